#!/bin/bash
# Round 6: small-shape kernels (gap, se_excite prefetch, rb1 init, split-K cap 8): affected tests + small A/B + timelines.
set -o pipefail
TAG=${1:-r06f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_gradcam.py tests/test_gpu_bf16x3.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/ab_small.py "" "M2S_KSPLIT_MAX=16" > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v "^#" "$OUT/ab.txt" | grep -v amdgpu.ids
bash tools/gpu_small.sh "$TAG/small" || exit 1
