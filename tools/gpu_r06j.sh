#!/bin/bash
# Round 6: per-parity W ring hand-off of ir_ws (M2S_IRWS_PAR=1): the ir_ws tests with it on, a same-box A/B of the CNN.
set -o pipefail
TAG=${1:-r06j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
M2S_IRWS_PAR=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_configs.py -m gpu -x -q \
  -k "ir_ws or config3 or every_block or timeout" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
AB_VALUES=0,1 timeout -k 10 300 python -u tools/ab_env.py M2S_IRWS_PAR 2 bf16x3 > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
AB_VALUES=1,0,1,0 timeout -k 10 300 python -u tools/ab_env.py M2S_IRWS_PAR 2 bf16x3 > "$OUT/ab2.txt" 2>&1 || { tail -20 "$OUT/ab2.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab2.txt"
