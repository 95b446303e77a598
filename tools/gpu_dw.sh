#!/bin/bash
# dwconv XCD order: parity tests that run the depthwise (fp32 / bf16x3 effnet taps), then one FETCH_SIZE pass and
# kernel stats of the bench step.  Usage: bash tools/gpu_dw.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-dw}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp STEPS=2
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "effnet or config or gemm128" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/fetch" -o run -- \
   python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/fetch.log" 2>&1) || exit 1
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
   python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/trace.log" 2>&1) || exit 1
python3 tools/kstats.py "$OUT/trace" 2 dwconv
