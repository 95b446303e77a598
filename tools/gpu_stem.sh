#!/bin/bash
# stem_b0 iteration: parity tests that run it (every-block taps fp32 / bf16x3 / bf16, configs), then kernel
# stats of the bench step in bf16x3 and bf16.  Usage: bash tools/gpu_stem.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-stem}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "effnet or config or smoke or bf16" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for dt in bf16x3 bf16; do
  (cd /tmp && export DTYPE=$dt && STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/$dt" -o run -- \
     python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/$dt.log" 2>&1) || exit 1
  echo "== $dt"; python3 tools/kstats.py "$OUT/$dt" 3 > "$OUT/$dt.txt"; grep -E "total|stem" "$OUT/$dt.txt"
done
