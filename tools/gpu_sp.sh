#!/bin/bash
# bf16x3 iteration: selected GPU tests, a short headline bench, kernel stats of the bench step with a kernel
# switch on and off.  Usage: bash tools/gpu_sp.sh <tag> "<pytest -k expr>" <ENV_SWITCH>   (e.g. M2S_SE_SP)
set -o pipefail
OUT=gpurun_out/${1:-sp}
ROOT=$(pwd)
SW=${3:-M2S_SE_SP}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${2:-bf16x3}" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-compare --no-cpu-baseline --no-long > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-330 "$OUT/bench.json"
for v in 1 0; do
  (cd /tmp && export $SW=$v && STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/p$v" -o run -- \
     python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/p$v.log" 2>&1) || exit 1
  echo "== $SW=$v"; python3 tools/kstats.py "$OUT/p$v" 3 | head -12
done
