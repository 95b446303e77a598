#!/bin/bash
# One quick GPU-box iteration: parity tests (optionally a -k filter), the headline bench line only,
# and a per-launch kernel trace of one step (tools/launches.py reads it).
# Usage (repo root, through gpurun): bash tools/gpu_iter.sh <tag> [pytest -k expression | all | none]
set -o pipefail
TAG=${1:-iter}
SEL=${2:-all}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
t=0
if [ "$SEL" = "all" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; t=$?
elif [ "$SEL" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$SEL" > "$OUT/pytest_gpu.log" 2>&1; t=$?
fi
[ $t -eq 0 ] \
&& timeout -k 10 300 python -u bench.py --steps 20 --no-compare --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& (cd /tmp && STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
      python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/trace.log" 2>&1)
rc=$?
tail -3 "$OUT/pytest_gpu.log" 2>/dev/null; cut -c1-400 "$OUT/bench.json" 2>/dev/null; tail -3 "$OUT/bench.err" 2>/dev/null
exit $rc
