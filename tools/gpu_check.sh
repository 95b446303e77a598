#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench (N=1), rocprofv3 kernel stats of the bench workload.
# Usage (from the repo root, through gpurun):  bash tools/gpu_check.sh [tag] [skip-tests]
# Every GPU step has its own time limit and the steps are chained with &&: the first failure ends it.
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
}
if [ "$2" = "skip-tests" ]; then t=0; else run_tests; t=$?; fi
[ $t -eq 0 ] \
&& timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/prof.err") \
&& timeout -k 10 300 python -u bench.py --ragged --steps 20 --no-cpu-baseline > "$OUT/bench_ragged.json" 2> "$OUT/bench_ragged.err"
rc=$?
tail -3 "$OUT/pytest_gpu.log" 2>/dev/null; tail -2 "$OUT/smoke.log" 2>/dev/null; cat "$OUT/bench.json" 2>/dev/null
exit $rc
