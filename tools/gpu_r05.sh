#!/bin/bash
# Round-5 pass on the current tree: [GPU tests (TESTS=1)], bench (N=1, default flags), then the PMC evidence
# (tools/gpu_evidence.sh: kernel trace, FETCH / WRITE / SQ passes with the stage-tagged launch log).
# Usage (GPU box, repo root): [TESTS=1] bash tools/gpu_r05.sh <tag>
set -o pipefail
TAG=${1:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
rc=0
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?
fi
[ $rc = 0 ] && timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
[ $rc = 0 ] && [ "${EVIDENCE:-1}" = 1 ] && bash tools/gpu_evidence.sh "${TAG}_ev" > "$OUT/evidence.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log" 2>/dev/null; tail -2 "$OUT/smoke.log" 2>/dev/null
cut -c1-400 "$OUT/bench.json" 2>/dev/null; tail -3 "$OUT/bench.err"; tail -3 "$OUT/evidence.log" 2>/dev/null
exit $rc
