#!/bin/bash
# Round 6: the whole GPU suite and smoke() on the current tree (one process each).  Usage: bash tools/gpu_r06_tests.sh <tag>
set -o pipefail
TAG=${1:-r06t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
grep smoke "$OUT/smoke.txt"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
