#!/bin/bash
# Round-4 closing pass on the final source: bench (N=1, default flags; its event table against rocprofv3),
# rocprofv3 kernel stats of the bench workload, then the PMC evidence of the same tree.
set -o pipefail
OUT=gpurun_out/${1:-r04fin2}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& bash tools/gpu_evidence.sh "${1:-r04fin2}_ev" > "$OUT/evidence.log" 2>&1
rc=$?
cut -c1-300 "$OUT/bench.json" 2>/dev/null; tail -3 "$OUT/evidence.log"
exit $rc
