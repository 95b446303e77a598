#!/bin/bash
# One GPU-box profiling pass of the bench workload: smoke(), rocprofv3 kernel-trace stats of bench.py,
# and the HBM traffic per kernel from two separate PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md
# HBM section) -> gpurun_out/<tag>/pmc_traffic.json.  Usage (repo root, through gpurun): bash tools/gpu_profile.sh <tag>
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp STEPS=2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-compare --no-parity > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/prof.err") \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/fetch" -o run -- \
      python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/fetch.log" 2>&1) \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$OUT/write" -o run -- \
      python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/write.log" 2>&1) \
&& python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.txt" 2>&1
rc=$?
cat "$OUT/smoke.log"; tail -3 "$OUT/prof.err"
exit $rc
