#!/bin/bash
# HBM traffic per kernel (rocprofv3 PMC, one counter group per pass, as MI355X_MICROARCH.md
# prescribes) plus a per-layer event profile of the bench workload.
# Usage (repo root, through gpurun):  bash tools/gpu_pmc.sh [tag]
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
export STEPS=2
M2S_PROF_DETAIL=1 M2S_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_detail.json" 2> "$OUT/bench_detail.err" \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/fetch" -o run -- \
      python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/fetch.log" 2>&1) \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$OUT/write" -o run -- \
      python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/write.log" 2>&1) \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
      -d "$ROOT/$OUT/mfma" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/mfma.log" 2>&1)
rc=$?
tail -5 "$OUT/bench_detail.err"
exit $rc
