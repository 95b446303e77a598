#!/bin/bash
# Evidence of the current tree on one MI355X (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the bench workload (per-kernel average durations),
#   2. PMC passes, one counter group per run as MI355X_MICROARCH.md prescribes (FETCH_SIZE; WRITE_SIZE;
#      SQ_INSTS_MFMA + SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE; SQ_INSTS_VALU +
#      SQ_INSTS_LDS + SQ_LDS_BANK_CONFLICT + SQ_WAVE_CYCLES),
#   2b. the same four passes of the fp8 engine at configs[4]'s per-GPU shape (8 x 1000 frames; its e4m3 kernels and
#       its per-stage record, profiles/<tag>_c4fp8_stages.json),
#   3. the source hash the files were made from (tools/evidence.py keys the JSON by it; bench.py only
#      uses a traffic record of the tree it runs).
# Usage: bash tools/gpu_evidence.sh <tag> [extra profile_step env, e.g. DTYPE=bf16]
set -o pipefail
TAG=${1:-evidence}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
export STEPS=${STEPS:-2}
python3 -c "import bench; print(bench.source_sha())" > "$OUT/src_sha.txt" || exit 1
pmc() {  # pmc <dir> <counters...>
  local d=$1; shift
  (cd /tmp && M2S_LAUNCH_LOG="$ROOT/$OUT/$d.launches.json" timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/$OUT/$d" -o run -- \
     python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/$d.log" 2>&1)
}
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
   python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-compare --no-parity \
   > "$ROOT/$OUT/bench_under_rocprof.json" 2> "$ROOT/$OUT/trace.err") \
&& pmc fetch FETCH_SIZE \
&& pmc write WRITE_SIZE \
&& pmc mfma SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
&& pmc valu SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
&& DTYPE=fp8 CLIPS=8 FRAMES=1000 pmc fetch8 FETCH_SIZE \
&& DTYPE=fp8 CLIPS=8 FRAMES=1000 pmc write8 WRITE_SIZE \
&& DTYPE=fp8 CLIPS=8 FRAMES=1000 pmc mfma8 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
&& DTYPE=fp8 CLIPS=8 FRAMES=1000 pmc valu8 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES
rc=$?
cat "$OUT/src_sha.txt"; cut -c1-300 "$OUT/bench_under_rocprof.json"
exit $rc
