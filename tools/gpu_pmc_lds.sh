#!/bin/bash
# LDS pressure per kernel on the bench workload: one PMC pass of SQ LDS counters (+ GRBM_GUI_ACTIVE), one
# step.  Usage (repo root, through gpurun): bash tools/gpu_pmc_lds.sh [tag]
TAG=${1:-lds}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp STEPS=1
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
   --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/a.log" 2>&1)
rc=$?
python3 tools/pmc_summary.py "$OUT/a" > "$OUT/summary.txt" 2>&1
head -40 "$OUT/summary.txt"
exit $rc
