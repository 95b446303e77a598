#!/bin/bash
# SQ instruction-mix and wait counters per kernel for the bench workload (two PMC passes, 8 SQ
# counters each).  Usage (repo root, through gpurun): bash tools/gpu_pmc_sq.sh [tag]
TAG=${1:-sq}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp STEPS=1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS \
   --output-format csv -d "$ROOT/$OUT/a" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/a.log" 2>&1) \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES \
   --output-format csv -d "$ROOT/$OUT/b" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/b.log" 2>&1)
