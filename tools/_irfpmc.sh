#!/bin/bash
OUT=gpurun_out/irfpmc; mkdir -p $OUT; export TMPDIR=/tmp; R=$(pwd)
for m in ${MODES:-0 1}; do
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --output-format csv -d $R/$OUT/a$m -o run -- $R/tools/irf_bench_$m > $R/$OUT/a$m.log 2>&1) || exit 1
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --output-format csv -d $R/$OUT/b$m -o run -- $R/tools/irf_bench_$m > $R/$OUT/b$m.log 2>&1) || exit 1
done
