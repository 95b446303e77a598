#!/bin/bash
# SQ counters of ir_block_kernel (one pass, 8 SQ counters)
OUT=gpurun_out/ibpmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "${IBPMC_RE:-ir_block|er2_fused}" --output-format csv -d /root/repo/$OUT -o pmc -- python3 /root/repo/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile > /root/repo/$OUT/log 2>&1
rc=$?
cd /root/repo && python3 - <<'P'
import csv, glob, collections
f = glob.glob('gpurun_out/ibpmc/**/*counter_collection.csv', recursive=True)
print(f)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for fn in f:
    for r in csv.DictReader(open(fn)):
        k = r.get('Kernel_Name', '')[:40]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {v:.4g}')
P
exit $rc
