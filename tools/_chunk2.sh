#!/bin/bash
# e2e frames/s vs CNN chunk size (ir_block off / on)
mkdir -p gpurun_out/chunk2
for ib in 0 1; do for c in 1920 960 640 480; do
  M2S_IR_BLOCK=$ib timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --chunk $c > gpurun_out/chunk2/b_${ib}_$c.json 2>gpurun_out/chunk2/e_${ib}_$c.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/chunk2/b_${ib}_$c.json'));print('ib=$ib chunk=$c', d['value'], d['ms_per_step'])"
done; done
