#!/bin/bash
# e2e frames/s under alternative env settings: bash tools/_gb.sh "VAR=a" "VAR=b" ...
for kv in "$@"; do
  env $kv timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/gb.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/gb.json'));print('$kv', d['value'], d['ms_per_step'])"
done
