#!/bin/bash
OUT=gpurun_out/chunk
mkdir -p $OUT
for c in 1920 960 480 240; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --chunk $c > $OUT/b$c.json 2> $OUT/b$c.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b$c.json'));print($c, d['value'], d['ms_per_step'])"
done
