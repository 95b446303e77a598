#!/bin/bash
# bench.py headline step time for several CNN chunk sizes (frames per CNN pass): smaller chunks keep
# each pass's intermediate maps within the 256 MB Infinity Cache.  Usage: bash tools/gpu_chunk_sweep.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-chunk}
mkdir -p "$OUT"
for c in 1920 960 640 480 384 320 256; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-compare --no-cpu-baseline --no-parity --no-profile --chunk $c \
    > "$OUT/chunk_$c.json" 2> "$OUT/chunk_$c.err" || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/chunk_$c.json')); print($c, d['ms_per_step'])"
done
