#!/bin/bash
# Same-box A/B of a process-level switch on the headline step: bench.py (event-profiled pass) with VAR=0 / VAR=1
# alternated, printing ms per step and the per-stage event times.  Usage: bash tools/ab_bench_stages.sh <tag> VAR [rounds]
# [values, default "0 1"]
set -o pipefail
TAG=$1; VAR=$2; R=${3:-2}; VALS=${4:-0 1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-compare --no-long --no-cpu-baseline \
      --no-caller --no-parity > "$OUT/b_${v}_$r.json" 2> "$OUT/b_${v}_$r.err" || { tail -20 "$OUT/b_${v}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b_${v}_$r.json')); st=d['roofline']['stages']; print('$VAR=$v', d['ms_per_step'], ' '.join(f'{k}={v[\"ms_per_step\"]}' for k, v in st.items() if v['ms_per_step'] > float('${MINMS:-0.3}')))"
  done
done
