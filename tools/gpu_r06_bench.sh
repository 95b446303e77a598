#!/bin/bash
# Round 6: the default bench line of the current tree (as the driver runs it) and a same-box stage A/B of a switch.
# Usage: bash tools/gpu_r06_bench.sh <tag> [VAR]
set -o pipefail
TAG=${1:-r06b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cut -c1-400 "$OUT/bench.json"
if [ -n "$2" ]; then bash tools/ab_bench_stages.sh "$TAG/ab" "$2" 2 || exit 1; fi
