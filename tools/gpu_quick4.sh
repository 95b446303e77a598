#!/bin/bash
# Round-4 quick iteration: selected GPU tests, the headline bench with the per-kernel event table
# (stderr), nothing else.  Usage (repo root, through gpurun): bash tools/gpu_quick4.sh <tag> "<pytest -k>" [bench args]
set -o pipefail
OUT=gpurun_out/${1:-q4}
SEL=${2:-ir_ws}
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$SEL" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$SEL" > "$OUT/pytest.log" 2>&1 \
    || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
M2S_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-compare --no-cpu-baseline --no-parity --no-long "$@" \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-300 "$OUT/bench.json"
grep "^#" "$OUT/bench.err" | head -25
