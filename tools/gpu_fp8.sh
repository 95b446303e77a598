#!/bin/bash
# fp8 iteration: the fp8 parity tests, then kernel stats of the configs[4]-style workload (8 x 1000 frames)
# in fp8 and the fp8 / bf16 bench lines at that shape.  Usage: bash tools/gpu_fp8.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-fp8}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread -k "${2:-fp8}" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
grep -E "cos|PASS|FAIL" "$OUT/pytest.log" | cut -c1-200
(cd /tmp && CLIPS=8 FRAMES=1000 CHUNK=1920 STEPS=3 DTYPE=fp8 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
   --output-format csv -d "$ROOT/$OUT/long_fp8" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/long_fp8.log" 2>&1) || exit 1
python3 tools/kstats.py "$OUT/long_fp8" 3 > "$OUT/kstats.txt" && head -25 "$OUT/kstats.txt"
for dt in fp8 bf16; do
  timeout -k 10 300 python -u bench.py --dtype $dt --clips 8 --frames 1000 --steps 3 --warmup 1 --no-compare --no-cpu-baseline \
    --no-long > "$OUT/bench_$dt.json" 2> "$OUT/bench_$dt.err" || { tail -20 "$OUT/bench_$dt.err"; exit 1; }
  cut -c1-300 "$OUT/bench_$dt.json"
done
