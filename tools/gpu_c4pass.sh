#!/bin/bash
# configs[4] shape after a CNN pass-size change: the chunking / configs[4] tests, then the 8 x 1000 lines per dtype.
# Usage (GPU box, repo root): bash tools/gpu_c4pass.sh <tag> [dtype ...]
set -o pipefail
TAG=${1:-c4pass}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs4.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "chunking or config4" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest.log" | tail -3 | cut -c1-200
for dt in "${@:-fp8 bf16}"; do
  timeout -k 10 300 python -u bench.py --dtype $dt --clips 8 --frames 1000 --steps 3 --warmup 1 --no-compare --no-cpu-baseline \
    --no-long > "$OUT/bench_$dt.json" 2> "$OUT/bench_$dt.err" || { tail -20 "$OUT/bench_$dt.err"; exit 1; }
  echo "$dt $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], 'ms', d['value'])" "$OUT/bench_$dt.json")"
done
