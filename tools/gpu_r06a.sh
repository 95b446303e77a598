#!/bin/bash
# Round 6, first check of the small-pass plan: the affected GPU tests, the configs[2] / configs[1] kernel timelines,
# and the bench's caller lines.  Usage: bash tools/gpu_r06a.sh <tag>
set -o pipefail
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bf16x3.py tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_plugin.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
bash tools/gpu_small.sh "$TAG/small" || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-compare --no-long --no-cpu-baseline --no-profile \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['parity']['wav_max_abs']); c=d['caller']; print('c2', c['configs2']['p50_ms'], c['configs2']['parity']['within_fp32_tol'], c['configs2']['parity']['wav_max_abs']); print('c1', c['configs1']['ms_per_call'], c['configs1']['parity'])"
