#!/bin/bash
# Round 6: se_ws half tiles: the ir_ws / config tests, a same-box A/B (M2S_IRWS_PARTS=1 vs auto) of the CNN and a
# short headline bench.  Usage: bash tools/gpu_r06h.sh <tag>
set -o pipefail
TAG=${1:-r06h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fp8.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
AB_VALUES=0,1 timeout -k 10 300 python -u tools/ab_env.py M2S_SEWS_HALF 2 bf16x3 > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-compare --no-long --no-cpu-baseline --no-caller \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['parity']['wav_max_abs'], r['kernel'], r['avg_launch_us'], r['bound'], r['frac'])"
