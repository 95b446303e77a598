#!/bin/bash
# fp8 ir_pwdw f16-depthwise A/B: per-kernel times vs the IRPW_F16=0 variant (same box), the fp8 tests, and the
# fp8 / bf16 lines at configs[4]'s shape.  Usage (GPU box, repo root): bash tools/gpu_f16dw.sh <tag> [variant]
set -o pipefail
TAG=${1:-f16dw}
VAR=${2:-variants/f16off}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
AB_DTYPE=fp8 AB_KERN=${AB_KERN:-ir_pwdw} AB_ROUNDS=2 timeout -k 10 300 python -u tools/ab_kern.py mri-to-speech_amd "$VAR" > "$OUT/ab.txt" 2>&1 \
  || { tail -30 "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt" | cut -c1-400
timeout -k 10 500 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_configs4.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "fp8" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
grep -E "passed|failed|cos" "$OUT/pytest.log" | tail -30 | cut -c1-200
for dt in fp8 bf16; do
  timeout -k 10 300 python -u bench.py --dtype $dt --clips 8 --frames 1000 --steps 3 --warmup 1 --no-compare --no-cpu-baseline \
    --no-long > "$OUT/bench_$dt.json" 2> "$OUT/bench_$dt.err" || { tail -20 "$OUT/bench_$dt.err"; exit 1; }
  cut -c1-300 "$OUT/bench_$dt.json"
done
