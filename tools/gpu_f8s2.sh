#!/bin/bash
# fp8 coverage pass: blocks.5.0 on e4m3 (M2S_F8_S2) and the C = 64 MRF on e4m3 (M2S_F8_MRF64): their tests, the
# fp8 CNN per-kernel A/B against a variant package, the fp8 tests, and the configs[4] fp8 line with each switch
# on and off plus the bf16 line.  Usage (GPU box, repo root): bash tools/gpu_f8s2.sh <tag> [variant]
set -o pipefail
TAG=${1:-f8s2}
VAR=${2:-variants/f16off}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "stride2 or mrf_narrow" > "$OUT/pytest_new.log" 2>&1 \
  || { tail -40 "$OUT/pytest_new.log"; exit 1; }
grep -E "passed|failed|cos" "$OUT/pytest_new.log" | tail -20 | cut -c1-200
AB_DTYPE=fp8 AB_KERN=ir_pwdw AB_ROUNDS=2 timeout -k 10 300 python -u tools/ab_kern.py mri-to-speech_amd "$VAR" > "$OUT/ab.txt" 2>&1 \
  || { tail -30 "$OUT/ab.txt"; exit 1; }
cut -c1-400 "$OUT/ab.txt"
bl() {  # bl <name> <dtype> [env...]
  local n=$1 dt=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --dtype $dt --clips 8 --frames 1000 --steps 3 --warmup 1 --no-compare \
    --no-cpu-baseline --no-long > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail -20 "$OUT/bench_$n.err"; return 1; }
  echo "$n $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], 'ms', d.get('parity'))" "$OUT/bench_$n.json" | cut -c1-300)"
}
bl fp8 fp8 && bl fp8_nos2 fp8 M2S_F8_S2=0 && bl fp8_nomrf64 fp8 M2S_F8_MRF64=0 && bl fp8_mrf32 fp8 M2S_F8_MRF32=1 && bl bf16 bf16 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_configs4.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "fp8" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest.log" | tail -3 | cut -c1-200
