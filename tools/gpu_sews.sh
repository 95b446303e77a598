#!/bin/bash
# se_ws A/B on one box: parity tests, then the headline bench (per-kernel event table) for the barrier ring
# (M2S_SE_WS=0) and each se_ws ring variant (M2S_SE_WS_CFG).  Usage: bash tools/gpu_sews.sh <tag> [pytest -k]
set -o pipefail
OUT=gpurun_out/${1:-sews}
SEL=${2:-"se_ws or ir_ws"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$SEL" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" M2S_BENCH_KERNELS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-compare --no-cpu-baseline \
    --no-parity --no-long > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail -20 "$OUT/bench_$n.err"; return 1; }
  echo "== $n: $(cut -c1-200 "$OUT/bench_$n.json")"
  grep -E "^# (se_ws|conv_gemm_kernel<128, 128, 4, 4, 2, 3, 2, 1>|ir_ws)" "$OUT/bench_$n.err"
}
run ring M2S_SE_WS=0 && run cfg0 M2S_SE_WS=1 M2S_SE_WS_CFG=0 && run cfg1 M2S_SE_WS=1 M2S_SE_WS_CFG=1 && run cfg2 M2S_SE_WS=1 M2S_SE_WS_CFG=2 && run cfg3 M2S_SE_WS=1 M2S_SE_WS_CFG=3
