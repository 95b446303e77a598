#!/bin/bash
# Round 5: fp8 e4m3 EdgeResidual blocks.2.1/.2 (er8w_fused) tests + A/B + configs[4] trace; cross-run NaN check;
# ir_ws per-phase stamps (diagnostic build under diag/).  Usage (GPU box, repo root): bash tools/gpu_r05b.sh TAG
set -o pipefail
TAG=${1:-r05b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_fp8.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_fp8.log"
  [ $rc = 0 ] || exit $rc
fi
timeout -k 10 200 python -u tools/nan_runs.py > "$OUT/nan_runs.txt" 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_env.py M2S_F8_ER2 8 fp8 > "$OUT/ab_f8er2.txt" 2>&1 || exit $?
bash tools/gpu_trace_c4.sh "$TAG/c4" fp8 bf16 || exit $?
M2S_IR_WS_TRACE=1 timeout -k 10 200 python -u tools/trace_ir_ws.py > "$OUT/irws_trace.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/ab_f8er2.txt"; cat "$OUT/nan_runs.txt" | grep -v amdgpu.ids | cut -c1-300
