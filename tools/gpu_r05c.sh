#!/bin/bash
# ir_ws on LDS counters: parity tests, the headline step's per-kernel event times, the per-phase stamps.
# Usage (GPU box, repo root): bash tools/gpu_r05c.sh TAG
set -o pipefail
TAG=${1:-r05c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "ir_ws or every_block or timeout or config or s2band" > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
M2S_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 20 --no-caller --no-long --no-compare --no-cpu-baseline \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
M2S_IR_WS_TRACE=1 timeout -k 10 200 python -u tools/trace_ir_ws.py > "$OUT/irws_trace.txt" 2>&1 || exit $?
cut -c1-300 "$OUT/bench.json"; grep -E "ir_ws|se_ws|stem|er_sp" "$OUT/bench.err" | head -8
