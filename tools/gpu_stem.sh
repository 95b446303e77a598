#!/bin/bash
# stem_b0 iteration: its parity tests, the diagnostic per-phase stamps, the headline bench's kernel table.
set -o pipefail
OUT=gpurun_out/${1:-stem}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "every_block or fused_kernels_vs_unfused or test_pipeline_bf16x3_end_to_end" > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
M2S_IR_WS_TRACE=1 timeout -k 10 200 python -u tools/trace_ir_ws.py > "$OUT/trace.txt" 2>&1 || { tail -20 "$OUT/trace.txt"; exit 1; }
grep -o "STEMTRACE.\{0,900\}" "$OUT/trace.txt" | head -1
M2S_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-compare --no-cpu-baseline --no-parity --no-long \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-250 "$OUT/bench.json"
grep "stem_b0\|lstm" "$OUT/bench.err"
