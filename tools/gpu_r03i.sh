#!/bin/bash
# Round-3 measurement bundle: ir_ws / stem_b0 phase traces (diagnostic build), the GPU test suite,
# the default bench line, and kernel stats of the bench step at a 256-frame CNN chunk vs one
# 1920-frame pass (is the SE GEMM faster when the expanded map it reads fits the Infinity Cache?).
# Usage: bash tools/gpu_r03i.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r03i}
mkdir -p "$OUT"
export TMPDIR=/tmp
M2S_IR_WS_TRACE=1 timeout -k 10 200 python -u tools/trace_ir_ws.py > "$OUT/trace.txt" 2>&1 || exit 1
echo "trace done"
for c in 256 1920; do
  CHUNK=$c STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/chunk$c" -o run -- python3 tools/profile_step.py \
    > "$OUT/chunk$c.log" 2>&1 || exit 1
  echo "chunk $c done"
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-600 "$OUT/bench.json"
