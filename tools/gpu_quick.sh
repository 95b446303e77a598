#!/bin/bash
# Quick GPU iteration: selected parity tests, the diagnostic stamps, a short headline bench.
# Usage: bash tools/gpu_quick.sh <tag> "<pytest -k expression>"
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${2:-effnet}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
M2S_IR_WS_TRACE=1 timeout -k 10 200 python -u tools/trace_ir_ws.py > "$OUT/trace.txt" 2>&1 || { tail -20 "$OUT/trace.txt"; exit 1; }
grep -o "STEMTRACE.\{0,700\}" "$OUT/trace.txt" | head -2
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-compare --no-cpu-baseline --no-parity --no-profile --no-long > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-400 "$OUT/bench.json"
CHUNK=1920 STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/profile_step.py > "$OUT/prof.log" 2>&1 || exit 1
python3 tools/rocpd_stats.py "$OUT/prof" > "$OUT/kstats.txt" && cut -c1-130 "$OUT/kstats.txt" | sed -n 1,18p
