#!/bin/bash
# Kernel traces of the reference CLI's shapes (configs[2] 1 x 30 bf16x3 end to end, configs[1] 8 x 4 bf16
# acoustic): per-call timelines -> gpurun_out/<tag>/{c2,c1}.timeline.txt.  Usage: bash tools/gpu_small.sh <tag>
set -o pipefail
TAG=${1:-small}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in c2 c1; do
  (cd /tmp && MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$m" -o run -- \
     python3 "$ROOT/tools/profile_small.py") > "$OUT/$m.log" 2>&1 || { tail -20 "$OUT/$m.log"; exit 1; }
  f=$(find "$OUT/$m" -name run_kernel_trace.csv)
  python3 tools/small_timeline.py "$f" > "$OUT/$m.timeline.txt" || exit 1
  grep "host wall" "$OUT/$m.log"; head -3 "$OUT/$m.timeline.txt"
  rm -f "$f"
done
