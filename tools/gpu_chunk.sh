#!/bin/bash
# Kernel stats of the bf16x3 bench step at CNN chunks of 256 and 1920 frames: does the SE GEMM read its
# expanded map faster when the map of one pass fits the 256 MB Infinity Cache?  Usage: bash tools/gpu_chunk.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-chunk}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in 256 1920; do
  (cd /tmp && export CHUNK=$c && STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/c$c" -o run -- \
     python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/c$c.log" 2>&1) || exit 1
  echo "== chunk $c"; python3 tools/kstats.py "$OUT/c$c" 3 > "$OUT/c$c.txt"; head -12 "$OUT/c$c.txt"
done
