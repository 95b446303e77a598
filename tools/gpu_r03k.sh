#!/bin/bash
# Round-3 state of the tree: GPU tests + smoke + default bench + rocprof of the bench (tools/gpu_check.sh),
# then kernel stats of the configs[4]-style workload (8 clips x 1000 frames) per dtype (bf16, fp8, bf16x3)
# for the fp8 plan.  Usage: bash tools/gpu_r03k.sh <tag>
set -o pipefail
TAG=${1:-r03k}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
bash tools/gpu_check.sh "$TAG" || exit 1
export TMPDIR=/tmp
for dt in bf16 fp8 bf16x3; do
  (cd /tmp && CLIPS=8 FRAMES=1000 CHUNK=1920 STEPS=3 DTYPE=$dt timeout -k 10 180 rocprofv3 --kernel-trace --stats \
     --output-format csv -d "$ROOT/$OUT/long_$dt" -o run -- python3 "$ROOT/tools/profile_step.py" \
     > "$ROOT/$OUT/long_$dt.log" 2>&1) || exit 1
  echo "long $dt done"
done
