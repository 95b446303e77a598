#!/bin/bash
# Per-kernel time of configs[4]'s per-GPU step (8 clips x 1000 frames) for each dtype given, in-tree package.
# Usage (GPU box, repo root): bash tools/gpu_trace_c4.sh TAG DTYPE [DTYPE ...]
set -o pipefail
TAG=$1; shift
ROOT=$(pwd)
export TMPDIR=/tmp AB_SHAPE=8x1000
mkdir -p "gpurun_out/$TAG"
for dt in "$@"; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$TAG/$dt" -o run -- \
    python3 "$ROOT/tools/ab_step.py" --child "${PKG:-mri-to-speech_amd}" "$dt") > "gpurun_out/$TAG/$dt.log" 2>&1 || exit $?
  f=$(find "gpurun_out/$TAG/$dt" -name run_kernel_trace.csv)
  python3 tools/trace_sum.py "$f" 4 > "gpurun_out/$TAG/$dt.sum.txt" || exit $?
  rm -f "$f"
done
