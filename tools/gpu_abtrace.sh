#!/bin/bash
# Kernel traces of the whole bench step for several m2s packages (tools/ab_step.py --child), for per-kernel
# A/B with tools/step_kstats.py.  Usage (GPU box, repo root): bash tools/gpu_abtrace.sh TAG PKG [PKG ...]
set -o pipefail
TAG=$1; shift
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p "gpurun_out/$TAG"
i=0
for pkg in "$@"; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$TAG/p$i" -o run -- \
    python3 "$ROOT/tools/ab_step.py" --child "$pkg" bf16x3) > "gpurun_out/$TAG/p$i.log" 2>&1 || exit $?
  f=$(find "gpurun_out/$TAG/p$i" -name run_kernel_trace.csv)
  echo "== $pkg" >> "gpurun_out/$TAG/kstats.txt"
  python3 tools/step_kstats.py "$f" >> "gpurun_out/$TAG/kstats.txt" || exit $?
  rm -f "$f"
  i=$((i+1))
done
