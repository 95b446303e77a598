#!/bin/bash
# Per-kernel A/B of an env switch read once per process (static), over the bf16x3 bench step, one process per
# value, alternating: bash tools/gpu_abenv_trace.sh TAG VAR V1 V2 [V1 V2 ...]   (GPU box, repo root)
set -o pipefail
TAG=$1; VAR=$2; shift 2
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p "gpurun_out/$TAG"
i=0
for v in "$@"; do
  (export "$VAR=$v" && cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/$TAG/p$i" \
    -o run -- python3 "$ROOT/tools/ab_step.py" --child mri-to-speech_amd bf16x3) > "gpurun_out/$TAG/p$i.log" 2>&1 || exit $?
  f=$(find "gpurun_out/$TAG/p$i" -name run_kernel_trace.csv)
  echo "== $VAR=$v" >> "gpurun_out/$TAG/kstats.txt"
  python3 tools/step_kstats.py "$f" >> "gpurun_out/$TAG/kstats.txt" || exit $?
  rm -f "$f"
  i=$((i+1))
done
