#!/bin/bash
# SE GEMM variant A/B on the bench step: kernel stats with env settings given as arguments (one run each).
# Usage: bash tools/gpu_se_ab.sh <tag> "A=1 B=2" "A=0" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  (cd /tmp && export $cfg && STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/v$i" -o run -- \
     python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/v$i.log" 2>&1) || exit 1
  echo "== $cfg"; python3 tools/kstats.py "$OUT/v$i" 3 > "$OUT/v$i.txt"; grep -E "total|gemm128|conv_gemm_kernel<128, 128, 4, 4, 2, 3, 2, 1>" "$OUT/v$i.txt"
done
