#!/bin/bash
# Ablation of the e4m3 SE GEMM (measurement only): per-launch time with the gate VALU, the MFMAs, or all
# compute removed (M2S_F8_ABLATE = 1 / 3 / 7), fp8 engine at 8 x 1000 frames.  Usage: bash tools/gpu_f8_ablate.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-f8abl}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 0 1 3 7; do
  (cd /tmp && M2S_F8_ABLATE=$v CLIPS=8 FRAMES=1000 CHUNK=1920 STEPS=2 DTYPE=fp8 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
     --output-format csv -d "$ROOT/$OUT/a$v" -o run -- python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/a$v.log" 2>&1) || exit 1
  echo "== ablate $v"; python3 tools/kstats.py "$OUT/a$v" 2 f8_gemm
done
