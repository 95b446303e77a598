#!/bin/bash
# Round-3 evidence of the current tree: tools/gpu_evidence.sh (rocprof kernel stats of the bench, PMC FETCH /
# WRITE / SQ passes) plus a FETCH_SIZE calibration on tools/bw_probe (kernels that read a known 1.447 GB with
# 16-byte lane loads / LDS-DMA over 2944-byte rows), for the dwconv over-fetch question.  Usage: bash tools/gpu_r03_evidence.sh <tag>
set -o pipefail
TAG=${1:-r03ev}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
bash tools/gpu_evidence.sh "$TAG" || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/cal" -o run -- \
   "$ROOT/tools/bw_probe" > "$ROOT/$OUT/cal.log" 2>&1) || exit 1
echo calibration done
