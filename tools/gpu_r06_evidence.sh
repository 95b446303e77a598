#!/bin/bash
# Round 6 evidence of the current tree, part 1 (run through gpurun from the repo root): the rocprofv3 kernel trace of
# the bench, the PMC passes of the headline and of the fp8 configs[4] step (tools/gpu_evidence.sh), the SQ wait
# breakdown, and the kernel traces of the reference CLI's small shapes.  Post-process here with
#   python3 tools/evidence.py gpurun_out/<tag> profiles/<tag>; python3 tools/step_kstats.py <trace csv>
# Usage: bash tools/gpu_r06_evidence.sh <tag>
set -o pipefail
TAG=${1:-r06ev}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_evidence.sh "$TAG" || exit 1
bash tools/gpu_pmc_wait.sh "$TAG/sqwait" > "$OUT/sq_wait.txt" 2>&1 || { tail -20 "$OUT/sq_wait.txt"; exit 1; }
head -14 "$OUT/sq_wait.txt"
bash tools/gpu_small.sh "$TAG/small" || exit 1
