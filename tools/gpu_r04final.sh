#!/bin/bash
# Round-4 closing pass on the final tree: the fp8 e4m3 EdgeResidual A/B (M2S_F8_ER), the GPU test suite +
# smoke, then tools/gpu_r04fin2.sh (bench N=1 default flags + rocprofv3 stats + PMC evidence).
# Usage (GPU box, repo root): bash tools/gpu_r04final.sh <tag>
set -o pipefail
TAG=${1:-r04final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_env.py M2S_F8_ER 5 fp8 > "$OUT/ab_f8er.txt" 2>&1 \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& bash tools/gpu_r04fin2.sh "$TAG"
rc=$?
grep -v amdgpu.ids "$OUT/ab_f8er.txt"; tail -2 "$OUT/pytest_gpu.log" 2>/dev/null; tail -2 "$OUT/smoke.log" 2>/dev/null
exit $rc
