#!/bin/bash
# Round-4 final pass: the fp8 e4m3-expand A/B, the GPU test suite + smoke, the bench (N=1, default flags),
# rocprofv3 kernel stats of the bench workload.  Usage: bash tools/gpu_r04fin.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r04fin}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_env.py M2S_F8_EXPAND 28 fp8 > "$OUT/ab_f8x.txt" 2>&1 \
&& timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/prof.err")
rc=$?
grep -v amdgpu.ids "$OUT/ab_f8x.txt"; tail -3 "$OUT/pytest_gpu.log" 2>/dev/null; tail -2 "$OUT/smoke.log" 2>/dev/null
cut -c1-400 "$OUT/bench.json" 2>/dev/null
exit $rc
