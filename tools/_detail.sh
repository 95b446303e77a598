#!/bin/bash
# per-layer event profile of the bench (M2S_PROF_DETAIL names carry kind, tile, K, N, M)
mkdir -p gpurun_out/detail
M2S_PROF_DETAIL=1 M2S_BENCH_KERNELS=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/detail/bench.json 2> gpurun_out/detail/kernels.txt
rc=$?
grep "^#" gpurun_out/detail/kernels.txt | head -45
exit $rc
