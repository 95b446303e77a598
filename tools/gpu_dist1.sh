#!/bin/bash
# The RCCL path of bench.py at one rank (M2S_BENCH_FORCE_DIST=1 under torchrun): state broadcast,
# length all-gather, result gather, barriers, max-reduce of the step time.  Usage: bash tools/gpu_dist1.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-dist1}
mkdir -p "$OUT"
M2S_BENCH_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline \
  > "$OUT/bench_dist1.json" 2> "$OUT/bench_dist1.err"
rc=$?
cut -c1-300 "$OUT/bench_dist1.json"; tail -3 "$OUT/bench_dist1.err"
exit $rc
