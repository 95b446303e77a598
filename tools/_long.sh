#!/bin/bash
# configs[4]-length clips (8 x 1000 frames per GPU): bench line + kernel stats
OUT=gpurun_out/long
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --clips 8 --frames 1000 --chunk 2000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$OUT/prof -o run -- python3 /root/repo/bench.py --clips 8 --frames 1000 --chunk 2000 --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /root/repo/$OUT/prof.log 2>&1)
rc=$?; cat $OUT/bench.json; exit $rc
