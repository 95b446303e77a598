#!/bin/bash
# fused-MRF check: vocoder parity tests + bench + kernel stats
OUT=gpurun_out/mrf1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k vocoder -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
&& M2S_MRF_FUSED=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_unfused.json 2>> $OUT/bench.err \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$OUT/prof -o run -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /root/repo/$OUT/prof.log 2>&1)
rc=$?
tail -5 $OUT/pytest.log; cat $OUT/bench.json $OUT/bench_unfused.json
exit $rc
