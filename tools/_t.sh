#!/bin/bash
# quick check: GPU parity subset + bench (no cpu baseline) + kernel stats
OUT=gpurun_out/${1:-t}
K=${2:-effnet or pipeline or vocoder}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "$K" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$OUT/prof -o run -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /root/repo/$OUT/prof.log 2>&1)
rc=$?
tail -3 $OUT/pytest.log; python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'])"
exit $rc
