#!/bin/bash
# rocprof kernel table of the bench under extra env settings: bash tools/_kt.sh TAG [VAR=value ...]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$OUT/prof -o run -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /root/repo/$OUT/bench.json 2> /root/repo/$OUT/err.log
rc=$?
cd /root/repo && python3 tools/kstats.py $OUT/prof 4 "" 2>/dev/null | head -${KT_N:-16}
exit $rc
