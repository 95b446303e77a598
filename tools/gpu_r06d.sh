#!/bin/bash
# Round 6: the fp32 ir_ws -> se_ws hand-off (tests + headline bench + kernel trace) and the split-K A/B on the small
# shapes.  Usage: bash tools/gpu_r06d.sh <tag>
set -o pipefail
TAG=${1:-r06d}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16x3.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-compare --no-long --no-cpu-baseline --no-caller \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['parity']['wav_max_abs'], r['kernel'], r['avg_launch_us'], r['bound'], r['frac']); print({k: v['ms_per_step'] for k, v in r['stages'].items()})"
(cd /tmp && CHUNK=1920 STEPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- \
   python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/prof.log" 2>&1) || exit 1
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY' > "$OUT/kstats.txt"
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:24]:
    print(f"{float(r['TotalDurationNs'])/1e6/3:9.3f} ms/step {int(r['Calls'])//3:5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
head -14 "$OUT/kstats.txt"
find "$OUT/prof" -name "*kernel_trace.csv" -delete
timeout -k 10 400 python -u tools/ab_small.py "" "M2S_KSPLIT=1" "M2S_KSPLIT_MAX=4" "M2S_KSPLIT_MAX=8" "M2S_KSPLIT_MINST=2" "M2S_KSPLIT_MINST=8" \
  > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v "^#" "$OUT/ab.txt"
