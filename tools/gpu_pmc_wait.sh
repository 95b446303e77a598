#!/bin/bash
# Where the waves of each kernel spend their cycles (one PMC pass, MI355X_MICROARCH.md SQ table): SQ_WAVE_CYCLES =
# SQ_WAIT_ANY (parked at s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall) + SQ_ACTIVE_INST_ANY, with
# SQ_ACTIVE_INST_VALU and SQ_INSTS_VALU.  Usage (GPU box, repo root): [DTYPE=fp8 CLIPS=8 FRAMES=1000] bash tools/gpu_pmc_wait.sh <tag>
set -o pipefail
TAG=${1:-pmcwait}
OUT=gpurun_out/$TAG
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp STEPS=${STEPS:-2}
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
   SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/wait" -o run -- \
   python3 "$ROOT/tools/profile_step.py" > "$ROOT/$OUT/wait.log" 2>&1) || { tail -20 "$OUT/wait.log"; exit 1; }
python3 - "$OUT/wait" <<'PY'
import collections, csv, glob, os, sys
sys.path.insert(0, "tools")
from pmc_traffic import short
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection*.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"] or 0)
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))
print(f"{'kernel':60s} {'gui Mcyc':>9s} {'wait':>6s} {'waitinst':>8s} {'active':>6s} {'valu':>6s} {'valu instr/wave-kcyc':>10s}")
for k, v in rows[:24]:
    w = v.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:60]:60s} {v.get('GRBM_GUI_ACTIVE', 0) / 8e6:9.2f} {v.get('SQ_WAIT_ANY', 0) / w:6.3f} {v.get('SQ_WAIT_INST_ANY', 0) / w:8.3f} "
          f"{v.get('SQ_ACTIVE_INST_ANY', 0) / w:6.3f} {v.get('SQ_ACTIVE_INST_VALU', 0) / w:6.3f} {1000 * v.get('SQ_INSTS_VALU', 0) / w:10.1f}")
PY
