"""Per-launch durations of the last profile_step.py step from a rocprofv3 --kernel-trace CSV.

python tools/launches.py gpurun_out/<tag>/trace [filter]   (tools/gpu_iter.sh writes the trace)
"""
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
step = rows[len(rows) // 2:]  # STEPS=2: the second step
tot = 0.0
groups = {}
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    nm = re.sub(r"m2s::\(anonymous namespace\)::|void |\(.*", "", r["Kernel_Name"])[:64]
    groups[nm] = groups.get(nm, 0.0) + d
    if flt and flt in nm:
        print(f"{d:8.1f} us  {nm:64s} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
print(f"step GPU time {tot / 1e3:.3f} ms, {len(step)} launches")
for nm, d in sorted(groups.items(), key=lambda x: -x[1])[:25]:
    print(f"{d / 1e3:8.3f} ms  {nm}")
