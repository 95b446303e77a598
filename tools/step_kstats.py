"""Per-kernel durations of the HEADLINE step only, from a rocprofv3 kernel trace of bench.py.

rocprofv3's --stats averages every launch of a kernel over the whole process, and bench.py also runs the
secondary lines (bf16 / fp8 / fp32) and the configs[4] lines, whose chunk sizes differ (a 320-frame tail
chunk launches the same ir_ws_kernel for 1/6 of the work): its 'AverageNs' is not the headline launch.
Here the headline steps are cut out of the trace (a step = the launches from one split stem_b0 to the
next whose grid matches the first step's) and every kernel is averaged over those steps only, so the
numbers compare with bench.py's event-timed roofline.avg_launch_us.
Usage: python3 tools/step_kstats.py <run_kernel_trace.csv> [stem kernel prefix]"""
import csv
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
stem = sys.argv[2] if len(sys.argv) > 2 else "void m2s::(anonymous namespace)::stem_b0_kernel<16, 1>"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(stem)]
# the headline steps come first (warm-up, timed steps, the event-timed pass): the leading run of segments
# with the first segment's launch count (later the secondary lines and the configs[4] CNN chunks follow)
segs = []
for a, b in zip(starts, starts[1:]):
    if segs and b - a != segs[0][1] - segs[0][0]:
        break
    segs.append((a, b))
n_mode = segs[0][1] - segs[0][0]
per = defaultdict(list)
walls = []
for a, b in segs:
    walls.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    for r in rows[a:b]:
        per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"# {len(segs)} headline steps of {n_mode} launches; step wall {statistics.mean(walls):.1f} us (min {min(walls):.1f})")
print(f"# {'ms/step':>8s} {'launches':>8s} {'avg us':>9s}  kernel")
for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(d) / len(segs) / 1e3:10.3f} {len(d) / len(segs):8.1f} {statistics.mean(d):9.1f}  {name[33:140] if name.startswith('void m2s') else name[:110]}")
