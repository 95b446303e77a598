"""Per-call kernel timeline from a rocprofv3 kernel trace of tools/profile_small.py: the calls are cut at the
marker kernels (torch's exp_), and the median call is printed launch by launch (start offset, duration, idle gap
before it), then the kernel time summed per name over all calls.  Usage:
  python3 tools/small_timeline.py run_kernel_trace.csv"""
import csv
import statistics
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("m2s::(anonymous namespace)::", "")
    return n[:100]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "exp_kernel" in r["Kernel_Name"]]
# the marker launches of the timed calls (calls + 1 of them; the warm-up calls launch none)
segs = list(zip(marks, marks[1:]))
if not segs:
    sys.exit("no marker kernels in the trace")
walls, busy = [], []
per = defaultdict(list)
for a, b in segs:
    ks = rows[a + 1:b]
    if not ks:
        continue
    t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    walls.append((t1 - t0) / 1e3)
    busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks) / 1e3)
    for r in ks:
        per[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
n = len(walls)
med = sorted(range(n), key=lambda i: walls[i])[n // 2]
print(f"# {n} calls; GPU span first launch -> last end: median {statistics.median(walls):.1f} us, "
      f"kernel busy {statistics.median(busy):.1f} us, launches per call {b - a - 1}")
a, b = segs[med]
ks = rows[a + 1:b]
t0 = int(ks[0]["Start_Timestamp"])
prev = t0
print(f"# median call: {walls[med]:.1f} us span")
print(f"{'start_us':>9s} {'dur_us':>8s} {'gap_us':>7s} {'grid':>14s}  kernel")
for r in ks:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    grid = f"{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
    wg = r.get("Workgroup_Size_X", "")
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev) / 1e3:7.1f} {grid:>14s} {wg:>4s}  {short(r['Kernel_Name'])}")
    prev = max(prev, e)
print("# kernel time per call, summed by name")
for k, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(d) / n:9.1f} us {len(d) / n:5.1f}x  {k}")
