"""Print per-step kernel times from a rocprofv3 --stats CSV: python tools/kstats.py DIR [steps] [filter]"""
import csv
import glob
import sys

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
flt = sys.argv[3] if len(sys.argv) > 3 else ""
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.3f} ms/step")
for r in rows:
    n = r["Name"].replace("void ", "").replace("m2s::(anonymous namespace)::", "")
    if flt and flt not in n:
        continue
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:5.1f}x {float(r['AverageNs']) / 1e3:9.1f}us  {n[:80]}")
