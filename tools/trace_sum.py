"""Per-kernel time per Pipeline.forward from a rocprofv3 kernel trace of tools/ab_step.py --child: every
launch of the process summed and divided by the number of forward calls (argv[2]; all calls are the same
workload).  Usage: python3 tools/trace_sum.py run_kernel_trace.csv CALLS"""
import csv
import sys
from collections import defaultdict

calls = int(sys.argv[2])
tot, cnt = defaultdict(float), defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("void ", "").replace("m2s::(anonymous namespace)::", "")[:90]
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cnt[k] += 1
print(f"# {sys.argv[1]}: kernel ms per forward (sum {sum(tot.values()) / calls:.3f} ms)")
for k in sorted(tot, key=tot.get, reverse=True):
    if tot[k] / calls >= 0.01:
        print(f"{tot[k] / calls:9.3f} {cnt[k] / calls:7.1f}  {k}")
