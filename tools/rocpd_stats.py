"""Kernel statistics from a rocprofv3 run: python tools/rocpd_stats.py <results.db | dir> [out.csv]

rocprofv3 7.x writes a rocpd SQLite database by default; this prints (and optionally writes) the
same per-kernel summary as `--stats` (calls, total/avg/min/max ns, % of kernel time), with kernel
names shortened and the grid size kept so that template variants stay apart.
"""
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name):
    name = name.replace("m2s::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*$", "", name)


def main(src, out=None):
    dbs = [src] if src.endswith(".db") else glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, dur in c.execute("select name, duration from kernels"):
            r = rows.setdefault(short(name), [0, 0, None, 0])
            r[0] += 1
            r[1] += dur
            r[2] = dur if r[2] is None else min(r[2], dur)
            r[3] = max(r[3], dur)
    tot = sum(r[1] for r in rows.values()) or 1
    table = [(k, r[0], r[1], r[1] / r[0], 100.0 * r[1] / tot, r[2], r[3]) for k, r in rows.items()]
    table.sort(key=lambda t: -t[2])
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]
    print(f"{'kernel':70s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'%':>6s}")
    for t in table:
        print(f"{t[0][:70]:70s} {t[1]:6d} {t[2] / 1e6:9.3f} {t[3] / 1e3:9.2f} {t[4]:6.2f}")
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(hdr)
            for t in table:
                w.writerow([t[0], t[1], t[2], round(t[3], 1), round(t[4], 3), t[5], t[6]])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
