"""Aggregate rocprofv3 --pmc CSVs per kernel family: python tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ...

Prints, per kernel symbol, the summed counter values (and the dispatch count).  FETCH_SIZE /
WRITE_SIZE are kB; on gfx950 FETCH_SIZE under-counts a wide coalesced stream by 2x
(MI355X_MICROARCH.md §HBM) - the 'fetch_x2_MB' column applies that correction.
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = name.replace("m2s::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)          # drop argument list
    return name[:110]


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        for r in load(d):
            k = short(r.get("Kernel_Name", r.get("Kernel-Name", "?")))
            c = r.get("Counter_Name", r.get("Counter-Name"))
            v = float(r.get("Counter_Value", r.get("Counter-Value", 0)) or 0)
            agg[k][c] += v
            disp[k].add((d, r.get("Dispatch_Id", r.get("Dispatch-Id"))))
    keys = sorted({c for v in agg.values() for c in v})
    for k in sorted(agg, key=lambda k: -agg[k].get("GRBM_GUI_ACTIVE", agg[k].get("FETCH_SIZE", 0))):
        v = agg[k]
        extra = ""
        if "FETCH_SIZE" in v:
            extra += f" fetch_x2_MB={2 * v['FETCH_SIZE'] / 1024:.1f}"
        if "WRITE_SIZE" in v:
            extra += f" write_MB={v['WRITE_SIZE'] / 1024:.1f}"
        if v.get("SQ_BUSY_CYCLES"):
            extra += f" mfma_busy/busy={v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / v['SQ_BUSY_CYCLES']:.3f}"
        print(f"{k}  n={len(disp[k])}{extra}")
        print("    " + "  ".join(f"{c}={v[c]:.4g}" for c in keys if c in v))


if __name__ == "__main__":
    main(sys.argv[1:])
