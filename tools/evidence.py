"""Post-process a tools/gpu_evidence.sh run into committed profiles/ records.

    python tools/evidence.py gpurun_out/<tag> profiles/<tag>

writes <prefix>_pmc_traffic.json (per-kernel HBM bytes per launch, keyed by the source hash of the
tree it was measured on, which bench.py matches), <prefix>_rocprof_kernel_stats.csv (rocprofv3
--stats of the bench run), and <prefix>_sq_mfma.txt: per kernel family the MFMA utilisation
    util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs, so / 8 = the dispatch's cycles; SQ_VALU_MFMA_BUSY_CYCLES
sums every SIMD's matrix-pipe busy cycles, MI355X_MICROARCH.md cycle-constants notes), with the
busy cycles per MFMA instruction as a check (16 for 16x16x32 bf16 / fp8, 32 for 16x16x4 f32), the
VALU instructions per MFMA and the LDS bank-conflict cycles per LDS instruction.
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from pmc_traffic import per_kernel, short  # noqa: E402


def counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"] or 0)
                disp[k].add(r["Dispatch_Id"])
    return agg, {k: len(v) for k, v in disp.items()}


def main(src, prefix):
    sha = open(os.path.join(src, "src_sha.txt")).read().strip()
    fe, wr = per_kernel(os.path.join(src, "fetch"), "FETCH_SIZE"), per_kernel(os.path.join(src, "write"), "WRITE_SIZE")
    if os.path.isdir(os.path.join(src, "fetch8")):  # the fp8 engine's passes (8 x 1000 frames): its own kernels
        for d, tgt, cn in (("fetch8", fe, "FETCH_SIZE"), ("write8", wr, "WRITE_SIZE")):
            for k, v in per_kernel(os.path.join(src, d), cn).items():
                tgt.setdefault(k, v)
    kern = {}
    for k in sorted(set(fe) | set(wr)):
        f_kib, nf = fe.get(k, (0.0, 0))
        w_kib, nw = wr.get(k, (0.0, 0))
        fb = 2.0 * f_kib * 1024 / nf if nf else None
        wb = w_kib * 1024 / nw if nw else None
        kern[k] = {"launches": max(nf, nw), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                   "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    meta = {"src_sha": sha, "source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes ({src}), "
            "tools/profile_step.py bench workload; FETCH_SIZE x2 (gfx950 correction), KiB -> bytes"}
    with open(prefix + "_pmc_traffic.json", "w") as fh:
        json.dump({"meta": meta, "kernels": kern}, fh, indent=1)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], prefix + "_rocprof_kernel_stats.csv")
    mf, nd = counters(os.path.join(src, "mfma"))
    va, _ = counters(os.path.join(src, "valu"))
    lines = [f"# src_sha {sha}; {src}; MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)",
             f"{'kernel':72s} {'n':>5s} {'util':>6s} {'cyc/mfma':>8s} {'valu/mfma':>9s} {'ldsconf/lds':>11s} "
             f"{'fetch MB':>9s} {'write MB':>9s}"]
    rows = []
    for k, v in mf.items():
        g = v.get("GRBM_GUI_ACTIVE", 0.0)
        util = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * g / 8.0) if g else 0.0
        mi = v.get("SQ_INSTS_MFMA", 0.0)
        cpm = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / mi if mi else 0.0
        w = va.get(k, {})
        vpm = w.get("SQ_INSTS_VALU", 0.0) / mi if mi else 0.0
        lds = w.get("SQ_INSTS_LDS", 0.0)
        lc = w.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else 0.0
        t = kern.get(k, {})
        rows.append((g, f"{k[:72]:72s} {nd.get(k, 0):5d} {util:6.3f} {cpm:8.1f} {vpm:9.1f} {lc:11.3f} "
                        f"{(t.get('fetch_bytes_per_launch') or 0) / 1e6:9.1f} {(t.get('write_bytes_per_launch') or 0) / 1e6:9.1f}"))
    lines += [r for _, r in sorted(rows, key=lambda x: -x[0])]
    with open(prefix + "_sq_mfma.txt", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
