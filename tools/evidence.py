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


def _base(name):
    return re.sub(r"[<(].*$", "", short(name)).strip()


def dispatch_stages(d):
    """{Dispatch_Id: stage} for a PMC pass directory: its dispatches in order, aligned with the launch sequence
    tools/profile_step.py logged (<d>.launches.json: libm2s's launches with their stage tags) by kernel name; a
    dispatch no launch matches (runtime fills, torch kernels) gets no stage.  Returns (map, steps, matched, n)."""
    log = d.rstrip("/") + ".launches.json"
    if not os.path.exists(log):
        return None, 0, 0, 0
    with open(log) as fh:
        rec = json.load(fh)
    launches = rec["launches"]
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    # the trace also holds the dispatches before the log was switched on (weight packing, the engines' set-up, which
    # can run the same kernels), and the logged steps are the process's last work: walk both sequences from the end
    disp = sorted(names, reverse=True)
    out, j, matched, i = {}, len(launches) - 1, 0, 0
    while i < len(disp) and j >= 0:
        want = _base(launches[j][0])
        # the previous dispatch of this kernel within a short window (fills / copies may sit between launches)
        hit = next((q for q in range(i, min(i + 8, len(disp))) if _base(names[disp[q]]) == want), None)
        if hit is None:  # this launch was not traced as named: skip it
            j -= 1
            continue
        out[disp[hit]] = launches[j][1]
        matched += 1
        i, j = hit + 1, j - 1
    return out, rec["steps"], matched, len(launches)


def stage_counters(d, st_map):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                st = st_map.get(int(r["Dispatch_Id"]))
                if st is not None:
                    agg[st][r["Counter_Name"]] += float(r["Counter_Value"] or 0)
    return agg


def stages(src, sha, prefix, suffix="", workload="headline"):
    """<prefix>_stages.json (suffix "8": <prefix>_c4fp8_stages.json from the fp8 engine's passes at configs[4]'s
    8 x 1000 frames): per stage of the path (libm2s's StageTag labels: cnn, bilstm, mrf_c<C>, ...), HBM bytes per
    step (FETCH_SIZE x2 + WRITE_SIZE, KiB -> bytes), MFMA utilisation and VALU per MFMA."""
    res = collections.defaultdict(dict)
    notes = {}
    for pas in ("fetch", "write", "mfma", "valu"):
        d = os.path.join(src, pas + suffix)
        st_map, steps, matched, n = dispatch_stages(d)
        if st_map is None:
            return None
        notes[pas] = f"{matched} of {n} launches aligned to dispatches over {steps} steps"
        for st, c in stage_counters(d, st_map).items():
            r = res[st]
            if pas == "fetch":
                r["fetch_bytes_per_step"] = 2.0 * c["FETCH_SIZE"] * 1024 / steps
            elif pas == "write":
                r["write_bytes_per_step"] = c["WRITE_SIZE"] * 1024 / steps
            elif pas == "mfma":
                g = c.get("GRBM_GUI_ACTIVE", 0.0)
                r["mfma_util"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * g / 8.0), 4) if g else None
                r["mfma_insts_per_step"] = c.get("SQ_INSTS_MFMA", 0.0) / steps
            else:
                r["valu_insts_per_step"] = c.get("SQ_INSTS_VALU", 0.0) / steps
                lds = c.get("SQ_INSTS_LDS", 0.0)
                r["lds_conflicts_per_lds_inst"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds, 3) if lds else None
    for r in res.values():
        r["hbm_bytes_per_step"] = r.get("fetch_bytes_per_step", 0.0) + r.get("write_bytes_per_step", 0.0)
        mi = r.get("mfma_insts_per_step")
        r["valu_per_mfma"] = round(r.get("valu_insts_per_step", 0.0) / mi, 2) if mi else None
    meta = {"src_sha": sha, "workload": workload,
            "source": f"rocprofv3 --pmc passes in {src} (tools/gpu_evidence.sh, tools/profile_step.py "
            f"{'bench workload' if workload == 'headline' else workload}), dispatches aligned with libm2s's stage-tagged "
            "launch log", "alignment": notes}
    with open(prefix + ("_c4fp8" if suffix else "") + "_stages.json", "w") as fh:
        json.dump({"meta": meta, "stages": res}, fh, indent=1)
    return res


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
    for suffix, wl in (("", "headline"), ("8", "configs4_fp8")):
        st = stages(src, sha, prefix, suffix, wl)
        for k, v in (st or {}).items():
            print(f"{wl} stage {k:10s} hbm {v['hbm_bytes_per_step'] / 1e6:9.1f} MB/step  mfma {v.get('mfma_util')}  "
                  f"valu/mfma {v.get('valu_per_mfma')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
