#!/usr/bin/env python3
"""Benchmark of the rtMRI -> mel -> 11 413 Hz waveform hot path on MI355X (libm2s).

Metric (BASELINE.json): rtMRI frames/s (and real-time factor) end to end, 256x256 frames.
Workload per GPU (weak scaling): ``--clips`` synthetic clips x ``--frames`` frames (default
64 x 30 = the per-GPU share of configs[3], 512 clips over 8 GPUs), CNN-BiLSTM + head + mel glue
+ HiFi-GAN generator.  One step = one pass of the whole path over the per-GPU batch with frames
already resident in HBM, followed by the RCCL gather of wav + mel to rank 0 (N > 1).  Weights are
random-init of the reference architecture (no checkpoints offline), broadcast from rank 0 over
RCCL once, outside the timing.

Precision.  The reference computes in fp32 (scripts/run_mri_video_inference.py:215-242, no
autocast).  The headline dtype is ``bf16x3``: split fp32, every activation and weight a bf16 pair
hi + lo and every product the three exact bf16 MFMA terms hi*hi + hi*lo + lo*hi accumulated in fp32
(include/m2s.h).  The line carries its measured error against the fp32 CPU oracle on clip 0 of the
same workload (``parity``), next to the fp32 tolerances of tests/test_gpu_configs.py.  At N = 1 a
second, shorter run of the bf16 path (configs[1]'s dtype) is reported under ``bf16`` with its own
error, and one of the fp8 path (configs[4]'s precision: e4m3 MFMA operands) under ``fp8`` with its
error and cosine similarity; neither is the headline.

Launch: ``python bench.py`` (N=1) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N``.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mri-to-speech_amd"))

from m2s import synth  # noqa: E402
from m2s.config import CNN_CHUNK, HIFIGAN_H  # noqa: E402

HOP = 420
SR = 11413
# dense MFMA peaks (MI355X_MICROARCH.md): per ALGORITHMIC flop, so bf16x3 (three bf16 MFMAs per
# product) peaks at a third of the bf16 rate
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3, "bf16x3": 2500.0 / 3,
               # e4m3 on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4: 2x bf16 (MI355X_MICROARCH.md)
               "fp8": 5000.0}
PEAK_HBM_GBS = 8000.0
FP32_TOL = {"mel_norm": 1e-4, "mel_log": 5e-4, "wav": 1e-4}  # tests/test_gpu_configs.py; wav: SURVEY.md §8(c)
# 1000-frame clips: fp32 summation order over 1000 recurrent steps (tests/test_gpu_configs4.py)
LONG_TOL = {"mel_norm": 2e-4, "mel_log": 1e-3, "wav": 1e-4}
PRECISION = {
    "bf16x3": "split fp32: bf16 hi+lo pairs (17-bit), 3 bf16 MFMA terms per product, fp32 accumulate; "
              "BiLSTM recurrence 3-term split products (lstm_x3, B > 4), input projection/head/glue fp32",
    "fp32": "exact f32 MFMA products (v_mfma_f32_16x16x4_f32), fp32 storage",
    "bf16": "bf16 storage and operands, fp32 accumulate; BiLSTM recurrence 3-term split products (B > 4), "
            "input projection/head/glue fp32",
    "fp8": "e4m3 storage + block-scaled e4m3 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4, per-output-channel "
           "weight scales) for the IR blocks' expand (stride 1 and blocks.5.0), expanded maps and SE-gated conv_pwl "
           "GEMMs (all IR blocks), the EdgeResidual blocks.1.1/.2 and blocks.2.1/.2 (conv_exp + conv_pwl) and the "
           "C=128/256 MRF convs; the other convs (stem, stride-2 EdgeResidual blocks.1.0/2.0, blocks.3.0 expand, IR "
           "depthwise on f16 / fp32 accumulation, C=32/64 MRF, upsamplers) bf16; BiLSTM recurrence 3-term split "
           "products (B > 4), input projection/head/glue fp32",
}

MFMA_KERNELS = ("conv_gemm_kernel", "gemm128_kernel", "conv_halo_kernel", "conv1d_halo", "conv_igemm_kernel", "ir_pwdw",
                "ir_ws_kernel", "se_ws_kernel", "lstm_persistent_kernel", "lstm_x3_kernel", "rb1_fused_kernel", "stem_b0_kernel", "se_excite_kernel",
                "er_fused_kernel", "er8_fused_kernel", "er8w_fused_kernel", "er2_fused_kernel", "ers2_fused_kernel", "er_sp_kernel", "ers2_sp_kernel")


def kernel_arith(name: str, dtype: str) -> str:
    """Arithmetic of a kernel in a run of `dtype`: the BiLSTM input projection is f32, its recurrence
    split fp32 (three bf16 terms) in every non-fp32 engine."""
    if name.startswith("lstm_persistent") or name.startswith("lstm_step") or "<float" in name:
        return "fp32"
    if name.startswith("lstm_x3"):  # the split recurrence of every non-fp32 engine
        return "bf16x3"
    if dtype == "fp8":  # only the e4m3 kernels run fp8 MFMA; the rest of an fp8 engine is bf16
        e4m3 = (name.startswith(("gemm128_kernel<0", "gemm128_kernel<1")) or (name.startswith("se_ws_kernel") and "true" in name)
                or (name.startswith("ir_pwdw_kernel<") and name.rstrip(">").endswith(", 3"))  # the e4m3 expand
                or name.startswith(("er8_fused_kernel", "er8w_fused_kernel")))
        return "fp8" if e4m3 else "bf16"
    return dtype


def source_sha() -> str:
    """sha256 (16 hex digits) of the HIP / C++ sources and the C ABI header: the identity of the
    kernels a measurement was taken on (the GPU box gets the tree without .git)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(REPO, "mri-to-speech_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(REPO, "mri-to-speech_amd", "csrc", "*.cpp")) +
                   glob.glob(os.path.join(REPO, "mri-to-speech_amd", "csrc", "*.hpp")) +
                   [os.path.join(REPO, "include", "m2s.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the profiles/*pmc_traffic.json record measured on THIS
    tree (its meta.src_sha equals source_sha(); rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes,
    tools/gpu_evidence.sh + tools/evidence.py).  No record of this tree: no traffic figure."""
    import glob
    sha = source_sha()
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic.json")), reverse=True):
        with open(f) as fh:
            rec = json.load(fh)
        if rec.get("meta", {}).get("src_sha") != sha:
            continue
        k = rec["kernels"].get(kernel)
        if not k:
            return None, os.path.relpath(f, REPO), sha
        return round(k["hbm_bytes_per_launch"]), os.path.relpath(f, REPO), sha
    return None, None, sha


def stage_records(workload="headline"):
    """Per-stage PMC record of THIS tree and workload (profiles/*_stages.json whose meta.src_sha equals source_sha()
    and meta.workload `workload`: "headline" = the 64 x 30 bench step, "configs4_fp8" = the fp8 engine at 8 x 1000;
    made by tools/evidence.py from the rocprofv3 FETCH_SIZE / WRITE_SIZE / SQ passes of tools/profile_step.py, each
    dispatch given the stage libm2s tagged its launch with): HBM bytes per step and MFMA utilisation."""
    import glob
    sha = source_sha()
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_stages.json")), reverse=True):
        with open(f) as fh:
            rec = json.load(fh)
        meta = rec.get("meta", {})
        if meta.get("src_sha") == sha and meta.get("workload", "headline") == workload:
            return rec, os.path.relpath(f, REPO)
    return None, None


# the stages north_star names: the memory-bound BiLSTM and dilated-conv (MRF) stages, the CNN backbone on MFMA
STAGE_ORDER = ("cnn", "bilstm", "head", "glue", "voc_pre", "ups_c256", "mrf_c256", "ups_c128", "mrf_c128", "ups_c64",
               "mrf_c64", "ups_c32", "mrf_c32", "voc_post", "other")


def stage_table(launches, steps, workload="headline"):
    """roofline.stages: per stage of the path, event time per step (the HIP-event pass over the timed region),
    algorithmic bytes / FLOP and their rates, and, from the PMC record of this tree, HBM bytes per step (FETCH x2
    + WRITE), achieved HBM GB/s = those bytes / the event time, its fraction of 8 TB/s, and MFMA utilisation."""
    from m2s import _native
    rec, src = stage_records(workload)
    pmc = (rec or {}).get("stages", {})
    out = {}
    agg = {a["name"]: a for a in _native.aggregate(launches, "stage")}
    for st in sorted(agg, key=lambda k: STAGE_ORDER.index(k) if k in STAGE_ORDER else len(STAGE_ORDER)):
        a = agg[st]
        ms = a["ms"] / steps
        kern = {}
        for r in launches:
            if r["stage"] == st:
                kern[r["name"]] = kern.get(r["name"], 0.0) + r["ms"] / steps
        row = {"ms_per_step": round(ms, 3), "launches_per_step": a["launches"] // steps,
               "algorithmic_GBs": round(a["bytes"] / steps / (ms * 1e-3) / 1e9, 1) if ms > 0 else None,
               "algorithmic_TFLOPs": round(a["flops"] / steps / (ms * 1e-3) / 1e12, 2) if ms > 0 else None,
               "top_kernels": {k: round(v, 3) for k, v in sorted(kern.items(), key=lambda kv: -kv[1])[:3]}}
        p = pmc.get(st)
        if p and ms > 0:
            hb = p["hbm_bytes_per_step"]
            row.update({"pmc_hbm_bytes_per_step": round(hb), "hbm_GBs": round(hb / (ms * 1e-3) / 1e9, 1),
                        "hbm_frac": round(hb / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                        "mfma_util": p.get("mfma_util"), "valu_per_mfma": p.get("valu_per_mfma")})
        out[st] = row
    return {"stages": out, "stages_source": src or f"no *_stages.json of source {source_sha()} and workload {workload} in "
            "profiles/ (tools/gpu_evidence.sh + tools/evidence.py)"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=80)  # ~3.4 s timed at ~42 ms per step
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--clips", type=int, default=64, help="clips per GPU")
    p.add_argument("--frames", type=int, default=30, help="frames per clip")
    p.add_argument("--hw", type=int, default=256)
    p.add_argument("--dtype", default="bf16x3", choices=["bf16x3", "fp32", "bf16", "fp8"])
    p.add_argument("--chunk", type=int, default=CNN_CHUNK,
                   help="frames per CNN pass (default: the engine's shipped m2s.config.CNN_CHUNK = one pass over the 64x30 step)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="C3 sample of the CPU baseline (seconds)")
    p.add_argument("--cpu-long-frames", type=int, default=1000, help="C5 clip length of the CPU baseline (0: skip)")
    p.add_argument("--no-profile", action="store_true")
    p.add_argument("--no-parity", action="store_true", help="skip the oracle check of clip 0")
    p.add_argument("--no-compare", action="store_true", help="skip the secondary bf16 / fp8 lines (N = 1)")
    p.add_argument("--no-caller", action="store_true",
                   help="skip the caller lines (configs[2] one-clip latency with host I/O, the I/O-inclusive step, configs[1])")
    p.add_argument("--no-long", action="store_true", help="skip the configs[4] lines (8 x 1000-frame clips, N = 1)")
    p.add_argument("--ragged", action="store_true",
                   help="clips x gpus clips of 0.8 / 1.0 / 1.2 x --frames frames, sharded by length over the ranks "
                        "(dp.shard_clips), one pipeline call per length group, results gathered to rank 0")
    return p.parse_args(argv)


# M2S_BENCH_FORCE_DIST=1 (under torchrun) takes the RCCL path even at one rank, so the collectives of
# the N-GPU run (broadcast, all-gather, gather, barrier, all-reduce) can be exercised on a 1-GPU box.
FORCE_DIST = os.environ.get("M2S_BENCH_FORCE_DIST") == "1"


def init_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or FORCE_DIST:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def multi(world):
    return world > 1 or FORCE_DIST


def timed_loop(step, k: int, world: int, sync, device) -> float:
    """Barrier + sync on both sides of exactly `k` steps; the max of the ranks' wall times."""
    if multi(world):
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    if multi(world):
        dist.barrier()
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if multi(world):
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item())


def ragged_lengths(n, mean_frames, seed=99):
    """Clip lengths of the ``--ragged`` workload: ``mean_frames`` x {0.8, 1.0, 1.2}, drawn per clip
    (seeded, the same list on every rank): 24 / 30 / 36 frames around configs[3]'s 30."""
    rng = np.random.default_rng(seed)
    choices = [max(1, int(round(mean_frames * f))) for f in (0.8, 1.0, 1.2)]
    return [int(c) for c in rng.choice(choices, size=n)]


class RaggedPlan:
    """The ``--ragged`` step: a global list of ragged clips sharded over the ranks by length
    (``dp.shard_clips``, the same plan on every rank, no communication), each rank's clips ordered by
    length so that every length group is one contiguous block of rows and ONE pipeline call; the
    results of a step land in padded per-rank (clips, max length) buffers that travel to rank 0 in one
    gather each (wav, dB mel) -- the product path of export_predicted_mels.py's torchrun mode."""

    def __init__(self, lens_all, world, rank):
        self.shards = [sorted(s, key=lambda i: (lens_all[i], i)) for s in dp_mod().shard_clips(lens_all, world)]
        self.mine = self.shards[rank]
        self.lens_by_rank = [[lens_all[i] for i in s] for s in self.shards]
        mine_lens = self.lens_by_rank[rank]
        self.tmax = max(mine_lens, default=0)
        self.groups = []  # (length, first row, last row + 1)
        for k, L in enumerate(mine_lens):
            if self.groups and self.groups[-1][0] == L:
                self.groups[-1][2] = k + 1
            else:
                self.groups.append([L, k, k + 1])

    def step(self, forward, frames_by_len, wav, mel, multi_rank):
        for L, r0, r1 in self.groups:
            o = forward(frames_by_len[L])
            wav[r0:r1, : L * HOP].copy_(o["wav"])
            mel[r0:r1, :L].copy_(o["mel_db"])
        if multi_rank:
            return (dp_mod().gather_results(wav, self.lens_by_rank, per_step=HOP),
                    dp_mod().gather_results(mel, self.lens_by_rank, per_step=1))
        return None


def dp_mod():
    from m2s import dp
    return dp


def make_frames(clips, frames, hw, rank, device):
    g = torch.Generator(device=device)
    g.manual_seed(1234 + rank)
    x = torch.rand(clips, frames, hw, hw, generator=g, device=device, dtype=torch.float32)
    lo = x.amin(dim=(2, 3), keepdim=True)
    hi = x.amax(dim=(2, 3), keepdim=True)
    return ((x - lo) / (hi - lo)).contiguous()


def cpu_threads():
    """Threads for the CPU leg: the host cores this process may run on (sched_getaffinity), capped by
    OMP_NUM_THREADS when the box sets one (the GPU box's CPU share)."""
    aff = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(aff, omp) if omp > 0 else aff), aff


def oracle_clip(ac_sd, gen_sd, mean, std, frames_np, cnn_chunk=64):
    sys.path.insert(0, REPO)
    from oracle import pipeline
    t = lambda sd: {k: torch.from_numpy(v) for k, v in sd.items()}  # noqa: E731
    return pipeline.e2e(t(ac_sd), t(gen_sd), HIFIGAN_H, frames_np, mean, std, cnn_chunk=cnn_chunk)


def parity_vs(ref, out, clip=0, tol=None):
    tol = tol or FP32_TOL
    got = {k: out[k][clip:clip + 1].float().cpu().numpy() for k in ("mel_norm", "mel_log", "wav")}
    w, rw = got["wav"].astype(np.float64), ref["wav"].astype(np.float64)
    res = {f"{k}_max_abs": float(np.abs(got[k] - ref[k]).max()) for k in got}
    res["wav_snr_db"] = round(float(10 * np.log10(np.sum(rw ** 2) / max(np.sum((w - rw) ** 2), 1e-30))), 2)
    res["within_fp32_tol"] = all(res[f"{k}_max_abs"] <= t for k, t in tol.items())
    return res


def cosine_vs(ref, out, clip=0):
    """Cosine similarity of mel_norm and wav against the oracle (the fp8 tolerance)."""
    res = {}
    for k in ("mel_norm", "wav"):
        a = out[k][clip:clip + 1].float().cpu().numpy().astype(np.float64).ravel()
        b = ref[k].astype(np.float64).ravel()
        res[f"{k}_cos"] = round(float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30)), 6)
    res["within_cos_0.99"] = all(v >= 0.99 for v in res.values())
    return res


def cpu_baseline(args, ac_sd, gen_sd, mean, std):
    """Oracle (torch-CPU fp32 restatement of the reference graph) on this host's cores, per BASELINE.md's CPU plan:
    C3 (one clip x args.frames end to end) repeated for ~cpu_seconds with per-stage wall time (CNN / BiLSTM / head +
    glue / Generator), C1 (mel only) from the same runs' CNN + BiLSTM + head stages, and C5 (ONE 1000-frame clip end to
    end, the CNN in chunks of args.frames frames, C3's clip: in 100-frame chunks the oracle's CNN ran 3x slower per frame
    on the box's 16-CPU share, 25 vs 8.3 ms).  `value` is the C3 end-to-end rate (the headline's workload per clip)."""
    sys.path.insert(0, REPO)
    from oracle import acoustic, effnet, hifigan

    threads, aff = cpu_threads()
    torch.set_num_threads(threads)
    sd = {k: torch.from_numpy(v) for k, v in ac_sd.items()}
    gsd = {k: torch.from_numpy(v) for k, v in gen_sd.items()}

    def clip(frames, T, acc, chunk=100):
        t0 = time.perf_counter()
        f = torch.cat([effnet.effnet_gap(sd, frames.reshape(T, args.hw, args.hw)[i:i + chunk])
                       for i in range(0, T, chunk)]).view(1, T, -1)
        t1 = time.perf_counter()
        h = acoustic.bilstm_summerge(sd, f)
        t2 = time.perf_counter()
        mn = acoustic.head(sd, h)
        ln = acoustic.mel_db_to_log(acoustic.denormalize_mel(mn[0], mean, std))
        t3 = time.perf_counter()
        hifigan.generator(gsd, HIFIGAN_H, ln.t().unsqueeze(0))
        t4 = time.perf_counter()
        for k, v in zip(("cnn", "bilstm", "head_glue", "generator"), (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            acc[k] = acc.get(k, 0.0) + v
        return t4 - t0

    T = args.frames
    frames = torch.from_numpy(synth.synth_frames(1, T, hw=(args.hw, args.hw), seed=77))
    st3, done, el = {}, 0, 0.0
    with torch.no_grad():
        while el < args.cpu_seconds and done < 50:
            el += clip(frames, T, st3)
            done += 1
    audio3 = T * HOP / SR
    mel_s = st3["cnn"] + st3["bilstm"] + st3["head_glue"]
    per = {"C1": {"what": f"1 clip x {T} frames -> mel (CNN-BiLSTM + head), from the C3 runs' stages",
                  "frames_per_s": round(done * T / mel_s, 3)},
           "C3": {"what": f"1 clip x {T} frames end to end", "clips": done, "frames_per_s": round(done * T / el, 3),
                  "rtf": round(el / done / audio3, 4),
                  "stage_ms_per_clip": {k: round(1e3 * v / done, 2) for k, v in st3.items()}}}
    if args.cpu_long_frames > 0:  # C5: one long clip, end to end
        TL = args.cpu_long_frames
        fl = torch.from_numpy(synth.synth_frames(1, TL, hw=(args.hw, args.hw), seed=78))
        st5 = {}
        with torch.no_grad():
            e5 = clip(fl, TL, st5, chunk=T)
        per["C5"] = {"what": f"1 clip x {TL} frames end to end (CNN in {T}-frame chunks)", "frames_per_s": round(TL / e5, 3),
                     "rtf": round(e5 / (TL * HOP / SR), 4), "stage_ms": {k: round(1e3 * v, 1) for k, v in st5.items()}}
    return {"value": round(done * T / el, 3), "unit": "rtMRI frames/s", "cores": threads, "affinity_cpus": aff,
            "kind": "port",
            "sample": f"C3: {done} clip(s) x {T} frames at {args.hw}x{args.hw}, end to end (CNN-BiLSTM + glue + HiFi-GAN), "
                      f"fp32 oracle (torch-CPU restatement of the reference graph), {el:.1f} s; C5: one "
                      f"{args.cpu_long_frames}-frame clip; {threads} threads",
            "threads_note": (f"{threads} threads = min(sched_getaffinity {aff}, OMP_NUM_THREADS): the GPU box grants one "
                             "GPU's job a 16-CPU share (OMP_NUM_THREADS=16 there) although the affinity mask shows the "
                             "whole host"),
            "per_config": per}


def long_clip_lines(args, build, device, sync, world, ref_args, clips=8, frames=1000, steps=3):
    """configs[4]'s shape on this GPU: 8 clips x 1000 frames (its per-GPU share of >= 1000-frame clips),
    end to end, in fp8 (its precision: e4m3 backbone / MRF convs), bf16x3 and bf16, with the fp8 run's
    dominant-kernel roofline from the HIP-event pass.  Frames resident in HBM, same timing rules as the
    headline; a secondary line, not the headline."""
    from m2s import _native
    x = make_frames(clips, frames, args.hw, 0, device)
    res = {"workload": f"e2e rtMRI->wav, {clips} clips x {frames} frames at {args.hw}x{args.hw} (configs[4] per-GPU)"}
    ref0 = None
    if not args.no_parity:  # clip 0 of this batch through the fp32 oracle, outside every timed loop
        torch.set_num_threads(cpu_threads()[0])
        ref0 = oracle_clip(*ref_args, x[:1].cpu().numpy(), cnn_chunk=100)
    for dt in ("fp8", "bf16x3", "bf16"):
        p = build(dt)
        out = p.forward(x)
        el = timed_loop(lambda: p.forward(x), steps, world, sync, device)
        p.ac.check()
        line = {"value": round(clips * frames * steps / el, 2), "ms_per_step": round(1000.0 * el / steps, 2),
                "rtf": round(el / (clips * frames * steps * HOP / SR), 6), "steps": steps}
        if ref0 is not None:  # the warm-up call's outputs (same inputs, same engine as the timed steps)
            par = dict(parity_vs(ref0, out, tol=LONG_TOL), **cosine_vs(ref0, out), clip=0, reference="fp32 CPU oracle")
            # within_tol against the tolerance this dtype is held to: the fp32 bars (1000-frame clips) for bf16x3,
            # cosine >= 0.99 for the narrower dtypes; within_fp32_tol only where that is the bar
            within = par.pop("within_fp32_tol")
            par["tolerance"] = LONG_TOL if dt == "bf16x3" else "cosine >= 0.99"
            par["within_tol"] = within if dt == "bf16x3" else par["within_cos_0.99"]
            if dt == "bf16x3":
                par["within_fp32_tol"] = within
            line["parity"] = par
        del out
        if dt == "fp8":
            _native.prof_enable(True)
            timed_loop(lambda: p.forward(x), steps, world, sync, device)
            _native.prof_enable(False)
            line["roofline"] = roofline(_native.prof_launches(), dt, steps, line["value"], clips * frames, stages=True,
                                        stage_workload="configs4_fp8")
        res[dt] = line
        del p
    res["fp8_over_bf16x3_step"] = round(res["fp8"]["ms_per_step"] / res["bf16x3"]["ms_per_step"], 3)
    del x
    return res


def host_frames_u8(clips, frames, hw, seed):
    """Decoded grey frames as the caller holds them before preprocessing: (clips, frames, hw, hw) uint8 in
    pinned host memory (FrameStream's staging buffers, scripts/run_mri_video_inference.py)."""
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.integers(0, 256, size=(clips, frames, hw, hw), dtype=np.uint8)).pin_memory()


def caller_lines(args, pipe, build, device, sync, world, ref_args, runs=60):
    """What a user of scripts/run_mri_video_inference.py experiences (reference :215-242: frames to the device,
    the no_grad forward, mel / wav back to the host), on this GPU:

    * ``configs2``: ONE 30-frame clip, decoded uint8 frames in pinned host memory -> H2D -> the device
      preprocessing (``preprocess_frames``, _preprocess_frame :34-54) -> ``pipeline_forward`` -> D2H of the wav,
      dB mel and ln mel -> host sync; latency percentiles over ``runs`` runs (each run timed alone, the engine
      warm), RTF = latency / audio seconds.
    * ``io``: the headline's 64 x 30 step with the same host legs, double-buffered as FrameStream does: the
      H2D of step k + 1's uint8 frames on a copy stream and the D2H of step k's results on another while step k
      computes; frames/s over the timed steps.
    * ``configs1``: BASELINE configs[1], the CNN-BiLSTM forward (acoustic model only, no vocoder), 8 clips x 4
      frames, bf16; frames/s and ms per call with frames resident on the device."""
    from m2s import runtime
    HW = args.hw
    res = {}
    # ---- configs[2]: one clip, host in -> host out -------------------------------------------------------
    T2 = 30
    hf = host_frames_u8(1, T2, HW, seed=2024)

    def one_clip():
        x8 = hf.to(device, non_blocking=True)
        x = runtime.preprocess_frames(x8.view(T2, HW, HW)).view(1, T2, HW, HW)
        o = pipe.forward(x)
        host = {k: o[k].to("cpu", non_blocking=True) for k in ("wav", "mel_db", "mel_log")}
        torch.cuda.synchronize(device)
        return host, o, x
    for _ in range(5):
        one_clip()
    lat = []
    for _ in range(runs):
        t0 = time.perf_counter()
        one_clip()
        lat.append(time.perf_counter() - t0)
    pipe.ac.check()
    lat_ms = np.sort(np.array(lat) * 1e3)
    audio_s = T2 * HOP / SR
    line = {"workload": f"1 clip x {T2} frames at {HW}x{HW}: pinned uint8 host frames -> H2D -> preprocess_frames -> "
                        "pipeline_forward (CNN-BiLSTM + glue + HiFi-GAN) -> D2H wav + dB mel + ln mel -> sync",
            "dtype": args.dtype, "runs": runs, "p50_ms": round(float(np.percentile(lat_ms, 50)), 3),
            "p90_ms": round(float(np.percentile(lat_ms, 90)), 3), "min_ms": round(float(lat_ms[0]), 3),
            "mean_ms": round(float(lat_ms.mean()), 3),
            "rtf_p50": round(float(np.percentile(lat_ms, 50)) / 1e3 / audio_s, 5), "audio_s": round(audio_s, 4),
            "frames_per_s_p50": round(T2 / (float(np.percentile(lat_ms, 50)) / 1e3), 1)}
    if not args.no_parity:  # the oracle on the frames the device preprocessing produced
        host, o, x = one_clip()
        ref = oracle_clip(*ref_args, x.cpu().numpy())
        par = parity_vs(ref, o)
        par["mel_db_host_max_abs"] = float(np.abs(host["mel_db"].numpy() - ref["mel_db"]).max())
        line["parity"] = dict(par, clip=0, tolerance=FP32_TOL, reference="fp32 CPU oracle on the device-preprocessed frames")
    res["configs2"] = line
    # ---- the headline step with the host legs, double-buffered -------------------------------------------
    B, T = args.clips, args.frames
    steps = max(5, args.steps // 4)
    h_in = [host_frames_u8(B, T, HW, seed=11), host_frames_u8(B, T, HW, seed=12)]
    d_in = [torch.empty(B, T, HW, HW, dtype=torch.uint8, device=device) for _ in range(2)]
    h_wav = [torch.empty(B, T * HOP, dtype=torch.float32).pin_memory() for _ in range(2)]
    h_mel = [torch.empty(B, T, 64, dtype=torch.float32).pin_memory() for _ in range(2)]
    cp_in, cp_out = torch.cuda.Stream(device), torch.cuda.Stream(device)
    comp = torch.cuda.current_stream(device)
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_free = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]
    state = {"k": 0}

    def prime():
        with torch.cuda.stream(cp_in):
            d_in[0].copy_(h_in[0], non_blocking=True)
            ev_in[0].record(cp_in)
            ev_free[1].record(cp_in)

    def io_step():
        k = state["k"]
        a, b = k & 1, (k + 1) & 1
        with torch.cuda.stream(cp_in):  # step k + 1's frames cross PCIe while step k computes
            cp_in.wait_event(ev_free[b])
            d_in[b].copy_(h_in[b], non_blocking=True)
            ev_in[b].record(cp_in)
        comp.wait_event(ev_in[a])
        x = runtime.preprocess_frames(d_in[a].view(B * T, HW, HW)).view(B, T, HW, HW)
        ev_free[a].record(comp)
        o = pipe.forward(x)
        ev_out[a].record(comp)
        with torch.cuda.stream(cp_out):  # step k's results back to the host behind the compute stream
            cp_out.wait_event(ev_out[a])
            h_wav[a].copy_(o["wav"], non_blocking=True)
            h_mel[a].copy_(o["mel_db"], non_blocking=True)
            o["wav"].record_stream(cp_out)
            o["mel_db"].record_stream(cp_out)
        state["k"] = k + 1
    prime()
    for _ in range(2):
        io_step()
    el = timed_loop(io_step, steps, world, sync, device)
    pipe.ac.check()
    res["io"] = {"workload": f"{B} clips x {T} frames at {HW}x{HW} per step: pinned uint8 host frames -> H2D (copy stream, "
                             "one step ahead) -> preprocess_frames -> pipeline_forward -> D2H wav + dB mel (second copy "
                             "stream) -- the headline step with the caller's host legs",
                 "dtype": args.dtype, "value": round(B * T * steps / el, 2), "unit": "rtMRI frames/s",
                 "ms_per_step": round(1000.0 * el / steps, 3), "steps": steps,
                 "h2d_bytes_per_step": B * T * HW * HW, "d2h_bytes_per_step": B * T * (HOP + 64) * 4,
                 "rtf": round(el / (B * T * steps * HOP / SR), 6)}
    del d_in, h_in, h_wav, h_mel
    # ---- configs[1]: CNN-BiLSTM forward, 8 x 4 frames, bf16 ----------------------------------------------
    ac = runtime.AcousticEngine(ref_args[0], dtype="bf16", device=device)
    x1 = make_frames(8, 4, HW, 5, device)
    for _ in range(5):
        mn = ac.forward(x1)
    k1 = 100
    el = timed_loop(lambda: ac.forward(x1), k1, world, sync, device)
    ac.check()
    line = {"workload": f"CNN-BiLSTM forward (acoustic model, no vocoder), 8 clips x 4 frames at {HW}x{HW}, frames resident "
                        "(BASELINE configs[1])", "dtype": "bf16", "value": round(8 * 4 * k1 / el, 2),
            "unit": "rtMRI frames/s", "ms_per_call": round(1000.0 * el / k1, 3), "calls": k1}
    if not args.no_parity:
        sys.path.insert(0, REPO)
        from oracle import pipeline
        sd = {k: torch.from_numpy(v) for k, v in ref_args[0].items()}
        ref = pipeline.acoustic_forward(sd, x1[:1].cpu().numpy()).numpy()
        got = mn[:1].float().cpu().numpy()
        a, b = got.ravel().astype(np.float64), ref.ravel().astype(np.float64)
        cos = float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))
        line["parity"] = {"mel_norm_max_abs": float(np.abs(got - ref).max()), "mel_norm_cos": round(cos, 6),
                          "within_tol": cos >= 0.99, "tolerance": "cosine >= 0.99 (bf16)", "clip": 0,
                          "reference": "fp32 CPU oracle"}
    res["configs1"] = line
    del ac
    return res


def roofline(launches, dtype, steps, fps, frames_per_step, stages=False, stage_workload="headline"):
    from m2s import _native
    stats = _native.aggregate(launches, "name")
    tot_ms = sum(s["ms"] for s in stats)
    dom = max(stats, key=lambda s: s["ms"])
    ar = kernel_arith(dom["name"], dtype)
    peak_tf = PEAK_TFLOPS[ar]
    ridge = peak_tf * 1e12 / (PEAK_HBM_GBS * 1e9)  # bound = the roof its algorithmic intensity hits first
    if dom["bytes"] <= 0 or dom["flops"] / dom["bytes"] > ridge:
        achieved = dom["flops"] / (dom["ms"] * 1e-3) / 1e12
        peak, unit, bound = peak_tf, "TFLOP/s", "mfma"
    else:
        achieved = dom["bytes"] / (dom["ms"] * 1e-3) / 1e9
        peak, unit, bound = PEAK_HBM_GBS, "GB/s", "hbm"
    mm = [s for s in stats if s["name"].startswith(MFMA_KERNELS)]
    mm_ms, mm_fl = sum(s["ms"] for s in mm), sum(s["flops"] for s in mm)
    flop_per_frame = sum(s["flops"] for s in stats) / (steps * frames_per_step)
    traffic, tsrc, sha = pmc_traffic(dom["name"])
    r = {
        "bound": bound, "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": unit,
        "frac": round(achieved / peak, 4), "traffic": traffic,
        "kernel": dom["name"], "arith": ar, "launches_per_step": dom["launches"] // steps,
        "avg_launch_us": round(1000.0 * dom["ms"] / dom["launches"], 2),
        "algorithmic_bytes_per_launch": round(dom["bytes"] / dom["launches"]),
        # an intermediate the kernel writes only for the next kernel of the same operation to read back (ir_ws: the
        # IR block's expanded depthwise map, read by the SE-gated conv_pwl; include/m2s.h spill_bytes): HBM traffic
        # the PMC record sees, not compulsory bytes, so not in `achieved` nor in the roof choice
        "spill_bytes_per_launch": round(dom.get("spill_bytes", 0.0) / dom["launches"]),
        "algorithmic_flop_per_launch": round(dom["flops"] / dom["launches"]),
        "kernel_share_of_gpu_time": round(dom["ms"] / tot_ms, 3),
        "all_mfma_kernels_tflops": round(mm_fl / (mm_ms * 1e-3) / 1e12, 2),
        "plan_gflop_per_frame": round(flop_per_frame / 1e9, 4),
        "e2e_tflops": round(flop_per_frame * fps / 1e12, 2),
        "e2e_frac_of_peak": round(flop_per_frame * fps / 1e12 / PEAK_TFLOPS[dtype], 4),
    }
    r["traffic_source"] = tsrc or f"no PMC record of source {sha} in profiles/ (tools/gpu_evidence.sh)"
    r["src_sha"] = sha
    r["bytes_note"] = ("algorithmic bytes on the real channel counts (compulsory: the operation's input + output + weights, "
                       "4 B an element in split fp32), not the padded channel strides of the layout; spilled intermediates "
                       "are spill_bytes_per_launch; bound = the roof the algorithmic intensity (flop / compulsory byte) meets "
                       "first")
    if traffic:
        r["traffic_over_compulsory_plus_spill"] = round(traffic / max(r["algorithmic_bytes_per_launch"] + r["spill_bytes_per_launch"], 1), 3)
    if stages:
        r.update(stage_table(launches, steps, stage_workload))
    return r


def main():
    args = parse()
    world, rank, local = init_dist()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    from m2s import _native, dp, runtime

    # weights: rank 0's state dicts reach every rank over RCCL (C1); every rank packs its own copy.
    # (Other ranks start from a differently seeded state so the broadcast is what makes them equal.)
    ac_sd = synth.synth_acoustic_state(0 if rank == 0 else 1000 + rank)
    gen_sd = synth.synth_generator_state(0 if rank == 0 else 1000 + rank)
    ac_sd = dp.broadcast_state(ac_sd, device)
    gen_sd = dp.broadcast_state(gen_sd, device)
    mean, std = synth.synth_scaler()

    def build(dtype):
        ac = runtime.AcousticEngine(ac_sd, dtype=dtype, device=device, chunk=args.chunk)
        voc = runtime.VocoderEngine(gen_sd, HIFIGAN_H, dtype=dtype, device=device)
        return runtime.Pipeline(ac, voc, mean, std)

    pipe = build(args.dtype)
    B, T, HW = args.clips, args.frames, args.hw
    out = {}
    if args.ragged:  # ragged clip list sharded by length; one pipeline call per length group
        lens_all = ragged_lengths(B * world, T)
        plan = RaggedPlan(lens_all, world, rank)
        fr_by_len = {L: make_frames(r1 - r0, L, HW, rank * 1000 + L, device) for L, r0, r1 in plan.groups}
        wav_buf = torch.zeros(len(plan.mine), plan.tmax * HOP, device=device)
        mel_buf = torch.zeros(len(plan.mine), plan.tmax, 64, device=device)
        frames = fr_by_len[plan.groups[0][0]] if plan.groups else make_frames(1, T, HW, rank, device)
        frames_per_step = sum(lens_all)
        local_frames = sum(plan.lens_by_rank[rank])
        args.no_compare = args.no_long = True

        def step(p=None):
            plan.step((p or pipe).forward, fr_by_len, wav_buf, mel_buf, multi(world))
    else:
        frames = make_frames(B, T, HW, rank, device)
        frames_per_step = world * B * T
        local_frames = B * T
        if multi(world):  # C3: clip lengths of every rank (the gather is sized from them)
            all_lens = dp.all_gather_lengths([T] * B, device)

        def step(p=None):
            out.update((p or pipe).forward(frames))  # torch.ops.m2s.pipeline_forward on the current stream
            if multi(world):  # C2: wav + dB mel of every clip to rank 0 over RCCL
                dp.gather_results(out["wav"], all_lens, per_step=HOP)
                dp.gather_results(out["mel_db"], all_lens, per_step=1)

    sync = lambda: torch.cuda.synchronize(device)  # noqa: E731
    for _ in range(args.warmup):
        step()
    elapsed = timed_loop(step, args.steps, world, sync, device)
    pipe.ac.check()  # a BiLSTM hand-off timeout in the timed steps raises here (m2s_acoustic_status)
    frames_total = frames_per_step * args.steps
    fps = frames_total / elapsed
    audio_s = frames_total * HOP / SR
    result = {
        "metric": "rtMRI frames/s end-to-end (256x256 frames -> 64-bin mel -> 11413 Hz wav)",
        "value": round(fps, 2),
        "unit": "rtMRI frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "precision": PRECISION[args.dtype],
        "data": "synthetic (seeded U[0,1) frames, per-frame min-max; random-init weights of the reference architecture)",
        "rtf": round(elapsed / audio_s, 6),
        "config": {"workload": (f"e2e rtMRI->wav, {B * world} ragged clips of {sorted(set(lens_all))} frames "
                                f"(mean {frames_per_step / (B * world):.1f}) sharded by length over {world} GPU(s) "
                                f"at {HW}x{HW}") if args.ragged else
                               (f"e2e rtMRI->wav, {B} clips x {T} frames per GPU at {HW}x{HW} " +
                                ("(configs[4] clip length)" if T >= 1000 else "(configs[3] per-GPU share)")),
                   "clips_per_gpu": B, "frames_per_clip": T, "global_batch_clips": B * world, "hw": HW,
                   "parallelism": f"dp{world}", "chunk": args.chunk},
    }

    # roofline: a second pass identical to the timed region with HIP events around every launch
    if not args.no_profile:
        _native.prof_enable(True)
        timed_loop(step, args.steps, world, sync, device)
        _native.prof_enable(False)
        launches = _native.prof_launches()
        result["roofline"] = roofline(launches, args.dtype, args.steps, fps, local_frames, stages=True)
        if rank == 0 and os.environ.get("M2S_BENCH_KERNELS"):
            for s in sorted(_native.aggregate(launches), key=lambda s: -s["ms"]):
                print(f"# {s['name']:40s} n={s['launches']:6d} ms={s['ms']:9.3f} "
                      f"TF/s={s['flops'] / max(s['ms'], 1e-9) / 1e9:8.2f} GB/s={s['bytes'] / max(s['ms'], 1e-9) / 1e6:8.1f}",
                      file=sys.stderr)

    ref0 = None
    if rank == 0 and not args.no_parity:  # clip 0 of this rank's workload through the fp32 oracle
        if args.ragged:  # clip 0 of the first length group
            out.update(pipe.forward(frames))
        ref0 = oracle_clip(ac_sd, gen_sd, mean, std, frames[:1].cpu().numpy())
        result["parity"] = dict(parity_vs(ref0, out), clip=0, tolerance=FP32_TOL, reference="fp32 CPU oracle")
    if world == 1 and not args.ragged and not args.no_caller:  # the caller's view: host I/O, one-clip latency, configs[1]
        result["caller"] = caller_lines(args, pipe, build, device, sync, world, (ac_sd, gen_sd, mean, std))
    if world == 1 and not args.no_compare:  # secondary lines: the narrower dtypes on the same workload
        del pipe
        for dt in ("bf16", "fp8", "fp32"):
            if dt == args.dtype:
                continue
            p2 = build(dt)
            for _ in range(args.warmup):
                step(p2)
            k = 5 if dt == "fp32" else max(5, args.steps // 2)  # exact f32: ~0.2 s per step
            el = timed_loop(lambda: step(p2), k, world, sync, device)
            result[dt] = {"value": round(B * T * k / el, 2), "ms_per_step": round(1000.0 * el / k, 3), "steps": k,
                          "precision": PRECISION[dt]}
            if ref0 is not None:
                par = dict(parity_vs(ref0, out), **cosine_vs(ref0, out))
                within = par.pop("within_fp32_tol")
                par["tolerance"] = FP32_TOL if dt == "fp32" else "cosine >= 0.99"
                par["within_tol"] = within if dt == "fp32" else par["within_cos_0.99"]
                result[dt]["parity"] = par
            del p2
    if world == 1 and not args.no_long and not (args.clips == 8 and args.frames == 1000):
        result["configs4"] = long_clip_lines(args, build, device, sync, world, (ac_sd, gen_sd, mean, std))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, ac_sd, gen_sd, mean, std)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if multi(world):
        dist.barrier()
        dist.destroy_process_group()
    # release the engines' device memory while the HIP runtime is still up
    del frames, out
    torch.cuda.synchronize(device)


if __name__ == "__main__":
    main()
