"""Predicted ln-mel export for HiFi-GAN fine-tuning on MI355X (drop-in for
scripts/export_predicted_mels.py).

Contract kept from the reference (export_predicted_mels.py:102-118 flags, :43-99 behaviour): reads
``{processed_dir}/samples/*/mri.npy`` ((T,H,W) float32 frames already /255,
preprocess_rtmri_data.py:113), writes one ``{output_dir}/{sample}.npy`` ln-mel of shape (n_mels, T)
float32 per sample (meldataset.py:195-218 consumes them), skips existing outputs unless
``--overwrite``, loads the model through the plug-in surface (``--mri_code_dir``,
``build_acoustic_model``, ``model_state_dict`` or a raw state dict, strict=False) and sizes n_mels
from ``--scaler_json``.

How it runs: the sample list is read first, clips with the same frame-stack shape go through the
acoustic model together (``--batch`` per call, m2s/drivers.py), and the de-normalisation
y*std+mean -> 10^(x/10) -> clamp(1e-5) -> ln runs on the device (``torch.ops.m2s.mel_glue``) before
the one copy back.  ``--cpu`` is refused: there is no CPU path.

Several GPUs (one process per GPU): ``python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 scripts/export_predicted_mels.py ...``.  Every rank lists the samples and reads
their frame counts from the .npy headers; the ragged clips are sharded by length (``dp.shard_clips``:
longest first onto the least-loaded rank); rank 0 loads the checkpoint and its state dict reaches the
other ranks in ONE broadcast (``dp.broadcast_state``); each rank reads and runs only its own clips;
the ln-mels are gathered to rank 0 in one padded gather (``drivers.run_sharded``) and rank 0 writes
every file.  Backend: RCCL ("nccl") over xGMI, or ``M2S_DIST_BACKEND=gloo``.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

PROJECT_ROOT = Path(__file__).resolve().parents[1]
if str(PROJECT_ROOT) not in sys.path:
    sys.path.insert(0, str(PROJECT_ROOT))

from m2s import drivers  # noqa: E402
from m2s.runtime import mel_glue  # noqa: E402


def scaler_arrays(path: Path):
    """scaler.json -> (mean, std) float32 tensors of equal length."""
    st = json.loads(Path(path).read_text(encoding="utf-8"))
    mean, std = (torch.tensor(st[k], dtype=torch.float32) for k in ("mean", "std"))
    if mean.numel() != std.numel():
        raise SystemExit("Scaler mean/std length mismatch")
    return mean, std


def pending_samples(samples_dir: Path, out_dir: Path, overwrite: bool, load: bool = True):
    """Jobs for the samples that still need a mel (frames loaded unless ``load`` is False: then only
    ``job.length``, the frame count from the .npy header, is read); missing mri.npy is reported."""
    if not samples_dir.is_dir():
        raise SystemExit(f"samples directory not found: {samples_dir}")
    dirs = sorted((p for p in samples_dir.iterdir() if p.is_dir()), key=lambda p: p.name)
    if not dirs:
        raise SystemExit(f"No sample folders found under {samples_dir}")
    jobs = []
    for d in dirs:
        if (out_dir / f"{d.name}.npy").exists() and not overwrite:
            continue
        job = drivers.Job(d / "mri.npy", d.name)
        if not job.src.is_file():
            print(f"[WARN] MRI file missing for {d.name}, skipping")
            continue
        if load:
            load_frames(job)
        else:
            try:
                job.length = int(np.load(job.src, mmap_mode="r", allow_pickle=False).shape[0])
            except Exception as e:  # noqa: BLE001 - reported per job (rank 0 writes the warning)
                job.error = f"{type(e).__name__}: {e}"
        jobs.append(job)
    return jobs


def load_frames(job):
    """(T,H,W) float32 frames of one sample into ``job.array`` (a read failure becomes ``job.error``)."""
    if job.error is not None or job.array is not None:
        return job
    try:
        job.array = np.load(job.src, allow_pickle=False).astype(np.float32, copy=False)
        job.length = int(job.array.shape[0])
    except Exception as e:  # noqa: BLE001 - reported per job
        job.error = f"{type(e).__name__}: {e}"
    return job


def init_distributed():
    """(world, rank, local_rank); joins the process group when launched by torch.distributed.run."""
    import os

    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("M2S_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def export_mels(args: argparse.Namespace) -> list:
    out_dir = Path(args.output_dir).resolve()
    out_dir.mkdir(parents=True, exist_ok=True)
    mean, std = scaler_arrays(Path(args.scaler_json).resolve())
    if args.cpu:
        raise SystemExit("--cpu: m2s runs on MI355X only (no CPU path); drop the flag")
    if not torch.cuda.is_available():
        raise SystemExit("m2s needs an MI355X (HIP) device; none is visible")
    world, rank, local = init_distributed()
    try:
        return _export(args, out_dir, mean, std, world, rank, local)
    finally:  # leave the group on every path, errors included, so no peer waits on this rank
        if world > 1:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()


def agree(ok: bool, device, world: int) -> bool:
    """True on every rank iff every rank passed ``ok`` (one all-reduce MIN); world 1: ``ok``."""
    if world == 1:
        return ok
    import torch.distributed as dist
    comm = device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=comm)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _export(args, out_dir, mean, std, world, rank, local) -> list:
    # one GPU per rank; more ranks than GPUs wrap round (a gloo rehearsal on a one-GPU box)
    device = torch.device("cuda", local % torch.cuda.device_count()) if world > 1 else torch.device("cuda")
    ckpt = Path(args.mri_checkpoint).resolve()
    # rank 0 reads the checkpoint; the other ranks build the same module tree and receive its weights.  A rank
    # that fails to build (rank 0: a missing or unreadable checkpoint) makes every rank stop before the
    # broadcast instead of leaving its peers blocked in it until the collective timeout.
    err = None
    try:
        model = drivers.build_acoustic(ckpt if rank == 0 else None, device, code_dir=args.mri_code_dir,
                                       n_mels=mean.numel(), dtype=args.dtype,
                                       log=print if rank == 0 else (lambda *a: None))
    except Exception as e:  # noqa: BLE001 - re-raised below on this rank, reported as a failure on the others
        err = e
    if not agree(err is None, device, world):
        if err is not None:
            raise err
        raise SystemExit(f"[rank {rank}] another rank failed to build the acoustic model (see rank 0's error)")
    if world > 1:
        broadcast_model_state(model, device)
    mean, std = mean.to(device), std.to(device)
    jobs = pending_samples(Path(args.processed_dir).resolve() / "samples", out_dir, args.overwrite,
                           load=world == 1)

    def mels(frames):  # (B,T,H,W) -> (B, n_mels, T) ln-mel
        _, ln = mel_glue(model(frames[:, :, None]), mean, std)
        return ln.transpose(1, 2)

    drivers.run_sharded(jobs, mels, device, lengths=[j.length for j in jobs], feat_shape=(mean.numel(),),
                        max_batch=args.batch, load=load_frames, time_axis=-1)
    if rank != 0:
        return []
    written = []
    for job in jobs:
        if job.result is None:
            print(f"[WARN] {job.stem}: {job.error}")
            continue
        path = out_dir / f"{job.stem}.npy"
        np.save(path, job.result.astype(np.float32))
        written.append(path)
    print(f"[INFO] {len(written)} mel file(s) written to {out_dir}")
    return written


def broadcast_model_state(model, device) -> None:
    """Rank 0's loaded weights to every rank in one flat broadcast (C1, m2s/dp.py)."""
    import torch.distributed as dist

    from m2s import dp

    comm = device if dist.get_backend() == "nccl" else torch.device("cpu")
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    got = dp.broadcast_state(sd, comm)
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in got.items()}, strict=True)


def parse_args(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description="Export predicted log-mel features for HiFi-GAN fine-tuning (MI355X).")
    p.add_argument("--processed_dir", required=True, help="rtMRI processed dataset root (contains samples/).")
    p.add_argument("--mri_checkpoint", required=True, help="Path to trained MRI->mel checkpoint (.pt).")
    p.add_argument("--scaler_json", required=True, help="Path to scaler.json (mean/std for denormalization).")
    p.add_argument("--output_dir", required=True, help="Directory for the log-mel .npy files (one per sample, [64, T]).")
    p.add_argument("--mri_code_dir", help="Directory containing mri_acoustic_model.py (if not importable by default).")
    p.add_argument("--cpu", action="store_true", help="Refused: m2s has no CPU execution path.")
    p.add_argument("--overwrite", action="store_true", help="Regenerate files even if they already exist.")
    p.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None,
                   help="m2s compute dtype (default: M2S_DTYPE or bf16x3)")
    p.add_argument("--batch", type=int, default=16, help="clips of equal length per forward call")
    return p.parse_args(argv)


def main(argv=None):
    return export_mels(parse_args(argv))


if __name__ == "__main__":
    main()
