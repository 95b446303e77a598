"""Batch drivers behind the stand-alone command lines (vocoder callers, mel export).

The reference's stand-alone scripts walk their inputs one file at a time and call the model once per
file (mel_to_audio_synthesis.py:218-223, inference_e2e.py:47-57, scripts/export_predicted_mels.py:78-99).
The m2s command lines keep those scripts' flags and output files but run a different plan:

1. ``Job`` list: every input is read and conformed on the host first (unreadable / malformed inputs
   become failed jobs with the reason kept, the rest go on);
2. ``plan_batches``: jobs whose arrays have the same shape form one batch (at most ``max_batch``);
3. ``vocode`` / the acoustic model: each batch is ONE pinned host block, ONE H2D copy, ONE device call
   (``Generator.forward`` on (B, n_mels, T) runs ``torch.ops.m2s.hifigan_forward``), ONE D2H copy;
4. the writers below produce the reference's files from the host results.

Clips are independent through the generator (every MRF conv is causal per clip and the transposed
convs never mix batch rows), so a batched call returns exactly the per-file results.
"""
from __future__ import annotations

import json
import wave
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

MAX_WAV_VALUE = 32768.0  # meldataset.py:14 (inference_e2e.py's int16 scale)


@dataclass
class Job:
    """One input file and what became of it."""

    src: Path
    stem: str
    array: Optional[np.ndarray] = None   # conformed input, host
    length: int = 0                      # time steps of the input (frames), for length-balanced sharding
    result: Optional[np.ndarray] = None  # model output, host
    notes: List[str] = field(default_factory=list)
    error: Optional[str] = None

    @property
    def ok(self) -> bool:
        return self.error is None and self.array is not None


# ------------------------------------------------------------------------------------------------
# planning and device execution
def plan_batches(jobs: Iterable[Job], max_batch: int = 64) -> List[List[Job]]:
    """Group the runnable jobs by input shape; first-seen order, chunks of at most ``max_batch``."""
    if max_batch < 1:
        raise ValueError("max_batch must be >= 1")
    by_shape: Dict[tuple, List[Job]] = {}
    for j in jobs:
        if j.ok:
            by_shape.setdefault(tuple(j.array.shape), []).append(j)
    return [grp[i:i + max_batch] for grp in by_shape.values() for i in range(0, len(grp), max_batch)]


def run_batches(batches: Sequence[Sequence[Job]], fn: Callable[[torch.Tensor], torch.Tensor],
                device: torch.device, stack: Callable[[List[np.ndarray]], np.ndarray] = np.stack) -> None:
    """For every batch: stack -> pinned host block -> device -> ``fn`` -> host, one result row per job.

    A batch whose device call raises marks each of its jobs failed with that error and the run goes on
    (the reference reports a failed file and continues, mel_to_audio_synthesis.py:132-136)."""
    for batch in batches:
        host = torch.from_numpy(np.ascontiguousarray(stack([j.array for j in batch]), dtype=np.float32))
        if device.type == "cuda":
            host = host.pin_memory()
        try:
            with torch.no_grad():
                out = fn(host.to(device, non_blocking=True)).float().cpu().numpy()
        except Exception as e:  # noqa: BLE001 - reported per job
            for j in batch:
                j.error = f"{type(e).__name__}: {e}"
            continue
        for j, row in zip(batch, out):
            j.result = row


def run_sharded(jobs: Sequence[Job], fn: Callable[[torch.Tensor], torch.Tensor], device: torch.device,
                lengths: Sequence[int], feat_shape: Sequence[int], max_batch: int = 16,
                load: Optional[Callable[[Job], Job]] = None, time_axis: int = -1, per_step: int = 1) -> List[Job]:
    """``run_batches`` over one process per GPU (torch.distributed; a no-op wrapper at world 1).

    Every rank holds the same job list and ``lengths`` (time steps per job, e.g. frames), so every rank
    derives the same length-balanced plan (``dp.shard_clips``) with no communication.  A rank loads
    (``load``) and runs only its own shard, batched by shape as in a single process; then every rank's
    results travel to rank 0 in ONE padded gather (``dp.gather_results``: RCCL "nccl" over xGMI on
    MI355X, gloo in the CPU tests), plus a gather of the per-job status and error text.  On rank 0
    every job of the list ends with ``result`` / ``error`` as a single-process ``run_batches`` leaves
    them; the other ranks return their own shard.

    A job's result is an array whose ``time_axis`` holds ``length * per_step`` steps and whose other
    axes are ``feat_shape`` (an ln-mel: (n_mels, T), time_axis -1)."""
    import torch.distributed as dist

    from . import dp

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        mine = [load(j) for j in jobs] if load else list(jobs)
        run_batches(plan_batches(mine, max_batch), fn, device)
        return list(jobs)
    world, rank = dist.get_world_size(), dist.get_rank()
    if len(lengths) != len(jobs):
        raise ValueError("one length per job")
    shards = dp.shard_clips(lengths, world)
    mine = [jobs[i] for i in shards[rank]]
    if load:
        mine = [load(j) for j in mine]
    run_batches(plan_batches(mine, max_batch), fn, device)

    comm = device if dist.get_backend() == "nccl" else torch.device("cpu")
    lens_by_rank = [[int(lengths[i]) for i in s] for s in shards]
    tmax = max(lens_by_rank[rank], default=0) * per_step
    local = torch.zeros((len(mine), tmax) + tuple(feat_shape), dtype=torch.float32)
    status = torch.zeros((len(mine), 1), dtype=torch.float32)
    errors = {}
    for k, j in enumerate(mine):
        if j.result is not None and j.error is None:
            r = np.moveaxis(np.asarray(j.result, np.float32), time_axis, 0)
            local[k, : r.shape[0]] = torch.from_numpy(np.ascontiguousarray(r))
            status[k, 0] = 1.0
        else:
            errors[shards[rank][k]] = j.error or "no result"
    got = dp.gather_results(local.to(comm), lens_by_rank, per_step=per_step)
    ok = dp.gather_results(status.to(comm), [[1] * len(s) for s in shards], per_step=1)
    errs = [None] * world if rank == 0 else None
    dist.gather_object(errors, errs, dst=0)
    if rank != 0:
        return mine
    all_errors = {i: e for d in errs for i, e in d.items()}
    for r, s in enumerate(shards):
        rows, flags = got[r].cpu().numpy(), ok[r].cpu().numpy()
        for k, i in enumerate(s):
            j = jobs[i]
            if flags[k, 0] > 0:
                j.result, j.error = np.moveaxis(rows[k, : int(lengths[i]) * per_step], 0, time_axis).copy(), None
            else:
                j.result = None
                j.error = all_errors.get(i, "no result") if r == 0 else f"rank {r}: {all_errors.get(i, 'no result')}"
    return list(jobs)


def vocode(generator, jobs: Sequence[Job], device: torch.device, max_batch: int = 64) -> None:
    """Every runnable job's (n_mels, T) ln-mel -> waveform (T * hop,) in ``job.result``."""
    run_batches(plan_batches(jobs, max_batch), lambda x: generator(x).reshape(x.shape[0], -1), device)


# ------------------------------------------------------------------------------------------------
# loading
def load_state(path) -> dict:
    """A checkpoint written by torch.save, loaded without executing anything from the file."""
    p = Path(path)
    if not p.is_file():
        raise FileNotFoundError(f"checkpoint not found: {p}")
    return torch.load(p, map_location="cpu", weights_only=True)


def strip_weight_norm(gen) -> int:
    """Best-effort weight-norm removal over ups, resblocks and conv_post (conv_pre never has one,
    models.py:94); returns how many modules had it.  Removal leaves the folded m2s weights as they are."""
    from torch.nn.utils import remove_weight_norm

    removed = 0
    for mod in list(gen.ups) + [gen.conv_post]:
        try:
            remove_weight_norm(mod)
            removed += 1
        except (ValueError, AttributeError):
            pass
    for rb in gen.resblocks:
        try:
            rb.remove_weight_norm()
            removed += 1
        except (ValueError, AttributeError):
            pass
    return removed


def build_generator(h, checkpoint, device: torch.device, dtype: Optional[str] = None):
    """``Generator(h)`` with ``ckpt['generator']`` loaded strictly, eval, weight norm stripped."""
    from models import Generator

    ck = load_state(checkpoint)
    if "generator" not in ck:
        raise KeyError(f"{checkpoint}: no 'generator' entry")
    gen = Generator(h).to(device)
    gen.load_state_dict(ck["generator"])
    gen.eval()
    n = strip_weight_norm(gen)
    if dtype:
        gen.m2s_dtype = dtype
    return gen, n


def build_acoustic(checkpoint, device: torch.device, code_dir=None, n_mels: int = 64, rnn_hidden: int = 640,
                   dropout: float = 0.5, dtype: Optional[str] = None, log=print):
    """The acoustic model through the plug-in surface: ``code_dir`` first on sys.path,
    ``build_acoustic_model(**kw)`` (mri_acoustic_model.py:139-156), a ``.pt`` holding
    ``model_state_dict`` or a raw state dict, ``load_state_dict(strict=False)`` with the key
    mismatches reported, eval."""
    import sys

    if code_dir is not None and Path(code_dir).is_dir() and str(Path(code_dir).resolve()) not in sys.path:
        sys.path.insert(0, str(Path(code_dir).resolve()))
    try:
        from mri_acoustic_model import build_acoustic_model
    except ImportError as e:
        raise ImportError("cannot import mri_acoustic_model; point the code-dir flag at the directory holding it") from e
    model = build_acoustic_model(n_mels=n_mels, cnn_pretrained=False, rnn_hidden=rnn_hidden, dropout=dropout,
                                 use_checkpoint=False, ckpt_segments=2, use_reentrant=False).to(device)
    if checkpoint is None:  # weights arrive later (a non-zero rank of a multi-GPU run: dp.broadcast_state)
        model.eval()
        if dtype:
            model.m2s_dtype = dtype
        return model
    ck = load_state(checkpoint)
    missing, unexpected = model.load_state_dict(ck.get("model_state_dict", ck), strict=False)
    for kind, keys in (("missing", missing), ("unexpected", unexpected)):
        if keys:
            log(f"[WARN] {len(keys)} {kind} key(s) in the MRI checkpoint: {list(keys)}")
    model.eval()
    if dtype:
        model.m2s_dtype = dtype
    return model


def read_mel(job: Job, n_mels: int, conform: bool = True) -> Job:
    """Load ``job.src`` (.npy) into a (n_mels, T) float32 array.  ``conform`` (the synthesis script,
    mel_to_audio_synthesis.py:62-87): a leading batch axis keeps its first row, extra bins are
    dropped, missing bins become zero rows.  Without it (inference_e2e.py:48-50 hands the array to
    the generator as is) a (1, n_mels, T) array is accepted and anything else of the wrong size fails.
    Failures land in ``job.error``."""
    try:
        a = np.load(job.src, allow_pickle=False)
        if a.ndim == 3:
            if a.shape[0] != 1:
                if not conform:
                    raise ValueError(f"batched mel {a.shape}: one utterance per file expected")
                job.notes.append(f"batch of {a.shape[0]}, first sample used")
            a = a[0]
        if a.ndim != 2:
            raise ValueError(f"Invalid mel spectrogram dimensions: {a.shape}")
        a = a.astype(np.float32, copy=False)
        if a.shape[0] != n_mels and not conform:
            raise ValueError(f"mel has {a.shape[0]} bins, the generator expects {n_mels}")
        if a.shape[0] > n_mels:
            job.notes.append(f"{a.shape[0]} bins truncated to {n_mels}")
            a = a[:n_mels]
        elif a.shape[0] < n_mels:
            job.notes.append(f"{a.shape[0]} bins zero-padded to {n_mels}")
            a = np.concatenate([a, np.zeros((n_mels - a.shape[0], a.shape[1]), np.float32)])
        if a.shape[1] < 1:
            raise ValueError("mel has no frames")
        job.array = np.ascontiguousarray(a)
    except Exception as e:  # noqa: BLE001 - reported per job
        job.error = f"{type(e).__name__}: {e}"
    return job


# ------------------------------------------------------------------------------------------------
# writers
def write_wav_pcm16(path, audio: np.ndarray, sr: int) -> None:
    """16-bit PCM wav with soundfile's float scaling (round(x * 32767), clipped); soundfile itself when
    installed (its WAV default subtype is PCM_16)."""
    try:
        import soundfile
    except ImportError:
        soundfile = None
    if soundfile is not None:
        soundfile.write(str(path), audio, sr)
        return
    pcm = np.clip(np.rint(np.asarray(audio, np.float64) * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sr))
        w.writeframes(pcm.tobytes())


def int16_truncated(audio: np.ndarray) -> np.ndarray:
    """inference_e2e.py:51-53: ``(audio * MAX_WAV_VALUE).astype('int16')`` (truncation toward zero)."""
    return (np.asarray(audio, np.float32) * MAX_WAV_VALUE).astype(np.int16)


def save_mel_png(mel: np.ndarray, title: str, path) -> bool:
    """(bins, T) image like the reference's figures; False when matplotlib is missing."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        from matplotlib import pyplot as plt
    except ImportError:  # pragma: no cover
        return False
    fig, ax = plt.subplots(figsize=(12, 4))
    im = ax.imshow(mel, aspect="auto", origin="lower")
    fig.colorbar(im, ax=ax)
    ax.set(title=title, xlabel="Time", ylabel="Mel Bins")
    fig.tight_layout()
    fig.savefig(path, dpi=150)
    plt.close(fig)
    return True


def write_json(path, obj) -> None:
    Path(path).write_text(json.dumps(obj, indent=2), encoding="utf-8")
