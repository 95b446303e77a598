"""Clip-level data parallelism for inference (one process per GPU, torch.distributed).

The reference runs one clip in one process (run_mri_video_inference.py:203-255); clips are
independent, so the path shards with no data-path collective.  The only collectives are:

* C1 ``broadcast_state``  - rank 0's reference-format state dict to every rank, one flat buffer;
* C3 ``all_gather_lengths`` - per-rank clip lengths (T varies per clip) so rank 0 can size the gather;
* C2 ``gather_results``   - wav / mel of every clip to rank 0 (point-to-point over xGMI: each rank's
  shard travels on its own link to rank 0; no all-reduce anywhere).

Backend-agnostic: "nccl" (= RCCL on ROCm) on MI355X, "gloo" for the CPU tests.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.distributed as dist


def shard_clips(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Greedy length-balanced partition: longest clip first onto the least-loaded rank.

    Deterministic (ties broken by clip index then rank), so every rank computes the same plan
    without communication."""
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    load = [0] * world
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        shards[r].append(i)
        load[r] += int(lengths[i])
    return [sorted(s) for s in shards]


def broadcast_state(state: Dict[str, np.ndarray], device: torch.device, src: int = 0) -> Dict[str, np.ndarray]:
    """C1.  Non-src ranks may pass a state with the right keys/shapes (e.g. freshly constructed)."""
    if not (dist.is_available() and dist.is_initialized()):
        return state
    keys = [k for k in state if np.asarray(state[k]).dtype == np.float32]
    sizes = [int(np.asarray(state[k]).size) for k in keys]
    if dist.get_rank() == src:
        flat = torch.from_numpy(np.concatenate([np.asarray(state[k], np.float32).ravel() for k in keys]))
    else:
        flat = torch.empty(sum(sizes), dtype=torch.float32)
    flat = flat.to(device)
    dist.broadcast(flat, src)
    host = flat.cpu().numpy()
    out, off = dict(state), 0
    for k, n in zip(keys, sizes):
        out[k] = host[off:off + n].reshape(np.asarray(state[k]).shape)
        off += n
    return out


def all_gather_lengths(local_lengths: Sequence[int], device: torch.device) -> List[List[int]]:
    """C3.  Every rank learns every rank's clip lengths (padded to the max clip count)."""
    world = dist.get_world_size()
    n = torch.tensor([len(local_lengths)], dtype=torch.int64, device=device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    cap = int(max(x.item() for x in ns))
    buf = torch.full((max(cap, 1),), -1, dtype=torch.int64, device=device)
    if len(local_lengths):
        buf[: len(local_lengths)] = torch.tensor(list(local_lengths), dtype=torch.int64, device=device)
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    return [[int(v) for v in b.tolist() if v >= 0] for b in bufs]


def gather_results(local: torch.Tensor, lengths_by_rank: List[List[int]], per_step: int, dst: int = 0):
    """C2.  ``local`` is this rank's (n_local, max_len_local * per_step, ...) result (``per_step`` =
    samples per mel frame: the hop for wav, 1 for mels); returns, on ``dst``, the per-rank list of
    tensors trimmed to (n_r, max_len_r * per_step, ...), else None.  Every rank pads to the same
    (max clips, max length) buffer, computed from ``lengths_by_rank`` alone, so ranks with no clips
    (world > clips) take part with an all-padding buffer and a single gather moves everything."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    if per_step < 1:
        raise ValueError("per_step must be >= 1")
    cap_n = max(max(len(l) for l in lengths_by_rank), 1)
    cap_t = max(max((max(l) if l else 0) for l in lengths_by_rank), 1)
    if local.dim() < 2:
        raise ValueError("expected (clips, time, ...) results")
    shape = (cap_n, cap_t * per_step) + tuple(local.shape[2:])
    send = torch.zeros(shape, dtype=local.dtype, device=local.device)
    if local.numel():
        send[: local.shape[0], : local.shape[1]] = local
    if rank == dst:
        recv = [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, recv, dst=dst)
        out = []
        for r in range(world):
            lens = lengths_by_rank[r]
            n, t = len(lens), (max(lens) if lens else 0) * per_step
            out.append(recv[r][:n, :t])
        return out
    dist.gather(send, None, dst=dst)
    return None
