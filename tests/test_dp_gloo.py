"""Multi-process data-parallel driver (m2s.dp) on CPU with the gloo backend, world_size 2 and 4.

The same functions run over RCCL ("nccl") on MI355X in bench.py; only the backend differs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from m2s import dp


def test_shard_clips_balanced_and_complete():
    lens = [30, 1000, 30, 5, 7, 999, 64, 64, 1, 30]
    for world in (1, 2, 3, 8):
        shards = dp.shard_clips(lens, world)
        assert sorted(i for s in shards for i in s) == list(range(len(lens)))
        loads = [sum(lens[i] for i in s) for s in shards]
        assert max(loads) - min(loads) <= max(lens)
    assert dp.shard_clips([30] * 512, 8) == [list(range(r, 512, 8)) for r in range(8)] or \
        all(len(s) == 64 for s in dp.shard_clips([30] * 512, 8))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, n_clips):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        # C1: rank 0's weights reach everyone
        state = {"a.weight": np.full((3, 4), rank, np.float32), "b": np.arange(5, dtype=np.float32) * (rank + 1),
                 "n": np.array(rank, np.int64)}
        got = dp.broadcast_state(state, dev)
        ok1 = np.array_equal(got["a.weight"], np.zeros((3, 4), np.float32)) and \
            np.array_equal(got["b"], np.arange(5, dtype=np.float32)) and int(got["n"]) == rank
        # shard a ragged clip list, C3 lengths, C2 gather of per-clip "wav" (T * 3 samples)
        lens = [5, 9, 2, 7, 7, 1, 4][:n_clips]
        mine = dp.shard_clips(lens, world)[rank]
        my_lens = [lens[i] for i in mine]
        all_lens = dp.all_gather_lengths(my_lens, dev)
        tmax = max(my_lens) if my_lens else 0
        wav = torch.zeros(len(mine), tmax * 3)
        for j, i in enumerate(mine):
            wav[j, : lens[i] * 3] = float(i + 1)
        res = dp.gather_results(wav, all_lens, per_step=3)
        if rank == 0:
            shards = dp.shard_clips(lens, world)
            ok2 = True
            for r in range(world):
                for j, i in enumerate(shards[r]):
                    row = res[r][j]
                    ok2 &= bool((row[: lens[i] * 3] == i + 1).all()) and bool((row[lens[i] * 3:] == 0).all())
            q.put(("gather", ok2))
        q.put(("bcast", rank, ok1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_clips", [(2, 7), (4, 7), (4, 3)])
def test_dp_collectives_gloo(world, n_clips):
    """world 4 with 3 clips: one rank has an empty shard and still joins every collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, n_clips)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=10) for _ in range(world + 1)]
    assert ("gather", True) in msgs
    assert all(m[2] for m in msgs if m[0] == "bcast")
