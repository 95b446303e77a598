"""The multi-GPU product path over a ragged clip list (drivers.run_sharded, export_predicted_mels.py's
torchrun mode) on CPU with the gloo backend, world_size 2 and 4.

The reference's mel export walks its samples in one process (scripts/export_predicted_mels.py:43-99).
Here every rank derives the same length-balanced plan, loads and runs only its own clips, and the
results come back to rank 0 in one padded gather; rank 0's jobs must end exactly as a single-process
run leaves them (results, per-job failures and their messages).  The device call is a stand-in
function on CPU tensors (run_batches' contract); on MI355X it is the acoustic model over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from m2s import drivers

LENS = [5, 9, 2, 7, 7, 1, 4, 3, 9, 6]
BAD = 3          # this sample's file cannot be read
RAISES_T = 1     # batches of this length make the device call raise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _jobs():
    return [drivers.Job(None, f"utt{i}", length=t) for i, t in enumerate(LENS)]


def _load(job):
    i = int(job.stem[3:])
    if i == BAD:
        job.error = "OSError: unreadable"
        return job
    job.array = np.random.default_rng(i).random((LENS[i], 4, 4), dtype=np.float32)
    return job


def _fn(x):  # (B,T,4,4) -> (B,3,T): a running mean over time, so padding or a wrong length shows
    if x.shape[1] == RAISES_T:
        raise RuntimeError("device call failed")
    m = x.mean(dim=(2, 3))
    return torch.cumsum(m, dim=1)[:, None, :] * torch.tensor([1.0, 2.0, 3.0])[None, :, None]


def _single():
    jobs = _jobs()
    drivers.run_sharded(jobs, _fn, torch.device("cpu"), LENS, (3,), max_batch=2, load=_load)
    return jobs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        jobs = _jobs()
        drivers.run_sharded(jobs, _fn, torch.device("cpu"), LENS, (3,), max_batch=2, load=_load)
        if rank == 0:
            q.put([(j.result, j.error) for j in jobs])
    finally:
        dist.destroy_process_group()


def test_run_sharded_single_process_is_run_batches():
    jobs = _single()
    ok = [j for j in jobs if j.error is None]
    assert len(ok) == len(LENS) - 2  # the unreadable file and the length-1 batch failed, the rest ran
    for j in ok:
        assert j.result.shape == (3, j.length)
    assert "unreadable" in jobs[BAD].error and "device call failed" in jobs[LENS.index(RAISES_T)].error


@pytest.mark.parametrize("world", [2, 4])
def test_run_sharded_gloo_equals_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    want = _single()
    for i, (res, err) in enumerate(got):
        if want[i].error is None:
            assert err is None, (i, err)
            assert res.shape == want[i].result.shape and np.array_equal(res, want[i].result), i
        else:
            assert res is None and err is not None and want[i].error.split(": ")[-1] in err, (i, err)


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib.util

        from m2s import synth
        from mri_acoustic_model import build_acoustic_model
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        spec = importlib.util.spec_from_file_location(
            "m2s_export_mels", os.path.join(repo, "mri-to-speech_amd", "scripts", "export_predicted_mels.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        model = build_acoustic_model()
        if rank == 0:
            model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synth_acoustic_state(9).items()})
        mod.broadcast_model_state(model, torch.device("cpu"))
        want = synth.synth_acoustic_state(9)
        q.put((rank, all(np.array_equal(v.numpy(), want[k]) for k, v in model.state_dict().items()
                         if not k.endswith("num_batches_tracked"))))
    finally:
        dist.destroy_process_group()


def test_export_broadcasts_rank0_weights_gloo():
    """export_predicted_mels.py's torchrun mode: only rank 0 reads the checkpoint; its weights reach every
    rank's plug-in model in one broadcast (C1)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert sorted(msgs) == [(0, True), (1, True)]


def test_export_pending_samples_reads_lengths_only(tmp_path):
    """Without loading, the sharding plan gets each sample's frame count from its .npy header."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "m2s_export_mels", os.path.join(repo, "mri-to-speech_amd", "scripts", "export_predicted_mels.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for stem, T in (("a", 4), ("b", 11)):
        d = tmp_path / "samples" / stem
        d.mkdir(parents=True)
        np.save(d / "mri.npy", np.zeros((T, 8, 8), np.float32))
    (tmp_path / "samples" / "c").mkdir()
    (tmp_path / "samples" / "c" / "mri.npy").write_text("garbage")
    jobs = mod.pending_samples(tmp_path / "samples", tmp_path / "out", overwrite=False, load=False)
    assert [(j.stem, j.length, j.array is None) for j in jobs[:2]] == [("a", 4, True), ("b", 11, True)]
    assert jobs[2].error is not None
    assert mod.load_frames(jobs[1]).array.shape == (11, 8, 8)


def _agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib.util
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        spec = importlib.util.spec_from_file_location(
            "m2s_export_mels", os.path.join(repo, "mri-to-speech_amd", "scripts", "export_predicted_mels.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        dev = torch.device("cpu")
        q.put((rank, mod.agree(True, dev, world), mod.agree(rank != 0, dev, world)))
    finally:
        dist.destroy_process_group()


def test_export_ranks_agree_on_a_failed_build_gloo():
    """export_predicted_mels.py's torchrun mode: when rank 0 cannot build the model (a bad checkpoint) every rank
    learns it from one all-reduce and stops, instead of waiting in the state broadcast until the timeout."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    msgs = sorted(q.get(timeout=180) for _ in range(3))
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert msgs == [(0, True, False), (1, True, False), (2, True, False)]
