"""bench.py host logic on CPU: the timed loop of the N-GPU path (barriers, max over ranks, the wav /
mel gather) under gloo with world 2, and the roofline arithmetic on synthetic profiler records."""
import os
import socket
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from m2s import dp  # noqa: E402


def test_parse_defaults_are_the_headline_workload():
    a = bench.parse([])
    assert (a.gpus, a.clips, a.frames, a.hw, a.dtype) == (1, 64, 30, 256, "bf16x3")
    assert a.steps * 0.04 >= 3.0  # a timed region of about three seconds or more at ~42 ms per step


def _launches(stats):
    """prof_launches()-style records (one per launch, in order, with a stage) from per-kernel totals."""
    out = []
    for s in stats:
        n = s["launches"]
        out += [dict(name=s["name"], stage=s["stage"], ms=s["ms"] / n, flops=s["flops"] / n, bytes=s["bytes"] / n)
                for _ in range(n)]
    return out


def test_roofline_picks_the_dominant_kernel_and_its_arithmetic():
    stats = [
        {"name": "dwconv_kernel<m2s::sp_t, 1>", "launches": 36, "ms": 20.0, "flops": 4e9 * 36, "bytes": 1.8e9 * 36,
         "stage": "cnn"},
        {"name": "lstm_persistent_kernel", "launches": 2, "ms": 1.2, "flops": 2e10, "bytes": 1e8, "stage": "bilstm"},
        {"name": "conv_gemm_kernel<128, 128, 4, 4, 2, 3, 0, 1>", "launches": 40, "ms": 10.0, "flops": 1e12, "bytes": 1e10,
         "stage": "mrf_c128"},
    ]
    r = bench.roofline(_launches(stats), "bf16x3", steps=2, fps=30000.0, frames_per_step=1920, stages=True)
    assert r["kernel"].startswith("dwconv") and r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert abs(r["achieved"] - 1.8e9 * 36 / 20e-3 / 1e9) < 1e-6 * r["achieved"]
    assert r["launches_per_step"] == 18
    assert bench.kernel_arith("lstm_persistent_kernel", "bf16x3") == "fp32"
    assert bench.kernel_arith("lstm_x3_kernel", "fp8") == "bf16x3"
    assert bench.kernel_arith("ir_pwdw_kernel<4, 1, 3>", "fp8") == "fp8"  # the e4m3 expand
    assert bench.kernel_arith("ir_pwdw_kernel<4, 1, 2>", "fp8") == "bf16"
    assert bench.kernel_arith("er8_fused_kernel", "fp8") == "fp8"  # the e4m3 EdgeResidual
    assert bench.kernel_arith("er_fused_kernel", "fp8") == "bf16"
    assert bench.kernel_arith("conv_igemm_kernel<float, 2, 4, 3>", "bf16") == "fp32"
    assert bench.PEAK_TFLOPS[bench.kernel_arith("conv_gemm_kernel<1>", "bf16x3")] == pytest.approx(2500.0 / 3)
    # fp8 engines: only the block-scaled e4m3 kernels (gemm128 KIND 0 / 1) are priced at the fp8 peak
    assert bench.kernel_arith("gemm128_kernel<0, 4, 1, 8, 3>", "fp8") == "fp8"
    assert bench.kernel_arith("gemm128_kernel<1, 2, 2, 8, 3>", "fp8") == "fp8"
    assert bench.kernel_arith("ir_pwdw_kernel<4, 1, 2>", "fp8") == "bf16"
    assert all(any(n.startswith(k) for k in bench.MFMA_KERNELS) for n in ("gemm128_kernel<2, 4, 2, 4, 3>", "er_sp_kernel<16>",
                                                                       "ir_ws_kernel<16, 4>", "conv1d_halo_sp_kernel<64>", "ers2_sp_kernel<16>"))
    fl = (4e9 * 36 + 2e10 + 1e12) / (2 * 1920)
    assert r["plan_gflop_per_frame"] == pytest.approx(fl / 1e9, rel=1e-3)
    # roofline.stages: per stage event time per step and algorithmic rates, in path order
    st = r["stages"]
    assert list(st) == ["cnn", "bilstm", "mrf_c128"]
    assert st["cnn"]["ms_per_step"] == pytest.approx(10.0) and st["cnn"]["launches_per_step"] == 18
    assert st["mrf_c128"]["algorithmic_GBs"] == pytest.approx(1e10 / 2 / 5e-3 / 1e9, rel=1e-3)
    assert "stages_source" in r


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        B, T, HOP = 3, 4, 5
        all_lens = dp.all_gather_lengths([T] * B, dev)
        wav = torch.full((B, T * HOP), float(rank + 1))
        mel = torch.full((B, T, 2), float(10 * (rank + 1)))
        got = {}

        def step():
            time.sleep(0.05 * (rank + 1))  # the slower rank sets the step time
            got["wav"] = dp.gather_results(wav, all_lens, per_step=HOP)
            got["mel"] = dp.gather_results(mel, all_lens, per_step=1)

        el = bench.timed_loop(step, 3, world, lambda: None, dev)
        ok = el >= 3 * 0.05 * world - 1e-3
        if rank == 0:
            ok &= all(bool((got["wav"][r] == r + 1).all()) and got["wav"][r].shape == (B, T * HOP) for r in range(world))
            ok &= all(bool((got["mel"][r] == 10 * (r + 1)).all()) and got["mel"][r].shape == (B, T, 2) for r in range(world))
        q.put((rank, ok, el))
    finally:
        dist.destroy_process_group()


def test_timed_loop_and_gather_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert all(ok for _, ok, _ in res), res
    assert res[0][2] == res[1][2]  # every rank reports the same (max) time


def _ragged_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lens_all = bench.ragged_lengths(13, 30)
        plan = bench.RaggedPlan(lens_all, world, rank)
        calls = []

        def forward(x):  # stand-in pipeline: every output row carries its clip id
            calls.append(tuple(x.shape))
            n, L = x.shape[:2]
            ids = x[:, 0, 0, 0]
            return {"wav": ids[:, None].expand(n, L * bench.HOP).clone(), "mel_db": ids[:, None, None].expand(n, L, 64).clone()}

        fr = {}
        for L, r0, r1 in plan.groups:  # frames whose first pixel is the global clip id
            fr[L] = torch.zeros(r1 - r0, L, 2, 2)
            fr[L][:, 0, 0, 0] = torch.tensor([float(i) for i in plan.mine[r0:r1]])
        wav = torch.zeros(len(plan.mine), plan.tmax * bench.HOP)
        mel = torch.zeros(len(plan.mine), plan.tmax, 64)
        got = plan.step(forward, fr, wav, mel, True)
        ok = len(calls) == len(plan.groups) == len({L for L, _, _ in plan.groups})
        if rank == 0:
            seen = []
            for r, s in enumerate(plan.shards):
                for k, i in enumerate(s):
                    L = lens_all[i]
                    ok &= bool((got[0][r][k, : L * bench.HOP] == i).all()) and bool((got[0][r][k, L * bench.HOP:] == 0).all())
                    ok &= bool((got[1][r][k, :L] == i).all())
                    seen.append(i)
            ok &= sorted(seen) == list(range(13))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ragged_bench_step_gloo(world):
    """bench.py --ragged: a ragged clip list sharded by length, one forward per length group, every
    clip's wav / mel back on rank 0 in its own row and length (rank 3 of 4 may hold few clips)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(ok for _, ok in res), res
    assert sorted(set(bench.ragged_lengths(64, 30))) == [24, 30, 36]


def test_cpu_baseline_reports_every_config_and_stage():
    """BASELINE.md's CPU plan: C3 end to end with per-stage wall time (CNN / BiLSTM / head + glue / Generator), C1 (mel
    only) from the same runs, C5 (one long clip); the thread count and why.  Tiny shapes here (the oracle on CPU)."""
    from m2s import synth
    args = bench.parse(["--frames", "3", "--hw", "64", "--cpu-seconds", "0.01", "--cpu-long-frames", "5"])
    ac, gen = synth.synth_acoustic_state(0), synth.synth_generator_state(0)
    mean, std = synth.synth_scaler()
    r = bench.cpu_baseline(args, ac, gen, mean, std)
    assert r["kind"] == "port" and r["cores"] >= 1 and r["value"] > 0 and "threads_note" in r
    per = r["per_config"]
    assert set(per) == {"C1", "C3", "C5"}
    assert set(per["C3"]["stage_ms_per_clip"]) == {"cnn", "bilstm", "head_glue", "generator"}
    assert per["C1"]["frames_per_s"] >= per["C3"]["frames_per_s"] > 0 and per["C5"]["rtf"] > 0
