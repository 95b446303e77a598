"""Split-fp32 ("bf16x3") path vs the CPU oracle and the reference goldens at the fp32 tolerances.

bf16x3 keeps every activation and weight as a bf16 pair hi + lo (17 significant bits) and forms
each product as the three exact bf16 MFMA terms hi*hi + hi*lo + lo*hi with fp32 accumulation
(include/m2s.h M2S_DT_BF16X3).  It must pass the SAME bars as the exact-f32 path
(tests/test_gpu_parity.py): wav max |d| <= 1e-4 vs the reference goldens, CNN taps <= 1e-4 of the
tensor's scale, mel_norm <= 1e-4 and wav <= 1e-4 end to end.  GPU box only.
"""
import json
import os

import numpy as np
import pytest
import torch

from m2s import synth
from m2s.config import HIFIGAN_H
from oracle import acoustic, effnet, hifigan

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = torch.device("cuda", 0)


def _gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-6))


@pytest.fixture(scope="module")
def rt():
    from m2s import runtime
    return runtime


@pytest.fixture(scope="module")
def ac_state():
    g = _gold("acoustic.npz")
    return synth.synth_acoustic_state(int(g["seed"]))


@pytest.mark.parametrize("case", ["r1", "r2"])
def test_vocoder_bf16x3_matches_reference_golden(rt, case):
    g = _gold("generator.npz")
    h = json.loads(bytes(g[f"{case}_h"]).decode())
    voc = rt.VocoderEngine(synth.synth_generator_state(int(g["seed"]), h), h, dtype="bf16x3", device=DEV)
    wav = voc.forward(torch.from_numpy(g[f"{case}_mel"]).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(wav, g[f"{case}_wav"], atol=1e-4, rtol=0)


@pytest.mark.parametrize("B,T", [(1, 1), (3, 17), (2, 64)])
def test_vocoder_bf16x3_vs_oracle_shapes(rt, B, T):
    sd = synth.synth_generator_state(5, HIFIGAN_H)
    voc = rt.VocoderEngine(sd, HIFIGAN_H, dtype="bf16x3", device=DEV)
    mel = synth.synth_mel_log(B, 64, T, seed=B * 100 + T)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, HIFIGAN_H, torch.from_numpy(mel)).numpy()
    wav = voc.forward(torch.from_numpy(mel).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(wav, ref, atol=1e-4, rtol=0)


@pytest.mark.parametrize("B,T", [(1, 1), (3, 17), (2, 64)])
def test_vocoder_bf16x3_mrf_fused(rt, monkeypatch, B, T):
    """Split fused ResBlock1 (mrf_fused.hip SP = 1, the C = 32 stage) against the oracle at the fp32
    bar and against the per-conv split path: a clip shorter than one tile, ragged last tiles, several
    clips.  Both are split fp32; they differ only by where the hi/lo re-splits round (~1e-6)."""
    sd = synth.synth_generator_state(7, HIFIGAN_H)
    mel = synth.synth_mel_log(B, 64, T, seed=B * 10 + T)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, HIFIGAN_H, torch.from_numpy(mel)).numpy()
    monkeypatch.setenv("M2S_MRF_FUSED", "1")
    fused = rt.VocoderEngine(sd, HIFIGAN_H, dtype="bf16x3", device=DEV).forward(torch.from_numpy(mel).to(DEV))
    monkeypatch.setenv("M2S_MRF_FUSED", "0")
    plain = rt.VocoderEngine(sd, HIFIGAN_H, dtype="bf16x3", device=DEV).forward(torch.from_numpy(mel).to(DEV))
    fused, plain = fused.cpu().numpy(), plain.cpu().numpy()
    np.testing.assert_allclose(fused, ref, atol=1e-4, rtol=0)
    np.testing.assert_allclose(fused, plain, atol=2e-5, rtol=0)


@pytest.mark.parametrize("hw",[(256, 256), (96, 80), (67, 101)])
def test_effnet_bf16x3_every_block(rt, ac_state, hw):
    sd = {k: torch.from_numpy(v) for k, v in ac_state.items()}
    fr = torch.from_numpy(synth.synth_frames(1, 3, hw=hw, seed=4)[0])
    taps = []
    effnet.effnet_features(sd, fr, taps=taps)
    eng = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    x = fr.to(DEV)
    for i, ref in enumerate(taps):
        got = eng.probe(x, i).cpu().numpy()
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        assert _rel(got, ref.numpy()) <= 1e-4, f"block {i}: rel err {_rel(got, ref.numpy())}"
    gap = eng.effnet(x).cpu().numpy()
    assert _rel(gap, effnet.effnet_gap(sd, fr).numpy()) <= 1e-4


def test_pipeline_bf16x3_end_to_end(rt, ac_state):
    sd = {k: torch.from_numpy(v) for k, v in ac_state.items()}
    gsd = synth.synth_generator_state(3)
    mean, std = synth.synth_scaler()
    pipe = rt.Pipeline(rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV),
                       rt.VocoderEngine(gsd, HIFIGAN_H, dtype="bf16x3", device=DEV), mean, std)
    fr = synth.synth_frames(2, 6, seed=21)
    out = {k: v.cpu().numpy() for k, v in pipe.forward(torch.from_numpy(fr).to(DEV)).items()}
    B, T = fr.shape[:2]
    f = effnet.effnet_gap(sd, torch.from_numpy(fr).reshape(B * T, 256, 256)).view(B, T, -1)
    mn = acoustic.head(sd, acoustic.bilstm_summerge(sd, f))
    db = acoustic.denormalize_mel(mn, mean, std)
    ln = acoustic.mel_db_to_log(db)
    wav = hifigan.generator({k: torch.from_numpy(v) for k, v in gsd.items()}, HIFIGAN_H, ln.transpose(1, 2))
    np.testing.assert_allclose(out["mel_norm"], mn.numpy(), atol=1e-4, rtol=0)
    np.testing.assert_allclose(out["mel_db"], db.numpy(), atol=2e-3, rtol=0)
    np.testing.assert_allclose(out["mel_log"], ln.numpy(), atol=5e-4, rtol=0)
    np.testing.assert_allclose(out["wav"], wav[:, 0].numpy(), atol=1e-4, rtol=0)


@pytest.mark.parametrize("hw,n", [((256, 256), 300), ((128, 128), 263)])
def test_ir_ws_matches_grid_kernel(rt, ac_state, monkeypatch, hw, n):
    """The persistent warp-specialised IR front half (ir_ws.hip: 16x16 and 8x8 maps, more images than
    workgroups) against the one-slice-per-workgroup kernel it replaces (M2S_IR_WS=0).  Same split fp32
    arithmetic except the order of the squeeze sums, which moves a few hi/lo roundings (17-bit
    values): the two differ by about their own distance from the fp32 oracle (~1e-5 of the scale,
    tools/diag_ir_ws.py), so the bar is the parity bar, 1e-4."""
    fr = torch.from_numpy(synth.synth_frames(1, n, hw=hw, seed=7)[0]).to(DEV)
    monkeypatch.setenv("M2S_IRWS_MIN", "0")  # ir_ws at any pass size (the product runs it from 512 frames a pass)
    monkeypatch.setenv("M2S_SEWS_MIN", "0")  # and se_ws after it, so ir_ws hands over fp32 rows (fm32) at both sizes
    ws = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    monkeypatch.setenv("M2S_IR_WS", "0")
    grid = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    for i in (10, 12, 13, 18, 24, 28):  # after blocks 3.1, 3.3, 4.0, 4.5, 5.5, 5.9
        a, b = ws.probe(fr, i).cpu().numpy(), grid.probe(fr, i).cpu().numpy()
        assert _rel(a, b) <= 1e-4, f"tap {i}: {_rel(a, b)}"
    assert _rel(ws.effnet(fr).cpu().numpy(), grid.effnet(fr).cpu().numpy()) <= 1e-4


@pytest.mark.parametrize("n", [3, 300])
def test_ir_ws_stride2_matches_grid_kernel_and_oracle(rt, ac_state, monkeypatch, n):
    """blocks.5.0 (the stride-2 IR block at 16x16 -> 8x8) on the persistent ir_ws kernel (ir_ws_kernel<16, 4, 2>)
    against the one-slice-per-workgroup ir_pwdw_s2 kernel it replaces (M2S_IR_WS_S2=0) and, at 3 frames, the fp32
    oracle's tap; 300 frames = more images than workgroups.  Same split fp32 arithmetic up to the squeeze's
    summation order: the 1e-4 parity bar."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state.items()}
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=23)[0])
    monkeypatch.setenv("M2S_IRWS_MIN", "0")  # ir_ws at any pass size (the product runs it from 512 frames a pass)
    ws = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    monkeypatch.setenv("M2S_IR_WS_S2", "0")
    grid = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    x = fr.to(DEV)
    from m2s import _native
    names = {}
    for key, eng in (("ws", ws), ("grid", grid)):  # the kernel each engine runs for blocks.5.0
        _native.prof_enable(True)
        eng.probe(x, 19)
        torch.cuda.synchronize()
        names[key] = {r["name"] for r in _native.prof_launches()}
        _native.prof_enable(False)
    assert "ir_ws_kernel<16, 4, 2>" in names["ws"] and "ir_pwdw_s2_kernel<1>" not in names["ws"], names["ws"]
    assert "ir_pwdw_s2_kernel<1>" in names["grid"], names["grid"]
    for i in (19, 20):  # after blocks.5.0 (stride 2) and blocks.5.1 (its SE-gated output feeds it)
        a, b = ws.probe(x, i).cpu().numpy(), grid.probe(x, i).cpu().numpy()
        assert np.isfinite(a).all() and _rel(a, b) <= 1e-4, (i, _rel(a, b))
    if n <= 3:
        taps = []
        effnet.effnet_features(sd, fr, taps=taps)
        assert _rel(ws.probe(x, 19).cpu().numpy(), taps[19].numpy()) <= 1e-4
    assert _rel(ws.effnet(x).cpu().numpy(), grid.effnet(x).cpu().numpy()) <= 1e-4


@pytest.mark.parametrize("n", [3, 37])
def test_ir_s2band_matches_unfused(rt, ac_state, monkeypatch, n):
    """blocks.3.0 as one banded kernel (ir_s2band.hip: conv_pw + stride-2 depthwise on 4-row bands, squeeze
    partials per band) against the conv_pw GEMM + dwconv + se_mean sequence it replaces (M2S_IR_S2BAND=0)
    and the fp32 oracle: the expanded activation stays fp32 in LDS instead of a hi/lo round trip, so the
    two agree to the split rounding; both at the 1e-4 parity bar."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state.items()}
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=17)[0])
    band = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    monkeypatch.setenv("M2S_IR_S2BAND", "0")
    plain = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    x = fr.to(DEV)
    for i in (9, 10):  # after blocks.3.0 (the banded block) and blocks.3.1 (its SE-gated output feeds it)
        a, b = band.probe(x, i).cpu().numpy(), plain.probe(x, i).cpu().numpy()
        assert np.isfinite(a).all() and _rel(a, b) <= 1e-4, (i, _rel(a, b))
    if n <= 3:
        taps = []
        effnet.effnet_features(sd, fr, taps=taps)
        assert _rel(band.probe(x, 9).cpu().numpy(), taps[9].numpy()) <= 1e-4
    assert _rel(band.effnet(x).cpu().numpy(), plain.effnet(x).cpu().numpy()) <= 1e-4


def test_er_sp_merged_ring_stages_are_bit_identical(rt, ac_state, monkeypatch):
    """er_sp_fused.hip MRG = 2 (blocks.1.1/.2: a W_hi stage and its W_lo stage share one ring slot, half
    the barriers) issues the same MFMAs in the same order as one stage per slot (M2S_ER_MRG=0), so the
    block outputs are equal bit for bit; 5 frames = several 16-row tiles per workgroup pass."""
    fr = torch.from_numpy(synth.synth_frames(1, 5, seed=13)[0]).to(DEV)
    merged = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    monkeypatch.setenv("M2S_ER_MRG", "0")
    single = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    for i in (4, 5):  # after blocks.1.1, blocks.1.2
        assert torch.equal(merged.probe(fr, i), single.probe(fr, i)), i


@pytest.mark.parametrize("B,T", [(1, 5), (3, 17), (4, 40)])
def test_vocoder_bf16x3_mrf_batched(rt, monkeypatch, B, T):
    """The batched split MRF stages (one launch per pair for every resblock, grid.z = resblock;
    LeakyReLU applied once by the producer and inverted for the residual: model.cpp
    mrf_stage_batched) against the oracle at the fp32 bar, the C = 64 / 128 halo-staged convs
    (conv1d_halo.hip) against the same batches through conv_gemm, and against the per-conv launches.
    T = 5 gives clips shorter than a 128-row tile at C = 128, T = 40 ragged tiles."""
    sd = synth.synth_generator_state(11, HIFIGAN_H)
    mel = synth.synth_mel_log(B, 64, T, seed=B * 7 + T)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, HIFIGAN_H, torch.from_numpy(mel)).numpy()
    monkeypatch.setenv("M2S_MRF_BATCH", "1")
    bat = rt.VocoderEngine(sd, HIFIGAN_H, dtype="bf16x3", device=DEV).forward(torch.from_numpy(mel).to(DEV))
    monkeypatch.setenv("M2S_MRF_HALO", "0")  # the same batches through conv_gemm's implicit GEMM
    gem = rt.VocoderEngine(sd, HIFIGAN_H, dtype="bf16x3", device=DEV).forward(torch.from_numpy(mel).to(DEV))
    np.testing.assert_allclose(bat.cpu().numpy(), gem.cpu().numpy(), atol=2e-5, rtol=0)
    monkeypatch.setenv("M2S_MRF_BATCH", "0")
    per = rt.VocoderEngine(sd, HIFIGAN_H, dtype="bf16x3", device=DEV).forward(torch.from_numpy(mel).to(DEV))
    bat, per = bat.cpu().numpy(), per.cpu().numpy()
    np.testing.assert_allclose(bat, ref, atol=1e-4, rtol=0)
    # the two round hi/lo at different points (lrelu before vs after the split, the residual
    # recovered from lrelu(x)): 17-bit values through 20 convs, ~3e-5 apart at most
    np.testing.assert_allclose(bat, per, atol=6e-5, rtol=0)
    assert np.abs(bat - ref).max() <= 1.5 * np.abs(per - ref).max() + 1e-5



def test_effnet_bf16x3_se_gemm128_path(rt, ac_state, monkeypatch):
    """The A/B split SE-gated conv_pwl (gemm128.hip KIND_SP_SE: 128-byte [hi|lo] K-step rows, gate applied to
    the activation fragments in registers; engine switch M2S_SE_SP=1) holds every IR block's tap and the GAP
    features to the fp32 bar at 7 frames (odd count: the 8x8 stage's last two-image tile is half empty)."""
    monkeypatch.setenv("M2S_SE_SP", "1")
    sd = {k: torch.from_numpy(v) for k, v in ac_state.items()}
    fr = torch.from_numpy(synth.synth_frames(1, 7, seed=12)[0])
    taps = []
    effnet.effnet_features(sd, fr, taps=taps)
    eng = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    x = fr.to(DEV)
    for i in range(9, len(taps)):  # blocks.3.0 on: the IR blocks
        got = eng.probe(x, i).cpu().numpy()
        assert _rel(got, taps[i].numpy()) <= 1e-4, f"block {i}: rel err {_rel(got, taps[i].numpy())}"
    assert _rel(eng.effnet(x).cpu().numpy(), effnet.effnet_gap(sd, fr).numpy()) <= 1e-4


@pytest.mark.parametrize("n", [5, 300, 600])
def test_se_ws_matches_barrier_ring(rt, ac_state, monkeypatch, n):
    """The SE-gated conv_pwl on the warp-specialised flag ring (se_ws.hip: loader / consumer waves, FULL /
    FREE counters in LDS, the ring running across tiles) against conv_gemm's barrier ring (M2S_SE_WS=0):
    the same split fp32 products in the same K order, so the two agree to the last split rounding.
    5 frames: a half-empty last 8x8 tile; 300 / 600: more 16x16 / 8x8 tiles than workgroups (each
    workgroup walks several tiles and its ring carries over)."""
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=41)[0]).to(DEV)
    monkeypatch.setenv("M2S_SE_WS", "1")
    monkeypatch.setenv("M2S_SEWS_MIN", "0")  # se_ws at any pass size (the product runs it from a full round of tiles)
    monkeypatch.setenv("M2S_KSPLIT", "1")    # the barrier ring unsplit: the same K order as the flag ring
    monkeypatch.setenv("M2S_IRWS_F32", "0")  # and the same split operand (ir_ws at 600 frames hands se_ws fp32 rows)
    monkeypatch.setenv("M2S_SEWS_HALF", "1")  # the tail's half tiles (300 / 600 frames: 44 / 88 tiles past the last
    ws = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)  # full round), off in the product
    monkeypatch.setenv("M2S_SE_WS", "0")
    ring = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    for i in (13, 18, 20, 28):  # after blocks 4.0 (16x16, no skip), 4.5, 5.1 (8x8, skip), 5.9
        a, b = ws.probe(fr, i).cpu().numpy(), ring.probe(fr, i).cpu().numpy()
        assert np.isfinite(a).all() and _rel(a, b) <= 1e-5, f"tap {i}: {_rel(a, b)}"
    assert _rel(ws.effnet(fr).cpu().numpy(), ring.effnet(fr).cpu().numpy()) <= 1e-5
    if n == 5:  # and against the fp32 oracle
        sd = {k: torch.from_numpy(v) for k, v in ac_state.items()}
        ref = effnet.effnet_gap(sd, fr.cpu()).numpy()
        assert _rel(ws.effnet(fr).cpu().numpy(), ref) <= 1e-4



@pytest.mark.parametrize("n", [520])
def test_ir_ws_fp32_handoff_matches_split(rt, ac_state, monkeypatch, n):
    """ir_ws -> se_ws hands the expanded depthwise map over as plain fp32 rows (launch_ir_ws fm32, se_ws XF): one
    16-byte store per 4 channels and no split in ir_ws's consumers, the gate applied to the fp32 value before se_ws's
    one split.  Against the split hand-off (M2S_IRWS_F32=0) the only difference is the dropped 17-bit rounding of the
    map, so every tap agrees within the parity bar; the launch log shows the XF se_ws."""
    from m2s import _native
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=43)[0]).to(DEV)
    f32 = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    monkeypatch.setenv("M2S_IRWS_F32", "0")
    spl = rt.AcousticEngine(ac_state, dtype="bf16x3", device=DEV)
    _native.prof_enable(True)
    f32.effnet(fr)
    torch.cuda.synchronize()
    names = {r["name"] for r in _native.prof_launches()}
    _native.prof_enable(False)
    assert any(k.startswith("ir_ws_kernel") for k in names), names
    assert any(k.endswith("false, true>") and k.startswith("se_ws_kernel") for k in names), names
    for i in (13, 18, 19, 20, 28):  # after blocks 4.0, 4.5, 5.0 (stride 2), 5.1, 5.9
        a, b = f32.probe(fr, i).cpu().numpy(), spl.probe(fr, i).cpu().numpy()
        assert np.isfinite(a).all() and _rel(a, b) <= 1e-4, f"tap {i}: {_rel(a, b)}"
