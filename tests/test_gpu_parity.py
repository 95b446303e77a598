"""HIP path (libm2s through its C ABI) vs the CPU oracle / reference golden vectors.  GPU box only.

Tolerances (fp32 path; the reference runs fp32 on CPU):
  * vocoder waveform       max |dwav|  <= 1e-4        (tanh output in [-1, 1])
  * BiLSTM / head          max |dy|    <= 2e-5 / 5e-5
  * CNN features / taps    max |d| / max|ref| <= 1e-4 (relative to the tensor's scale)
  * mel_norm end to end    max |d|     <= 1e-4 ; mel_log <= 5e-4 (x ln10/10 * std amplification)
bf16 path (compute dtype of configs[1]): waveform SNR >= 25 dB, mel cosine >= 0.999 / max |d| <= 5e-2.
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


def _snr_db(ref, x):
    ref, x = np.asarray(ref, np.float64), np.asarray(x, np.float64)
    return 10 * np.log10(np.sum(ref ** 2) / max(np.sum((ref - x) ** 2), 1e-30))


@pytest.fixture(scope="module")
def rt():
    from m2s import runtime
    return runtime


@pytest.fixture(scope="module")
def ac_state():
    g = _gold("acoustic.npz")
    return int(g["seed"]), synth.synth_acoustic_state(int(g["seed"]))


@pytest.fixture(scope="module")
def ac_f32(rt, ac_state):
    return rt.AcousticEngine(ac_state[1], dtype="fp32", device=DEV)


@pytest.fixture(scope="module")
def ac_bf16(rt, ac_state):
    return rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)


# ------------------------------------------------------------------------------ vocoder
@pytest.mark.parametrize("case", ["r1", "r2"])
def test_vocoder_fp32_matches_reference_golden(rt, case):
    g = _gold("generator.npz")
    h = json.loads(bytes(g[f"{case}_h"]).decode())
    voc = rt.VocoderEngine(synth.synth_generator_state(int(g["seed"]), h), h, dtype="fp32", device=DEV)
    wav = voc.forward(torch.from_numpy(g[f"{case}_mel"]).to(DEV)).cpu().numpy()
    assert wav.shape == g[f"{case}_wav"].shape
    np.testing.assert_allclose(wav, g[f"{case}_wav"], atol=1e-4, rtol=0)


def test_vocoder_fp32_long_and_layouts(rt):
    g = _gold("generator.npz")
    h = json.loads(bytes(g["r1_h"]).decode())
    voc = rt.VocoderEngine(synth.synth_generator_state(int(g["seed"]), h), h, dtype="fp32", device=DEV)
    mel = torch.from_numpy(g["r1_mel30"]).to(DEV)
    np.testing.assert_allclose(voc.forward(mel).cpu().numpy(), g["r1_wav30"], atol=1e-4, rtol=0)
    nlc = voc.forward(mel.transpose(1, 2).contiguous(), layout=1).cpu().numpy()
    np.testing.assert_allclose(nlc, g["r1_wav30"], atol=1e-4, rtol=0)


@pytest.mark.parametrize("B,T", [(1, 1), (3, 17), (2, 64)])
def test_vocoder_fp32_vs_oracle_shapes(rt, B, T):
    h = HIFIGAN_H
    sd = synth.synth_generator_state(5, h)
    voc = rt.VocoderEngine(sd, h, dtype="fp32", device=DEV)
    mel = synth.synth_mel_log(B, 64, T, seed=B * 100 + T)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, h, torch.from_numpy(mel)).numpy()
    wav = voc.forward(torch.from_numpy(mel).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(wav, ref, atol=1e-4, rtol=0)


def test_vocoder_bf16_snr(rt):
    h = HIFIGAN_H
    sd = synth.synth_generator_state(5, h)
    voc = rt.VocoderEngine(sd, h, dtype="bf16", device=DEV)
    mel = synth.synth_mel_log(2, 64, 30, seed=9)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, h, torch.from_numpy(mel)).numpy()
    wav = voc.forward(torch.from_numpy(mel).to(DEV)).cpu().numpy()
    assert _snr_db(ref, wav) >= 25.0


@pytest.mark.parametrize("B,T", [(1, 1), (3, 17), (2, 64)])
def test_vocoder_bf16_mrf_fused(rt, monkeypatch, B, T):
    """The fused ResBlock1 kernel (mrf_fused.hip: the C=64 and C=32 MRF stages, one launch per
    resblock) against the fp32 oracle and against the per-conv bf16 path: clips shorter than one
    tile (T=1: 420 samples), ragged last tiles, several clips.  Both bf16 paths round at different
    points, so the bar is the oracle SNR, and the fused path may not lose more than 1.5 dB."""
    h = HIFIGAN_H
    sd = synth.synth_generator_state(7, h)
    mel = synth.synth_mel_log(B, 64, T, seed=B * 10 + T)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, h, torch.from_numpy(mel)).numpy()
    monkeypatch.setenv("M2S_MRF_FUSED", "1")
    fused = rt.VocoderEngine(sd, h, dtype="bf16", device=DEV).forward(torch.from_numpy(mel).to(DEV)).cpu().numpy()
    monkeypatch.setenv("M2S_MRF_FUSED", "0")
    plain = rt.VocoderEngine(sd, h, dtype="bf16", device=DEV).forward(torch.from_numpy(mel).to(DEV)).cpu().numpy()
    s_f, s_p = _snr_db(ref, fused), _snr_db(ref, plain)
    assert np.isfinite(fused).all()
    assert s_f >= 25.0 and s_f >= s_p - 1.5, (s_f, s_p)


# ------------------------------------------------------------------------------ BiLSTM + head
@pytest.mark.parametrize("bt", ["2x7", "1x1", "8x4", "1x30"])
def test_bilstm_head_matches_reference_golden(ac_f32, bt):
    g = _gold("acoustic.npz")
    y, m = ac_f32.bilstm(torch.from_numpy(g[f"lstm_{bt}_in"]).to(DEV))
    np.testing.assert_allclose(y.cpu().numpy(), g[f"lstm_{bt}_y"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(m.cpu().numpy(), g[f"lstm_{bt}_head"], atol=5e-5, rtol=0)


def test_bilstm_batch_over_32(ac_f32, ac_state):
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    x = torch.from_numpy(np.random.default_rng(1).normal(0, 0.5, (37, 5, 208)).astype(np.float32))
    ref_y = acoustic.bilstm_summerge(sd, x)
    y, m = ac_f32.bilstm(x.to(DEV))
    np.testing.assert_allclose(y.cpu().numpy(), ref_y.numpy(), atol=2e-5, rtol=0)
    np.testing.assert_allclose(m.cpu().numpy(), acoustic.head(sd, ref_y).numpy(), atol=5e-5, rtol=0)


@pytest.mark.parametrize("B,T", [(1, 30), (8, 4), (2, 32), (3, 40)])
def test_bilstm_small_pass_projection(ac_f32, ac_state, B, T):
    """Passes of <= 64 frames run the fp32 BiLSTM input projection with its K chunks split over the four waves of a
    row tile (conv_igemm.hip kw, ConvArgs::kwave); larger passes keep one wave per row group.  Both against the
    oracle at the fp32 bar, and the same clip inside a > 64-frame batch agrees with itself alone to fp32 rounding."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    x = torch.from_numpy(np.random.default_rng(7 + B).normal(0, 0.5, (B, T, 208)).astype(np.float32))
    ref_y = acoustic.bilstm_summerge(sd, x)
    y, m = ac_f32.bilstm(x.to(DEV))
    np.testing.assert_allclose(y.cpu().numpy(), ref_y.numpy(), atol=2e-5, rtol=0)
    np.testing.assert_allclose(m.cpu().numpy(), acoustic.head(sd, ref_y).numpy(), atol=5e-5, rtol=0)
    extra = max(4, 70 // T)
    big = torch.cat([x, torch.from_numpy(np.random.default_rng(99).normal(0, 0.5, (extra, T, 208)).astype(np.float32))])
    assert big.shape[0] * T > 64
    yb, _ = ac_f32.bilstm(big.to(DEV))
    np.testing.assert_allclose(yb[:B].cpu().numpy(), y.cpu().numpy(), atol=1e-5, rtol=0)


# ------------------------------------------------------------------------------ CNN encoder
def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-6))


def test_effnet_every_block_fp32(ac_f32, ac_state):
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    fr = torch.from_numpy(synth.synth_frames(1, 2, seed=4)[0])
    taps = []
    effnet.effnet_features(sd, fr, taps=taps)
    x = fr.to(DEV)
    for i, ref in enumerate(taps):
        got = ac_f32.probe(x, i).cpu().numpy()
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        assert _rel(got, ref.numpy()) <= 1e-4, f"block {i}: rel err {_rel(got, ref.numpy())}"


@pytest.mark.parametrize("hw", [(256, 256), (96, 80), (67, 101)])
def test_effnet_gap_fp32_sizes(ac_f32, ac_state, hw):
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    fr = torch.from_numpy(synth.synth_frames(1, 3, hw=hw, seed=8)[0])
    ref = effnet.effnet_gap(sd, fr).numpy()
    got = ac_f32.effnet(fr.to(DEV)).cpu().numpy()
    assert _rel(got, ref) <= 1e-4


def test_effnet_chunking_is_exact(rt, ac_state):
    eng = rt.AcousticEngine(ac_state[1], dtype="fp32", device=DEV, chunk=2)
    ref_eng = rt.AcousticEngine(ac_state[1], dtype="fp32", device=DEV, chunk=256)
    fr = torch.from_numpy(synth.synth_frames(1, 5, seed=12)[0]).to(DEV)
    assert torch.equal(eng.effnet(fr), ref_eng.effnet(fr))
    # 33 frames at chunk 16: two passes of 17 (one pass fewer of <= chunk + chunk / 16 frames) instead of 16, 16, 1
    eng16 = rt.AcousticEngine(ac_state[1], dtype="fp32", device=DEV, chunk=16)
    fr = torch.from_numpy(synth.synth_frames(1, 33, seed=13)[0]).to(DEV)
    assert torch.equal(eng16.effnet(fr), ref_eng.effnet(fr))


def test_effnet_bf16_close(ac_bf16, ac_state):
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    fr = torch.from_numpy(synth.synth_frames(1, 4, seed=8)[0])
    ref = effnet.effnet_gap(sd, fr).numpy()
    got = ac_bf16.effnet(fr.to(DEV)).cpu().numpy()
    cos = float((got * ref).sum() / np.sqrt((got ** 2).sum() * (ref ** 2).sum()))
    assert cos >= 0.999, cos


def _cos(a, b):
    return float((a * b).sum() / np.sqrt((a ** 2).sum() * (b ** 2).sum()))


@pytest.mark.parametrize("hw", [(256, 256), (256, 128), (96, 80), (67, 101)])
def test_effnet_bf16_ir_fused_every_block(rt, ac_state, monkeypatch, hw):
    """The fused conv_pw+conv_dw+SE-squeeze kernel (ir_fused.hip) against the unfused bf16
    sequence and the fp32 oracle, block by block (both bf16 paths round the expanded activation
    to bf16 at the same point, so they agree to accumulation order)."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    fr = torch.from_numpy(synth.synth_frames(1, 3, hw=hw, seed=31)[0])
    taps = []
    effnet.effnet_features(sd, fr, taps=taps)
    monkeypatch.setenv("M2S_IR_FUSED", "1")
    fused = rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)
    monkeypatch.setenv("M2S_IR_FUSED", "0")
    plain = rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)
    x = fr.to(DEV)
    for i, ref in enumerate(taps):
        a = fused.probe(x, i).float().cpu().numpy()
        b = plain.probe(x, i).float().cpu().numpy()
        assert _rel(a, b) <= 2e-2, f"block {i}: fused vs unfused rel {_rel(a, b)}"
        assert _cos(a, ref.numpy()) >= 0.999, f"block {i}: cos vs oracle {_cos(a, ref.numpy())}"
    ga = fused.effnet(x).cpu().numpy()
    gb = plain.effnet(x).cpu().numpy()
    assert _cos(ga, gb) >= 0.99999


def test_effnet_bf16_ir_s2band_matches_unfused(rt, ac_state, monkeypatch):
    """blocks.3.0 in bf16 as one banded kernel (ir_s2band.hip SP = 0) against conv_pw + dwconv + se_mean
    (M2S_IR_S2BAND=0): the banded kernel keeps the expanded activation fp32 in LDS where the unfused
    sequence stores it as bf16, so they agree to bf16 rounding; both at the bf16 cosine bar vs the oracle."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    fr = torch.from_numpy(synth.synth_frames(1, 3, seed=19)[0])
    taps = []
    effnet.effnet_features(sd, fr, taps=taps)
    band = rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)
    monkeypatch.setenv("M2S_IR_S2BAND", "0")
    plain = rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)
    x = fr.to(DEV)
    for i in (9, 10):
        a, b = band.probe(x, i).float().cpu().numpy(), plain.probe(x, i).float().cpu().numpy()
        assert np.isfinite(a).all() and _rel(a, b) <= 2e-2, (i, _rel(a, b))
        assert _cos(a, taps[i].numpy()) >= 0.999, (i, _cos(a, taps[i].numpy()))
    assert _cos(band.effnet(x).cpu().numpy(), plain.effnet(x).cpu().numpy()) >= 0.99999


@pytest.mark.parametrize("env,blocks", [("M2S_STEM_FUSED", (2, 3, 6, -1)), ("M2S_SE_FUSED", (9, 14, 20, -1)), ("M2S_IR_FUSED", (9, 10, 18, 19, -1)),
                                        ("M2S_ER_FUSED", (3, 4, 5, 6, 7, 8, -1))])
@pytest.mark.parametrize("hw", [(256, 256), (96, 80), (67, 101)])
def test_effnet_bf16_fused_kernels_vs_unfused(rt, ac_state, monkeypatch, hw, env, blocks):
    """The fused stem + blocks.0 kernel (stem_b0.hip), the one-kernel SE excitation (se_excite.hip)
    the fused EdgeResidual (er_fused.hip / er2_fused.hip: blocks.1.1/.2 at 64x64, blocks.2.1/.2 at 32x32;
    ers2_fused.hip: the stride-2 blocks.1.0 / blocks.2.0)
    against the separate launches they replace and the fp32 oracle, block by block
    and on the pooled features; odd sizes exercise the TF-SAME bottom/right stem pad and partial
    16 x 16 tiles, and a 3-frame batch a partial 8-image SE group."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    fr = torch.from_numpy(synth.synth_frames(1, 3, hw=hw, seed=47)[0])
    taps = []
    effnet.effnet_features(sd, fr, taps=taps)
    monkeypatch.setenv(env, "1")
    fused = rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)
    monkeypatch.setenv(env, "0")
    plain = rt.AcousticEngine(ac_state[1], dtype="bf16", device=DEV)
    x = fr.to(DEV)
    for i in [b if b >= 0 else len(taps) - 1 for b in blocks]:
        a = fused.probe(x, i).float().cpu().numpy()
        b = plain.probe(x, i).float().cpu().numpy()
        assert np.isfinite(a).all()
        assert _rel(a, b) <= 2e-2, f"block {i}: fused vs unfused rel {_rel(a, b)}"
        assert _cos(a, taps[i].numpy()) >= 0.999, f"block {i}: cos vs oracle {_cos(a, taps[i].numpy())}"
    assert _cos(fused.effnet(x).cpu().numpy(), plain.effnet(x).cpu().numpy()) >= 0.99999


# ------------------------------------------------------------------------------ acoustic model / pipeline
def test_acoustic_forward_matches_reference_wiring(ac_f32):
    g = _gold("acoustic.npz")
    fr = synth.synth_frames(2, 3, seed=int(g["model_frames_seed"]))
    out = ac_f32.forward(torch.from_numpy(fr[:1]).unsqueeze(2).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(out, g["model_out"], atol=1e-4, rtol=0)
    out4 = ac_f32.forward(torch.from_numpy(fr[:, :2]).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(out4, g["model_out4d"], atol=1e-4, rtol=0)


def test_mel_glue_matches_reference_golden(rt):
    g = _gold("glue.npz")
    db, ln = rt.mel_glue(torch.from_numpy(g["pred_norm"]).to(DEV), torch.from_numpy(g["scaler_mean"]),
                         torch.from_numpy(g["scaler_std"]))
    np.testing.assert_array_equal(db.cpu().numpy(), g["mel_db"])
    np.testing.assert_allclose(ln.cpu().numpy(), g["mel_log"], atol=2e-6, rtol=0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_pipeline_end_to_end(rt, ac_state, dtype):
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    gsd = synth.synth_generator_state(3)
    mean, std = synth.synth_scaler()
    ac = rt.AcousticEngine(ac_state[1], dtype=dtype, device=DEV)
    voc = rt.VocoderEngine(gsd, HIFIGAN_H, dtype=dtype, device=DEV)
    pipe = rt.Pipeline(ac, voc, mean, std)
    fr = synth.synth_frames(2, 6, seed=21)
    out = pipe.forward(torch.from_numpy(fr).to(DEV))
    # oracle: reference graph on CPU
    B, T = fr.shape[:2]
    f = effnet.effnet_gap(sd, torch.from_numpy(fr).reshape(B * T, 256, 256)).view(B, T, -1)
    mn = acoustic.head(sd, acoustic.bilstm_summerge(sd, f))
    db = acoustic.denormalize_mel(mn, mean, std)
    ln = acoustic.mel_db_to_log(db)
    wav = hifigan.generator({k: torch.from_numpy(v) for k, v in gsd.items()}, HIFIGAN_H, ln.transpose(1, 2))
    got = {k: v.cpu().numpy() for k, v in out.items()}
    if dtype == "fp32":
        np.testing.assert_allclose(got["mel_norm"], mn.numpy(), atol=1e-4, rtol=0)
        np.testing.assert_allclose(got["mel_db"], db.numpy(), atol=2e-3, rtol=0)
        np.testing.assert_allclose(got["mel_log"], ln.numpy(), atol=5e-4, rtol=0)
        np.testing.assert_allclose(got["wav"], wav[:, 0].numpy(), atol=1e-4, rtol=0)
    else:
        assert np.abs(got["mel_norm"] - mn.numpy()).max() <= 5e-2
        assert _snr_db(wav[:, 0].numpy(), got["wav"]) >= 20.0


# ------------------------------------------------------------------------------ persistent BiLSTM
@pytest.mark.parametrize("B,T", [(1, 1000), (3, 64), (4, 40), (70, 6), (8, 1000), (5, 17), (20, 33), (64, 30),
                                 (64, 200), (12, 33), (16, 200), (9, 1000)])
def test_bilstm_persistent_long_and_wide(rt, ac_state, monkeypatch, B, T):
    """One-launch recurrence (lstm_persistent.hip) vs the oracle and vs the per-step kernel:
    B <= 4 runs the granule-exchange lstm_small_kernel (1 x 1000 = configs[4]'s clip length); 4 < B
    <= 16 the chunked granule-exchange lstm_mid_kernel, 4-sequence chunks up to B = 8 (8 x 1000 =
    configs[4]'s per-GPU batch, a ragged last chunk at 5) and 8-sequence chunks above (12 x 33 and
    9 x 1000 with ragged last chunks, 16 x 200 full); B > 16 the counter-barrier kernel (20 x 33, the
    bench's 64 x 30, 70 x 6)."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    x = torch.from_numpy(np.random.default_rng(B * 7 + T).normal(0, 0.5, (B, T, 208)).astype(np.float32))
    monkeypatch.setenv("M2S_LSTM_PERSISTENT", "1")
    y, m = rt.AcousticEngine(ac_state[1], dtype="fp32", device=DEV).bilstm(x.to(DEV))
    monkeypatch.setenv("M2S_LSTM_PERSISTENT", "0")
    y_step, _ = rt.AcousticEngine(ac_state[1], dtype="fp32", device=DEV).bilstm(x.to(DEV))
    ref_y = acoustic.bilstm_summerge(sd, x).numpy()
    y = y.cpu().numpy()
    assert np.isfinite(y).all()
    tol = 2e-5 if T <= 64 else 1e-4  # fp32 summation order over 1000 recurrent steps
    np.testing.assert_allclose(y, ref_y, atol=tol, rtol=0)
    np.testing.assert_allclose(y, y_step.cpu().numpy(), atol=tol, rtol=0)
    np.testing.assert_allclose(m.cpu().numpy(), acoustic.head(sd, torch.from_numpy(ref_y)).numpy(), atol=5 * tol, rtol=0)


@pytest.mark.parametrize("B,T", [(5, 17), (8, 1000), (12, 33), (16, 200), (17, 1), (20, 33), (64, 30), (64, 200),
                                 (70, 6), (40, 1000)])
def test_bilstm_split_x3(rt, ac_state, monkeypatch, B, T):
    """B > 4 in the split-fp32 engines (lstm_x3_kernel): three bf16 MFMA terms over W_hh and h split
    hi / lo, h_t handed over by write-through stores behind per-workgroup flags.  Against the oracle and
    the exact-product f32 kernel (M2S_LSTM_X3=0) in the same engine; the split costs ~2^-16 per product,
    so the bar is the split engines' 1e-4 (a 64-sequence full launch, a ragged 6-sequence second launch at
    70, one sequence half at 5-20, configs[4]'s 8 x 1000, 1000 recurrent steps at 40)."""
    sd = {k: torch.from_numpy(v) for k, v in ac_state[1].items()}
    x = torch.from_numpy(np.random.default_rng(B * 11 + T).normal(0, 0.5, (B, T, 208)).astype(np.float32))
    monkeypatch.setenv("M2S_LSTM_X3", "1")
    y, m = rt.AcousticEngine(ac_state[1], dtype="bf16x3", device=DEV).bilstm(x.to(DEV))
    monkeypatch.setenv("M2S_LSTM_X3", "0")
    y_f32, _ = rt.AcousticEngine(ac_state[1], dtype="bf16x3", device=DEV).bilstm(x.to(DEV))
    ref_y = acoustic.bilstm_summerge(sd, x).numpy()
    y = y.cpu().numpy()
    assert np.isfinite(y).all()
    np.testing.assert_allclose(y, ref_y, atol=1e-4, rtol=0)
    np.testing.assert_allclose(y, y_f32.cpu().numpy(), atol=1e-4, rtol=0)
    np.testing.assert_allclose(m.cpu().numpy(), acoustic.head(sd, torch.from_numpy(ref_y)).numpy(), atol=5e-4, rtol=0)
    print(f"lstm_x3 B={B} T={T}: max |d| vs oracle {np.abs(y - ref_y).max():.2e}")


@pytest.mark.parametrize("B,T", [(5, 17), (8, 1000), (16, 200)])
def test_bilstm_x3g_matches_flag_handoff(rt, ac_state, monkeypatch, B, T):
    """5..16 sequences in the split engines run lstm_x3g_kernel: lstm_x3's split arithmetic with h_t handed over as
    data-tagged granules {step + 1 | hi | lo} swept into LDS instead of write-through rows behind per-workgroup flags.
    The products, their order and the K-slice sums are lstm_x3's, so the two agree to fp32 rounding of the same
    operations; the launch log names the kernel."""
    from m2s import _native
    x = torch.from_numpy(np.random.default_rng(B * 7 + T).normal(0, 0.5, (B, T, 208)).astype(np.float32)).to(DEV)
    eng = rt.AcousticEngine(ac_state[1], dtype="bf16x3", device=DEV)
    _native.prof_enable(True)
    y, _ = eng.bilstm(x)
    torch.cuda.synchronize()
    names = {r["name"] for r in _native.prof_launches()}
    _native.prof_enable(False)
    assert "lstm_x3g_kernel" in names, names
    monkeypatch.setenv("M2S_LSTM_X3G", "0")
    y3, _ = rt.AcousticEngine(ac_state[1], dtype="bf16x3", device=DEV).bilstm(x)
    eng.check()
    np.testing.assert_allclose(y.cpu().numpy(), y3.cpu().numpy(), atol=1e-5, rtol=0)


# ------------------------------------------------------------------------------ frame preprocessing
def test_preprocess_matches_reference_golden(rt):
    """Device _preprocess_frame (preprocess.hip) vs the reference's own outputs (glue.npz)."""
    g = _gold("glue.npz")
    out = rt.preprocess_frames(torch.from_numpy(g["frames_u8"]).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(out, g["preprocessed"], atol=1e-6, rtol=0)


@pytest.mark.parametrize("shape", [(5, 256, 256), (2, 67, 101), (3, 256, 256, 3)])
def test_preprocess_vs_oracle_shapes_and_bgr(rt, shape):
    rng = np.random.default_rng(len(shape) * 100 + shape[1])
    u8 = rng.integers(0, 256, size=shape, dtype=np.uint8)
    u8[0] = 77  # a constant frame: zeros (reference :52-53)
    out = rt.preprocess_frames(torch.from_numpy(u8).to(DEV)).cpu().numpy()
    grey = np.stack([acoustic.bgr_to_grey(f) for f in u8]) if len(shape) == 4 else u8
    ref = np.stack([acoustic.preprocess_frame(f) for f in grey])
    assert out.shape == ref.shape and not out[0].any()
    np.testing.assert_allclose(out, ref, atol=1e-6, rtol=0)


def test_bilstm_epoch_tags_across_calls(rt, ac_state):
    """The granule BiLSTM kernels (lstm_small B = 1, lstm_x3g B = 5..16) keep one sync buffer per engine whose tags
    continue an epoch count instead of a memset per call (lstm_persistent.hip lstm_epoch): calls of both kinds and
    different lengths interleaved on one engine give bit-identical outputs to fresh engines (a stale granule of an
    earlier call never passes for a current one)."""
    eng = rt.AcousticEngine(ac_state[1], dtype="bf16x3", device=DEV)
    xs = [torch.randn(b, t, 208, device=DEV, generator=torch.Generator(device=DEV).manual_seed(40 + i))
          for i, (b, t) in enumerate([(1, 30), (8, 50), (1, 31), (8, 17), (12, 30)])]
    want = []
    for x in xs:
        fresh = rt.AcousticEngine(ac_state[1], dtype="bf16x3", device=DEV)
        want.append(fresh.bilstm(x)[0].cpu())
        fresh.check()
    for rnd in range(3):
        for x, w in zip(xs, want):
            y = eng.bilstm(x)[0].cpu()
            eng.check()
            assert torch.equal(y, w), (rnd, tuple(x.shape))


# ------------------------------------------------------------------------------ asynchronous failure report
@pytest.mark.parametrize("B,dtype", [(1, "fp32"), (8, "fp32"), (12, "fp32"), (70, "fp32"), (8, "bf16x3"), (70, "bf16x3")])
def test_bilstm_barrier_timeout_is_reported(rt, ac_state, B, dtype):
    """A BiLSTM hand-off wait that times out (forced: spin limit 0 = the first wait fails) poisons the outputs and is
    reported: m2s_acoustic_status -> M2SError, and the next forward on the engine fails too.  B = 1:
    lstm_small_kernel, 8 / 12: lstm_mid_kernel with 4- / 8-sequence chunks (granule sweeps), 70: the counter
    barrier (fp32); 8 bf16x3: the granule hand-off of lstm_x3g_kernel, 70 bf16x3: the flag hand-off of lstm_x3_kernel."""
    import ctypes
    from m2s import _native
    eng = rt.AcousticEngine(ac_state[1], dtype=dtype, device=DEV)
    _native.check(_native.lib().m2s_acoustic_set_lstm_spin_limit(ctypes.c_void_p(eng.handle), 0))
    x = torch.randn(B, 30, 208, device=DEV)
    y, _ = eng.bilstm(x)
    with pytest.raises(_native.M2SError, match="timed out"):
        eng.check()
    assert torch.isnan(y).any()
    eng.check()  # the report is consumed once
    _native.check(_native.lib().m2s_acoustic_set_lstm_spin_limit(ctypes.c_void_p(eng.handle), 1 << 24))
    y2, _ = eng.bilstm(x)
    eng.check()
    assert torch.isfinite(y2).all()


@pytest.mark.parametrize("dtype", ["bf16x3", "fp8"])
def test_ws_flag_timeout_is_reported(rt, ac_state, dtype, monkeypatch):
    """The persistent CNN kernels' LDS flag waits (ir_ws producers' weight-slot wait, se_ws FULL / FREE) are bounded;
    forced to time out (spin limit 0 = every wait fails), the launch poisons its outputs and reports it:
    m2s_acoustic_status -> M2SError naming the flag ring, then a normal limit gives finite features again.
    bf16x3: ir_ws + the split se_ws; fp8: the e4m3 se_ws."""
    import ctypes
    from m2s import _native
    monkeypatch.setenv("M2S_IRWS_MIN", "0")  # the persistent kernels at this 4-frame pass (the product's small-pass
    monkeypatch.setenv("M2S_SEWS_MIN", "0")  # plan runs the grid forms there)
    eng = rt.AcousticEngine(ac_state[1], dtype=dtype, device=DEV)
    fr = torch.rand(4, 256, 256, device=DEV)
    _native.check(_native.lib().m2s_acoustic_set_ws_spin_limit(ctypes.c_void_p(eng.handle), 0))
    f = eng.effnet(fr)
    with pytest.raises(_native.M2SError, match="flag-ring"):
        eng.check()
    assert torch.isnan(f).any()
    eng.check()  # the report is consumed once
    _native.check(_native.lib().m2s_acoustic_set_ws_spin_limit(ctypes.c_void_p(eng.handle), 1 << 20))
    f2 = eng.effnet(fr)
    eng.check()
    assert torch.isfinite(f2).all()
