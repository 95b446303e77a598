"""fp8 path (configs[4]: "fp8 MFMA CNN encoder + HiFi-GAN MRF dilated-conv path, >=1000-frame clips").

M2S_DT_FP8 (include/m2s.h): OCP e4m3 storage and block-scaled e4m3 MFMA
(v_mfma_scale_f32_16x16x128_f8f6f4, per-output-channel fp32 weight scales) in the fp8 engine's e4m3
kernels; the remaining convs run the bf16 path.  Tolerance: cosine similarity >= 0.99 against
the fp32 oracle for the mel at 1 x 1000 frames; the vocoder's wav is held to the same cosine.  The
measured values are printed (pytest -s).  GPU box only.
"""
import numpy as np
import pytest
import torch

from m2s import synth
from m2s.config import HIFIGAN_H
from oracle import acoustic, effnet, hifigan

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
COS_MIN = 0.99


def _cos(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))


@pytest.fixture(scope="module")
def rt():
    from m2s import runtime
    return runtime


@pytest.fixture(scope="module")
def clip1000():
    """1 x 1000 frames at 256 x 256 (configs[4] length) and the oracle's features, mel."""
    st = synth.synth_acoustic_state(11)
    sd = {k: torch.from_numpy(v) for k, v in st.items()}
    fr = synth.synth_frames(1, 1000, seed=5)
    torch.set_num_threads(16)
    f = torch.cat([effnet.effnet_gap(sd, torch.from_numpy(fr[0, i:i + 100])) for i in range(0, 1000, 100)]).view(1, 1000, -1)
    mn = acoustic.head(sd, acoustic.bilstm_summerge(sd, f)).numpy()
    return st, fr, f.numpy(), mn


def test_effnet_fp8_features_cosine(rt, clip1000):
    st, fr, f_ref, _ = clip1000
    eng = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    f = eng.effnet(torch.from_numpy(fr[0]).to(DEV)).cpu().numpy()
    c = _cos(f, f_ref[0])
    print(f"\nfp8 effnet GAP features (1000 frames): cos {c:.5f}, rel max {np.abs(f - f_ref[0]).max() / np.abs(f_ref).max():.3e}")
    assert c >= COS_MIN


def test_effnet_fp8_propagates_nan(rt):
    """A NaN pixel must reach the features as NaN (the e4m3 operand saturation keeps NaN), not be
    clamped to -448 and come out as finite data; the clean frames of the same batch stay finite."""
    st = synth.synth_acoustic_state(3)
    eng = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    fr = torch.from_numpy(synth.synth_frames(1, 4, seed=2)[0]).to(DEV)
    fr[1, 100, 100] = float("nan")
    f = eng.effnet(fr).cpu()
    assert torch.isnan(f[1]).any()
    assert torch.isfinite(f[[0, 2, 3]]).all()


def test_acoustic_fp8_mel_cosine_1x1000(rt, clip1000):
    st, fr, _, mn_ref = clip1000
    eng = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    mn = eng.forward(torch.from_numpy(fr).to(DEV)).cpu().numpy()
    c = _cos(mn, mn_ref)
    per_frame = min(_cos(mn[0, t], mn_ref[0, t]) for t in range(0, 1000, 37))
    print(f"\nfp8 mel_norm 1x1000: cos {c:.5f} (worst sampled frame {per_frame:.5f}), max|d| {np.abs(mn - mn_ref).max():.3e}")
    assert c >= COS_MIN


def test_vocoder_fp8_wav_cosine_1x1000(rt):
    sd = synth.synth_generator_state(5, HIFIGAN_H)
    mel = synth.synth_mel_log(1, 64, 1000, seed=9)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, HIFIGAN_H, torch.from_numpy(mel)).numpy()
    voc = rt.VocoderEngine(sd, HIFIGAN_H, dtype="fp8", device=DEV)
    wav = voc.forward(torch.from_numpy(mel).to(DEV)).cpu().numpy()
    c = _cos(wav, ref)
    snr = 10 * np.log10((ref ** 2).sum() / max(((wav.reshape(ref.shape) - ref) ** 2).sum(), 1e-30))
    print(f"\nfp8 vocoder 1x1000 frames: wav cos {c:.5f}, SNR {snr:.1f} dB")
    assert c >= COS_MIN


def test_pipeline_fp8_end_to_end_1x1000(rt, clip1000):
    """configs[4] end to end at its clip length: frames -> mel -> wav in ONE fp8 pipeline_forward call
    (e4m3 backbone and MRF convs), mel_norm and wav cosine vs the fp32 oracle of the same clip."""
    st, fr, _, mn_ref = clip1000
    gen_sd = synth.synth_generator_state(5, HIFIGAN_H)
    mean, std = synth.synth_scaler()
    pipe = rt.Pipeline(rt.AcousticEngine(st, dtype="fp8", device=DEV),
                       rt.VocoderEngine(gen_sd, HIFIGAN_H, dtype="fp8", device=DEV), mean, std)
    out = pipe.forward(torch.from_numpy(fr).to(DEV))
    pipe.ac.check()
    ln_ref = acoustic.mel_db_to_log(acoustic.denormalize_mel(torch.from_numpy(mn_ref), mean, std))
    wav_ref = hifigan.generator({k: torch.from_numpy(v) for k, v in gen_sd.items()}, HIFIGAN_H,
                                ln_ref.transpose(1, 2))[:, 0].numpy()
    c_mel, c_wav = _cos(out["mel_norm"].cpu().numpy(), mn_ref), _cos(out["wav"].cpu().numpy(), wav_ref)
    print(f"\nfp8 pipeline 1x1000: mel_norm cos {c_mel:.5f}, wav cos {c_wav:.5f}")
    assert out["wav"].shape == (1, 1000 * 420)
    assert c_mel >= COS_MIN and c_wav >= COS_MIN


def test_vocoder_fp8_ragged_batch_is_batch_invariant(rt):
    """3 clips x 37 frames (stage lengths 370 / 2590 / ..., not multiples of any tile): each clip's wav
    from the batch equals, bit for bit, the wav of that clip alone (the causal taps of the e4m3 MRF convs
    never read across a clip boundary), and each is within the cosine bar of the fp32 oracle."""
    sd = synth.synth_generator_state(7, HIFIGAN_H)
    mel = synth.synth_mel_log(3, 64, 37, seed=4)
    voc = rt.VocoderEngine(sd, HIFIGAN_H, dtype="fp8", device=DEV)
    wav = voc.forward(torch.from_numpy(mel).to(DEV)).cpu().numpy().reshape(3, -1)
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, HIFIGAN_H, torch.from_numpy(mel)).numpy()
    for b in range(3):
        alone = voc.forward(torch.from_numpy(mel[b:b + 1]).to(DEV)).cpu().numpy().reshape(-1)
        assert np.array_equal(alone, wav[b]), b
        assert _cos(wav[b], ref[b]) >= COS_MIN, b


def test_effnet_fp8_odd_batch_per_frame(rt):
    """5 frames: the 8x8 stage's e4m3 SE GEMM runs two-image tiles, the last one half empty; every frame's
    GAP features stay within the cosine bar of the fp32 oracle (per frame, not only over the batch)."""
    st = synth.synth_acoustic_state(4)
    sd = {k: torch.from_numpy(v) for k, v in st.items()}
    fr = synth.synth_frames(1, 5, seed=8)[0]
    ref = effnet.effnet_gap(sd, torch.from_numpy(fr)).numpy()
    f = rt.AcousticEngine(st, dtype="fp8", device=DEV).effnet(torch.from_numpy(fr).to(DEV)).cpu().numpy()
    cs = [_cos(f[i], ref[i]) for i in range(5)]
    print("\nfp8 per-frame feature cos (5 frames):", " ".join(f"{c:.5f}" for c in cs))
    assert min(cs) >= 0.999


def test_effnet_fp8_non_square_frames(rt):
    """256 x 512 frames: the 8 x 16 maps of blocks.5 put two images in an e4m3-output ir_pwdw workgroup
    (ir_group G = 2, the ir_pwdw_kernel<4, 2, 2> variant) in front of the e4m3 SE GEMM; every frame stays
    within the cosine bar of the fp32 oracle."""
    st = synth.synth_acoustic_state(6)
    sd = {k: torch.from_numpy(v) for k, v in st.items()}
    fr = synth.synth_frames(1, 3, hw=(256, 512), seed=12)[0]
    ref = effnet.effnet_gap(sd, torch.from_numpy(fr)).numpy()
    f = rt.AcousticEngine(st, dtype="fp8", device=DEV).effnet(torch.from_numpy(fr).to(DEV)).cpu().numpy()
    cs = [_cos(f[i], ref[i]) for i in range(3)]
    print("\nfp8 per-frame feature cos (256x512):", " ".join(f"{c:.5f}" for c in cs))
    assert min(cs) >= 0.999


@pytest.mark.parametrize("n", [5, 600])
def test_se_ws_f8_matches_gemm128(rt, monkeypatch, n):
    """The fp8 engine's SE-gated conv_pwl on the warp-specialised flag ring (se_ws.hip F8: loader / consumer
    waves, FULL / FREE counters in LDS, ring across tiles) against gemm128.hip's barrier ring (M2S_SE_WS=0):
    the same e4m3 operands and block-scaled MFMAs in the same K order.  5 frames: a half-empty last 8x8 tile;
    600: more tiles than workgroups.  Plus the cosine bar against the fp32 oracle at 5 frames."""
    st = synth.synth_acoustic_state(8)
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=44)[0]).to(DEV)
    ws = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    monkeypatch.setenv("M2S_SE_WS", "0")
    ring = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    for i in (13, 18, 20, 28):  # after blocks 4.0, 4.5, 5.1, 5.9
        a, b = ws.probe(fr, i).cpu().numpy(), ring.probe(fr, i).cpu().numpy()
        rel = float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-6))
        assert np.isfinite(a).all() and rel <= 1e-3, (i, rel)
    if n == 5:
        sd = {k: torch.from_numpy(v) for k, v in st.items()}
        ref = effnet.effnet_gap(sd, fr.cpu()).numpy()
        f = ws.effnet(fr).cpu().numpy()
        assert min(_cos(f[i], ref[i]) for i in range(n)) >= 0.999


@pytest.mark.parametrize("n", [5, 300])
def test_fp8_e4m3_expand(rt, monkeypatch, n):
    """The fp8 engine's stride-1 IR expand (conv_pw + bn1) on e4m3 (ir_pwdw mode 3: the block input as e4m3
    rows written by the previous block's SE GEMM epilogue or converted, per-channel-scaled e4m3 weights,
    v_mfma_scale_f32_16x16x128_f8f6f4) against the bf16 expand (M2S_F8_EXPAND=0) and the fp32 oracle.  One
    more e4m3 rounding per IR block, so the bars are cosines: every probed tap >= 0.995 against the bf16
    expand, pooled features per frame >= 0.995 against the oracle (0.99 end to end)."""
    st = synth.synth_acoustic_state(8)
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=45)[0]).to(DEV)
    monkeypatch.setenv("M2S_F8_EXPAND", "1")
    e8 = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    monkeypatch.setenv("M2S_F8_EXPAND", "0")
    eb = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    for i in (10, 13, 18, 20, 28):  # after blocks 3.1, 4.0, 4.5, 5.1, 5.9
        a, b = e8.probe(fr, i).cpu().numpy(), eb.probe(fr, i).cpu().numpy()
        assert np.isfinite(a).all()
        c = _cos(a.ravel(), b.ravel())
        print(f"tap {i}: cos(e4m3 expand, bf16 expand) {c:.6f}")
        assert c >= 0.995, (i, c)
    if n == 5:
        sd = {k: torch.from_numpy(v) for k, v in st.items()}
        ref = effnet.effnet_gap(sd, fr.cpu()).numpy()
        f = e8.effnet(fr).cpu().numpy()
        cmin = min(_cos(f[i], ref[i]) for i in range(n))
        print(f"features vs oracle: min per-frame cos {cmin:.6f}")
        assert cmin >= 0.995


@pytest.mark.parametrize("n", [5, 300])
def test_fp8_e4m3_edge_residual(rt, monkeypatch, n):
    """The fp8 engine's EdgeResidual blocks.1.1/.2 on e4m3 (er8_fused.hip: conv_exp 3x3 in tap groups of four
    and conv_pwl on v_mfma_scale_f32_16x16x128_f8f6f4, per-channel-scaled e4m3 weights, the halo and the
    128-channel map as e4m3) and blocks.2.1/.2 (er8w_fused.hip: 56 -> 224 -> 56, conv_exp in K steps of two taps x
    64 channels with its e4m3 weights streamed through an LDS ring, the 224-channel map in registers) against the
    bf16 er_fused / er2_fused (M2S_F8_ER=0) and the fp32 oracle.  Two more e4m3
    roundings per block, so the bars are cosines: the blocks' own outputs >= 0.995 and every later probed tap
    >= 0.99 against the bf16 blocks, pooled features per frame >= 0.995 against the oracle (SURVEY.md §8(c):
    0.99 end to end).  300 frames = 4800 tiles: the persistent loop's halo double buffer over many tiles."""
    st = synth.synth_acoustic_state(8)
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=46)[0]).to(DEV)
    monkeypatch.setenv("M2S_F8_ER", "1")
    e8 = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    monkeypatch.setenv("M2S_F8_ER", "0")
    eb = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    # after 1.1, 1.2 (er8_fused), 2.1, 2.2 (er8w_fused), 4.5, 5.9
    for i, bar in ((4, 0.995), (5, 0.995), (7, 0.99), (8, 0.99), (18, 0.99), (28, 0.99)):
        a, b = e8.probe(fr, i).cpu().numpy(), eb.probe(fr, i).cpu().numpy()
        assert np.isfinite(a).all()
        c = _cos(a.ravel(), b.ravel())
        print(f"tap {i}: cos(e4m3 er, bf16 er) {c:.6f}")
        assert c >= bar, (i, c)
    if n == 5:
        sd = {k: torch.from_numpy(v) for k, v in st.items()}
        ref = effnet.effnet_gap(sd, fr.cpu()).numpy()
        f = e8.effnet(fr).cpu().numpy()
        cmin = min(_cos(f[i], ref[i]) for i in range(n))
        print(f"features vs oracle: min per-frame cos {cmin:.6f}")
        assert cmin >= 0.995


def test_fp8_er8_e4m3_handoff_is_exact(rt, monkeypatch):
    """blocks.1.0 (ers2_fused) and blocks.1.1 (er8_fused) store their outputs' e4m3 bytes for the next er8 block
    (y8 -> x8), which then DMAs them instead of converting its bf16 input in the kernel (M2S_ER8_X8=0): the
    same bytes (e4m3 of the stored bf16 values, NaN kept), so the two paths agree bit for bit."""
    st = synth.synth_acoustic_state(8)
    fr = torch.from_numpy(synth.synth_frames(1, 37, seed=47)[0]).to(DEV)
    monkeypatch.setenv("M2S_ER8_X8", "1")
    ex = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    monkeypatch.setenv("M2S_ER8_X8", "0")
    ec = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    for i in (4, 5, 8):
        assert torch.equal(ex.probe(fr, i), ec.probe(fr, i)), i
    assert torch.equal(ex.effnet(fr), ec.effnet(fr))


def test_fp8_se_y8_e4m3_handoff_is_exact(rt, monkeypatch):
    """The SE GEMMs of the fp8 engine (se_ws / gemm128 KIND_F8_SE) store the next IR block's e4m3 expand operand
    (y8) as the e4m3 bytes of the bf16 values they store, so the next block reads the same bytes as when
    launch_rows_e4m3 converts its bf16 input (M2S_SE_Y8=0): the two paths agree bit for bit (one rounding chain)."""
    st = synth.synth_acoustic_state(8)
    fr = torch.from_numpy(synth.synth_frames(1, 37, seed=48)[0]).to(DEV)
    monkeypatch.setenv("M2S_SE_Y8", "1")
    ey = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    monkeypatch.setenv("M2S_SE_Y8", "0")
    ec = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    for i in (10, 12, 14, 18, 20, 28):
        assert torch.equal(ey.probe(fr, i), ec.probe(fr, i)), i
    assert torch.equal(ey.effnet(fr), ec.effnet(fr))


@pytest.mark.parametrize("n", [5, 300])
def test_fp8_e4m3_stride2_block(rt, monkeypatch, n):
    """The stride-2 IR blocks on e4m3 in the fp8 engine: blocks.5.0 (16x16 -> 8x8) on ir_pwdw_s2 mode 3 (the expand
    on the e4m3 block input written by blocks.4.5's SE GEMM, the f16 depthwise, e4m3 output) and the e4m3 SE-gated
    conv_pwl (se_ws f8); blocks.3.0 (32x32 -> 16x16) on ir_s2band mode 2 (bf16 expand, e4m3 depthwise output) and
    the e4m3 SE GEMM (gemm128), against the bf16 blocks (M2S_F8_S2=0) and the fp32 oracle.  The launch log shows
    which kernels ran.  Bars as for the stride-1 e4m3 expand: taps >= 0.995 against the bf16 blocks, pooled
    features per frame >= 0.995 against the oracle (0.99 end to end)."""
    from m2s import _native
    st = synth.synth_acoustic_state(8)
    fr = torch.from_numpy(synth.synth_frames(1, n, seed=49)[0]).to(DEV)
    monkeypatch.setenv("M2S_F8_S2", "1")
    e8 = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    monkeypatch.setenv("M2S_F8_S2", "0")
    eb = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    names = {}
    for key, eng in (("f8", e8), ("bf16", eb)):
        _native.prof_enable(True)
        eng.probe(fr, 19)
        torch.cuda.synchronize()
        names[key] = {r["name"] for r in _native.prof_launches()}
        _native.prof_enable(False)
    assert "ir_pwdw_s2_kernel<3>" in names["f8"] and "ir_pwdw_s2_kernel<0>" not in names["f8"], names["f8"]
    assert "ir_s2band_kernel<2, 2>" in names["f8"] and "ir_s2band_kernel<2, 0>" not in names["f8"], names["f8"]
    assert "ir_pwdw_s2_kernel<0>" in names["bf16"] and "ir_s2band_kernel<2, 0>" in names["bf16"], names["bf16"]
    # after blocks.3.0, 3.1 (its e4m3 input now from 3.0's SE GEMM), 5.0, 5.1, 5.9
    for i in (9, 10, 19, 20, 28):
        a, b = e8.probe(fr, i).cpu().numpy(), eb.probe(fr, i).cpu().numpy()
        assert np.isfinite(a).all()
        c = _cos(a.ravel(), b.ravel())
        print(f"tap {i}: cos(e4m3 blocks.5.0, bf16 blocks.5.0) {c:.6f}")
        assert c >= 0.995, (i, c)
    if n == 5:
        sd = {k: torch.from_numpy(v) for k, v in st.items()}
        ref = effnet.effnet_gap(sd, fr.cpu()).numpy()
        f = e8.effnet(fr).cpu().numpy()
        cmin = min(_cos(f[i], ref[i]) for i in range(n))
        print(f"features vs oracle: min per-frame cos {cmin:.6f}")
        assert cmin >= 0.995


@pytest.mark.parametrize("frames", [37, 300])
@pytest.mark.parametrize("var,C,kern", [("M2S_F8_MRF64", 64, "gemm128_kernel<1, 4, 1, 4, 3>"),
                                        ("M2S_F8_MRF32", 32, "gemm128_kernel<1, 4, 1, 2, 3>")])
def test_fp8_mrf_narrow_e4m3(rt, monkeypatch, frames, var, C, kern):
    """The C = 64 (M2S_F8_MRF64=1) and C = 32 (M2S_F8_MRF32=1) MRF stages on e4m3 in the fp8 vocoder (conv1d_f8 with
    128 / C taps per 128-byte K step, a tap count not a multiple ending on zero taps) against the fused bf16
    ResBlock1 (switch off, the default: faster at configs[4]) and the fp32 oracle: wav cosine >= 0.999 between the two engines and >= 0.99
     against the oracle, the launch log showing which kernel ran.  Ragged: 3 clips, stage lengths
    not multiples of any tile."""
    from m2s import _native
    sd = synth.synth_generator_state(5, HIFIGAN_H)
    mel = synth.synth_mel_log(3, 64, frames, seed=12)
    monkeypatch.setenv(var, "1")
    v8 = rt.VocoderEngine(sd, HIFIGAN_H, dtype="fp8", device=DEV)
    monkeypatch.setenv(var, "0")
    vb = rt.VocoderEngine(sd, HIFIGAN_H, dtype="fp8", device=DEV)
    x = torch.from_numpy(mel).to(DEV)
    out, names = {}, {}
    for key, v in (("f8", v8), ("bf16", vb)):
        _native.prof_enable(True)
        out[key] = v.forward(x).cpu().numpy().reshape(3, -1)
        torch.cuda.synchronize()
        names[key] = {r["name"] for r in _native.prof_launches()}
        _native.prof_enable(False)
    fused = f"rb1_fused_kernel<{C},"
    assert kern in names["f8"] and not any(fused in n for n in names["f8"]), names["f8"]
    assert any(fused in n for n in names["bf16"]) and kern not in names["bf16"], names["bf16"]
    ref = hifigan.generator({k: torch.from_numpy(v) for k, v in sd.items()}, HIFIGAN_H, torch.from_numpy(mel)).numpy()
    for b in range(3):
        c2, cr = _cos(out["f8"][b], out["bf16"][b]), _cos(out["f8"][b], ref[b])
        print(f"clip {b}: wav cos(e4m3 C={C}, bf16 C={C}) {c2:.6f}, vs oracle {cr:.6f}")
        assert np.isfinite(out["f8"][b]).all()
        assert c2 >= 0.999 and cr >= COS_MIN, (b, c2, cr)
