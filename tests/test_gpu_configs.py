"""Every BASELINE.json config at its real size through the HIP path, against the CPU oracle.

  configs[0]  1 clip x 30 frames -> 64-bin mel (CNN-BiLSTM), fp32 and bf16x3
  configs[1]  8 clips x 4 frames (ref_frames = 4) CNN-BiLSTM, bf16
  configs[2]  1 clip x 30 frames end to end to the 11 413 Hz wav, fp32 and bf16x3
  configs[3]  the per-GPU share of 512 clips over 8 GPUs: 64 clips x 30 frames end to end in the
              bench dtype (bf16x3); 17 clips (every 4th and the last) against the fp32 oracle in one
              batched oracle run (all 64 passed once: profiles/r03_cfg3_all64_oracle.txt), every clip against the bf16 path
  configs[4]  a 1000-frame clip end to end (bf16x3), the clip length of the fp8 config
Tolerances (fp32 = the reference's precision): mel_norm <= 1e-4, mel_log <= 5e-4, wav <= 1e-4
(1000 frames: mel_norm <= 2e-4 — fp32 summation order over 1000 recurrent steps); bf16:
mel_norm <= 5e-2 and cosine >= 0.999, wav SNR >= 20 dB.  (scripts/run_mri_video_inference.py:218-242)
"""
import numpy as np
import pytest
import torch

from m2s import synth
from m2s.config import HIFIGAN_H
from oracle import pipeline

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
FP32_TOL = {"mel_norm": 1e-4, "mel_db": 2e-3, "mel_log": 5e-4, "wav": 1e-4}


@pytest.fixture(scope="module")
def rt():
    from m2s import runtime
    return runtime


@pytest.fixture(scope="module")
def weights():
    ac, gen = synth.synth_acoustic_state(11), synth.synth_generator_state(12)
    mean, std = synth.synth_scaler()
    return ac, gen, mean, std


def _t(sd):
    return {k: torch.from_numpy(v) for k, v in sd.items()}


def _snr_db(ref, x):
    ref, x = np.asarray(ref, np.float64), np.asarray(x, np.float64)
    return 10 * np.log10(np.sum(ref ** 2) / max(np.sum((ref - x) ** 2), 1e-30))


def _cos(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(a @ b / np.sqrt((a @ a) * (b @ b)))


def _pipe(rt, weights, dtype):
    ac, gen, mean, std = weights
    return rt.Pipeline(rt.AcousticEngine(ac, dtype=dtype, device=DEV), rt.VocoderEngine(gen, HIFIGAN_H, dtype=dtype, device=DEV),
                       mean, std)


@pytest.fixture(scope="module")
def clip30(weights):
    ac, gen, mean, std = weights
    fr = synth.synth_frames(1, 30, seed=300)
    return fr, pipeline.e2e(_t(ac), _t(gen), HIFIGAN_H, fr, mean, std)


@pytest.mark.parametrize("dtype", ["fp32", "bf16x3"])
def test_config0_1x30_mel(rt, weights, clip30, dtype):
    fr, ref = clip30
    eng = rt.AcousticEngine(weights[0], dtype=dtype, device=DEV)
    mn = eng.forward(torch.from_numpy(fr).unsqueeze(2).to(DEV)).cpu().numpy()  # (1,T,1,H,W) as the script feeds it
    assert mn.shape == (1, 30, 64)
    np.testing.assert_allclose(mn, ref["mel_norm"], atol=FP32_TOL["mel_norm"], rtol=0)


def test_config1_8x4_bf16(rt, weights):
    ac = weights[0]
    fr = synth.synth_frames(8, 4, seed=301)
    ref = pipeline.acoustic_forward(_t(ac), fr).numpy()
    mn = rt.AcousticEngine(ac, dtype="bf16", device=DEV).forward(torch.from_numpy(fr).to(DEV)).cpu().numpy()
    assert mn.shape == (8, 4, 64) and np.isfinite(mn).all()
    assert np.abs(mn - ref).max() <= 5e-2
    assert _cos(mn, ref) >= 0.999
    x3 = rt.AcousticEngine(ac, dtype="bf16x3", device=DEV).forward(torch.from_numpy(fr).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(x3, ref, atol=FP32_TOL["mel_norm"], rtol=0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16x3"])
def test_config2_1x30_end_to_end(rt, weights, clip30, dtype):
    fr, ref = clip30
    out = {k: v.cpu().numpy() for k, v in _pipe(rt, weights, dtype).forward(torch.from_numpy(fr).to(DEV)).items()}
    assert out["wav"].shape == (1, 30 * 420)
    for k, tol in FP32_TOL.items():
        np.testing.assert_allclose(out[k], ref[k], atol=tol, rtol=0, err_msg=k)


@pytest.mark.timeout(600)
def test_config3_64x30_per_gpu_share(rt, weights):
    ac, gen, mean, std = weights
    fr = synth.synth_frames(64, 30, seed=302)
    x = torch.from_numpy(fr).to(DEV)
    out = {k: v.cpu().numpy() for k, v in _pipe(rt, weights, "bf16x3").forward(x).items()}
    bf = {k: v.cpu().numpy() for k, v in _pipe(rt, weights, "bf16").forward(x).items()}
    assert out["wav"].shape == (64, 30 * 420)
    for k in out:
        assert np.isfinite(out[k]).all() and np.isfinite(bf[k]).all(), k
    for c in range(64):
        assert _snr_db(out["wav"][c], bf["wav"][c]) >= 20.0, c
    for c0 in range(0, 64, 16):  # every clip through the fp32 oracle, 16 at a time (~1 min of CPU in all)
        ref = pipeline.e2e(_t(ac), _t(gen), HIFIGAN_H, fr[c0:c0 + 16], mean, std)
        for k, tol in FP32_TOL.items():
            for j in range(16):
                np.testing.assert_allclose(out[k][c0 + j], ref[k][j], atol=tol, rtol=0, err_msg=f"clip {c0 + j} {k}")


def test_config4_1x1000_end_to_end(rt, weights):
    ac, gen, mean, std = weights
    fr = synth.synth_frames(1, 1000, seed=303)
    out = {k: v.cpu().numpy() for k, v in _pipe(rt, weights, "bf16x3").forward(torch.from_numpy(fr).to(DEV)).items()}
    ref = pipeline.e2e(_t(ac), _t(gen), HIFIGAN_H, fr, mean, std, cnn_chunk=100)
    assert out["wav"].shape == (1, 1000 * 420)
    tol = dict(FP32_TOL, mel_norm=2e-4, mel_log=1e-3, mel_db=4e-3)
    for k, t in tol.items():
        np.testing.assert_allclose(out[k], ref[k], atol=t, rtol=0, err_msg=k)


def _launches(fn):
    from m2s import _native
    _native.prof_enable(True)
    out = fn()
    torch.cuda.synchronize()
    names = [r["name"] for r in _native.prof_launches()]
    _native.prof_enable(False)
    return out, names


def test_config2_small_pass_plan(rt, weights, clip30, monkeypatch):
    """The one-clip shape of the reference CLI (run_mri_video_inference.py:215-242) runs the small-pass plan: the grid
    IR front halves (ir_pwdw / ir_pwdw_s2) instead of the one-workgroup-per-image ir_ws, the split-K conv_gemm SE
    GEMM instead of se_ws, and split-K vocoder convs (conv_gemm_ksum_kernel).  Same split fp32 arithmetic up to
    summation order: within 1e-4 of the persistent plan (M2S_IRWS_MIN=0, M2S_SEWS_MIN=0, M2S_KSPLIT=1) and of the
    fp32 oracle at the configs[2] bar."""
    fr, ref = clip30
    x = torch.from_numpy(fr).to(DEV)
    small, names = _launches(lambda: {k: v.cpu().numpy() for k, v in _pipe(rt, weights, "bf16x3").forward(x).items()})
    assert not any(n.startswith(("ir_ws_kernel", "se_ws_kernel")) for n in names), sorted(set(names))
    assert any(n.startswith("ir_pwdw_kernel") for n in names) and any(n.startswith("conv_gemm_ksum_kernel") for n in names)
    monkeypatch.setenv("M2S_IRWS_MIN", "0")
    monkeypatch.setenv("M2S_SEWS_MIN", "0")
    monkeypatch.setenv("M2S_KSPLIT", "1")
    big, names = _launches(lambda: {k: v.cpu().numpy() for k, v in _pipe(rt, weights, "bf16x3").forward(x).items()})
    assert any(n.startswith("ir_ws_kernel") for n in names) and any(n.startswith("se_ws_kernel") for n in names)
    assert not any(n.startswith("conv_gemm_ksum_kernel") for n in names)
    for k, tol in FP32_TOL.items():
        np.testing.assert_allclose(small[k], ref[k], atol=tol, rtol=0, err_msg=k)
        np.testing.assert_allclose(small[k], big[k], atol=tol, rtol=0, err_msg=k)


@pytest.mark.parametrize("dtype,nc,nf,parts", [("bf16", 8, 4, None), ("bf16x3", 1, 30, None), ("bf16x3", 2, 30, "3"),
                                               ("bf16", 1, 30, "8")])
def test_stem_strip_parts_bitwise(rt, weights, monkeypatch, dtype, nc, nf, parts):
    """Small batches cut the fused stem's strips (image, 16-column tile column) into tile-row ranges so the units
    fill the workgroup slots (stem_b0.hip): a range's first tile recomputes the S / A rows a whole strip carries
    over from the tile above, with the same arithmetic, so the mel is bit-identical to whole strips
    (M2S_STEM_PARTS=1).  parts None = the automatic cut (3 at 8 x 4 bf16, 2 at one bf16x3 clip); "3" = uneven
    ranges (3 + 3 + 2 tile rows); "8" = one tile row a unit."""
    ac = weights[0]
    x = torch.from_numpy(synth.synth_frames(nc, nf, seed=311)).to(DEV)
    if parts is not None:
        monkeypatch.setenv("M2S_STEM_PARTS", parts)
    a = rt.AcousticEngine(ac, dtype=dtype, device=DEV).forward(x).cpu().numpy()
    monkeypatch.setenv("M2S_STEM_PARTS", "1")
    b = rt.AcousticEngine(ac, dtype=dtype, device=DEV).forward(x).cpu().numpy()
    assert np.isfinite(a).all() and np.array_equal(a, b)


def test_config1_split_k_matches_unsplit(rt, weights, monkeypatch):
    """configs[1] (8 x 4, bf16): the SE GEMMs of the small pass run split K (fp32 partial sums added in split order by
    conv_gemm_ksum_kernel); against the unsplit launches (M2S_KSPLIT=1) the mel differs only by fp32 summation
    order before the bf16 rounding of each layer's output."""
    ac = weights[0]
    x = torch.from_numpy(synth.synth_frames(8, 4, seed=301)).to(DEV)
    a, names = _launches(lambda: rt.AcousticEngine(ac, dtype="bf16", device=DEV).forward(x).cpu().numpy())
    assert any(n.startswith("conv_gemm_ksum_kernel") for n in names)
    monkeypatch.setenv("M2S_KSPLIT", "1")
    b = rt.AcousticEngine(ac, dtype="bf16", device=DEV).forward(x).cpu().numpy()
    assert np.isfinite(a).all() and _cos(a, b) >= 0.9999 and np.abs(a - b).max() <= 2e-2
