"""configs[4] at the shape bench.py times: 8 clips x 1000 frames per GPU, end to end, one pipeline call.

configs[4] (BASELINE.json): "fp8 MFMA CNN encoder + HiFi-GAN MRF dilated-conv path, >=1000-frame clips".
bench.py's ``configs4`` lines time 8 x 1000 frames (8 000 CNN frames over several CNN chunks, the
8-sequence split ``lstm_x3`` BiLSTM, the batched e4m3 MRF stages); these tests hold that exact batch to the
fp32 oracle (oracle/pipeline.py e2e, the no_grad section of scripts/run_mri_video_inference.py:218-242)
on clips 0 and 7 (the first and last rows of every batched launch):

* fp8     cosine >= 0.99 (SURVEY.md §8(c)'s fp8 tolerance) for mel_norm and wav, every clip finite;
* bf16x3  the fp32 tolerances of test_config4_1x1000_end_to_end (1000 recurrent steps);
* bf16    cosine >= 0.999 for mel_norm, wav SNR >= 20 dB (the bf16 bars of test_gpu_configs.py).

The 2-clip oracle run takes ~30-60 s of host CPU, so the tests carry their own timeout.
"""
import numpy as np
import pytest
import torch

from m2s import synth
from m2s.config import HIFIGAN_H
from oracle import pipeline

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]
DEV = torch.device("cuda", 0)
B, T = 8, 1000
CLIPS = (0, 7)
TOL_X3 = {"mel_norm": 2e-4, "mel_db": 4e-3, "mel_log": 1e-3, "wav": 1e-4}


def _t(sd):
    return {k: torch.from_numpy(v) for k, v in sd.items()}


def _cos(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))


def _snr_db(ref, x):
    ref, x = np.asarray(ref, np.float64), np.asarray(x, np.float64)
    return 10 * np.log10(np.sum(ref ** 2) / max(np.sum((ref - x) ** 2), 1e-30))


@pytest.fixture(scope="module")
def c4():
    ac, gen = synth.synth_acoustic_state(11), synth.synth_generator_state(12)
    mean, std = synth.synth_scaler()
    fr = synth.synth_frames(B, T, seed=304)
    torch.set_num_threads(16)
    ref = pipeline.e2e(_t(ac), _t(gen), HIFIGAN_H, fr[list(CLIPS)], mean, std, cnn_chunk=100)
    return ac, gen, mean, std, fr, ref


def _run(c4, dtype):
    from m2s import runtime as rt
    ac, gen, mean, std, fr, _ = c4
    pipe = rt.Pipeline(rt.AcousticEngine(ac, dtype=dtype, device=DEV),
                       rt.VocoderEngine(gen, HIFIGAN_H, dtype=dtype, device=DEV), mean, std)
    out = pipe.forward(torch.from_numpy(fr).to(DEV))
    pipe.ac.check()
    out = {k: v.cpu().numpy() for k, v in out.items()}
    assert out["wav"].shape == (B, T * 420) and out["mel_norm"].shape == (B, T, 64)
    for k, v in out.items():
        assert np.isfinite(v).all(), (dtype, k)
    return out


def test_config4_8x1000_fp8(c4):
    out, ref = _run(c4, "fp8"), c4[5]
    for j, c in enumerate(CLIPS):
        cm, cw = _cos(out["mel_norm"][c], ref["mel_norm"][j]), _cos(out["wav"][c], ref["wav"][j])
        print(f"\nfp8 8x1000 clip {c}: mel_norm cos {cm:.5f}, wav cos {cw:.5f}")
        assert cm >= 0.99 and cw >= 0.99, (c, cm, cw)


def test_config4_8x1000_bf16x3(c4):
    out, ref = _run(c4, "bf16x3"), c4[5]
    for j, c in enumerate(CLIPS):
        for k, t in TOL_X3.items():
            np.testing.assert_allclose(out[k][c], ref[k][j], atol=t, rtol=0, err_msg=f"clip {c} {k}")


def test_config4_8x1000_bf16(c4):
    out, ref = _run(c4, "bf16"), c4[5]
    for j, c in enumerate(CLIPS):
        cm, snr = _cos(out["mel_norm"][c], ref["mel_norm"][j]), _snr_db(ref["wav"][j], out["wav"][c])
        print(f"\nbf16 8x1000 clip {c}: mel_norm cos {cm:.6f}, wav SNR {snr:.1f} dB")
        assert cm >= 0.999 and snr >= 20.0, (c, cm, snr)
