"""Pin the CPU oracle against golden vectors produced by the reference's own code
(tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from m2s import synth
from oracle import acoustic, effnet, hifigan

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="module")
def gen_gold():
    return _load("generator.npz")


@pytest.mark.parametrize("case", ["r1", "r2"])
def test_generator_matches_reference(gen_gold, case):
    h = json.loads(bytes(gen_gold[f"{case}_h"]).decode())
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_generator_state(int(gen_gold["seed"]), h).items()}
    wav = hifigan.generator(sd, h, torch.from_numpy(gen_gold[f"{case}_mel"]))
    ref = gen_gold[f"{case}_wav"]
    assert wav.shape == ref.shape == (2, 1, 6 * 420)
    np.testing.assert_allclose(wav.numpy(), ref, atol=2e-6, rtol=0)


def test_generator_folded_weightnorm(gen_gold):
    h = json.loads(bytes(gen_gold["r1_h"]).decode())
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_generator_state(int(gen_gold["seed"]), h).items()}
    np.testing.assert_allclose(hifigan.generator(sd, h, torch.from_numpy(gen_gold["r1_mel"])).numpy(),
                               gen_gold["r1_wav_folded"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(hifigan.generator(sd, h, torch.from_numpy(gen_gold["r1_mel30"])).numpy(),
                               gen_gold["r1_wav30"], atol=2e-6, rtol=0)


def test_generator_is_causal_with_lookahead():
    """Receptive field: conv_pre/conv_post look 6 frames/samples ahead; MRF is causal (utils.py:33-34)."""
    from m2s.config import HIFIGAN_H as h
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_generator_state(0, h).items()}
    mel = torch.from_numpy(synth.synth_mel_log(1, 64, 40))
    a = hifigan.generator(sd, h, mel)
    mel2 = mel.clone()
    mel2[:, :, 30] += 1.0
    b = hifigan.generator(sd, h, mel2)
    changed = torch.nonzero((a - b).abs()[0, 0] > 0).flatten()
    assert changed.min().item() >= (30 - 7) * 420 and changed.min().item() < 30 * 420


@pytest.fixture(scope="module")
def ac_gold():
    g = _load("acoustic.npz")
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_acoustic_state(int(g["seed"])).items()}
    return g, sd


@pytest.mark.parametrize("bt", ["2x7", "1x1", "8x4", "1x30"])
def test_bilstm_head_matches_reference(ac_gold, bt):
    g, sd = ac_gold
    x = torch.from_numpy(g[f"lstm_{bt}_in"])
    for fn in (acoustic.bilstm_summerge, acoustic.bilstm_summerge_loop):
        y = fn(sd, x)
        np.testing.assert_allclose(y.numpy(), g[f"lstm_{bt}_y"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(acoustic.head(sd, torch.from_numpy(g[f"lstm_{bt}_y"])).numpy(),
                               g[f"lstm_{bt}_head"], atol=1e-5, rtol=0)


def test_acoustic_wiring_matches_reference(ac_gold):
    """Reference OTNLikeCNNBiLSTM.forward with the oracle backbone == oracle composition."""
    g, sd = ac_gold
    fr = torch.from_numpy(synth.synth_frames(2, 3, seed=int(g["model_frames_seed"])))
    for frames, key in ((fr[:1], "model_out"), (fr[:, :2], "model_out4d")):
        B, T = frames.shape[:2]
        f = effnet.effnet_gap(sd, frames.reshape(B * T, 1, 256, 256)).view(B, T, -1)
        out = acoustic.head(sd, acoustic.bilstm_summerge(sd, f))
        np.testing.assert_allclose(out.numpy(), g[key], atol=2e-5, rtol=0)


def test_glue_matches_reference():
    g = _load("glue.npz")
    pre = np.stack([acoustic.preprocess_frame(f) for f in g["frames_u8"]])
    np.testing.assert_allclose(pre, g["preprocessed"], atol=1e-6, rtol=0)
    assert not pre[2].any()
    assert tuple(g["frames_tensor_shape"]) == (1, 3, 1, 256, 256)
    db = acoustic.denormalize_mel(torch.from_numpy(g["pred_norm"]), g["scaler_mean"], g["scaler_std"])
    np.testing.assert_array_equal(db.numpy(), g["mel_db"])
    np.testing.assert_array_equal(acoustic.mel_db_to_log(db).numpy(), g["mel_log"])
    assert g["mel_log"].min() >= np.log(np.float32(1e-5)) - 1e-6


def test_effnet_structure():
    """timm absent: parity unpinned, structure pinned (keys, shapes, channel widths, output size)."""
    from m2s.state_layout import effnet_state_shapes
    assert dict(effnet.effnet_state_shapes()) == dict(effnet_state_shapes())
    blocks = effnet.block_table()
    assert [sum(1 for b in blocks if b["stage"] == s) for s in range(6)] == [2, 3, 3, 4, 6, 10]
    assert [b["mid"] for b in blocks if b["type"] == "ir" and b["idx"] == 1] == [416, 720, 1248]
    assert [b["rd"] for b in blocks if b["type"] == "ir" and b["idx"] <= 1] == [14, 26, 26, 30, 30, 52]
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_acoustic_state(0).items()}
    x = torch.from_numpy(synth.synth_frames(1, 1))[0]
    f = effnet.effnet_features(sd, x)
    assert f.shape == (1, 208, 8, 8)
    fl = effnet.effnet_flops_per_frame()
    assert abs(fl["total"] / 1e9 - 3.011) < 0.01


def test_effnet_same_padding_is_asymmetric():
    """TF SAME on a stride-2 3x3 conv of an even input pads (0,1,0,1), unlike PyTorch's symmetric pad."""
    x = torch.randn(1, 1, 8, 8)
    w = torch.randn(1, 1, 3, 3)
    y = effnet._conv(x, w, 3, 2)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(x, [0, 1, 0, 1]), w, stride=2)
    assert torch.equal(y, ref)
