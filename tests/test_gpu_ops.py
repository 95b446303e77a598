"""torch.ops.m2s.* on the GPU: torch.library.opcheck (schema, fake kernels vs the HIP kernels,
AOT dispatch) for every op, and the drop-in plug-in forwards dispatching through them."""
import numpy as np
import pytest
import torch

from m2s import ops, runtime, synth
from m2s.config import HIFIGAN_H
from oracle import effnet

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def engines():
    ac = runtime.AcousticEngine(synth.synth_acoustic_state(2), dtype="bf16x3", device=DEV)
    voc = runtime.VocoderEngine(synth.synth_generator_state(2), HIFIGAN_H, dtype="bf16x3", device=DEV)
    return ac, voc


def _frames(b, t, hw=(96, 80)):
    return torch.from_numpy(synth.synth_frames(b, t, hw=hw, seed=b * 10 + t)).to(DEV)


def test_opcheck_every_op(engines):
    ac, voc = engines
    o = ops.load()
    from m2s.autograd import CamEngine
    cam = CamEngine({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synth_acoustic_state(2).items()}, DEV)
    g = torch.Generator().manual_seed(0)
    lw = [(torch.rand(*s, generator=g) * 0.1 - 0.05).to(DEV)
          for s in [(2560, 208), (2560, 640), (2560,), (2560,)] * 2]
    mean, std = (torch.from_numpy(a).to(DEV) for a in synth.synth_scaler())
    cases = {
        "acoustic_forward": (ac.handle, _frames(2, 3), 64),
        "effnet_forward": (ac.handle, _frames(1, 4)[0]),
        "effnet_features": (ac.handle, _frames(1, 2)[0], 18),
        "bilstm_summerge": (ac.handle, torch.randn(2, 5, 208, device=DEV), 640, 64),
        "mel_glue": (torch.randn(6, 64, device=DEV), mean, std),
        "hifigan_forward": (voc.handle, torch.from_numpy(synth.synth_mel_log(2, 64, 7)).to(DEV), 0, voc.hop),
        "pipeline_forward": (ac.handle, voc.handle, _frames(2, 4), mean, std, 64, voc.hop),
        "preprocess_frames": (torch.randint(0, 256, (3, 40, 36), dtype=torch.uint8, device=DEV),),
        "cam_backbone": (cam.handle, _frames(1, 3, hw=(64, 48))[0]),
        "bilstm_train_forward": (torch.randn(2, 3, 208, device=DEV), lw),
        "bilstm_train_backward": (torch.randn(2, 3, 640, device=DEV), torch.randn(2, 3, 208, device=DEV), lw,
                                  *o.bilstm_train_forward(torch.randn(2, 3, 208, device=DEV), lw)[1:]),
        "linear_forward": (torch.randn(2, 3, 640, device=DEV), torch.randn(64, 640, device=DEV),
                           torch.randn(64, device=DEV)),
        "linear_backward": (torch.randn(2, 3, 64, device=DEV), torch.randn(2, 3, 640, device=DEV),
                            torch.randn(64, 640, device=DEV)),
        "gap_forward": (torch.randn(2, 208, 8, 8, device=DEV),),
        "gap_backward": (torch.randn(2, 208, device=DEV), 8, 8),
    }
    assert set(cases) == set(ops.OPS)
    for name, args in cases.items():
        torch.library.opcheck(getattr(o, name).default, args,
                              test_utils=("test_schema", "test_faketensor", "test_aot_dispatch_dynamic"))


def _dispatched(fn):
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        fn()
    return {e.name for e in prof.events()}


def test_plugin_forwards_dispatch_through_torch_ops():
    from env import AttrDict
    from models import Generator
    from mri_acoustic_model import build_acoustic_model
    m = build_acoustic_model().to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synth.synth_acoustic_state(3).items()},
                      strict=False)
    m.eval()
    gen = Generator(AttrDict(HIFIGAN_H)).to(DEV)
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_generator_state(3).items()})
    gen.eval()
    x = _frames(1, 3)
    with torch.no_grad():
        assert "m2s::acoustic_forward" in _dispatched(lambda: m(x))
        assert "m2s::effnet_forward" in _dispatched(lambda: m.cnn(x[0].unsqueeze(1)))
        assert "m2s::bilstm_summerge" in _dispatched(lambda: m.rnn(torch.randn(1, 3, 208, device=DEV)))
        mel = torch.from_numpy(synth.synth_mel_log(1, 64, 5)).to(DEV)
        assert "m2s::hifigan_forward" in _dispatched(lambda: gen(mel))


def test_backbone_feature_maps_for_gradcam():
    """mri_gradcam_formant.py:153-158: backbone(x.repeat(1, 3, 1, 1)) -> list, last map (N,208,H/32,W/32)."""
    from mri_acoustic_model import build_acoustic_model
    sd = synth.synth_acoustic_state(5)
    m = build_acoustic_model().to(DEV)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=False)
    m.eval()
    fr = torch.from_numpy(synth.synth_frames(1, 2, seed=9)[0])
    x = fr.unsqueeze(1).to(DEV).repeat(1, 3, 1, 1)
    with torch.no_grad():
        feats = m.cnn.backbone(x)
    assert isinstance(feats, list) and len(feats) == 5
    assert [tuple(f.shape) for f in feats] == [(2, c, 256 // s, 256 // s) for c, s in
                                                zip((16, 32, 56, 120, 208), (2, 4, 8, 16, 32))]
    taps = []
    effnet.effnet_features({k: torch.from_numpy(v) for k, v in sd.items()}, fr, taps=taps)
    for f, i in zip(feats, (2, 5, 8, 18, 28)):
        ref = taps[i].numpy()
        assert np.abs(f.cpu().numpy() - ref).max() <= 1e-4 * np.abs(ref).max(), i
