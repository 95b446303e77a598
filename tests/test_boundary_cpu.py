"""Drop-in boundary checks that need no GPU: the C ABI library, the plug-in module trees and
state-dict keys, loader semantics, the CLI surface, and the no-fallback rule."""
import os
import re

import numpy as np
import pytest
import torch

from m2s import _native as N
from m2s import synth
from m2s.config import HIFIGAN_H
from m2s.state_layout import acoustic_state_shapes, generator_state_shapes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(REPO, "include", "m2s.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(m2s_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    declared = _header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(N.exported_symbols()) == declared
    assert L.m2s_abi_version() == N.ABI_VERSION == 6


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device error path")
def test_no_device_fails_loudly():
    L = N.lib()
    assert L.m2s_device_check(0) == 4  # M2S_E_NODEV
    from m2s import runtime
    with pytest.raises(N.M2SError):
        runtime.AcousticEngine(synth.synth_acoustic_state(0), dtype="fp32")


def test_acoustic_plugin_tree_and_keys():
    from mri_acoustic_model import build_acoustic_model
    m = build_acoustic_model(n_mels=64, cnn_pretrained=False, rnn_hidden=640, dropout=0.5,
                             use_checkpoint=False, ckpt_segments=2, use_reentrant=False)
    sd = m.state_dict()
    want = acoustic_state_shapes()
    assert list(sd.keys()) == list(want.keys())
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(want[k]), k
    assert m.cnn.out_channels == 208
    assert isinstance(m.rnn.dropout, torch.nn.Dropout) and m.rnn.dropout.p == 0.5
    assert isinstance(m.head, torch.nn.Linear)


def test_acoustic_plugin_load_state_dict_strict_false():
    from mri_acoustic_model import build_acoustic_model
    m = build_acoustic_model()
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in synth.synth_acoustic_state(1).items()}
    sd["optimizer_junk"] = torch.zeros(1)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert missing == [] and unexpected == ["optimizer_junk"]
    assert torch.equal(m.head.weight, sd["head.weight"])


def test_acoustic_plugin_refuses_cpu_and_training():
    from mri_acoustic_model import build_acoustic_model
    m = build_acoustic_model().eval()
    with torch.no_grad(), pytest.raises(RuntimeError):
        m(torch.zeros(1, 2, 1, 64, 64))
    m.train()
    with pytest.raises(NotImplementedError):
        m(torch.zeros(1, 2, 1, 64, 64))


def test_generator_plugin_keys_and_loader():
    from env import AttrDict
    from models import Generator
    g = Generator(AttrDict(HIFIGAN_H))
    want = generator_state_shapes(HIFIGAN_H)
    sd = g.state_dict()
    assert sorted(sd.keys()) == sorted(want.keys())
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(want[k]), k
    g.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_generator_state(2).items()})  # strict
    # the reference loader's best-effort weight-norm removal (run_mri_video_inference.py:99-115)
    from torch.nn.utils import remove_weight_norm
    for m in list(g.ups) + [g.conv_post]:
        remove_weight_norm(m)
    for r in g.resblocks:
        r.remove_weight_norm()
    assert "ups.0.weight" in g.state_dict() and "ups.0.weight_g" not in g.state_dict()
    with pytest.raises(ValueError):  # second removal raises, like the reference
        g.resblocks[0].remove_weight_norm()


def test_generator_remove_weight_norm_mirrors_reference_failure():
    """models.py:133-140 removes ups/resblocks then fails on the never-normed conv_pre."""
    from env import AttrDict
    from models import Generator
    g = Generator(AttrDict(HIFIGAN_H))
    with pytest.raises(ValueError):
        g.remove_weight_norm()
    assert "ups.3.weight" in g.state_dict()


def test_resblock2_generator_keys():
    from env import AttrDict
    from models import Generator
    h = dict(HIFIGAN_H, resblock="2", resblock_dilation_sizes=[[1, 3], [1, 3], [1, 3]])
    g = Generator(AttrDict(h))
    assert sorted(g.state_dict().keys()) == sorted(generator_state_shapes(h).keys())


def test_cli_matches_reference_flags():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "m2s_cli", os.path.join(REPO, "mri-to-speech_amd", "scripts", "run_mri_video_inference.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    a = cli.parse_args(["--video", "v.mp4", "--mri-checkpoint", "c.pt", "--scaler-json", "s.json",
                        "--hifigan-config", "h.json", "--hifigan-checkpoint", "g", "--output-dir", "o",
                        "--mri-code-dir", "d", "--max-frames", "10", "--n-mels", "64", "--rnn-hidden", "640",
                        "--dropout", "0.5"])
    assert (a.video, a.max_frames, a.n_mels, a.rnn_hidden, a.dropout) == ("v.mp4", 10, 64, 640, 0.5)
    assert a.dtype is None and a.decode_chunk == 64  # additive flags
    g = np.load(os.path.join(REPO, "tests", "golden", "glue.npz"))
    pre = torch.from_numpy(g["preprocessed"])  # the device kernel's output is checked against it on the GPU
    assert tuple(cli.frames_to_tensor(pre).shape) == tuple(g["frames_tensor_shape"])


def test_cli_frame_stream_chunks_a_npy_stack(tmp_path):
    """Host half of the pipelined decode: a (T,H,W) uint8 .npy stack in chunks, --max-frames honoured."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "m2s_cli3", os.path.join(REPO, "mri-to-speech_amd", "scripts", "run_mri_video_inference.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    stack = np.random.default_rng(0).integers(0, 256, (11, 256, 256), dtype=np.uint8)
    np.save(tmp_path / "v.npy", stack)
    fs = cli.FrameStream(tmp_path / "v.npy", torch.device("cpu"), max_frames=10, chunk=4)
    chunks = list(fs._host_chunks())
    assert [len(c) for c in chunks] == [4, 4, 2]
    np.testing.assert_array_equal(np.concatenate([np.stack(c) for c in chunks]), stack[:10])


def test_cli_wav_writer_pcm16(tmp_path):
    import importlib.util
    import wave
    spec = importlib.util.spec_from_file_location(
        "m2s_cli2", os.path.join(REPO, "mri-to-speech_amd", "scripts", "run_mri_video_inference.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    audio = np.array([0.0, 0.5, -1.0, 1.0, 1.5], dtype=np.float32)
    p = tmp_path / "x.wav"
    cli.write_wav(p, audio, 11413)
    with wave.open(str(p)) as w:
        assert (w.getframerate(), w.getsampwidth(), w.getnchannels()) == (11413, 2, 1)
        pcm = np.frombuffer(w.readframes(5), dtype="<i2")
    assert pcm.tolist() == [0, 16384, -32767, 32767, 32767]


def test_plugin_ships_the_benched_cnn_chunk(monkeypatch):
    """The engine the plug-in builds (and so the CLI and export_predicted_mels.py) runs the CNN in the
    chunk bench.py times (the plug-in shipped 256-frame passes while bench.py timed 1920)."""
    import inspect

    import bench
    from m2s import runtime
    from m2s.config import CNN_CHUNK
    from mri_acoustic_model import build_acoustic_model
    monkeypatch.delenv("M2S_CHUNK", raising=False)
    assert build_acoustic_model().m2s_chunk == bench.parse([]).chunk == CNN_CHUNK
    assert inspect.signature(runtime.AcousticEngine).parameters["chunk"].default == CNN_CHUNK
