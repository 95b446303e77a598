"""Host logic of the stand-alone command lines (m2s/drivers.py): input conforming, batch planning,
per-job failure handling, the wav writers and the plug-in / generator loaders.  No GPU: the device
call is a stand-in function on CPU tensors (run_batches' contract), never a model."""
import json
import wave

import numpy as np
import pytest
import torch

from m2s import drivers


def _job(tmp_path, name, arr):
    p = tmp_path / f"{name}.npy"
    np.save(p, arr)
    return drivers.Job(p, name)


def test_read_mel_conform_rules(tmp_path):
    """mel_to_audio_synthesis.py:62-87: first row of a batch, truncate / zero-pad bins."""
    a = np.arange(2 * 70 * 5, dtype=np.float32).reshape(2, 70, 5)
    j = drivers.read_mel(_job(tmp_path, "batch", a), 64)
    assert j.ok and j.array.shape == (64, 5) and np.array_equal(j.array, a[0, :64])
    assert any("first sample" in n for n in j.notes) and any("truncated" in n for n in j.notes)
    b = np.ones((60, 3), np.float32)
    j = drivers.read_mel(_job(tmp_path, "short", b), 64)
    assert j.array.shape == (64, 3) and not j.array[60:].any() and j.array[:60].all()
    j = drivers.read_mel(_job(tmp_path, "bad", np.zeros((2, 3, 4, 5), np.float32)), 64)
    assert not j.ok and "dimensions" in j.error


def test_read_mel_strict_for_inference_e2e(tmp_path):
    """inference_e2e.py passes the array as is: a (1, n_mels, T) array is fine, other shapes fail."""
    assert drivers.read_mel(_job(tmp_path, "one", np.zeros((1, 64, 7), np.float32)), 64, conform=False).ok
    assert not drivers.read_mel(_job(tmp_path, "two", np.zeros((2, 64, 7), np.float32)), 64, conform=False).ok
    assert not drivers.read_mel(_job(tmp_path, "bins", np.zeros((80, 7), np.float32)), 64, conform=False).ok
    (tmp_path / "notnpy.npy").write_text("garbage")
    assert not drivers.read_mel(drivers.Job(tmp_path / "notnpy.npy", "x"), 64).ok


def test_plan_batches_groups_equal_shapes_in_order():
    jobs = [drivers.Job(None, f"j{i}", array=np.zeros(s, np.float32)) for i, s in
            enumerate([(64, 5), (64, 7), (64, 5), (64, 5), (64, 7)])]
    jobs.append(drivers.Job(None, "failed", error="x"))
    plan = drivers.plan_batches(jobs, max_batch=2)
    assert [[j.stem for j in b] for b in plan] == [["j0", "j2"], ["j3"], ["j1", "j4"]]
    with pytest.raises(ValueError):
        drivers.plan_batches(jobs, 0)


def test_run_batches_one_call_per_batch_and_failures_stay_per_batch():
    calls = []

    def fn(x):
        calls.append(tuple(x.shape))
        if x.shape[-1] == 7:
            raise RuntimeError("boom")
        return x.sum(dim=1)

    jobs = [drivers.Job(None, f"j{i}", array=np.full((4, t), i, np.float32)) for i, t in enumerate([5, 7, 5])]
    drivers.run_batches(drivers.plan_batches(jobs), fn, torch.device("cpu"))
    assert calls == [(2, 4, 5), (1, 4, 7)]
    assert np.allclose(jobs[0].result, 0) and np.allclose(jobs[2].result, 8)
    assert jobs[1].result is None and "boom" in jobs[1].error


def test_pcm_writers(tmp_path):
    audio = np.array([0.0, 0.5, -1.0, 1.0, 1.5, -0.99999], np.float32)
    drivers.write_wav_pcm16(tmp_path / "a.wav", audio, 11413)
    with wave.open(str(tmp_path / "a.wav")) as w:
        assert (w.getframerate(), w.getsampwidth(), w.getnchannels()) == (11413, 2, 1)
        pcm = np.frombuffer(w.readframes(6), dtype="<i2")
    assert pcm.tolist() == [0, 16384, -32767, 32767, 32767, -32767]
    # inference_e2e.py:51-53: scale by 32768 and truncate toward zero
    assert drivers.int16_truncated(np.array([0.5, -0.25, 0.99999], np.float32)).tolist() == [16384, -8192, 32767]


def test_build_generator_strips_weight_norm_best_effort(tmp_path):
    from env import AttrDict
    from m2s import synth
    from m2s.config import HIFIGAN_H
    torch.save({"generator": {k: torch.from_numpy(v) for k, v in synth.synth_generator_state(1).items()}},
               tmp_path / "g_00000001")
    gen, n = drivers.build_generator(AttrDict(HIFIGAN_H), tmp_path / "g_00000001", torch.device("cpu"), "fp32")
    assert n == 4 + 12 + 1 and not gen.training and gen.m2s_dtype == "fp32"
    assert "ups.0.weight" in gen.state_dict() and "conv_post.weight" in gen.state_dict()
    with pytest.raises(KeyError):
        torch.save({"g": {}}, tmp_path / "bad")
        drivers.build_generator(AttrDict(HIFIGAN_H), tmp_path / "bad", torch.device("cpu"))


def test_build_acoustic_plugin_surface(tmp_path):
    from m2s import synth
    import os
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in synth.synth_acoustic_state(2).items()}
    sd["extra_key"] = torch.zeros(1)
    torch.save({"epoch": 1, "model_state_dict": sd}, tmp_path / "best.pt")
    logs = []
    code = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mri-to-speech_amd", "mri2speech_code")
    m = drivers.build_acoustic(tmp_path / "best.pt", torch.device("cpu"), code_dir=code, dtype="bf16", log=logs.append)
    assert not m.training and m.m2s_dtype == "bf16"
    assert len(logs) == 1 and "unexpected" in logs[0] and "extra_key" in logs[0]
    assert torch.equal(m.head.weight, sd["head.weight"])


def test_write_json_roundtrip(tmp_path):
    drivers.write_json(tmp_path / "s.json", {"a": [1, 2], "b": 0.5})
    assert json.loads((tmp_path / "s.json").read_text()) == {"a": [1, 2], "b": 0.5}
