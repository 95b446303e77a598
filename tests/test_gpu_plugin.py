"""The drop-in surface on the GPU: plug-in acoustic model, models.Generator and the CLI script,
driven exactly as the reference drives them, checked against the oracle / reference goldens."""
import importlib.util
import json
import os

import numpy as np
import pytest
import torch

from m2s import synth
from m2s.config import HIFIGAN_H
from oracle import acoustic, effnet, hifigan

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")


def _t(sd):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}


def test_plugin_forward_matches_reference_wiring():
    from mri_acoustic_model import build_acoustic_model
    g = np.load(os.path.join(GOLD, "acoustic.npz"))
    m = build_acoustic_model(n_mels=64, cnn_pretrained=False, rnn_hidden=640, dropout=0.5).to("cuda")
    missing, unexpected = m.load_state_dict(_t(synth.synth_acoustic_state(int(g["seed"]))), strict=False)
    assert not missing and not unexpected
    m.eval()
    fr = synth.synth_frames(2, 3, seed=int(g["model_frames_seed"]))
    with torch.no_grad():
        out = m(torch.from_numpy(fr[:1]).unsqueeze(2).cuda())
        feats = m.cnn(torch.from_numpy(fr[0]).unsqueeze(1).cuda())
        y = m.rnn(feats.view(1, 3, 208))
        head_out = m.head(y)
    np.testing.assert_allclose(out.cpu().numpy(), g["model_out"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(head_out.cpu().numpy(), g["model_out"], atol=1e-4, rtol=0)
    # re-loading weights invalidates the packed engine
    m.load_state_dict(_t(synth.synth_acoustic_state(0)), strict=False)
    with torch.no_grad():
        out2 = m(torch.from_numpy(fr[:1]).unsqueeze(2).cuda())
    assert not torch.allclose(out, out2)


def test_generator_plugin_after_reference_loader():
    from env import AttrDict
    from models import Generator
    from torch.nn.utils import remove_weight_norm
    g = np.load(os.path.join(GOLD, "generator.npz"))
    h = AttrDict(json.loads(bytes(g["r1_h"]).decode()))
    gen = Generator(h).to("cuda")
    gen.load_state_dict(_t(synth.synth_generator_state(int(g["seed"]), h)))
    gen.eval()
    with torch.no_grad():
        w1 = gen(torch.from_numpy(g["r1_mel"]).cuda()).cpu().numpy()
    for mod in list(gen.ups) + [gen.conv_post]:
        remove_weight_norm(mod)
    for r in gen.resblocks:
        r.remove_weight_norm()
    with torch.no_grad():
        w2 = gen(torch.from_numpy(g["r1_mel"]).cuda()).cpu().numpy()
    np.testing.assert_allclose(w1, g["r1_wav"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(w2, g["r1_wav_folded"], atol=1e-4, rtol=0)


def _cli():
    spec = importlib.util.spec_from_file_location(
        "m2s_cli_gpu", os.path.join(REPO, "mri-to-speech_amd", "scripts", "run_mri_video_inference.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_cli_end_to_end(tmp_path, dtype):
    """The reference CLI contract: checkpoint formats, plug-in dir, output files, numerics."""
    T = 9
    ac_sd = synth.synth_acoustic_state(4)
    gen_sd = synth.synth_generator_state(4)
    mean, std = synth.synth_scaler()
    ckdir = tmp_path / "ck" / "mri"
    ckdir.mkdir(parents=True)
    torch.save({"epoch": 3, "model_state_dict": _t(ac_sd), "val_loss": 0.1}, ckdir / "best.pt")
    torch.save({"generator": _t(gen_sd)}, tmp_path / "g_00000001")
    (tmp_path / "config.json").write_text(json.dumps(dict(HIFIGAN_H)))
    (tmp_path / "scaler.json").write_text(json.dumps({"mean": mean.tolist(), "std": std.tolist(), "count_frames": 5}))
    rng = np.random.default_rng(0)
    video = rng.integers(0, 256, size=(T + 2, 256, 256), dtype=np.uint8)
    np.save(tmp_path / "clip01.npy", video)
    cli = _cli()
    res = cli.main(["--video", str(tmp_path / "clip01.npy"), "--mri-checkpoint", str(ckdir / "best.pt"),
                    "--scaler-json", str(tmp_path / "scaler.json"), "--hifigan-config", str(tmp_path / "config.json"),
                    "--hifigan-checkpoint", str(tmp_path / "g_00000001"), "--output-dir", str(tmp_path / "out"),
                    "--mri-code-dir", os.path.join(REPO, "mri-to-speech_amd", "mri2speech_code"),
                    "--max-frames", str(T), "--dtype", dtype])
    out = tmp_path / "out"
    for f in ("clip01_generated.wav", "clip01_mel.npy", "clip01_mel_log.npy", "clip01_mel.png"):
        assert (out / f).exists(), f
    mel_db = np.load(out / "clip01_mel.npy")
    assert mel_db.shape == (T, 64) and res["audio"].shape == (T * 420,)
    # oracle of the same call
    frames = np.stack([acoustic.preprocess_frame(f) for f in video[:T]])
    sd = _t(ac_sd)
    f = effnet.effnet_gap(sd, torch.from_numpy(frames)).view(1, T, -1)
    mn = acoustic.head(sd, acoustic.bilstm_summerge(sd, f))[0]
    db = acoustic.denormalize_mel(mn, mean, std)
    ln = acoustic.mel_db_to_log(db)
    wav = hifigan.generator(_t(gen_sd), HIFIGAN_H, ln.t().unsqueeze(0))[0, 0].numpy()
    if dtype == "fp32":
        np.testing.assert_allclose(mel_db, db.numpy(), atol=2e-3, rtol=0)
        np.testing.assert_allclose(np.load(out / "clip01_mel_log.npy"), ln.numpy(), atol=5e-4, rtol=0)
        np.testing.assert_allclose(res["audio"], wav, atol=1e-4, rtol=0)
    else:
        assert np.abs(mel_db - db.numpy()).max() < 1.0  # dB; mel_norm x std(<=15) amplifies bf16 error


def _load(relpath, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "mri-to-speech_amd", relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_export_predicted_mels(tmp_path):
    """scripts/export_predicted_mels.py drop-in: samples/*/mri.npy (/255 frames) -> (64, T) ln-mel
    per sample (export_predicted_mels.py:84-99), equal-length samples batched, vs the oracle."""
    ac_sd = synth.synth_acoustic_state(6)
    mean, std = synth.synth_scaler()
    ck = tmp_path / "best.pt"
    torch.save({"model_state_dict": _t(ac_sd)}, ck)
    (tmp_path / "scaler.json").write_text(json.dumps({"mean": mean.tolist(), "std": std.tolist(), "count_frames": 9}))
    rng = np.random.default_rng(3)
    lens = {"utt_a": 5, "utt_b": 3, "utt_c": 5}
    for stem, T in lens.items():
        d = tmp_path / "proc" / "samples" / stem
        d.mkdir(parents=True)
        np.save(d / "mri.npy", (rng.integers(0, 256, (T, 256, 256)) / 255.0).astype(np.float32))
    (tmp_path / "proc" / "samples" / "utt_nomri").mkdir()
    mod = _load(os.path.join("scripts", "export_predicted_mels.py"), "m2s_export_mels")
    out_dir = tmp_path / "mels"
    written = mod.main(["--processed_dir", str(tmp_path / "proc"), "--mri_checkpoint", str(ck),
                        "--scaler_json", str(tmp_path / "scaler.json"), "--output_dir", str(out_dir),
                        "--mri_code_dir", os.path.join(REPO, "mri-to-speech_amd", "mri2speech_code")])
    assert sorted(p.name for p in written) == ["utt_a.npy", "utt_b.npy", "utt_c.npy"]
    sd = _t(ac_sd)
    for stem, T in lens.items():
        fr = torch.from_numpy(np.load(tmp_path / "proc" / "samples" / stem / "mri.npy"))
        f = effnet.effnet_gap(sd, fr).view(1, T, -1)
        mn = acoustic.head(sd, acoustic.bilstm_summerge(sd, f))[0]
        ref = acoustic.mel_db_to_log(acoustic.denormalize_mel(mn, mean, std)).t().numpy()
        got = np.load(out_dir / f"{stem}.npy")
        assert got.shape == (64, T) and got.dtype == np.float32
        np.testing.assert_allclose(got, ref, atol=5e-4, rtol=0)
    # existing outputs are kept unless --overwrite
    assert mod.main(["--processed_dir", str(tmp_path / "proc"), "--mri_checkpoint", str(ck),
                     "--scaler_json", str(tmp_path / "scaler.json"), "--output_dir", str(out_dir)]) == []


def test_export_predicted_mels_torchrun_ragged(tmp_path):
    """export_predicted_mels.py under torch.distributed.run, 2 ranks on this box's GPU (gloo for the
    collectives: RCCL takes one rank per GPU): ragged clips sharded by length, rank 0's weights broadcast,
    the mels gathered to rank 0, which writes every file.  Every file equals the single-process run's
    (1e-5: a clip may share its CNN / BiLSTM launch with other clips) and the oracle (5e-4)."""
    import socket
    import subprocess
    import sys
    ac_sd = synth.synth_acoustic_state(7)
    mean, std = synth.synth_scaler()
    ck = tmp_path / "best.pt"
    torch.save({"model_state_dict": _t(ac_sd)}, ck)
    (tmp_path / "scaler.json").write_text(json.dumps({"mean": mean.tolist(), "std": std.tolist()}))
    rng = np.random.default_rng(4)
    lens = {"utt_a": 5, "utt_b": 3, "utt_c": 5, "utt_d": 7, "utt_e": 2}
    for stem, T in lens.items():
        d = tmp_path / "proc" / "samples" / stem
        d.mkdir(parents=True)
        np.save(d / "mri.npy", (rng.integers(0, 256, (T, 256, 256)) / 255.0).astype(np.float32))
    script = os.path.join(REPO, "mri-to-speech_amd", "scripts", "export_predicted_mels.py")
    common = ["--processed_dir", str(tmp_path / "proc"), "--mri_checkpoint", str(ck),
              "--scaler_json", str(tmp_path / "scaler.json"),
              "--mri_code_dir", os.path.join(REPO, "mri-to-speech_amd", "mri2speech_code")]
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ, M2S_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), script, *common,
                        "--output_dir", str(tmp_path / "dist")], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    single = _load(os.path.join("scripts", "export_predicted_mels.py"), "m2s_export_mels_1")
    single.main([*common, "--output_dir", str(tmp_path / "one")])
    sd = _t(ac_sd)
    for stem, T in lens.items():
        got, one = np.load(tmp_path / "dist" / f"{stem}.npy"), np.load(tmp_path / "one" / f"{stem}.npy")
        assert got.shape == (64, T)
        np.testing.assert_allclose(got, one, atol=1e-5, rtol=0, err_msg=stem)
        fr = torch.from_numpy(np.load(tmp_path / "proc" / "samples" / stem / "mri.npy"))
        mn = acoustic.head(sd, acoustic.bilstm_summerge(sd, effnet.effnet_gap(sd, fr).view(1, T, -1)))[0]
        ref = acoustic.mel_db_to_log(acoustic.denormalize_mel(mn, mean, std)).t().numpy()
        np.testing.assert_allclose(got, ref, atol=5e-4, rtol=0, err_msg=stem)


def test_vocoder_only_callers(tmp_path):
    """inference_e2e.py and mel_to_audio_synthesis.py drop-ins: (64, T) ln-mel files -> wav, files of
    equal length batched into one generator call, malformed files reported and skipped."""
    from scipy.io import wavfile
    gen_sd = synth.synth_generator_state(8)
    ckdir = tmp_path / "cp"
    ckdir.mkdir()
    torch.save({"generator": _t(gen_sd)}, ckdir / "g_00000010")
    cfg = dict(HIFIGAN_H, seed=1234, sampling_rate=11413, n_fft=1024, hop_size=420, win_size=1024)
    (ckdir / "config.json").write_text(json.dumps(cfg))
    mels = tmp_path / "mels"
    mels.mkdir()
    inputs = {"utt_mel": synth.synth_mel_log(1, 64, 11, seed=2)[0], "b": synth.synth_mel_log(1, 64, 11, seed=4)[0],
              "c": synth.synth_mel_log(1, 64, 7, seed=5)[0]}
    for k, v in inputs.items():
        np.save(mels / f"{k}.npy", v)
    np.save(mels / "bad.npy", synth.synth_mel_log(2, 64, 5, seed=6))  # a batch of two: e2e refuses, synthesis takes row 0
    ref = {k: hifigan.generator(_t(gen_sd), HIFIGAN_H, torch.from_numpy(v)[None])[0, 0].numpy() for k, v in inputs.items()}
    ref["bad"] = hifigan.generator(_t(gen_sd), HIFIGAN_H, torch.from_numpy(synth.synth_mel_log(2, 64, 5, seed=6)[:1]))[0, 0].numpy()

    e2e = _load("inference_e2e.py", "m2s_inference_e2e")
    out = e2e.main(["--input_mels_dir", str(mels), "--output_dir", str(tmp_path / "e2e"),
                    "--checkpoint_file", str(ckdir / "g_00000010")])
    assert sorted(os.path.basename(p) for p in out) == ["b_generated_e2e.wav", "c_generated_e2e.wav",
                                                         "utt_mel_generated_e2e.wav"]
    for k in inputs:
        sr, pcm = wavfile.read(tmp_path / "e2e" / f"{k}_generated_e2e.wav")
        assert sr == 11413 and pcm.dtype == np.int16 and pcm.shape == (inputs[k].shape[1] * 420,)
        np.testing.assert_allclose(pcm.astype(np.float64), (ref[k] * 32768.0).astype(np.int16), atol=8)

    syn = _load("mel_to_audio_synthesis.py", "m2s_mel_to_audio")
    done = syn.main(["--input", str(mels), "--checkpoint_file", str(ckdir / "g_00000010"),
                     "--config", str(ckdir / "config.json"), "--output_dir", str(tmp_path / "syn")])
    assert done == ["b", "bad", "c", "utt"]
    stats = json.loads((tmp_path / "syn" / "utt_synthesis_stats.json").read_text())
    assert stats["audio_shape"] == [11 * 420] and stats["sampling_rate"] == 11413 and stats["mel_shape"] == [1, 64, 11]
    for f in ("utt_from_mel.wav", "utt_input_mel.png", "mel_synthesis_results.html", "overall_synthesis_stats.json"):
        assert (tmp_path / "syn" / f).exists(), f
    overall = json.loads((tmp_path / "syn" / "overall_synthesis_stats.json").read_text())
    assert overall["total_files"] == 4 and overall["successful_syntheses"] == 4
    for k in ("b", "bad", "c"):
        with open(tmp_path / "syn" / f"{k}_from_mel.wav", "rb") as fh:
            import wave
            with wave.open(fh) as w:
                pcm = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2")
        want = np.clip(np.rint(ref[k].astype(np.float64) * 32767.0), -32768, 32767)
        np.testing.assert_allclose(pcm.astype(np.float64), want, atol=8)
