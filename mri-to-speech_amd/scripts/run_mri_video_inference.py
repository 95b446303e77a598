"""rtMRI video -> mel -> waveform, drop-in for scripts/run_mri_video_inference.py on MI355X.

Same command line (--video --mri-checkpoint --scaler-json --hifigan-config --hifigan-checkpoint
--output-dir [--mri-code-dir --max-frames --n-mels --rnn-hidden --dropout]), same plug-in loading
(``--mri-code-dir`` on sys.path, ``build_acoustic_model(**kw)``, ``load_state_dict(strict=False)``),
same HiFi-GAN loading (``Generator(AttrDict(config))``, strict ``ckpt['generator']``, best-effort
weight-norm removal) and the same output files ({stem}_generated.wav, {stem}_mel.npy (T,64) dB,
{stem}_mel.png, {stem}_mel_log.npy (T,64)).  Additive flag: ``--dtype {fp32,bf16}``.

The acoustic model, the mel glue and the generator run in libm2s on the GPU; there is no CPU
fallback (the reference's ``device = cuda if available else cpu`` becomes a hard requirement).
Host I/O: OpenCV decodes video when installed; a ``.npy`` (T,H,W[,3]) frame stack is accepted
too.  The wav is written by soundfile when installed, else as 16-bit PCM by ``wave``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import wave
from pathlib import Path

import numpy as np
import torch

PROJECT_ROOT = Path(__file__).resolve().parents[1]
if str(PROJECT_ROOT) not in sys.path:
    sys.path.insert(0, str(PROJECT_ROOT))

from env import AttrDict  # noqa: E402
from models import Generator  # noqa: E402
from m2s.runtime import mel_glue, preprocess_frames  # noqa: E402

try:  # optional host-side decoders, exactly as the reference uses them
    import cv2  # noqa: F401
except ImportError:  # pragma: no cover - absent in this image
    cv2 = None
try:
    import soundfile as sf
except ImportError:  # pragma: no cover
    sf = None


def _ensure_sys_path(path: Path):
    if path and path.exists():
        sys.path.insert(0, str(path))


def _preprocess_frame(frame: np.ndarray, target_size=(256, 256)) -> np.ndarray:
    """Grey, resize to 256x256, per-frame z-score then min-max to [0, 1] (reference :34-54)."""
    if frame.ndim == 3:
        if cv2 is not None:
            gray = cv2.cvtColor(frame, cv2.COLOR_BGR2GRAY)
        else:  # ITU-R 601 luma, the weights COLOR_BGR2GRAY applies
            f = frame.astype(np.float32)
            gray = np.clip(np.rint(0.114 * f[..., 0] + 0.587 * f[..., 1] + 0.299 * f[..., 2]), 0, 255).astype(np.uint8)
    else:
        gray = frame
    if gray.shape[::-1] != tuple(target_size):
        if cv2 is None:
            raise ValueError(f"frame size {gray.shape} != {target_size} and OpenCV is not installed to resize")
        gray = cv2.resize(gray, target_size, interpolation=cv2.INTER_LINEAR)
    gray = gray.astype(np.float32)
    mean, std = gray.mean(), gray.std()
    gray = (gray - mean) / std if std > 0 else gray - mean
    lo, hi = gray.min(), gray.max()
    return (gray - lo) / (hi - lo) if hi > lo else np.zeros_like(gray)


def decode_video_frames(video_path: Path, target_size=(256, 256), max_frames=None) -> np.ndarray:
    """Host half of load_video_frames: decoded uint8 frames, (T,H,W) grey or (T,H,W,3) BGR at
    `target_size`.  Frames of another size are converted to grey and resized here (cv2, as the
    reference does); the z-score / min-max normalisation runs on the device
    (m2s.runtime.preprocess_frames)."""
    if video_path.suffix.lower() == ".npy":
        raw = np.load(video_path, allow_pickle=False)
        if max_frames is not None:
            raw = raw[:max_frames]
        raw = list(raw)
    else:
        if cv2 is None:
            raise RuntimeError("OpenCV is not installed; pass the frames as a .npy (T,H,W) array instead")
        cap = cv2.VideoCapture(str(video_path))
        if not cap.isOpened():
            raise ValueError(f"Unable to open video: {video_path}")
        total = int(cap.get(cv2.CAP_PROP_FRAME_COUNT))
        if max_frames is not None:
            total = min(total, max_frames)
        raw = []
        for _ in range(total):
            ret, frame = cap.read()
            if not ret:
                break
            raw.append(frame)
        cap.release()
    if not len(raw):
        raise ValueError("No frames could be read from video")
    out = []
    for f in raw:
        f = np.asarray(f)
        if f.dtype != np.uint8:
            raise ValueError(f"expected 8-bit frames, got {f.dtype}")
        if f.shape[:2][::-1] != tuple(target_size):
            if cv2 is None:
                raise ValueError(f"frame size {f.shape[:2]} != {target_size} and OpenCV is not installed to resize")
            g = cv2.cvtColor(f, cv2.COLOR_BGR2GRAY) if f.ndim == 3 else f
            f = cv2.resize(g, target_size, interpolation=cv2.INTER_LINEAR)
        out.append(f)
    if len({a.shape for a in out}) != 1:
        out = [cv2.cvtColor(a, cv2.COLOR_BGR2GRAY) if a.ndim == 3 else a for a in out]
    return np.ascontiguousarray(np.stack(out))


def load_video_frames(video_path: Path, target_size=(256, 256), max_frames=None) -> torch.Tensor:
    if video_path.suffix.lower() == ".npy":
        raw = np.load(video_path, allow_pickle=False)
        if max_frames is not None:
            raw = raw[:max_frames]
        frames = [_preprocess_frame(f, target_size) for f in raw]
    else:
        if cv2 is None:
            raise RuntimeError("OpenCV is not installed; pass the frames as a .npy (T,H,W) array instead")
        cap = cv2.VideoCapture(str(video_path))
        if not cap.isOpened():
            raise ValueError(f"Unable to open video: {video_path}")
        total = int(cap.get(cv2.CAP_PROP_FRAME_COUNT))
        if max_frames is not None:
            total = min(total, max_frames)
        frames = []
        for _ in range(total):
            ret, frame = cap.read()
            if not ret:
                break
            frames.append(_preprocess_frame(frame, target_size))
        cap.release()
    if not len(frames):
        raise ValueError("No frames could be read from video")
    return torch.from_numpy(np.asarray(frames, dtype=np.float32))


def load_scaler(stats_path: Path):
    with open(stats_path, "r", encoding="utf-8") as f:
        stats = json.load(f)
    if "mean" not in stats or "std" not in stats:
        raise KeyError("Scaler JSON must contain 'mean' and 'std' lists")
    mean = np.asarray(stats["mean"], dtype=np.float32)
    std = np.asarray(stats["std"], dtype=np.float32)
    if mean.ndim != 1 or std.ndim != 1:
        raise ValueError("Scaler mean/std must be 1-D lists")
    return mean, std


def _set_dtype(module, dtype):
    if dtype:
        module.m2s_dtype = dtype


def load_hifigan(config_path: Path, checkpoint_path: Path, device: torch.device, dtype=None):
    with open(config_path, "r", encoding="utf-8") as f:
        h = AttrDict(json.load(f))
    generator = Generator(h).to(device)
    ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    if "generator" not in ckpt:
        raise KeyError("HiFi-GAN checkpoint missing 'generator' state")
    generator.load_state_dict(ckpt["generator"])
    generator.eval()
    from torch.nn.utils import remove_weight_norm
    for module in list(generator.ups) + [generator.conv_post]:
        try:
            remove_weight_norm(module)
        except (ValueError, AttributeError):
            pass
    for res in generator.resblocks:
        try:
            res.remove_weight_norm()
        except (ValueError, AttributeError):
            pass
    _set_dtype(generator, dtype)
    return generator, h


def build_mri_model(args, device: torch.device):
    code_dir = Path(args.mri_code_dir) if args.mri_code_dir else None
    if code_dir is None:
        code_dir = Path(args.mri_checkpoint).resolve().parent.parent / "mri2speech_code"
    _ensure_sys_path(code_dir)
    try:
        from mri_acoustic_model import build_acoustic_model
    except ImportError as exc:
        raise ImportError("Failed to import mri_acoustic_model. Use --mri-code-dir to point to the "
                          "mri2speech_code directory.") from exc
    model_kwargs = {"n_mels": args.n_mels, "cnn_pretrained": False, "rnn_hidden": args.rnn_hidden,
                    "dropout": args.dropout, "use_checkpoint": False, "ckpt_segments": 2, "use_reentrant": False}
    model = build_acoustic_model(**model_kwargs).to(device)
    checkpoint = torch.load(args.mri_checkpoint, map_location="cpu", weights_only=True)
    state_dict = checkpoint.get("model_state_dict", checkpoint)
    missing, unexpected = model.load_state_dict(state_dict, strict=False)
    if missing:
        print(f"[WARN] Missing keys when loading MRI model: {missing}")
    if unexpected:
        print(f"[WARN] Unexpected keys when loading MRI model: {unexpected}")
    model.eval()
    _set_dtype(model, getattr(args, "dtype", None))
    return model


def frames_to_tensor(frames: torch.Tensor, use_channel: bool = True) -> torch.Tensor:
    if frames.dim() != 3:
        raise ValueError(f"Expected frames tensor of shape (T,H,W), got {tuple(frames.shape)}")
    frames = frames.unsqueeze(0)
    if use_channel:
        frames = frames.unsqueeze(2)
    return frames


def denormalize_mel(mel_normalized: torch.Tensor, mean: np.ndarray, std: np.ndarray) -> torch.Tensor:
    return mel_glue(mel_normalized, torch.from_numpy(mean), torch.from_numpy(std))[0]


def _write_wav(path: Path, audio: np.ndarray, sr: int):
    if sf is not None:
        sf.write(path, audio, sr)
        return
    pcm = np.clip(np.rint(np.asarray(audio, np.float64) * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sr))
        w.writeframes(pcm.tobytes())


def save_outputs(audio: np.ndarray, mel: np.ndarray, output_dir: Path, sampling_rate: int, stem: str):
    output_dir.mkdir(parents=True, exist_ok=True)
    audio_path = output_dir / f"{stem}_generated.wav"
    _write_wav(audio_path, audio, sampling_rate)
    mel_path = output_dir / f"{stem}_mel.npy"
    np.save(mel_path, mel)
    fig_path = output_dir / f"{stem}_mel.png"
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        plt.figure(figsize=(12, 4))
        plt.imshow(mel.T, aspect="auto", origin="lower", cmap="viridis")
        plt.colorbar()
        plt.title(f"Generated Mel Spectrogram - {stem}")
        plt.xlabel("Time")
        plt.ylabel("Mel bins")
        plt.tight_layout()
        plt.savefig(fig_path, dpi=150)
        plt.close()
    except ImportError:  # pragma: no cover
        fig_path = None
    return audio_path, mel_path, fig_path


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="rtMRI -> Speech inference (OTN-like MRI model + HiFi-GAN) on MI355X")
    p.add_argument("--video", required=True, help="Input rtMRI video (.mp4) or frame stack (.npy)")
    p.add_argument("--mri-checkpoint", required=True, help="Path to OTN-like MRI checkpoint (.pt)")
    p.add_argument("--scaler-json", required=True, help="Path to scaler.json (contains per-mel mean/std)")
    p.add_argument("--hifigan-config", required=True, help="HiFi-GAN config JSON")
    p.add_argument("--hifigan-checkpoint", required=True, help="HiFi-GAN generator checkpoint")
    p.add_argument("--output-dir", required=True, help="Directory to save generated artifacts")
    p.add_argument("--mri-code-dir", help="Directory containing mri_acoustic_model.py (defaults to sibling mri2speech_code)")
    p.add_argument("--max-frames", type=int, default=None, help="Optional max number of frames to process")
    p.add_argument("--n-mels", type=int, default=64)
    p.add_argument("--rnn-hidden", type=int, default=640)
    p.add_argument("--dropout", type=float, default=0.5)
    p.add_argument("--dtype", choices=["fp32", "bf16"], default=None,
                   help="m2s compute dtype (default: M2S_DTYPE env or fp32)")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    video_path = Path(args.video)
    if not video_path.exists():
        raise FileNotFoundError(f"Video file not found: {video_path}")
    mean, std = load_scaler(Path(args.scaler_json))
    if len(mean) != args.n_mels or len(std) != args.n_mels:
        raise ValueError("Scaler mean/std length does not match n_mels")
    if not torch.cuda.is_available():
        raise RuntimeError("m2s needs an MI355X (HIP) device; no CPU fallback")
    device = torch.device("cuda")
    print(f"[INFO] Using device: {device}")

    # host: decode (+ resize when needed); device: grey, z-score, min-max (libm2s preprocess kernel)
    frames_u8 = decode_video_frames(video_path, target_size=(256, 256), max_frames=args.max_frames)
    frames = preprocess_frames(torch.from_numpy(frames_u8).to(device))
    frames_tensor = frames_to_tensor(frames, use_channel=True)

    mri_model = build_mri_model(args, device)
    with torch.no_grad():
        pred_norm = mri_model(frames_tensor)
    pred_norm = pred_norm.squeeze(0)
    print(f"[INFO] Predicted normalized mel shape: {tuple(pred_norm.shape)}")

    mel_denorm, mel_log = mel_glue(pred_norm, torch.from_numpy(mean), torch.from_numpy(std))
    mel_denorm_np = mel_denorm.cpu().numpy().astype(np.float32)
    print(f"[INFO] Mel (denormalized dB) range: {mel_denorm_np.min():.3f} .. {mel_denorm_np.max():.3f}")
    mel_log_np = mel_log.cpu().numpy().astype(np.float32)
    print(f"[INFO] Mel (log-power) range: {mel_log_np.min():.3f} .. {mel_log_np.max():.3f}")

    generator, hifigan_config = load_hifigan(Path(args.hifigan_config), Path(args.hifigan_checkpoint), device,
                                             args.dtype)
    mel_for_hifigan = mel_log.transpose(0, 1).unsqueeze(0).float().to(device)
    with torch.no_grad():
        audio = generator(mel_for_hifigan).squeeze().cpu().numpy()
    print(f"[INFO] Generated audio length: {audio.shape[0]} samples")

    stem = video_path.stem
    output_dir = Path(args.output_dir)
    audio_path, mel_path, fig_path = save_outputs(audio, mel_denorm_np, output_dir, hifigan_config.sampling_rate, stem)
    log_mel_path = output_dir / f"{stem}_mel_log.npy"
    np.save(log_mel_path, mel_log_np)
    print("[DONE] Inference complete.")
    print(f"  Audio : {audio_path}")
    print(f"  Mel   : {mel_path}")
    print(f"  LogMel: {log_mel_path}")
    print(f"  Figure: {fig_path}")
    return {"audio": audio, "mel_db": mel_denorm_np, "mel_log": mel_log_np}


if __name__ == "__main__":
    main()
