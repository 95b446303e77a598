"""Command-line driver: rtMRI video -> 64-bin mel -> 11 413 Hz waveform on MI355X.

Drop-in for the reference's scripts/run_mri_video_inference.py: the same flags (:187-200), the same
plug-in loading (``--mri-code-dir`` on sys.path, ``build_acoustic_model(**kw)``, ``.pt`` with or
without ``model_state_dict``, ``load_state_dict(strict=False)``; :119-148), the same HiFi-GAN loading
(``Generator(AttrDict(config))``, strict ``ckpt['generator']``, best-effort weight-norm removal;
:89-116) and the same output files (``{stem}_generated.wav`` PCM-16, ``{stem}_mel.npy`` (T, n_mels)
dB, ``{stem}_mel.png``, ``{stem}_mel_log.npy`` (T, n_mels) ln-power; :166-184, :245-249).  The helper
names the Grad-CAM tool imports from this module (``build_mri_model``, ``frames_to_tensor``,
``load_scaler``, ``load_video_frames``; mri_gradcam_formant.py:25-30) keep their signatures.

How it runs (this is not the reference's control flow):

* ``FrameStream`` decodes on a worker thread in chunks (OpenCV for video files, or a ``.npy``
  (T,H,W[,3]) uint8 stack), stages each chunk in pinned host memory, copies it on a side HIP stream
  and normalises it there (``torch.ops.m2s.preprocess_frames``: BGR -> grey, per-frame z-score +
  min-max, :34-54), so chunk k+1 decodes while chunk k crosses PCIe and normalises.
* ``run`` hands the whole clip to ONE ``torch.ops.m2s.pipeline_forward`` call when both loaded
  modules are the m2s plug-ins: CNN -> BiLSTM -> head -> de-normalise -> dB -> ln -> generator stay on
  the device, with no host round trip between the mel and the waveform.  Any other plug-in module
  is driven through its own ``forward`` with the device mel glue in between.
* ``--dtype`` (additive) picks bf16x3 (default, fp32 tolerance), fp32 (exact f32 MFMA) or bf16.

No CPU fallback: without a HIP device the script stops.  The wav goes through soundfile when it is
installed, else through ``wave`` as 16-bit PCM with soundfile's scaling (round(x * 32767)).
"""
from __future__ import annotations

import argparse
import json
import queue
import sys
import threading
from pathlib import Path

import numpy as np
import torch

PROJECT_ROOT = Path(__file__).resolve().parents[1]
if str(PROJECT_ROOT) not in sys.path:
    sys.path.insert(0, str(PROJECT_ROOT))

from env import AttrDict  # noqa: E402
from models import Generator  # noqa: E402
from m2s import drivers, runtime  # noqa: E402

try:  # host-side decoders the reference uses; absent from this image
    import cv2
except ImportError:  # pragma: no cover
    cv2 = None

TARGET = (256, 256)


# ------------------------------------------------------------------------------------------------
# frames
class FrameStream:
    """Chunked decode (worker thread) -> pinned staging -> H2D + device normalisation (side stream)."""

    def __init__(self, path: Path, device: torch.device, max_frames=None, chunk: int = 64, target=TARGET):
        self.path, self.device, self.max_frames, self.chunk, self.target = Path(path), device, max_frames, chunk, target

    def _host_chunks(self):
        """uint8 frame arrays at the target size, `chunk` frames at a time."""
        limit = self.max_frames if self.max_frames is not None else 1 << 62
        if self.path.suffix.lower() == ".npy":
            stack = np.load(self.path, mmap_mode="r", allow_pickle=False)
            stack = stack[:limit]
            for i in range(0, len(stack), self.chunk):
                yield [self._fit(np.asarray(f)) for f in stack[i:i + self.chunk]]
            return
        if cv2 is None:
            raise RuntimeError("OpenCV is not installed; pass the frames as a .npy (T,H,W) uint8 stack")
        cap = cv2.VideoCapture(str(self.path))
        if not cap.isOpened():
            raise ValueError(f"cannot open video {self.path}")
        n = min(int(cap.get(cv2.CAP_PROP_FRAME_COUNT)), limit)
        buf = []
        try:
            for _ in range(n):
                ok, f = cap.read()
                if not ok:
                    break
                buf.append(self._fit(f))
                if len(buf) == self.chunk:
                    yield buf
                    buf = []
        finally:
            cap.release()
        if buf:
            yield buf

    def _fit(self, f: np.ndarray) -> np.ndarray:
        if f.dtype != np.uint8:
            raise ValueError(f"expected 8-bit frames, got {f.dtype}")
        if f.shape[:2][::-1] == tuple(self.target):
            return f
        if cv2 is None:
            raise ValueError(f"frame of size {f.shape[:2]} needs a resize to {self.target} and OpenCV is missing")
        g = cv2.cvtColor(f, cv2.COLOR_BGR2GRAY) if f.ndim == 3 else f  # the reference resizes the grey frame
        return cv2.resize(g, self.target, interpolation=cv2.INTER_LINEAR)

    def read(self) -> torch.Tensor:
        """All frames as one (T,H,W) fp32 device tensor in [0, 1], on the current stream."""
        q: "queue.Queue" = queue.Queue(maxsize=2)

        def worker():
            try:
                for c in self._host_chunks():
                    shapes = {a.shape for a in c}
                    if len(shapes) > 1:  # mixed grey / colour frames: grey them on the host
                        c = [cv2.cvtColor(a, cv2.COLOR_BGR2GRAY) if a.ndim == 3 else a for a in c]
                    q.put(torch.from_numpy(np.ascontiguousarray(np.stack(c))).pin_memory())
            except BaseException as e:  # surfaced in the consumer
                q.put(e)
            q.put(None)

        threading.Thread(target=worker, daemon=True).start()
        side = torch.cuda.Stream(self.device)
        parts = []
        while True:
            item = q.get()
            if item is None:
                break
            if isinstance(item, BaseException):
                raise item
            with torch.cuda.stream(side):  # the pinned block stays reserved until this copy completes
                parts.append(runtime.preprocess_frames(item.to(self.device, non_blocking=True)))
        torch.cuda.current_stream(self.device).wait_stream(side)
        if not parts:
            raise ValueError(f"no frames could be read from {self.path}")
        for p in parts:
            p.record_stream(torch.cuda.current_stream(self.device))
        return parts[0] if len(parts) == 1 else torch.cat(parts)


def load_video_frames(video_path: Path, target_size=TARGET, max_frames=None) -> torch.Tensor:
    """(T,H,W) fp32 frames in [0, 1] on the host (the Grad-CAM tool moves them itself)."""
    return FrameStream(Path(video_path), torch.device("cuda"), max_frames, target=target_size).read().cpu()


def frames_to_tensor(frames: torch.Tensor, use_channel: bool = True) -> torch.Tensor:
    """(T,H,W) -> (1,T,1,H,W) (or (1,T,H,W) without the channel axis)."""
    if frames.dim() != 3:
        raise ValueError(f"expected (T,H,W) frames, got {tuple(frames.shape)}")
    return frames[None, :, None] if use_channel else frames[None]


def load_scaler(stats_path: Path):
    """scaler.json {"mean": [n_mels], "std": [n_mels], ...} -> float32 arrays."""
    stats = json.loads(Path(stats_path).read_text(encoding="utf-8"))
    try:
        mean, std = (np.asarray(stats[k], dtype=np.float32) for k in ("mean", "std"))
    except KeyError as e:
        raise KeyError("scaler JSON needs 'mean' and 'std' lists") from e
    if mean.ndim != 1 or std.ndim != 1:
        raise ValueError("scaler mean/std must be 1-D lists")
    return mean, std


# ------------------------------------------------------------------------------------------------
# models
def build_mri_model(args, device: torch.device):
    """The acoustic model through the plug-in surface: --mri-code-dir (default <ckpt>/../../mri2speech_code)."""
    code_dir = Path(args.mri_code_dir) if getattr(args, "mri_code_dir", None) else \
        Path(args.mri_checkpoint).resolve().parent.parent / "mri2speech_code"
    return drivers.build_acoustic(args.mri_checkpoint, device, code_dir=code_dir, n_mels=args.n_mels,
                                  rnn_hidden=args.rnn_hidden, dropout=args.dropout,
                                  dtype=getattr(args, "dtype", None))


def load_hifigan(config_path: Path, checkpoint_path: Path, device: torch.device, dtype=None):
    h = AttrDict(json.loads(Path(config_path).read_text(encoding="utf-8")))
    gen, _ = drivers.build_generator(h, checkpoint_path, device, dtype)
    return gen, h


# ------------------------------------------------------------------------------------------------
# run
def run(model, gen, frames: torch.Tensor, mean: np.ndarray, std: np.ndarray):
    """(T,H,W) device frames -> dict mel_db (T,n_mels), mel_log (T,n_mels), audio (T*hop,) on the host.

    On the m2s path the acoustic engine's asynchronous failure report (a BiLSTM barrier timeout
    poisons the outputs with NaN, include/m2s.h m2s_acoustic_status) is read after the results reach
    the host, and raises instead of letting NaN outputs be written."""
    dev = frames.device
    if hasattr(model, "_engine") and hasattr(gen, "_engine"):  # both are m2s plug-ins: one device call
        eng = model._engine(dev)
        pipe = runtime.Pipeline(eng, gen._engine(dev), mean, std)
        out = pipe.forward(frames[None])
        res = {"mel_db": out["mel_db"][0], "mel_log": out["mel_log"][0], "audio": out["wav"][0]}
        res = {k: v.float().cpu().numpy() for k, v in res.items()}
        eng.check()
        return res
    with torch.no_grad():  # a foreign plug-in: its forward, then the device glue and the generator
        mn = model(frames_to_tensor(frames))[0]
        db, ln = runtime.mel_glue(mn, torch.from_numpy(mean), torch.from_numpy(std))
        wav = gen(ln.t()[None]).reshape(-1)
    return {"mel_db": db.float().cpu().numpy(), "mel_log": ln.float().cpu().numpy(), "audio": wav.float().cpu().numpy()}


def write_wav(path: Path, audio: np.ndarray, sr: int):
    drivers.write_wav_pcm16(path, audio, sr)


def write_outputs(res, out_dir: Path, stem: str, sr: int):
    out_dir.mkdir(parents=True, exist_ok=True)
    paths = {"audio": out_dir / f"{stem}_generated.wav", "mel": out_dir / f"{stem}_mel.npy",
             "figure": out_dir / f"{stem}_mel.png", "mel_log": out_dir / f"{stem}_mel_log.npy"}
    write_wav(paths["audio"], res["audio"], sr)
    np.save(paths["mel"], res["mel_db"].astype(np.float32))
    np.save(paths["mel_log"], res["mel_log"].astype(np.float32))
    try:
        import matplotlib
        matplotlib.use("Agg")
        from matplotlib import pyplot as plt
        fig, ax = plt.subplots(figsize=(12, 4))
        im = ax.imshow(res["mel_db"].T, aspect="auto", origin="lower", cmap="viridis")
        fig.colorbar(im, ax=ax)
        ax.set(title=f"Generated Mel Spectrogram - {stem}", xlabel="Time", ylabel="Mel bins")
        fig.tight_layout()
        fig.savefig(paths["figure"], dpi=150)
        plt.close(fig)
    except ImportError:  # pragma: no cover
        paths["figure"] = None
    return paths


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="rtMRI video -> mel -> waveform (CNN-BiLSTM + HiFi-GAN) on MI355X")
    req = [("--video", "rtMRI video, or a (T,H,W[,3]) uint8 .npy frame stack"),
           ("--mri-checkpoint", "acoustic-model checkpoint (.pt)"),
           ("--scaler-json", "scaler.json with the per-bin mel mean/std"),
           ("--hifigan-config", "HiFi-GAN config JSON"),
           ("--hifigan-checkpoint", "HiFi-GAN generator checkpoint (g_XXXXXXXX)"),
           ("--output-dir", "where the wav / npy / png outputs go")]
    for flag, help_ in req:
        p.add_argument(flag, required=True, help=help_)
    p.add_argument("--mri-code-dir", help="directory with mri_acoustic_model.py (default: <ckpt>/../../mri2speech_code)")
    p.add_argument("--max-frames", type=int, default=None, help="decode at most this many frames")
    p.add_argument("--n-mels", type=int, default=64)
    p.add_argument("--rnn-hidden", type=int, default=640)
    p.add_argument("--dropout", type=float, default=0.5)
    p.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None,
                   help="m2s compute dtype (default: M2S_DTYPE or bf16x3)")
    p.add_argument("--decode-chunk", type=int, default=64, help="frames per decode / H2D chunk")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    video = Path(args.video)
    if not video.exists():
        raise FileNotFoundError(f"video not found: {video}")
    mean, std = load_scaler(Path(args.scaler_json))
    if len(mean) != args.n_mels or len(std) != args.n_mels:
        raise ValueError("scaler mean/std length does not match --n-mels")
    if not torch.cuda.is_available():
        raise RuntimeError("m2s needs an MI355X (HIP) device; there is no CPU path")
    device = torch.device("cuda")

    model = build_mri_model(args, device)
    gen, h = load_hifigan(Path(args.hifigan_config), Path(args.hifigan_checkpoint), device, args.dtype)
    frames = FrameStream(video, device, args.max_frames, chunk=args.decode_chunk).read()
    res = run(model, gen, frames, mean, std)
    paths = write_outputs(res, Path(args.output_dir), video.stem, int(h.sampling_rate))
    print(f"[m2s] {frames.shape[0]} frames -> mel {res['mel_db'].shape} -> {res['audio'].shape[0]} samples "
          f"@ {int(h.sampling_rate)} Hz ({model.m2s_dtype if hasattr(model, 'm2s_dtype') else 'plug-in'})")
    for k, v in paths.items():
        print(f"  {k:8s}: {v}")
    return res


if __name__ == "__main__":
    main()
