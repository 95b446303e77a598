"""Export predicted log-mel features, drop-in for scripts/export_predicted_mels.py on MI355X.

Same command line (--processed_dir --mri_checkpoint --scaler_json --output_dir [--mri_code_dir
--overwrite]), same plug-in (``build_acoustic_model(**kw)`` from --mri_code_dir, checkpoint
``model_state_dict`` or raw state dict, ``load_state_dict(strict=False)`` with the missing /
unexpected keys printed; export_predicted_mels.py:19-40), same input (``samples/*/mri.npy``, (T,H,W)
float32 frames already /255, preprocess_rtmri_data.py:113) and the same output: one
``{sample}.npy`` ln-mel of shape (n_mels, T) float32 per sample (export_predicted_mels.py:84-99),
existing files skipped unless --overwrite.

The acoustic model and the mel glue (y*std + mean -> 10^(x/10) -> clamp(1e-5) -> ln) run in libm2s
on the GPU.  Additive: ``--dtype`` and ``--batch`` (samples of equal length go through one forward
call, up to --batch clips).  ``--cpu`` is rejected: there is no CPU path.
"""
from __future__ import annotations

import argparse
import json
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np
import torch

PROJECT_ROOT = Path(__file__).resolve().parents[1]
if str(PROJECT_ROOT) not in sys.path:
    sys.path.insert(0, str(PROJECT_ROOT))

from m2s.runtime import mel_glue  # noqa: E402

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    def tqdm(x, **_):
        return x


def load_scaler(scaler_path: Path):
    with scaler_path.open("r", encoding="utf-8") as handle:
        stats = json.load(handle)
    return torch.tensor(stats["mean"], dtype=torch.float32), torch.tensor(stats["std"], dtype=torch.float32)


def build_model(checkpoint_path: Path, n_mels: int, device: torch.device, dtype=None):
    from mri_acoustic_model import build_acoustic_model

    model = build_acoustic_model(n_mels=n_mels, cnn_pretrained=False, rnn_hidden=640, dropout=0.5,
                                 use_checkpoint=False, ckpt_segments=2, use_reentrant=False).to(device)
    checkpoint = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    state_dict = checkpoint.get("model_state_dict", checkpoint)
    missing, unexpected = model.load_state_dict(state_dict, strict=False)
    if missing:
        print(f"[WARN] missing keys when loading MRI model: {missing}")
    if unexpected:
        print(f"[WARN] unexpected keys when loading MRI model: {unexpected}")
    model.eval()
    if dtype:
        model.m2s_dtype = dtype
    return model


def export_mels(args: argparse.Namespace) -> list:
    processed_dir = Path(args.processed_dir).resolve()
    samples_dir = processed_dir / "samples"
    if not samples_dir.is_dir():
        raise SystemExit(f"samples directory not found: {samples_dir}")
    output_dir = Path(args.output_dir).resolve()
    output_dir.mkdir(parents=True, exist_ok=True)
    mean, std = load_scaler(Path(args.scaler_json).resolve())
    if mean.numel() != std.numel():
        raise SystemExit("Scaler mean/std length mismatch")
    n_mels = mean.numel()
    if args.cpu:
        raise SystemExit("--cpu: m2s runs on MI355X only (no CPU path); drop the flag")
    if not torch.cuda.is_available():
        raise SystemExit("m2s needs an MI355X (HIP) device; none is visible")
    device = torch.device("cuda")
    print(f"[INFO] Using device: {device}")
    if args.mri_code_dir:
        code_dir = Path(args.mri_code_dir).resolve()
        if code_dir.is_dir() and str(code_dir) not in sys.path:
            sys.path.insert(0, str(code_dir))
    model = build_model(Path(args.mri_checkpoint).resolve(), n_mels, device, args.dtype)
    mean, std = mean.to(device), std.to(device)

    sample_dirs = sorted([p for p in samples_dir.iterdir() if p.is_dir()], key=lambda p: p.name)
    if not sample_dirs:
        raise SystemExit(f"No sample folders found under {samples_dir}")
    todo = defaultdict(list)  # frame shape -> [(stem, frames)]
    for sample_path in sample_dirs:
        stem = sample_path.name
        out_path = output_dir / f"{stem}.npy"
        if out_path.exists() and not args.overwrite:
            continue
        mri_path = sample_path / "mri.npy"
        if not mri_path.is_file():
            print(f"[WARN] MRI file missing for {stem}, skipping")
            continue
        mri = np.load(mri_path, allow_pickle=False).astype(np.float32)
        todo[mri.shape].append((stem, mri))

    written = []
    with torch.no_grad():
        groups = [(shape, items[i:i + args.batch]) for shape, items in todo.items()
                  for i in range(0, len(items), args.batch)]
        for _, group in tqdm(groups, desc="Exporting mels"):
            frames = torch.from_numpy(np.stack([m for _, m in group])).unsqueeze(2).to(device)  # (B,T,1,H,W)
            pred_norm = model(frames)  # (B, T, n_mels)
            _, mel_log = mel_glue(pred_norm, mean, std)
            mel_log_np = mel_log.transpose(1, 2).cpu().numpy().astype(np.float32)  # (B, n_mels, T)
            for (stem, _), m in zip(group, mel_log_np):
                out_path = output_dir / f"{stem}.npy"
                np.save(out_path, m)
                written.append(out_path)
    return written


def parse_args(argv=None) -> argparse.Namespace:
    parser = argparse.ArgumentParser(description="Export predicted log-mel features for HiFi-GAN fine-tuning (MI355X).")
    parser.add_argument("--processed_dir", required=True, help="rtMRI processed dataset root (contains samples/).")
    parser.add_argument("--mri_checkpoint", required=True, help="Path to trained MRI->mel checkpoint (.pt).")
    parser.add_argument("--scaler_json", required=True, help="Path to scaler.json (mean/std for denormalization).")
    parser.add_argument("--output_dir", required=True,
                        help="Directory to store generated log-mel numpy files (one per sample, shape [64, T]).")
    parser.add_argument("--mri_code_dir", help="Directory containing mri_acoustic_model.py (if not importable by default).")
    parser.add_argument("--cpu", action="store_true", help="Rejected: m2s has no CPU execution path.")
    parser.add_argument("--overwrite", action="store_true", help="Regenerate files even if they already exist.")
    parser.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None, help="m2s compute dtype (default fp32)")
    parser.add_argument("--batch", type=int, default=16, help="clips of equal length per forward call")
    return parser.parse_args(argv)


def main(argv=None):
    return export_mels(parse_args(argv))


if __name__ == "__main__":
    main()
