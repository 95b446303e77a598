"""Oracle: the whole no_grad section of run_mri_video_inference.py main(), torch-CPU fp32.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Composes the restatements of this package in the reference's order
(scripts/run_mri_video_inference.py:218-242): time-distributed CNN + GAP (mri_acoustic_model.py:105-114),
BiLSTM sum-merge + head (:67-72,135), denormalize_mel + dB -> ln-power (:160-163,227-233), transpose to
(B, n_mels, T) (:238) and Generator.forward (models.py:113-131).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from . import acoustic, effnet, hifigan


def acoustic_forward(sd: Dict[str, torch.Tensor], frames: np.ndarray, cnn_chunk: int = 64) -> torch.Tensor:
    """frames (B,T,H,W) fp32 -> mel_norm (B,T,n_mels); the CNN runs in chunks of frames (exact: it is per frame)."""
    B, T, H, W = frames.shape
    flat = torch.from_numpy(np.ascontiguousarray(frames)).reshape(B * T, H, W)
    with torch.no_grad():
        feats = torch.cat([effnet.effnet_gap(sd, flat[i:i + cnn_chunk]) for i in range(0, B * T, cnn_chunk)])
        return acoustic.head(sd, acoustic.bilstm_summerge(sd, feats.view(B, T, -1)))


def e2e(ac_sd: Dict[str, torch.Tensor], gen_sd: Dict[str, torch.Tensor], h, frames: np.ndarray, mean, std,
        cnn_chunk: int = 64) -> Dict[str, np.ndarray]:
    """frames (B,T,H,W) -> mel_norm, mel_db, mel_log (B,T,n_mels) and wav (B, T*hop)."""
    mn = acoustic_forward(ac_sd, frames, cnn_chunk)
    with torch.no_grad():
        db = acoustic.denormalize_mel(mn, mean, std)
        ln = acoustic.mel_db_to_log(db)
        wav = hifigan.generator(gen_sd, h, ln.transpose(1, 2))[:, 0]
    return {"mel_norm": mn.numpy(), "mel_db": db.numpy(), "mel_log": ln.numpy(), "wav": wav.numpy()}
