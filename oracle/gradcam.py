"""Oracle: the reference's Grad-CAM computation, torch-CPU fp32 autograd over the oracle modules.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates scripts/mri_gradcam_formant.py of the reference:
* ``_forward_with_features`` (:128-166): (B,T,1,H,W) frames -> (B*T,3,H,W) repeat -> backbone in train
  mode -> last feature map as a gradient leaf -> mean over (H,W) -> BiLSTM sum merge -> head;
* ``compute_gradcam`` (:203-279): model.train() with the rnn dropout in eval (:221-225), de-normalised
  mel (:230-231, denormalize_mel :122-125), power 10^(dB/10), band power summed over ``band_indices``
  (:233-234), target = mean or sum over (B,T) (:243-247), backward, and per requested frame a target of
  that frame's band power (:254-266);
* ``_compute_cam_from_grads`` (:169-200): channel weights = spatial mean of the gradient, ReLU of the
  weighted feature sum, bilinear resize (align_corners=False) to the frame size, per-frame min-max
  normalisation with +1e-6.

The backbone's train-mode BatchNorm (batch statistics, running statistics updated) is
oracle/effnet.py ``effnet_features(train=True)``; the BiLSTM is oracle/acoustic.py's explicit loop,
which autograd differentiates.  Parity of the pieces: BiLSTM / head pinned by tests/golden
(acoustic.npz); the timm backbone is parity unpinned (oracle/effnet.py).
"""
from __future__ import annotations

from typing import Dict, Iterable, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import acoustic, effnet


def forward_with_features(sd: Dict[str, torch.Tensor], frames: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """frames (B,T,1,H,W) -> (pred_norm (B,T,n_mels), feats (B*T,208,h,w) gradient leaf).
    ``sd``'s BatchNorm running statistics are updated (train mode)."""
    B, T = frames.shape[:2]
    x = frames.reshape(B * T, *frames.shape[2:])
    x = x.repeat(1, 3, 1, 1)
    with torch.no_grad():
        feats = effnet.effnet_features(sd, x, train=True)
    feats = feats.detach().requires_grad_(True)
    seq = feats.mean(dim=(2, 3)).view(B, T, -1)
    pred = acoustic.head(sd, acoustic.bilstm_summerge_loop(sd, seq))
    return pred, feats


def cam_from_grads(feats: torch.Tensor, grads: torch.Tensor, B: int, T: int, hw: Tuple[int, int]) -> torch.Tensor:
    w = grads.mean(dim=(2, 3), keepdim=True)
    cam = torch.relu((w * feats).sum(dim=1, keepdim=True)).view(B, T, *feats.shape[-2:]).detach()
    out = []
    for t in range(T):
        c = F.interpolate(cam[:, t].unsqueeze(1), size=hw, mode="bilinear", align_corners=False).squeeze(1)
        c = c - c.amin(dim=(-2, -1), keepdim=True)
        out.append(c / (c.amax(dim=(-2, -1), keepdim=True) + 1e-6))
    return torch.stack(out, dim=1)[0]


def gradcam(sd: Dict[str, torch.Tensor], frames: torch.Tensor, mean: np.ndarray, std: np.ndarray,
            band: Iterable[int], reduction: str = "mean", frame_indices: Iterable[int] = ()):
    """-> (heatmaps (T,H,W), {frame: heatmap (H,W)}, feats.grad of the full target)."""
    sd = {k: v.clone() for k, v in sd.items()}
    pred, feats = forward_with_features(sd, frames)
    B, T = pred.shape[:2]
    db = pred * torch.from_numpy(std) + torch.from_numpy(mean)
    power = torch.pow(10.0, db / 10.0)
    band_power = power.index_select(-1, torch.as_tensor(list(band), dtype=torch.long)).sum(-1)
    target = band_power.mean() if reduction == "mean" else band_power.sum()
    frames_l = list(frame_indices)
    g = torch.autograd.grad(target, feats, retain_graph=bool(frames_l))[0]
    hw = tuple(frames.shape[-2:])
    maps = cam_from_grads(feats.detach(), g, B, T, hw)
    per = {}
    for i, t in enumerate(frames_l):
        gt = torch.autograd.grad(band_power[:, t].mean(), feats, retain_graph=i < len(frames_l) - 1)[0]
        per[t] = cam_from_grads(feats.detach(), gt, B, T, hw)[t]
    return maps, per, g
