"""Oracle: BiLSTM sum-merge, Linear head and the mel glue, torch-CPU fp32.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* ``bilstm_summerge`` restates mri2speech_code/mri_acoustic_model.py:50-72:
  ``nn.LSTM(in, H, 1 layer, batch_first, bidirectional)``; PyTorch gate order i,f,g,o;
  c' = f*c + i*g, h' = o*tanh(c'); h0 = c0 = 0; output chunk -> y_fwd + y_bwd;
  Dropout is identity in eval.  Written as an explicit loop (``bilstm_summerge_loop``)
  and as the fused torch op (``bilstm_summerge``, used for CPU timing); both are pinned
  against tests/golden/acoustic.npz produced by the reference module itself.
* ``head`` restates mri_acoustic_model.py:103,135 (``nn.Linear(640, n_mels)``).
* ``preprocess_frame`` restates scripts/run_mri_video_inference.py:34-54 for grey
  frames already at the target size (resize not exercised).  ``bgr_to_grey`` restates the
  cv2.cvtColor(COLOR_BGR2GRAY) call at :36 as OpenCV's published 8-bit fixed-point formula
  (Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14); cv2 is not installed, so that step is parity
  unpinned.
* ``denormalize_mel`` / ``mel_db_to_log`` restate run_mri_video_inference.py:160-163 and
  the inline glue at :227-233 (10**(x/10) -> clamp(min=1e-5) -> ln).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


def lstm_params(sd: Dict[str, torch.Tensor], prefix: str = "rnn.lstm."):
    """(w_ih, w_hh, b_ih, b_hh) per direction, PyTorch nn.LSTM key names."""
    out = []
    for sfx in ("", "_reverse"):
        out.append(tuple(sd[f"{prefix}{n}_l0{sfx}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")))
    return out


def bilstm_summerge_loop(sd: Dict[str, torch.Tensor], x: torch.Tensor, prefix: str = "rnn.lstm.") -> torch.Tensor:
    """Explicit-loop restatement. x: (B,T,C) fp32 -> (B,T,H)."""
    B, T, _ = x.shape
    outs = []
    for d, (w_ih, w_hh, b_ih, b_hh) in enumerate(lstm_params(sd, prefix)):
        H = w_hh.shape[1]
        h = x.new_zeros(B, H)
        c = x.new_zeros(B, H)
        pre = x @ w_ih.t() + b_ih + b_hh  # (B,T,4H)
        ys = [None] * T
        steps = range(T) if d == 0 else range(T - 1, -1, -1)
        for t in steps:
            g = pre[:, t] + h @ w_hh.t()
            i, f, gg, o = g.chunk(4, dim=1)
            i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
            c = f * c + i * gg
            h = o * torch.tanh(c)
            ys[t] = h
        outs.append(torch.stack(ys, dim=1))
    return outs[0] + outs[1]


def bilstm_summerge(sd: Dict[str, torch.Tensor], x: torch.Tensor, prefix: str = "rnn.lstm.") -> torch.Tensor:
    """Same computation through torch's fused CPU LSTM (the op the reference calls)."""
    (wf, hf, bf1, bf2), (wr, hr, br1, br2) = lstm_params(sd, prefix)
    H = hf.shape[1]
    lstm = torch.nn.LSTM(wf.shape[1], H, 1, batch_first=True, bidirectional=True)
    with torch.no_grad():
        for name, t in zip(("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0",
                            "weight_ih_l0_reverse", "weight_hh_l0_reverse", "bias_ih_l0_reverse",
                            "bias_hh_l0_reverse"), (wf, hf, bf1, bf2, wr, hr, br1, br2)):
            getattr(lstm, name).copy_(t)
        y, _ = lstm(x)
    yf, yb = y.chunk(2, dim=-1)
    return yf + yb


def head(sd: Dict[str, torch.Tensor], y: torch.Tensor, prefix: str = "head.") -> torch.Tensor:
    return torch.nn.functional.linear(y, sd[prefix + "weight"], sd[prefix + "bias"])


def preprocess_frame(gray: np.ndarray) -> np.ndarray:
    """run_mri_video_inference.py:34-54 for a 2-D frame already at 256x256."""
    g = gray.astype(np.float32)
    mean = g.mean()
    std = g.std()
    g = (g - mean) / std if std > 0 else g - mean
    lo, hi = g.min(), g.max()
    return (g - lo) / (hi - lo) if hi > lo else np.zeros_like(g)


def bgr_to_grey(frame: np.ndarray) -> np.ndarray:
    """cv2.COLOR_BGR2GRAY for uint8 (H,W,3) BGR (run_mri_video_inference.py:36)."""
    f = frame.astype(np.int64)
    return ((1868 * f[..., 0] + 9617 * f[..., 1] + 4899 * f[..., 2] + (1 << 13)) >> 14).astype(np.uint8)


def denormalize_mel(mel_norm: torch.Tensor, mean: np.ndarray, std: np.ndarray) -> torch.Tensor:
    return mel_norm * torch.from_numpy(std) + torch.from_numpy(mean)


def mel_db_to_log(mel_db: torch.Tensor) -> torch.Tensor:
    mel_power = torch.pow(10.0, mel_db / 10.0)
    return torch.log(torch.clamp(mel_power, min=1e-5))
