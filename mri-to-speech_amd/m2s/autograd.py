"""Autograd over libm2s: the Grad-CAM path of the acoustic model.

The reference's scripts/mri_gradcam_formant.py (compute_gradcam, :203-279) does, on the loaded plug-in:

* ``model.train()`` with ``model.rnn.dropout`` kept in eval (:221-225), so the backbone's BatchNorms use
  the batch statistics of the clip's frames and update their running statistics;
* ``feats = model.cnn.backbone(x.repeat(1, 3, 1, 1))[-1]``, made a gradient leaf (:153-160);
* ``pooled = feats.mean((2, 3))`` -> ``model.rnn`` -> ``model.head`` (:162-165), the mel band power, and
  ``backward()`` to read ``feats.grad`` (:238-248).

Here those pieces are HIP kernels (csrc/cam.hip, csrc/cam.cpp) behind ``torch.ops.m2s.*``:

* ``CamEngine.backbone`` - train-mode backbone forward (``cam_backbone``): raw fp32 convs, two-pass
  batch statistics, (x - mean) * gamma / sqrt(var + eps) + beta, SiLU / residual;
* ``BiLSTMFunction`` - BiLSTM forward with saved gates / cells / hidden states and the backward through
  time, including the weight gradients nn.LSTM would accumulate (``bilstm_train_*``);
* ``LinearFunction`` - the head (``linear_*``), ``GapFunction`` - GlobalAvgPool (``gap_*``).

No CPU path: CPU tensors raise.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Tuple

import torch

from . import _native as N
from . import ops as _ops


def _need_hip(t: torch.Tensor, what: str):
    if t.device.type != "cuda":
        raise N.M2SError(f"{what}: m2s runs on MI355X (HIP) tensors only; got a {t.device} tensor")


class CamEngine:
    """Backbone weights packed for the train-mode forward (BatchNorm gamma / beta unfolded)."""

    def __init__(self, state_dict: Dict, device: torch.device):
        from .runtime import _device
        self.device = _device(device)
        L = N.lib()
        self.ops = _ops.load()
        N.check(L.m2s_device_check(self.device.index))
        sd = {k: v for k, v in state_dict.items() if k.startswith("cnn.backbone.")}
        arr, keep = N.tensor_array(sd)
        h = C.c_void_p()
        N.check(L.m2s_cam_create(arr, len(arr), self.device.index, C.byref(h)))
        del keep
        self._h = h
        self._destroy = L.m2s_cam_destroy
        self.layers = _ops.cam_bn_layers()
        n = L.m2s_cam_bn_layers(h)
        if n != len(self.layers) or any(L.m2s_cam_bn_channels(h, i) != c for i, (_, c, _) in enumerate(self.layers)):
            raise N.M2SError("libm2s BatchNorm layer table does not match the timm block table")

    def __del__(self):
        h, destroy = getattr(self, "_h", None), getattr(self, "_destroy", None)
        if h is not None and h.value and destroy is not None:
            destroy(h)
            self._h = None

    @property
    def handle(self) -> int:
        """The m2s_cam* as the int torch.ops.m2s.cam_backbone takes."""
        return int(self._h.value)

    def backbone(self, frames: torch.Tensor) -> Tuple[List[torch.Tensor], torch.Tensor]:
        """frames (N,H,W) -> ([5 feature maps (N,C,OH,OW)], BN batch stats [mean C | var C] per layer)."""
        _need_hip(frames, "cam backbone")
        out = self.ops.cam_backbone(self.handle, frames.to(torch.float32).contiguous())
        return list(out[:5]), out[5]

    def update_running_stats(self, buffers: Dict[str, torch.Tensor], stats: torch.Tensor, n: int, h: int, w: int,
                             momenta: Dict[str, float]):
        """What torch's BatchNorm does in train mode after normalising with the batch statistics:
        running_mean += m (mean - running_mean), running_var likewise with the unbiased variance
        (count / (count - 1)), num_batches_tracked += 1 (momentum None: cumulative average)."""
        off = 0
        with torch.no_grad():
            for name, c, red in self.layers:
                mean, var = stats[off:off + c], stats[off + c:off + 2 * c]
                off += 2 * c
                oh, ow = h, w
                r = 1
                while r < red:
                    oh, ow, r = (oh + 1) // 2, (ow + 1) // 2, r * 2
                cnt = n * oh * ow
                rm, rv = buffers.get(name + ".running_mean"), buffers.get(name + ".running_var")
                if name not in momenta or rm is None or rv is None:
                    continue  # track_running_stats=False: torch's BatchNorm keeps no running statistics
                nbt = buffers.get(name + ".num_batches_tracked")
                if nbt is not None:
                    nbt.add_(1)
                m = momenta[name]
                if m is None:
                    m = 1.0 / float(nbt.item()) if nbt is not None else 0.0
                unbiased = var * (cnt / max(cnt - 1, 1))
                rm.mul_(1.0 - m).add_(mean.to(rm.device), alpha=m)
                rv.mul_(1.0 - m).add_(unbiased.to(rv.device), alpha=m)


class BiLSTMFunction(torch.autograd.Function):
    """nn.LSTM(bidirectional, batch_first) with the sum merge (mri_acoustic_model.py:67-71)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, w_ih_r, w_hh_r, b_ih_r, b_hh_r):
        w = [t.detach().to(torch.float32).contiguous() for t in (w_ih, w_hh, b_ih, b_hh, w_ih_r, w_hh_r, b_ih_r, b_hh_r)]
        xc = x.detach().to(torch.float32).contiguous()
        y, gates, cells, hid = _ops.load().bilstm_train_forward(xc, w)
        ctx.save_for_backward(xc, gates, cells, hid, *w)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, gates, cells, hid, *w = ctx.saved_tensors
        dx, g = _ops.load().bilstm_train_backward(dy.to(torch.float32).contiguous(), xc, w, gates, cells, hid)
        need = ctx.needs_input_grad
        dx = dx if need[0] else None
        # b_ih and b_hh enter the gates as one sum: both receive the same gradient (nn.LSTM)
        grads = [g[0], g[1], g[2], g[2], g[3], g[4], g[5], g[5]]
        return (dx, *[gr if need[i + 1] else None for i, gr in enumerate(grads)])


def bilstm(x: torch.Tensor, lstm: torch.nn.LSTM) -> torch.Tensor:
    _need_hip(x, "BiLSTM")
    p = [getattr(lstm, f"{n}_l0{s}") for s in ("", "_reverse") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    return BiLSTMFunction.apply(x, *p)


class LinearFunction(torch.autograd.Function):
    """nn.Linear: y = x W^T + b (mri_acoustic_model.py:103,135)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        xc, wc = x.detach().to(torch.float32).contiguous(), weight.detach().to(torch.float32).contiguous()
        ctx.save_for_backward(xc, wc)
        ctx.has_bias = bias is not None
        return _ops.load().linear_forward(xc, wc, None if bias is None else bias.detach().to(torch.float32))

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        dx, dw, db = _ops.load().linear_backward(dy.to(torch.float32).contiguous(), xc, wc)
        need = ctx.needs_input_grad
        return (dx if need[0] else None, dw if need[1] else None, db if (need[2] and ctx.has_bias) else None)


def linear(x: torch.Tensor, weight: torch.Tensor, bias) -> torch.Tensor:
    _need_hip(x, "Linear")
    return LinearFunction.apply(x, weight, bias)


class GapFunction(torch.autograd.Function):
    """GlobalAvgPool: mean over (H, W) of (N,C,H,W) (mri_acoustic_model.py:15-18)."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return _ops.load().gap_forward(x.detach().to(torch.float32).contiguous())

    @staticmethod
    def backward(ctx, dy):
        return _ops.load().gap_backward(dy.to(torch.float32).contiguous(), *ctx.hw)


def gap(x: torch.Tensor) -> torch.Tensor:
    _need_hip(x, "GlobalAvgPool")
    return GapFunction.apply(x)
