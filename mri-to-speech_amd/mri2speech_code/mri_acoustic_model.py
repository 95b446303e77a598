"""Drop-in ``mri_acoustic_model`` plug-in backed by libm2s (MI355X / gfx950).

Same import path and factory as the reference plug-in (mri2speech_code/mri_acoustic_model.py:139-156):
``--mri-code-dir`` -> ``from mri_acoustic_model import build_acoustic_model`` ->
``build_acoustic_model(n_mels, cnn_pretrained, rnn_hidden, dropout, use_checkpoint, ckpt_segments,
use_reentrant)``.  The returned module has the reference's tree (``cnn.backbone``, ``cnn.gap``,
``rnn.lstm``, ``rnn.dropout``, ``head``) and state-dict keys (timm ``EfficientNetFeatures`` names for
the backbone), so ``load_state_dict(checkpoint['model_state_dict'], strict=False)`` behaves the same.

Inference (eval, HIP tensors): ``forward`` runs the whole CNN -> BiLSTM -> head graph in libm2s
through ``torch.ops.m2s.acoustic_forward``; ``model.cnn.backbone(x)`` returns timm's five feature maps
(strides 2..32: 16/32/56/120/208 channels, ``torch.ops.m2s.effnet_features``).

Grad-CAM (scripts/mri_gradcam_formant.py:203-279, m2s/autograd.py): after ``model.train()`` the
backbone normalises with the batch statistics of the frames it is given and updates the BatchNorm
running statistics (timm / torch train-mode semantics, ``torch.ops.m2s.cam_backbone``); ``model.rnn``,
``model.head`` and ``model.cnn.gap`` are autograd functions over HIP kernels (BiLSTM backward through
time with the weight gradients nn.LSTM would produce, Linear, GAP), so ``feats.grad`` of a
leaf feature map is filled by ``backward()``.  The backbone itself has no backward: a train-mode
``model(x)`` with gradients enabled (training the CNN) raises.

Compute dtype of the inference engine: ``M2S_DTYPE`` env var or ``model.m2s_dtype``: "bf16x3"
(default; split fp32, meets the fp32 tolerances of the parity tests), "fp32" (exact f32 MFMA
products), "bf16" (fast, lower precision), "fp8".  The Grad-CAM path is exact fp32.
The packed engines are rebuilt after ``load_state_dict`` / ``.to()``, a dtype / chunk change, or an
in-place parameter edit that bumps the tensor version (``p.copy_()``, ``p.mul_()``, ``p.data = t``);
call ``model.m2s_refresh()`` after edits through ``p.data.copy_()``, which torch does not version.
No CPU fallback: CPU tensors raise.
"""
from __future__ import annotations

import os
import sys
from typing import Optional

import torch
import torch.nn as nn

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from m2s.config import BN_EPS, CNN_CHUNK, EFFNET_STEM, effnet_blocks  # noqa: E402


def _bn(c):
    return nn.BatchNorm2d(c, eps=BN_EPS)


class _ConvBnAct(nn.Module):  # timm ConvBnAct ('cn')
    def __init__(self, b):
        super().__init__()
        self.conv = nn.Conv2d(b["cin"], b["cout"], b["k"], b["stride"], bias=False)
        self.bn1 = _bn(b["cout"])


class _EdgeResidual(nn.Module):  # timm EdgeResidual ('er')
    def __init__(self, b):
        super().__init__()
        self.conv_exp = nn.Conv2d(b["cin"], b["mid"], b["k"], b["stride"], bias=False)
        self.bn1 = _bn(b["mid"])
        self.conv_pwl = nn.Conv2d(b["mid"], b["cout"], 1, bias=False)
        self.bn2 = _bn(b["cout"])


class _SqueezeExcite(nn.Module):
    def __init__(self, c, rd):
        super().__init__()
        self.conv_reduce = nn.Conv2d(c, rd, 1, bias=True)
        self.conv_expand = nn.Conv2d(rd, c, 1, bias=True)


class _InvertedResidual(nn.Module):  # timm InvertedResidual ('ir', SE)
    def __init__(self, b):
        super().__init__()
        m = b["mid"]
        self.conv_pw = nn.Conv2d(b["cin"], m, 1, bias=False)
        self.bn1 = _bn(m)
        self.conv_dw = nn.Conv2d(m, m, b["k"], b["stride"], groups=m, bias=False)
        self.bn2 = _bn(m)
        self.se = _SqueezeExcite(m, b["rd"])
        self.conv_pwl = nn.Conv2d(m, b["cout"], 1, bias=False)
        self.bn3 = _bn(b["cout"])


class _FeatureInfo:
    def channels(self):
        return [16, 32, 56, 120, 208]

    def reduction(self):
        return [2, 4, 8, 16, 32]


# n_blocks (effnet_features) after which each of timm's five features is taken: the end of
# blocks.0 / .1 / .2 / .4 / .5 (features_only out_indices of tf_efficientnetv2_b2)
_FEATURE_TAPS = (2, 5, 8, 18, 28)


class _EffNetV2B2Features(nn.Module):
    """Parameter container with timm ``tf_efficientnetv2_b2`` features_only key names."""

    def __init__(self):
        super().__init__()
        self.conv_stem = nn.Conv2d(3, EFFNET_STEM, 3, 2, bias=False)
        self.bn1 = _bn(EFFNET_STEM)
        stages = {}
        for b in effnet_blocks():
            cls = {"cn": _ConvBnAct, "er": _EdgeResidual, "ir": _InvertedResidual}[b["type"]]
            stages.setdefault(b["stage"], []).append(cls(b))
        self.blocks = nn.Sequential(*[nn.Sequential(*stages[s]) for s in sorted(stages)])
        self.feature_info = _FeatureInfo()

    def forward(self, x):
        """(N,3,H,W) repeated-grey or (N,1,H,W) frames -> [5 feature maps (N,C,H/s,W/s)] (eval only;
        mri_gradcam_formant.py:153-158 passes x.repeat(1, 3, 1, 1) and keeps the last map)."""
        if x.dim() != 4 or x.size(1) not in (1, 3):
            raise ValueError(f"expected (N,1,H,W) or (N,3,H,W) frames, got {tuple(x.shape)}")
        if x.size(1) == 3:
            if not (torch.equal(x[:, 0], x[:, 1]) and torch.equal(x[:, 0], x[:, 2])):
                raise ValueError("m2s folds the grey->RGB repeat into conv_stem; the 3 channels must be equal")
        g = x[:, 0]
        root = self._root()
        if root.training:  # timm train mode: BatchNorm on this batch's statistics (Grad-CAM, :223)
            cam = root._cam_engine(x.device)
            maps, stats = cam.backbone(g)
            bns = {n: m for n, m in self.named_modules() if isinstance(m, nn.BatchNorm2d)}
            bufs = {f"cnn.backbone.{n}.{b}": t for n, m in bns.items() for b, t in m.named_buffers()}
            momenta = {f"cnn.backbone.{n}": m.momentum for n, m in bns.items() if m.track_running_stats}
            if momenta:
                cam.update_running_stats(bufs, stats, g.shape[0], g.shape[1], g.shape[2], momenta)
            return maps
        eng = root._engine(x.device)
        return [eng.probe(g, n) for n in _FEATURE_TAPS]


class GlobalAvgPool(nn.Module):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(N,C,H,W) -> (N,C) mean over (H, W) (mri_acoustic_model.py:15-18), HIP forward + backward."""
        from m2s import autograd
        return autograd.gap(x)


class EffNetV2B2Backbone(nn.Module):
    def __init__(self, pretrained: bool = False):
        super().__init__()
        if pretrained:
            raise ValueError("pretrained timm weights cannot be fetched offline; load a checkpoint instead")
        self.backbone = _EffNetV2B2Features()
        self.out_channels = self.backbone.feature_info.channels()[-1]
        self.gap = GlobalAvgPool()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(N,1,H,W) or (N,H,W) grey frames -> (N, 208) (mri_acoustic_model.py:39-48)."""
        if x.dim() == 4:
            if x.size(1) != 1:
                raise ValueError("m2s expects grey (1-channel) frames")
            x = x[:, 0]
        if self._root().training:  # batch-statistics BatchNorm, then GAP (autograd from the pooled map on)
            return self.gap(self.backbone(x[:, None])[-1])
        return self._root()._engine(x.device).effnet(x)


class BiLSTMSumMerge(nn.Module):
    def __init__(self, in_dim: int, hidden_size: int = 640, dropout: float = 0.0):
        super().__init__()
        self.lstm = nn.LSTM(input_size=in_dim, hidden_size=hidden_size, num_layers=1, batch_first=True,
                            bidirectional=True, dropout=0.0)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B,T,C) -> (B,T,H) forward + backward hidden states, then dropout (mri_acoustic_model.py:67-72).

        With autograd live (training, or gradients enabled for x or the LSTM weights) it runs the
        saved-activation kernels and their backward through time; otherwise the inference engine."""
        root = self._root()
        grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.lstm.parameters()))
        if root.training or grad:
            from m2s import autograd
            y = autograd.bilstm(x, self.lstm)
        else:
            y = root._engine(x.device).bilstm(x)[0]
        return self.dropout(y)


class _Head(nn.Linear):
    """nn.Linear(rnn_hidden, n_mels) (mri_acoustic_model.py:103) on HIP kernels, forward and backward."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from m2s import autograd
        return autograd.linear(x, self.weight, self.bias)


class OTNLikeCNNBiLSTM(nn.Module):
    def __init__(self, n_mels: int = 64, cnn_pretrained: bool = False, rnn_hidden: int = 640,
                 dropout: float = 0.5, use_checkpoint: bool = False, ckpt_segments: int = 2,
                 use_reentrant: bool = False):
        super().__init__()
        self.n_mels = n_mels
        self.use_checkpoint = use_checkpoint
        self.ckpt_segments = ckpt_segments
        self.use_reentrant = use_reentrant
        self.cnn = EffNetV2B2Backbone(pretrained=cnn_pretrained)
        self.rnn = BiLSTMSumMerge(in_dim=self.cnn.out_channels, hidden_size=rnn_hidden, dropout=dropout)
        self.head = _Head(rnn_hidden, n_mels)
        self.m2s_dtype = os.environ.get("M2S_DTYPE", "bf16x3")
        self.m2s_chunk = int(os.environ.get("M2S_CHUNK", str(CNN_CHUNK)))
        root = lambda: self  # noqa: E731  (children reach the engine without registering a cycle)
        for m in (self.cnn, self.rnn, self.cnn.backbone):
            object.__setattr__(m, "_root", root)
        object.__setattr__(self, "_eng", None)
        object.__setattr__(self, "_eng_key", None)
        object.__setattr__(self, "_cam", None)
        object.__setattr__(self, "_cam_key", None)
        object.__setattr__(self, "_gen", 0)
        self.register_load_state_dict_post_hook(lambda mod, keys: mod.m2s_refresh())

    def m2s_refresh(self):
        """Repack the weights at the next forward (after in-place parameter edits)."""
        object.__setattr__(self, "_gen", self._gen + 1)

    def _apply(self, fn, *a, **k):  # .to() / .cuda() / .float() move or replace the parameters
        r = super()._apply(fn, *a, **k)
        self.m2s_refresh()
        return r

    def _signature(self, device):
        # (data_ptr, _version) of every parameter and buffer: in-place edits (p.copy_() under no_grad,
        # EMA updates, vector_to_parameters) bump _version and `p.data = ...` moves data_ptr, so the
        # packed engine is rebuilt without an explicit m2s_refresh(); edits through `p.data.copy_()`
        # bypass the version counter and still need m2s_refresh().
        params = tuple((t.data_ptr(), t._version) for t in self.parameters())
        bufs = tuple((t.data_ptr(), t._version) for t in self.buffers())
        return (str(device), self.m2s_dtype, self.m2s_chunk, self._gen, params, bufs)

    def _engine(self, device: torch.device):
        if self.training:
            raise NotImplementedError("the fused m2s inference engine runs in eval(); in train() the Grad-CAM "
                                      "path (cnn.backbone / rnn / head) is available, CNN training is not")
        if device.type != "cuda":
            raise RuntimeError("m2s runs on MI355X (HIP) tensors only; move the model and frames to 'cuda'")
        key = self._signature(device)
        if self._eng is None or self._eng_key != key:
            from m2s.runtime import AcousticEngine
            sd = {k: v.detach().to("cpu") for k, v in self.state_dict().items()}
            object.__setattr__(self, "_eng", AcousticEngine(sd, n_mels=self.n_mels,
                                                            rnn_hidden=self.rnn.lstm.hidden_size,
                                                            dtype=self.m2s_dtype, device=device,
                                                            chunk=self.m2s_chunk))
            object.__setattr__(self, "_eng_key", key)
        return self._eng

    def _cam_engine(self, device: torch.device):
        """Train-mode backbone weights (conv weights + BN gamma / beta; running statistics are not
        packed, so their updates do not repack it)."""
        if device.type != "cuda":
            raise RuntimeError("m2s runs on MI355X (HIP) tensors only; move the model and frames to 'cuda'")
        key = (str(device), self._gen, tuple((p.data_ptr(), p._version) for p in self.cnn.backbone.parameters()))
        if self._cam is None or self._cam_key != key:
            from m2s.autograd import CamEngine
            sd = {k: v.detach().to("cpu") for k, v in self.state_dict().items() if k.startswith("cnn.backbone.")}
            object.__setattr__(self, "_cam", CamEngine(sd, device))
            object.__setattr__(self, "_cam_key", key)
        return self._cam

    def _check_grad(self, x):
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            if x.requires_grad:
                raise NotImplementedError("m2s forward has no autograd; run under torch.no_grad()")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B,T,1,H,W) or (B,T,H,W) -> (B,T,n_mels)  (mri_acoustic_model.py:116-136).

        eval: one fused libm2s call.  train (no_grad only): the train-mode backbone (batch-statistics
        BatchNorm) -> GAP -> BiLSTM -> head, as the reference's training branch computes it (:118-130)."""
        if self.training:
            if torch.is_grad_enabled():
                raise NotImplementedError("m2s has no backward through the CNN backbone: train-mode forward runs "
                                          "under torch.no_grad() only (Grad-CAM uses cnn.backbone / rnn / head)")
            if x.device.type != "cuda":
                raise RuntimeError("m2s runs on MI355X (HIP) tensors only; move the model and frames to 'cuda'")
            B, T = x.shape[0], x.shape[1]
            g = x.reshape(B * T, 1, *x.shape[-2:])
            feats = self.cnn.gap(self.cnn.backbone(g)[-1]).view(B, T, -1)
            return self.head(self.rnn(feats))
        self._check_grad(x)
        return self._engine(x.device).forward(x)


def build_acoustic_model(n_mels: int = 64, cnn_pretrained: bool = False, rnn_hidden: int = 640,
                         dropout: float = 0.5, use_checkpoint: bool = False, ckpt_segments: int = 2,
                         use_reentrant: bool = False) -> nn.Module:
    return OTNLikeCNNBiLSTM(n_mels=n_mels, cnn_pretrained=cnn_pretrained, rnn_hidden=rnn_hidden,
                            dropout=dropout, use_checkpoint=use_checkpoint, ckpt_segments=ckpt_segments,
                            use_reentrant=use_reentrant)
