"""Drop-in ``models.Generator`` (HiFi-GAN generator with the reference's causal MRF) on libm2s.

Same import (``from models import Generator``, scripts/run_mri_video_inference.py:8-19), constructor
(``Generator(h)`` reading h.resblock / upsample_* / resblock_* / num_mels / upsample_initial_channel,
models.py:88-109), state-dict keys (``weight_g``/``weight_v`` on ups, resblocks and conv_post; plain
``conv_pre``) and weight-norm API (``remove_weight_norm`` per ResBlock; ``ups`` / ``conv_post``
accept ``torch.nn.utils.remove_weight_norm``) as the reference models.py:11-140, so
``load_state_dict(ckpt['generator'])`` (strict) and the loader's best-effort removal
(run_mri_video_inference.py:96-115) behave identically.

``forward`` (eval, HIP tensors) runs the whole generator in libm2s (conv_pre -> 4 x [LeakyReLU ->
polyphase ConvTranspose1d -> 3 causal ResBlocks averaged] -> LeakyReLU(0.01) -> conv_post -> tanh).
The torch sub-modules only hold parameters.  Discriminators and losses (training only) are not part
of this path.  ``forward`` dispatches to ``torch.ops.m2s.hifigan_forward``.  Compute dtype:
``M2S_DTYPE`` / ``generator.m2s_dtype``: "bf16x3" (default; split fp32 within the fp32 tolerances),
"fp32" (exact f32 MFMA), "bf16".  The packed engine is rebuilt after ``load_state_dict`` / ``.to()`` /
a dtype change or a versioned in-place parameter edit; ``generator.m2s_refresh()`` after
``p.data.copy_()`` edits.  Weight-norm removal
does not change the folded weights, so it needs no repack.
"""
from __future__ import annotations

import os
import sys
import warnings

import torch
import torch.nn as nn
from torch.nn import Conv1d, ConvTranspose1d

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

LRELU_SLOPE = 0.1

with warnings.catch_warnings():
    warnings.simplefilter("ignore")
    from torch.nn.utils import remove_weight_norm, weight_norm  # weight_g / weight_v key layout


def _init(m, std=0.01):  # utils.init_weights (utils.py:22-25)
    if isinstance(m, (Conv1d, ConvTranspose1d)):
        m.weight.data.normal_(0.0, std)


def _wn(m):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return weight_norm(m)


def get_padding(kernel_size, dilation=1):
    """utils.py:33-34 - full (k-1)*d padding; with output truncation it makes every MRF conv causal."""
    return int(kernel_size * dilation - dilation)


class ResBlock1(nn.Module):
    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3, 5)):
        super().__init__()
        self.h = h
        self.kernel_size, self.dilation = kernel_size, tuple(dilation)
        self.convs1 = nn.ModuleList([_wn(Conv1d(channels, channels, kernel_size, 1, dilation=d,
                                                padding=get_padding(kernel_size, d))) for d in dilation])
        self.convs2 = nn.ModuleList([_wn(Conv1d(channels, channels, kernel_size, 1, dilation=1,
                                                padding=get_padding(kernel_size, 1))) for _ in dilation])
        self.convs1.apply(_init)
        self.convs2.apply(_init)

    def forward(self, x):
        raise NotImplementedError("ResBlocks run fused inside Generator.forward (libm2s)")

    def remove_weight_norm(self):
        for layer in self.convs1:
            remove_weight_norm(layer)
        for layer in self.convs2:
            remove_weight_norm(layer)


class ResBlock2(nn.Module):
    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3)):
        super().__init__()
        self.h = h
        self.kernel_size, self.dilation = kernel_size, tuple(dilation)
        self.convs = nn.ModuleList([_wn(Conv1d(channels, channels, kernel_size, 1, dilation=d,
                                               padding=get_padding(kernel_size, d))) for d in dilation])
        self.convs.apply(_init)

    def forward(self, x):
        raise NotImplementedError("ResBlocks run fused inside Generator.forward (libm2s)")

    def remove_weight_norm(self):
        for layer in self.convs:
            remove_weight_norm(layer)


class Generator(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.h = h
        self.num_kernels = len(h.resblock_kernel_sizes)
        self.num_upsamples = len(h.upsample_rates)
        self.conv_pre = Conv1d(h.num_mels, h.upsample_initial_channel, 7, 1, padding=0)
        resblock = ResBlock1 if h.resblock == "1" else ResBlock2
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
            self.ups.append(_wn(ConvTranspose1d(h.upsample_initial_channel // (2 ** i),
                                                h.upsample_initial_channel // (2 ** (i + 1)), k, u,
                                                padding=(k - u) // 2)))
        self.resblocks = nn.ModuleList()
        ch = h.upsample_initial_channel
        for i in range(len(self.ups)):
            ch = h.upsample_initial_channel // (2 ** (i + 1))
            for k, d in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes):
                self.resblocks.append(resblock(h, ch, k, d))
        self.conv_post = _wn(Conv1d(ch, 1, 7, 1, padding=0))
        self.ups.apply(_init)
        self.conv_post.apply(_init)
        self.m2s_dtype = os.environ.get("M2S_DTYPE", "bf16x3")
        object.__setattr__(self, "_eng", None)
        object.__setattr__(self, "_eng_key", None)
        object.__setattr__(self, "_gen", 0)
        self.register_load_state_dict_post_hook(lambda mod, keys: mod.m2s_refresh())

    def m2s_refresh(self):
        """Repack the weights at the next forward (after in-place parameter edits)."""
        object.__setattr__(self, "_gen", self._gen + 1)

    def _apply(self, fn, *a, **k):  # .to() / .cuda() / .float() move or replace the parameters
        r = super()._apply(fn, *a, **k)
        self.m2s_refresh()
        return r

    def _config(self):
        h = self.h
        return {k: (h[k] if isinstance(h, dict) else getattr(h, k)) for k in
                ("resblock", "upsample_rates", "upsample_kernel_sizes", "upsample_initial_channel",
                 "resblock_kernel_sizes", "resblock_dilation_sizes", "num_mels")}

    def _engine(self, device):
        if self.training:
            raise NotImplementedError("m2s implements generator inference only; call .eval()")
        if device.type != "cuda":
            raise RuntimeError("m2s runs on MI355X (HIP) tensors only; move the generator and mel to 'cuda'")
        # in-place edits that bump a tensor's version or move its storage repack too (see the plug-in's
        # OTNLikeCNNBiLSTM._signature); `p.data.copy_()` edits still need m2s_refresh()
        key = (str(device), self.m2s_dtype, self._gen, tuple((t.data_ptr(), t._version) for t in self.parameters()),
               tuple((t.data_ptr(), t._version) for t in self.buffers()))
        if self._eng is None or self._eng_key != key:
            from m2s.runtime import VocoderEngine
            host = {k: v.detach().to("cpu") for k, v in self.state_dict().items()}
            object.__setattr__(self, "_eng", VocoderEngine(host, self._config(), dtype=self.m2s_dtype, device=device))
            object.__setattr__(self, "_eng_key", key)
        return self._eng

    def forward(self, x):
        """(B, num_mels, T) ln-mel -> (B, 1, T * prod(upsample_rates)) waveform in [-1, 1].
        An unbatched (num_mels, T) mel gives (1, T * hop), as torch's unbatched conv1d chain does
        for the reference module (inference_e2e.py:48-50 passes the stored (64, T) arrays as is)."""
        if torch.is_grad_enabled() and x.requires_grad:
            raise NotImplementedError("m2s generator has no autograd; run under torch.no_grad()")
        if x.dim() == 2:
            return self._engine(x.device).forward(x.unsqueeze(0), layout=0)[0]
        return self._engine(x.device).forward(x, layout=0)

    def remove_weight_norm(self):
        """Mirrors models.py:133-140, including its failure on the never-normed conv_pre."""
        print("Removing weight norm...")
        for layer in self.ups:
            remove_weight_norm(layer)
        for layer in self.resblocks:
            layer.remove_weight_norm()
        remove_weight_norm(self.conv_pre)
        remove_weight_norm(self.conv_post)
