"""Oracle: HiFi-GAN Generator with the reference's causal MRF resblocks, torch-CPU fp32.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates models.py:11-131 functionally over a reference-format state dict:

* ``get_padding(k, d) = k*d - d`` (utils.py:33-34) is applied on BOTH sides, then the
  conv output is truncated to the input length (models.py:43-47, :76-80) - i.e. a
  causal dilated conv: y[t] = sum_j w[j] x[t - (k-1)d + j d].
* ResBlock1 (models.py:11-55): 3 x [lrelu(0.1) -> c1(dil d) -> lrelu(0.1) -> c2(dil 1) -> +x].
* ResBlock2 (models.py:58-85): 2 x [lrelu(0.1) -> c(dil d) -> +x].
* Generator.forward (models.py:113-131): pad right 6 -> conv_pre (k7, no weight norm)
  -> 4 x [lrelu(0.1) -> ConvTranspose1d(k, u, pad (k-u)//2) -> sum_j resblock_j / 3]
  -> leaky_relu (default slope **0.01**) -> pad right 6 -> conv_post (k7) -> tanh.
* weight norm: w = g * v / ||v|| (norm over every dim except 0; for ConvTranspose1d
  dim 0 is in_channels), as ``torch._weight_norm(v, g, 0)`` (models.py:94-101;
  run_mri_video_inference.py:99-115 folds it once at load).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.1


def get_padding(kernel_size: int, dilation: int = 1) -> int:
    return int(kernel_size * dilation - dilation)


def fold_weight(sd: Dict[str, torch.Tensor], p: str) -> torch.Tensor:
    if p + ".weight" in sd:
        return sd[p + ".weight"]
    return torch._weight_norm(sd[p + ".weight_v"], sd[p + ".weight_g"], 0)


def _causal_conv(x, w, b, k, d):
    pad = get_padding(k, d)
    y = F.conv1d(x, w, b, 1, pad, d)
    return y[:, :, : x.shape[2]]


def resblock1(sd, p, x, k, dil):
    for i, d in enumerate(dil):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = _causal_conv(xt, fold_weight(sd, f"{p}.convs1.{i}"), sd[f"{p}.convs1.{i}.bias"], k, d)
        xt = F.leaky_relu(xt, LRELU_SLOPE)
        xt = _causal_conv(xt, fold_weight(sd, f"{p}.convs2.{i}"), sd[f"{p}.convs2.{i}.bias"], k, 1)
        x = xt + x
    return x


def resblock2(sd, p, x, k, dil):
    for i, d in enumerate(dil):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = _causal_conv(xt, fold_weight(sd, f"{p}.convs.{i}"), sd[f"{p}.convs.{i}.bias"], k, d)
        x = xt + x
    return x


def generator(sd: Dict[str, torch.Tensor], h, mel: torch.Tensor) -> torch.Tensor:
    """mel (B, num_mels, T) fp32 -> wav (B, 1, T * prod(upsample_rates))."""
    x = F.pad(mel, (0, 6), "constant")
    x = F.conv1d(x, fold_weight(sd, "conv_pre"), sd["conv_pre.bias"])
    nk = len(h["resblock_kernel_sizes"])
    rb = resblock1 if h["resblock"] == "1" else resblock2
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        x = F.leaky_relu(x, LRELU_SLOPE)
        x = F.conv_transpose1d(x, fold_weight(sd, f"ups.{i}"), sd[f"ups.{i}.bias"], u, (k - u) // 2)
        xs = None
        for j, (rk, rd) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            y = rb(sd, f"resblocks.{i * nk + j}", x, rk, rd)
            xs = y if xs is None else xs + y
        x = xs / nk
    x = F.leaky_relu(x)
    x = F.pad(x, (0, 6), "constant")
    x = F.conv1d(x, fold_weight(sd, "conv_post"), sd["conv_post.bias"])
    return torch.tanh(x)


def generator_state_shapes(h) -> Dict[str, tuple]:
    """Key -> shape of the reference Generator's state dict (weight-normed form)."""
    s: Dict[str, tuple] = {}
    c0 = h["upsample_initial_channel"]
    s["conv_pre.weight"] = (c0, h["num_mels"], 7)
    s["conv_pre.bias"] = (c0,)
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        ci, co = c0 // 2 ** i, c0 // 2 ** (i + 1)
        s[f"ups.{i}.bias"] = (co,)
        s[f"ups.{i}.weight_g"] = (ci, 1, 1)
        s[f"ups.{i}.weight_v"] = (ci, co, k)
    nk = len(h["resblock_kernel_sizes"])
    for i in range(len(h["upsample_rates"])):
        ch = c0 // 2 ** (i + 1)
        for j, (k, d) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            p = f"resblocks.{i * nk + j}"
            groups = ("convs1", "convs2") if h["resblock"] == "1" else ("convs",)
            for g in groups:
                for n in range(len(d)):
                    s[f"{p}.{g}.{n}.bias"] = (ch,)
                    s[f"{p}.{g}.{n}.weight_g"] = (ch, 1, 1)
                    s[f"{p}.{g}.{n}.weight_v"] = (ch, ch, k)
    ch = c0 // 2 ** len(h["upsample_rates"])
    s["conv_post.bias"] = (1,)
    s["conv_post.weight_g"] = (1, 1, 1)
    s["conv_post.weight_v"] = (1, ch, 7)
    return s


def generator_flops_per_frame(h) -> Dict[str, float]:
    """Algorithmic FLOPs (2*MAC) per mel frame (causal outputs only)."""
    c0 = h["upsample_initial_channel"]
    f = {"conv_pre": 2.0 * c0 * h["num_mels"] * 7, "ups": 0.0, "mrf": 0.0}
    L = 1
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        ci, co = c0 // 2 ** i, c0 // 2 ** (i + 1)
        f["ups"] += 2.0 * ci * co * k * L  # each input sample meets k taps
        L *= u
        per = 2 if h["resblock"] == "1" else 1
        for rk, rd in zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"]):
            f["mrf"] += per * len(rd) * 2.0 * co * co * rk * L
    f["conv_post"] = 2.0 * (c0 // 2 ** len(h["upsample_rates"])) * 7 * L
    f["total"] = sum(f.values())
    return f
