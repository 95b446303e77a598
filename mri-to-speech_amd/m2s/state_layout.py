"""State-dict layouts of the two plug-in modules (key -> shape), reference names.

* Acoustic model (``build_acoustic_model`` -> OTNLikeCNNBiLSTM, mri_acoustic_model.py:74-136):
  ``cnn.backbone.*`` (timm EfficientNetFeatures key names), ``rnn.lstm.*`` (nn.LSTM),
  ``head.*`` (nn.Linear).  The trainer saves ``model.state_dict()`` under
  ``model_state_dict`` (train_mri_acoustic_model.py:511-520).
* Generator (models.py:88-109), weight-normed form as saved by train.py:199-203
  (``{'generator': state_dict}``): ``weight_g``/``weight_v`` everywhere except ``conv_pre``.
"""
from __future__ import annotations

from collections import OrderedDict

from .config import EFFNET_STEM, effnet_blocks


def _bn(s, q, c):
    for n in ("weight", "bias", "running_mean", "running_var"):
        s[f"{q}.{n}"] = (c,)
    s[f"{q}.num_batches_tracked"] = ()


def effnet_state_shapes(prefix: str = "cnn.backbone."):
    s = OrderedDict()
    s[prefix + "conv_stem.weight"] = (EFFNET_STEM, 3, 3, 3)
    _bn(s, prefix + "bn1", EFFNET_STEM)
    for b in effnet_blocks():
        q = f"{prefix}blocks.{b['stage']}.{b['idx']}."
        k, ci, co, m = b["k"], b["cin"], b["cout"], b["mid"]
        if b["type"] == "cn":
            s[q + "conv.weight"] = (co, ci, k, k)
            _bn(s, q + "bn1", co)
        elif b["type"] == "er":
            s[q + "conv_exp.weight"] = (m, ci, k, k)
            _bn(s, q + "bn1", m)
            s[q + "conv_pwl.weight"] = (co, m, 1, 1)
            _bn(s, q + "bn2", co)
        else:
            rd = b["rd"]
            s[q + "conv_pw.weight"] = (m, ci, 1, 1)
            _bn(s, q + "bn1", m)
            s[q + "conv_dw.weight"] = (m, 1, k, k)
            _bn(s, q + "bn2", m)
            s[q + "se.conv_reduce.weight"] = (rd, m, 1, 1)
            s[q + "se.conv_reduce.bias"] = (rd,)
            s[q + "se.conv_expand.weight"] = (m, rd, 1, 1)
            s[q + "se.conv_expand.bias"] = (m,)
            s[q + "conv_pwl.weight"] = (co, m, 1, 1)
            _bn(s, q + "bn3", co)
    return s


def acoustic_state_shapes(n_mels: int = 64, rnn_hidden: int = 640, in_dim: int = 208):
    s = effnet_state_shapes()
    H = rnn_hidden
    for sfx in ("", "_reverse"):
        s[f"rnn.lstm.weight_ih_l0{sfx}"] = (4 * H, in_dim)
        s[f"rnn.lstm.weight_hh_l0{sfx}"] = (4 * H, H)
        s[f"rnn.lstm.bias_ih_l0{sfx}"] = (4 * H,)
        s[f"rnn.lstm.bias_hh_l0{sfx}"] = (4 * H,)
    s["head.weight"] = (n_mels, H)
    s["head.bias"] = (n_mels,)
    return s


def generator_state_shapes(h):
    s = OrderedDict()
    c0 = h["upsample_initial_channel"]
    s["conv_pre.weight"] = (c0, h["num_mels"], 7)
    s["conv_pre.bias"] = (c0,)
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        ci, co = c0 // 2 ** i, c0 // 2 ** (i + 1)
        s[f"ups.{i}.bias"] = (co,)
        s[f"ups.{i}.weight_g"] = (ci, 1, 1)
        s[f"ups.{i}.weight_v"] = (ci, co, k)
    nk = len(h["resblock_kernel_sizes"])
    groups = ("convs1", "convs2") if h["resblock"] == "1" else ("convs",)
    for i in range(len(h["upsample_rates"])):
        ch = c0 // 2 ** (i + 1)
        for j, (k, d) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            p = f"resblocks.{i * nk + j}"
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
