"""Oracle: timm ``tf_efficientnetv2_b2`` (features_only) + global average pool, torch-CPU fp32.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference call site: mri2speech_code/mri_acoustic_model.py:20-48
  ``timm.create_model("tf_efficientnetv2_b2", pretrained=False, features_only=True,
  drop_rate=0, drop_path_rate=0)``; grey input repeated to 3 channels (:41-44);
  last feature map (:46); ``GlobalAvgPool`` = mean over (H, W) (:15-18, :47).

timm==1.0.21 (requirements.lab.txt:11) is a third-party dependency absent from this
image and from /root/reference.  Its published builder semantics are restated here:

* ``_gen_efficientnetv2_base`` arch_def
    cn_r1_k3_s1_e1_c16_skip | er_r2_k3_s2_e4_c32 | er_r2_k3_s2_e4_c48 |
    ir_r3_k3_s2_e4_c96_se0.25 | ir_r5_k3_s1_e6_c112_se0.25 | ir_r8_k3_s2_e6_c192_se0.25
  with channel_multiplier 1.1 (make_divisible(c*1.1, 8)) and depth_multiplier 1.2
  (ceil) for "b2"  ->  repeats (2,3,3,4,6,10), widths (16,32,56,104,120,208), stem 32.
* ``tf_`` variants: BatchNorm eps 1e-3, padding 'same' (TF SAME: static pad 1 for
  3x3/s1, dynamic asymmetric pad (0,1,0,1) for 3x3/s2 on even sizes = Conv2dSame).
* ConvBnAct: conv -> BN+SiLU (+ shortcut iff stride 1 and in == out).
* EdgeResidual: conv_exp kxk (stride) -> BN+SiLU -> conv_pwl 1x1 -> BN (+ shortcut).
* InvertedResidual: conv_pw 1x1 -> BN+SiLU -> conv_dw kxk (stride, depthwise) -> BN+SiLU
  -> SqueezeExcite(rd = round(mid * 0.25 / exp) , SiLU, sigmoid gate) -> conv_pwl 1x1 -> BN
  (+ shortcut).
* No conv_head in features_only mode; last feature = output of blocks.5 (N,208,H/32,W/32).

PARITY UNPINNED: no test in the reference and no timm install can pin these numerics;
checked structurally (state-dict key names / shapes, output shape (N,208,8,8)).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

BN_EPS = 1e-3

# (block_type, repeats, kernel, stride, exp_ratio, out_ch, se_ratio)
STAGES: List[Tuple[str, int, int, int, int, int, float]] = [
    ("cn", 2, 3, 1, 1, 16, 0.0),
    ("er", 3, 3, 2, 4, 32, 0.0),
    ("er", 3, 3, 2, 4, 56, 0.0),
    ("ir", 4, 3, 2, 4, 104, 0.25),
    ("ir", 6, 3, 1, 6, 120, 0.25),
    ("ir", 10, 3, 2, 6, 208, 0.25),
]
STEM_CH = 32
OUT_CH = 208


def make_divisible(v: float, divisor: int = 8) -> int:
    """timm.layers.make_divisible with round_limit=0 (channel rounding of the builder)."""
    return max(divisor, int(v + divisor / 2) // divisor * divisor)


def block_table() -> List[dict]:
    """Expanded per-block description: one dict per timm block, in state-dict order."""
    blocks = []
    cin = STEM_CH
    for s, (bt, reps, k, stride, exp, cout, se) in enumerate(STAGES):
        for b in range(reps):
            st = stride if b == 0 else 1
            d = dict(stage=s, idx=b, type=bt, k=k, stride=st, cin=cin, cout=cout,
                     skip=(st == 1 and cin == cout))
            if bt in ("er", "ir"):
                d["mid"] = make_divisible(cin * exp)
            if bt == "ir" and se > 0:
                d["rd"] = int(round(d["mid"] * (se / exp)))
            blocks.append(d)
            cin = cout
    return blocks


def _same_pad(x: torch.Tensor, k: int, s: int) -> torch.Tensor:
    """TF 'SAME' padding (timm pad_same): total = max((ceil(i/s)-1)*s + k - i, 0), left = total//2."""
    ih, iw = x.shape[-2:]
    ph = max((math.ceil(ih / s) - 1) * s + k - ih, 0)
    pw = max((math.ceil(iw / s) - 1) * s + k - iw, 0)
    return F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])


def _conv(x, w, k, s, groups=1):
    if k == 1:
        return F.conv2d(x, w, None, s, 0, 1, groups)
    if s == 1:  # static symmetric padding ((s-1) + (k-1)) // 2
        return F.conv2d(x, w, None, 1, (k - 1) // 2, 1, groups)
    return F.conv2d(_same_pad(x, k, s), w, None, s, 0, 1, groups)


BN_MOMENTUM = 0.1  # torch.nn.BatchNorm2d default, kept by timm's BatchNormAct2d


def _bn(x, sd, p, act, train=False):
    """timm BatchNormAct2d.  eval: running statistics.  train (model.train(), as the reference's
    Grad-CAM runs it, scripts/mri_gradcam_formant.py:223): the batch's statistics, and the running
    statistics in ``sd`` updated in place the way torch does (momentum 0.1, unbiased variance)."""
    y = F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                     sd[p + ".bias"], train, BN_MOMENTUM if train else 0.0, BN_EPS)
    return F.silu(y) if act else y


def effnet_features(sd: Dict[str, torch.Tensor], x: torch.Tensor, prefix: str = "cnn.backbone.",
                    taps: list | None = None, train: bool = False) -> torch.Tensor:
    """(N,1,H,W) or (N,H,W) or (N,3,H,W) fp32 -> last feature map (N,208,H/32,W/32).

    ``taps``, if given, receives the output of the stem and of every block (29 tensors).
    ``train``: BatchNorm in training mode (see ``_bn``); ``sd``'s running statistics are updated."""
    if x.dim() == 3:
        x = x.unsqueeze(1)
    if x.size(1) == 1:  # mri_acoustic_model.py:43-44
        x = x.repeat(1, 3, 1, 1)
    p = prefix
    x = _conv(x, sd[p + "conv_stem.weight"], 3, 2)
    x = _bn(x, sd, p + "bn1", True, train)
    if taps is not None:
        taps.append(x)
    for b in block_table():
        q = f"{p}blocks.{b['stage']}.{b['idx']}."
        sc = x
        if b["type"] == "cn":
            x = _conv(x, sd[q + "conv.weight"], b["k"], b["stride"])
            x = _bn(x, sd, q + "bn1", True, train)
        elif b["type"] == "er":
            x = _conv(x, sd[q + "conv_exp.weight"], b["k"], b["stride"])
            x = _bn(x, sd, q + "bn1", True, train)
            x = _conv(x, sd[q + "conv_pwl.weight"], 1, 1)
            x = _bn(x, sd, q + "bn2", False, train)
        else:
            x = _conv(x, sd[q + "conv_pw.weight"], 1, 1)
            x = _bn(x, sd, q + "bn1", True, train)
            x = _conv(x, sd[q + "conv_dw.weight"], b["k"], b["stride"], groups=b["mid"])
            x = _bn(x, sd, q + "bn2", True, train)
            s = x.mean((2, 3), keepdim=True)
            s = F.conv2d(s, sd[q + "se.conv_reduce.weight"], sd[q + "se.conv_reduce.bias"])
            s = F.silu(s)
            s = F.conv2d(s, sd[q + "se.conv_expand.weight"], sd[q + "se.conv_expand.bias"])
            x = x * torch.sigmoid(s)
            x = _conv(x, sd[q + "conv_pwl.weight"], 1, 1)
            x = _bn(x, sd, q + "bn3", False, train)
        if b["skip"]:
            x = x + sc
        if taps is not None:
            taps.append(x)
    return x


def effnet_gap(sd: Dict[str, torch.Tensor], x: torch.Tensor, prefix: str = "cnn.backbone.") -> torch.Tensor:
    """EffNetV2B2Backbone.forward (mri_acoustic_model.py:39-48): -> (N, 208)."""
    return torch.mean(effnet_features(sd, x, prefix), dim=(2, 3))


def effnet_state_shapes(prefix: str = "cnn.backbone.") -> Dict[str, Tuple[int, ...]]:
    """State-dict keys/shapes timm's EfficientNetFeatures would expose for this model."""
    shapes: Dict[str, Tuple[int, ...]] = {}

    def bn(q, c):
        for n in ("weight", "bias", "running_mean", "running_var"):
            shapes[q + "." + n] = (c,)
        shapes[q + ".num_batches_tracked"] = ()

    p = prefix
    shapes[p + "conv_stem.weight"] = (STEM_CH, 3, 3, 3)
    bn(p + "bn1", STEM_CH)
    for b in block_table():
        q = f"{p}blocks.{b['stage']}.{b['idx']}."
        k, ci, co = b["k"], b["cin"], b["cout"]
        if b["type"] == "cn":
            shapes[q + "conv.weight"] = (co, ci, k, k)
            bn(q + "bn1", co)
        elif b["type"] == "er":
            m = b["mid"]
            shapes[q + "conv_exp.weight"] = (m, ci, k, k)
            bn(q + "bn1", m)
            shapes[q + "conv_pwl.weight"] = (co, m, 1, 1)
            bn(q + "bn2", co)
        else:
            m, rd = b["mid"], b["rd"]
            shapes[q + "conv_pw.weight"] = (m, ci, 1, 1)
            bn(q + "bn1", m)
            shapes[q + "conv_dw.weight"] = (m, 1, k, k)
            bn(q + "bn2", m)
            shapes[q + "se.conv_reduce.weight"] = (rd, m, 1, 1)
            shapes[q + "se.conv_reduce.bias"] = (rd,)
            shapes[q + "se.conv_expand.weight"] = (m, rd, 1, 1)
            shapes[q + "se.conv_expand.bias"] = (m,)
            shapes[q + "conv_pwl.weight"] = (co, m, 1, 1)
            bn(q + "bn3", co)
    return shapes


def effnet_flops_per_frame(h: int = 256, w: int = 256) -> Dict[str, float]:
    """Algorithmic FLOPs (2*MAC) per frame, 3-channel stem as in the reference graph."""
    dense = dw = se = 0.0
    oh, ow = math.ceil(h / 2), math.ceil(w / 2)
    dense += 2 * oh * ow * STEM_CH * 3 * 9
    for b in block_table():
        k, s = b["k"], b["stride"]
        nh, nw = math.ceil(oh / s), math.ceil(ow / s)
        if b["type"] == "cn":
            dense += 2 * nh * nw * b["cout"] * b["cin"] * k * k
        elif b["type"] == "er":
            dense += 2 * nh * nw * b["mid"] * b["cin"] * k * k
            dense += 2 * nh * nw * b["cout"] * b["mid"]
        else:
            dense += 2 * oh * ow * b["mid"] * b["cin"]
            dw += 2 * nh * nw * b["mid"] * k * k
            se += 2 * 2 * b["mid"] * b["rd"]
            dense += 2 * nh * nw * b["cout"] * b["mid"]
        oh, ow = nh, nw
    return {"dense": dense, "depthwise": dw, "se": se, "total": dense + dw + se}
