"""torch.ops.m2s.* - the PyTorch-ROCm custom ops of libm2s (csrc/torch_ops.cpp) and their fake kernels.

``load()`` loads ``libm2s_torch.so`` (built in-tree next to ``libm2s.so``, which it links) with
``torch.ops.load_library``; there is no fallback: a missing library raises ``M2SError``.  The ops
take the packed model as an opaque int handle (``AcousticEngine.handle`` / ``VocoderEngine.handle``)
and run on the current HIP stream.  The fake (meta) kernels below give every op its output shapes
for FakeTensor tracing / torch.compile / ``torch.library.opcheck``.

Reference interfaces: mri2speech_code/mri_acoustic_model.py:15-18,39-48,67-72,116-136 (acoustic model),
models.py:113-131 (Generator.forward), scripts/run_mri_video_inference.py:34-54,160-163,222-242.
"""
from __future__ import annotations

import os

import torch

from ._native import M2SError

TORCH_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libm2s_torch.so")
OPS = ("acoustic_forward", "effnet_forward", "effnet_features", "bilstm_summerge", "mel_glue", "hifigan_forward",
       "pipeline_forward", "preprocess_frames", "cam_backbone", "bilstm_train_forward", "bilstm_train_backward",
       "linear_forward", "linear_backward", "gap_forward", "gap_backward")

# timm tf_efficientnetv2_b2 (features_only): stride and output channels of the stem (index 0) and of
# the 29 blocks that follow (effnet_features' n_blocks = how many of them ran)
_FEAT_STRIDE = [2] + [1, 1] + [2, 1, 1] + [2, 1, 1] + [2, 1, 1, 1] + [1] * 6 + [2] + [1] * 9
_FEAT_CH = [32] + [16] * 2 + [32] * 3 + [56] * 3 + [104] * 4 + [120] * 6 + [208] * 10

def cam_bn_layers():
    """(state-dict prefix, channels, input reduction) of every BatchNorm in cam_backbone's statistics
    order: conv_stem's bn1, then per block bn1 / bn2 / bn3 (timm key names).  The reduction is the
    layer's spatial stride w.r.t. the frame (its map is ceil-halved that many times)."""
    from .config import EFFNET_STEM, effnet_blocks
    out = [("cnn.backbone.bn1", EFFNET_STEM, 2)]
    red = 2
    for b in effnet_blocks():
        q = f"cnn.backbone.blocks.{b['stage']}.{b['idx']}."
        r_in, red = red, red * b["stride"]
        layers = {"cn": [(b["cout"], red)], "er": [(b["mid"], red), (b["cout"], red)],
                  "ir": [(b["mid"], r_in), (b["mid"], red), (b["cout"], red)]}[b["type"]]
        out += [(f"{q}bn{i + 1}", c, r) for i, (c, r) in enumerate(layers)]
    return out


# floats of cam_backbone's BatchNorm statistics: [mean C | var C] per layer
CAM_BN_STATS = 2 * sum(c for _, c, _ in cam_bn_layers())

_loaded = False


def load():
    """Load libm2s_torch.so once (registers torch.ops.m2s.*) and the fake kernels."""
    global _loaded
    if _loaded:
        return torch.ops.m2s
    if not os.path.exists(TORCH_LIB_PATH):
        raise M2SError(f"libm2s_torch.so not found at {TORCH_LIB_PATH}; build it with `make -C mri-to-speech_amd/csrc` "
                       "(there is no CPU fallback)")
    torch.ops.load_library(TORCH_LIB_PATH)
    _register_fakes()
    _loaded = True
    return torch.ops.m2s


def feature_shape(n: int, h: int, w: int, n_blocks: int):
    """(N, C, OH, OW) of effnet_features after `n_blocks` blocks (TF-SAME: out = ceil(in / stride))."""
    oh, ow = h, w
    for s in _FEAT_STRIDE[: n_blocks + 1]:
        oh, ow = (oh + s - 1) // s, (ow + s - 1) // s
    return n, _FEAT_CH[n_blocks], oh, ow


def _register_fakes():
    f = torch.library.register_fake

    @f("m2s::acoustic_forward")
    def _acoustic(handle, frames, n_mels):
        return frames.new_empty((frames.shape[0], frames.shape[1], n_mels), dtype=torch.float32)

    @f("m2s::effnet_forward")
    def _effnet(handle, frames):
        return frames.new_empty((frames.shape[0], 208), dtype=torch.float32)

    @f("m2s::effnet_features")
    def _features(handle, frames, n_blocks):
        return frames.new_empty(feature_shape(frames.shape[0], frames.shape[1], frames.shape[2], n_blocks),
                                dtype=torch.float32)

    @f("m2s::bilstm_summerge")
    def _bilstm(handle, feats, hidden, n_mels):
        b, t = feats.shape[0], feats.shape[1]
        return (feats.new_empty((b, t, hidden), dtype=torch.float32),
                feats.new_empty((b, t, n_mels), dtype=torch.float32))

    @f("m2s::mel_glue")
    def _glue(mel_norm, mean, std):
        return (torch.empty_like(mel_norm, dtype=torch.float32), torch.empty_like(mel_norm, dtype=torch.float32))

    @f("m2s::hifigan_forward")
    def _hifigan(handle, mel, layout, hop):
        t = mel.shape[2] if layout == 0 else mel.shape[1]
        return mel.new_empty((mel.shape[0], 1, t * hop), dtype=torch.float32)

    @f("m2s::pipeline_forward")
    def _pipeline(acoustic, vocoder, frames, mean, std, n_mels, hop):
        b, t = frames.shape[0], frames.shape[1]
        mel = [frames.new_empty((b, t, n_mels), dtype=torch.float32) for _ in range(3)]
        return mel[0], mel[1], mel[2], frames.new_empty((b, t * hop), dtype=torch.float32)

    @f("m2s::preprocess_frames")
    def _pre(frames):
        return frames.new_empty(tuple(frames.shape[:3]), dtype=torch.float32)

    @f("m2s::cam_backbone")
    def _cam(handle, frames):
        n, h, w = frames.shape
        maps = [frames.new_empty(feature_shape(n, h, w, k), dtype=torch.float32) for k in (2, 5, 8, 18, 28)]
        return (*maps, frames.new_empty((CAM_BN_STATS,), dtype=torch.float32))

    @f("m2s::bilstm_train_forward")
    def _lstm_fwd(x, weights):
        b, t, hd = x.shape[0], x.shape[1], weights[1].shape[1]
        return (x.new_empty((b, t, hd)), x.new_empty((2, b, t, 4 * hd)), x.new_empty((2, b, t, hd)),
                x.new_empty((2, b, t, hd)))

    @f("m2s::bilstm_train_backward")
    def _lstm_bwd(dy, x, weights, gates, cells, hid):
        return torch.empty_like(x), [torch.empty_like(weights[i]) for i in (0, 1, 2, 4, 5, 6)]

    @f("m2s::linear_forward")
    def _lin(x, weight, bias):
        return x.new_empty((*x.shape[:-1], weight.shape[0]))

    @f("m2s::linear_backward")
    def _lin_bwd(dy, x, weight):
        return torch.empty_like(x), torch.empty_like(weight), weight.new_empty((weight.shape[0],))

    @f("m2s::gap_forward")
    def _gap(x):
        return x.new_empty((x.shape[0], x.shape[1]))

    @f("m2s::gap_backward")
    def _gap_bwd(dy, h, w):
        return dy.new_empty((dy.shape[0], dy.shape[1], h, w))
