"""Synthetic, seeded inputs and weights for the hot path (no checkpoints or datasets exist offline).

The recipe is numpy ``default_rng(seed)`` (stable across numpy versions), drawn key by
key in ``state_layout`` order, and scaled so activations stay O(1) through the whole
graph (random-init weights at the reference's std 0.01, utils.py:22-25, would make every
output ~0 and every tolerance meaningless).  Golden fixtures store only the seed.
"""
from __future__ import annotations

import math

import numpy as np

from .config import HIFIGAN_H
from .state_layout import acoustic_state_shapes, generator_state_shapes


def _fan_in(shape):
    return int(np.prod(shape[1:])) if len(shape) > 1 else 1


def synth_acoustic_state(seed: int = 0, n_mels: int = 64, rnn_hidden: int = 640):
    rng = np.random.default_rng(seed)
    out = {}
    for key, shape in acoustic_state_shapes(n_mels, rnn_hidden).items():
        if key.endswith("num_batches_tracked"):
            out[key] = np.array(0, dtype=np.int64)
            continue
        leaf = key.rsplit(".", 1)[-1]
        if key.startswith("rnn.lstm."):
            b = 1.0 / math.sqrt(rnn_hidden)
            a = rng.uniform(-b, b, size=shape)
        elif key.startswith("head."):
            a = rng.normal(0.0, 3.0 / math.sqrt(shape[-1]), size=shape) if leaf == "weight" else rng.normal(0, 0.1, shape)
        elif ".bn" in key:
            if leaf == "weight":
                a = rng.uniform(0.8, 1.2, size=shape)
            elif leaf == "bias":
                a = rng.normal(0.0, 0.1, size=shape)
            elif leaf == "running_mean":
                a = rng.normal(0.0, 0.1, size=shape)
            else:
                a = rng.uniform(0.5, 1.5, size=shape)
        elif leaf == "bias":
            a = rng.normal(0.0, 0.1, size=shape)
        else:
            fan = shape[1] * shape[2] * shape[3] if len(shape) == 4 else _fan_in(shape)
            gain = 0.6 if "conv_pwl" in key else math.sqrt(2.0)
            if "conv_dw" in key:
                fan = 9
            if "conv_stem" in key:
                fan = 9  # the three input channels are identical (grey repeat)
                gain = 1.0
            a = rng.normal(0.0, gain / math.sqrt(fan), size=shape)
        out[key] = a.astype(np.float32)
    return out


def synth_generator_state(seed: int = 0, h=None):
    h = h or HIFIGAN_H
    rng = np.random.default_rng(seed)
    out = {}
    rates = dict(enumerate(h["upsample_rates"]))
    for key, shape in generator_state_shapes(h).items():
        leaf = key.rsplit(".", 1)[-1]
        if leaf == "bias":
            a = rng.normal(0.0, 0.05, size=shape)
        elif leaf == "weight_v":
            a = rng.normal(0.0, 1.0, size=shape)
        elif leaf == "weight_g":
            if key.startswith("ups."):
                g = math.sqrt(rates[int(key.split(".")[1])] / 2.0) * 1.4
            elif key.startswith("conv_post"):
                g = 0.3
            else:
                g = 0.6
            a = rng.uniform(0.8, 1.2, size=shape) * g
        else:  # conv_pre.weight (plain Conv1d, models.py:94)
            a = rng.normal(0.0, 1.0 / math.sqrt(_fan_in(shape)), size=shape) * 0.5
        out[key] = a.astype(np.float32)
    return out


def synth_frames(n_clips: int, n_frames: int, hw=(256, 256), seed: int = 1234):
    """(n_clips, T, H, W) fp32 in [0,1], per-frame min-max normalised."""
    rng = np.random.default_rng(seed)
    x = rng.random((n_clips, n_frames) + tuple(hw), dtype=np.float32)
    lo = x.min(axis=(2, 3), keepdims=True)
    hi = x.max(axis=(2, 3), keepdims=True)
    return ((x - lo) / (hi - lo)).astype(np.float32)


def synth_scaler(n_mels: int = 64, seed: int = 7):
    rng = np.random.default_rng(seed)
    mean = rng.normal(-40.0, 10.0, size=n_mels).astype(np.float32)
    std = rng.uniform(5.0, 15.0, size=n_mels).astype(np.float32)
    return mean, std


def synth_mel_log(batch: int, n_mels: int, T: int, seed: int = 3):
    """ln-power mels in the range the glue produces (>= ln 1e-5)."""
    rng = np.random.default_rng(seed)
    m = rng.normal(-4.0, 2.0, size=(batch, n_mels, T)).astype(np.float32)
    return np.maximum(m, np.float32(math.log(1e-5)))
