"""Shapes of the hot path, as the reference configures it.

* ``HIFIGAN_H``: the Generator hyper-parameters of config_custom.json:2,10-44,46,49,51
  (only the keys ``Generator`` and the inference script read: models.py:89-109,
  run_mri_video_inference.py:247).
* ``EFFNET_*``: timm ``tf_efficientnetv2_b2`` features_only (mri_acoustic_model.py:28-36),
  see DESIGN.md for the builder rules these follow.
* ``ACOUSTIC_DEFAULTS``: ``build_acoustic_model`` defaults (mri_acoustic_model.py:139-156).
"""
from __future__ import annotations

HIFIGAN_H = {
    "resblock": "1",
    "upsample_rates": [10, 7, 3, 2],
    "upsample_kernel_sizes": [20, 15, 7, 4],
    "upsample_initial_channel": 512,
    "resblock_kernel_sizes": [3, 7, 11],
    "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
    "num_mels": 64,
    "hop_size": 420,
    "sampling_rate": 11413,
}

ACOUSTIC_DEFAULTS = dict(n_mels=64, cnn_pretrained=False, rnn_hidden=640, dropout=0.5,
                         use_checkpoint=False, ckpt_segments=2, use_reentrant=False)

FRAME_HW = (256, 256)

# Frames per CNN pass of the acoustic engine: the one default the plug-in, the CLI, the drivers and
# bench.py share (bench.py's 64 x 30 step is one pass; DESIGN.md §2.2 measured 256-frame passes 25 %
# slower: 53.7 vs 43.0 ms per step).  The engine sizes its workspace for min(frames, CNN_CHUNK).
CNN_CHUNK = 1920

# (block_type, repeats, kernel, stride, exp_ratio, out_ch, se_ratio) per timm stage
EFFNET_STAGES = [
    ("cn", 2, 3, 1, 1, 16, 0.0),
    ("er", 3, 3, 2, 4, 32, 0.0),
    ("er", 3, 3, 2, 4, 56, 0.0),
    ("ir", 4, 3, 2, 4, 104, 0.25),
    ("ir", 6, 3, 1, 6, 120, 0.25),
    ("ir", 10, 3, 2, 6, 208, 0.25),
]
EFFNET_STEM = 32
EFFNET_OUT = 208
BN_EPS = 1e-3


def make_divisible(v: float, divisor: int = 8) -> int:
    return max(divisor, int(v + divisor / 2) // divisor * divisor)


def effnet_blocks():
    """One dict per timm block (stage, idx, type, k, stride, cin, cout, mid, rd, skip)."""
    out, cin = [], EFFNET_STEM
    for s, (bt, reps, k, stride, exp, cout, se) in enumerate(EFFNET_STAGES):
        for b in range(reps):
            st = stride if b == 0 else 1
            d = dict(stage=s, idx=b, type=bt, k=k, stride=st, cin=cin, cout=cout,
                     skip=(st == 1 and cin == cout), mid=0, rd=0)
            if bt != "cn":
                d["mid"] = make_divisible(cin * exp)
            if bt == "ir":
                d["rd"] = int(round(d["mid"] * se / exp))
            out.append(d)
            cin = cout
    return out
