"""Mel files -> 16-bit wav with the HiFi-GAN generator on MI355X; drop-in for inference_e2e.py.

Same command line (--input_mels_dir --output_dir --checkpoint_file), same config lookup
(``config.json`` next to the checkpoint, inference_e2e.py:69-75), same loading (strict
``load_state_dict(ckpt['generator'])``), same outputs (``{name}_generated_e2e.wav``, int16 PCM
of ``audio * MAX_WAV_VALUE`` at ``h.sampling_rate`` via scipy, inference_e2e.py:47-57).

One deliberate fix: the reference calls ``generator.remove_weight_norm()``,
which raises on the never-normed ``conv_pre`` (models.py:94,139) and stops the script; here the
weight norm is removed best-effort per module, as run_mri_video_inference.py:99-115 does.  The
generator runs in libm2s (``M2S_DTYPE`` / ``--dtype`` selects fp32 or bf16).
"""
from __future__ import absolute_import, division, print_function, unicode_literals

import argparse
import glob
import json
import os
import sys

import numpy as np
import torch
from scipy.io.wavfile import write

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from env import AttrDict  # noqa: E402
from models import Generator  # noqa: E402

MAX_WAV_VALUE = 32768.0  # meldataset.py:14
h = None
device = None


def load_checkpoint(filepath, device):
    assert os.path.isfile(filepath)
    print("Loading '{}'".format(filepath))
    checkpoint_dict = torch.load(filepath, map_location="cpu", weights_only=True)
    print("Complete.")
    return checkpoint_dict


def scan_checkpoint(cp_dir, prefix):
    cp_list = glob.glob(os.path.join(cp_dir, prefix + "*"))
    if len(cp_list) == 0:
        return ""
    return sorted(cp_list)[-1]


def remove_weight_norm_best_effort(generator):
    from torch.nn.utils import remove_weight_norm
    for module in list(generator.ups) + [generator.conv_post]:
        try:
            remove_weight_norm(module)
        except (ValueError, AttributeError):
            pass
    for res in generator.resblocks:
        try:
            res.remove_weight_norm()
        except (ValueError, AttributeError):
            pass


def inference(a):
    generator = Generator(h).to(device)
    state_dict_g = load_checkpoint(a.checkpoint_file, device)
    generator.load_state_dict(state_dict_g["generator"])
    if getattr(a, "dtype", None):
        generator.m2s_dtype = a.dtype
    filelist = sorted(os.listdir(a.input_mels_dir))
    os.makedirs(a.output_dir, exist_ok=True)
    generator.eval()
    remove_weight_norm_best_effort(generator)
    outputs = []
    with torch.no_grad():
        for filname in filelist:
            x = np.load(os.path.join(a.input_mels_dir, filname), allow_pickle=False)
            x = torch.FloatTensor(x).to(device)
            y_g_hat = generator(x)
            audio = y_g_hat.squeeze()
            audio = audio * MAX_WAV_VALUE
            audio = audio.cpu().numpy().astype("int16")
            output_file = os.path.join(a.output_dir, os.path.splitext(filname)[0] + "_generated_e2e.wav")
            write(output_file, h.sampling_rate, audio)
            print(output_file)
            outputs.append(output_file)
    return outputs


def main(argv=None):
    print("Initializing Inference Process..")
    parser = argparse.ArgumentParser()
    parser.add_argument("--input_mels_dir", default="test_mel_files")
    parser.add_argument("--output_dir", default="generated_files_from_mel")
    parser.add_argument("--checkpoint_file", required=True)
    parser.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None, help="m2s compute dtype")
    a = parser.parse_args(argv)
    config_file = os.path.join(os.path.split(a.checkpoint_file)[0], "config.json")
    with open(config_file) as f:
        data = f.read()
    global h, device
    h = AttrDict(json.loads(data))
    torch.manual_seed(h.seed)
    if not torch.cuda.is_available():
        raise RuntimeError("m2s needs an MI355X (HIP) device; no CPU fallback")
    torch.cuda.manual_seed(h.seed)
    device = torch.device("cuda")
    return inference(a)


if __name__ == "__main__":
    main()
