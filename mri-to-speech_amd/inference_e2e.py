"""ln-mel files -> int16 wav files with the m2s HiFi-GAN generator (drop-in for inference_e2e.py).

Contract kept from the reference (inference_e2e.py:60-90): the flags ``--input_mels_dir``,
``--output_dir``, ``--checkpoint_file``; ``config.json`` read from the checkpoint's directory;
``Generator(h)`` with ``ckpt['generator']`` loaded strictly; one ``{name}_generated_e2e.wav`` per
input file at ``h.sampling_rate``, holding ``(audio * MAX_WAV_VALUE).astype(int16)`` (scipy writer).

How it runs: every file in the directory is read up front, files of equal length are synthesised
together in one generator call (m2s/drivers.py), and the wavs are written afterwards.  Files that
cannot be read or have the wrong number of bins are reported and skipped.  The weight norm is removed
best-effort: the reference's ``generator.remove_weight_norm()`` raises on the never-normed conv_pre
(models.py:94,139), which SURVEY.md §8f-3 lists as the thing to fix.  ``--dtype`` and ``--batch`` are
additive.  There is no CPU path.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import torch

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from env import AttrDict  # noqa: E402
from m2s import drivers  # noqa: E402

MAX_WAV_VALUE = drivers.MAX_WAV_VALUE


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="ln-mel .npy files -> int16 wav (HiFi-GAN generator on MI355X)")
    p.add_argument("--input_mels_dir", default="test_mel_files")
    p.add_argument("--output_dir", default="generated_files_from_mel")
    p.add_argument("--checkpoint_file", required=True)
    p.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None,
                   help="m2s compute dtype (default: M2S_DTYPE or bf16x3)")
    p.add_argument("--batch", type=int, default=64, help="files of equal length per generator call")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    ckpt = Path(args.checkpoint_file)
    h = AttrDict(json.loads((ckpt.parent / "config.json").read_text(encoding="utf-8")))
    if not torch.cuda.is_available():
        raise RuntimeError("m2s needs an MI355X (HIP) device; there is no CPU path")
    torch.manual_seed(h.seed)
    device = torch.device("cuda")
    gen, _ = drivers.build_generator(h, ckpt, device, args.dtype)

    src = Path(args.input_mels_dir)
    jobs = [drivers.read_mel(drivers.Job(src / name, Path(name).stem), int(h.num_mels), conform=False)
            for name in sorted(os.listdir(src))]
    drivers.vocode(gen, jobs, device, args.batch)

    out_dir = Path(args.output_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    from scipy.io.wavfile import write

    written = []
    for job in jobs:
        if job.result is None:
            print(f"[skip] {job.src}: {job.error}")
            continue
        path = out_dir / f"{job.stem}_generated_e2e.wav"
        write(str(path), int(h.sampling_rate), drivers.int16_truncated(job.result))
        print(path)
        written.append(str(path))
    return written


if __name__ == "__main__":
    main()
