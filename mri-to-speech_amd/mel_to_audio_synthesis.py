"""Mel .npy file(s) -> wav, figure and stats with the m2s HiFi-GAN generator
(drop-in for mel_to_audio_synthesis.py).

Contract kept from the reference (mel_to_audio_synthesis.py:138-333): the flags ``--input`` (one .npy
or a directory of them), ``--checkpoint_file``, ``--config``, ``--output_dir``, ``--max_files``; the
input conforming rules (first row of a batched array, mel bins truncated / zero-padded to
``h.num_mels``); per input ``{base}_from_mel.wav`` (16-bit PCM), ``{base}_input_mel.png`` and
``{base}_synthesis_stats.json`` (input_file, mel_shape, mel_range, audio_shape, audio_range,
duration_seconds, sampling_rate), with a trailing ``_mel`` dropped from ``base``; then
``mel_synthesis_results.html`` and ``overall_synthesis_stats.json`` over the run.  A file that fails is
reported and the run continues.

How it runs: all inputs are read and conformed first, equal-length mels share one generator call
(m2s/drivers.py), outputs are written afterwards.  ``--dtype`` / ``--batch`` are additive; there is no
CPU path.
"""
from __future__ import annotations

import argparse
import html
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


def find_inputs(path: Path, limit: int):
    """The .npy files named by ``--input``; None for an unusable argument."""
    if path.is_file() and path.suffix == ".npy":
        return [path]
    if path.is_dir():
        found = sorted(p for p in path.iterdir() if p.suffix.lower() == ".npy")
        if len(found) > limit:
            print(f"{len(found)} .npy files in {path}; taking the first {limit}")
        return found[:limit]
    return None


def stem_of(p: Path) -> str:
    s = p.stem
    return s[:-4] if s.endswith("_mel") else s


def file_stats(job, sr: int) -> dict:
    m, a = job.array, job.result
    return {"input_file": str(job.src), "mel_shape": [1, *m.shape],
            "mel_range": [float(m.min()), float(m.max())], "audio_shape": list(a.shape),
            "audio_range": [float(a.min()), float(a.max())], "duration_seconds": a.shape[0] / sr,
            "sampling_rate": sr}


def report_html(h, done) -> str:
    """One page: the run summary and, per synthesised file, its stats, player and input figure."""
    rows = []
    for i, (base, st) in enumerate(done, 1):
        b = html.escape(base)
        rows.append(
            f'<section class="file"><h2>{i}. {b}</h2>'
            f'<p class="stats">mel {st["mel_shape"]}, range {st["mel_range"][0]:.3f} .. {st["mel_range"][1]:.3f}; '
            f'audio {st["duration_seconds"]:.2f} s, range {st["audio_range"][0]:.3f} .. {st["audio_range"][1]:.3f}</p>'
            f'<audio controls src="{b}_from_mel.wav"></audio>'
            f'<img src="{b}_input_mel.png" alt="input mel {b}"></section>')
    return ("<!DOCTYPE html><html><head><meta charset='utf-8'><title>HiFi-GAN Mel-to-Audio Synthesis</title>"
            "<style>body{font-family:sans-serif;margin:20px}.file{border:1px solid #ccc;padding:12px;margin:12px 0}"
            "audio,img{width:100%}.stats{font-family:monospace;font-size:12px}</style></head><body>"
            f"<h1>HiFi-GAN Mel-to-Audio Synthesis</h1><p>{len(done)} file(s) synthesised; "
            f"{h.num_mels} mel bins, {h.sampling_rate} Hz.</p>" + "".join(rows) + "</body></html>\n")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="mel .npy -> wav with the HiFi-GAN generator on MI355X")
    p.add_argument("--input", required=True, help="Input .npy mel file or directory with .npy files")
    p.add_argument("--checkpoint_file", required=True, help="Generator checkpoint file")
    p.add_argument("--config", default="config_custom.json", help="HiFi-GAN config file")
    p.add_argument("--output_dir", default="mel_synthesis_result", help="Output directory")
    p.add_argument("--max_files", default=20, type=int, help="Maximum number of files to process (if directory)")
    p.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None,
                   help="m2s compute dtype (default: M2S_DTYPE or bf16x3)")
    p.add_argument("--batch", type=int, default=64, help="mels of equal length per generator call")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    h = AttrDict(json.loads(Path(args.config).read_text(encoding="utf-8")))
    out_dir = Path(args.output_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    inputs = find_inputs(Path(args.input), args.max_files)
    if not inputs:
        print(f"Nothing to synthesise from {args.input} (expects a .npy file or a directory holding some)")
        return None
    if not torch.cuda.is_available():
        raise RuntimeError("m2s needs an MI355X (HIP) device; there is no CPU path")
    device = torch.device("cuda")
    gen, n_wn = drivers.build_generator(h, args.checkpoint_file, device, args.dtype)
    print(f"generator ready on {device}; weight norm stripped from {n_wn} module(s)")

    sr = int(h.sampling_rate)
    jobs = [drivers.read_mel(drivers.Job(p, stem_of(p)), int(h.num_mels)) for p in inputs]
    drivers.vocode(gen, jobs, device, args.batch)

    done = []
    for job in jobs:
        for note in job.notes:
            print(f"[{job.stem}] {note}")
        if job.result is None:
            print(f"[{job.stem}] failed: {job.error}")
            continue
        drivers.write_wav_pcm16(out_dir / f"{job.stem}_from_mel.wav", job.result, sr)
        drivers.save_mel_png(job.array, f"Input Mel Spectrogram - {job.stem}", out_dir / f"{job.stem}_input_mel.png")
        st = file_stats(job, sr)
        drivers.write_json(out_dir / f"{job.stem}_synthesis_stats.json", st)
        done.append((job.stem, st))
        print(f"[{job.stem}] {st['duration_seconds']:.2f} s of audio")

    (out_dir / "mel_synthesis_results.html").write_text(report_html(h, done), encoding="utf-8")
    cfg = {k: h.get(k) for k in ("num_mels", "sampling_rate", "n_fft", "hop_size", "win_size")}
    drivers.write_json(out_dir / "overall_synthesis_stats.json",
                       {"total_files": len(jobs), "successful_syntheses": len(done), "model_config": cfg,
                        "individual_stats": [st for _, st in done]})
    print(f"{len(done)}/{len(jobs)} file(s) synthesised into {out_dir}")
    return [b for b, _ in done]


if __name__ == "__main__":
    main()
