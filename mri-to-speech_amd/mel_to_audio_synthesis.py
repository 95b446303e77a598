"""Stand-alone mel -> audio synthesis on MI355X; drop-in for mel_to_audio_synthesis.py.

Same command line (--input file-or-dir --checkpoint_file --config --output_dir --max_files) and
the same per-file behaviour as mel_to_audio_synthesis.py:47-136: a (n_mels, T) or (B, n_mels, T)
array (first sample used), mel bins truncated / zero-padded to ``h.num_mels``, the generator run,
``{base}_from_mel.wav`` (soundfile, or 16-bit PCM through ``wave`` when soundfile is absent),
``{base}_input_mel.png`` (matplotlib), ``{base}_synthesis_stats.json``; then
``mel_synthesis_results.html`` and ``overall_synthesis_stats.json``.  Weight norm is removed
best-effort (ups, resblocks, conv_post; conv_pre has none), as the reference does (:193-211).
The generator runs in libm2s; there is no CPU fallback.
"""
import argparse
import gc
import json
import os
import sys
import wave

import numpy as np
import torch

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from env import AttrDict  # noqa: E402
from models import Generator  # noqa: E402

try:
    import soundfile as sf
except ImportError:  # pragma: no cover - absent in this image
    sf = None


def load_checkpoint(filepath, device):
    assert os.path.isfile(filepath)
    print(f"Loading '{filepath}'...")
    checkpoint_dict = torch.load(filepath, map_location="cpu", weights_only=True)
    print("Complete.")
    return checkpoint_dict


def safe_remove_weight_norm(module):
    try:
        from torch.nn.utils import remove_weight_norm
        remove_weight_norm(module)
        return True
    except (ValueError, AttributeError):
        return False


def load_mel_spectrogram(mel_path):
    if not os.path.exists(mel_path):
        raise FileNotFoundError(f"Mel file not found: {mel_path}")
    mel_np = np.load(mel_path, allow_pickle=False)
    print(f"Loaded mel spectrogram from: {mel_path}")
    print(f"Mel shape: {mel_np.shape}")
    print(f"Mel range: {mel_np.min():.3f} to {mel_np.max():.3f}")
    return mel_np


def write_wav(path, audio, sr):
    if sf is not None:
        sf.write(path, audio, sr)
        return
    pcm = np.clip(np.rint(np.asarray(audio, np.float64) * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sr))
        w.writeframes(pcm.tobytes())


def save_mel_png(mel, title, path):
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:  # pragma: no cover
        return
    plt.figure(figsize=(12, 4))
    plt.imshow(mel, aspect="auto", origin="lower")
    plt.colorbar()
    plt.title(title)
    plt.xlabel("Time")
    plt.ylabel("Mel Bins")
    plt.tight_layout()
    plt.savefig(path, dpi=150)
    plt.close()


def process_mel_file(mel_path, h, generator, device, output_dir):
    basename = os.path.splitext(os.path.basename(mel_path))[0]
    if basename.endswith("_mel"):
        basename = basename[:-4]
    print(f"\n=== Processing: {mel_path} ===")
    try:
        mel_tensor = torch.FloatTensor(load_mel_spectrogram(mel_path)).to(device)
        if mel_tensor.dim() == 2:
            mel_tensor = mel_tensor.unsqueeze(0)
        elif mel_tensor.dim() == 3:
            if mel_tensor.size(0) != 1:
                print(f"Warning: Batch size is {mel_tensor.size(0)}, using first sample")
                mel_tensor = mel_tensor[0:1]
        else:
            raise ValueError(f"Invalid mel spectrogram dimensions: {mel_tensor.shape}")
        print(f"Mel tensor shape for synthesis: {mel_tensor.shape}")
        expected_mels, actual_mels = h.num_mels, mel_tensor.size(1)
        if actual_mels != expected_mels:
            print(f"Warning: Mel bins mismatch. Expected: {expected_mels}, Got: {actual_mels}")
            if actual_mels > expected_mels:
                print(f"Truncating to {expected_mels} mel bins")
                mel_tensor = mel_tensor[:, :expected_mels, :]
            else:
                print(f"Padding to {expected_mels} mel bins")
                mel_tensor = torch.nn.functional.pad(mel_tensor, (0, 0, 0, expected_mels - actual_mels), "constant", 0)
        with torch.no_grad():
            print("Generating audio from mel spectrogram...")
            audio_output = generator(mel_tensor.contiguous()).squeeze().cpu().numpy()
            print(f"Generated audio shape: {audio_output.shape}")
            print(f"Generated audio range: {audio_output.min():.3f} to {audio_output.max():.3f}")
            print(f"Generated audio duration: {len(audio_output) / h.sampling_rate:.2f} seconds")
        output_path = os.path.join(output_dir, f"{basename}_from_mel.wav")
        write_wav(output_path, audio_output, h.sampling_rate)
        print(f"Generated audio saved to: {output_path}")
        save_mel_png(mel_tensor.squeeze().cpu().numpy(), f"Input Mel Spectrogram - {basename}",
                     os.path.join(output_dir, f"{basename}_input_mel.png"))
        stats = {
            "input_file": mel_path,
            "mel_shape": list(mel_tensor.shape),
            "mel_range": [float(mel_tensor.min()), float(mel_tensor.max())],
            "audio_shape": list(audio_output.shape),
            "audio_range": [float(audio_output.min()), float(audio_output.max())],
            "duration_seconds": len(audio_output) / h.sampling_rate,
            "sampling_rate": h.sampling_rate,
        }
        with open(os.path.join(output_dir, f"{basename}_synthesis_stats.json"), "w") as f:
            json.dump(stats, f, indent=2)
        return True, basename, stats
    except Exception as e:  # the reference reports and continues with the next file (:132-136)
        print(f"Error processing {mel_path}: {e}")
        import traceback
        traceback.print_exc()
        return False, None, None


def _html(h, processed_files, all_stats, success_count):
    parts = ["<!DOCTYPE html>\n<html>\n<head>\n<title>HiFi-GAN Mel-to-Audio Synthesis</title>\n</head>\n<body>\n",
             "<h1>HiFi-GAN Mel-to-Audio Synthesis</h1>\n",
             f"<div class=\"info\"><strong>Mel Spectrogram to Audio Synthesis</strong><br>Processed {success_count} "
             f"files successfully<br>Model config: {h.num_mels} mels, {h.sampling_rate}Hz sampling rate</div>\n"]
    for i, (basename, stats) in enumerate(zip(processed_files, all_stats)):
        parts.append(
            f"<div class=\"file-section\"><h2>File {i + 1}: {basename}</h2>\n"
            f"<div class=\"stats\">Input mel shape: {stats['mel_shape']}<br>"
            f"Mel range: {stats['mel_range'][0]:.3f} to {stats['mel_range'][1]:.3f}<br>"
            f"Generated audio duration: {stats['duration_seconds']:.2f} seconds<br>"
            f"Audio range: {stats['audio_range'][0]:.3f} to {stats['audio_range'][1]:.3f}</div>\n"
            f"<audio controls><source src=\"{basename}_from_mel.wav\" type=\"audio/wav\"></audio>\n"
            f"<img src=\"{basename}_input_mel.png\" alt=\"Input Mel Spectrogram - {basename}\"></div>\n")
    parts.append("</body>\n</html>\n")
    return "".join(parts)


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--input", required=True, help="Input .npy mel file or directory with .npy files")
    parser.add_argument("--checkpoint_file", required=True, help="Generator checkpoint file")
    parser.add_argument("--config", default="config_custom.json", help="HiFi-GAN config file")
    parser.add_argument("--output_dir", default="mel_synthesis_result", help="Output directory")
    parser.add_argument("--max_files", default=20, type=int, help="Maximum number of files to process (if directory)")
    parser.add_argument("--dtype", choices=["bf16x3", "fp32", "bf16", "fp8"], default=None, help="m2s compute dtype")
    args = parser.parse_args(argv)
    with open(args.config) as f:
        h = AttrDict(json.loads(f.read()))
    os.makedirs(args.output_dir, exist_ok=True)
    if not torch.cuda.is_available():
        raise RuntimeError("m2s needs an MI355X (HIP) device; no CPU fallback")
    device = torch.device("cuda")
    print(f"Using device: {device}")
    if os.path.isfile(args.input) and args.input.endswith(".npy"):
        mel_files = [args.input]
    elif os.path.isdir(args.input):
        mel_files = sorted(os.path.join(args.input, f) for f in os.listdir(args.input) if f.lower().endswith(".npy"))
        if not mel_files:
            print(f"No .npy files found in {args.input}")
            return None
        mel_files = mel_files[:args.max_files]
        print(f"Processing {len(mel_files)} mel files from directory")
    else:
        print(f"Invalid input: {args.input} (must be .npy file or directory)")
        return None
    with torch.no_grad():
        generator = Generator(h).to(device)
        state_dict_g = load_checkpoint(args.checkpoint_file, device)
        generator.load_state_dict(state_dict_g["generator"])
        generator.eval()
        if args.dtype:
            generator.m2s_dtype = args.dtype
        print("Removing weight norm...")
        removed = sum(safe_remove_weight_norm(u) for u in generator.ups)
        for resblock in generator.resblocks:
            try:
                resblock.remove_weight_norm()
            except (ValueError, AttributeError):
                pass
        removed += safe_remove_weight_norm(generator.conv_post)
        print(f"Weight norm removal completed. Removed from {removed} layers.")
        processed_files, all_stats = [], []
        for mel_file in mel_files:
            ok, basename, stats = process_mel_file(mel_file, h, generator, device, args.output_dir)
            if ok:
                processed_files.append(basename)
                all_stats.append(stats)
        print("\n=== Processing Complete ===")
        print(f"Successfully processed: {len(processed_files)}/{len(mel_files)} files")
        with open(os.path.join(args.output_dir, "mel_synthesis_results.html"), "w", encoding="utf-8") as f:
            f.write(_html(h, processed_files, all_stats, len(processed_files)))
        overall = {"total_files": len(mel_files), "successful_syntheses": len(processed_files),
                   "model_config": {k: h.get(k) for k in ("num_mels", "sampling_rate", "n_fft", "hop_size", "win_size")},
                   "individual_stats": all_stats}
        with open(os.path.join(args.output_dir, "overall_synthesis_stats.json"), "w") as f:
            json.dump(overall, f, indent=2)
        del generator, state_dict_g
        gc.collect()
    return processed_files


if __name__ == "__main__":
    main()
