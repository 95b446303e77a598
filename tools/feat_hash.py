"""Hash of the CNN features of a fixed synthetic batch (argv[1] = dtype, default fp8): same-bytes checks between
kernel-selection switches set in the environment of separate processes.  Diagnostic only (GPU box)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mri-to-speech_amd"))
from m2s import runtime as rt, synth  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(5)
x = torch.rand(256, 256, 256, generator=g).to(dev)
eng = rt.AcousticEngine(synth.synth_acoustic_state(1), dtype=sys.argv[1] if len(sys.argv) > 1 else "fp8", device=dev)
f = eng.effnet(x).float().cpu()
print(hashlib.sha256(f.numpy().tobytes()).hexdigest()[:16], float(f.abs().mean()), bool(torch.isfinite(f).all()))
