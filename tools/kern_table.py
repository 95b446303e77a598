"""Per-kernel table of the bench step for each dtype in argv (default bf16 fp8): mean ms per step by kernel
name and by stage tag, from libm2s's launch log (HIP events on each launch's stream).  Diagnostic only (GPU box)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mri-to-speech_amd"))
sys.path.insert(0, REPO)
from m2s import runtime, synth, _native  # noqa: E402
from m2s.config import HIFIGAN_H  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
x = bench.make_frames(64, 30, 256, 0, dev)
mean, std = synth.synth_scaler()
steps = int(os.environ.get("STEPS", "5"))
for dt in sys.argv[1:] or ["bf16", "fp8"]:
    ac = runtime.AcousticEngine(synth.synth_acoustic_state(0), dtype=dt, device=dev)
    voc = runtime.VocoderEngine(synth.synth_generator_state(0), HIFIGAN_H, dtype=dt, device=dev)
    pipe = runtime.Pipeline(ac, voc, mean, std)
    for _ in range(3):
        pipe.forward(x)
    torch.cuda.synchronize()
    _native.prof_enable(True)
    for _ in range(steps):
        pipe.forward(x)
    torch.cuda.synchronize()
    launches = _native.prof_launches()
    _native.prof_enable(False)
    tot = sum(l["ms"] for l in launches) / steps
    print(f"== {dt}: {tot:.3f} ms/step of kernel time")
    for key in ("stage", "name"):
        for s in sorted(_native.aggregate(launches, key=key), key=lambda s: -s["ms"])[:int(os.environ.get("TOP", "40"))]:
            print(f"  {s['name']:58s} n/step={s['launches'] / steps:6.1f} ms/step={s['ms'] / steps:7.3f}")
        print()
