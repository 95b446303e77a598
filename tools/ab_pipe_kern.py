"""Same-box A/B of per-kernel times over the whole pipeline step (CNN-BiLSTM + glue + HiFi-GAN) between m2s packages
(argv = package parent dirs, e.g. mri-to-speech_amd variants/old): each package in its own subprocess, alternating,
runs Pipeline.forward on AB_SHAPE (default 64x30) in each of AB_DTYPES (default bf16x3) with the launch log on and
prints the mean duration of every kernel whose name contains one of AB_KERN (comma-separated, default rb1_fused),
plus their sum per step.  Diagnostic only (GPU box)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, torch
sys.path.insert(0, sys.argv[1])
from m2s import runtime as rt, synth, _native
from m2s.config import HIFIGAN_H
dev = torch.device("cuda", 0)
dt = sys.argv[2]
nc, nf = (int(v) for v in os.environ.get("AB_SHAPE", "64x30").split("x"))
frames = torch.rand(nc, nf, 256, 256, generator=torch.Generator().manual_seed(0)).to(dev)
mean, std = synth.synth_scaler()
pipe = rt.Pipeline(rt.AcousticEngine(synth.synth_acoustic_state(0), dtype=dt, device=dev),
                   rt.VocoderEngine(synth.synth_generator_state(0), HIFIGAN_H, dtype=dt, device=dev), mean, std)
reps = 2 if nc * nf > 4000 else 5
for _ in range(2):
    pipe.forward(frames)
torch.cuda.synchronize()
_native.prof_enable(True)
for _ in range(reps):
    pipe.forward(frames)
torch.cuda.synchronize()
agg = _native.aggregate(_native.prof_launches())
_native.prof_enable(False)
keys = os.environ.get("AB_KERN", "rb1_fused").split(",")
sel = [s for s in agg if any(k in s["name"] for k in keys)]
print(f"{dt:7s} " + "  ".join(f"{s['name']} {1000 * s['ms'] / s['launches']:7.1f} us" for s in sel),
      f"| selected {sum(s['ms'] for s in sel) / reps:7.3f} ms/step | all {sum(s['ms'] for s in agg) / reps:7.3f} ms/step",
      flush=True)
'''
for rnd in range(int(os.environ.get("AB_ROUNDS", "2"))):
    for dt in os.environ.get("AB_DTYPES", "bf16x3").split(","):
        for pkg in sys.argv[1:]:
            r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(REPO, pkg), dt], capture_output=True, text=True,
                               timeout=300)
            sys.stdout.write(f"{pkg:28s} " + r.stdout)
            if r.returncode:
                sys.stdout.write(r.stderr[-2000:])
                sys.exit(r.returncode)
