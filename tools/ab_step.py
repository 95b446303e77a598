"""Same-box A/B of the whole bench step (Pipeline.forward over 64 clips x 30 frames, bf16x3; AB_SHAPE=8x1000
and AB_DTYPES=fp8,bf16 for configs[4]) between m2s
packages: argv = package parent dirs (e.g. mri-to-speech_amd variants/base).  Each package runs in its own
subprocess, alternating A B A B; prints ms per step (median of 5 groups of 5).  GPU box only."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, statistics, torch
sys.path.insert(0, sys.argv[1])
from m2s import runtime as rt, synth
from m2s.config import HIFIGAN_H
dev = torch.device("cuda", 0)
dt = sys.argv[2]
g = torch.Generator(device="cpu").manual_seed(0)
import os
nc, nf = (int(v) for v in os.environ.get("AB_SHAPE", "64x30").split("x"))
frames = torch.rand(nc, nf, 256, 256, generator=g).to(dev)
ac = rt.AcousticEngine(synth.synth_acoustic_state(0), dtype=dt, device=dev)
voc = rt.VocoderEngine(synth.synth_generator_state(0), HIFIGAN_H, dtype=dt, device=dev)
mean, std = synth.synth_scaler()
pipe = rt.Pipeline(ac, voc, mean, std)
nw, ng = (2, 2) if nf * nc > 4000 else (3, 5)
for _ in range(nw):
    pipe.forward(frames)
torch.cuda.synchronize()
res = []
for _ in range(ng):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        pipe.forward(frames)
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / 5)
print(f"{sys.argv[1]:28s} {dt:7s} step {statistics.median(res):7.3f} ms  (min {min(res):7.3f})", flush=True)
'''

if sys.argv[1] == "--child":  # one package in this process (for rocprofv3 -- python3 tools/ab_step.py --child PKG DT)
    sys.argv = [sys.argv[0], os.path.join(REPO, sys.argv[2]), sys.argv[3]]
    exec(CHILD)
    sys.exit(0)
dtypes = os.environ.get("AB_DTYPES", "bf16x3").split(",")
for rnd in range(2):
    for dt in dtypes:
        for pkg in sys.argv[1:]:
            r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(REPO, pkg), dt], capture_output=True,
                               text=True, timeout=300)
            sys.stdout.write(r.stdout)
            if r.returncode:
                sys.stdout.write(r.stderr[-2000:])
                sys.exit(r.returncode)
