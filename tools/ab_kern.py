"""Same-box A/B of per-kernel times between m2s packages (argv = package parent dirs, e.g. mri-to-speech_amd
variants/b): each package in its own subprocess, alternating, runs the bf16x3 CNN over 1920 frames with the
launch log on and prints the mean duration of every kernel whose name contains $AB_KERN (default ir_ws).
Diagnostic only (GPU box)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, torch
sys.path.insert(0, sys.argv[1])
from m2s import runtime as rt, synth, _native
dev = torch.device("cuda", 0)
x = torch.rand(1920, 256, 256, device=dev)
eng = rt.AcousticEngine(synth.synth_acoustic_state(1), dtype=os.environ.get("AB_DTYPE", "bf16x3"), device=dev)
for _ in range(3):
    eng.effnet(x)
torch.cuda.synchronize()
_native.prof_enable(True)
for _ in range(5):
    eng.effnet(x)
torch.cuda.synchronize()
agg = _native.aggregate(_native.prof_launches())
_native.prof_enable(False)
key = os.environ.get("AB_KERN", "ir_ws")
print("  ".join(f"{s['name']} {1000 * s['ms'] / s['launches']:7.1f} us" for s in agg if key in s["name"]),
      f"| cnn total {sum(s['ms'] for s in agg) / 5:7.3f} ms", flush=True)
'''
for rnd in range(int(os.environ.get("AB_ROUNDS", "2"))):
    for pkg in sys.argv[1:]:
        r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(REPO, pkg)], capture_output=True, text=True,
                           timeout=300)
        sys.stdout.write(f"{pkg:28s} " + r.stdout)
        if r.returncode:
            sys.stdout.write(r.stderr[-2000:])
            sys.exit(r.returncode)
