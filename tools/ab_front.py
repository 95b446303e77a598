"""Same-box A/B of the encoder front (stem + blocks.0 + blocks.1.0: AcousticEngine.probe(x, 2)) and of the
whole CNN, between m2s packages: argv = package parent dirs (e.g. mri-to-speech_amd variants/old).  Each
package runs in its own subprocess, alternating A B A B, 1920 frames, bf16x3 and bf16.  GPU box only."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
from m2s import runtime as rt, synth
dev = torch.device("cuda", 0)
x = torch.rand(1920, 256, 256, device=dev)
for dt in ("bf16x3", "bf16"):
    eng = rt.AcousticEngine(synth.synth_acoustic_state(1), dtype=dt, device=dev)
    res = []
    for fn in (lambda: eng.probe(x, 2), lambda: eng.effnet(x)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 10)
    print(f"{sys.argv[1]:28s} {dt:7s} front {res[0]:7.3f} ms  cnn {res[1]:7.3f} ms", flush=True)
'''

for rnd in range(2):
    for pkg in sys.argv[1:]:
        r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(REPO, pkg)], capture_output=True, text=True,
                           timeout=300)
        sys.stdout.write(r.stdout)
        if r.returncode:
            sys.stdout.write(r.stderr[-2000:])
            sys.exit(r.returncode)
