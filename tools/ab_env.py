"""Same-process A/B of a kernel-selection switch read at engine construction (M2S_STEM_WS, M2S_SE_WS, ...):
usage: python tools/ab_env.py VAR [probe_blocks] [dtype ...].  Times AcousticEngine.probe(x, probe_blocks)
(default 2: stem + blocks.0) and the whole CNN over 1920 frames with VAR=1 and VAR=0, alternating.  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mri-to-speech_amd"))
from m2s import runtime as rt, synth  # noqa: E402

var = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dtypes = sys.argv[3:] or ["bf16x3", "bf16"]
dev = torch.device("cuda", 0)
x = torch.rand(1920, 256, 256, device=dev)
st = synth.synth_acoustic_state(1)


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for dt in dtypes:
    engs = {}
    for v in os.environ.get("AB_VALUES", "1,0").split(","):  # e.g. AB_VALUES=4,0 for a config switch
        os.environ[var] = v
        engs[v] = rt.AcousticEngine(st, dtype=dt, device=dev)
    for rnd in range(2):
        for v, e in engs.items():
            os.environ[var] = v  # (switches read per launch, e.g. M2S_IRWS_PARTS, take the engine's value here too)
            print(f"{var}={v} {dt:7s} probe({nb}) {timed(lambda: e.probe(x, nb)):7.3f} ms  cnn {timed(lambda: e.effnet(x)):7.3f} ms",
                  flush=True)
