"""Same-process A/B of launch-time switches on the reference CLI's small shapes: configs[2] (1 clip x 30 frames,
bf16x3 pipeline_forward) and configs[1] (8 x 4 frames, bf16 acoustic forward), GPU time per call by HIP events,
settings alternated over rounds.  Switches read per launch (M2S_KSPLIT, M2S_KSPLIT_MAX, M2S_KSPLIT_MINST) take
effect at once; engine-construction switches need fresh engines (built per setting here).
usage: python tools/ab_small.py "M2S_KSPLIT_MAX=4" "M2S_KSPLIT_MAX=8" ...   ("" = defaults).  GPU only."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mri-to-speech_amd"))
from m2s import runtime as rt, synth  # noqa: E402
from m2s.config import HIFIGAN_H  # noqa: E402

dev = torch.device("cuda", 0)
settings = sys.argv[1:] or [""]
ac_sd, gen_sd = synth.synth_acoustic_state(0), synth.synth_generator_state(0)
mean, std = synth.synth_scaler()
x2 = torch.rand(1, 30, 256, 256, device=dev)
x1 = torch.rand(8, 4, 256, 256, device=dev)
KEYS = ("M2S_KSPLIT", "M2S_KSPLIT_MAX", "M2S_KSPLIT_MINST", "M2S_IRWS_MIN", "M2S_SEWS_MIN", "M2S_STEM_PARTS", "M2S_SE_FOLD")


def apply(s):
    for k in KEYS:
        os.environ.pop(k, None)
    for kv in filter(None, s.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v


def timed(fn, n=30):
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


engines = {}
for s in settings:
    apply(s)
    pipe = rt.Pipeline(rt.AcousticEngine(ac_sd, dtype="bf16x3", device=dev),
                       rt.VocoderEngine(gen_sd, HIFIGAN_H, dtype="bf16x3", device=dev), mean, std)
    engines[s] = (pipe, rt.AcousticEngine(ac_sd, dtype="bf16", device=dev))
    print(f"# engines for {s or 'default'} built", flush=True)
res = {s: ([], []) for s in settings}
for rnd in range(3):
    for s in settings:
        apply(s)
        pipe, a1 = engines[s]
        res[s][0].append(timed(lambda: pipe.forward(x2)))
        res[s][1].append(timed(lambda: a1.forward(x1)))
        print(f"# round {rnd} {s or 'default'}: {res[s][0][-1]:.3f} / {res[s][1][-1]:.3f} ms", flush=True)
for s in settings:
    print(f"{s or 'default':40s} configs2 {np.median(res[s][0]):.3f} ms  configs1 {np.median(res[s][1]):.3f} ms  "
          f"(rounds {' '.join(f'{v:.3f}' for v in res[s][0])} | {' '.join(f'{v:.3f}' for v in res[s][1])})", flush=True)
