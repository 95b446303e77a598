"""Does a HIP graph (torch.cuda.CUDAGraph capture of the engine's launch sequence) shorten the reference CLI's small
shapes?  configs[2] (1 clip x 30 frames, bf16x3 pipeline_forward) and configs[1] (8 x 4, bf16 acoustic forward):
GPU time per call by HIP events, eager vs graph replay, alternated; outputs compared.  GPU only."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mri-to-speech_amd"))
from m2s import runtime as rt, synth  # noqa: E402
from m2s.config import HIFIGAN_H  # noqa: E402

dev = torch.device("cuda", 0)
ac_sd, gen_sd = synth.synth_acoustic_state(0), synth.synth_generator_state(0)
mean, std = synth.synth_scaler()
x2 = torch.rand(1, 30, 256, 256, device=dev)
x1 = torch.rand(8, 4, 256, 256, device=dev)
pipe = rt.Pipeline(rt.AcousticEngine(ac_sd, dtype="bf16x3", device=dev),
                   rt.VocoderEngine(gen_sd, HIFIGAN_H, dtype="bf16x3", device=dev), mean, std)
a1 = rt.AcousticEngine(ac_sd, dtype="bf16", device=dev)


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


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    torch.cuda.synchronize()
    return g, out


ref2 = {k: v.clone() for k, v in pipe.forward(x2).items()}
ref1 = a1.forward(x1).clone()
g2, o2 = capture(lambda: pipe.forward(x2))
g1, o1 = capture(lambda: a1.forward(x1))
g2.replay()
g1.replay()
torch.cuda.synchronize()
pipe.ac.check()
a1.check()
print("graph outputs == eager:", {k: float((o2[k] - ref2[k]).abs().max()) for k in ref2}, float((o1 - ref1).abs().max()),
      flush=True)
res = {"eager2": [], "graph2": [], "eager1": [], "graph1": []}
for rnd in range(3):
    res["eager2"].append(timed(lambda: pipe.forward(x2)))
    res["graph2"].append(timed(g2.replay))
    res["eager1"].append(timed(lambda: a1.forward(x1)))
    res["graph1"].append(timed(g1.replay))
    print(f"# round {rnd}: " + " ".join(f"{k} {v[-1]:.3f}" for k, v in res.items()), flush=True)
for k, v in res.items():
    print(f"{k}: {np.median(v):.3f} ms per call")
