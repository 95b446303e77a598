"""BiLSTM recurrence timing at the configs[4] shape (1 clip x 1000 frames) and the bench shape (64 x 30).

Prints the per-recurrent-step time of the one-launch kernel (torch.cuda events around engine.bilstm
minus nothing: the input projection GEMM is a separate, short launch; rocprofv3 --kernel-trace
--stats on this script gives the kernel's own duration).  GPU box only.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mri-to-speech_amd"))
from m2s import runtime as rt, synth  # noqa: E402

DEV = torch.device("cuda", 0)
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "acoustic.npz"), allow_pickle=False)
# M2S_LSTM_MID=0 in the environment times the counter-barrier kernel at 4 < B <= 64 instead; argv[1] = engine
# dtype (fp32 default; bf16x3 / bf16 / fp8 run lstm_x3_kernel above 16 sequences unless M2S_LSTM_X3=0)
eng = rt.AcousticEngine(synth.synth_acoustic_state(int(g["seed"])), dtype=sys.argv[1] if len(sys.argv) > 1 else "fp32",
                        device=DEV)
shapes = ((1, 1000), (1, 30), (8, 1000), (16, 200), (32, 100), (64, 30), (64, 200))
for B, T in shapes:
    x = torch.randn(B, T, 208, device=DEV)
    for _ in range(3):
        eng.bilstm(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 5
    e0.record()
    for _ in range(n):
        eng.bilstm(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"bilstm B={B} T={T}: {ms:.3f} ms per call, {1000 * ms / T:.2f} us per recurrent step")
eng.check()
