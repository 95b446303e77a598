"""Drive ir_ws launches for its per-phase cycle trace.

Diagnostic only: rebuild mri-to-speech_amd/csrc/ir_ws.hip with -DIRWS_TRACE (relink libm2s.so),
run with M2S_IR_WS_TRACE=1 on the GPU box; stamps of workgroup 0 print to stderr.
"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mri-to-speech_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "diag"))  # tools/build_diag.sh
from m2s import runtime as rt, synth
DEV = torch.device("cuda", 0)
st = synth.synth_acoustic_state(1)
eng = rt.AcousticEngine(st, dtype="bf16x3", device=DEV)
fr = torch.rand(1920, 256, 256, device=DEV)
for _ in range(2):
    eng.effnet(fr)
torch.cuda.synchronize()
