"""ir_ws ablation timing (diagnostic build only: tools/build_diag.sh, env M2S_IRWS_ABL = 0..3, see ir_ws.hip).
Prints the HIP-event time per launch of each ir_ws variant over a 1920-frame bf16x3 effnet pass."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mri-to-speech_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "diag"))
from m2s import _native, runtime as rt, synth  # noqa: E402

DEV = torch.device("cuda", 0)
eng = rt.AcousticEngine(synth.synth_acoustic_state(1), dtype="bf16x3", device=DEV)
fr = torch.rand(1920, 256, 256, device=DEV)
eng.effnet(fr)
torch.cuda.synchronize()
_native.prof_enable(True)
for _ in range(3):
    eng.effnet(fr)
torch.cuda.synchronize()
_native.prof_enable(False)
abl = os.environ.get("M2S_IRWS_ABL", "0")
for s in _native.prof_collect():
    if s["name"].startswith(("ir_ws", "se_ws")):
        print(f"abl {abl} {s['name']:30s} {1000 * s['ms'] / s['launches']:8.1f} us/launch")
