"""Which frames carry NaN after each block of the fp8 engine when one frame holds a NaN pixel
(M2S_F8_EXPAND on / off).  Diagnostic, GPU box only."""
import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mri-to-speech_amd"))
from m2s import runtime as rt, synth
DEV = torch.device("cuda", 0)
st = synth.synth_acoustic_state(3)
fr = torch.from_numpy(synth.synth_frames(1, 4, seed=2)[0]).to(DEV)
fr[1, 100, 100] = float("nan")
for v in ("1", "0"):
    os.environ["M2S_F8_EXPAND"] = v
    eng = rt.AcousticEngine(st, dtype="fp8", device=DEV)
    rows = []
    for i in (2, 8, 9, 10, 12, 13, 18, 19, 20, 28):
        t = eng.probe(fr, i).cpu()
        rows.append(f"{i}:" + "".join("N" if torch.isnan(t[j]).any() else "." for j in range(4)))
    f = eng.effnet(fr).cpu()
    print(f"M2S_F8_EXPAND={v}", " ".join(rows), "feat:" + "".join("N" if torch.isnan(f[j]).any() else "." for j in range(4)), flush=True)
