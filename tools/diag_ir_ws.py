"""Diagnostic: split-fp32 engines with and without ir_ws vs the fp32 oracle, per tap and per image."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mri-to-speech_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from m2s import runtime as rt, synth
from oracle import effnet

DEV = torch.device("cuda", 0)
g = np.load("tests/golden/acoustic.npz", allow_pickle=False)
st = synth.synth_acoustic_state(int(g["seed"]))
sd = {k: torch.from_numpy(v) for k, v in st.items()}
fr = torch.from_numpy(synth.synth_frames(1, 3, hw=(256, 256), seed=7)[0])
taps = []
effnet.effnet_features(sd, fr, taps=taps)
ws = rt.AcousticEngine(st, dtype="bf16x3", device=DEV)
os.environ["M2S_IR_WS"] = "0"
gr = rt.AcousticEngine(st, dtype="bf16x3", device=DEV)
x = fr.to(DEV)
for i in (9, 10, 11, 12, 13, 18, 19, 20, 28):
    ref = taps[i].numpy()
    a = ws.probe(x, i).cpu().numpy()
    b = gr.probe(x, i).cpu().numpy()
    s = np.abs(ref).max()
    d = np.abs(a - b)
    idx = np.unravel_index(d.argmax(), d.shape)
    print(f"tap {i} shape {ref.shape} ws {np.abs(a-ref).max()/s:.2e} grid {np.abs(b-ref).max()/s:.2e} ws-grid {d.max()/s:.2e} at {idx}"
          f" per-image {[float(np.abs(a[n]-b[n]).max()/s) for n in range(a.shape[0])]}")
