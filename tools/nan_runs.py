"""Cross-run NaN contamination check (diagnostic, GPU box only): run 1 poisons (a NaN frame, or the flag-ring
timeout with M2S spin limit 0), run 2 is clean; print which frames carry NaN after each probed block of run 2.
Workspace memory is reused between the runs (torch caching allocator), so a NaN left in a pad region that a
kernel reads (pad x 0 weight = NaN) shows up here."""
import ctypes
import os
import sys

import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mri-to-speech_amd"))
from m2s import _native, runtime as rt, synth  # noqa: E402

DEV = torch.device("cuda", 0)
st = synth.synth_acoustic_state(3)
clean = torch.from_numpy(synth.synth_frames(1, 4, seed=2)[0]).to(DEV)
taps = list(range(1, 29))
for dtype in ("fp8", "bf16", "bf16x3"):
    for mode in ("nanframe", "timeout"):
        eng = rt.AcousticEngine(st, dtype=dtype, device=DEV)
        fr = clean.clone()
        if mode == "nanframe":
            fr[1, 100, 100] = float("nan")
        else:
            _native.check(_native.lib().m2s_acoustic_set_ws_spin_limit(ctypes.c_void_p(eng.handle), 0))
        eng.effnet(fr)
        try:
            eng.check()
        except _native.M2SError:
            pass
        _native.check(_native.lib().m2s_acoustic_set_ws_spin_limit(ctypes.c_void_p(eng.handle), 1 << 20))
        rows = []
        for i in taps:
            t = eng.probe(clean, i).cpu()
            rows.append(f"{i}:" + "".join("N" if torch.isnan(t[j]).any() else "." for j in range(4)))
        f = eng.effnet(clean).cpu()
        print(f"{dtype} {mode}: run 2", " ".join(rows), "feat:" + "".join("N" if torch.isnan(f[j]).any() else "." for j in range(4)),
              flush=True)
