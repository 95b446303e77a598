"""Run the bench workload for a few steps with no timing/extras (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mri-to-speech_amd"))
sys.path.insert(0, REPO)
from m2s import runtime, synth  # noqa: E402
from m2s.config import HIFIGAN_H  # noqa: E402
import bench  # noqa: E402

steps = int(os.environ.get("STEPS", "2"))
clips, frames = int(os.environ.get("CLIPS", "64")), int(os.environ.get("FRAMES", "30"))
dev = torch.device("cuda", 0)
dt = os.environ.get("DTYPE", "bf16x3")
ac = runtime.AcousticEngine(synth.synth_acoustic_state(0), dtype=dt, device=dev, chunk=int(os.environ.get("CHUNK", "1920")))
voc = runtime.VocoderEngine(synth.synth_generator_state(0), HIFIGAN_H, dtype=dt, device=dev)
mean, std = synth.synth_scaler()
pipe = runtime.Pipeline(ac, voc, mean, std)
x = bench.make_frames(clips, frames, 256, 0, dev)
log = os.environ.get("M2S_LAUNCH_LOG")  # the launch sequence with libm2s's stage tags (tools/evidence.py aligns the
if log:                                 # PMC dispatches with it)
    from m2s import _native
    _native.prof_enable(True)
for _ in range(steps):
    pipe.forward(x)
torch.cuda.synchronize()
if log:
    import json
    _native.prof_enable(False)
    with open(log, "w") as fh:
        json.dump({"steps": steps, "launches": [[r["name"], r["stage"]] for r in _native.prof_launches()]}, fh)
print("done")
