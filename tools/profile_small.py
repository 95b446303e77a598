"""The reference CLI's own shapes for a rocprofv3 kernel trace (verdict r05 item 2):

* MODE=c2 -- configs[2]: one clip x 30 frames, pinned uint8 host frames -> H2D -> preprocess_frames ->
  pipeline_forward (bf16x3) -> D2H, CALLS calls (scripts/run_mri_video_inference.py:215-242);
* MODE=c1 -- configs[1]: the CNN-BiLSTM forward, 8 clips x 4 frames resident, bf16, CALLS calls.

Each call is bracketed by a one-thread marker kernel (torch's exp_ of a 1-element tensor) so that
tools/small_timeline.py can cut the trace into calls.  Usage (GPU box):
  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/profile_small.py"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mri-to-speech_amd"))
sys.path.insert(0, REPO)
from m2s import runtime, synth  # noqa: E402
from m2s.config import HIFIGAN_H  # noqa: E402
import bench  # noqa: E402

mode = os.environ.get("MODE", "c2")
calls = int(os.environ.get("CALLS", "20"))
dev = torch.device("cuda", 0)
mark = torch.zeros(1, device=dev)
lat = []
if mode == "c2":
    dt = os.environ.get("DTYPE", "bf16x3")
    ac = runtime.AcousticEngine(synth.synth_acoustic_state(0), dtype=dt, device=dev)
    voc = runtime.VocoderEngine(synth.synth_generator_state(0), HIFIGAN_H, dtype=dt, device=dev)
    mean, std = synth.synth_scaler()
    pipe = runtime.Pipeline(ac, voc, mean, std)
    T = int(os.environ.get("FRAMES", "30"))
    hf = bench.host_frames_u8(1, T, 256, seed=2024)

    def call():
        x8 = hf.to(dev, non_blocking=True)
        x = runtime.preprocess_frames(x8.view(T, 256, 256)).view(1, T, 256, 256)
        o = pipe.forward(x)
        host = {k: o[k].to("cpu", non_blocking=True) for k in ("wav", "mel_db", "mel_log")}
        torch.cuda.synchronize(dev)
        return host
else:
    dt = os.environ.get("DTYPE", "bf16")
    ac = runtime.AcousticEngine(synth.synth_acoustic_state(0), dtype=dt, device=dev)
    B, T = int(os.environ.get("CLIPS", "8")), int(os.environ.get("FRAMES", "4"))
    x1 = bench.make_frames(B, T, 256, 5, dev)

    def call():
        ac.forward(x1)
        torch.cuda.synchronize(dev)

for _ in range(5):
    call()
for _ in range(calls):
    mark.exp_()
    t0 = time.perf_counter()
    call()
    lat.append((time.perf_counter() - t0) * 1e3)
mark.exp_()
torch.cuda.synchronize(dev)
ac.check()
lat = np.sort(np.array(lat))
print(f"{mode} {dt}: host wall per call p50 {np.percentile(lat, 50):.3f} ms, min {lat[0]:.3f} ms over {calls} calls")
