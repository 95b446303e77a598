"""Device-side engines over libm2s.

The packed models are created and destroyed through the C ABI (ctypes, ``_native``); every compute
call goes through the PyTorch-ROCm custom ops ``torch.ops.m2s.*`` (``ops``, csrc/torch_ops.cpp), which
allocate outputs and workspace with the torch caching allocator on the current HIP stream.

* ``AcousticEngine``  - packed CNN + BiLSTM + head (replaces OTNLikeCNNBiLSTM.forward,
                        mri2speech_code/mri_acoustic_model.py:116-136)
* ``VocoderEngine``   - packed HiFi-GAN generator (replaces Generator.forward, models.py:113-131)
* ``mel_glue``        - denormalize_mel + dB -> ln-power (run_mri_video_inference.py:160-163,227-233)
* ``Pipeline``        - frames -> mel_norm / mel_db / mel_log / wav in one call on one stream
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import torch

from . import _native as N
from . import ops as _ops
from .config import CNN_CHUNK


def _device(device) -> torch.device:
    if not torch.cuda.is_available():
        raise N.M2SError("m2s needs a HIP device (MI355X / gfx950); none is visible and there is no CPU fallback")
    d = torch.device(device if device is not None else "cuda")
    if d.type != "cuda":
        raise N.M2SError(f"m2s runs on HIP devices only, got {d}")
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def _as_f32(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    if t.device != device:
        raise N.M2SError(f"input on {t.device}, engine on {device}")
    return t.to(torch.float32).contiguous()


class AcousticEngine:
    """libm2s's acoustic model on one device.  ``chunk``: frames per CNN pass (include/m2s.h
    m2s_acoustic_set_chunk); a pass may hold up to chunk + chunk // 16 frames when that saves a short tail
    pass, so size limits chosen through ``chunk`` have ~6 % of headroom to leave."""

    def __init__(self, state_dict: Dict, n_mels: int = 64, rnn_hidden: int = 640, dtype: str = "bf16x3",
                 device=None, chunk: int = CNN_CHUNK):
        self.device = _device(device)
        self.n_mels, self.rnn_hidden, self.dtype = n_mels, rnn_hidden, dtype
        if dtype not in N.DTYPES:
            raise N.M2SError(f"unknown dtype {dtype!r}; one of {sorted(N.DTYPES)}")
        L = N.lib()
        self.ops = _ops.load()
        N.check(L.m2s_device_check(self.device.index))
        arr, keep = N.tensor_array(state_dict)
        h = C.c_void_p()
        N.check(L.m2s_acoustic_create(arr, len(arr), n_mels, rnn_hidden, N.DTYPES[dtype], self.device.index,
                                      C.byref(h)))
        del keep
        self._h = h
        self._destroy = L.m2s_acoustic_destroy  # bound now: module globals may be gone at exit
        N.check(L.m2s_acoustic_set_chunk(self._h, int(chunk)))

    def __del__(self):
        h, destroy = getattr(self, "_h", None), getattr(self, "_destroy", None)
        if h is not None and h.value and destroy is not None:
            destroy(h)
            self._h = None

    @property
    def handle(self) -> int:
        """The m2s_acoustic* as the int the torch.ops.m2s ops take."""
        return int(self._h.value)

    def check(self):
        """Synchronise the device and raise M2SError if a launch of this engine failed asynchronously
        (a BiLSTM grid-barrier timeout: its outputs hold NaN; include/m2s.h m2s_acoustic_status)."""
        torch.cuda.synchronize(self.device)
        N.check(N.lib().m2s_acoustic_status(self._h))

    def forward(self, frames: torch.Tensor) -> torch.Tensor:
        """frames (B,T,1,H,W) or (B,T,H,W) fp32 -> normalised mel (B,T,n_mels) fp32."""
        if frames.dim() == 5:
            if frames.size(2) != 1:
                raise N.M2SError("expected a single grey channel")
            frames = frames[:, :, 0]
        if frames.dim() != 4:
            raise N.M2SError(f"expected (B,T,H,W) frames, got {tuple(frames.shape)}")
        return self.ops.acoustic_forward(self.handle, _as_f32(frames, self.device), self.n_mels)

    def effnet(self, frames: torch.Tensor) -> torch.Tensor:
        """frames (N,H,W) -> GAP features (N,208)."""
        return self.ops.effnet_forward(self.handle, _as_f32(frames, self.device))

    def probe(self, frames: torch.Tensor, n_blocks: int) -> torch.Tensor:
        """Feature map after ``n_blocks`` timm blocks (0 = stem), (N,C,OH,OW) fp32."""
        return self.ops.effnet_features(self.handle, _as_f32(frames, self.device), int(n_blocks))

    def bilstm(self, feats: torch.Tensor):
        """feats (B,T,208) -> (sum-merged BiLSTM output (B,T,H), head output (B,T,n_mels))."""
        return self.ops.bilstm_summerge(self.handle, _as_f32(feats, self.device), self.rnn_hidden, self.n_mels)


class VocoderEngine:
    def __init__(self, state_dict: Dict, h, dtype: str = "bf16x3", device=None):
        self.device = _device(device)
        self.h, self.dtype = dict(h), dtype
        if dtype not in N.DTYPES:
            raise N.M2SError(f"unknown dtype {dtype!r}; one of {sorted(N.DTYPES)}")
        L = N.lib()
        self.ops = _ops.load()
        N.check(L.m2s_device_check(self.device.index))
        arr, keep = N.tensor_array(state_dict)
        self._hh = N.hifigan_h(h)
        v = C.c_void_p()
        N.check(L.m2s_vocoder_create(arr, len(arr), C.byref(self._hh), N.DTYPES[dtype], self.device.index,
                                     C.byref(v)))
        del keep
        self._h = v
        self._destroy = L.m2s_vocoder_destroy
        self.hop = 1
        for u in h["upsample_rates"]:
            self.hop *= int(u)

    def __del__(self):
        h, destroy = getattr(self, "_h", None), getattr(self, "_destroy", None)
        if h is not None and h.value and destroy is not None:
            destroy(h)
            self._h = None

    @property
    def handle(self) -> int:
        return int(self._h.value)

    def forward(self, mel: torch.Tensor, layout: int = 0) -> torch.Tensor:
        """mel (B,num_mels,T) [layout 0, as Generator.forward] or (B,T,num_mels) [layout 1] -> (B,1,T*hop)."""
        x = _as_f32(mel, self.device)
        if x.dim() != 3:
            raise N.M2SError(f"expected a 3-D mel, got {tuple(x.shape)}")
        C_ = x.shape[1] if layout == 0 else x.shape[2]
        if C_ != self.h["num_mels"]:
            raise N.M2SError(f"mel has {C_} bins, generator expects {self.h['num_mels']}")
        return self.ops.hifigan_forward(self.handle, x, int(layout), self.hop)


def mel_glue(mel_norm: torch.Tensor, mean: torch.Tensor, std: torch.Tensor):
    """(rows..., n_mels) -> (mel_db, mel_log), same shape."""
    d = mel_norm.device
    return _ops.load().mel_glue(mel_norm.to(torch.float32).contiguous(), torch.as_tensor(mean).to(d),
                                torch.as_tensor(std).to(d))


def preprocess_frames(frames: torch.Tensor) -> torch.Tensor:
    """Decoded uint8 frames on the device, (T,H,W) grey or (T,H,W,3) BGR -> (T,H,W) fp32 in [0, 1]
    (_preprocess_frame, run_mri_video_inference.py:34-54; resizing stays on the host)."""
    if frames.dtype != torch.uint8:
        raise N.M2SError(f"expected uint8 frames, got {frames.dtype}")
    if frames.device.type != "cuda":
        raise N.M2SError("preprocess_frames runs on the HIP device; move the decoded frames there first")
    if not (frames.dim() == 3 or (frames.dim() == 4 and frames.shape[-1] == 3)):
        raise N.M2SError(f"expected (T,H,W) or (T,H,W,3) frames, got {tuple(frames.shape)}")
    return _ops.load().preprocess_frames(frames.contiguous())


class Pipeline:
    """frames -> (mel_norm, mel_db, mel_log, wav) on one stream (run_mri_video_inference.py:218-242)."""

    def __init__(self, acoustic: AcousticEngine, vocoder: VocoderEngine, mean, std):
        if acoustic.device != vocoder.device:
            raise N.M2SError("acoustic model and vocoder must share a device")
        self.ac, self.voc, self.device = acoustic, vocoder, acoustic.device
        self.mean = torch.as_tensor(mean, dtype=torch.float32).to(self.device).contiguous()
        self.std = torch.as_tensor(std, dtype=torch.float32).to(self.device).contiguous()

    def forward(self, frames: torch.Tensor, out: Optional[Dict[str, torch.Tensor]] = None):
        """frames (B,T,[1,]H,W) -> dict mel_norm / mel_db / mel_log (B,T,n_mels), wav (B,T*hop)."""
        if frames.dim() == 5:
            frames = frames[:, :, 0]
        x = _as_f32(frames, self.device)
        mn, db, ln, wav = self.ac.ops.pipeline_forward(self.ac.handle, self.voc.handle, x, self.mean, self.std,
                                                       self.ac.n_mels, self.voc.hop)
        res = {"mel_norm": mn, "mel_db": db, "mel_log": ln, "wav": wav}
        if out is not None:  # caller-owned buffers (kept for API compatibility)
            for k, v in res.items():
                if k in out:
                    out[k].copy_(v)
            return out
        return res
