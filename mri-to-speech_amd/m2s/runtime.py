"""Device-side engines over libm2s (torch is used only for device memory and streams).

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


def _device(device) -> torch.device:
    if not torch.cuda.is_available():
        raise N.M2SError("m2s needs a HIP device (MI355X / gfx950); none is visible and there is no CPU fallback")
    d = torch.device(device if device is not None else "cuda")
    if d.type != "cuda":
        raise N.M2SError(f"m2s runs on HIP devices only, got {d}")
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _as_f32(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    if t.device != device:
        raise N.M2SError(f"input on {t.device}, engine on {device}")
    return t.to(torch.float32).contiguous()


class _WS:
    """Grow-only device workspace owned by an engine (stream-ordered by torch's allocator)."""

    def __init__(self, device):
        self.device, self.buf = device, None

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
        return self.buf


class AcousticEngine:
    def __init__(self, state_dict: Dict, n_mels: int = 64, rnn_hidden: int = 640, dtype: str = "bf16",
                 device=None, chunk: int = 256):
        self.device = _device(device)
        self.n_mels, self.rnn_hidden, self.dtype = n_mels, rnn_hidden, dtype
        L = N.lib()
        N.check(L.m2s_device_check(self.device.index))
        arr, keep = N.tensor_array(state_dict)
        h = C.c_void_p()
        N.check(L.m2s_acoustic_create(arr, len(arr), n_mels, rnn_hidden, N.DTYPES[dtype], self.device.index,
                                      C.byref(h)))
        del keep
        self._h = h
        self._ws = _WS(self.device)
        N.check(L.m2s_acoustic_set_chunk(self._h, int(chunk)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            N.lib().m2s_acoustic_destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def workspace_bytes(self, B, T, H, W) -> int:
        return int(N.lib().m2s_acoustic_workspace_bytes(self._h, B, T, H, W))

    def forward(self, frames: torch.Tensor) -> torch.Tensor:
        """frames (B,T,1,H,W) or (B,T,H,W) fp32 -> normalised mel (B,T,n_mels) fp32."""
        if frames.dim() == 5:
            if frames.size(2) != 1:
                raise N.M2SError("expected a single grey channel")
            frames = frames[:, :, 0]
        if frames.dim() != 4:
            raise N.M2SError(f"expected (B,T,H,W) frames, got {tuple(frames.shape)}")
        x = _as_f32(frames, self.device)
        B, T, H, W = x.shape
        out = torch.empty(B, T, self.n_mels, dtype=torch.float32, device=self.device)
        ws = self._ws.get(self.workspace_bytes(B, T, H, W))
        N.check(N.lib().m2s_acoustic_forward(self._h, _ptr(x), B, T, H, W, _ptr(out), _ptr(ws), ws.numel(),
                                             _stream(self.device)))
        return out

    def effnet(self, frames: torch.Tensor) -> torch.Tensor:
        """frames (N,H,W) -> GAP features (N,208)."""
        x = _as_f32(frames, self.device)
        n, H, W = x.shape
        out = torch.empty(n, 208, dtype=torch.float32, device=self.device)
        ws = self._ws.get(self.workspace_bytes(n, 1, H, W))
        N.check(N.lib().m2s_effnet_forward(self._h, _ptr(x), n, H, W, _ptr(out), _ptr(ws), ws.numel(),
                                           _stream(self.device)))
        return out

    def probe(self, frames: torch.Tensor, n_blocks: int) -> torch.Tensor:
        """Feature map after ``n_blocks`` timm blocks (0 = stem), (N,C,OH,OW) fp32."""
        x = _as_f32(frames, self.device)
        n, H, W = x.shape
        out = torch.empty(n * ((H + 1) // 2) * ((W + 1) // 2) * 32, dtype=torch.float32, device=self.device)
        ws = self._ws.get(self.workspace_bytes(n, 1, H, W))
        oh, ow, oc = C.c_int(), C.c_int(), C.c_int()
        N.check(N.lib().m2s_effnet_probe(self._h, _ptr(x), n, H, W, int(n_blocks), _ptr(out), C.byref(oh),
                                         C.byref(ow), C.byref(oc), _ptr(ws), ws.numel(), _stream(self.device)))
        return out[: n * oh.value * ow.value * oc.value].view(n, oh.value, ow.value, oc.value).permute(0, 3, 1, 2)

    def bilstm(self, feats: torch.Tensor):
        """feats (B,T,208) -> (sum-merged BiLSTM output (B,T,H), head output (B,T,n_mels))."""
        x = _as_f32(feats, self.device)
        B, T, _ = x.shape
        y = torch.empty(B, T, self.rnn_hidden, dtype=torch.float32, device=self.device)
        m = torch.empty(B, T, self.n_mels, dtype=torch.float32, device=self.device)
        ws = self._ws.get(self.workspace_bytes(B, T, 64, 64))
        N.check(N.lib().m2s_bilstm_summerge(self._h, _ptr(x), B, T, _ptr(y), _ptr(m), _ptr(ws), ws.numel(),
                                            _stream(self.device)))
        return y, m


class VocoderEngine:
    def __init__(self, state_dict: Dict, h, dtype: str = "bf16", device=None):
        self.device = _device(device)
        self.h, self.dtype = dict(h), dtype
        L = N.lib()
        N.check(L.m2s_device_check(self.device.index))
        arr, keep = N.tensor_array(state_dict)
        self._hh = N.hifigan_h(h)
        v = C.c_void_p()
        N.check(L.m2s_vocoder_create(arr, len(arr), C.byref(self._hh), N.DTYPES[dtype], self.device.index,
                                     C.byref(v)))
        del keep
        self._h = v
        self._ws = _WS(self.device)
        self.hop = 1
        for u in h["upsample_rates"]:
            self.hop *= int(u)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            N.lib().m2s_vocoder_destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def forward(self, mel: torch.Tensor, layout: int = 0) -> torch.Tensor:
        """mel (B,num_mels,T) [layout 0, as Generator.forward] or (B,T,num_mels) [layout 1] -> (B,1,T*hop)."""
        x = _as_f32(mel, self.device)
        if x.dim() != 3:
            raise N.M2SError(f"expected a 3-D mel, got {tuple(x.shape)}")
        B = x.shape[0]
        T = x.shape[2] if layout == 0 else x.shape[1]
        C_ = x.shape[1] if layout == 0 else x.shape[2]
        if C_ != self.h["num_mels"]:
            raise N.M2SError(f"mel has {C_} bins, generator expects {self.h['num_mels']}")
        wav = torch.empty(B, 1, T * self.hop, dtype=torch.float32, device=self.device)
        ws = self._ws.get(int(N.lib().m2s_vocoder_workspace_bytes(self._h, B, T)))
        N.check(N.lib().m2s_vocoder_forward(self._h, _ptr(x), int(layout), B, T, _ptr(wav), _ptr(ws), ws.numel(),
                                            _stream(self.device)))
        return wav


def mel_glue(mel_norm: torch.Tensor, mean: torch.Tensor, std: torch.Tensor):
    """(rows..., n_mels) -> (mel_db, mel_log), same shape."""
    d = mel_norm.device
    x = mel_norm.to(torch.float32).contiguous()
    n_mels = x.shape[-1]
    rows = x.numel() // n_mels
    mean = mean.to(device=d, dtype=torch.float32).contiguous()
    std = std.to(device=d, dtype=torch.float32).contiguous()
    db, ln = torch.empty_like(x), torch.empty_like(x)
    N.check(N.lib().m2s_mel_glue(_ptr(x), rows, n_mels, _ptr(mean), _ptr(std), _ptr(db), _ptr(ln), _stream(d)))
    return db, ln


def preprocess_frames(frames: torch.Tensor) -> torch.Tensor:
    """Decoded uint8 frames on the device, (T,H,W) grey or (T,H,W,3) BGR -> (T,H,W) fp32 in [0, 1]
    (_preprocess_frame, run_mri_video_inference.py:34-54; resizing stays on the host)."""
    if frames.dtype != torch.uint8:
        raise N.M2SError(f"expected uint8 frames, got {frames.dtype}")
    if frames.device.type != "cuda":
        raise N.M2SError("preprocess_frames runs on the HIP device; move the decoded frames there first")
    x = frames.contiguous()
    if x.dim() == 4 and x.shape[-1] == 3:
        ch = 3
    elif x.dim() == 3:
        ch = 1
    else:
        raise N.M2SError(f"expected (T,H,W) or (T,H,W,3) frames, got {tuple(x.shape)}")
    n, h, w = x.shape[:3]
    out = torch.empty(n, h, w, dtype=torch.float32, device=x.device)
    N.check(N.lib().m2s_preprocess_frames(_ptr(x), n, h, w, ch, _ptr(out), _stream(x.device)))
    return out


class Pipeline:
    """frames -> (mel_norm, mel_db, mel_log, wav) on one stream (run_mri_video_inference.py:218-242)."""

    def __init__(self, acoustic: AcousticEngine, vocoder: VocoderEngine, mean, std):
        if acoustic.device != vocoder.device:
            raise N.M2SError("acoustic model and vocoder must share a device")
        self.ac, self.voc, self.device = acoustic, vocoder, acoustic.device
        self.mean = torch.as_tensor(mean, dtype=torch.float32).to(self.device).contiguous()
        self.std = torch.as_tensor(std, dtype=torch.float32).to(self.device).contiguous()
        self._ws = _WS(self.device)

    def workspace_bytes(self, B, T, H, W) -> int:
        return int(N.lib().m2s_pipeline_workspace_bytes(self.ac.handle, self.voc.handle, B, T, H, W))

    def forward(self, frames: torch.Tensor, out: Optional[Dict[str, torch.Tensor]] = None, want_mels: bool = True):
        if frames.dim() == 5:
            frames = frames[:, :, 0]
        x = _as_f32(frames, self.device)
        B, T, H, W = x.shape
        nm = self.ac.n_mels
        if out is None:
            out = {"wav": torch.empty(B, T * self.voc.hop, dtype=torch.float32, device=self.device)}
            if want_mels:
                for k in ("mel_norm", "mel_db", "mel_log"):
                    out[k] = torch.empty(B, T, nm, dtype=torch.float32, device=self.device)
        ws = self._ws.get(self.workspace_bytes(B, T, H, W))
        N.check(N.lib().m2s_pipeline_forward(
            self.ac.handle, self.voc.handle, _ptr(x), B, T, H, W, _ptr(self.mean), _ptr(self.std),
            _ptr(out.get("mel_norm")), _ptr(out.get("mel_db")), _ptr(out.get("mel_log")), _ptr(out["wav"]),
            _ptr(ws), ws.numel(), _stream(self.device)))
        return out
