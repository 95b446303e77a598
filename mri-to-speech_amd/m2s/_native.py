"""ctypes binding of libm2s.so (C ABI: include/m2s.h).

The library is built in-tree (``make -C mri-to-speech_amd/csrc``) next to this file.  There
is no fallback: if the library is missing, or no gfx950 device is visible, every entry point
raises ``M2SError``.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Tuple

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libm2s.so")

F32, BF16, BF16X3, FP8 = 0, 1, 2, 3
# "bf16x3": split fp32 (hi + lo bf16 pairs, three-term MFMA products), fp32 tolerance;
# "fp8": e4m3 MFMA operands with per-channel weight scales (configs[4]; include/m2s.h)
DTYPES = {"fp32": F32, "float32": F32, "f32": F32, "bf16": BF16, "bfloat16": BF16, "bf16x3": BF16X3,
          "fp8": FP8, "e4m3": FP8}
ELEM_F32, ELEM_I64 = 0, 1
ABI_VERSION = 6  # include/m2s.h M2S_ABI_VERSION


class M2SError(RuntimeError):
    pass


class Tensor(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data", C.c_void_p), ("elem", C.c_int), ("ndim", C.c_int),
                ("shape", C.c_int64 * 4)]


class HifiganH(C.Structure):
    _fields_ = [("resblock", C.c_int), ("num_mels", C.c_int), ("upsample_initial_channel", C.c_int),
                ("n_up", C.c_int), ("upsample_rates", C.c_int * 8), ("upsample_kernel_sizes", C.c_int * 8),
                ("n_kernels", C.c_int), ("resblock_kernel_sizes", C.c_int * 8), ("n_dilations", C.c_int * 8),
                ("resblock_dilation_sizes", (C.c_int * 8) * 8)]


class ProfStat(C.Structure):
    _fields_ = [("name", C.c_char * 96), ("launches", C.c_int64), ("ms", C.c_double), ("flops", C.c_double),
                ("bytes", C.c_double)]


class ProfLaunch(C.Structure):
    _fields_ = [("name", C.c_char * 96), ("stage", C.c_char * 24), ("ms", C.c_double), ("flops", C.c_double),
                ("bytes", C.c_double), ("spill_bytes", C.c_double)]


_lib = None


def lib():
    """Load libm2s.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise M2SError(f"libm2s.so not found at {LIB_PATH}; build it with `make -C mri-to-speech_amd/csrc` "
                       "(there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp, i, sz, fp = C.c_void_p, C.c_int, C.c_size_t, C.c_void_p
    sig = {
        "m2s_abi_version": (i, []),
        "m2s_last_error": (C.c_char_p, []),
        "m2s_device_check": (i, [i]),
        "m2s_acoustic_create": (i, [C.POINTER(Tensor), i, i, i, i, i, C.POINTER(vp)]),
        "m2s_acoustic_destroy": (None, [vp]),
        "m2s_acoustic_set_chunk": (i, [vp, i]),
        "m2s_acoustic_status": (i, [vp]),
        "m2s_acoustic_set_lstm_spin_limit": (i, [vp, C.c_uint]),
        "m2s_acoustic_set_ws_spin_limit": (i, [vp, C.c_uint]),
        "m2s_acoustic_workspace_bytes": (sz, [vp, i, i, i, i]),
        "m2s_acoustic_forward": (i, [vp, fp, i, i, i, i, fp, vp, sz, vp]),
        "m2s_effnet_forward": (i, [vp, fp, i, i, i, fp, vp, sz, vp]),
        "m2s_effnet_probe": (i, [vp, fp, i, i, i, i, fp, C.POINTER(i), C.POINTER(i), C.POINTER(i), vp, sz, vp]),
        "m2s_bilstm_summerge": (i, [vp, fp, i, i, fp, fp, vp, sz, vp]),
        "m2s_mel_glue": (i, [fp, i, i, fp, fp, fp, fp, vp]),
        "m2s_preprocess_frames": (i, [fp, i, i, i, i, fp, vp]),
        "m2s_vocoder_create": (i, [C.POINTER(Tensor), i, C.POINTER(HifiganH), i, i, C.POINTER(vp)]),
        "m2s_vocoder_destroy": (None, [vp]),
        "m2s_vocoder_workspace_bytes": (sz, [vp, i, i]),
        "m2s_vocoder_forward": (i, [vp, fp, i, i, i, fp, vp, sz, vp]),
        "m2s_pipeline_workspace_bytes": (sz, [vp, vp, i, i, i, i]),
        "m2s_pipeline_forward": (i, [vp, vp, fp, i, i, i, i, fp, fp, fp, fp, fp, fp, vp, sz, vp]),
        "m2s_cam_create": (i, [C.POINTER(Tensor), i, i, C.POINTER(vp)]),
        "m2s_cam_destroy": (None, [vp]),
        "m2s_cam_bn_layers": (i, [vp]),
        "m2s_cam_bn_channels": (i, [vp, i]),
        "m2s_cam_workspace_bytes": (sz, [vp, i, i, i]),
        "m2s_cam_backbone": (i, [vp, fp, i, i, i, vp, fp, vp, sz, vp]),
        "m2s_bilstm_train_workspace_bytes": (sz, [i, i, i, i]),
        "m2s_bilstm_train_forward": (i, [fp, i, i, i, i, vp, fp, fp, fp, fp, vp, sz, vp]),
        "m2s_bilstm_train_backward": (i, [fp, fp, i, i, i, i, vp, fp, fp, fp, fp, vp, vp, sz, vp]),
        "m2s_linear_forward": (i, [fp, i, i, i, fp, fp, fp, vp]),
        "m2s_linear_backward": (i, [fp, fp, i, i, i, fp, fp, fp, fp, vp]),
        "m2s_gap_forward": (i, [fp, C.c_int64, i, fp, vp]),
        "m2s_gap_backward": (i, [fp, C.c_int64, i, fp, vp]),
        "m2s_prof_enable": (i, [i]),
        "m2s_prof_collect": (i, [C.POINTER(ProfStat), i, C.POINTER(i)]),
        "m2s_prof_launches": (i, [C.POINTER(ProfLaunch), i, C.POINTER(i)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.m2s_abi_version() != ABI_VERSION:
        raise M2SError("libm2s ABI version mismatch")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().m2s_last_error().decode(errors="replace")
        raise M2SError(f"libm2s error {rc}: {msg}")


def exported_symbols() -> List[str]:
    return [n for n in ("m2s_abi_version", "m2s_last_error", "m2s_device_check", "m2s_acoustic_create",
                        "m2s_acoustic_destroy", "m2s_acoustic_set_chunk", "m2s_acoustic_status",
                        "m2s_acoustic_set_lstm_spin_limit", "m2s_acoustic_set_ws_spin_limit", "m2s_acoustic_workspace_bytes",
                        "m2s_acoustic_forward", "m2s_effnet_forward", "m2s_effnet_probe", "m2s_bilstm_summerge",
                        "m2s_mel_glue", "m2s_preprocess_frames", "m2s_vocoder_create", "m2s_vocoder_destroy",
                        "m2s_vocoder_workspace_bytes", "m2s_vocoder_forward", "m2s_pipeline_workspace_bytes",
                        "m2s_pipeline_forward", "m2s_cam_create", "m2s_cam_destroy", "m2s_cam_bn_layers",
                        "m2s_cam_bn_channels", "m2s_cam_workspace_bytes", "m2s_cam_backbone",
                        "m2s_bilstm_train_workspace_bytes", "m2s_bilstm_train_forward", "m2s_bilstm_train_backward",
                        "m2s_linear_forward", "m2s_linear_backward", "m2s_gap_forward", "m2s_gap_backward",
                        "m2s_prof_enable", "m2s_prof_collect", "m2s_prof_launches")]


def tensor_array(state: Dict[str, "np.ndarray"]) -> Tuple[C.Array, list]:
    """Reference-format state dict (numpy / CPU torch) -> m2s_tensor[] plus the keep-alive list."""
    keep, items = [], []
    for k, v in state.items():
        a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        if a.dtype == np.int64:
            elem = ELEM_I64
        else:
            a = np.ascontiguousarray(a, dtype=np.float32)
            elem = ELEM_F32
        a = np.ascontiguousarray(a)
        if a.ndim > 4:
            raise M2SError(f"{k}: rank {a.ndim} > 4")
        name = k.encode()
        keep += [a, name]
        shape = (C.c_int64 * 4)(*(list(a.shape) + [0] * (4 - a.ndim)))
        items.append(Tensor(name, a.ctypes.data, elem, a.ndim, shape))
    arr = (Tensor * len(items))(*items)
    return arr, keep


def hifigan_h(h) -> HifiganH:
    s = HifiganH()
    rb = str(h["resblock"])
    if rb not in ("1", "2"):
        raise M2SError(f"unsupported resblock type {rb!r}")
    s.resblock = int(rb)
    s.num_mels = int(h["num_mels"])
    s.upsample_initial_channel = int(h["upsample_initial_channel"])
    ur, uk = list(h["upsample_rates"]), list(h["upsample_kernel_sizes"])
    rk, rd = list(h["resblock_kernel_sizes"]), list(h["resblock_dilation_sizes"])
    if len(ur) != len(uk) or len(rk) != len(rd) or not (1 <= len(ur) <= 8) or not (1 <= len(rk) <= 8):
        raise M2SError("inconsistent generator config")
    s.n_up = len(ur)
    for i, (u, k) in enumerate(zip(ur, uk)):
        s.upsample_rates[i], s.upsample_kernel_sizes[i] = int(u), int(k)
    s.n_kernels = len(rk)
    for j, (k, d) in enumerate(zip(rk, rd)):
        s.resblock_kernel_sizes[j] = int(k)
        s.n_dilations[j] = len(d)
        for q, dd in enumerate(d):
            s.resblock_dilation_sizes[j][q] = int(dd)
    return s


def prof_enable(on: bool) -> None:
    check(lib().m2s_prof_enable(1 if on else 0))


def prof_launches() -> List[dict]:
    """Every launch recorded since prof_enable(True), in launch order: name, stage, ms, flops, bytes
    (m2s_prof_launches); clears the record."""
    n = C.c_int(0)
    check(lib().m2s_prof_launches(None, 0, C.byref(n)))  # count only (records kept)
    cap = max(n.value, 1)
    buf = (ProfLaunch * cap)()
    check(lib().m2s_prof_launches(buf, cap, C.byref(n)))
    return [dict(name=buf[i].name.decode(), stage=buf[i].stage.decode(), ms=buf[i].ms, flops=buf[i].flops,
                 bytes=buf[i].bytes, spill_bytes=buf[i].spill_bytes) for i in range(min(n.value, cap))]


def aggregate(launches: List[dict], key: str = "name") -> List[dict]:
    """Per-kernel (key="name") or per-stage (key="stage") sums of prof_launches() records."""
    agg: Dict[str, dict] = {}
    for r in launches:
        a = agg.setdefault(r[key], dict(name=r[key], launches=0, ms=0.0, flops=0.0, bytes=0.0, spill_bytes=0.0))
        a["launches"] += 1
        for f in ("ms", "flops", "bytes", "spill_bytes"):
            a[f] += r.get(f, 0.0)
    return list(agg.values())


def prof_collect() -> List[dict]:
    """Per-kernel sums of the recorded launches (name, launches, ms, flops, bytes); clears the record."""
    return aggregate(prof_launches(), "name")
