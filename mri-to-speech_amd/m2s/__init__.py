"""m2s: MI355X-native rtMRI -> mel -> waveform hot path (host side).

The compute lives in ``libm2s.so`` (HIP, gfx950) behind the C ABI of include/m2s.h;
``m2s._native`` binds it with ctypes and raises when it is missing or no GPU is present.
"""
