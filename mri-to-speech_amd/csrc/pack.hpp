// Host-side packing helpers shared by the model plans (model.cpp) and the Grad-CAM path (cam.cpp):
// state-dict lookup, host bf16 / split / e4m3 conversions, dense-conv packing into the conv kernels'
// [phase][n_pad][kp] rows, ConvArgs set-up, TF-SAME padding and the tf_efficientnetv2_b2 stage table.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "model.hpp"

namespace m2s {

inline const HostTensor& need(const StateDict& sd, const std::string& k, std::vector<int64_t> shape) {
  auto it = sd.find(k);
  if (it == sd.end()) throw Error(M2S_E_ARG, "missing state-dict key: " + k);
  if (it->second.shape != shape) {
    std::string got, want;
    for (auto d : it->second.shape) got += std::to_string(d) + ",";
    for (auto d : shape) want += std::to_string(d) + ",";
    throw Error(M2S_E_ARG, "shape mismatch for " + k + ": got (" + got + ") want (" + want + ")");
  }
  return it->second;
}

inline uint16_t f2bf_host(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float bf2f_host(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline void split_host(float f, uint16_t* hi, uint16_t* lo) {
  *hi = f2bf_host(f);
  *lo = f2bf_host(f - bf2f_host(*hi));
}

// Event-profiler record names = the kernels' demangled symbols as rocprofv3 prints them, so the
// two profiles can be joined on the name.
template <typename T>
inline std::string tname(const char* base, const char* extra = "") {
  return std::string(base) + (std::is_same<T, bf16_t>::value ? "<unsigned short" : std::is_same<T, sp_t>::value ? "<m2s::sp_t" : "<float") +
         extra + ">";
}

inline int kc_of(int dtype) { return dtype == M2S_DT_F32 ? Elem<float>::KC : Elem<bf16_t>::KC; }
// bytes per activation element of a dtype's storage (split fp32: hi + lo; e4m3 operands keep bf16)
inline size_t act_bytes(int dtype) { return dtype == M2S_DT_BF16 || dtype == M2S_DT_FP8 ? 2 : 4; }

// OCP e4m3fn rounding of a float (round to nearest even; 3 mantissa bits, exponents -6..8 with
// subnormals down to 2^-9, largest finite 448): the grid gfx950's v_cvt_pk_fp8_f32 rounds onto.
inline float e4m3_host(float x) {
  if (!(x == x) || x == 0.f) return 0.f;
  const float a = std::fabs(x);
  if (a >= 448.f) return std::copysign(448.f, x);
  int e;
  std::frexp(a, &e);                       // a = m * 2^e, m in [0.5, 1): leading bit 2^(e-1)
  const float step = std::ldexp(1.f, std::max(e - 1, -6) - 3);
  return std::copysign(std::nearbyint(a / step) * step, x);
}


// OCP e4m3fn bit pattern of a value on the e4m3 grid (e4m3_host output; -0 -> +0)
inline uint8_t e4m3_bits_host(float v) {
  if (v == 0.f) return 0;
  const uint8_t sgn = v < 0.f ? 0x80 : 0;
  const float a = std::fabs(v);
  int e;
  std::frexp(a, &e);
  const int E = e - 1;  // a = 1.m x 2^E
  if (E < -6) return sgn | (uint8_t)std::nearbyint(a / std::ldexp(1.f, -9));  // subnormal: m x 2^-9
  return sgn | (uint8_t)((E + 7) << 3) | (uint8_t)std::nearbyint((a / std::ldexp(1.f, E) - 1.f) * 8.f);
}

// A 1x1 conv as e4m3 bytes for the K = 128 block-scaled MFMA (gemm128.hip): rows [n_pad][kp], kp = cin
// rounded up to 128, w[n][c] / s[n] on the e4m3 grid with s[n] = amax_n / 448; scales and bias [n_pad].
template <class Get, class Bias>
inline void pack_gemm_f8(Arena& ar, int cin, int cout, int n_pad, int kp, Get get, Bias bias, size_t* w_off,
                         size_t* s_off, size_t* b_off) {
  std::vector<uint8_t> w((size_t)n_pad * kp, 0);
  std::vector<float> sc(n_pad, 1.f), b(n_pad, 0.f);
  for (int n = 0; n < cout; ++n) {
    float amax = 0.f;
    for (int c = 0; c < cin; ++c) amax = std::max(amax, std::fabs(get(n, c)));
    if (amax > 0.f) sc[n] = amax / 448.f;
    for (int c = 0; c < cin; ++c) w[(size_t)n * kp + c] = e4m3_bits_host(e4m3_host(get(n, c) / sc[n]));
    b[n] = bias(n);
  }
  *w_off = ar.add_vec(w);
  *s_off = ar.add_vec(sc);
  *b_off = ar.add_vec(b);
}

inline PConv make_pconv(int kind, int cin, int cout, int ntaps, int dtype) {
  PConv p;
  p.kind = kind;
  p.cin = cin;
  p.cout = cout;
  p.cs_in = chan_stride(cin);
  p.cs_out = chan_stride(cout);
  p.ntaps = ntaps;
  const int kc = kc_of(dtype);
  p.tpc = conv_tpc(p.cs_in, kc);
  p.kp = conv_kp(ntaps, p.cs_in, kc);
  p.n_pad = round_up(p.cs_out, 64);
  return p;
}

// get(phase, n, tap, c) for n < cout, tap < ntaps, c < cin; bias(n)
template <class Get, class Bias>
inline void pack_conv(Arena& ar, int dtype, PConv& p, Get get, Bias bias) {
  std::vector<float> w((size_t)p.phases * p.n_pad * p.kp, 0.f);
  for (int ph = 0; ph < p.phases; ++ph)
    for (int n = 0; n < p.cout; ++n)
      for (int t = 0; t < p.ntaps; ++t)
        for (int c = 0; c < p.cin; ++c)
          w[((size_t)ph * p.n_pad + n) * p.kp + (size_t)t * p.cs_in + c] = get(ph, n, t, c);
  if (dtype == M2S_DT_FP8) {  // per output channel: s = amax / 448, w / s on the e4m3 grid (exact in bf16)
    std::vector<float> sc(p.n_pad, 1.f);
    for (int n = 0; n < p.n_pad; ++n) {
      float amax = 0.f;
      for (int ph = 0; ph < p.phases; ++ph)
        for (int k = 0; k < p.kp; ++k) amax = std::max(amax, std::fabs(w[((size_t)ph * p.n_pad + n) * p.kp + k]));
      if (amax > 0.f) sc[n] = amax / 448.f;
    }
    std::vector<uint16_t> h(w.size());
    for (size_t i = 0; i < w.size(); ++i) h[i] = f2bf_host(e4m3_host(w[i] / sc[(i / p.kp) % p.n_pad]));
    p.w_off = ar.add_vec(h);
    p.ws_off = ar.add_vec(sc);
    p.fp8 = true;
  } else if (dtype == M2S_DT_BF16) {
    std::vector<uint16_t> h(w.size());
    for (size_t i = 0; i < w.size(); ++i) h[i] = f2bf_host(w[i]);
    p.w_off = ar.add_vec(h);
  } else if (dtype == M2S_DT_BF16X3) {  // rows [hi kp | lo kp]
    std::vector<uint16_t> h(2 * w.size());
    const size_t rows = w.size() / p.kp;
    for (size_t r = 0; r < rows; ++r)
      for (int k = 0; k < p.kp; ++k) split_host(w[r * p.kp + k], &h[2 * r * p.kp + k], &h[(2 * r + 1) * p.kp + k]);
    p.w_off = ar.add_vec(h);
  } else {
    p.w_off = ar.add_vec(w);
  }
  std::vector<float> b(p.n_pad, 0.f);
  for (int n = 0; n < p.cout; ++n) b[n] = bias(n);
  p.b_off = ar.add_vec(b);
}

inline ConvArgs conv_args(const PConv& p) {
  ConvArgs a;
  std::memset(&a, 0, sizeof(a));
  a.w = p.w;
  a.bias = p.b;
  a.kind = p.kind;
  a.cs_in = p.cs_in;
  a.cs_out = p.cs_out;
  a.n_pad = p.n_pad;
  a.kp = p.kp;
  a.ntaps = p.ntaps;
  a.tpc = p.tpc;
  a.ks = p.ks;
  a.stride = p.stride;
  a.dil = p.dil;
  a.pad_left = p.pad_left;
  a.ct_u = p.ct_u;
  a.ct_pad = p.ct_pad;
  a.ct_k = p.ct_k;
  a.OH = 1;
  a.accum_div = 1.f;
  a.wscale = p.wscale;
  return a;
}

// algorithmic work of one conv launch (profiler records): flops, and compulsory traffic = input
// once, output once (+ residual / accumulator read), weights once
template <typename T>
inline void conv_cost(const ConvArgs& a, const PConv& p, double* flops_out, double* bytes_out) {
  const double rows = (double)a.M;
  const double flops = 2.0 * p.macs_per_row * rows;
  const double es = sizeof(T) * Elem<T>::R;
  // compulsory traffic: input once, output once (+ residual/accum read), weights once
  double in_rows = p.kind == KIND_CONV2D ? (double)a.IH * a.IW * (a.M / ((double)a.OH * a.OW))
                                         : (p.kind == KIND_GEMM ? rows : 0.0);
  if (p.kind == KIND_CONV1D || p.kind == KIND_CONVT) in_rows = (double)a.L_in * (a.M / (double)(p.kind == KIND_CONV1D ? a.L_out : a.L_in));
  const double out_rows = rows * (p.kind == KIND_CONVT ? p.ct_u : 1);
  const double bytes = es * (in_rows * p.cin + out_rows * p.cout * (1 + (a.res ? 1 : 0) + (a.accum ? 1 : 0)) +
                             (double)p.phases * p.cout * p.ntaps * p.cin);
  *flops_out = flops;
  *bytes_out = bytes;
}

template <typename T>
inline void run_conv(const ConvArgs& a, const PConv& p, hipStream_t s) {
  double flops, bytes;
  conv_cost<T>(a, p, &flops, &bytes);
  launch_conv<T>(a, s, flops, bytes);
}

// TF "SAME": out = ceil(in / s), total pad = max((out - 1) * s + k - in, 0), top/left = total / 2
inline void same_pad(int in, int k, int s, int* out, int* pad) {
  *out = (in + s - 1) / s;
  if (s == 1) {
    *pad = (k - 1) / 2;  // timm static padding for odd k, stride 1
  } else {
    int total = std::max((*out - 1) * s + k - in, 0);
    *pad = total / 2;
  }
}

constexpr int EFF_STEM = 32, EFF_OUT = 208;
constexpr int SE_RD_MAX = 64;  // SE reduce width of tf_efficientnetv2_b2 is <= 52 (chan_stride <= 64)
struct StageDef {
  int type, reps, k, stride, exp, cout;
  float se;
};
constexpr StageDef kStages[6] = {{0, 2, 3, 1, 1, 16, 0.f},   {1, 3, 3, 2, 4, 32, 0.f},
                                    {1, 3, 3, 2, 4, 56, 0.f},   {2, 4, 3, 2, 4, 104, 0.25f},
                                    {2, 6, 3, 1, 6, 120, 0.25f}, {2, 10, 3, 2, 6, 208, 0.25f}};
inline int make_divisible(double v, int d = 8) { return std::max(d, (int)(v + d / 2.0) / d * d); }

}  // namespace m2s
