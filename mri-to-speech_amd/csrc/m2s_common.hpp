// Shared device/host helpers for libm2s (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace m2s {

typedef uint16_t bf16_t;  // storage type of bf16 activations / weights
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define M2S_HIP(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      throw ::m2s::Error(2, std::string(#expr) + ": " + hipGetErrorString(e_) + " @" +       \
                                std::string(__FILE__) + ":" + std::to_string(__LINE__));     \
  } while (0)

#define M2S_CHECK(cond, msg)                                                                 \
  do {                                                                                       \
    if (!(cond)) throw ::m2s::Error(1, std::string(msg));                                    \
  } while (0)

// ---- scalar conversions ---------------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return *reinterpret_cast<bf16_t*>(&b);
}

// Two floats -> one dword of bf16 (lo = a): a single v_cvt_pk_bf16_f32 (RNE).
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}

// Split-fp32 ("bf16x3") storage: an fp32 value v is kept as the bf16 pair hi = bf16(v),
// lo = bf16(v - hi) (17 significant bits, relative error <= 2^-17), so a product of two such
// values is three exact bf16 MFMA terms hi*hi + hi*lo + lo*hi accumulated in fp32.  A channel-last
// tensor with channel stride cs stores every position as [hi: cs][lo: cs] bf16 (4 bytes per
// channel, the footprint of fp32): a DMA of the hi chunk and one of the lo chunk at +cs.
struct sp_t {
  uint16_t v;
};

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int VEC = 4;  // elements per 16-byte lane load
  static constexpr int KC = 16;  // K covered by one 16-byte load set (4 x mfma 16x16x4 f32)
  static constexpr int R = 1;    // planes per position
  __device__ static __forceinline__ float to_f(float v) { return v; }
  __device__ static __forceinline__ float from_f(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int VEC = 8;
  static constexpr int KC = 32;  // one mfma 16x16x32 bf16
  static constexpr int R = 1;
  __device__ static __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
  __device__ static __forceinline__ bf16_t from_f(float v) { return f2bf(v); }
};
template <> struct Elem<sp_t> {
  static constexpr int VEC = 8;
  static constexpr int KC = 32;
  static constexpr int R = 2;  // [hi cs][lo cs] per position
};

// Element access by (position p, channel c) for the three storage types.
template <typename T>
__device__ __forceinline__ float act_ld(const T* x, long p, int cs, int c) {
  if constexpr (Elem<T>::R == 2) {
    const uint16_t* u = reinterpret_cast<const uint16_t*>(x) + p * 2 * cs + c;
    return bf2f(u[0]) + bf2f(u[cs]);
  } else {
    return Elem<T>::to_f(x[p * cs + c]);
  }
}
template <typename T>
__device__ __forceinline__ void act_st(T* x, long p, int cs, int c, float v) {
  if constexpr (Elem<T>::R == 2) {
    uint16_t* u = reinterpret_cast<uint16_t*>(x) + p * 2 * cs + c;
    const bf16_t h = f2bf(v);
    u[0] = h;
    u[cs] = f2bf(v - bf2f(h));
  } else {
    x[p * cs + c] = Elem<T>::from_f(v);
  }
}

// 4 / 8 consecutive channels (c % 4 == 0 / c % 8 == 0) of one position, vectorised.
__device__ __forceinline__ void unpack_bf16x4(uint2 u, float* v) {
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xffff0000u);
}
template <typename T>
__device__ __forceinline__ void act_ld4(const T* x, long p, int cs, int c, float* v) {
  if constexpr (std::is_same<T, float>::value) {
    const float4 f = *reinterpret_cast<const float4*>(x + p * cs + c);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  } else if constexpr (Elem<T>::R == 1) {
    unpack_bf16x4(*reinterpret_cast<const uint2*>(x + p * cs + c), v);
  } else {
    const uint16_t* u = reinterpret_cast<const uint16_t*>(x) + p * 2 * cs + c;
    float l[4];
    unpack_bf16x4(*reinterpret_cast<const uint2*>(u), v);
    unpack_bf16x4(*reinterpret_cast<const uint2*>(u + cs), l);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += l[j];
  }
}
// split of 4 values: hi = bf16(v), lo = bf16(v - hi), each as 4 packed bf16
__device__ __forceinline__ void split4(const float* v, uint2& hi, uint2& lo) {
  hi.x = pack_bf16x2(v[0], v[1]);
  hi.y = pack_bf16x2(v[2], v[3]);
  float h[4];
  unpack_bf16x4(hi, h);
  lo.x = pack_bf16x2(v[0] - h[0], v[1] - h[1]);
  lo.y = pack_bf16x2(v[2] - h[2], v[3] - h[3]);
}
template <typename T>
__device__ __forceinline__ void act_st4(T* x, long p, int cs, int c, const float* v) {
  if constexpr (std::is_same<T, float>::value) {
    *reinterpret_cast<float4*>(x + p * cs + c) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (Elem<T>::R == 1) {
    *reinterpret_cast<uint2*>(x + p * cs + c) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  } else {
    uint16_t* u = reinterpret_cast<uint16_t*>(x) + p * 2 * cs + c;
    uint2 hi, lo;
    split4(v, hi, lo);
    *reinterpret_cast<uint2*>(u) = hi;
    *reinterpret_cast<uint2*>(u + cs) = lo;
  }
}
template <typename T>
__device__ __forceinline__ void act_ld8(const T* x, long p, int cs, int c, float* v) {
  act_ld4<T>(x, p, cs, c, v);
  act_ld4<T>(x, p, cs, c + 4, v + 4);
}
template <typename T>
__device__ __forceinline__ void act_st8(T* x, long p, int cs, int c, const float* v) {
  if constexpr (Elem<T>::R == 2) {  // split: one 16-byte store for the 8 hi halves, one for the lo
    uint16_t* u = reinterpret_cast<uint16_t*>(x) + p * 2 * cs + c;
    uint2 h0, l0, h1, l1;
    split4(v, h0, l0);
    split4(v + 4, h1, l1);
    *reinterpret_cast<uint4*>(u) = make_uint4(h0.x, h0.y, h1.x, h1.y);
    *reinterpret_cast<uint4*>(u + cs) = make_uint4(l0.x, l0.y, l1.x, l1.y);
  } else {
    act_st4<T>(x, p, cs, c, v);
    act_st4<T>(x, p, cs, c + 4, v + 4);
  }
}

// Interleaved split layout ("sp32") of the IR blocks' depthwise output, the operand of the SE-gated
// conv_pwl GEMM (conv_gemm.hip, IN_SE_SCALE with SP = 1): per position and 32-channel group, [hi 32 | lo 32]
// bf16 (cs % 32 == 0, same footprint as sp_t), so one 32-channel K step of the GEMM reads one 128-byte line
// per row instead of two half lines (hi at c, lo at cs + c).
__device__ __forceinline__ uint16_t* il_addr(sp_t* x, long p, int cs, int c) {
  return reinterpret_cast<uint16_t*>(x) + p * 2 * cs + (c & ~31) * 2 + (c & 31);
}
__device__ __forceinline__ void il_st4(sp_t* x, long p, int cs, int c, const float* v) {  // c % 4 == 0
  uint16_t* u = il_addr(x, p, cs, c);
  uint2 hi, lo;
  split4(v, hi, lo);
  *reinterpret_cast<uint2*>(u) = hi;
  *reinterpret_cast<uint2*>(u + 32) = lo;
}
__device__ __forceinline__ void il_st8(sp_t* x, long p, int cs, int c, const float* v) {  // c % 8 == 0
  uint16_t* u = il_addr(x, p, cs, c);
  uint2 h0, l0, h1, l1;
  split4(v, h0, l0);
  split4(v + 4, h1, l1);
  *reinterpret_cast<uint4*>(u) = make_uint4(h0.x, h0.y, h1.x, h1.y);
  *reinterpret_cast<uint4*>(u + 32) = make_uint4(l0.x, l0.y, l1.x, l1.y);
}

// OCP e4m3fn storage (fp8 engines): 8 floats -> 8 bytes (v_cvt_pk_fp8_f32, round to nearest even),
// finite values saturated to +-448 (the conversion has no saturating mode), NaN kept
__device__ __forceinline__ float sat_e4m3(float x) { return x != x ? x : fminf(fmaxf(x, -448.f), 448.f); }
__device__ __forceinline__ uint2 e4m3x8(const float* v) {
  int q[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(v[4 * h]), sat_e4m3(v[4 * h + 1]), 0, false);
    q[h] = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(v[4 * h + 2]), sat_e4m3(v[4 * h + 3]), r, true);
  }
  return make_uint2((uint32_t)q[0], (uint32_t)q[1]);
}

// 8 values already within +-448 (or NaN: kept) -> 8 e4m3
__device__ __forceinline__ uint2 e4m3x8_nosat(const float* v) {
  int q[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * h], v[4 * h + 1], 0, false);
    q[h] = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * h + 2], v[4 * h + 3], r, true);
  }
  return make_uint2((uint32_t)q[0], (uint32_t)q[1]);
}

// 4 bf16 (a uint2 as stored) -> 4 e4m3 (saturated as sat_e4m3: NaN kept), the same bytes er8_fused's own
// conversion of a bf16 operand gives
__device__ __forceinline__ uint32_t e4m3x4_bf16(uint2 u) {
  const int r = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(__uint_as_float(u.x << 16)),
                                                sat_e4m3(__uint_as_float(u.x & 0xffff0000u)), 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(__uint_as_float(u.y << 16)),
                                                   sat_e4m3(__uint_as_float(u.y & 0xffff0000u)), r, true);
}

// bf16-path activations: one v_exp_f32 + one v_rcp_f32 (1 ulp) instead of an IEEE divide and
// __expf's denormal-range fix-up (a compare + select + multiply per value); e^-x underflowing to
// 0 or overflowing to inf gives silu = x or -0 as the exact function does.  These run in every
// conv epilogue, where VALU issue, not the MFMA, bounds the small-K layers.
__device__ __forceinline__ float exp_neg(float x) { return __builtin_amdgcn_exp2f(x * -1.4426950408889634f); }
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + exp_neg(x)); }
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + exp_neg(x)); }
// SiLU saturated for e4m3 (SiLU >= -0.28, so only the top needs the clamp): min(x, 448) * sigmoid(x), where a
// NaN x still yields NaN through the sigmoid factor, so e4m3x8_nosat needs no NaN test (sat_e4m3's two ops)
__device__ __forceinline__ float silu_e4m3(float x) { return fminf(x, 448.f) * __builtin_amdgcn_rcpf(1.0f + exp_neg(x)); }

// Exact-libm variants used by the fp32 parity path (the reference runs fp32 libm on CPU).
__device__ __forceinline__ float silu_exact(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float sigmoid_exact(float x) { return 1.0f / (1.0f + expf(-x)); }

// Per-device launch attributes (device_attr.cpp), cached per (device[, kernel]) so engines on
// different devices in one process each get their own: the current device's CU count, the 160 KB
// dynamic-LDS opt-in of `kernel` on the current device, and how many workgroups of `kernel` (block
// threads, dynamic LDS) the current device holds at once.
int device_cus();
void allow_lds(const void* kernel);
int device_resident(const void* kernel, int block, size_t lds);

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int round_up(int a, int b) { return ceil_div(a, b) * b; }

// Channel stride of an activation tensor with C real channels: rows are padded so the
// implicit-GEMM K loop never splits a 16-byte lane load across taps.
inline int chan_stride(int c) { return c <= 16 ? round_up(c, 16) : round_up(c, 32); }

}  // namespace m2s
