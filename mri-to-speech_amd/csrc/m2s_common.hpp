// Shared device/host helpers for libm2s (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

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

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int VEC = 4;  // elements per 16-byte lane load
  static constexpr int KC = 16;  // K covered by one 16-byte load set (4 x mfma 16x16x4 f32)
  __device__ static __forceinline__ float to_f(float v) { return v; }
  __device__ static __forceinline__ float from_f(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int VEC = 8;
  static constexpr int KC = 32;  // one mfma 16x16x32 bf16
  __device__ static __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
  __device__ static __forceinline__ bf16_t from_f(float v) { return f2bf(v); }
};

// bf16-path activations: one v_exp_f32 + one v_rcp_f32 (1 ulp) instead of an IEEE divide and
// __expf's denormal-range fix-up (a compare + select + multiply per value); e^-x underflowing to
// 0 or overflowing to inf gives silu = x or -0 as the exact function does.  These run in every
// conv epilogue, where VALU issue, not the MFMA, bounds the small-K layers.
__device__ __forceinline__ float exp_neg(float x) { return __builtin_amdgcn_exp2f(x * -1.4426950408889634f); }
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + exp_neg(x)); }
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + exp_neg(x)); }

// Exact-libm variants used by the fp32 parity path (the reference runs fp32 libm on CPU).
__device__ __forceinline__ float silu_exact(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float sigmoid_exact(float x) { return 1.0f / (1.0f + expf(-x)); }

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int round_up(int a, int b) { return ceil_div(a, b) * b; }

// Channel stride of an activation tensor with C real channels: rows are padded so the
// implicit-GEMM K loop never splits a 16-byte lane load across taps.
inline int chan_stride(int c) { return c <= 16 ? round_up(c, 16) : round_up(c, 32); }

}  // namespace m2s
