// Implicit-GEMM convolution kernels (see conv_igemm.hpp for the contract).
//
// Tiling: a 256-thread workgroup = 4 waves stacked along M (output positions); each wave owns
// an (NT*16 channels) x (MT*16 positions) tile of 16x16 MFMA accumulators.  Per K chunk each
// lane issues one 16-byte load per M subtile (8 bf16 / 4 f32 input channels of one position
// at one tap, zero for padding) and one per N subtile (packed weight row), then
// NT*MT MFMAs (f32: 4 x v_mfma_f32_16x16x4_f32, exact f32).  Only the exact-f32 path (M2S_DT_F32)
// instantiates it; bf16 and split fp32 run the LDS-DMA pipeline of conv_gemm.hip.
#include "conv_igemm.hpp"

#include "prof.hpp"

namespace m2s {

namespace {

template <typename T>
__device__ __forceinline__ void xform_lrelu(uint4& v, float slope) {
  if constexpr (sizeof(T) == 4) {
    float* f = reinterpret_cast<float*>(&v);
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = f[e] > 0.f ? f[e] : f[e] * slope;
  } else {
    bf16_t* h = reinterpret_cast<bf16_t*>(&v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float f = bf2f(h[e]);
      h[e] = f > 0.f ? h[e] : f2bf(f * slope);
    }
  }
}

template <typename T>
__device__ __forceinline__ void xform_scale(uint4& v, const T* __restrict__ s) {
  if constexpr (sizeof(T) == 4) {
    float* f = reinterpret_cast<float*>(&v);
    const float4 sc = *reinterpret_cast<const float4*>(s);
    f[0] *= sc.x; f[1] *= sc.y; f[2] *= sc.z; f[3] *= sc.w;
  } else {
    bf16_t* h = reinterpret_cast<bf16_t*>(&v);
    const uint4 su = *reinterpret_cast<const uint4*>(s);
    const bf16_t* sc = reinterpret_cast<const bf16_t*>(&su);
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = f2bf(bf2f(h[e]) * bf2f(sc[e]));
  }
}

template <typename T>
__device__ __forceinline__ void mfma_step(f32x4& acc, const uint4& a, const uint4& b) {
  if constexpr (sizeof(T) == 4) {
    const float* fa = reinterpret_cast<const float*>(&a);
    const float* fb = reinterpret_cast<const float*>(&b);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[e], fb[e], acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                  acc, 0, 0, 0);
  }
}

template <typename T>
__device__ __forceinline__ float act_apply(float v, int act, float slope) {
  if (act == ACT_SILU) return sizeof(T) == 4 ? silu_exact(v) : silu(v);
  if (act == ACT_LRELU) return v > 0.f ? v : v * slope;
  if (act == ACT_SIGMOID) return sizeof(T) == 4 ? sigmoid_exact(v) : sigmoidf_(v);
  return v;
}

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* v) {
  if constexpr (sizeof(T) == 4) {
    float4 f = *reinterpret_cast<const float4*>(p);
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
  } else {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
}

template <typename T>
__device__ __forceinline__ void store4(T* p, const float* v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  }
}

template <typename T, int MT, int NT, int KIND>
__global__ void __launch_bounds__(256) conv_igemm_kernel(const ConvArgs a) {
  constexpr int VEC = Elem<T>::VEC;
  constexpr int KC = Elem<T>::KC;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // kw (ConvArgs::kwave): the four waves take the same MT x 16 rows and split the K chunks (chunk i to wave i % 4),
  // adding their partial sums in LDS in a fixed order.  For the BiLSTM input projection of a small pass (M = 30
  // frames) one wave walking 88 chunks x 32 MFMAs alone, three idle, was a 20 us launch on 80 workgroups.
  const bool kw = a.kwave != 0;
  const int m_base = kw ? blockIdx.x * (MT * 16) : (blockIdx.x * 4 + wave) * (MT * 16);
  const int n_base = blockIdx.y * (NT * 16);
  const int phase = blockIdx.z;
  if (m_base >= a.M) return;

  const T* __restrict__ X = static_cast<const T*>(a.x);
  const T* __restrict__ W = static_cast<const T*>(a.w) + (size_t)phase * a.n_pad * a.kp;

  // ---- per-row (output position) state, computed once -------------------------------------
  int rb[MT], rp0[MT], rp1[MT];
  bool rok[MT];
  const int delta = (KIND == KIND_CONVT) ? (phase + a.ct_pad) / a.ct_u : 0;
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m_base + mi * 16 + r16;
    rok[mi] = m < a.M;
    const int mm = rok[mi] ? m : 0;
    if constexpr (KIND == KIND_CONV2D) {
      const int hw = a.OH * a.OW;
      const int img = mm / hw;
      const int rem = mm - img * hw;
      const int oy = rem / a.OW;
      const int ox = rem - oy * a.OW;
      rb[mi] = img;
      rp0[mi] = oy * a.stride - a.pad_t;
      rp1[mi] = ox * a.stride - a.pad_l;
    } else if constexpr (KIND == KIND_CONV1D) {
      const int b = mm / a.L_out;
      rb[mi] = b;
      rp0[mi] = mm - b * a.L_out - a.pad_left;
      rp1[mi] = 0;
    } else if constexpr (KIND == KIND_CONVT) {
      const int b = mm / a.L_in;
      rb[mi] = b;
      rp0[mi] = mm - b * a.L_in + delta;
      rp1[mi] = mm - b * a.L_in;  // q
    } else {
      rb[mi] = mm / a.OH;  // KIND_GEMM: OH = rows per image (SE scale row)
      rp0[mi] = mm;
      rp1[mi] = 0;
    }
  }

  f32x4 acc[NT][MT];
#pragma unroll
  for (int ni = 0; ni < NT; ++ni)
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool multi_tap = a.tpc > 1;
  const int tap_off = multi_tap ? (g * VEC) / a.cs_in : 0;
  const int c_off = multi_tap ? (g * VEC) % a.cs_in : g * VEC;
  const int cchunks = multi_tap ? 1 : a.cs_in / KC;
  const uint4 zero4 = make_uint4(0, 0, 0, 0);

  int it = 0;  // K chunk counter (kw)
  for (int tap0 = 0; tap0 < a.ntaps; tap0 += a.tpc) {
    const int tap = tap0 + tap_off;
    long xo[MT];
    int img_row[MT];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      long off = -1;
      img_row[mi] = rb[mi];
      if (rok[mi] && tap < a.ntaps) {
        if constexpr (KIND == KIND_CONV2D) {
          const int ky = tap / a.ks;
          const int kx = tap - ky * a.ks;
          const int iy = rp0[mi] + ky, ix = rp1[mi] + kx;
          if (iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW)
            off = ((long)(rb[mi] * a.IH + iy) * a.IW + ix) * a.cs_in;
        } else if constexpr (KIND == KIND_CONV1D) {
          const int it = rp0[mi] + tap * a.dil;
          if (it >= 0 && it < a.L_in) off = ((long)rb[mi] * a.L_in + it) * a.cs_in;
        } else if constexpr (KIND == KIND_CONVT) {
          const int it = rp0[mi] - tap;
          if (it >= 0 && it < a.L_in) off = ((long)rb[mi] * a.L_in + it) * a.cs_in;
        } else {
          off = (long)rp0[mi] * a.cs_in;
        }
      }
      xo[mi] = off;
    }
    const T* wrow[NT];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
      wrow[ni] = W + (size_t)(n_base + ni * 16 + r16) * a.kp + (size_t)tap * a.cs_in + c_off;

    for (int cc = 0; cc < cchunks; ++cc) {
      const bool mine = !kw || (it & 3) == wave;
      ++it;
      if (!mine) continue;
      uint4 bx[MT], aw[NT];
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        bx[mi] = xo[mi] >= 0 ? *reinterpret_cast<const uint4*>(X + xo[mi] + c_off + cc * KC) : zero4;
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) aw[ni] = *reinterpret_cast<const uint4*>(wrow[ni] + cc * KC);
      if (a.in_xform == IN_LRELU) {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) xform_lrelu<T>(bx[mi], a.in_slope);
      } else if (a.in_xform == IN_SE_SCALE) {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
          if (xo[mi] >= 0)
            xform_scale<T>(bx[mi], static_cast<const T*>(a.in_scale) + (size_t)img_row[mi] * a.cs_in + c_off + cc * KC);
      }
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) mfma_step<T>(acc[ni][mi], aw[ni], bx[mi]);
    }
  }

  if (kw) {  // waves 1-3 hand their partial sums to wave 0: ((w0 + w1) + (w2 + w3))
    extern __shared__ __attribute__((aligned(16))) char kw_lds[];
    f32x4* red = reinterpret_cast<f32x4*>(kw_lds);  // [3][NT * MT][64]
    if (wave > 0)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) red[((wave - 1) * NT * MT + ni * MT + mi) * 64 + lane] = acc[ni][mi];
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int i = ni * MT + mi;
        acc[ni][mi] = (acc[ni][mi] + red[i * 64 + lane]) + (red[(NT * MT + i) * 64 + lane] + red[(2 * NT * MT + i) * 64 + lane]);
      }
  }

  // ---- epilogue: bias, activation, residual, MRF accumulation; 4 channels per lane ----------
  T* __restrict__ Y = static_cast<T*>(a.y);
  const T* __restrict__ R = static_cast<const T*>(a.res);
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    if (!rok[mi]) continue;
    const int m = m_base + mi * 16 + r16;
    long orow;
    if constexpr (KIND == KIND_CONVT)
      orow = ((long)rb[mi] * a.L_out + (long)rp1[mi] * a.ct_u + phase) * a.cs_out;
    else
      orow = (long)m * a.cs_out;
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int n4 = n_base + ni * 16 + 4 * g;
      if (n4 >= a.cs_out) continue;
      const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
      float v[4] = {acc[ni][mi][0] + bb.x, acc[ni][mi][1] + bb.y, acc[ni][mi][2] + bb.z, acc[ni][mi][3] + bb.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = act_apply<T>(v[j], a.act, a.act_slope);
      if (R) {
        float r[4];
        load4<T>(R + orow + n4, r);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += r[j];
      }
      if (a.accum) {
        float p[4];
        load4<T>(Y + orow + n4, p);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = p[j] + v[j];
        if (a.accum == 2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = v[j] / a.accum_div;
        }
      }
      store4<T>(Y + orow + n4, v);
    }
  }
}


template <typename T, int MT, int NT, int KIND>
void launch_tile(const ConvArgs& a, hipStream_t s, int phases, double flops, double bytes) {
  dim3 grid(ceil_div(a.M, (a.kwave ? 1 : 4) * MT * 16), ceil_div(a.cs_out, NT * 16), phases);
  M2S_CHECK(grid.y * NT * 16 <= a.n_pad, "conv: weight rows not padded to the N tile");
  char name[96];
  snprintf(name, sizeof(name), "conv_igemm_kernel<%s, %d, %d, %d>", sizeof(T) == 4 ? "float" : "unsigned short", MT, NT, KIND);
  ProfScope ps(name, flops, bytes, s);
  const size_t lds = a.kwave ? (size_t)3 * NT * MT * 64 * sizeof(f32x4) : 0;  // the kernel's kw reduction
  hipLaunchKernelGGL((conv_igemm_kernel<T, MT, NT, KIND>), grid, dim3(256), lds, s, a);
}

template <typename T, int KIND>
void launch_kind(const ConvArgs& a, hipStream_t s, int phases, double flops, double bytes) {
  if (a.kwave && a.cs_out > 32)  // K split over the waves: 16-column tiles spread the N dimension over more workgroups
    return launch_tile<T, 2, 1, KIND>(a, s, phases, flops, bytes);
  if (a.cs_out <= 16)
    launch_tile<T, 4, 1, KIND>(a, s, phases, flops, bytes);
  else if (a.cs_out <= 32)
    launch_tile<T, 4, 2, KIND>(a, s, phases, flops, bytes);
  else
    launch_tile<T, 2, 4, KIND>(a, s, phases, flops, bytes);
}

}  // namespace

template <typename T>
void launch_conv(const ConvArgs& a, hipStream_t s, double flops, double bytes) {
  if constexpr (!std::is_same<T, float>::value) {  // bf16 / split fp32: LDS-DMA pipeline (conv_gemm.hip)
    M2S_CHECK(a.kind != KIND_CONV2D || a.ks == 3, "conv: bf16 / split 2-D convs are 3x3");
    launch_conv_gemm(a, std::is_same<T, sp_t>::value, s, flops, bytes);
  } else {  // exact f32 products: the direct-load kernel of this file
    constexpr int KC = Elem<T>::KC;
    M2S_CHECK(a.cs_in % KC == 0 || KC % a.cs_in == 0, "conv: cs_in incompatible with K chunk");
    M2S_CHECK(a.cs_out % 4 == 0, "conv: cs_out must be a multiple of 4");
    M2S_CHECK(a.tpc == conv_tpc(a.cs_in, KC), "conv: tpc mismatch");
    M2S_CHECK(a.kp == conv_kp(a.ntaps, a.cs_in, KC), "conv: kp mismatch");
    if (a.M <= 0) return;
    switch (a.kind) {
      case KIND_CONV2D: launch_kind<T, KIND_CONV2D>(a, s, 1, flops, bytes); break;
      case KIND_CONV1D: launch_kind<T, KIND_CONV1D>(a, s, 1, flops, bytes); break;
      case KIND_CONVT: launch_kind<T, KIND_CONVT>(a, s, a.ct_u, flops, bytes); break;
      case KIND_GEMM: launch_kind<T, KIND_GEMM>(a, s, 1, flops, bytes); break;
      default: M2S_CHECK(false, "conv: bad kind");
    }
    M2S_HIP(hipGetLastError());
  }
}

template void launch_conv<float>(const ConvArgs&, hipStream_t, double, double);
template void launch_conv<bf16_t>(const ConvArgs&, hipStream_t, double, double);
template void launch_conv<sp_t>(const ConvArgs&, hipStream_t, double, double);

}  // namespace m2s
