// InvertedResidual middle: depthwise 3x3 + BN + SiLU with the SE squeeze (timm conv_dw / bn2 /
// se.*; mri_acoustic_model.py:28-34 builds them).  The SE excitation itself (conv_reduce -> SiLU
// -> conv_expand -> sigmoid over all images at once) runs as two GEMMs on MFMA (model.cpp); this
// file provides the depthwise conv and the squeeze (channel means) that feeds them.
#include "kernels.hpp"

namespace m2s {
namespace {

template <typename T>
__device__ __forceinline__ float silu_t(float v) {
  return sizeof(T) == 4 ? silu_exact(v) : silu(v);
}

// ---------------------------------------------------------------------------------------------
// Depthwise.  Workgroup = 256 channels (512 contiguous bytes of every pixel row in bf16) x
// DW_PIX output pixels: DW_PIX / P whole images when an image is smaller, else one pixel block of
// one image.  grid (ceil(cs/256), image groups, pixel blocks).  Thread = 8 channels (one 16-byte
// vector) x every 8th pixel; the 9 tap loads of a pixel are issued together.  The 256x9 folded
// weights are staged once per workgroup in LDS.  SE partial sums per (image, pixel block,
// channel): each thread flushes its 8 sums to LDS when its image changes; the 8 pixel lanes are
// then added in a fixed order -> psum[n][pb][cs] (deterministic).
constexpr int DW_PIX = 256;
constexpr int DW_MAXG = DW_PIX / 64;  // images per workgroup at most (grouping needs P >= 64)
// channels per workgroup: 64, or 32 for split storage, whose lo half starts cs * 2 bytes into the row -
// with cs = 224 that is 64 B off a 128-byte line, so a 64-channel (128 B) lo read touched two lines
// (PMC: 1.64x the input bytes fetched); 32 channels = 64 B pieces that never cross a line
template <typename T>
constexpr int dw_cb() {
  return Elem<T>::R == 2 ? 32 : 64;
}

template <typename T, int S>
__global__ void __launch_bounds__(256) dwconv_kernel(const T* __restrict__ x, int N, int IH, int IW, int OH, int OW,
                                                     int pad_t, int pad_l, int cs, int G,
                                                     const float* __restrict__ w9, const float* __restrict__ bias,
                                                     T* __restrict__ y, float* __restrict__ psum) {
  constexpr int DW_CB = dw_cb<T>(), DW_PL = 256 / (DW_CB / 8);
  __shared__ float red[DW_MAXG][DW_PL][DW_CB + 1];
  __shared__ __attribute__((aligned(16))) float wsm[10][DW_CB];  // 9 taps + bias
  const int cg = threadIdx.x % (DW_CB / 8), pl = threadIdx.x / (DW_CB / 8);
  // XCD-aware work order: the hardware deals linear block ids round-robin over the 8 XCDs, so consecutive ids
  // of one image's channel slices landed on different L2s; a slice is 32 channels = 64 B of a 128-byte line
  // at split cs = 224, whose other half belongs to the neighbouring slice, and every L2 fetched the whole
  // line (PMC: 2.1x the input bytes).  Here the slices (and pixel blocks) of one image share an XCD.
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xq = nwg / 8, xr = nwg % 8, xcd = lin % 8;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + lin / 8;
  const int bx = wid % gridDim.x, byz = wid / gridDim.x, by = byz % gridDim.y, bz = byz / gridDim.y;
  const int cb = bx * DW_CB;
  const int c0 = cb + cg * 8;
  const int P = OH * OW;
  const int n0 = by * G, pb = bz;
  for (int i = threadIdx.x; i < 10 * DW_CB; i += 256) {
    const int t = i / DW_CB, c = cb + (i % DW_CB);
    wsm[t][i % DW_CB] = c < cs ? (t < 9 ? w9[(long)t * cs + c] : bias[c]) : 0.f;
  }
  for (int i = threadIdx.x; i < G * DW_PL * DW_CB; i += 256)
    red[i / (DW_PL * DW_CB)][(i / DW_CB) % DW_PL][i % DW_CB] = 0.f;
  __syncthreads();
  if (c0 < cs) {
    float w[9][8], b[8];
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      const float4 lo = *reinterpret_cast<const float4*>(&wsm[t][cg * 8]);
      const float4 hi = *reinterpret_cast<const float4*>(&wsm[t][cg * 8 + 4]);
      float* d = t < 9 ? w[t] : b;
      d[0] = lo.x; d[1] = lo.y; d[2] = lo.z; d[3] = lo.w;
      d[4] = hi.x; d[5] = hi.y; d[6] = hi.z; d[7] = hi.w;
    }
    const int npix = G > 1 ? G * P : min(DW_PIX, P - pb * DW_PIX);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int g_cur = 0;
    for (int lp = pl; lp < npix; lp += DW_PL) {
      const int g = G > 1 ? lp / P : 0;
      const int p = G > 1 ? lp - g * P : pb * DW_PIX + lp;
      const int n = n0 + g;
      if (n >= N) break;
      if (g != g_cur) {  // flush the previous image's partial sums
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red[g_cur][pl][cg * 8 + j] = s[j];
          s[j] = 0.f;
        }
        g_cur = g;
      }
      constexpr int R = Elem<T>::R;
      const T* xn = x + (long)n * IH * IW * cs * R + c0;
      const int oy = p / OW, ox = p - (p / OW) * OW;
      uint4 in[9], inl[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int iy = oy * S - pad_t + t / 3, ix = ox * S - pad_l + t % 3;
        const bool ok = iy >= 0 && iy < IH && ix >= 0 && ix < IW;
        in[t] = ok ? *reinterpret_cast<const uint4*>(xn + ((long)iy * IW + ix) * cs * R) : make_uint4(0, 0, 0, 0);
        if constexpr (R == 2)  // split storage: the lo half of the same 8 channels, cs elements on
          inl[t] = ok ? *reinterpret_cast<const uint4*>(xn + ((long)iy * IW + ix) * cs * R + cs) : make_uint4(0, 0, 0, 0);
      }
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = b[j];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        float v[8];
        if constexpr (sizeof(T) == 4) {
          // fp32: 8 channels span two 16-byte vectors; in[] holds the first, load the second
          const float* f = reinterpret_cast<const float*>(&in[t]);
          const int iy = oy * S - pad_t + t / 3, ix = ox * S - pad_l + t % 3;
          const bool ok = iy >= 0 && iy < IH && ix >= 0 && ix < IW;
          const float4 hi = ok ? *reinterpret_cast<const float4*>(xn + ((long)iy * IW + ix) * cs + 4)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
          v[0] = f[0]; v[1] = f[1]; v[2] = f[2]; v[3] = f[3];
          v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        } else {
          const uint32_t u[4] = {in[t].x, in[t].y, in[t].z, in[t].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[2 * j] = __uint_as_float(u[j] << 16);
            v[2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u);
          }
          if constexpr (R == 2) {
            const uint32_t l[4] = {inl[t].x, inl[t].y, inl[t].z, inl[t].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[2 * j] += __uint_as_float(l[j] << 16);
              v[2 * j + 1] += __uint_as_float(l[j] & 0xffff0000u);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += w[t][j] * v[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j] = silu_t<T>(acc[j]);
        s[j] += acc[j];
      }
      T* o = y + ((long)n * P + p) * cs + c0;
      if constexpr (R == 2) {  // split: the SE GEMM's interleaved operand (m2s_common.hpp il_st8)
        il_st8(reinterpret_cast<sp_t*>(y), (long)n * P + p, cs, c0, acc);
      } else if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      } else {
        uint4 u;
        u.x = (uint32_t)f2bf(acc[0]) | ((uint32_t)f2bf(acc[1]) << 16);
        u.y = (uint32_t)f2bf(acc[2]) | ((uint32_t)f2bf(acc[3]) << 16);
        u.z = (uint32_t)f2bf(acc[4]) | ((uint32_t)f2bf(acc[5]) << 16);
        u.w = (uint32_t)f2bf(acc[6]) | ((uint32_t)f2bf(acc[7]) << 16);
        *reinterpret_cast<uint4*>(o) = u;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[g_cur][pl][cg * 8 + j] = s[j];
  }
  __syncthreads();
  const int npb = gridDim.z;  // (pb = bz above)
  for (int i = threadIdx.x; i < G * DW_CB; i += 256) {
    const int g = i / DW_CB, cl = i % DW_CB, c = cb + cl;
    if (c >= cs || n0 + g >= N) continue;
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < DW_PL; ++r) t += red[g][r][cl];
    psum[((long)(n0 + g) * npb + pb) * cs + c] = t;
  }
}

// SE squeeze: mean[n][c] = (sum over pixel blocks of psum) / P, in the compute dtype (the A
// operand of the conv_reduce GEMM).  Pad channels carry zeros (their depthwise output is 0).
template <typename T>
__global__ void __launch_bounds__(256) se_mean_kernel(const float* __restrict__ psum, int N, int npb, int cs,
                                                      float inv_count, T* __restrict__ mean) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * cs) return;
  const long n = i / cs;
  const int c = (int)(i - n * cs);
  float acc = 0.f;
  for (int q = 0; q < npb; ++q) acc += psum[(n * npb + q) * cs + c];
  act_st<T>(mean, n, cs, c, acc * inv_count);
}

int dw_group(int OH, int OW) {
  const int P = OH * OW;
  return P >= DW_PIX || P < 64 ? 1 : DW_PIX / P;
}

}  // namespace

int dw_pixel_blocks(int OH, int OW) { return dw_group(OH, OW) > 1 ? 1 : (OH * OW + DW_PIX - 1) / DW_PIX; }

template <typename T>
void launch_dwconv(const T* x, int N, int IH, int IW, int OH, int OW, int stride, int pad_t, int pad_l, int C, int cs,
                   const float* w9, const float* bias, T* y, float* sums, hipStream_t s) {
  (void)C;
  M2S_CHECK(cs % 8 == 0, "dwconv: cs % 8");
  M2S_CHECK(stride == 1 || stride == 2, "dwconv: stride");
  const int G = dw_group(OH, OW);
  const dim3 grid(ceil_div(cs, dw_cb<T>()), ceil_div(N, G), dw_pixel_blocks(OH, OW));
  if (stride == 1)
    hipLaunchKernelGGL((dwconv_kernel<T, 1>), grid, dim3(256), 0, s, x, N, IH, IW, OH, OW, pad_t, pad_l, cs, G, w9,
                       bias, y, sums);
  else
    hipLaunchKernelGGL((dwconv_kernel<T, 2>), grid, dim3(256), 0, s, x, N, IH, IW, OH, OW, pad_t, pad_l, cs, G, w9,
                       bias, y, sums);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_se_mean(const float* psum, int N, int npb, int cs, float inv_count, T* mean, hipStream_t s) {
  hipLaunchKernelGGL(se_mean_kernel<T>, dim3(ceil_div(N * cs, 256)), dim3(256), 0, s, psum, N, npb, cs, inv_count,
                     mean);
  M2S_HIP(hipGetLastError());
}

template void launch_dwconv<float>(const float*, int, int, int, int, int, int, int, int, int, int, const float*,
                                   const float*, float*, float*, hipStream_t);
template void launch_dwconv<bf16_t>(const bf16_t*, int, int, int, int, int, int, int, int, int, int, const float*,
                                    const float*, bf16_t*, float*, hipStream_t);
template void launch_se_mean<float>(const float*, int, int, int, float, float*, hipStream_t);
template void launch_se_mean<bf16_t>(const float*, int, int, int, float, bf16_t*, hipStream_t);
template void launch_dwconv<sp_t>(const sp_t*, int, int, int, int, int, int, int, int, int, int, const float*,
                                  const float*, sp_t*, float*, hipStream_t);
template void launch_se_mean<sp_t>(const float*, int, int, int, float, sp_t*, hipStream_t);

}  // namespace m2s
