// Frame preprocessing on the device: decoded uint8 frames -> the [0, 1] fp32 frames the acoustic
// model consumes.  Restates scripts/run_mri_video_inference.py:34-54 (_preprocess_frame) after
// the host decode: BGR -> grey (cv2.COLOR_BGR2GRAY's 8-bit fixed point: (1868 B + 9617 G +
// 4899 R + 2^13) >> 14), per-frame z-score (numpy mean / population std), then min-max to [0, 1]
// (zeros when the frame is constant).  Resizing stays on the host (cv2.resize), so H x W here is
// already the model's input size.
//
// One 1024-thread workgroup per frame, two passes over the frame's bytes (L2-resident between
// them): pass 1 reduces sum, sum of squares, min and max of the grey values in integers (exact);
// pass 2 writes ((g - mean) / std - zmin) / (zmax - zmin) with the reference's float32 operation
// order.  mean = sum / n is exact in float32 while sum < 2^24 (256 x 256 frames), like numpy's
// float32 pairwise sum; std is computed in double and rounded, so outputs differ from numpy by
// rounding only (the min-max step cancels std mathematically).  HBM-bound: n (or 3n) bytes in,
// 4n bytes out per frame.
#include "kernels.hpp"

namespace m2s {
namespace {

constexpr int PP_THREADS = 1024;

__device__ __forceinline__ int grey_at(const uint8_t* f, long p, int ch) {
  if (ch == 1) return f[p];
  const uint8_t* q = f + 3 * p;  // B, G, R
  return (1868 * q[0] + 9617 * q[1] + 4899 * q[2] + (1 << 13)) >> 14;
}

__global__ void __launch_bounds__(PP_THREADS) preprocess_kernel(const uint8_t* __restrict__ frames, int HW, int ch,
                                                                float* __restrict__ out) {
  __shared__ unsigned long long s_sum[PP_THREADS / 64], s_sq[PP_THREADS / 64];
  __shared__ int s_min[PP_THREADS / 64], s_max[PP_THREADS / 64];
  __shared__ float s_par[4];
  const uint8_t* f = frames + (size_t)blockIdx.x * HW * ch;
  float* o = out + (size_t)blockIdx.x * HW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  unsigned long long sum = 0, sq = 0;
  int mn = 255, mx = 0;
  // grey frames of whole dwords: 4 pixels a load (one-byte loads made a small batch's pass latency-bound)
  const bool v4 = ch == 1 && (HW & 3) == 0 && ((uintptr_t)f & 3) == 0;
  if (v4) {
    for (long p = tid; p < HW / 4; p += PP_THREADS) {
      const uint32_t w = reinterpret_cast<const uint32_t*>(f)[p];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int g = (w >> (8 * j)) & 255;
        sum += g;
        sq += (unsigned)(g * g);
        mn = min(mn, g);
        mx = max(mx, g);
      }
    }
  } else {
    for (long p = tid; p < HW; p += PP_THREADS) {
      const int g = grey_at(f, p, ch);
      sum += g;
      sq += (unsigned)(g * g);
      mn = min(mn, g);
      mx = max(mx, g);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    sum += __shfl_xor(sum, m);
    sq += __shfl_xor(sq, m);
    mn = min(mn, __shfl_xor(mn, m));
    mx = max(mx, __shfl_xor(mx, m));
  }
  if (lane == 0) {
    s_sum[wave] = sum;
    s_sq[wave] = sq;
    s_min[wave] = mn;
    s_max[wave] = mx;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned long long S = 0, Q = 0;
    int lo = 255, hi = 0;
    for (int w = 0; w < PP_THREADS / 64; ++w) {
      S += s_sum[w];
      Q += s_sq[w];
      lo = min(lo, s_min[w]);
      hi = max(hi, s_max[w]);
    }
    const double n = (double)HW;
    const float mean = (float)((double)S / n);
    const double var = ((double)Q - (double)S * (double)S / n) / n;
    const float sd = (float)sqrt(var > 0.0 ? var : 0.0);
    float zlo, zhi;
    {
#pragma clang fp contract(off)
      zlo = sd > 0.f ? ((float)lo - mean) / sd : (float)lo - mean;
      zhi = sd > 0.f ? ((float)hi - mean) / sd : (float)hi - mean;
    }
    s_par[0] = mean;
    s_par[1] = sd;
    s_par[2] = zlo;
    s_par[3] = zhi;
  }
  __syncthreads();
  const float mean = s_par[0], sd = s_par[1], zlo = s_par[2], zhi = s_par[3];
  const bool flat = !(zhi > zlo);
  auto norm = [&](int gi) {
#pragma clang fp contract(off)
    const float g = (float)gi;
    const float z = sd > 0.f ? (g - mean) / sd : g - mean;
    return flat ? 0.f : (z - zlo) / (zhi - zlo);
  };
  if (v4 && ((uintptr_t)o & 15) == 0) {
    for (long p = tid; p < HW / 4; p += PP_THREADS) {
      const uint32_t w = reinterpret_cast<const uint32_t*>(f)[p];
      reinterpret_cast<float4*>(o)[p] = make_float4(norm(w & 255), norm((w >> 8) & 255), norm((w >> 16) & 255), norm(w >> 24));
    }
  } else {
    for (long p = tid; p < HW; p += PP_THREADS) o[p] = norm(grey_at(f, p, ch));
  }
}

}  // namespace

void launch_preprocess(const uint8_t* frames, int N, int H, int W, int channels, float* out, hipStream_t s) {
  M2S_CHECK(N >= 0 && H > 0 && W > 0 && (channels == 1 || channels == 3), "preprocess: bad shape");
  if (N == 0) return;
  hipLaunchKernelGGL(preprocess_kernel, dim3(N), dim3(PP_THREADS), 0, s, frames, H * W, channels, out);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
