// SqueezeExcite excitation for a batch of images in one kernel (bf16 engines):
//   hidden = SiLU(W_reduce · mean + b_reduce) ; gate = sigmoid(W_expand · hidden + b_expand)
// (timm SqueezeExcite conv_reduce -> act -> conv_expand -> gate, inside the InvertedResidual blocks
// that mri_acoustic_model.py:28-34 builds).  As two GEMMs over M = images these ran with 8..15
// workgroups and 20-40 serial k-steps each (~35 us per block for ~0.3 GFLOP).  Here a workgroup
// owns 16 images - the MFMA N dimension - so both layers are a handful of v_mfma_f32_16x16x32_bf16
// per wave: reduce = 4 waves x (rd/16 <= 4 row tiles) x (cs_mid/32) k-steps with the squeeze
// vectors read straight into B fragments; the hidden layer (bf16) goes through LDS; expand = the
// cs_mid/16 channel tiles spread over the waves, 2 k-steps each.  Weights are the GEMM path's
// packed rows ([>= rd][cs_mid] and [>= mid][cs(rd)]).
#include <algorithm>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

constexpr int SE_IMG = 16;   // images per workgroup (MFMA N)
constexpr int SE_RDMAX = 64;
constexpr int SE_HROW = SE_RDMAX + 8;  // LDS row of the hidden layer (bf16), padded

__global__ void __launch_bounds__(256) se_excite_kernel(const bf16_t* __restrict__ mean, int N, int mid, int cs_mid,
                                                        const bf16_t* __restrict__ w1, int kp1,
                                                        const float* __restrict__ b1, int rd,
                                                        const bf16_t* __restrict__ w2, int kp2,
                                                        const float* __restrict__ b2, bf16_t* __restrict__ gate) {
  __shared__ __attribute__((aligned(16))) bf16_t hid[SE_IMG][SE_HROW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = blockIdx.x * SE_IMG;
  const bool img_ok = n0 + r16 < N;
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);

  // ---- conv_reduce + SiLU: wave w owns hidden rows [16w, 16w + 16) ------------------------------
  {
    const int row = 16 * wave + r16;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (16 * wave < rd) {
      const bf16_t* wr = w1 + (size_t)row * kp1 + 8 * g;
      const bf16_t* mr = mean + (size_t)(n0 + r16) * cs_mid + 8 * g;
      // 8 k-steps of loads in flight per batch: the chain is load-latency bound, not MFMA bound
      const bool rok = row < rd;
      for (int k0 = 0; k0 < cs_mid; k0 += 8 * 32) {
        uint4 a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + 32 * u;
          a[u] = rok && k < cs_mid ? *reinterpret_cast<const uint4*>(wr + k) : z4;
          b[u] = img_ok && k < cs_mid ? *reinterpret_cast<const uint4*>(mr + k) : z4;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[u]), __builtin_bit_cast(bf16x8, b[u]),
                                                        acc, 0, 0, 0);
      }
    }
    // lane holds hidden rows 16w + 4g .. + 3 of image r16
    float h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 16 * wave + 4 * g + j;
      h[j] = r < rd ? silu(acc[j] + b1[r]) : 0.f;
    }
    *reinterpret_cast<uint2*>(&hid[r16][16 * wave + 4 * g]) = make_uint2(pack_bf16x2(h[0], h[1]), pack_bf16x2(h[2], h[3]));
  }
  __syncthreads();

  // ---- conv_expand + sigmoid: channel tiles of 16 over the waves ---------------------------------
  bf16x8 hb[SE_RDMAX / 32];
#pragma unroll
  for (int ks = 0; ks < SE_RDMAX / 32; ++ks) hb[ks] = *reinterpret_cast<const bf16x8*>(&hid[r16][32 * ks + 8 * g]);
  const int nks = kp2 / 32;
  const int ntile = cs_mid / 16;
  // 4 channel tiles per batch, all their weight fragments loaded before the MFMAs
  for (int t0 = wave; t0 < ntile; t0 += 4 * 4) {
    uint4 a[4][SE_RDMAX / 32];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = 16 * (t0 + 4 * u) + r16;  // weight row of this lane's A fragment
#pragma unroll
      for (int ks = 0; ks < SE_RDMAX / 32; ++ks)
        a[u][ks] = c < mid && ks < nks ? *reinterpret_cast<const uint4*>(w2 + (size_t)c * kp2 + 32 * ks + 8 * g) : z4;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + 4 * u;
      if (t >= ntile) break;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < SE_RDMAX / 32; ++ks)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[u][ks]), hb[ks], acc, 0, 0, 0);
      // lane holds gates of channels 16t + 4g .. + 3 for image r16
      const int c4 = 16 * t + 4 * g;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c4 + j < mid ? sigmoidf_(acc[j] + b2[c4 + j]) : 0.f;
      if (img_ok)
        *reinterpret_cast<uint2*>(gate + (size_t)(n0 + r16) * cs_mid + c4) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
}

}  // namespace

bool se_excite_supported(int rd, int kp2, int cs_mid) {
  return rd >= 1 && rd <= SE_RDMAX && kp2 >= rd && kp2 % 32 == 0 && kp2 <= SE_RDMAX && cs_mid % 32 == 0;
}

void launch_se_excite(const bf16_t* mean, int N, int mid, int cs_mid, const bf16_t* w1, int kp1, const float* b1,
                      int rd, const bf16_t* w2, int kp2, const float* b2, bf16_t* gate, hipStream_t s) {
  M2S_CHECK(se_excite_supported(rd, kp2, cs_mid) && kp1 >= cs_mid && N > 0, "se_excite: unsupported shape");
  ProfScope ps("se_excite_kernel", 2.0 * 2.0 * N * mid * rd, 2.0 * (2.0 * N * cs_mid) + 2.0 * 2.0 * mid * rd, s);
  hipLaunchKernelGGL(se_excite_kernel, dim3(ceil_div(N, SE_IMG)), dim3(256), 0, s, mean, N,
                     mid, cs_mid, w1, kp1, b1, rd, w2, kp2, b2, gate);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
