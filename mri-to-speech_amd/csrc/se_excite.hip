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
// Split fp32 (SP = 1, m2s_common.hpp sp_t): the squeeze vectors, the weights (rows [hi kp | lo kp])
// and the gates are hi/lo pairs, every product is the three MFMA terms hi*hi + hi*lo + lo*hi, and
// the hidden layer goes through LDS as two bf16 planes.  (The split engine used to run the two
// GEMMs through conv_gemm: 40 launches per step at 60-90 us, ~3 ms of a 56 ms step.)
#include <algorithm>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

constexpr int SE_IMG = 16;   // images per workgroup (MFMA N)
constexpr int SE_RDMAX = 64;
constexpr int SE_HROW = SE_RDMAX + 8;  // LDS row of the hidden layer (bf16), padded

__device__ __forceinline__ bf16x8 ld8(const bf16_t* p, bool ok) {
  return __builtin_bit_cast(bf16x8, ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u));
}

// acc += a * b over the split terms (SP) or the single bf16 term
template <int SP>
__device__ __forceinline__ f32x4 mma(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 acc) {
  if constexpr (SP) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  }
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// 4 values -> the dtype's storage at (row base u, channel c): bf16, or a hi/lo pair at +cs
template <int SP>
__device__ __forceinline__ void st4(bf16_t* u, int cs, const float* v) {
  if constexpr (SP) {
    uint2 hi, lo;
    split4(v, hi, lo);
    *reinterpret_cast<uint2*>(u) = hi;
    *reinterpret_cast<uint2*>(u + cs) = lo;
  } else {
    *reinterpret_cast<uint2*>(u) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
}

// NW waves a workgroup: 4, or 16 for small batches (the reduce's K chain split NW / RT ways instead of 4 / RT:
// at one clip the 8 x 8 blocks' 39-step chain made a 16-workgroup launch ~23 us)
template <int SP, int NW>
__global__ void __launch_bounds__(64 * NW) se_excite_kernel(const bf16_t* __restrict__ mean, int N, int mid, int cs_mid,
                                                        const bf16_t* __restrict__ w1, int kp1,
                                                        const float* __restrict__ b1, int rd,
                                                        const bf16_t* __restrict__ w2, int kp2,
                                                        const float* __restrict__ b2, bf16_t* __restrict__ gate) {
  constexpr int R = SP ? 2 : 1;
  constexpr int UB = SP ? 4 : 8;  // k-steps of loads in flight per batch
  __shared__ __attribute__((aligned(16))) bf16_t hid[R][SE_IMG][SE_HROW];
  __shared__ __attribute__((aligned(16))) f32x4 part[NW][64];  // K-split partial sums
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = blockIdx.x * SE_IMG;
  const bool img_ok = n0 + r16 < N;
  // the expand weights of this wave's first channel tile, fetched before the reduce so their latency hides under it
  // (a small batch's launch is a chain of dependent load round trips)
  const int nks = kp2 / 32, ntile = cs_mid / 16, t_first = NW * blockIdx.y + wave;
  bf16x8 pa[SE_RDMAX / 32], pal[SE_RDMAX / 32];
  {
    const int c = 16 * t_first + r16;
#pragma unroll
    for (int ks = 0; ks < SE_RDMAX / 32; ++ks) {
      const bf16_t* wp = w2 + (size_t)c * kp2 * R + 32 * ks + 8 * g;
      pa[ks] = ld8(wp, t_first < ntile && c < mid && ks < nks);
      if constexpr (SP) pal[ks] = ld8(wp + kp2, t_first < ntile && c < mid && ks < nks);
    }
  }

  // ---- conv_reduce + SiLU: RT = ceil(rd / 16) row tiles; the NW waves split K NW / RT ways -------
  // (wave w: row tile w % RT, k-steps w / RT, w / RT + KSP, ...), partials summed in LDS in a fixed
  // order.  One wave per row tile walked all cs_mid / 32 k-steps alone with two or three waves idle.
  {
    const int RT = (rd + 15) / 16, KSP = NW / RT;
    const int rt = wave % RT, kq = wave / RT;
    const int row = 16 * rt + r16;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kq < KSP) {
      const bf16_t* wr = w1 + (size_t)row * kp1 * R + 8 * g;
      const bf16_t* mr = mean + (size_t)(n0 + r16) * cs_mid * R + 8 * g;
      // UB k-steps of loads in flight per batch: the chain is load-latency bound, not MFMA bound
      const bool rok = row < rd;
      for (int k0 = 32 * kq; k0 < cs_mid; k0 += UB * 32 * KSP) {
        bf16x8 a[UB], b[UB], al[UB], bl[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int k = k0 + 32 * KSP * u;
          a[u] = ld8(wr + k, rok && k < cs_mid);
          b[u] = ld8(mr + k, img_ok && k < cs_mid);
          if constexpr (SP) {
            al[u] = ld8(wr + kp1 + k, rok && k < cs_mid);
            bl[u] = ld8(mr + cs_mid + k, img_ok && k < cs_mid);
          }
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) acc = mma<SP>(a[u], al[u], b[u], bl[u], acc);
      }
    }
    part[wave][lane] = acc;
    __syncthreads();
    if (wave < RT) {
      for (int q = 1; q < KSP; ++q) acc += part[wave + RT * q][lane];
      // lane holds hidden rows 16w + 4g .. + 3 of image r16
      float h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * wave + 4 * g + j;
        h[j] = r < rd ? silu(acc[j] + b1[r]) : 0.f;
      }
      st4<SP>(&hid[0][r16][16 * wave + 4 * g], SE_IMG * SE_HROW, h);
    } else if (wave < 4 && 16 * wave < SE_RDMAX) {  // rows past rd: zeros (read by the expand's k-steps)
      const float z[4] = {0.f, 0.f, 0.f, 0.f};
      st4<SP>(&hid[0][r16][16 * wave + 4 * g], SE_IMG * SE_HROW, z);
    }
  }
  __syncthreads();

  // ---- conv_expand + sigmoid: channel tiles of 16 over the waves ---------------------------------
  bf16x8 hb[SE_RDMAX / 32], hl[SE_RDMAX / 32];
#pragma unroll
  for (int ks = 0; ks < SE_RDMAX / 32; ++ks) {
    hb[ks] = *reinterpret_cast<const bf16x8*>(&hid[0][r16][32 * ks + 8 * g]);
    if constexpr (SP) hl[ks] = *reinterpret_cast<const bf16x8*>(&hid[R - 1][r16][32 * ks + 8 * g]);
  }
  // channel tiles dealt over the gridDim.y workgroups of these images and their 4 waves (tile
  // 4 * (y + gridDim.y * v) + wave); 4 tiles per batch, all their weight fragments loaded first
  const int ts = NW * gridDim.y;
  for (int t0 = NW * blockIdx.y + wave; t0 < ntile; t0 += 4 * ts) {
    bf16x8 a[4][SE_RDMAX / 32], al[4][SE_RDMAX / 32];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = 16 * (t0 + ts * u) + r16;  // weight row of this lane's A fragment
#pragma unroll
      for (int ks = 0; ks < SE_RDMAX / 32; ++ks) {
        if (u == 0 && t0 == t_first) {  // prefetched
          a[u][ks] = pa[ks];
          if constexpr (SP) al[u][ks] = pal[ks];
          continue;
        }
        const bf16_t* wp = w2 + (size_t)c * kp2 * R + 32 * ks + 8 * g;
        a[u][ks] = ld8(wp, c < mid && ks < nks);
        if constexpr (SP) al[u][ks] = ld8(wp + kp2, c < mid && ks < nks);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + ts * u;
      if (t >= ntile) break;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < SE_RDMAX / 32; ++ks) acc = mma<SP>(a[u][ks], al[u][ks], hb[ks], hl[ks], acc);
      // lane holds gates of channels 16t + 4g .. + 3 for image r16
      const int c4 = 16 * t + 4 * g;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c4 + j < mid ? sigmoidf_(acc[j] + b2[c4 + j]) : 0.f;
      if (img_ok) st4<SP>(gate + (size_t)(n0 + r16) * cs_mid * R + c4, cs_mid, v);
    }
  }
}

}  // namespace

bool se_excite_supported(int rd, int kp2, int cs_mid) {
  return rd >= 1 && rd <= SE_RDMAX && kp2 >= rd && kp2 % 32 == 0 && kp2 <= SE_RDMAX && cs_mid % 32 == 0;
}

void launch_se_excite(const void* mean, int N, int mid, int cs_mid, const void* w1, int kp1, const float* b1,
                      int rd, const void* w2, int kp2, const float* b2, void* gate, bool split, hipStream_t s) {
  M2S_CHECK(se_excite_supported(rd, kp2, cs_mid) && kp1 >= cs_mid && N > 0, "se_excite: unsupported shape");
  const double es = split ? 4.0 : 2.0;
  // expand tiles split over ES workgroups per 16 images (each recomputes the reduce) while the grid
  // stays within one workgroup per CU: 1920 images were 120 workgroups (0.67 ms per step); ES = 2
  // gives 0.50, and ES = 3 / 4 / 8 (past one per CU) 0.64 / 0.61 / 0.87.  Under a quarter of the CUs
  // busy (a few dozen images) the workgroups run 16 waves
  const int cus = device_cus();
  const int nwg = ceil_div(N, SE_IMG), ES = std::max(1, std::min(std::min(cus / nwg, cs_mid / 64), 8));
  const bool wide = nwg * ES * 4 <= cus;
  static const char* const names[2][2] = {{"se_excite_kernel<0, 4>", "se_excite_kernel<1, 4>"},
                                          {"se_excite_kernel<0, 16>", "se_excite_kernel<1, 16>"}};
  ProfScope ps(names[wide][split], 2.0 * 2.0 * N * mid * rd, es * (2.0 * N * cs_mid) + es * 2.0 * mid * rd, s);
  auto k = wide ? (split ? se_excite_kernel<1, 16> : se_excite_kernel<0, 16>) : (split ? se_excite_kernel<1, 4> : se_excite_kernel<0, 4>);
  hipLaunchKernelGGL(k, dim3(nwg, ES), dim3(wide ? 1024 : 256), 0, s, static_cast<const bf16_t*>(mean), N, mid, cs_mid,
                     static_cast<const bf16_t*>(w1), kp1, b1, rd, static_cast<const bf16_t*>(w2), kp2, b2,
                     static_cast<bf16_t*>(gate));
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
