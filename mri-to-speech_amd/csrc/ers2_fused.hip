// Fused stride-2 EdgeResidual block (bf16, no shortcut): conv_exp 3x3/s2 TF-SAME + bn1 + SiLU ->
// conv_pwl 1x1 + bn2, for tf_efficientnetv2_b2 blocks.1.0 (16 -> 64 -> 32, 128x128 -> 64x64) and
// blocks.2.0 (32 -> 128 -> 56, 64x64 -> 32x32) (timm EdgeResidual; mri_acoustic_model.py:28-34).
//
// Same dataflow as er_fused.hip: the conv_exp accumulators (lane = 4 consecutive channels of one
// pixel) become conv_pwl's B fragments through the permuted conv_pwl K order, so the expanded map
// never exists in memory.  Differences: stride 2, and one output tile is 8 rows x 16 columns (wave w
// owns row w).  Its haloed input (17 x 33 pixels) sits in LDS split by column parity,
// [8-channel chunk][parity][row][column / 2] with 17-pixel rows, so the 16 pixels of a B-fragment read
// (input columns 2 x + kx) are 16 consecutive 16-byte slots: conflict-free at every tap.  With
// CIN = 16 a 32-deep k-step covers two taps (lane groups 0-1: tap 2s, 2-3: tap 2s + 1).
// Persistent workgroups (8 waves; one per CU, two for blocks.1.0): conv_exp's weights are DMA'd into LDS once, the next
// tile's halo lands in the second buffer while the current tile computes, conv_pwl's weights and the
// biases stay in VGPRs.
#include <algorithm>
#include <cstdio>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_es2_zero[4];  // DMA source for padding pixels

constexpr int ES_TH = 8, ES_TW = 16;     // output tile rows / columns
constexpr int ES_HR = 2 * ES_TH + 1;     // 17 halo rows
constexpr int ES_HC = ES_TW + 1;         // 17 slots per parity row (33 halo columns)
constexpr int ES_PPL = 5;                // 1 KB DMA pieces per (chunk, parity) plane: 17 x 17 <= 320
constexpr int ES_PLANE = ES_PPL * 1024;

struct Es2Args {
  const bf16_t* x;     // (N, H, W, CIN)
  const bf16_t* wexp;  // [KS][MID / 16][64][8]
  const float* bexp;   // [MID]
  const bf16_t* wpwl;  // [CO / 16][MID / 32][64][8], permuted K
  const float* bpwl;   // [CO] (zero past cout)
  bf16_t* y;           // (N, OH, OW, CO)
  uint8_t* y8;         // bf16 kernel, fp8 engines: e4m3 of the stored y, (N, OH, OW, CO) bytes (the next
                       // block's er8_fused operand), or null
  int N, H, W, OH, OW, pad_t, pad_l, tiles_x, tiles_y;
};

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Y8: also store y's e4m3 bytes (a.y8).  A template parameter, so the per-tile store count the counted vmcnt wait
// at the top of the tile loop relies on (ON, 2 ON with y8) is fixed when the kernel is compiled.
template <int CIN, int MID, int CO, bool Y8>
__global__ void __launch_bounds__(512, (CIN == 16 ? 2 : 1)) ers2_fused_kernel(const Es2Args a) {
  constexpr int NCH = CIN / 8;             // input chunks
  constexpr int KS = (9 * CIN + 31) / 32;  // conv_exp k-steps
  constexpr int NT = MID / 16;             // conv_exp n16 tiles
  constexpr int PK = MID / 32;             // conv_pwl k-steps
  constexpr int ON = CO / 16;              // conv_pwl n16 tiles
  constexpr int BUF = NCH * 2 * ES_PLANE;
  constexpr int WEXP = KS * NT * 1024;
  constexpr int NPIECE = NCH * 2 * ES_PPL;  // halo DMA pieces per tile
  static_assert(CIN == 16 || CIN == 32, "CIN");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;
  char* hbuf = smem + WEXP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifndef ERB_PRIO
#define ERB_PRIO 1
#endif
  // the younger half at static priority (er_sp_fused.hip): configs[4] bf16 A/B -4 % (CIN 16) / -1 % (CIN 32);
  // er_fused / er2_fused measured -0.4 % / +1 % that way and do not take it (profiles/r04_prio_kstats.txt)
  if (ERB_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int g = lane >> 4, r16 = lane & 15;
  const int tpi = a.tiles_x * a.tiles_y, ntiles = a.N * tpi;

  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_es2_zero;
  asm volatile("" : "+s"(zpage));
  auto issue_halo = [&](int tile, char* buf) {
    const int n = tile / tpi, tr = tile - n * tpi, ty = tr / a.tiles_x, tx = tr - ty * a.tiles_x;
    const int iy0 = 2 * ES_TH * ty - a.pad_t, ix0 = 2 * ES_TW * tx - a.pad_l;
    const bf16_t* xi = a.x + (size_t)n * a.H * a.W * CIN;
#pragma unroll
    for (int p = wave; p < NPIECE; p += 8) {
      const int pl = p / ES_PPL, pb = p - pl * ES_PPL, c = pl >> 1, par = pl & 1;
      const int slot = pb * 64 + lane, hy = slot / ES_HC, hx = 2 * (slot - hy * ES_HC) + par;
      const int iy = iy0 + hy, ix = ix0 + hx;
      const void* src = zpage;
      if (hy < ES_HR && hx <= 2 * ES_TW && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        src = xi + ((size_t)iy * a.W + ix) * CIN + c * 8;
      dma16(src, buf + pl * ES_PLANE + pb * 1024);
    }
  };

  // ---- once: conv_exp fragments -> LDS; conv_pwl fragments + biases -> VGPRs ---------------------
  for (int p = wave; p < KS * NT; p += 8) dma16(a.wexp + (size_t)p * 512 + lane * 8, wl + p * 1024);
  bf16x8 wp[ON][PK];
#pragma unroll
  for (int on = 0; on < ON; ++on)
#pragma unroll
    for (int ks = 0; ks < PK; ++ks)
      wp[on][ks] = *reinterpret_cast<const bf16x8*>(a.wpwl + ((size_t)(on * PK + ks) * 64 + lane) * 8);
  float4 be[NT], bp[ON];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) be[nt] = *reinterpret_cast<const float4*>(a.bexp + nt * 16 + 4 * g);
#pragma unroll
  for (int on = 0; on < ON; ++on) bp[on] = *reinterpret_cast<const float4*>(a.bpwl + on * 16 + 4 * g);
  if ((int)blockIdx.x < ntiles) issue_halo(blockIdx.x, hbuf);
  wait_vm<0>();
  __syncthreads();

  for (int it = 0, tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    char* hb = hbuf + (it & 1) * BUF;
    if (it > 0) {
      if constexpr (Y8) wait_vm<2 * ON>();  // this tile's halo landed (the younger ops are the last tile's stores)
      else wait_vm<ON>();
      __builtin_amdgcn_s_barrier();  // ... for every wave; every wave is done with the other buffer
      asm volatile("" ::: "memory");  // (a raw barrier: __syncthreads would also wait for the stores)
    }
    if (tile + (int)gridDim.x < ntiles) issue_halo(tile + gridDim.x, hbuf + ((it + 1) & 1) * BUF);

    // ---- conv_exp: 16 pixels of output row `wave` x MID channels, K = 9 taps x CIN -------------
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int t = CIN == 16 ? min(2 * s + (g >> 1), 8) : s;  // tap 9 (CIN 16) has zero weights
      const int c = CIN == 16 ? (g & 1) : g;
      const int ky = t / 3, kx = t - (t / 3) * 3;
      const bf16x8 bx = *reinterpret_cast<const bf16x8*>(hb + (c * 2 + (kx & 1)) * ES_PLANE +
                                                         ((2 * wave + ky) * ES_HC + r16 + (kx >> 1)) * 16);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + ((s * NT + nt) * 64 + lane) * 16);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bx, acc[nt], 0, 0, 0);
      }
    }

    // ---- bias + SiLU -> bf16 B fragments of conv_pwl (permuted K) -> conv_pwl -> + bias -> y -----
    f32x4 o[ON];
#pragma unroll
    for (int on = 0; on < ON; ++on) o[on] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < PK; ++ks) {
      uint32_t u[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int nt = 2 * ks + h;
        u[2 * h] = pack_bf16x2(silu(acc[nt][0] + be[nt].x), silu(acc[nt][1] + be[nt].y));
        u[2 * h + 1] = pack_bf16x2(silu(acc[nt][2] + be[nt].z), silu(acc[nt][3] + be[nt].w));
      }
      const bf16x8 mb = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
#pragma unroll
      for (int on = 0; on < ON; ++on) o[on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[on][ks], mb, o[on], 0, 0, 0);
    }
    const int n = tile / tpi, tr = tile - n * tpi, ty = tr / a.tiles_x, tx = tr - ty * a.tiles_x;
    const int oy = ty * ES_TH + wave, ox = tx * ES_TW + r16;
    // every tile is whole (OH % 8 == 0, OW % 16 == 0): exactly ON stores (2 ON with y8) per wave per
    // tile, which the counted wait at the top of the loop relies on
#pragma unroll
    for (int on = 0; on < ON; ++on) {
      const int c4 = on * 16 + 4 * g;
      const size_t px = ((size_t)n * a.OH + oy) * a.OW + ox;
      const uint2 yb = make_uint2(pack_bf16x2(o[on][0] + bp[on].x, o[on][1] + bp[on].y),
                                  pack_bf16x2(o[on][2] + bp[on].z, o[on][3] + bp[on].w));
      *reinterpret_cast<uint2*>(a.y + px * CO + c4) = yb;
      if constexpr (Y8) *reinterpret_cast<uint32_t*>(a.y8 + px * CO + c4) = e4m3x4_bf16(yb);
    }
  }
  wait_vm<0>();
}


// Split fp32 (m2s_common.hpp sp_t) for blocks.1.0 (CIN 16): the halo carries hi and lo planes
// ([hi/lo][chunk][parity][row][column / 2]), conv_exp's W_hi / W_lo fragments stay in LDS
// ([hi/lo][k-step][n16][lane][8], 40 KB), conv_pwl's in VGPRs; every product is the three MFMA
// terms, the conv_exp accumulators are re-split into conv_pwl's B fragments, y is stored as hi/lo
// rows.  One workgroup per CU (120 KB of LDS).
template <int CIN, int MID, int CO>
__global__ void __launch_bounds__(512, 1) ers2_sp_kernel(const Es2Args a) {
  constexpr int NCH = CIN / 8;
  constexpr int KS = (9 * CIN + 31) / 32;
  constexpr int NT = MID / 16, PK = MID / 32, ON = CO / 16;
  constexpr int HPL = 2 * NCH * 2;  // halo planes: (hi / lo, chunk, column parity)
  constexpr int BUF = HPL * ES_PLANE;
  constexpr int WEXP = 2 * KS * NT * 1024;
  constexpr int NPIECE = HPL * ES_PPL;
  static_assert(CIN == 16 && NPIECE % 8 == 0, "split stride-2 EdgeResidual: blocks.1.0 shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;
  char* hbuf = smem + WEXP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifndef ERS2_PRIO
#define ERS2_PRIO 1
#endif
  // the younger half at static priority (er_sp_fused.hip): same-box A/B -2 %
  if (ERS2_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int g = lane >> 4, r16 = lane & 15;
  const int tpi = a.tiles_x * a.tiles_y, ntiles = a.N * tpi;

  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_es2_zero;
  asm volatile("" : "+s"(zpage));
  auto issue_halo = [&](int tile, char* buf) {
    const int n = tile / tpi, tr = tile - n * tpi, ty = tr / a.tiles_x, tx = tr - ty * a.tiles_x;
    const int iy0 = 2 * ES_TH * ty - a.pad_t, ix0 = 2 * ES_TW * tx - a.pad_l;
    const bf16_t* xi = a.x + (size_t)n * a.H * a.W * CIN * 2;
#pragma unroll
    for (int p = wave; p < NPIECE; p += 8) {
      const int pl = p / ES_PPL, pb = p - pl * ES_PPL, hl = pl / (2 * NCH), c = (pl >> 1) % NCH, par = pl & 1;
      const int slot = pb * 64 + lane, hy = slot / ES_HC, hx = 2 * (slot - hy * ES_HC) + par;
      const int iy = iy0 + hy, ix = ix0 + hx;
      const void* src = zpage;
      if (hy < ES_HR && hx <= 2 * ES_TW && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        src = xi + ((size_t)iy * a.W + ix) * CIN * 2 + hl * CIN + c * 8;
      dma16(src, buf + pl * ES_PLANE + pb * 1024);
    }
  };

  for (int p = wave; p < 2 * KS * NT; p += 8) dma16(a.wexp + (size_t)p * 512 + lane * 8, wl + p * 1024);
  bf16x8 wph[ON][PK], wpl[ON][PK];
#pragma unroll
  for (int on = 0; on < ON; ++on)
#pragma unroll
    for (int ks = 0; ks < PK; ++ks) {
      wph[on][ks] = *reinterpret_cast<const bf16x8*>(a.wpwl + ((size_t)(on * PK + ks) * 64 + lane) * 8);
      wpl[on][ks] = *reinterpret_cast<const bf16x8*>(a.wpwl + ((size_t)((ON + on) * PK + ks) * 64 + lane) * 8);
    }
  float4 be[NT], bp[ON];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) be[nt] = *reinterpret_cast<const float4*>(a.bexp + nt * 16 + 4 * g);
#pragma unroll
  for (int on = 0; on < ON; ++on) bp[on] = *reinterpret_cast<const float4*>(a.bpwl + on * 16 + 4 * g);
  if ((int)blockIdx.x < ntiles) issue_halo(blockIdx.x, hbuf);
  wait_vm<0>();
  __syncthreads();

  uint16_t* Y = reinterpret_cast<uint16_t*>(a.y);
  for (int it = 0, tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    char* hb = hbuf + (it & 1) * BUF;
    if (it > 0) {
      wait_vm<2 * ON>();  // this tile's halo landed (the 2 ON younger ops: the last tile's hi / lo stores)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (tile + (int)gridDim.x < ntiles) issue_halo(tile + gridDim.x, hbuf + ((it + 1) & 1) * BUF);

    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int t = min(2 * s + (g >> 1), 8), c = g & 1;  // tap 9 has zero weights
      const int ky = t / 3, kx = t - (t / 3) * 3;
      const int off = ((2 * wave + ky) * ES_HC + r16 + (kx >> 1)) * 16;
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(hb + (c * 2 + (kx & 1)) * ES_PLANE + off);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(hb + ((NCH + c) * 2 + (kx & 1)) * ES_PLANE + off);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(wl + ((s * NT + nt) * 64 + lane) * 16);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(wl + (((KS + s) * NT + nt) * 64 + lane) * 16);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[nt], 0, 0, 0);
      }
    }

    f32x4 o[ON];
#pragma unroll
    for (int on = 0; on < ON; ++on) o[on] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < PK; ++ks) {
      float v[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int nt = 2 * ks + h;
        v[4 * h] = silu(acc[nt][0] + be[nt].x);
        v[4 * h + 1] = silu(acc[nt][1] + be[nt].y);
        v[4 * h + 2] = silu(acc[nt][2] + be[nt].z);
        v[4 * h + 3] = silu(acc[nt][3] + be[nt].w);
      }
      uint2 h0, l0, h1, l1;
      split4(v, h0, l0);
      split4(v + 4, h1, l1);
      const bf16x8 mh = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
      const bf16x8 ml = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
#pragma unroll
      for (int on = 0; on < ON; ++on) {
        o[on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wpl[on][ks], mh, o[on], 0, 0, 0);
        o[on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wph[on][ks], ml, o[on], 0, 0, 0);
        o[on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wph[on][ks], mh, o[on], 0, 0, 0);
      }
    }
    const int n = tile / tpi, tr = tile - n * tpi, ty = tr / a.tiles_x, tx = tr - ty * a.tiles_x;
    const int oy = ty * ES_TH + wave, ox = tx * ES_TW + r16;
    // every tile is whole: exactly 2 ON stores per wave per tile (the counted wait above)
#pragma unroll
    for (int on = 0; on < ON; ++on) {
      const int c4 = on * 16 + 4 * g;
      const float w4[4] = {o[on][0] + bp[on].x, o[on][1] + bp[on].y, o[on][2] + bp[on].z, o[on][3] + bp[on].w};
      uint2 hi, lo;
      split4(w4, hi, lo);
      uint16_t* yp = Y + (((size_t)n * a.OH + oy) * a.OW + ox) * CO * 2 + c4;
      *reinterpret_cast<uint2*>(yp) = hi;
      *reinterpret_cast<uint2*>(yp + CO) = lo;
    }
  }
  wait_vm<0>();
}

template <int CIN, int MID, int CO>
void launch_cfg_sp(const Es2Args& a, double flops, double bytes, hipStream_t s) {
  constexpr int KS = (9 * CIN + 31) / 32;
  const size_t lds = (size_t)2 * KS * (MID / 16) * 1024 + 2 * (size_t)2 * (CIN / 8) * 2 * ES_PLANE;
  allow_lds(reinterpret_cast<const void*>(&ers2_sp_kernel<CIN, MID, CO>));
  M2S_CHECK(lds <= 160 * 1024, "ers2_sp: LDS budget");
  const int cus = device_cus();
  const int grid = std::min(a.N * a.tiles_x * a.tiles_y, cus);
  char name[64];
  snprintf(name, sizeof(name), "ers2_sp_kernel<%d, %d, %d>", CIN, MID, CO);
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((ers2_sp_kernel<CIN, MID, CO>), dim3(grid), dim3(512), lds, s, a);
  M2S_HIP(hipGetLastError());
}

template <int CIN, int MID, int CO, bool Y8>
void launch_cfg(const Es2Args& a, double flops, double bytes, hipStream_t s) {
  constexpr int KS = (9 * CIN + 31) / 32;
  const size_t lds = (size_t)KS * (MID / 16) * 1024 + 2 * (size_t)(CIN / 8) * 2 * ES_PLANE;
  allow_lds(reinterpret_cast<const void*>(&ers2_fused_kernel<CIN, MID, CO, Y8>));
  M2S_CHECK(lds <= 160 * 1024, "ers2_fused: LDS budget");
  const int cus = device_cus();
  // CIN 16: 60 KB of LDS and < 128 VGPRs, so two workgroups per CU
  const int grid = std::min(a.N * a.tiles_x * a.tiles_y, (CIN == 16 ? 2 : 1) * cus);
  char name[64];
  snprintf(name, sizeof(name), "ers2_fused_kernel<%d, %d, %d, %s>", CIN, MID, CO, Y8 ? "true" : "false");
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((ers2_fused_kernel<CIN, MID, CO, Y8>), dim3(grid), dim3(512), lds, s, a);
  M2S_HIP(hipGetLastError());
}

}  // namespace

bool ers2_fused_supported(int OH, int OW, int cs_in, int mid, int cs_out, int kp_exp, int kp_pwl) {
  const bool shape = (cs_in == 16 && mid == 64 && cs_out == 32) || (cs_in == 32 && mid == 128 && cs_out == 64);
  return shape && kp_exp >= 9 * cs_in && kp_pwl == mid && OH > 0 && OW > 0 && OH % ES_TH == 0 && OW % ES_TW == 0;
}

int ers2_exp_elems(int cs_in, int mid) { return (9 * cs_in + 31) / 32 * (mid / 16) * 512; }

bool ers2_sp_supported(int OH, int OW, int cs_in, int mid, int cs_out) {
  return cs_in == 16 && mid == 64 && cs_out == 32 && OH > 0 && OW > 0 && OH % ES_TH == 0 && OW % ES_TW == 0;
}

void launch_ers2_sp(const void* x, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, int cs_in, int mid,
                    int cs_out, const void* wexp, const float* bexp, const void* wpwl, const float* bpwl, void* y,
                    double flops, double bytes, hipStream_t s) {
  M2S_CHECK(N > 0 && ers2_sp_supported(OH, OW, cs_in, mid, cs_out), "ers2_sp: unsupported shape");
  Es2Args a;
  a.x = static_cast<const bf16_t*>(x);
  a.wexp = static_cast<const bf16_t*>(wexp);
  a.bexp = bexp;
  a.wpwl = static_cast<const bf16_t*>(wpwl);
  a.bpwl = bpwl;
  a.y = static_cast<bf16_t*>(y);
  a.y8 = nullptr;
  a.N = N;
  a.H = H;
  a.W = W;
  a.OH = OH;
  a.OW = OW;
  a.pad_t = pad_t;
  a.pad_l = pad_l;
  a.tiles_x = OW / ES_TW;
  a.tiles_y = OH / ES_TH;
  launch_cfg_sp<16, 64, 32>(a, flops, bytes, s);
}

void launch_ers2_fused(const bf16_t* x, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, int cs_in, int mid,
                       int cs_out, const bf16_t* wexp, const float* bexp, const bf16_t* wpwl, const float* bpwl,
                       bf16_t* y, double flops, double bytes, hipStream_t s, uint8_t* y8) {
  M2S_CHECK(N > 0 && ers2_fused_supported(OH, OW, cs_in, mid, cs_out, 9 * cs_in, mid), "ers2_fused: unsupported shape");
  Es2Args a;
  a.x = x;
  a.wexp = wexp;
  a.bexp = bexp;
  a.wpwl = wpwl;
  a.bpwl = bpwl;
  a.y = y;
  a.y8 = y8;
  a.N = N;
  a.H = H;
  a.W = W;
  a.OH = OH;
  a.OW = OW;
  a.pad_t = pad_t;
  a.pad_l = pad_l;
  a.tiles_x = OW / ES_TW;
  a.tiles_y = OH / ES_TH;
  if (cs_in == 16) {
    if (y8) launch_cfg<16, 64, 32, true>(a, flops, bytes, s);
    else launch_cfg<16, 64, 32, false>(a, flops, bytes, s);
  } else {
    if (y8) launch_cfg<32, 128, 64, true>(a, flops, bytes, s);
    else launch_cfg<32, 128, 64, false>(a, flops, bytes, s);
  }
}

}  // namespace m2s
