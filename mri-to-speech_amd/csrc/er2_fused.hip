// Fused EdgeResidual block (bf16), stride 1 with skip, 56 -> 224 -> 56 channels (channel strides
// 64 / 224 / 64): tf_efficientnetv2_b2 blocks.2.1/.2 at 32x32 (timm EdgeResidual conv_exp 3x3 + bn1 +
// SiLU -> conv_pwl 1x1 + bn2 -> + shortcut; mri_acoustic_model.py:28-34 builds the backbone).
//
// Same dataflow as er_fused.hip (conv_exp accumulators -> bias + SiLU -> conv_pwl B fragments through
// a permuted K order; the 224-channel map never leaves the registers), but conv_exp's weights are
// 258 KB, so they cannot sit in LDS: every 16x16 output tile streams them, with conv_pwl's, through a
// 3-slot LDS ring of 16 KB stages (20 stages per tile: 18 conv_exp k-steps of 14 fragments, 2 conv_pwl
// stages), two 1 KB LDS-DMA pieces per wave per stage, in the fragment order the host packs.  The ring
// runs across tiles, and the next tile's haloed input (8 planes of 18x18 pixels) lands in the second
// halo buffer while the current tile computes.  Waits are counted `vmcnt`s over a fixed per-tile issue
// order (the table in the stage loop), including exactly 8 output stores per wave and tile.
#include <algorithm>
#include <cstdio>
#include <type_traits>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_er2_zero[4];

constexpr int E2_TW = 16, E2_HW = 18, E2_HPIX = E2_HW * E2_HW;
constexpr int E2_PLANE = 384 * 16;          // 6 pieces of 64 pixels
constexpr int E2_BUF = 8 * E2_PLANE;        // 64 channels = 8 planes (48 KB)
constexpr int E2_STAGE = 16 * 1024;         // 16 pieces
constexpr int E2_SLOTS = 3;
constexpr int E2_NST = 20;                  // stages per tile
constexpr int E2_MID = 224, E2_NT = 14, E2_ON = 4;

struct Er2Args {
  const bf16_t* x;      // (N, H, W, 64)
  const bf16_t* wst;    // stage stream [20][16][64][8]
  const float* bexp;    // [224]
  const float* bpwl;    // [64] (zero past 56)
  bf16_t* y;            // (N, H, W, 64)
  int N, H, W, tiles_x, tiles_y;
};

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
// LDS reads the compiler does not see: an ordinary ds_read after an LDS-DMA gets a conservative
// s_waitcnt vmcnt(0), which would drain the ring's prefetch.  These wait only for themselves.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ uint2 lds_u2(const void* p) {
  uint2 r;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_off(p)));
  return r;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ void __launch_bounds__(512, 1) er2_fused_kernel(const Er2Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;                                              // 3 x 16 KB
  char* hbuf = smem + E2_SLOTS * E2_STAGE;                        // 2 x 48 KB
  float* bexp_l = reinterpret_cast<float*>(hbuf + 2 * E2_BUF);    // 224 floats
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int tpi = a.tiles_x * a.tiles_y, ntiles = a.N * tpi;

  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_er2_zero;
  asm volatile("" : "+s"(zpage));
  auto stage_dma = [&](int ls, int slot) {  // 2 pieces per wave
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = wave * 2 + j;
      dma16(a.wst + ((size_t)(ls * 16 + piece) * 64 + lane) * 8, ring + slot * E2_STAGE + piece * 1024);
    }
  };
  auto halo_dma = [&](int tile, char* buf) {  // 6 pieces per wave: 8 planes x 6 pixel blocks
    const int n = tile / tpi, tr = tile - n * tpi;
    const int ty0 = (tr / a.tiles_x) * E2_TW - 1, tx0 = (tr - (tr / a.tiles_x) * a.tiles_x) * E2_TW - 1;
    const bf16_t* xi = a.x + (size_t)n * a.H * a.W * 64;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int piece = wave * 6 + j, c = piece / 6, pb = piece - c * 6;
      const int p = pb * 64 + lane, hy = p / E2_HW, hx = p - hy * E2_HW;
      const int iy = ty0 + hy, ix = tx0 + hx;
      const void* src = zpage;
      if (p < E2_HPIX && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) src = xi + ((size_t)iy * a.W + ix) * 64 + c * 8;
      dma16(src, buf + c * E2_PLANE + pb * 1024);
    }
  };

  for (int i = tid; i < E2_MID; i += 512) bexp_l[i] = a.bexp[i];
  __syncthreads();  // bexp_l is read through lds_f4, which the compiler's waits do not cover
  float4 bp[E2_ON];
#pragma unroll
  for (int on = 0; on < E2_ON; ++on) bp[on] = *reinterpret_cast<const float4*>(a.bpwl + on * 16 + 4 * g);

  int q = 0;  // global stage index (ring slot = q % 3)
  if ((int)blockIdx.x < ntiles) {
    stage_dma(0, 0);
    stage_dma(1, 1);
    halo_dma(blockIdx.x, hbuf);
  }
  for (int it = 0, tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    const bool has_next = tile + (int)gridDim.x < ntiles;
    const char* hb = hbuf + (it & 1) * E2_BUF;
    const int n = tile / tpi, tr = tile - n * tpi;
    const int oy0 = (tr / a.tiles_x) * E2_TW, ox = (tr - (tr / a.tiles_x) * a.tiles_x) * E2_TW + r16;

    f32x4 acc[2][E2_NT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int nt = 0; nt < E2_NT; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 o[2][E2_ON];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int on = 0; on < E2_ON; ++on) o[i][on] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Issue order per wave and tile: ls = 0: S(2), then H(next); ls = k < 18: S(k + 2); ls = 18, 19:
    // the next tile's S(0), S(1); after the stages the tile's 8 stores.  Stage ls has landed once only
    // the ops issued after it are outstanding.  Returns this lane's view of the stage's ring slot.
    auto begin_stage = [&](int ls) -> const char* {
      if (ls == 0) {
        if (it == 0) wait_vm<0>();  // prologue: S(0), S(1) and the halo
        else wait_vm<10>();         // younger: S(1), 8 stores
      } else if (ls == 1) {
        if (it == 0) wait_vm<0>();
        else if (has_next) wait_vm<16>();  // younger: 8 stores, S(2), H(next)
        else wait_vm<10>();
      } else if (ls == 2) {
        if (has_next) wait_vm<8>();  // younger: H(next), S(3)
        else wait_vm<2>();
      } else if (ls < 19 || has_next) {
        wait_vm<2>();  // younger: S(ls + 1)
      } else {
        wait_vm<0>();  // last tile, last stage
      }
      __builtin_amdgcn_s_barrier();  // every wave's pieces of stage ls landed; slot (q - 1) % 3 is free
      asm volatile("" ::: "memory");
      if (ls + 2 < E2_NST) stage_dma(ls + 2, (q + 2) % E2_SLOTS);
      else if (has_next) stage_dma(ls + 2 - E2_NST, (q + 2) % E2_SLOTS);
      if (ls == 0 && has_next) halo_dma(tile + gridDim.x, hbuf + ((it + 1) & 1) * E2_BUF);
      const char* ws = ring + (q % E2_SLOTS) * E2_STAGE + lane * 16;
      ++q;
      return ws;
    };

    // ---- conv_exp: 18 k-steps (tap ls / 2, input channels 32 (ls % 2) .. + 31) -------------------
#pragma unroll 1
    for (int ls = 0; ls < 18; ++ls) {
      const char* ws = begin_stage(ls);
      const int t = ls >> 1, h = ls & 1, ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bx[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        bx[i] = *reinterpret_cast<const bf16x8*>(hb + (h * 4 + g) * E2_PLANE + ((2 * wave + i + ky) * E2_HW + r16 + kx) * 16);
#pragma unroll
      for (int nt = 0; nt < E2_NT; ++nt) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ws + nt * 1024);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bx[i], acc[i][nt], 0, 0, 0);
      }
    }
    // ---- bn1 bias + SiLU: the accumulators of n-tiles (2 ks, 2 ks + 1) become conv_pwl's B fragment of
    // k-step ks (the compiler puts a vmcnt(0) before these bias reads, for the DMA of stage 19) -----
    bf16x8 mb[2][E2_MID / 32];
#pragma unroll
    for (int ks = 0; ks < E2_MID / 32; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        uint32_t u[4];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int nt = 2 * ks + hh;
          const float4 bb = *reinterpret_cast<const float4*>(bexp_l + nt * 16 + 4 * g);
          u[2 * hh] = pack_bf16x2(silu(acc[i][nt][0] + bb.x), silu(acc[i][nt][1] + bb.y));
          u[2 * hh + 1] = pack_bf16x2(silu(acc[i][nt][2] + bb.z), silu(acc[i][nt][3] + bb.w));
        }
        mb[i][ks] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
      }
    // ---- conv_pwl: stage 18 = k-steps 0..3, stage 19 = 4..6 (piece = local k-step * 4 + on) -------
    auto pwl_stage = [&](auto ks0_c, auto nks_c) {
      constexpr int ks0 = decltype(ks0_c)::value, nks = decltype(nks_c)::value;
      const char* ws = begin_stage(ks0 == 0 ? 18 : 19);
#pragma unroll
      for (int kk = 0; kk < nks; ++kk)
#pragma unroll
        for (int on = 0; on < E2_ON; ++on) {
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(ws + (kk * 4 + on) * 1024);
#pragma unroll
          for (int i = 0; i < 2; ++i) o[i][on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, mb[i][ks0 + kk], o[i][on], 0, 0, 0);
        }
    };
    pwl_stage(std::integral_constant<int, 0>(), std::integral_constant<int, 4>());
    pwl_stage(std::integral_constant<int, 4>(), std::integral_constant<int, 3>());

    // ---- + bn2 bias + shortcut (halo centre); 8 stores per wave --------------------------------
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ry = 2 * wave + i, oy = oy0 + ry;
#pragma unroll
      for (int on = 0; on < E2_ON; ++on) {
        const int c4 = on * 16 + 4 * g;
        const uint2 r = lds_u2(hb + (c4 >> 3) * E2_PLANE + ((ry + 1) * E2_HW + r16 + 1) * 16 + (c4 & 7) * 2);
        const float v0 = o[i][on][0] + bp[on].x + __uint_as_float(r.x << 16);
        const float v1 = o[i][on][1] + bp[on].y + __uint_as_float(r.x & 0xffff0000u);
        const float v2 = o[i][on][2] + bp[on].z + __uint_as_float(r.y << 16);
        const float v3 = o[i][on][3] + bp[on].w + __uint_as_float(r.y & 0xffff0000u);
        *reinterpret_cast<uint2*>(a.y + (((size_t)n * a.H + oy) * a.W + ox) * 64 + c4) =
            make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
      }
    }
  }
  wait_vm<0>();
}

}  // namespace

bool er2_fused_supported(int H, int W, int cs_in, int mid, int cout, int kp_exp, int kp_pwl) {
  return cs_in == 64 && mid == E2_MID && cout <= 64 && cout > 32 && kp_exp == 9 * 64 && kp_pwl == E2_MID &&
         H % E2_TW == 0 && W % E2_TW == 0 && H > 0 && W > 0;
}

int er2_stage_elems() { return E2_NST * 16 * 64 * 8; }

void launch_er2_fused(const bf16_t* x, int N, int H, int W, const bf16_t* wst, const float* bexp, const float* bpwl,
                      bf16_t* y, double flops, double bytes, hipStream_t s) {
  M2S_CHECK(N > 0 && H % E2_TW == 0 && W % E2_TW == 0, "er2_fused: unsupported shape");
  Er2Args a;
  a.x = x;
  a.wst = wst;
  a.bexp = bexp;
  a.bpwl = bpwl;
  a.y = y;
  a.N = N;
  a.H = H;
  a.W = W;
  a.tiles_x = W / E2_TW;
  a.tiles_y = H / E2_TW;
  const size_t lds = E2_SLOTS * E2_STAGE + 2 * E2_BUF + E2_MID * sizeof(float);
  allow_lds(reinterpret_cast<const void*>(&er2_fused_kernel));
  const int cus = device_cus();
  const int grid = std::min(N * a.tiles_x * a.tiles_y, cus);
  ProfScope ps("er2_fused_kernel", flops, bytes, s);
  hipLaunchKernelGGL(er2_fused_kernel, dim3(grid), dim3(512), lds, s, a);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
