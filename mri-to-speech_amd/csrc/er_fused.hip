// Fused EdgeResidual block (bf16), stride 1 with skip, 32 -> 128 -> 32 channels (timm EdgeResidual
// conv_exp 3x3 + bn1 + SiLU -> conv_pwl 1x1 + bn2 -> + shortcut: tf_efficientnetv2_b2 blocks.1.1/.2,
// built by mri_acoustic_model.py:28-34).
//
// Unfused, conv_exp writes its 128-channel map (2 GB per 1920 frames at 64x64) and conv_pwl reads it
// back; here it never leaves the registers.  The conv_exp accumulators of one 16-pixel subtile hold,
// per lane, 4 consecutive channels of each 16-channel tile; two adjacent tiles give the 8 values a
// lane needs as the B fragment of one 32-deep conv_pwl k-step, provided conv_pwl's K is permuted the
// same way (host packing: k-slot 8g+e of k-step s is channel 32s + 4g + e for e < 4, 32s + 16 + 4g +
// e - 4 otherwise).  So: conv_exp MFMAs -> bias + SiLU -> pack -> conv_pwl MFMAs -> bias + skip.
//
// Persistent workgroups (one per CU, 8 waves): conv_exp's weights (72 KB, fragment order) are
// DMA'd into LDS once; each 16x16 output tile's haloed input (18x18 x 32 channels) is DMA'd into
// one of two planar LDS buffers ([16-byte chunk][pixel], conflict-free fragment reads at any tap
// offset) while the previous tile computes.  conv_pwl's weights (8 KB) and all biases stay in VGPRs.
// Wave w computes output rows 2w and 2w+1 of the tile.
#include <algorithm>
#include <cstdio>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_er_zero[4];  // DMA source for padding pixels

constexpr int ER_TW = 16, ER_HW = 18;            // tile / halo width
constexpr int ER_HPIX = ER_HW * ER_HW;           // 324 halo pixels
constexpr int ER_PLANE = 384 * 16;               // 6 DMA pieces of 64 pixels per plane (24 x 256 B)
constexpr int ER_BUF = 4 * ER_PLANE;             // 4 planes of 8 channels
constexpr int ER_WEXP = 9 * 8 * 1024;            // conv_exp fragments: [tap][n16][lane][16 B]

struct ErArgs {
  const bf16_t* x;      // (N, H, W, 32)
  const bf16_t* wexp;   // fragment order [9][8][64][8]
  const float* bexp;    // [128]
  const bf16_t* wpwl;   // permuted fragment order [2][4][64][8]
  const float* bpwl;    // [32]
  bf16_t* y;            // (N, H, W, 32)
  int N, H, W, tiles_x, tiles_y;
};

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
// An LDS read the compiler does not see: an ordinary ds_read after an LDS-DMA (the next tile's halo)
// gets a conservative s_waitcnt vmcnt(0), which would also wait for this tile's stores.
__device__ __forceinline__ uint2 lds_u2(const void* p) {
  uint2 r;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(r)
               : "v"((uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p));
  return r;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ void __launch_bounds__(512, 1) er_fused_kernel(const ErArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;                 // conv_exp fragments
  char* hbuf = smem + ER_WEXP;     // two halo buffers
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int tpi = a.tiles_x * a.tiles_y, ntiles = a.N * tpi;

  // this wave's 3 halo pieces per tile: plane c, 64-pixel block pb
  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_er_zero;
  asm volatile("" : "+s"(zpage));
  auto issue_halo = [&](int tile, char* buf) {
    const int n = tile / tpi, tr = tile - n * tpi;
    const int ty0 = (tr / a.tiles_x) * ER_TW - 1, tx0 = (tr - (tr / a.tiles_x) * a.tiles_x) * ER_TW - 1;
    const bf16_t* xi = a.x + (size_t)n * a.H * a.W * 32;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int piece = wave * 3 + j, c = piece / 6, pb = piece - c * 6;
      const int p = pb * 64 + lane, hy = p / ER_HW, hx = p - hy * ER_HW;
      const int iy = ty0 + hy, ix = tx0 + hx;
      const void* src = zpage;
      if (p < ER_HPIX && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) src = xi + ((size_t)iy * a.W + ix) * 32 + c * 8;
      dma16(src, buf + c * ER_PLANE + pb * 1024);
    }
  };

  // ---- once: conv_exp fragments -> LDS (9 pieces per wave); conv_pwl fragments + biases -> VGPRs -
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int piece = wave * 9 + j;
    dma16(a.wexp + (size_t)piece * 512 + lane * 8, wl + piece * 1024);
  }
  bf16x8 wp[2][4];
#pragma unroll
  for (int on = 0; on < 2; ++on)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      wp[on][ks] = *reinterpret_cast<const bf16x8*>(a.wpwl + ((size_t)(on * 4 + ks) * 64 + lane) * 8);
  float4 be[8], bp[2];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) be[nt] = *reinterpret_cast<const float4*>(a.bexp + nt * 16 + 4 * g);
#pragma unroll
  for (int on = 0; on < 2; ++on) bp[on] = *reinterpret_cast<const float4*>(a.bpwl + on * 16 + 4 * g);
  if ((int)blockIdx.x < ntiles) issue_halo(blockIdx.x, hbuf);
  wait_vm<0>();
  __syncthreads();

  for (int it = 0, tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    char* hb = hbuf + (it & 1) * ER_BUF;
    if (it > 0) {
      wait_vm<4>();  // this tile's halo landed (the 4 younger ops are the last tile's stores)
      __builtin_amdgcn_s_barrier();  // ... for every wave; every wave is done with the other buffer
      asm volatile("" ::: "memory");  // (a raw barrier: __syncthreads would also wait for the stores)
    }
    if (tile + (int)gridDim.x < ntiles) issue_halo(tile + gridDim.x, hbuf + ((it + 1) & 1) * ER_BUF);

    // ---- conv_exp: 2 rows x 16 pixels x 128 channels per wave, K = 9 taps x 32 ----------------
    f32x4 acc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bx[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        bx[i] = *reinterpret_cast<const bf16x8*>(hb + g * ER_PLANE + ((2 * wave + i + ky) * ER_HW + r16 + kx) * 16);
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + ((t * 8 + nt) * 64 + lane) * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bx[i], acc[i][nt], 0, 0, 0);
      }
    }

    // ---- bias + SiLU -> bf16 B fragments of conv_pwl (permuted K) -> conv_pwl -------------------
    const int n = tile / tpi, tr = tile - n * tpi;
    const int oy0 = (tr / a.tiles_x) * ER_TW, ox = (tr - (tr / a.tiles_x) * a.tiles_x) * ER_TW + r16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        uint32_t u[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int nt = 2 * ks + h;
          u[2 * h] = pack_bf16x2(silu(acc[i][nt][0] + be[nt].x), silu(acc[i][nt][1] + be[nt].y));
          u[2 * h + 1] = pack_bf16x2(silu(acc[i][nt][2] + be[nt].z), silu(acc[i][nt][3] + be[nt].w));
        }
        const bf16x8 mb = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
#pragma unroll
        for (int on = 0; on < 2; ++on) o[on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wp[on][ks], mb, o[on], 0, 0, 0);
      }
      // + bn2 bias + shortcut (the tile's centre pixels of the halo buffer); 4 channels per lane
      const int ry = 2 * wave + i, oy = oy0 + ry;
#pragma unroll
      for (int on = 0; on < 2; ++on) {
        const int c4 = on * 16 + 4 * g;
        const uint2 r = lds_u2(hb + (c4 >> 3) * ER_PLANE + ((ry + 1) * ER_HW + r16 + 1) * 16 + (c4 & 7) * 2);
        const float v0 = o[on][0] + bp[on].x + __uint_as_float(r.x << 16);
        const float v1 = o[on][1] + bp[on].y + __uint_as_float(r.x & 0xffff0000u);
        const float v2 = o[on][2] + bp[on].z + __uint_as_float(r.y << 16);
        const float v3 = o[on][3] + bp[on].w + __uint_as_float(r.y & 0xffff0000u);
        // every tile is whole (H, W multiples of 16): exactly 4 stores per wave per tile, which the
        // counted wait at the top of the loop relies on
        *reinterpret_cast<uint2*>(a.y + (((size_t)n * a.H + oy) * a.W + ox) * 32 + c4) =
            make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
      }
    }
  }
  wait_vm<0>();
}

}  // namespace

bool er_fused_supported(int H, int W, int cin, int mid, int cout, int kp_exp, int kp_pwl) {
  return cin == 32 && mid == 128 && cout == 32 && kp_exp == 288 && kp_pwl == 128 && H % ER_TW == 0 && W % ER_TW == 0 &&
         H > 0 && W > 0;
}

void launch_er_fused(const bf16_t* x, int N, int H, int W, const bf16_t* wexp, const float* bexp, const bf16_t* wpwl,
                     const float* bpwl, bf16_t* y, double flops, double bytes, hipStream_t s) {
  M2S_CHECK(er_fused_supported(H, W, 32, 128, 32, 288, 128) && N > 0, "er_fused: unsupported shape");
  ErArgs a;
  a.x = x;
  a.wexp = wexp;
  a.bexp = bexp;
  a.wpwl = wpwl;
  a.bpwl = bpwl;
  a.y = y;
  a.N = N;
  a.H = H;
  a.W = W;
  a.tiles_x = W / ER_TW;
  a.tiles_y = H / ER_TW;
  const size_t lds = ER_WEXP + 2 * ER_BUF;
  allow_lds(reinterpret_cast<const void*>(&er_fused_kernel));
  const int cus = device_cus();
  const int grid = std::min(N * a.tiles_x * a.tiles_y, cus);
  ProfScope ps("er_fused_kernel", flops, bytes, s);
  hipLaunchKernelGGL(er_fused_kernel, dim3(grid), dim3(512), lds, s, a);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
