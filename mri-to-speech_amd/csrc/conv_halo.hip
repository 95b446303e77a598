// bf16 3x3 stride-1 convolution (TF-SAME pad 1) with LDS-resident weights and haloed input tiles:
// the EfficientNetV2 conv_stem-adjacent stages (timm ConvBnAct / EdgeResidual conv_exp at 128x128,
// 64x64 and 32x32; mri_acoustic_model.py:28-34 builds the backbone).
//
// Why a second conv kernel.  The implicit-GEMM pipeline (conv_gemm.hip) gathers a fresh A tile per
// K step, so every input pixel crosses L2 -> LDS nine times, and every output tile re-streams the
// full weight matrix: on these layers that fill, not the MFMA, set the time (~330 TF/s at best and
// ~1.1 TB/s on the 16-channel b0 layers).  Here a persistent workgroup owns one N tile of the
// weights for its whole life (DMA'd into LDS once, [k-step][n] rows of 64 B) and walks a strided
// list of 16-wide output tiles; per tile it DMAs the (TH+2) x 18 haloed input pixels once into one
// of two LDS buffers - the next tile's halo lands while the current one computes - and every MFMA
// fragment then comes from LDS: A = weights [n][k], B = input pixel (ty+ky, tx+kx) for the tap of
// the k-step.  64-byte LDS rows carry a source-side XOR swizzle (chunk ^ ((row >> 2) & 3)) as in
// conv_gemm.hip, so the 16-byte fragment reads stay bank-conflict free.
// Channel strides must be multiples of 32 (one or two 64-byte rows per pixel).
#include <algorithm>
#include <cstdio>

#include "conv_igemm.hpp"
#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_halo_zero[4];  // DMA source for padding pixels

constexpr int ROWB = 64;  // bytes per LDS row (32 bf16 = one k-step of one pixel)
constexpr int TW = 16;    // output tile width (one MFMA position subtile = one tile row)

__device__ __forceinline__ int swz(int row, int chunk) { return row * ROWB + ((chunk ^ ((row >> 2) & 3)) << 4); }

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void ld4f(const bf16_t* p, float* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xffff0000u);
}

struct HaloArgs {
  const bf16_t* x;
  const bf16_t* w;     // packed [n_pad][kp], k = tap * cs_in + c
  const float* bias;   // [n_pad]
  const bf16_t* res;   // residual (or null), layout of y
  bf16_t* y;
  int H, W;            // input = output size (stride 1)
  int cs_in, kc;       // kc = cs_in / 32 (64-byte rows per pixel)
  int kp, n_pad, cs_out;
  int tiles_x, tiles_y, m_tiles, n_tiles;
  int act;
  float act_slope;
};

template <int MTW, int NTW, int WM, int WN, int KC>
__global__ void __launch_bounds__(256) conv_halo_kernel(const HaloArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int BN = WN * NTW * 16;
  constexpr int TH = WM * MTW;        // tile rows (one 16-position subtile per row)
  constexpr int HW = TW + 2;          // halo width
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nsteps = a.kp / 32;
  // kc = 64-byte rows per pixel (cs_in / 32); kc = 0: cs_in = 16, two pixels per row
  const int hrows = KC ? (TH + 2) * HW * KC : (TH + 2) * HW / 2;
  const int hblocks = (hrows + 15) / 16;
  char* wbuf = smem;
  char* hbuf0 = smem + nsteps * BN * ROWB;
  const int hbytes = hblocks * 16 * ROWB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, r16 = lane & 15;
  const int lrow = lane >> 2;
  const int q = (lane & 3) ^ ((lane >> 4) & 3);  // logical 16-byte chunk this lane fetches

  const int nt = blockIdx.x % a.n_tiles;
  const int n0 = nt * BN;
  const int mstride = gridDim.x / a.n_tiles;
  int mt = blockIdx.x / a.n_tiles;

  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_halo_zero;
  asm volatile("" : "+s"(zpage));
  // ---- weights of this N tile -> LDS, once ----------------------------------------------------
  for (int blk = wave; blk < nsteps * BN / 16; blk += 4) {
    const int row = blk * 16 + lrow, st = row / BN, n = n0 + (row - st * BN);
    const void* src = n < a.n_pad ? (const void*)(a.w + (size_t)n * a.kp + st * 32 + q * 8) : zpage;
    dma16(src, wbuf + blk * 16 * ROWB);
  }

  auto issue_halo = [&](int m, char* hb) {
    const int img = m / (a.tiles_x * a.tiles_y), rem = m - img * (a.tiles_x * a.tiles_y);
    const int ty0 = (rem / a.tiles_x) * TH - 1, tx0 = (rem - (rem / a.tiles_x) * a.tiles_x) * TW - 1;
    const bf16_t* xi = a.x + (size_t)img * a.H * a.W * a.cs_in;
    for (int blk = wave; blk < hblocks; blk += 4) {
      const int row = blk * 16 + lrow;
      int hp, coff;  // halo pixel and channel offset of this lane's 16 bytes
      if (KC == 0) {
        hp = 2 * row + (q >> 1);
        coff = (q & 1) * 8;
      } else {
        hp = KC == 2 ? row >> 1 : row;
        coff = (KC == 2 ? row & 1 : 0) * 32 + q * 8;
      }
      const int hy = hp / HW, hx = hp - (hp / HW) * HW;
      const int iy = ty0 + hy, ix = tx0 + hx;
      const void* src = zpage;
      if (row < hrows && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        src = xi + ((size_t)iy * a.W + ix) * a.cs_in + coff;
      dma16(src, hb + blk * 16 * ROWB);
    }
  };

  if (mt < a.m_tiles) issue_halo(mt, hbuf0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int it = 0; mt < a.m_tiles; mt += mstride, ++it) {
    char* hb = hbuf0 + (it & 1) * hbytes;
    if (mt + mstride < a.m_tiles) issue_halo(mt + mstride, hbuf0 + ((it + 1) & 1) * hbytes);

    f32x4 acc[NTW][MTW];
#pragma unroll
    for (int ni = 0; ni < NTW; ++ni)
#pragma unroll
      for (int mi = 0; mi < MTW; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int st = 0; st < nsteps; ++st) {
      // cs_in = 16: a k-step spans taps 2st (lanes g < 2) and 2st+1; the pad tap 9 (zero
      // weights) reads tap 0's pixel so the product stays finite
      int tap = KC == 0 ? 2 * st + (g >> 1) : (KC == 2 ? st >> 1 : st);
      if (tap > 8) tap = 0;
      const int kc = KC == 2 ? st & 1 : 0;
      const int ky = tap / 3, kx = tap - (tap / 3) * 3;
      bf16x8 af[NTW], bx[MTW];
#pragma unroll
      for (int ni = 0; ni < NTW; ++ni)
        af[ni] = *reinterpret_cast<const bf16x8*>(wbuf + swz(st * BN + wn * NTW * 16 + ni * 16 + r16, g));
#pragma unroll
      for (int mi = 0; mi < MTW; ++mi) {
        const int ty = wm * MTW + mi;
        const int p = (ty + ky) * HW + r16 + kx;
        const int off = KC == 0 ? swz(p >> 1, ((p & 1) << 1) | (g & 1)) : swz(p * KC + kc, g);
        bx[mi] = *reinterpret_cast<const bf16x8*>(hb + off);
      }
#pragma unroll
      for (int ni = 0; ni < NTW; ++ni)
#pragma unroll
        for (int mi = 0; mi < MTW; ++mi)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ni], bx[mi], acc[ni][mi], 0, 0, 0);
    }
    // residual = this block's input (cs_in == cs_out): take it from the halo tile now, before the
    // barrier releases the buffer to the next prefetch
    uint2 rres[NTW][MTW];
    const bool res_lds = KC == 0 && a.res == a.x;  // cs_in == cs_out == 16 (b0 skip)
    if (KC == 0 && res_lds) {
#pragma unroll
      for (int mi = 0; mi < MTW; ++mi)
#pragma unroll
        for (int ni = 0; ni < NTW; ++ni) {
          const int n4 = n0 + wn * NTW * 16 + ni * 16 + 4 * g;
          const int p = (wm * MTW + mi + 1) * HW + r16 + 1;
          const int off = KC == 0 ? swz(p >> 1, ((p & 1) << 1) | (n4 >> 3)) + (n4 & 7) * 2
                                    : swz(p * KC + (n4 >> 5), (n4 & 31) >> 3) + (n4 & 7) * 2;
          rres[ni][mi] = n4 < a.cs_in ? *reinterpret_cast<const uint2*>(hb + off) : make_uint2(0, 0);
        }
    }
    // the next halo has landed (it had the whole K loop) and every wave is done with this one
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // ---- epilogue: 4 consecutive channels of one position per lane ----------------------------
    const int img = mt / (a.tiles_x * a.tiles_y), rem = mt - img * (a.tiles_x * a.tiles_y);
    const int oy0 = (rem / a.tiles_x) * TH, ox = (rem - (rem / a.tiles_x) * a.tiles_x) * TW + r16;
#pragma unroll
    for (int mi = 0; mi < MTW; ++mi) {
      const int oy = oy0 + wm * MTW + mi;
      if (oy >= a.H || ox >= a.W) continue;
      const size_t orow = ((size_t)img * a.H * a.W + (size_t)oy * a.W + ox) * a.cs_out;
#pragma unroll
      for (int ni = 0; ni < NTW; ++ni) {
        const int n4 = n0 + wn * NTW * 16 + ni * 16 + 4 * g;
        if (n4 >= a.cs_out) continue;
        const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
        float v[4] = {acc[ni][mi][0] + bb.x, acc[ni][mi][1] + bb.y, acc[ni][mi][2] + bb.z, acc[ni][mi][3] + bb.w};
        if (a.act == ACT_SILU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = silu(v[j]);
        } else if (a.act == ACT_LRELU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * a.act_slope;
        }
        if (KC == 0 && res_lds) {
          const uint2 u = rres[ni][mi];
          v[0] += __uint_as_float(u.x << 16);
          v[1] += __uint_as_float(u.x & 0xffff0000u);
          v[2] += __uint_as_float(u.y << 16);
          v[3] += __uint_as_float(u.y & 0xffff0000u);
        } else if (a.res) {
          float r[4];
          ld4f(a.res + orow + n4, r);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] += r[j];
        }
        uint2 u;
        u.x = pack_bf16x2(v[0], v[1]);
        u.y = pack_bf16x2(v[2], v[3]);
        *reinterpret_cast<uint2*>(a.y + orow + n4) = u;
      }
    }
  }
}

int num_cus() {
  const int n = device_cus();
  return n;
}

template <int MTW, int NTW, int WM, int WN, int KC>
bool launch_cfg(const ConvArgs& c, hipStream_t s, double flops, double bytes) {
  constexpr int BN = WN * NTW * 16, TH = WM * MTW;
  HaloArgs a;
  a.x = static_cast<const bf16_t*>(c.x);
  a.w = static_cast<const bf16_t*>(c.w);
  a.bias = c.bias;
  a.res = static_cast<const bf16_t*>(c.res);
  a.y = static_cast<bf16_t*>(c.y);
  a.H = c.OH;
  a.W = c.OW;
  a.cs_in = c.cs_in;
  a.kc = c.cs_in / 32;  // 0 for cs_in = 16
  a.kp = c.kp;
  a.n_pad = c.n_pad;
  a.cs_out = c.cs_out;
  a.tiles_x = ceil_div(c.OW, TW);
  a.tiles_y = ceil_div(c.OH, TH);
  const int nimg = c.M / (c.OH * c.OW);
  a.m_tiles = nimg * a.tiles_x * a.tiles_y;
  a.n_tiles = ceil_div(c.cs_out, BN);
  a.act = c.act;
  a.act_slope = c.act_slope;
  const int hrows = a.kc ? (TH + 2) * (TW + 2) * a.kc : (TH + 2) * (TW + 2) / 2;
  const int hblocks = ceil_div(hrows, 16);
  const size_t lds = (size_t)(a.kp / 32) * BN * ROWB + 2 * (size_t)hblocks * 16 * ROWB;
  if (lds > 160 * 1024) return false;
  allow_lds(reinterpret_cast<const void*>(&conv_halo_kernel<MTW, NTW, WM, WN, KC>));
  const int per_cu = std::max(1, (int)((160 * 1024) / lds));
  int wgs = std::min(a.m_tiles * a.n_tiles, num_cus() * std::min(per_cu, 4));
  wgs = std::max(a.n_tiles, wgs / a.n_tiles * a.n_tiles);
  char name[64];
  snprintf(name, sizeof(name), "conv_halo_kernel<%d, %d, %d, %d, %d>", MTW, NTW, WM, WN, KC);
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((conv_halo_kernel<MTW, NTW, WM, WN, KC>), dim3(wgs), dim3(256), lds, s, a);
  M2S_HIP(hipGetLastError());
  return true;
}

}  // namespace

bool conv_halo_supported(const ConvArgs& a) {
  return a.kind == KIND_CONV2D && a.ks == 3 && a.stride == 1 && a.ntaps == 9 && a.IH == a.OH && a.IW == a.OW &&
         a.pad_t == 1 && a.pad_l == 1 && ((a.cs_in == 32 && a.kp == 9 * 32) || (a.cs_in == 16 && a.kp == 10 * 16)) &&
         a.in_xform == IN_NONE && !a.accum && a.cs_out <= 256;
}

void launch_conv_halo(const ConvArgs& a, hipStream_t s, double flops, double bytes) {
  M2S_CHECK(conv_halo_supported(a), "conv_halo: unsupported conv");
  // Tile shapes measured with tools/halo_bench.hip (1920 frames): 16x16 output tiles; 64-channel
  // N tiles beat 128 (the 128-wide tile needs 1 wave/SIMD: 1.81 vs 1.28 ms on b1 conv_exp) and
  // 32 (1.61 ms); 8x16 tiles lose to 16x16 at every width.
  bool done;
  if (a.cs_in == 16)
    done = launch_cfg<4, 1, 4, 1, 0>(a, s, flops, bytes);  // b0 16 -> 16
  else if (a.cs_out <= 16)
    done = launch_cfg<4, 1, 4, 1, 1>(a, s, flops, bytes);  // b0 32 -> 16
  else
    done = launch_cfg<4, 4, 4, 1, 1>(a, s, flops, bytes);  // b1 32 -> 128 (two 64-wide N tiles)
  M2S_CHECK(done, "conv_halo: LDS budget");
}

}  // namespace m2s
