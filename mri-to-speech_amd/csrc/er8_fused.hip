// Fused EdgeResidual block of the fp8 engines on e4m3 operands, stride 1 with skip, 32 -> 128 -> 32
// channels (timm EdgeResidual conv_exp 3x3 + bn1 + SiLU -> conv_pwl 1x1 + bn2 -> + shortcut:
// tf_efficientnetv2_b2 blocks.1.1/.2 at 64x64, built by mri_acoustic_model.py:28-34).
//
// er_fused.hip's dataflow (the 128-channel map never leaves the registers) on the block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales; K = 128 per instruction, 2x the bf16 rate):
//   conv_exp: K = (tap, input channel) in groups of four taps, 3 MFMAs per (16 channels, 16 pixels)
//     (taps 0-3, 4-7, 8 + three zero taps) instead of 9 bf16 ones.  A lane's 32 B of a B fragment are one
//     tap's 32 input channels of one pixel: lane (r16, g) reads pixel (row + ky, r16 + kx) of tap 4q + g
//     from an e4m3 copy of the haloed rows (two 16-channel planes, 16 B per pixel: a fragment read of 16
//     consecutive pixels is bank-conflict free), or a zero slot for the padding taps.
//   weights: e4m3 of W / s with s = amax / 448 per output channel (host), the epilogues multiply by s.
//   conv_exp -> conv_pwl: a lane's accumulators hold channels 16 nt + 4 g + e (nt < 8, e < 4) of its
//     pixel; after scale + bias + SiLU their 32 e4m3 bytes, in (nt, e) order, are the lane's B fragment of
//     conv_pwl's single K = 128 step, with the host packing conv_pwl's K in the same permuted order
//     (k-slot 32 g + 4 nt + e = mid channel 16 nt + 4 g + e).
//
// Schedule.  On e4m3 the MFMAs are the smaller half of a tile: the epilogue (scale, bias, SiLU and the e4m3
// packing of 128 channels per pixel) is ~570 VALU instructions a wave against 52 MFMAs.  With every wave in
// the same phase (one barrier per tile) a SIMD's two waves ran them back to back (the first form: 5.8 ms per
// 8000 frames, no faster than bf16 er_fused).  Here the workgroup's two halves (waves 0-3, 4-7: one wave of
// each on every SIMD) run one phase apart on their own 8 x 16 tiles: phase p, half h computes conv_exp of its
// tile (p - h) / 2 or the epilogue of tile (p - h - 1) / 2, so on each SIMD one wave's MFMAs run beside the
// other's VALU.  One barrier per phase.  Each half double-buffers its tiles' bf16 halo (10 x 18 x 32, LDS-DMA
// two phases ahead; it also serves the bf16 shortcut); each wave converts the 4 halo rows it reads to its own
// e4m3 rows (no barrier between the conversion and the fragment reads).  The e4m3 conv_exp fragments (48 KB)
// are DMA'd once.  LDS reads are inline asm consumed behind counted lgkmcnt waits (a plain ds_read after an
// LDS-DMA makes hipcc drain the DMA in flight), the conv_exp weight fragments three deep.
#include <algorithm>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int E8M0_ONE = 0x7f7f7f7f;

__device__ __attribute__((aligned(16))) uint4 g_er8_zero[4];  // DMA source for padding pixels

constexpr int E8_TW = 16, E8_TH = 8;                        // tile: 8 rows x 16 pixels per half-workgroup
constexpr int E8_HW = E8_TW + 2, E8_HH = E8_TH + 2;         // halo 10 x 18
constexpr int E8_HPIX = E8_HH * E8_HW;                      // 180 pixels
constexpr int E8_PLANE = 192 * 16;                          // bf16 halo: 3 DMA pieces per 8-channel plane
constexpr int E8_BUF = 4 * E8_PLANE;                        // 4 planes (12 KB)
constexpr int E8_WEXP = 3 * 8 * 2 * 1024;                   // conv_exp fragments [q][nt][half][lane][16 B]
constexpr int E8_WP8 = 4 * E8_HW * 16;                      // a wave's e4m3 plane: 4 halo rows x 18 pixels
constexpr int E8_W8 = 2 * E8_WP8;                           // two 16-channel planes per wave (2304 B)
constexpr int E8_ZS = 8 * E8_W8;                            // zero slot (32 B) after the 8 waves' rows
constexpr int E8_H8 = E8_ZS + 64;
// with an e4m3 input from the producer (x8): [half][2] e4m3 halo buffers of two 16-channel planes instead
constexpr int E8_P8 = 192 * 16;                             // e4m3 plane: 3 DMA pieces of 64 pixels
constexpr int E8_XBUF = 2 * E8_P8;
constexpr int E8_ZSX = 4 * E8_XBUF;
constexpr int E8_H8X = E8_ZSX + 64;
constexpr int e8_lds(bool x8) { return E8_WEXP + 4 * E8_BUF + (x8 ? E8_H8X : E8_H8) + 2 * 128 * 4; }  // + scales, biases

struct Er8Args {
  const bf16_t* x;       // (N, H, W, 32)
  const uint8_t* wexp;   // e4m3 [3][8][2][64][16]
  const float* sexp;     // [128] conv_exp per-channel scales
  const float* bexp;     // [128] bn1 bias
  const uint8_t* wpwl;   // e4m3 [2][2][64][16] (permuted K)
  const float* spwl;     // [32]
  const float* bpwl;     // [32]
  bf16_t* y;             // (N, H, W, 32)
  const uint8_t* x8;     // X8: the input as e4m3 bytes (N, H, W, 32), written by the producer block
  uint8_t* y8;           // Y8: e4m3 of the stored y (the next er8 block's x8)
  int N, H, W, tiles_x, tiles_y;  // 8 x 16 tiles
};

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ i32x8 cat8(u32x4 a, u32x4 b) {
  return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

template <bool X8, bool Y8>
__global__ void __launch_bounds__(512, 1) er8_fused_kernel(const Er8Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;                        // conv_exp fragments
  char* hbuf = smem + E8_WEXP;            // [half][2] bf16 halo buffers
  char* h8 = hbuf + 4 * E8_BUF;           // per-wave e4m3 halo rows (X8: [half][2] e4m3 halos) + zero slot
  float* sb = reinterpret_cast<float*>(h8 + (X8 ? E8_H8X : E8_H8));  // [128] scales, [128] biases
  constexpr int ZS = X8 ? E8_ZSX : E8_ZS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, lw = wave & 3;  // lw: output rows 2 lw, 2 lw + 1 of the half's tile
  const int g = lane >> 4, r16 = lane & 15;
  const int tpi = a.tiles_x * a.tiles_y, ntiles = a.N * tpi;
  // the half's tiles: T(j) = (j * gridDim.x + blockIdx.x) * 2 + half; J = how many are < ntiles
  auto tile_of = [&](int h, int j) { return (j * (int)gridDim.x + (int)blockIdx.x) * 2 + h; };
  auto count = [&](int h) {
    const int t0 = (int)blockIdx.x * 2 + h, step = 2 * (int)gridDim.x;
    return t0 < ntiles ? (ntiles - 1 - t0) / step + 1 : 0;
  };
  const int J = count(half), J0 = count(0);

  // this wave's 3 halo pieces of tile T: plane c, 64-pixel block pb
  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_er8_zero;
  asm volatile("" : "+s"(zpage));
  auto issue_halo = [&](int T, char* buf) {
    const int n = T / tpi, tr = T - n * tpi;
    const int ty0 = (tr / a.tiles_x) * E8_TH - 1, tx0 = (tr - (tr / a.tiles_x) * a.tiles_x) * E8_TW - 1;
    const bf16_t* xi = a.x + (size_t)n * a.H * a.W * 32;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int piece = lw * 3 + j, c = piece / 3, pb = piece - c * 3;
      const int p = pb * 64 + lane, hy = p / E8_HW, hx = p - hy * E8_HW;
      const int iy = ty0 + hy, ix = tx0 + hx;
      const void* src = zpage;
      if (p < E8_HPIX && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) src = xi + ((size_t)iy * a.W + ix) * 32 + c * 8;
      dma16(src, buf + c * E8_PLANE + pb * 1024);
    }
  };
  char* hb_half = hbuf + half * 2 * E8_BUF;
  // X8: this wave's pieces (lw, lw + 4 < 6) of tile T's e4m3 halo: plane pl, 64-pixel block pb
  auto issue_halo8 = [&](int T, char* buf) {
    const int n = T / tpi, tr = T - n * tpi;
    const int ty0 = (tr / a.tiles_x) * E8_TH - 1, tx0 = (tr - (tr / a.tiles_x) * a.tiles_x) * E8_TW - 1;
    const uint8_t* xi = a.x8 + (size_t)n * a.H * a.W * 32;
    for (int piece = lw; piece < 6; piece += 4) {
      const int pl = piece / 3, pb = piece - pl * 3;
      const int p = pb * 64 + lane, hy = p / E8_HW, hx = p - hy * E8_HW;
      const int iy = ty0 + hy, ix = tx0 + hx;
      const void* src = zpage;
      if (p < E8_HPIX && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) src = xi + ((size_t)iy * a.W + ix) * 32 + pl * 16;
      dma16(src, buf + pl * E8_P8 + pb * 1024);
    }
  };
  char* x8_half = h8 + half * 2 * E8_XBUF;

  // ---- once: conv_exp fragments -> LDS (6 pieces per wave); conv_pwl fragments, its scales and biases ->
  // VGPRs; conv_exp scales and biases -> LDS; the zero slot; both halves' first halo
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int piece = wave * 6 + j;
    dma16(a.wexp + (size_t)piece * 1024 + lane * 16, wl + piece * 1024);
  }
  i32x8 wp[2];
#pragma unroll
  for (int on = 0; on < 2; ++on) {
    const u32x4 h0 = *reinterpret_cast<const u32x4*>(a.wpwl + ((size_t)(on * 2 + 0) * 64 + lane) * 16);
    const u32x4 h1 = *reinterpret_cast<const u32x4*>(a.wpwl + ((size_t)(on * 2 + 1) * 64 + lane) * 16);
    wp[on] = cat8(h0, h1);
  }
  float4 sp[2], bp[2];
#pragma unroll
  for (int on = 0; on < 2; ++on) {
    sp[on] = *reinterpret_cast<const float4*>(a.spwl + on * 16 + 4 * g);
    bp[on] = *reinterpret_cast<const float4*>(a.bpwl + on * 16 + 4 * g);
  }
  if (tid < 128) sb[tid] = a.sexp[tid];
  else if (tid < 256) sb[tid] = a.bexp[tid - 128];
  else if (tid < 260) *reinterpret_cast<uint4*>(h8 + ZS + (tid - 256) * 16) = make_uint4(0u, 0u, 0u, 0u);
  if (J > 0) issue_halo(tile_of(half, 0), hb_half);
  if (X8 && J > 0) issue_halo8(tile_of(half, 0), x8_half);
  wait_vm<0>();
  __syncthreads();

  const uint32_t wl0 = lds_off(wl) + lane * 16, sb0 = lds_off(sb);
  const uint32_t w80 = lds_off(h8) + wave * E8_W8, zs0 = lds_off(h8) + ZS;
  f32x4 acc[2][8];
  // phases: half 0 conv_exp(j) at 2 j, epilogue(j) at 2 j + 1; half 1 one phase later; J0 >= J (half 1)
  const int nphase = 2 * J0 + 1;
  for (int p = 0; p < nphase; ++p) {
    const int ph = p - half;
    if (ph >= 0 && (ph & 1) == 0 && (ph >> 1) < J) {
      // ================= conv_exp of tile j =================
      const int j = ph >> 1;
      const uint32_t hb0 = lds_off(hb_half + (j & 1) * E8_BUF);
      if (j + 1 < J) issue_halo(tile_of(half, j + 1), hb_half + ((j + 1) & 1) * E8_BUF);  // its epilogue read
      // buffer (j + 1) & 1 last in phase p - 1
      if (X8 && j + 1 < J) issue_halo8(tile_of(half, j + 1), x8_half + ((j + 1) & 1) * E8_XBUF);  // read in p - 2
      const uint32_t xb0 = lds_off(x8_half + (j & 1) * E8_XBUF);

      // without x8: this wave's halo rows 2 lw .. 2 lw + 3 as e4m3: item = (row, pixel, 16-channel plane)
      for (int w = lane; w < (X8 ? 0 : 4 * E8_HW * 2); w += 64) {
        const int pl = w & 1, rp = w >> 1;  // rp = local row * 18 + pixel
        const int hp = 2 * lw * E8_HW + rp;  // halo pixel
        u32x4 u0, u1;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(u0), "=&v"(u1)
                     : "v"(hb0 + (2 * pl) * E8_PLANE + hp * 16), "v"(hb0 + (2 * pl + 1) * E8_PLANE + hp * 16)
                     : "memory");
        float f[16];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f[2 * e] = __uint_as_float(u0[e] << 16);
          f[2 * e + 1] = __uint_as_float(u0[e] & 0xffff0000u);
          f[8 + 2 * e] = __uint_as_float(u1[e] << 16);
          f[8 + 2 * e + 1] = __uint_as_float(u1[e] & 0xffff0000u);
        }
        const uint2 q0 = e4m3x8(f), q1 = e4m3x8(f + 8);
        const u32x4 q = {q0.x, q0.y, q1.x, q1.y};
        asm volatile("ds_write_b128 %0, %1" ::"v"(w80 + pl * E8_WP8 + rp * 16), "v"(q) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's own rows: no barrier needed

      // B fragments of all 3 tap groups, then the 24 (q, nt) weight fragments three deep
      u32x4 b0[2][3], b1[2][3];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int tap = 4 * q + g, ky = tap / 3, kx = tap - (tap / 3) * 3;
          const int rp = (i + ky) * E8_HW + r16 + kx, hp = 2 * lw * E8_HW + rp;
          const uint32_t b = X8 ? xb0 + hp * 16 : w80 + rp * 16, pl1 = X8 ? E8_P8 : E8_WP8;
          const uint32_t o0 = tap < 9 ? b : zs0, o1 = tap < 9 ? b + pl1 : zs0 + 16;
          asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3" : "=&v"(b0[i][q]), "=&v"(b1[i][q]) : "v"(o0), "v"(o1) : "memory");
        }
      u32x4 a0[3], a1[3];
      auto read_a = [&](int f) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024"
                     : "=&v"(a0[f % 3]), "=&v"(a1[f % 3])
                     : "v"(wl0 + f * 2048)
                     : "memory");
      };
      read_a(0);
      read_a(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      i32x8 bx[2][3];
#pragma unroll
      for (int f = 0; f < 24; ++f) {
        const int q = f / 8, nt = f % 8;
        if (f + 2 < 24) read_a(f + 2);
        // reads younger than A(f): A(f + 1), A(f + 2) (2 each, while issued)
        if (f + 2 < 24) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a0[f % 3]), "+v"(a1[f % 3]));
        else if (f + 1 < 24) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a0[f % 3]), "+v"(a1[f % 3]));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0[f % 3]), "+v"(a1[f % 3]));
        if (nt == 0) {  // the B reads were issued before every A read
          asm volatile("" : "+v"(b0[0][q]), "+v"(b1[0][q]), "+v"(b0[1][q]), "+v"(b1[1][q]));
          bx[0][q] = cat8(b0[0][q], b1[0][q]);
          bx[1][q] = cat8(b0[1][q], b1[1][q]);
        }
        const i32x8 af = cat8(a0[f % 3], a1[f % 3]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][nt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bx[i][q], acc[i][nt], 0, 0, 0, E8M0_ONE, 0,
                                                                        E8M0_ONE);
      }
    } else if (ph >= 1 && (ph & 1) == 1 && (ph >> 1) < J) {
      // ================= epilogue of tile j =================
      const int j = ph >> 1, T = tile_of(half, j);
      const uint32_t hb0 = lds_off(hb_half + (j & 1) * E8_BUF);
      // scale + bias + SiLU -> e4m3 B fragment of conv_pwl (dword nt = channels 16 nt + 4 g + e)
      i32x8 mid[2];
#pragma unroll
      for (int nt = 0; nt < 8; nt += 2) {
        u32x4 s0, s1, c0, c1;
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:512\n\t"
                     "ds_read_b128 %3, %4 offset:576\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(s0), "=&v"(s1), "=&v"(c0), "=&v"(c1)
                     : "v"(sb0 + (nt * 16 + 4 * g) * 4)
                     : "memory");
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = silu_e4m3(acc[i][nt][e] * __uint_as_float(s0[e]) + __uint_as_float(c0[e]));
            v[4 + e] = silu_e4m3(acc[i][nt + 1][e] * __uint_as_float(s1[e]) + __uint_as_float(c1[e]));
          }
          const uint2 m = e4m3x8_nosat(v);
          mid[i][nt] = (int)m.x;
          mid[i][nt + 1] = (int)m.y;
        }
      }
      // conv_pwl (one K = 128 MFMA per 16 output channels) + scale + bn2 bias + shortcut
      const int n = T / tpi, tr = T - n * tpi;
      const int oy0 = (tr / a.tiles_x) * E8_TH, ox = (tr - (tr / a.tiles_x) * a.tiles_x) * E8_TW + r16;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ry = 2 * lw + i, oy = oy0 + ry;
#pragma unroll
        for (int on = 0; on < 2; ++on) {
          const f32x4 o = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wp[on], mid[i], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0,
                                                                           0, E8M0_ONE, 0, E8M0_ONE);
          const int c4 = on * 16 + 4 * g;
          uint2 r;
          asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=v"(r)
                       : "v"(hb0 + (c4 >> 3) * E8_PLANE + ((ry + 1) * E8_HW + r16 + 1) * 16 + (c4 & 7) * 2)
                       : "memory");
          const float v0 = o[0] * sp[on].x + bp[on].x + __uint_as_float(r.x << 16);
          const float v1 = o[1] * sp[on].y + bp[on].y + __uint_as_float(r.x & 0xffff0000u);
          const float v2 = o[2] * sp[on].z + bp[on].z + __uint_as_float(r.y << 16);
          const float v3 = o[3] * sp[on].w + bp[on].w + __uint_as_float(r.y & 0xffff0000u);
          // every tile is whole (H a multiple of 8, W of 16): exactly 4 stores (8 with y8) per wave per tile
          const size_t px = ((size_t)n * a.H + oy) * a.W + ox;
          const uint2 yb = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
          *reinterpret_cast<uint2*>(a.y + px * 32 + c4) = yb;
          if (Y8) *reinterpret_cast<uint32_t*>(a.y8 + px * 32 + c4) = e4m3x4_bf16(yb);
        }
      }
      // the next tile's halo (issued in the conv_exp phase of tile j, before these stores) must have landed
      // for every wave of the half by the next phase: the barrier below follows each wave's own wait
      if (Y8) wait_vm<8>();
      else wait_vm<4>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  wait_vm<0>();
}

}  // namespace

bool er8_fused_supported(int H, int W, int cin, int mid, int cout) {
  return cin == 32 && mid == 128 && cout == 32 && H % E8_TH == 0 && W % E8_TW == 0 && H > 0 && W > 0;
}

void launch_er8_fused(const bf16_t* x, int N, int H, int W, const uint8_t* wexp, const float* sexp, const float* bexp,
                      const uint8_t* wpwl, const float* spwl, const float* bpwl, bf16_t* y, double flops, double bytes,
                      hipStream_t s, const uint8_t* x8, uint8_t* y8) {
  M2S_CHECK(er8_fused_supported(H, W, 32, 128, 32) && N > 0, "er8_fused: unsupported shape");
  Er8Args a;
  a.x = x;
  a.wexp = wexp;
  a.sexp = sexp;
  a.bexp = bexp;
  a.wpwl = wpwl;
  a.spwl = spwl;
  a.bpwl = bpwl;
  a.y = y;
  a.x8 = x8;
  a.y8 = y8;
  a.N = N;
  a.H = H;
  a.W = W;
  a.tiles_x = W / E8_TW;
  a.tiles_y = H / E8_TH;
  M2S_CHECK(x8 || !y8, "er8_fused: an e4m3 output needs the e4m3 input path");
  auto k = x8 ? (y8 ? er8_fused_kernel<true, true> : er8_fused_kernel<true, false>) : er8_fused_kernel<false, false>;
  allow_lds(reinterpret_cast<const void*>(k));
  // two tiles per workgroup in flight (one per half)
  const int grid = std::min((N * a.tiles_x * a.tiles_y + 1) / 2, device_cus());
  ProfScope ps("er8_fused_kernel", flops, bytes + (x8 ? N * (double)H * W * 32 : 0.0) + (y8 ? N * (double)H * W * 32 : 0.0), s);
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), e8_lds(x8 != nullptr), s, a);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
