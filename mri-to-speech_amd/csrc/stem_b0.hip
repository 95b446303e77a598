// Fused encoder front (bf16): conv_stem 3x3/s2 (TF-SAME) + bn1 + SiLU  ->  blocks.0.0 ConvBnAct 3x3
// 32->16 + SiLU  ->  blocks.0.1 ConvBnAct 3x3 16->16 + SiLU + skip, for one 16 x TH output tile per
// workgroup (timm tf_efficientnetv2_b2 conv_stem/bn1/blocks.0; mri_acoustic_model.py:28-46 builds it).
//
// Unfused, the stem writes its 32-channel map (2 MB per 256x256 frame in bf16), blocks.0.0 reads it
// back and writes 16 channels, blocks.0.1 reads those twice (conv + skip) and writes again: ~8.5 GB
// of HBM traffic per 1920 frames.  Here only the fp32 frame is read and the blocks.0.1 output
// written (1.5 GB); the two intermediate maps live in LDS with the halos the next 3x3 needs:
//   S = stem output on (TH+4) x 20 pixels (32 ch), A = blocks.0.0 output on (TH+2) x 18 (16 ch).
// Pixels outside the image are stored as exact zeros: they are the next conv's zero padding.
//
//   phase 1  stem on MFMA 16x16x32 bf16, split into three terms (hi*hi + hi*lo + lo*hi, both engines):
//            A = the 32 x 9 weights resident in VGPRs, B = 16 S pixels x their 9 frame values, prefetched a
//            tile ahead in registers.  K = 32 holds tap row ky at k = 8 ky .. 8 ky + 2 (lane group g = ky < 3
//            carries the three taps of one frame row; the other k are zero), so a lane keeps 3 values a pixel
//   phase 2  blocks.0.0 on MFMA 16x16x32 bf16: weights (16 x 288) resident in VGPRs as 9 A
//            fragments, B = 16 A-pixels x 32 channels of one tap from S
//   phase 3  blocks.0.1 likewise (16 x 160: two taps of 16 channels per K step), + skip from A.
// Both LDS images are planar ([16-byte chunk][pixel]) so a B-fragment read of 16 consecutive
// pixels is bank-conflict free at any tap offset (see mrf_fused.hip).
// Split fp32 (SP = 1, m2s_common.hpp sp_t): S and A keep a hi and a lo plane set (double the LDS,
// two workgroups per CU), the conv weights come as [hi kp | lo kp] rows (A fragments hi and lo
// resident), every product is the three MFMA terms and y is written as (N, OH, OW, [hi 16 | lo 16]).
//
// Persistent: a workgroup per CU slot walks a sequence of tiles with its weights resident (loaded
// once), and the frame pixels of its next tile's phase 1 are loaded into registers right after the
// current tile's phase 1 (they land while phases 2 and 3 run).  Launched one workgroup per tile, a
// tile's life was a chain of exposed latencies (weights from L2, frame from HBM, two barriers): 16 us
// per workgroup at two per CU.  Tiles are dealt per XCD in contiguous ranges, so the workgroups of
// one XCD work on neighbouring tiles of the same frames at any time (shared halos stay in its L2).
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

#ifndef STEM_P2_DB
#define STEM_P2_DB 0  // phase 2's B fragments double-buffered across taps (spills at 256 VGPRs: off)
#endif
constexpr int SB_TW = 16;           // output tile width (one MFMA position subtile per tile row)
constexpr int SB_SW = SB_TW + 4;    // S row width
constexpr int SB_AV = SB_TW + 2;    // A row width (valid pixels)
// A rows are stored at the S pitch: a phase-2 subtile of 16 consecutive A positions then reads 16
// consecutive S pixels for every tap (conflict-free planes).  At the 18-pixel pitch a subtile crossed
// an A row break and its S pixels jumped by 2 there: 2-way bank conflicts on most phase-2 reads
// (SQ_LDS_BANK_CONFLICT 1.4x the LDS-active cycles).  Columns 18-19 of A are computed and ignored.
constexpr int SB_AW = SB_SW;

struct StemB0Args {
  const float* frames;  // (N, H, W) fp32
  const float* w9;      // stem [32][9] (grey repeat folded), BN folded
  const float* b9;      // [32]
  const bf16_t* w0;     // blocks.0.0 packed [>=16][kp0 = 288] (SP: [hi kp0 | lo kp0] rows)
  const float* b0;
  const bf16_t* w1;     // blocks.0.1 packed [>=16][kp1 = 160] (SP: [hi kp1 | lo kp1] rows)
  const float* b1;
  bf16_t* y;            // (N, OH, OW, 16) (SP: (N, OH, OW, [hi 16 | lo 16]))
  int N, H, W, OH, OW, pad_t, pad_l, kp0, kp1, tiles_x, tiles_y;
  int per_xcd;  // units (strip part) per XCD range (gridDim.x is a multiple of 8)
  int parts, tpp;  // a strip's tile rows cut into `parts` ranges of tpp rows (small batches; 1 = whole strips)
  unsigned long long* trace;  // diagnostic build (-DIRWS_TRACE): per-phase s_memtime stamps, else null
};

__device__ __forceinline__ bf16x8 frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ f32x4 mma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

template <int TH, int SP>
__global__ void __launch_bounds__(256, SP ? 2 : 3) stem_b0_kernel(const StemB0Args a) {
  static_assert(TH == 16, "line buffer: 16 new S / A rows per tile");
  // Plane index of S pixel / A position (row, col) = OFS + row * SB_SW + col: the pad makes A row 2 start
  // on a 16-position subtile, so a strip's later tiles recompute exactly A rows 2..17 (20 subtiles).
  constexpr int OFS = 8;
  constexpr int SH = TH + 4, AH = TH + 2;
  constexpr int SPIX = OFS + SH * SB_SW, APIX = OFS + AH * SB_AW;
  static_assert(APIX % 16 == 0 && (OFS + 2 * SB_AW) % 16 == 0, "A subtiles");
  constexpr int SPLANE = (SPIX * 16 + 255) / 256 * 256;      // bytes per S plane (4 planes)
  // A: four planes of 4 channels (8 bytes a position) per set, plane p at a4(p): blocks.0.0's epilogue
  // stores a 16-lane group's 16 positions as 128 contiguous bytes (with 8-channel planes the two halves
  // of a position interleaved and every store was 2-way bank-conflicted: 0.29 conflict cycles per LDS
  // instruction, profiles/r04ev2_sq_mfma.txt), and the plane offsets are 0 / 128 / 128 / 0 mod 256 bytes so
  // the paired 8-byte reads of blocks.0.1 (planes 0 + 2, 1 + 3) and of the skip (0 + 1, 2 + 3) land on
  // disjoint banks
  constexpr int A4 = (APIX * 8 + 255) / 256 * 256;           // bytes per 4-channel A plane, a multiple of 256
  constexpr int ASUB = APIX / 16;                             // A position subtiles of a strip's first tile
  constexpr int ASUB0 = (OFS + 2 * SB_AW) / 16;               // first subtile of A row 2 (later tiles)
  constexpr int AMS = (ASUB + 3) / 4;                         // subtiles per wave, at most
  constexpr int OMS = TH / 4;                                 // output subtiles (rows) per wave
  constexpr int SHIFT = TH * SB_SW;                           // carried rows move up by TH rows
  static_assert(SB_SW == SB_AW, "S and A share the pitch");
  constexpr int R = SP ? 2 : 1;  // plane sets: hi (+ lo)
  __shared__ __attribute__((aligned(16))) char sS[R * 4 * SPLANE + 256];  // + the overrun of columns 18-19
  constexpr int ALO = 4 * A4 + 256;                           // offset of the lo plane set
  __shared__ __attribute__((aligned(16))) char sA[R * ALO];
  constexpr int SLO = 4 * SPLANE;  // offset of the lo S plane set
  auto a4 = [](int p) { return p * A4 + ((p == 1 || p == 2) ? 128 : 0); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  // Strips = (image, 16-column tile column): a workgroup walks a strip's tiles top to bottom and keeps
  // the rows the next tile shares (S rows 16..19 -> 0..3, A rows 16..17 -> 0..1: halo recompute 1.56x ->
  // 1.25x of the stem, 1.44x -> 1.25x of blocks.0.0).  Strips of XCD x (= blockIdx % 8) are
  // [x * per_xcd, (x + 1) * per_xcd) (neighbouring columns of the same frames share one L2).
  // Units = (strip, part): part p is tile rows [p tpp, min((p + 1) tpp, tiles_y)); its first tile computes every S / A
  // row (no rows carried in), as a strip's first tile does.  Parts > 1 only where whole strips leave workgroup slots
  // idle (one clip: 240 strips for 512 slots).
  const int nunit = a.N * a.tiles_x * a.parts;
  const int gx = gridDim.x / 8, xcd = blockIdx.x % 8;
  const int s_end = min(nunit, (xcd + 1) * a.per_xcd);
  auto strip_of = [&](int u) { return u / a.parts; };
  auto ty_lo = [&](int u) { return (u - (u / a.parts) * a.parts) * a.tpp; };
  auto ty_hi = [&](int u) { return min(ty_lo(u) + a.tpp, a.tiles_y); };

  // ---- phase-1 work of a tile: S position subtiles j (16 S pixels OFS + 16 j ..), j = j0 + wave + 4 i: a
  // strip's first tile all 25 (rows 0..19), later tiles the 20 of rows 4..19 (j0 = 5; rows 0..3 are carried).
  // A lane's B operand: pixel r16 of its subtile, k = 8 g + kx = tap (ky = g, kx) for g < 3 and kx < 3, else 0.
  constexpr int SJ = SPIX / 16 - OFS / 16;  // 25 S subtiles
  static_assert(OFS % 16 == 8 || OFS % 16 == 0, "subtile base");
  constexpr int NPF = 5;                    // subtiles a wave prefetches (later tiles: exactly 5)
  // raw loads at clamped (always valid) addresses; the padding mask (3 bits) is applied when the values are used,
  // so nothing consumes a prefetched load before the next tile (a select right after each load made the compiler
  // wait for every one of them, ~4k cycles of exposed HBM latency a tile)
  auto load3 = [&](float* x3, int st, int ty, int j) -> unsigned {
    const int n = st / a.tiles_x, tx0 = (st - n * a.tiles_x) * SB_TW, ty0 = ty * TH;
    const float* fr = a.frames + (size_t)n * a.H * a.W;
    const int i = 16 * j + r16, sy = i / SB_SW, sx = i - (i / SB_SW) * SB_SW;
    const int oy = ty0 - 2 + sy, ox = tx0 - 2 + sx;  // stem output pixel
    const int iy = oy * 2 - a.pad_t + g, ix0 = ox * 2 - a.pad_l;
    const bool ok = j < SJ && g < 3 && oy >= 0 && oy < a.OH && ox >= 0 && ox < a.OW && iy >= 0 && iy < a.H;
    // unconditional loads at clamped addresses, then the zero padding by select
    const float* row = fr + (size_t)min(max(iy, 0), a.H - 1) * a.W;
    unsigned m = 0;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ix0 + kx;
      x3[kx] = row[min(max(ix, 0), a.W - 1)];
      m |= (ok && ix >= 0 && ix < a.W) ? 1u << kx : 0u;
    }
    return m;
  };
  float xin[NPF][3];
  unsigned xm = 0;  // 3 mask bits per prefetched subtile
  auto load_in = [&](int u, int ty) {
    const int j0 = ty == ty_lo(u) ? 0 : 5;
    xm = 0;
#pragma unroll
    for (int i = 0; i < NPF; ++i) xm |= load3(xin[i], strip_of(u), ty, j0 + wave + 4 * i) << (3 * i);
  };
  int u = xcd * a.per_xcd + (int)blockIdx.x / 8, ty = ty_lo(u);
  if (u < s_end) load_in(u, ty);

  // resident weights of both convs (A fragments)
  bf16x8 wf0[9], wf1[5], wl0[SP ? 9 : 1], wl1[SP ? 5 : 1];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const bf16_t* w = a.w0 + (size_t)r16 * a.kp0 * R + k * 32 + 8 * g;
    wf0[k] = *reinterpret_cast<const bf16x8*>(w);
    if constexpr (SP) wl0[k] = *reinterpret_cast<const bf16x8*>(w + a.kp0);
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const bf16_t* w = a.w1 + (size_t)r16 * a.kp1 * R + k * 32 + 8 * g;
    wf1[k] = *reinterpret_cast<const bf16x8*>(w);
    if constexpr (SP) wl1[k] = *reinterpret_cast<const bf16x8*>(w + a.kp1);
  }
  // the stem's weights in LDS as the lanes' A-fragments, split once here: [channel tile][lane (g, r16)] the
  // bf16 hi and lo halves of the taps (ky = g, kx = 0..2) of channel ni * 16 + r16 and 0 (g = 3: zeros) in one
  // 16-byte entry, then the fp32 biases; a subtile reads its two fragments and biases instead of keeping them
  // in registers, which phase 2's resident weights leave none of
  __shared__ __attribute__((aligned(16))) uint32_t sw9[2 * 64 * 4 + 32];
  for (int i = tid; i < 2 * 64 + 32; i += 256) {
    if (i < 128) {
      const int ni = i >> 6, ln = i & 63, gg = ln >> 4;
      float wv[4] = {0.f, 0.f, 0.f, 0.f};
      if (gg < 3)
        for (int kx = 0; kx < 3; ++kx) wv[kx] = a.w9[(ni * 16 + (ln & 15)) * 9 + 3 * gg + kx];
      uint2 wh, wl;
      split4(wv, wh, wl);
      *reinterpret_cast<uint4*>(&sw9[i * 4]) = make_uint4(wh.x, wh.y, wl.x, wl.y);
    } else {
      sw9[512 + i - 128] = __float_as_uint(a.b9[i - 128]);
    }
  }
  const float4 bb0 = *reinterpret_cast<const float4*>(a.b0 + 4 * g);
  const float4 bb1 = *reinterpret_cast<const float4*>(a.b1 + 4 * g);
  __syncthreads();  // sw9

  auto copy16 = [&](char* base, int from, int to) {  // one 16-byte LDS chunk, hi (and lo) planes
    *reinterpret_cast<uint4*>(base + to) = *reinterpret_cast<const uint4*>(base + from);
  };

  int it = 0;  // tile iteration (diagnostic stamps)
  auto TR = [&](int k) {
#ifdef IRWS_TRACE
    if (a.trace && blockIdx.x == 0 && lane == 0 && it < 32) a.trace[(it * 4 + wave) * 8 + k] = __builtin_amdgcn_s_memtime();
#else
    (void)k;
#endif
  };
  while (u < s_end) {
    const int st = strip_of(u);
    const int n = st / a.tiles_x, tx0 = (st - n * a.tiles_x) * SB_TW, ty0 = ty * TH;
    const bool first = ty == ty_lo(u);
    TR(0);
    // ---- phase 1: stem (fp32 VALU) -> S -----------------------------------------------------
    // (S is free: every wave passed the previous tile's phase-2 barrier before reaching here.)
    {
      const int j0 = first ? 0 : 5;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const int j = j0 + wave + 4 * i;  // wave-uniform
        if (j >= SJ) break;
        float xl[3];
        const float* x3 = xin[i < NPF ? i : 0];
        unsigned m3 = (xm >> (3 * (i < NPF ? i : 0))) & 7u;
        if (i >= NPF) {  // a strip's first tile: its last rows, loaded now
          m3 = load3(xl, st, ty, j);
          x3 = xl;
        }
        const int px = OFS + 16 * j + r16;
        // a later tile's rows 16..19 move to 0..3 first (this wave's subtiles j >= 20: the copy's reads precede
        // its own writes in LDS order); lane (g, r16) = plane g of pixel r16
        if (!first && j >= 20) {
#pragma unroll
          for (int h = 0; h < R; ++h) copy16(sS + h * SLO + g * SPLANE, px * 16, (px - SHIFT) * 16);
        }
        const float x4[4] = {m3 & 1u ? x3[0] : 0.f, m3 & 2u ? x3[1] : 0.f, m3 & 4u ? x3[2] : 0.f, 0.f};
        uint2 xh, xlo;
        split4(x4, xh, xlo);
        const bf16x8 bh = __builtin_bit_cast(bf16x8, make_uint4(xh.x, xh.y, 0u, 0u));
        const bf16x8 bl = __builtin_bit_cast(bf16x8, make_uint4(xlo.x, xlo.y, 0u, 0u));
        int ln = lane;  // rebuilt per subtile: hoisted, the weight addresses stayed live across phases 2 and 3
        asm volatile("" : "+v"(ln));
        const int si = 16 * j + r16, sy = si / SB_SW, sx = si - (si / SB_SW) * SB_SW;
        const int oy = ty0 - 2 + sy, ox = tx0 - 2 + sx;
        const bool ok = oy >= 0 && oy < a.OH && ox >= 0 && ox < a.OW;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const uint4 w4 = *reinterpret_cast<const uint4*>(&sw9[(ni * 64 + ln) * 4]);
          const float4 b4 = *reinterpret_cast<const float4*>(&sw9[512 + ni * 16 + 4 * (ln >> 4)]);
          const bf16x8 wsh = __builtin_bit_cast(bf16x8, make_uint4(w4.x, w4.y, 0u, 0u));
          const bf16x8 wsl = __builtin_bit_cast(bf16x8, make_uint4(w4.z, w4.w, 0u, 0u));
          const f32x4 acc = mma3(wsh, wsl, bh, bl, f32x4{b4.x, b4.y, b4.z, b4.w});
          const float v[4] = {silu(acc[0]), silu(acc[1]), silu(acc[2]), silu(acc[3])};
          uint2 hi = make_uint2(0u, 0u), lo = make_uint2(0u, 0u);
          if (ok) {
            if constexpr (SP) {
              split4(v, hi, lo);
            } else {
              hi.x = pack_bf16x2(v[0], v[1]);
              hi.y = pack_bf16x2(v[2], v[3]);
            }
          }
          // channels ni * 16 + 4 g .. : plane 2 ni + g / 2, the (g & 1) half of its 16 bytes.  The odd lane rows
          // hand their halves to the even rows (v_permlane16_swap), which store whole 16-byte chunks: 8-byte
          // stores of the halves were 2-way bank-conflicted (16 lanes 16 bytes apart; 0.36 conflict cycles per
          // LDS instruction over the kernel, profiles/r05fin2_sq_mfma.txt)
          auto up = [](uint32_t v) { return __builtin_amdgcn_permlane16_swap(v, v, false, false)[1]; };
          const uint4 hq = make_uint4(hi.x, hi.y, up(hi.x), up(hi.y));
          uint4 lq = make_uint4(0u, 0u, 0u, 0u);
          if constexpr (SP) lq = make_uint4(lo.x, lo.y, up(lo.x), up(lo.y));
          if ((g & 1) == 0) {
            char* d = sS + (2 * ni + (g >> 1)) * SPLANE + px * 16;
            *reinterpret_cast<uint4*>(d) = hq;
            if constexpr (SP) *reinterpret_cast<uint4*>(d + SLO) = lq;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // the next tile's frame pixels, in flight through phases 2 and 3
      const bool endu = ty + 1 >= ty_hi(u);
      const int nu = endu ? u + gx : u, nty = endu ? ty_lo(nu) : ty + 1;
      if (nu < s_end) load_in(nu, nty);
    }
    TR(1);
    __syncthreads();
    TR(2);

    // ---- phase 2: blocks.0.0 (32 -> 16) on MFMA -> A ------------------------------------------
    {
      const int sub0 = first ? 0 : ASUB0;  // later tiles: A rows 2..17 (rows 0, 1 carried)
      int sbase[AMS];
#pragma unroll
      for (int i = 0; i < AMS; ++i) {
        const int pa = min(16 * (sub0 + wave + 4 * i) + r16, APIX - 1);
        sbase[i] = pa * 16 + g * SPLANE;  // (A and S share the pitch; the taps of columns 18-19 may read
                                          // into the next plane or the pad: ignored results)
      }
      f32x4 acc[AMS];
#pragma unroll
      for (int i = 0; i < AMS; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      // the wave's subtiles (a uniform count: 5 or 6 with the 23-subtile A map) as a straight-line body: every
      // B fragment of a tap read at once and the next tap's issued before this tap's MFMAs (the per-subtile
      // guarded form waited out a full LDS round trip for each of its 54 (tap, subtile) pairs: ~8.5 k cycles)
      const int nsub = (ASUB - sub0 - wave + 3) / 4;
      auto body = [&](auto nic) {
        constexpr int NI = decltype(nic)::value;
        constexpr int NB = STEM_P2_DB ? 2 : 1;  // tap buffers: 2 = the next tap's reads ahead of this tap's MFMAs
        bf16x8 bh[NB][NI], bl[NB][SP ? NI : 1];
        auto ld = [&](int k, int buf) {
          const int toff = ((k / 3) * SB_SW + (k % 3)) * 16;
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            bh[buf][i] = frag(sS + sbase[i] + toff);
            if constexpr (SP) bl[buf][i] = frag(sS + SLO + sbase[i] + toff);
          }
        };
        if (NB == 2) ld(0, 0);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int cb = NB == 2 ? (k & 1) : 0;
          if (NB == 1) ld(k, 0);
          else if (k + 1 < 9) ld(k + 1, (k + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            if constexpr (SP)
              acc[i] = mma3(wf0[k], wl0[k], bh[cb][i], bl[cb][i], acc[i]);
            else
              acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf0[k], bh[cb][i], acc[i], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      static_assert(AMS == 6, "the straight-line bodies cover 5 and 6 subtiles");
      // (split only: the bf16 kernel's three workgroups per CU leave 168 VGPRs, and the bodies spilled there)
      if (SP && nsub == 6) {
        body(std::integral_constant<int, 6>());
      } else if (SP && nsub == 5) {
        body(std::integral_constant<int, 5>());
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int toff = ((k / 3) * SB_SW + (k % 3)) * 16;
#pragma unroll
          for (int i = 0; i < AMS; ++i) {
            if (sub0 + wave + 4 * i < ASUB) {
              const bf16x8 b = frag(sS + sbase[i] + toff);
              if constexpr (SP)
                acc[i] = mma3(wf0[k], wl0[k], b, frag(sS + SLO + sbase[i] + toff), acc[i]);
              else
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf0[k], b, acc[i], 0, 0, 0);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < AMS; ++i) {
        const int pa = 16 * (sub0 + wave + 4 * i) + r16, ai = pa - OFS;
        const int ay = ai / SB_AW, ax = ai - (ai / SB_AW) * SB_AW;
        if (sub0 + wave + 4 * i >= ASUB || ai < 0 || ax >= SB_AV) continue;
        const int oy = ty0 - 1 + ay, ox = tx0 - 1 + ax;
        uint2 u = make_uint2(0u, 0u), ul = make_uint2(0u, 0u);
        if (oy >= 0 && oy < a.OH && ox >= 0 && ox < a.OW) {
          const float v[4] = {silu(acc[i][0] + bb0.x), silu(acc[i][1] + bb0.y), silu(acc[i][2] + bb0.z),
                              silu(acc[i][3] + bb0.w)};
          if constexpr (SP) {
            split4(v, u, ul);
          } else {
            u.x = pack_bf16x2(v[0], v[1]);
            u.y = pack_bf16x2(v[2], v[3]);
          }
        }
        const int ao = a4(g) + pa * 8;
        if (!first && pa >= OFS + SHIFT) {  // carry A rows 16, 17 -> 0, 1 before overwriting them
          *reinterpret_cast<uint2*>(sA + ao - SHIFT * 8) = *reinterpret_cast<const uint2*>(sA + ao);
          if constexpr (SP) *reinterpret_cast<uint2*>(sA + ALO + ao - SHIFT * 8) = *reinterpret_cast<const uint2*>(sA + ALO + ao);
        }
        *reinterpret_cast<uint2*>(sA + ao) = u;
        if constexpr (SP) *reinterpret_cast<uint2*>(sA + ALO + ao) = ul;
      }
    }
    TR(3);
    __syncthreads();
    TR(4);

    // ---- phase 3: blocks.0.1 (16 -> 16) + skip on MFMA -> y -----------------------------------
    {
      // K step st covers taps 2st (lanes g < 2) and 2st + 1 (g >= 2), 16 channels each; the pad tap
      // 9 (zero weights) reads tap 0's pixel so the product stays finite
      // a lane's 8 channels 8 (g & 1) .. of its tap are planes 2 (g & 1) and 2 (g & 1) + 1: two 8-byte reads
      int toff[5];
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        int k = 2 * ks + (g >> 1);
        if (k > 8) k = 0;
        toff[ks] = ((k / 3) * SB_AW + (k % 3)) * 8 + a4(2 * (g & 1));
      }
      const int pdel = a4(2 * (g & 1) + 1) - a4(2 * (g & 1));  // second plane of the pair
      auto afrag = [&](const char* p) {
        const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + pdel);
        return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      };
      f32x4 acc[OMS];
#pragma unroll
      for (int i = 0; i < OMS; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 5; ++ks)
#pragma unroll
        for (int i = 0; i < OMS; ++i) {
          const int row = wave + 4 * i;  // output tile row = subtile
          const char* p = sA + (OFS + row * SB_AW + r16) * 8 + toff[ks];
          if constexpr (SP)
            acc[i] = mma3(wf1[ks], wl1[ks], afrag(p), afrag(p + ALO), acc[i]);
          else
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf1[ks], afrag(p), acc[i], 0, 0, 0);
        }
      const int ox = tx0 + r16;
#pragma unroll
      for (int i = 0; i < OMS; ++i) {
        const int row = wave + 4 * i, oy = ty0 + row;
        if (oy >= a.OH || ox >= a.OW) continue;
        const int soff = a4(g) + (OFS + (row + 1) * SB_AW + r16 + 1) * 8;
        float r[4];
        unpack_bf16x4(*reinterpret_cast<const uint2*>(sA + soff), r);
        if constexpr (SP) {
          float rl[4];
          unpack_bf16x4(*reinterpret_cast<const uint2*>(sA + ALO + soff), rl);
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] += rl[j];
        }
        const float v[4] = {silu(acc[i][0] + bb1.x) + r[0], silu(acc[i][1] + bb1.y) + r[1],
                            silu(acc[i][2] + bb1.z) + r[2], silu(acc[i][3] + bb1.w) + r[3]};
        bf16_t* yo = a.y + (((size_t)n * a.OH + oy) * a.OW + ox) * 16 * R + 4 * g;
        if constexpr (SP) {
          uint2 h, l;
          split4(v, h, l);
          *reinterpret_cast<uint2*>(yo) = h;
          *reinterpret_cast<uint2*>(yo + 16) = l;
        } else {
          *reinterpret_cast<uint2*>(yo) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
      }
    }
    TR(5);
    ++it;
    if (++ty == ty_hi(u)) {
      u += gx;
      ty = ty_lo(u);
    }
  }
}

}  // namespace

void launch_stem_b0(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, const float* w9,
                    const float* b9, const void* w0, const float* b0, int kp0, const void* w1, const float* b1,
                    int kp1, void* y, bool split, double flops, double bytes, hipStream_t s) {
  M2S_CHECK(kp0 == 288 && kp1 == 160 && N > 0 && OH > 0 && OW > 0, "stem_b0: unsupported shape");
  constexpr int TH = 16;
  StemB0Args a;
  a.frames = frames;
  a.w9 = w9;
  a.b9 = b9;
  a.w0 = static_cast<const bf16_t*>(w0);
  a.b0 = b0;
  a.w1 = static_cast<const bf16_t*>(w1);
  a.b1 = b1;
  a.y = static_cast<bf16_t*>(y);
  a.N = N;
  a.H = H;
  a.W = W;
  a.OH = OH;
  a.OW = OW;
  a.pad_t = pad_t;
  a.pad_l = pad_l;
  a.kp0 = kp0;
  a.kp1 = kp1;
  a.trace = nullptr;
#ifdef IRWS_TRACE
  static unsigned long long* tr = [] {
    unsigned long long* p = nullptr;
    if (getenv("M2S_IR_WS_TRACE")) M2S_HIP(hipMalloc(&p, 32 * 4 * 8 * 8));
    return p;
  }();
  a.trace = tr;
#endif
  a.tiles_x = ceil_div(OW, SB_TW);
  a.tiles_y = ceil_div(OH, TH);
  M2S_CHECK((double)N * a.tiles_x * a.tiles_y < 2147483647.0, "stem_b0: grid");
  // persistent grid: the resident workgroups of the device (two per CU split, three bf16), a multiple
  // of 8 (one equal share per XCD); small inputs take fewer
  const int cus = device_cus();
  const int nstrip = N * a.tiles_x;  // a workgroup walks whole strips (image, tile column) top to bottom
  const int per_cu = split ? 2 : 3;
  // small batches: strips cut into tile-row ranges so the units fill the workgroup slots (a cut costs one more
  // first tile, ~1.2 tiles of work).  M2S_STEM_PARTS=n forces n (tests, A/B).
  const char* fp = getenv("M2S_STEM_PARTS");
  int parts = fp ? atoi(fp) : (cus * per_cu) / std::max(1, nstrip);
  parts = std::max(1, std::min(parts, a.tiles_y));
  a.tpp = ceil_div(a.tiles_y, parts);
  a.parts = ceil_div(a.tiles_y, a.tpp);  // (no empty parts)
  a.per_xcd = ceil_div(nstrip * a.parts, 8);
  const int grid = 8 * std::max(1, std::min(ceil_div(cus * per_cu, 8), a.per_xcd));
  if (split) {
    ProfScope ps("stem_b0_kernel<16, 1>", flops, bytes, s);
    hipLaunchKernelGGL((stem_b0_kernel<TH, 1>), dim3(grid), dim3(256), 0, s, a);
#ifdef IRWS_TRACE
    if (tr) {  // per-phase cycles of workgroup 0's four waves, first tiles: p1 bar1 p2 bar2 p3
      static int calls = 0;
      if (++calls <= 4) {
        std::vector<unsigned long long> h(32 * 4 * 8);
        M2S_HIP(hipStreamSynchronize(s));
        M2S_HIP(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
        fprintf(stderr, "STEMTRACE");
        for (int i = 2; i < 12; ++i)
          for (int w = 0; w < 4; w += 3) {
            const unsigned long long* q = &h[(i * 4 + w) * 8];
            fprintf(stderr, " [t%d w%d p1 %lld bar1 %lld p2 %lld bar2 %lld p3 %lld next %lld]", i, w, (long long)(q[1] - q[0]),
                    (long long)(q[2] - q[1]), (long long)(q[3] - q[2]), (long long)(q[4] - q[3]), (long long)(q[5] - q[4]),
                    (long long)(h[((i + 1) * 4 + w) * 8] - q[5]));
          }
        fprintf(stderr, "\n");
      }
    }
#endif
  } else {
    ProfScope ps("stem_b0_kernel<16, 0>", flops, bytes, s);
    hipLaunchKernelGGL((stem_b0_kernel<TH, 0>), dim3(grid), dim3(256), 0, s, a);
  }
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
