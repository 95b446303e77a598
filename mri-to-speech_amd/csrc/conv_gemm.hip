// bf16 implicit-GEMM convolution with an LDS-DMA (global_load_lds) pipeline: the fast path of every
// bf16 conv.  ConvArgs contract: conv_igemm.hpp (shared with the fp32 parity kernel).
//
// Why this shape.  The hot-path GEMMs are short in K (64..1248 = 2..39 steps of 32) and long in M
// (positions x frames), so per-step load latency, not arithmetic, is what a workgroup waits on.
// Each workgroup (4 waves) keeps S-1 K-steps of its A (activation) and B (weight) tiles in flight
// as LDS-DMA transfers - no staging registers - retired by a counted `s_waitcnt vmcnt` and a raw
// s_barrier (cdna_hip_programming.md §5 "Pipelining across barriers").  A tile row = one output
// position, gathered per lane (implicit GEMM: the lane's source address is the input position for
// its tap; padding lanes read a zero page).  LDS rows are 64 B (32 bf16 = one MFMA k-step); the
// 16-byte chunks are XOR-swizzled on the SOURCE side (chunk p of row r holds logical chunk
// p ^ ((r >> 2) & 3)) so the ds_read_b128 fragment reads are bank-conflict free (rule 21).
// LeakyReLU / SE scales are applied to the activation fragments after the LDS read; the SE table
// of the workgroup's images is staged in LDS once.  Blocks are remapped so that the N tiles of
// one M tile run on one XCD (shared A rows stay in that XCD's L2).
#include "conv_igemm.hpp"

#include <cstring>
#include <map>
#include <mutex>

#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_zero_page[4];  // padding lanes' DMA source

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ bf16x8 lrelu_frag(bf16x8 v, float slope) {
  uint4 u = __builtin_bit_cast(uint4, v);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float lo = __uint_as_float(w[j] << 16), hi = __uint_as_float(w[j] & 0xffff0000u);
    lo = lo > 0.f ? lo : lo * slope;
    hi = hi > 0.f ? hi : hi * slope;
    w[j] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
  }
  return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
}

// SE scales come from an LDS table.  Read through inline asm (loads + wait in ONE statement,
// cdna_hip_programming.md §5.7 form (i)): a plain ds_read there makes hipcc assume it may alias
// the in-flight LDS-DMA and drain the whole pipeline with vmcnt(0) every step.
__device__ __forceinline__ void load_scales(const float* s, float* sc) {
  float4 s0, s1;
  const uint32_t addr = (uint32_t)(uintptr_t)s;
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(s0), "=&v"(s1)
               : "v"(addr)
               : "memory");
  sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
  sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
}
__device__ __forceinline__ bf16x8 scale_with(bf16x8 v, const float* sc) {
  uint4 u = __builtin_bit_cast(uint4, v);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = pack_bf16x2(__uint_as_float(w[j] << 16) * sc[2 * j], __uint_as_float(w[j] & 0xffff0000u) * sc[2 * j + 1]);
  return __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
}
__device__ __forceinline__ bf16x8 scale_frag(bf16x8 v, const float* s) {
  float sc[8];
  load_scales(s, sc);
  return scale_with(v, sc);
}

// Split-fp32 fragments (SP = 1): hi/lo pairs of 8 values.  An input transform computes in fp32 on
// hi + lo and re-splits the result, so the transformed operand keeps 17 significant bits.
__device__ __forceinline__ void resplit_frag(const float* v, bf16x8& h, bf16x8& l) {
  uint2 h0, h1, l0, l1;
  split4(v, h0, l0);
  split4(v + 4, h1, l1);
  h = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
  l = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
}
__device__ __forceinline__ void frag_sum(bf16x8 h, bf16x8 l, float* v) {
  const uint4 a = __builtin_bit_cast(uint4, h), b = __builtin_bit_cast(uint4, l);
  unpack_bf16x4(make_uint2(a.x, a.y), v);
  unpack_bf16x4(make_uint2(a.z, a.w), v + 4);
  float w[8];
  unpack_bf16x4(make_uint2(b.x, b.y), w);
  unpack_bf16x4(make_uint2(b.z, b.w), w + 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] += w[j];
}
__device__ __forceinline__ void lrelu_split(bf16x8& h, bf16x8& l, float slope) {
  float v[8];
  frag_sum(h, l, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * slope;
  resplit_frag(v, h, l);
}
__device__ __forceinline__ void scale_split(bf16x8& h, bf16x8& l, const float* sc) {
  float v[8];
  frag_sum(h, l, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= sc[j];
  resplit_frag(v, h, l);
}

// 8 bf16 -> 8 OCP e4m3fn (gfx950 v_cvt_pk_fp8_f32, round to nearest even), saturated by sat_e4m3
// (m2s_common.hpp: finite values clamped to +-448, a NaN stays NaN so an upstream fault is not hidden)
__device__ __forceinline__ long fp8x8(bf16x8 v) {
  const uint4 u = __builtin_bit_cast(uint4, v);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  int q[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float f[4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f[2 * j] = sat_e4m3(__uint_as_float(w[2 * h + j] << 16));
      f[2 * j + 1] = sat_e4m3(__uint_as_float(w[2 * h + j] & 0xffff0000u));
    }
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    q[h] = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], r, true);
  }
  return (long)(((unsigned long)(uint32_t)q[1] << 32) | (uint32_t)q[0]);
}

__device__ __forceinline__ void ld4f(const bf16_t* p, float* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xffff0000u);
}

constexpr int ROW = 64;  // bytes per LDS row = 32 bf16 = one k-step

// Physical chunk of logical chunk c in row r: c ^ f((r >> 2) & 3) with f = [0, 2, 3, 1].  A fragment read
// (lane = (g = lane >> 4, r16 = lane & 15): row r16, chunk g) is then conflict-free for ds_read_b128's
// lane groups on gfx950 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...; MI355X_MICROARCH.md LDS table):
// within each group the four lanes that share (r16 & 3) land in four different 16-byte bank slots.
// (The plain c ^ ((r >> 2) & 3) put lanes 0-3 and 20-23 on the same slots: 2-way conflicts, SQ
// LDS_BANK_CONFLICT ~3x the LDS-active cycles.)
__device__ __forceinline__ int swz_f(int x) { return (0x1320 >> (4 * x)) & 3; }
__device__ __forceinline__ int swz(int row, int chunk) { return row * ROW + ((chunk ^ swz_f((row >> 2) & 3)) << 4); }

// SP = 1: split-fp32 operands (m2s_common.hpp sp_t): every activation and weight row is [hi | lo],
// each K step DMAs both halves into two planes of the slot and runs the three MFMA terms
// hi*hi + hi*lo + lo*hi (the dropped lo*lo term is below 2^-16 of the product).
// SP = 2: e4m3 operands over bf16 storage (conv_igemm.hpp launch_conv_gemm, a.wscale).
template <int BM, int BN, int MT, int NT, int S, int KIND, int XF, int SP>
__global__ void __launch_bounds__(256, (BN >= 256 || (BM >= 256 && BN >= 128) ? 2 : 1)) conv_gemm_kernel(const ConvBatch ab, int n_tiles, int se_imgs,
                                                                                                      float* __restrict__ kpart) {
  // KIND_CONV1D launches may batch convs of one shape over grid.z (launch_conv_gemm_batch)
  const ConvArgs a = ab.a[KIND == KIND_CONV1D ? blockIdx.z : 0];  // a copy: fields land in SGPRs once, not re-loaded per K step
  constexpr int WN = BN / (NT * 16);
  constexpr int WM = 4 / WN;
  static_assert(WM * WN == 4 && WM * MT * 16 == BM, "bad tile");
  constexpr int R = SP == 1 ? 2 : 1;               // planes per operand row
  constexpr int A_PER_WAVE = BM / 64;              // 16-row DMA blocks per wave for A
  constexpr int B_BLOCKS = BN / 16;                // 16-row DMA blocks for B
  constexpr int B_PER_WAVE = (B_BLOCKS + 3) / 4;   // waves >= B_BLOCKS issue into a scratch block
  constexpr int SLOT = (R * (BM + BN) + 16) * ROW; // +16 rows: scratch for surplus B DMAs
  constexpr int PER_STAGE = R * (A_PER_WAVE + B_PER_WAVE);
  constexpr bool PRE = SP == 1 && XF == IN_SE_SCALE;  // split SE scale applied in LDS (below)
  constexpr bool SE = XF == IN_SE_SCALE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* se_tab = reinterpret_cast<float*>(smem + S * SLOT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, r16 = lane & 15;

  // XCD-aware block -> (m tile, n tile): the n tiles of one m tile share blockIdx % 8 (one XCD).
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int mt = wid / n_tiles, nt = wid - (wid / n_tiles) * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int phase = KIND == KIND_CONVT ? (int)blockIdx.z : 0;

  const bf16_t* __restrict__ X = static_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ W = static_cast<const bf16_t*>(a.w) + (size_t)phase * a.n_pad * a.kp * R;
  const int xs = a.cs_in * R;  // elements per input position
  // split K (grid.y > 1, small grids: launch_tile): this workgroup runs K steps [kb, kb + nsteps) of its tile and
  // stores fp32 partial sums to kpart; conv_gemm_ksum_kernel adds them in split order and runs the epilogue
  const int nks = gridDim.y, ks = blockIdx.y;
  const int kb = (a.kp / 32) * ks / nks;
  const int nsteps = (a.kp / 32) * (ks + 1) / nks - kb;

  // ---- DMA roles: lane -> (row within a 16-row block, physical chunk) -------------------------
  // Per A row the geometry is resolved once: `rbase` = element offset of the row's tap-0 input
  // position (may lie outside the tensor) and `rmask` bit t = tap t reads inside the tensor (the
  // TF-SAME / causal / look-ahead zero padding).  Per K step a lane then needs only its tap's
  // uniform offset, one bit test and one add per row (the address math used to be ~40 VALU per
  // row per step, which made VALU issue, not the MFMA, the limit of these kernels).
  const int lrow = lane >> 2;
  const int q = (lane & 3) ^ swz_f((lane >> 4) & 3);  // logical chunk this lane fetches ((row>>2)&3 = lane>>4 & 3)
  int rbase[A_PER_WAVE];
  uint32_t rmask[A_PER_WAVE];
  const int delta = (KIND == KIND_CONVT) ? (phase + a.ct_pad) / a.ct_u : 0;
#pragma unroll
  for (int j = 0; j < A_PER_WAVE; ++j) {
    const int m = m0 + (wave * A_PER_WAVE + j) * 16 + lrow;
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    uint32_t msk = 0;
    if constexpr (KIND == KIND_CONV2D) {
      const int hw = a.OH * a.OW;
      const int img = mm / hw, rem = mm - (mm / hw) * hw;
      const int oy = rem / a.OW, ox = rem - (rem / a.OW) * a.OW;
      const int iy0 = oy * a.stride - a.pad_t, ix0 = ox * a.stride - a.pad_l;
      rbase[j] = ((img * a.IH + iy0) * a.IW + ix0) * xs;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int iy = iy0 + t / 3, ix = ix0 + t % 3;
        msk |= (uint32_t)(iy >= 0 && iy < a.IH && ix >= 0 && ix < a.IW) << t;
      }
    } else if constexpr (KIND == KIND_CONV1D) {
      const int b = mm / a.L_out, t0 = mm - b * a.L_out - a.pad_left;
      rbase[j] = (b * a.L_in + t0) * xs;
      for (int t = 0; t < a.ntaps; ++t) {
        const int it = t0 + t * a.dil;
        msk |= (uint32_t)(it >= 0 && it < a.L_in) << t;
      }
    } else if constexpr (KIND == KIND_CONVT) {
      const int b = mm / a.L_in, t0 = mm - b * a.L_in + delta;
      rbase[j] = (b * a.L_in + t0) * xs;
      for (int t = 0; t < a.ntaps; ++t) {
        const int it = t0 - t;
        msk |= (uint32_t)(it >= 0 && it < a.L_in) << t;
      }
    } else {
      rbase[j] = mm * xs;
      msk = 1u;
    }
    rmask[j] = ok ? msk : 0u;
  }
  // this lane's tap and channel within the current K step, and the tap's input offset
  // (K step kb's element offset: cs_in >= 32 is a multiple of 32, smaller cs_in divide 32)
  int s_tap = (kb * 32 + q * 8) / a.cs_in, s_c = (kb * 32 + q * 8) % a.cs_in;
  const int row_stride = a.IW * xs;  // CONV2D: one input row
  auto tap_off = [&](int t) -> int {
    if constexpr (KIND == KIND_CONV2D) return (t / 3) * row_stride + (t - (t / 3) * 3) * xs;
    else if constexpr (KIND == KIND_CONV1D) return t * a.dil * xs;
    else if constexpr (KIND == KIND_CONVT) return -t * xs;
    else return 0;
  };
  int s_off = tap_off(s_tap) + s_c;
  const char* zp = reinterpret_cast<const char*>(g_zero_page);
  asm volatile("" : "+s"(zp));  // keep the zero page address in SGPRs (no per-use reload)
  const bf16_t* bsrc[B_PER_WAVE];
#pragma unroll
  for (int j = 0; j < B_PER_WAVE; ++j) {
    const int blk = wave * B_PER_WAVE + j;
    const int n = n0 + blk * 16 + lrow;
    bsrc[j] = (blk < B_BLOCKS && n < a.n_pad) ? W + (size_t)n * a.kp * R + q * 8 : nullptr;
  }

  // split SE-gated GEMM: the operand is in the interleaved layout (m2s_common.hpp il_st8: per 32-channel
  // group [hi 32 | lo 32]); the K step's hi chunk q sits at 64 st + 8 q, its lo chunk 32 further
  constexpr bool IL = PRE && KIND == KIND_GEMM;
  auto issue = [&](int st, int slot) {
    char* As = smem + slot * SLOT;
    char* Bs = As + R * BM * ROW;
#pragma unroll
    for (int j = 0; j < A_PER_WAVE; ++j) {
      const bool v = s_tap < 32 && ((rmask[j] >> s_tap) & 1u);
      const bf16_t* src = X + (unsigned)(rbase[j] + (IL ? 2 * s_off - q * 8 : s_off));
      dma16(v ? static_cast<const void*>(src) : static_cast<const void*>(zp), As + (wave * A_PER_WAVE + j) * 16 * ROW);
      if constexpr (SP == 1)
        dma16(v ? static_cast<const void*>(src + (IL ? 32 : a.cs_in)) : static_cast<const void*>(zp),
              As + (BM + (wave * A_PER_WAVE + j) * 16) * ROW);
    }
#pragma unroll
    for (int j = 0; j < B_PER_WAVE; ++j) {
      const int blk = wave * B_PER_WAVE + j;
      const void* src = bsrc[j] ? (const void*)(bsrc[j] + st * 32) : (const void*)zp;
      dma16(src, blk < B_BLOCKS ? Bs + blk * 16 * ROW : As + R * (BM + BN) * ROW);
      if constexpr (SP == 1)
        dma16(bsrc[j] ? (const void*)(bsrc[j] + st * 32 + a.kp) : (const void*)zp,
              blk < B_BLOCKS ? Bs + (BN + blk * 16) * ROW : As + R * (BM + BN) * ROW);
    }
    // advance one K step (32 channels): cs_in >= 32 is a multiple of 32, smaller cs_in divide 32
    if (a.cs_in >= 32) {
      s_c += 32;
      if (s_c >= a.cs_in) {
        s_c -= a.cs_in;
        ++s_tap;
      }
    } else {
      s_tap += 32 / a.cs_in;
    }
    s_off = tap_off(s_tap) + s_c;
  };

  // ---- SE scale table for this workgroup's images (GEMM kind only) ---------------------------
  int img0 = 0;
  if constexpr (SE) {
    // only this workgroup's K range (split K: 1 / nks of the channels), 8 channels a 16-byte load, every load of a
    // thread issued before the first conversion (the element-wise loop over every channel was a chain of global
    // round trips: configs[1] 1.065 -> 1.034 ms, configs[2] 2.254 -> 2.245 ms, gpurun_out/r06r)
    img0 = m0 / a.OH;
    const int c_lo = kb * 32, nc8 = (min(a.cs_in, (kb + nsteps) * 32) - c_lo) / 8, tot = se_imgs * nc8;
    const bf16_t* gb = static_cast<const bf16_t*>(a.in_scale);
    for (int i0 = tid; i0 < tot; i0 += 4 * 256) {
      uint4 h[4], l[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 256 * u, im = i / max(nc8, 1), c = c_lo + 8 * (i - im * nc8);
        h[u] = l[u] = make_uint4(0u, 0u, 0u, 0u);
        if (i < tot && (img0 + im) * a.OH < a.M) {
          const bf16_t* g = gb + (size_t)(img0 + im) * xs + c;
          h[u] = *reinterpret_cast<const uint4*>(g);
          if constexpr (SP == 1) l[u] = *reinterpret_cast<const uint4*>(g + a.cs_in);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 256 * u, im = i / max(nc8, 1), c = c_lo + 8 * (i - im * nc8);
        if (i >= tot) break;
        float v[8];
        unpack_bf16x4(make_uint2(h[u].x, h[u].y), v);
        unpack_bf16x4(make_uint2(h[u].z, h[u].w), v + 4);
        if constexpr (SP == 1) {
          float w[8];
          unpack_bf16x4(make_uint2(l[u].x, l[u].y), w);
          unpack_bf16x4(make_uint2(l[u].z, l[u].w), w + 4);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += w[e];
        }
        float* d = se_tab + im * a.cs_in + c;
        *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    }
  }
  // SE scale on the weight fragments when the tile is one image (its k-scales are shared by every
  // row): NT fragments and one table read per k-step instead of MT fragments and MT reads
  bool one_img = false;
  if constexpr (SE) one_img = img0 == (min(m0 + BM, a.M) - 1) / a.OH;
  int frow_img[MT];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + wm * MT * 16 + mi * 16 + r16;
    frow_img[mi] = SE ? (m < a.M ? m / a.OH : img0) - img0 : 0;
  }

  f32x4 acc[NT][MT];
#pragma unroll
  for (int ni = 0; ni < NT; ++ni)
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one K step of MFMAs on the operands in `slot` (input transforms applied to the fragments)
  auto compute = [&](int st, int slot) {
    const char* As = smem + slot * SLOT;
    const char* Bs = As + R * BM * ROW;
    bf16x8 af[NT], bx[MT];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
      af[ni] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn * NT * 16 + ni * 16 + r16, g));
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
      bx[mi] = *reinterpret_cast<const bf16x8*>(As + swz(wm * MT * 16 + mi * 16 + r16, g));
    if constexpr (SP == 1) {
      bf16x8 afl[NT], bxl[MT];
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
        afl[ni] = *reinterpret_cast<const bf16x8*>(Bs + BN * ROW + swz(wn * NT * 16 + ni * 16 + r16, g));
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        bxl[mi] = *reinterpret_cast<const bf16x8*>(As + BM * ROW + swz(wm * MT * 16 + mi * 16 + r16, g));
      if constexpr (XF == IN_LRELU) {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) lrelu_split(bx[mi], bxl[mi], a.in_slope);
      }
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[ni], bx[mi], acc[ni][mi], 0, 0, 0);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ni], bxl[mi], acc[ni][mi], 0, 0, 0);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ni], bx[mi], acc[ni][mi], 0, 0, 0);
        }
      return;
    }
    if constexpr (XF == IN_LRELU) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) bx[mi] = lrelu_frag(bx[mi], a.in_slope);
    } else if constexpr (XF == IN_SE_SCALE) {
      if (one_img) {  // the whole tile is one image: scale the NT weight fragments, one table read
        float sc[8];
        load_scales(se_tab + st * 32 + g * 8, sc);
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) af[ni] = scale_with(af[ni], sc);
      } else {
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) bx[mi] = scale_frag(bx[mi], se_tab + frow_img[mi] * a.cs_in + st * 32 + g * 8);
      }
    }
    if constexpr (SP == 2) {  // e4m3: weights are on the grid (exact), activations round here
      long a8[NT], b8[MT];
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) a8[ni] = fp8x8(af[ni]);
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) b8[mi] = fp8x8(bx[mi]);
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a8[ni], b8[mi], acc[ni][mi], 0, 0, 0);
      return;
    }
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ni], bx[mi], acc[ni][mi], 0, 0, 0);
  };

  // split SE GEMM and split 1-D convs (the MRF c2's residual): the skip operand is fetched before the
  // K loop (the epilogue's residual read was an exposed HBM round trip at the end of every tile)
  constexpr bool PREF = PRE || (SP == 1 && KIND == KIND_CONV1D);
  uint2 pres[PREF ? MT : 1][PREF ? NT : 1][2];
  if constexpr (PREF) {
    const bf16_t* __restrict__ R0 = static_cast<const bf16_t*>(a.res);
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int m = m0 + wm * MT * 16 + mi * 16 + r16, n4 = n0 + wn * NT * 16 + ni * 16 + 4 * g;
        pres[mi][ni][0] = pres[mi][ni][1] = make_uint2(0u, 0u);
        if (R0 && nks == 1 && m < a.M && n4 < a.cs_out) {
          const size_t orow = (size_t)m * a.cs_out * 2;
          pres[mi][ni][0] = *reinterpret_cast<const uint2*>(R0 + orow + n4);
          pres[mi][ni][1] = *reinterpret_cast<const uint2*>(R0 + orow + a.cs_out + n4);
        }
      }
  }

  if constexpr (PRE) {
    // Split SE-scaled GEMM: the A tile is scaled IN LDS once per K step by the whole workgroup (each
    // thread BM / 64 16-byte hi/lo chunk pairs) between two barriers, instead of per wave on its
    // fragments (WN-fold redundant; the fp32 re-split is ~56 VALU per 8 values).  The second
    // workgroup on the CU runs its MFMAs meanwhile.  Measured per launch (20 a step, split fp32):
    // per-fragment 419 us, in-LDS on two slots 405 us, in-LDS one step ahead on three slots 568 us
    // (one workgroup per CU).
    static_assert(S == 2, "pre-scaled SE GEMM runs two slots");
    constexpr int UPT = BM * 4 / 256;
    uint32_t u_lds[UPT], u_tab[UPT];
    const uint32_t tab0 = (uint32_t)(uintptr_t)se_tab;
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const int u = tid + 256 * j, row = u >> 2, p = u & 3;
      const int c = p ^ swz_f((row >> 2) & 3);
      const int m = m0 + row;
      const int im = (m < a.M ? m / a.OH : img0) - img0;
      u_lds[j] = (uint32_t)(row * ROW + p * 16);
      u_tab[j] = tab0 + (uint32_t)((im * a.cs_in + c * 8) * 4);
    }
    const uint32_t smem0 = (uint32_t)(uintptr_t)smem;
    auto scale_slot = [&](int st, int slot) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      u32x4 h[UPT], l[UPT];
      f32x4 s0[UPT], s1[UPT];
#pragma unroll
      for (int j = 0; j < UPT; ++j) {
        const uint32_t ah = smem0 + slot * SLOT + u_lds[j], ta = u_tab[j] + st * 128;
        // plain ds_reads here would let hipcc drain the in-flight DMA (vmcnt(0)): see load_scales
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:%6\n\tds_read_b128 %2, %5\n\tds_read_b128 %3, %5 offset:16"
                     : "=&v"(h[j]), "=&v"(l[j]), "=&v"(s0[j]), "=&v"(s1[j])
                     : "v"(ah), "v"(ta), "n"(BM * ROW)
                     : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < UPT; ++j) {
        asm volatile("" : "+v"(h[j]), "+v"(l[j]), "+v"(s0[j]), "+v"(s1[j]));
        const float sc[8] = {s0[j][0], s0[j][1], s0[j][2], s0[j][3], s1[j][0], s1[j][1], s1[j][2], s1[j][3]};
        bf16x8 hv = __builtin_bit_cast(bf16x8, h[j]), lv = __builtin_bit_cast(bf16x8, l[j]);
        scale_split(hv, lv, sc);
        const uint32_t ah = smem0 + slot * SLOT + u_lds[j];
        asm volatile("ds_write_b128 %0, %1\n\tds_write_b128 %0, %2 offset:%3"
                     :
                     : "v"(ah), "v"(__builtin_bit_cast(u32x4, hv)), "v"(__builtin_bit_cast(u32x4, lv)), "n"(BM * ROW)
                     : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible at the next barrier
    };
    if (nsteps > 0) issue(kb, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the SE table stores
    for (int i = 0; i < nsteps; ++i) {
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();  // step i landed everywhere; slot (i + 1) % 2 free
      if (i + 1 < nsteps) issue(kb + i + 1, (i + 1) % 2);
      scale_slot(kb + i, i % 2);
      __builtin_amdgcn_s_barrier();
      compute(kb + i, i % 2);
    }
  } else {
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nsteps) issue(kb + s, s);

  for (int i = 0; i < nsteps; ++i) {
    // step i has landed once at most min(S-2, nsteps-1-i) younger steps are outstanding
    const int younger = min(S - 2, nsteps - 1 - i);
    if (younger >= 2)
      wait_vm<2 * PER_STAGE>();
    else if (younger == 1)
      wait_vm<PER_STAGE>();
    else
      wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave's DMA for step i landed; slot (i-1)%S is free
    if (i + S - 1 < nsteps) issue(kb + i + S - 1, (i + S - 1) % S);
    compute(kb + i, i % S);
  }
  }

  if (nks > 1) {  // split K: raw fp32 partial sums [z][ks][M][cs_out], the epilogue runs in conv_gemm_ksum_kernel
    float* __restrict__ P = kpart + ((size_t)blockIdx.z * nks + ks) * a.M * a.cs_out;
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      const int m = m0 + wm * MT * 16 + mi * 16 + r16;
      if (m >= a.M) continue;
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int n4 = n0 + wn * NT * 16 + ni * 16 + 4 * g;
        if (n4 < a.cs_out)
          *reinterpret_cast<float4*>(P + (size_t)m * a.cs_out + n4) =
              make_float4(acc[ni][mi][0], acc[ni][mi][1], acc[ni][mi][2], acc[ni][mi][3]);
      }
    }
    return;
  }

  // ---- epilogue: 4 consecutive channels of one position per lane ------------------------------
  bf16_t* __restrict__ Y = static_cast<bf16_t*>(a.y);
  const bf16_t* __restrict__ Rs = static_cast<const bf16_t*>(a.res);
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + wm * MT * 16 + mi * 16 + r16;
    if (m >= a.M) continue;
    long orow;  // output position
    if constexpr (KIND == KIND_CONVT) {
      const int b = m / a.L_in, qq = m - (m / a.L_in) * a.L_in;
      orow = (long)b * a.L_out + (long)qq * a.ct_u + phase;
    } else {
      orow = m;
    }
    orow *= (long)a.cs_out * R;
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int n4 = n0 + wn * NT * 16 + ni * 16 + 4 * g;
      if (n4 >= a.cs_out) continue;
      const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
      float v[4] = {acc[ni][mi][0] + bb.x, acc[ni][mi][1] + bb.y, acc[ni][mi][2] + bb.z, acc[ni][mi][3] + bb.w};
      if constexpr (SP == 2) {  // e4m3 weights carry a per-output-channel scale
        const float4 ws = *reinterpret_cast<const float4*>(a.wscale + n4);
        v[0] = fmaf(acc[ni][mi][0], ws.x, bb.x);
        v[1] = fmaf(acc[ni][mi][1], ws.y, bb.y);
        v[2] = fmaf(acc[ni][mi][2], ws.z, bb.z);
        v[3] = fmaf(acc[ni][mi][3], ws.w, bb.w);
      }
      auto apply_act = [&]() {
        if (a.act == ACT_SILU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = silu(v[j]);
        } else if (a.act == ACT_LRELU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * a.act_slope;
        } else if (a.act == ACT_SIGMOID) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = sigmoidf_(v[j]);
        }
      };
      if (!a.act_after_res) apply_act();
      if (Rs) {
        float r[4];
        if constexpr (PREF) {
          float rl[4];
          unpack_bf16x4(pres[mi][ni][0], r);
          unpack_bf16x4(pres[mi][ni][1], rl);
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] += rl[j];
        } else {
          ld4f(Rs + orow + n4, r);
          if constexpr (SP == 1) {
            float rl[4];
            ld4f(Rs + orow + a.cs_out + n4, rl);
#pragma unroll
            for (int j = 0; j < 4; ++j) r[j] += rl[j];
          }
        }
        if (a.res_unslope != 0.f) {  // the residual was stored as lrelu(x): invert it
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = r[j] > 0.f ? r[j] : r[j] * a.res_unslope;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += r[j];
      }
      if (a.accum) {
        float p[4];
        ld4f(Y + orow + n4, p);
        if constexpr (SP == 1) {
          float pl[4];
          ld4f(Y + orow + a.cs_out + n4, pl);
#pragma unroll
          for (int j = 0; j < 4; ++j) p[j] += pl[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = p[j] + v[j];
        if (a.accum == 2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = v[j] / a.accum_div;
        }
      }
      if (a.act_after_res) apply_act();
      if constexpr (SP == 1) {
        uint2 hi, lo;
        split4(v, hi, lo);
        *reinterpret_cast<uint2*>(Y + orow + n4) = hi;
        *reinterpret_cast<uint2*>(Y + orow + a.cs_out + n4) = lo;
      } else {
        uint2 u;
        u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(Y + orow + n4) = u;
      }
    }
  }
}

// Split-K epilogue: the partial sums of the nks K ranges added in split order (deterministic), then the main
// kernel's epilogue (bias / e4m3 weight scale, activation, residual, MRF accumulation, bf16 or split store);
// lane = 4 consecutive channels of one output position, grid.z = the main launch's grid.z.
template <int KIND, int SP>
__global__ void __launch_bounds__(256) conv_gemm_ksum_kernel(const ConvBatch ab, const float* __restrict__ kpart, int nks) {
  const ConvArgs a = ab.a[KIND == KIND_CONV1D ? blockIdx.z : 0];
  constexpr int R = SP == 1 ? 2 : 1;
  const int nq = a.cs_out / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)a.M * nq) return;
  const int m = (int)(i / nq), n4 = (int)(i - (long)m * nq) * 4;
  const size_t plane = (size_t)a.M * a.cs_out;
  const float* p = kpart + (size_t)blockIdx.z * nks * plane + (size_t)m * a.cs_out + n4;
  float4 acc = *reinterpret_cast<const float4*>(p);
  for (int k = 1; k < nks; ++k) {
    const float4 t = *reinterpret_cast<const float4*>(p + k * plane);
    acc.x += t.x;
    acc.y += t.y;
    acc.z += t.z;
    acc.w += t.w;
  }
  long orow = m;
  if constexpr (KIND == KIND_CONVT) {
    const int b = m / a.L_in, qq = m - (m / a.L_in) * a.L_in;
    orow = (long)b * a.L_out + (long)qq * a.ct_u + blockIdx.z;
  }
  orow *= (long)a.cs_out * R;
  const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
  float v[4] = {acc.x + bb.x, acc.y + bb.y, acc.z + bb.z, acc.w + bb.w};
  if constexpr (SP == 2) {
    const float4 ws = *reinterpret_cast<const float4*>(a.wscale + n4);
    v[0] = fmaf(acc.x, ws.x, bb.x);
    v[1] = fmaf(acc.y, ws.y, bb.y);
    v[2] = fmaf(acc.z, ws.z, bb.z);
    v[3] = fmaf(acc.w, ws.w, bb.w);
  }
  auto apply_act = [&]() {
    if (a.act == ACT_SILU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = silu(v[j]);
    } else if (a.act == ACT_LRELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * a.act_slope;
    } else if (a.act == ACT_SIGMOID) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = sigmoidf_(v[j]);
    }
  };
  if (!a.act_after_res) apply_act();
  bf16_t* __restrict__ Y = static_cast<bf16_t*>(a.y);
  const bf16_t* __restrict__ Rs = static_cast<const bf16_t*>(a.res);
  if (Rs) {
    float r[4];
    ld4f(Rs + orow + n4, r);
    if constexpr (SP == 1) {
      float rl[4];
      ld4f(Rs + orow + a.cs_out + n4, rl);
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] += rl[j];
    }
    if (a.res_unslope != 0.f) {
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = r[j] > 0.f ? r[j] : r[j] * a.res_unslope;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += r[j];
  }
  if (a.accum) {
    float pv[4];
    ld4f(Y + orow + n4, pv);
    if constexpr (SP == 1) {
      float pl[4];
      ld4f(Y + orow + a.cs_out + n4, pl);
#pragma unroll
      for (int j = 0; j < 4; ++j) pv[j] += pl[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = pv[j] + v[j];
    if (a.accum == 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = v[j] / a.accum_div;
    }
  }
  if (a.act_after_res) apply_act();
  if constexpr (SP == 1) {
    uint2 hi, lo;
    split4(v, hi, lo);
    *reinterpret_cast<uint2*>(Y + orow + n4) = hi;
    *reinterpret_cast<uint2*>(Y + orow + a.cs_out + n4) = lo;
  } else {
    uint2 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(Y + orow + n4) = u;
  }
}

// Split-K partial sums live in one device buffer per (device, stream), grown on demand (only small grids split,
// so it stays a few MB); launches on one stream are ordered, so one buffer per stream is race-free.  A stream under
// HIP graph capture cannot allocate: it borrows the device's largest buffer (the eager warm-up calls made it) and,
// if none is large enough, gets nullptr, and the launch runs unsplit.
float* ksplit_scratch(hipStream_t s, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> bufs;
  int dev = 0;
  M2S_HIP(hipGetDevice(&dev));
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  M2S_HIP(hipStreamIsCapturing(s, &cap));
  std::lock_guard<std::mutex> g(mu);
  if (cap != hipStreamCaptureStatusNone) {
    void* best = nullptr;
    size_t best_sz = 0;
    for (auto& kv : bufs)
      if (kv.first.first == dev && kv.second.second > best_sz) {
        best = kv.second.first;
        best_sz = kv.second.second;
      }
    return best_sz >= bytes ? static_cast<float*>(best) : nullptr;
  }
  auto& b = bufs[{dev, s}];
  if (b.second < bytes) {
    if (b.first) {
      M2S_HIP(hipStreamSynchronize(s));  // the old buffer may still be read by queued launches
      M2S_HIP(hipFree(b.first));
    }
    const size_t sz = (bytes + (16u << 20) - 1) / (16u << 20) * (16u << 20);
    M2S_HIP(hipMalloc(&b.first, sz));
    b.second = sz;
  }
  return static_cast<float*>(b.first);
}

const char* kname(int k) {
  switch (k) {
    case KIND_CONV2D: return "conv2d";
    case KIND_CONV1D: return "conv1d";
    case KIND_CONVT: return "convT";
    default: return "gemm";
  }
}

// rows of SE gates a tile needs: the images its BM rows touch
inline int se_images(int BM, int OH) { return BM % OH == 0 ? BM / OH : OH % BM == 0 ? 1 : (BM + OH - 1) / OH + 1; }

template <int BM, int BN, int MT, int NT, int KIND, int XF, int SP, int SF = 0>
void launch_tile(const ConvBatch& b, hipStream_t s, int phases, double flops, double bytes) {
  const ConvArgs& a = b.a[0];
  // keep two workgroups' LDS per CU (128 x 256: the SE gate table too, and 256 registers a wave);
  // split operands double the slot, so they run two stages (SF: a forced stage count, A/B builds)
  constexpr int S = SF ? SF : SP == 1 ? (BM == 128 && BN == 64 && XF != IN_SE_SCALE ? 3 : 2) : (BN >= 256 || BM + BN >= 384) ? 2 : (BM >= 256 ? 3 : 4);
  constexpr int R = SP == 1 ? 2 : 1;
  allow_lds(reinterpret_cast<const void*>(&conv_gemm_kernel<BM, BN, MT, NT, S, KIND, XF, SP>));
  const int m_tiles = ceil_div(a.M, BM), n_tiles = ceil_div(a.cs_out, BN);
  int se_imgs = 0;
  if (a.in_xform == IN_SE_SCALE) {
    M2S_CHECK(KIND == KIND_GEMM && a.OH > 0 && a.cs_in % 8 == 0, "SE scale needs the GEMM kind with OH = rows per image");
    se_imgs = se_images(BM, a.OH);
  }
  const size_t lds = (size_t)S * (R * (BM + BN) + 16) * ROW + (size_t)se_imgs * a.cs_in * sizeof(float);
  M2S_CHECK(lds <= 160 * 1024, "conv_gemm: LDS budget");
  // Split K where the tiles fill under half a round of the chip's workgroup slots (one clip, the 8 x 4 acoustic
  // batch: a few dozen tiles walking 20..88 K steps each): nks K ranges of >= 4 steps, up to a full round and at
  // most 8 (the partial sums' round trip grows with nks: same-box A/B at one clip / configs[1], M2S_KSPLIT_MAX 4 / 8
  // / 16: 2.378 / 2.286 / 2.300 ms and 1.106 / 1.107 / 1.119 ms, gpurun_out/r06d/ab.txt).
  // M2S_KSPLIT=n forces n ranges (A/B, tests; 1 = never split).
  int nst = 0;
  for (int i = 0; i < (KIND == KIND_CONV1D ? phases : 1); ++i) nst = std::max(nst, b.a[i].kp / 32);
  const int tiles = m_tiles * n_tiles * phases;
  const int slots = device_cus() * std::max(1, std::min(2, (int)(160 * 1024 / lds)));
  const char* fe = getenv("M2S_KSPLIT");  // read per launch: tests switch it between engines of one process
  const int force = fe ? atoi(fe) : 0;
  int nks = 1;
  if (force > 0)
    nks = std::min(force, std::max(1, nst));
  else if (2 * tiles <= slots && nst >= 8) {
    const char* mx = getenv("M2S_KSPLIT_MAX");  // A/B of the split count (tools/ab_env.py)
    const char* ms = getenv("M2S_KSPLIT_MINST");
    nks = std::max(1, std::min({slots / tiles, nst / (ms ? std::max(1, atoi(ms)) : 4), mx ? std::max(1, atoi(mx)) : 8}));
  }
  const size_t part_bytes = (size_t)phases * nks * a.M * a.cs_out * sizeof(float);
  if (nks > 1 && part_bytes > ((size_t)256 << 20)) nks = 1;
  float* kpart = nks > 1 ? ksplit_scratch(s, part_bytes) : nullptr;
  if (!kpart) nks = 1;  // (a stream under graph capture with no scratch large enough)
  dim3 grid(m_tiles * n_tiles, nks, phases);
  char name[96];
  static const bool detail = getenv("M2S_PROF_DETAIL") != nullptr;
  if (detail)  // per-layer records for analysis: K x N and rows per launch
    snprintf(name, sizeof(name), "conv_gemm<%s,%dx%d%s> K%d N%d M%d", kname(KIND), BM, BN, SP == 1 ? ",x3" : SP == 2 ? ",e4m3" : "", a.kp, a.cs_out, a.M);
  else
    snprintf(name, sizeof(name), "conv_gemm_kernel<%d, %d, %d, %d, %d, %d, %d, %d>", BM, BN, MT, NT, S, KIND, XF, SP);
  {
    ProfScope ps(name, flops, bytes, s);
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MT, NT, S, KIND, XF, SP>), grid, dim3(256), lds, s, b, n_tiles, se_imgs, kpart);
  }
  if (nks > 1) {
    // the partial sums are a spill (written and read back once), not compulsory bytes
    snprintf(name, sizeof(name), "conv_gemm_ksum_kernel<%d, %d>", KIND, SP);
    ProfScope ps(name, 0.0, 0.0, s, 2.0 * part_bytes);
    const long threads = (long)a.M * (a.cs_out / 4);
    hipLaunchKernelGGL((conv_gemm_ksum_kernel<KIND, SP>), dim3((unsigned)((threads + 255) / 256), 1, phases), dim3(256), 0, s, b,
                       kpart, nks);
  }
}

template <int KIND, int XF, int SP>
void launch_kind_xf(const ConvBatch& a, hipStream_t s, int phases, double flops, double bytes) {
  const int n = a.a[0].cs_out;
  if constexpr (SP != 0) {  // split / e4m3 operands: 16/32/64-wide tiles for narrow outputs, else 128 x 128
    if (n <= 16)
      return launch_tile<256, 16, 4, 1, KIND, XF, SP>(a, s, phases, flops, bytes);
    if (n <= 32)  // (a 128 x 32 tile at three stages: 0.1 ms per step slower on the C = 32 MRF convs)
      return launch_tile<256, 32, 4, 2, KIND, XF, SP>(a, s, phases, flops, bytes);
    if (n <= 64 || (n % 128 != 0 && ceil_div(n, 64) * 64 < ceil_div(n, 128) * 128)) {
      // split 64-wide outputs: 128 x 64 at three stages (77 KB, two workgroups per CU) instead of
      // 256 x 64 at two (84 KB, one per CU): the C = 64 MRF convs 3.7 -> 3.1 ms per step
      if (SP == 1 && n <= 64) return launch_tile<128, 64, 4, 2, KIND, XF, SP>(a, s, phases, flops, bytes);
      return launch_tile<256, 64, 4, 4, KIND, XF, SP>(a, s, phases, flops, bytes);
    }
    if constexpr (SP == 1 && KIND == KIND_CONV1D && XF == IN_NONE) {  // A/B: the split MRF convs on 128 x 64 tiles
      static const bool bn64 = getenv("M2S_CG_BN64") && atoi(getenv("M2S_CG_BN64")) == 1;  // (3 stages, 2 per CU)
      if (bn64) return launch_tile<128, 64, 4, 2, KIND, XF, SP>(a, s, phases, flops, bytes);
      // A/B: 3 or 4 stages at one workgroup per CU (101 / 135 KB) instead of 2 stages at two
      static const int stg = getenv("M2S_CG_STAGES") ? atoi(getenv("M2S_CG_STAGES")) : 0;
      if (stg == 3) return launch_tile<128, 128, 4, 4, KIND, XF, SP, 3>(a, s, phases, flops, bytes);
      if (stg == 4) return launch_tile<128, 128, 4, 4, KIND, XF, SP, 4>(a, s, phases, flops, bytes);
    }
    return launch_tile<128, 128, 4, 4, KIND, XF, SP>(a, s, phases, flops, bytes);
  } else {
  if constexpr (KIND == KIND_GEMM || KIND == KIND_CONV2D) if (a.a[0].M >= 256 * 256 && n > 128 &&
                                                               ((n <= 256 && a.a[0].kp >= 512) || KIND == KIND_GEMM)) {
    // long-K 1x1 GEMMs and 3x3 convs with 129..256 outputs: one 256-wide n tile reads (gathers)
    // the activations once instead of twice (b5 conv_pwl 1248 -> 208: 13.5 -> 10.0 ms per 4 steps;
    // b2 conv_exp 3x3 56 -> 224: 1.10 -> 0.91 ms per launch); also every wide 1x1 GEMM (the
    // stride-2 IR expansions K 64 / 128 -> 224 / 736: 526 -> 457 us per launch).  A 256x128 tile
    // for n <= 128 measured slower at every K (one wave per SIMD at 272 registers).
    return launch_tile<128, 256, 4, 8, KIND, XF, 0>(a, s, phases, flops, bytes);
  }
  if constexpr (KIND == KIND_GEMM)
    if (a.a[0].M >= 256 * 256 && n > 64 && n <= 128 && a.a[0].kp >= 384) {
      // 256 rows x 128 outputs at two waves per SIMD: the weight tile (K x 128) is re-read from L2
      // once per 256 rows instead of per 128 (the SE-scaled conv_pwl of blocks.3/4: K 416..736)
      return launch_tile<256, 128, 8, 4, KIND, XF, 0>(a, s, phases, flops, bytes);
    }
  if (n <= 16)
    launch_tile<256, 16, 4, 1, KIND, XF, 0>(a, s, phases, flops, bytes);
  else if (n <= 32)
    launch_tile<256, 32, 4, 2, KIND, XF, 0>(a, s, phases, flops, bytes);
  else if (n <= 64 || (n % 128 != 0 && ceil_div(n, 64) * 64 < ceil_div(n, 128) * 128))
    launch_tile<256, 64, 4, 4, KIND, XF, 0>(a, s, phases, flops, bytes);
  else
    launch_tile<128, 128, 4, 4, KIND, XF, 0>(a, s, phases, flops, bytes);
  }
}

// Only the (kind, input transform) pairs the hot path uses are instantiated.
template <int KIND, int SP>
void launch_kind(const ConvArgs& a0, hipStream_t s, int phases, double flops, double bytes, const ConvBatch* batch = nullptr) {
  ConvBatch bl;
  if (!batch) {
    std::memset(&bl, 0, sizeof(bl));
    bl.a[0] = a0;
  }
  const ConvBatch& a = batch ? *batch : bl;
  if (a0.in_xform == IN_NONE) {
    launch_kind_xf<KIND, IN_NONE, SP>(a, s, phases, flops, bytes);
  } else if constexpr (KIND == KIND_CONV1D || KIND == KIND_CONVT) {
    M2S_CHECK(a0.in_xform == IN_LRELU, "conv_gemm: 1-D kinds take LeakyReLU inputs only");
    launch_kind_xf<KIND, IN_LRELU, SP>(a, s, phases, flops, bytes);
  } else if constexpr (KIND == KIND_GEMM) {
    M2S_CHECK(a0.in_xform == IN_SE_SCALE, "conv_gemm: GEMM kind takes SE-scaled inputs only");
    launch_kind_xf<KIND, IN_SE_SCALE, SP>(a, s, phases, flops, bytes);
  } else {
    M2S_CHECK(false, "conv_gemm: 2-D convs take untransformed inputs");
  }
}

}  // namespace

void launch_conv_gemm_batch(const ConvArgs* as, int n, hipStream_t s, double flops, double bytes) {
  M2S_CHECK(n >= 1 && n <= CONV_BATCH, "conv_gemm batch: 1..CONV_BATCH convs");
  const ConvArgs& a = as[0];
  M2S_CHECK(a.kind == KIND_CONV1D && a.cs_in >= 32 && a.cs_in % 32 == 0 && a.cs_out % 4 == 0, "conv_gemm batch: 1-D convs, cs_in % 32 == 0");
  ConvBatch b;
  std::memset(&b, 0, sizeof(b));
  for (int i = 0; i < n; ++i) {
    const ConvArgs& c = as[i];
    M2S_CHECK(c.kind == a.kind && c.M == a.M && c.cs_in == a.cs_in && c.cs_out == a.cs_out && c.n_pad == a.n_pad &&
                  c.in_xform == a.in_xform && c.L_in == a.L_in && c.L_out == a.L_out,
              "conv_gemm batch: convs of one shape");
    M2S_CHECK(c.kp % 32 == 0 && c.kp >= c.ntaps * c.cs_in && c.ntaps <= 31, "conv_gemm batch: kp / taps");
    // every conv of the batch reads its own operands and writes its own output (grid.z = i below):
    // no null pointer, and no output aliasing an input or another conv's output
    M2S_CHECK(c.x && c.w && c.bias && c.y && c.y != c.x && c.y != c.res, "conv_gemm batch: operand pointers");
    for (int j = 0; j < i; ++j) M2S_CHECK(as[j].y != c.y, "conv_gemm batch: two convs write one output");
    M2S_CHECK((double)(c.M / c.L_out) * c.L_in * c.cs_in * 2 < 2147483647.0, "conv_gemm batch: 32-bit offsets");
    b.a[i] = c;
  }
  if (a.M <= 0) return;
  launch_kind<KIND_CONV1D, 1>(a, s, n, flops, bytes, &b);
  M2S_HIP(hipGetLastError());
}

void launch_conv_gemm(const ConvArgs& a, bool split, hipStream_t s, double flops, double bytes) {
  M2S_CHECK(a.cs_in % 8 == 0 && a.cs_out % 4 == 0, "conv_gemm: channel strides");
  M2S_CHECK(a.cs_in >= 32 ? a.cs_in % 32 == 0 : 32 % a.cs_in == 0, "conv_gemm: channel stride vs the 32-wide K step");
  M2S_CHECK(a.ntaps <= 31, "conv_gemm: at most 31 taps");
  {  // input element offsets are 32-bit in the kernel
    const double in_elems = a.kind == KIND_CONV2D ? (double)(a.M / (a.OH * a.OW)) * a.IH * a.IW * a.cs_in
                            : a.kind == KIND_CONV1D ? (double)(a.M / a.L_out) * a.L_in * a.cs_in
                            : a.kind == KIND_CONVT  ? (double)a.M * a.cs_in
                                                    : (double)a.M * a.cs_in;
    M2S_CHECK(in_elems * (split ? 2 : 1) < 2147483647.0, "conv_gemm: input too large for 32-bit offsets (use a smaller chunk)");
  }
  M2S_CHECK(a.kp % 32 == 0 && a.kp >= a.ntaps * a.cs_in, "conv_gemm: kp");
  M2S_CHECK(a.kind != KIND_CONV2D || a.ks == 3, "conv_gemm: 2-D kernels are 3x3 (1x1 runs as GEMM)");
  if (a.M <= 0) return;
  M2S_CHECK(!(split && a.wscale), "conv_gemm: e4m3 operands take bf16 storage");
  if (split) {
    switch (a.kind) {
      case KIND_CONV2D: launch_kind<KIND_CONV2D, 1>(a, s, 1, flops, bytes); break;
      case KIND_CONV1D: launch_kind<KIND_CONV1D, 1>(a, s, 1, flops, bytes); break;
      case KIND_CONVT: launch_kind<KIND_CONVT, 1>(a, s, a.ct_u, flops, bytes); break;
      case KIND_GEMM: launch_kind<KIND_GEMM, 1>(a, s, 1, flops, bytes); break;
      default: M2S_CHECK(false, "conv_gemm: bad kind");
    }
    M2S_HIP(hipGetLastError());
    return;
  }
  if (a.wscale) {  // e4m3 operands
    switch (a.kind) {
      case KIND_CONV2D: launch_kind<KIND_CONV2D, 2>(a, s, 1, flops, bytes); break;
      case KIND_CONV1D: launch_kind<KIND_CONV1D, 2>(a, s, 1, flops, bytes); break;
      case KIND_CONVT: launch_kind<KIND_CONVT, 2>(a, s, a.ct_u, flops, bytes); break;
      case KIND_GEMM: launch_kind<KIND_GEMM, 2>(a, s, 1, flops, bytes); break;
      default: M2S_CHECK(false, "conv_gemm: bad kind");
    }
    M2S_HIP(hipGetLastError());
    return;
  }
  if (conv_halo_supported(a)) return launch_conv_halo(a, s, flops, bytes);
  switch (a.kind) {
    case KIND_CONV2D: launch_kind<KIND_CONV2D, 0>(a, s, 1, flops, bytes); break;
    case KIND_CONV1D: launch_kind<KIND_CONV1D, 0>(a, s, 1, flops, bytes); break;
    case KIND_CONVT: launch_kind<KIND_CONVT, 0>(a, s, a.ct_u, flops, bytes); break;
    case KIND_GEMM: launch_kind<KIND_GEMM, 0>(a, s, 1, flops, bytes); break;
    default: M2S_CHECK(false, "conv_gemm: bad kind");
  }
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
