// GEMMs over 128-byte K-step rows: one LDS row of an operand row per K step, filled by LDS-DMA through a
// 3-slot ring.  Three kinds (one kernel template, gemm128_kernel<KIND, WM, WN, NT, S>):
//
// KIND_F8_SE (fp8 engines, the IR blocks' SE-gated conv_pwl), on the block-scaled MFMA
//   v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate per clock; MI355X_MICROARCH.md Matrix cores),
//   K step = 128 e4m3 channels:
//   y[m][n] = wscale[n] * sum_k W8[n][k] * e4m3(gate[img(m)][k] * X8[m][k]) + bias[n] (+ res[m][n])
// KIND_F8_C1D (fp8 engines, the HiFi-GAN MRF convs at C = 64 / 128 / 256, models.py:11-49: causal dilated
//   Conv1d, the operand already LeakyReLU'd by its producer), same MFMA (C = 64 / 32: a K step holds 128 / C taps,
//   C / 16 of the row's 16-byte chunks each, in tap order; a tap count not a multiple ends on zero taps):
//   v[m][n] = wscale[n] * sum_{t,c} W8[n][t C + c] * X8[b, l + t dil - (k - 1) dil][c] + bias[n] (+ res[m][n])
//   y (bf16) = v, or the MRF running sum (y + v) [/ nk]; y8 (e4m3) = lrelu(v) for the next conv's operand.
// KIND_SP_SE (bf16x3 engines, the same SE-gated conv_pwl in split fp32), K step = 32 channels as
//   [hi 32 | lo 32] bf16 (the interleaved operand ir_ws / ir_pwdw write, m2s_common.hpp il_st8), three
//   v_mfma_f32_16x16x32_bf16 terms per product (hi*hi + hi*lo + lo*hi), gate applied in fp32 and re-split:
//   y[m][n] = sum_k W[n][k] * (gate[img(m)][k] * X[m][k]) + bias[n] (+ res[m][n]), all split fp32.
//
// The InvertedResidual tail of timm's EfficientNetV2 (se.conv_expand gate x conv_pwl + bn3 + skip;
// mri_acoustic_model.py:28-34,46).  Every wave owns 64 rows that lie in ONE image (P % 64 == 0), so its gates
// per K step are shared by its four row fragments and the gate is applied to the activation fragments in
// registers (the gate is in (0, 1): no new saturation in e4m3).  The per-channel fp8 weight scale is applied
// in the epilogue; the E8M0 block scales are 1.
#include "conv_igemm.hpp"
#include "kernels.hpp"
#include "prof.hpp"

#include <cstdlib>
#include <cstdlib>
#include <cstring>

namespace m2s {
namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int F8_ROW = 128;            // bytes per LDS row: 128 e4m3 = one K step
constexpr int E8M0_ONE = 0x7f7f7f7f;   // 2^0 block scale in every byte

__device__ __attribute__((aligned(16))) uint4 g_zero_f8[4];  // padding lanes' DMA source

// Physical 16-byte chunk of logical chunk c in row r: c ^ f(r), f(r) = ((r >> 1) & 1) | (r & 4).  A
// fragment is two ds_read_b128 (lane (g = lane >> 4, r = lane & 15) reads chunks 2g and 2g + 1 of row r);
// with 128-byte rows a row pair spans the 64 banks, and this f puts the 16 lanes of each of ds_read_b128's
// lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...; MI355X_MICROARCH.md LDS table) on 16 distinct
// 16-byte bank quads for both reads (exhaustive check over the XOR swizzles of the row's low 4 bits).
__device__ __forceinline__ int f8_swz(int r) { return ((r >> 1) & 1) | (r & 4); }
// SP: a fragment reads chunks g (hi) and g + 4 (lo); f(r) = r & 6 is conflict-free for that pair (same check)
template <bool SP>
__device__ __forceinline__ int swz128(int r) { return SP ? (r & 6) : f8_swz(r); }

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 4 e4m3 (one dword) x 4 gates -> 4 e4m3
__device__ __forceinline__ int gate4(int d, const float* s) {
  const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(d, false);
  const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(d, true);
  const int r = __builtin_amdgcn_cvt_pk_fp8_f32(lo[0] * s[0], lo[1] * s[1], 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(hi[0] * s[2], hi[1] * s[3], r, true);
}

enum { KIND_F8_SE = 0, KIND_F8_C1D = 1, KIND_SP_SE = 2 };

struct G128Args {
  const uint8_t* x;     // e4m3 [M][cs_in]; SP: interleaved split [M][cs_in / 32][hi 32 | lo 32] bf16
  const uint8_t* w;     // e4m3 [n_pad][kp], zero beyond the input channels; SP: bf16 rows [hi kp | lo kp]
  const float* wscale;  // [n_pad]
  const float* bias;    // [n_pad]
  const bf16_t* gate;   // SE: [M / P][cs_in] (SP: split [M / P][hi cs_in | lo cs_in])
  const bf16_t* res;    // [M][cs_out] or null (SP: split [M][hi cs_out | lo cs_out])
  bf16_t* y;            // [M][cs_out] bf16 or null (SP: split)
  uint8_t* y8;          // C1D: [M][cs_out] e4m3 of lrelu(v, slope8); F8 SE: [M][ld8] e4m3 of v; or null
  int M, P, cs_in, kp, cs_out, n_tiles, nimg;  // P: SE rows per image, C1D sequence length L
  int ld8;                                      // F8 SE: y8 row bytes
  int dil, pad_left, accum;                     // C1D: tap dilation, causal left pad, MRF sum mode (0 / 1 / 2)
  int ntap;                                     // C1D: taps (C < 128: a K step holds 128 / C)
  float accum_div, slope8;
};

template <int KIND, int WM, int WN, int NT, int S>
__global__ void __launch_bounds__(64 * WM * WN, 1) gemm128_kernel(const G128Args a) {
  constexpr int NW = WM * WN, NTHR = 64 * NW;  // 4 waves (one per SIMD) or 8 (two per SIMD)
  constexpr bool SP = KIND == KIND_SP_SE;  // split fp32 operands, three bf16 MFMA terms
  constexpr bool SE = KIND == KIND_F8_SE || SP;
  constexpr int BM = 64 * WM, BN = 16 * NT * WN, MT = 4;
  constexpr int A_BLK = BN / 8, TB = A_BLK + BM / 8;  // 8-row (1 KB) DMA blocks: weights, then activations
  static_assert((NW == 4 || NW == 8) && TB % NW == 0, "bad tile");
  constexpr int PER = TB / NW;  // DMA instructions per wave per stage
  constexpr int SLOT = (BN + BM) * F8_ROW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* gtab = reinterpret_cast<float*>(smem + S * SLOT);  // [nimg][kp] gates of the tile's images

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, r16 = lane & 15;

  // XCD-aware block -> (m tile, n tile): the n tiles of one m tile share blockIdx % 8 (one XCD)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int mt = wid / a.n_tiles, nt = wid - mt * a.n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nsteps = SP ? a.kp / 32 : a.kp / F8_ROW;
  const int img0 = m0 / a.P;

  // ---- SE: gate table of the tile's images (fp32, zero past cs_in) ---------------------------------
  if constexpr (SE) {
    for (int i = tid; i < a.nimg * a.kp; i += NTHR) {
      const int im = i / a.kp, k = i - im * a.kp;
      const int img = img0 + im;
      const bf16_t* gp = a.gate + (size_t)img * a.cs_in * (SP ? 2 : 1) + k;
      gtab[i] = (k < a.cs_in && img * a.P < a.M) ? (SP ? bf2f(gp[0]) + bf2f(gp[a.cs_in]) : bf2f(gp[0])) : 0.f;
    }
    __syncthreads();
  }

  // ---- DMA roles: block b = wave + 4 j; lane -> (row lane >> 3 of the block, physical chunk lane & 7) --
  const int lrow = lane >> 3, pch = lane & 7;
  const char* zp = reinterpret_cast<const char*>(g_zero_f8);
  asm volatile("" : "+s"(zp));
  // SE: K step st = input channels [128 st, 128 st + 128) of the row.  C1D: tap t = st / gpt, channels
  // 128 (st % gpt) .. of input position l + t dil - pad_left of the row's sequence (zero outside [0, L)).
  const int tpk = !SE && a.cs_in < F8_ROW ? F8_ROW / a.cs_in : 1;  // C1D: taps a K step (C = 64: 2, C = 32: 4)
  const int cpt = 8 / tpk;                                        // ... and 16-byte chunks a tap
  const bool two = tpk > 1;
  const int gpt = two ? 1 : a.cs_in / F8_ROW;                      // C1D: K steps per tap
  const uint8_t* srow[PER];  // row base (+ logical chunk offset; C1D: at tap 0 with the pad), or null
  int cofs[PER];             // SE: logical chunk byte offset within the K step
  int lpos[PER];             // C1D: position of tap 0 within the sequence (l - pad_left)
  int thalf[PER];            // C1D, C < 128: the chunk's tap within the K step
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int blk = wave + NW * j;
    const int lr = blk * 8 + lrow;  // LDS row within the slot
    const int c = pch ^ swz128<SP>(lr & 15);
    cofs[j] = c * 16;
    lpos[j] = 0;
    thalf[j] = two ? c / cpt : 0;
    if (blk < A_BLK) {  // SP: hi chunks 0-3 from the row's hi half, lo chunks 4-7 from its lo half
      srow[j] = SP ? a.w + (size_t)(n0 + lr) * a.kp * 4 + (c < 4 ? c * 16 : a.kp * 2 + (c - 4) * 16)
                   : a.w + (size_t)(n0 + lr) * a.kp + c * 16;
    } else {
      const int m = m0 + lr - BN;
      if constexpr (SE) {
        srow[j] = m < a.M ? a.x + (size_t)m * a.cs_in * (SP ? 4 : 1) + c * 16 : nullptr;
      } else {
        const int l = m - (m / a.P) * a.P;
        lpos[j] = l - a.pad_left;
        srow[j] = m < a.M ? a.x + ((long)m - a.pad_left) * a.cs_in + (two ? c % cpt : c) * 16 : nullptr;
      }
    }
  }
  auto issue = [&](int st, int slot) {
    char* base = smem + slot * SLOT;
    const int t = SE ? 0 : st / gpt, cg = SE ? st : st - t * gpt;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int blk = wave + NW * j;
      const void* src;
      if (blk < A_BLK) {
        src = srow[j] + st * (SP ? 64 : F8_ROW);
      } else if constexpr (SP) {
        src = srow[j] ? static_cast<const void*>(srow[j] + st * F8_ROW) : static_cast<const void*>(zp);
      } else if constexpr (SE) {
        src = srow[j] && st * F8_ROW + cofs[j] < a.cs_in ? static_cast<const void*>(srow[j] + st * F8_ROW) : zp;
      } else if (two) {
        const int tt = tpk * st + thalf[j], lp = lpos[j] + tt * a.dil;
        src = srow[j] && tt < a.ntap && lp >= 0 && lp < a.P ? static_cast<const void*>(srow[j] + (long)tt * a.dil * a.cs_in)
                                                             : static_cast<const void*>(zp);
      } else {
        const int lp = lpos[j] + t * a.dil;
        src = srow[j] && lp >= 0 && lp < a.P ? static_cast<const void*>(srow[j] + ((long)t * a.dil * a.cs_in + cg * F8_ROW))
                                             : static_cast<const void*>(zp);
      }
      dma16(src, base + blk * 1024);
    }
  };

  f32x4 acc[NT][MT];
#pragma unroll
  for (int ni = 0; ni < NT; ++ni)
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wimg = SE ? (min(m0 + wm * 64, a.M - 1)) / a.P - img0 : 0;  // this wave's image within the table
  const uint32_t gaddr0 = (uint32_t)(uintptr_t)(gtab + wimg * a.kp + g * (SP ? 8 : 32));
  const int sw = swz128<SP>(r16);
  // a lane's two 16-byte chunks of a fragment row: e4m3 2g, 2g + 1 (32 consecutive k); SP hi g, lo g + 4
  const int ch0 = ((SP ? g : 2 * g) ^ sw) << 4, ch1 = ((SP ? g + 4 : 2 * g + 1) ^ sw) << 4;

  // LDS reads through inline asm: a plain ds_read after an LDS-DMA makes hipcc wait for every DMA in
  // flight (vmcnt(0)) before it, which would drain the pipeline each K step; the data dependence on the
  // DMA is the barrier after the counted vmcnt wait of the loop.  Outputs of a read statement are consumed
  // only through a later `s_waitcnt lgkmcnt` statement that takes them as "+v" operands.
  const uint32_t sm0 = (uint32_t)(uintptr_t)smem;
  const uint32_t a_lds0 = sm0 + (uint32_t)((wn * NT * 16 + r16) * F8_ROW);
  const uint32_t b_lds0 = sm0 + (uint32_t)((BN + wm * 64 + r16) * F8_ROW);
  auto compute = [&](int st, int slot) {
    const uint32_t so = (uint32_t)(slot * SLOT);
    if constexpr (SP) {
      // 8 gates (k = 32 st + 8 g + j) and the MT activation fragments (hi chunk g, lo chunk g + 4 of a row)
      f32x4 q0, q1;
      u32x4 bh[MT], bl[MT];
      const uint32_t ga = gaddr0 + st * 32 * 4, ba0 = b_lds0 + so + ch0, ba1 = b_lds0 + so + ch1;
      asm volatile(
          "ds_read_b128 %0, %10\n\tds_read_b128 %1, %10 offset:16\n\t"
          "ds_read_b128 %2, %11\n\tds_read_b128 %3, %12\n\tds_read_b128 %4, %11 offset:2048\n\t"
          "ds_read_b128 %5, %12 offset:2048\n\tds_read_b128 %6, %11 offset:4096\n\tds_read_b128 %7, %12 offset:4096\n\t"
          "ds_read_b128 %8, %11 offset:6144\n\tds_read_b128 %9, %12 offset:6144\n\ts_waitcnt lgkmcnt(0)"
          : "=&v"(q0), "=&v"(q1), "=&v"(bh[0]), "=&v"(bl[0]), "=&v"(bh[1]), "=&v"(bl[1]), "=&v"(bh[2]), "=&v"(bl[2]),
            "=&v"(bh[3]), "=&v"(bl[3])
          : "v"(ga), "v"(ba0), "v"(ba1)
          : "memory");
      static_assert(MT == 4, "the read statement above covers four 16-row fragments");
      u32x4 ah[NT], al[NT];
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const uint32_t aa = a_lds0 + so + ni * 16 * F8_ROW;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3" : "=&v"(ah[ni]), "=&v"(al[ni]) : "v"(aa + ch0), "v"(aa + ch1) : "memory");
      }
      // gate in fp32 on hi + lo, re-split (17 significant bits kept)
      const float gsc[8] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
      bf16x8 xh[MT], xl[MT];
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        float v[8], w[8];
        unpack_bf16x4(make_uint2(bh[mi][0], bh[mi][1]), v);
        unpack_bf16x4(make_uint2(bh[mi][2], bh[mi][3]), v + 4);
        unpack_bf16x4(make_uint2(bl[mi][0], bl[mi][1]), w);
        unpack_bf16x4(make_uint2(bl[mi][2], bl[mi][3]), w + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (v[j] + w[j]) * gsc[j];
        uint2 h0, l0, h1, l1;
        split4(v, h0, l0);
        split4(v + 4, h1, l1);
        xh[mi] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
        xl[mi] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
      }
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(ah[ni]), "+v"(al[ni]) : "n"(2 * (NT - 1 - ni)));
        const bf16x8 wh = __builtin_bit_cast(bf16x8, ah[ni]), wl = __builtin_bit_cast(bf16x8, al[ni]);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh[mi], acc[ni][mi], 0, 0, 0);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl[mi], acc[ni][mi], 0, 0, 0);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh[mi], acc[ni][mi], 0, 0, 0);
        }
      }
      return;
    }
    // the wave's 32 gates of this K step (k = 128 st + 32 g + j) and its MT activation fragments
    f32x4 q[8];
    u32x4 b0[MT], b1[MT];
    if constexpr (!SE) {
      const uint32_t ba0 = b_lds0 + so + ch0, ba1 = b_lds0 + so + ch1;
      asm volatile(
          "ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %8 offset:2048\n\t"
          "ds_read_b128 %3, %9 offset:2048\n\tds_read_b128 %4, %8 offset:4096\n\tds_read_b128 %5, %9 offset:4096\n\t"
          "ds_read_b128 %6, %8 offset:6144\n\tds_read_b128 %7, %9 offset:6144"
          : "=&v"(b0[0]), "=&v"(b1[0]), "=&v"(b0[1]), "=&v"(b1[1]), "=&v"(b0[2]), "=&v"(b1[2]), "=&v"(b0[3]), "=&v"(b1[3])
          : "v"(ba0), "v"(ba1)
          : "memory");
    } else {
      const uint32_t ga = gaddr0 + st * F8_ROW * 4, ba0 = b_lds0 + so + ch0, ba1 = b_lds0 + so + ch1;
      asm volatile(
          "ds_read_b128 %0, %16\n\tds_read_b128 %1, %16 offset:16\n\tds_read_b128 %2, %16 offset:32\n\t"
          "ds_read_b128 %3, %16 offset:48\n\tds_read_b128 %4, %16 offset:64\n\tds_read_b128 %5, %16 offset:80\n\t"
          "ds_read_b128 %6, %16 offset:96\n\tds_read_b128 %7, %16 offset:112\n\t"
          "ds_read_b128 %8, %17\n\tds_read_b128 %9, %18\n\tds_read_b128 %10, %17 offset:2048\n\t"
          "ds_read_b128 %11, %18 offset:2048\n\tds_read_b128 %12, %17 offset:4096\n\tds_read_b128 %13, %18 offset:4096\n\t"
          "ds_read_b128 %14, %17 offset:6144\n\tds_read_b128 %15, %18 offset:6144\n\ts_waitcnt lgkmcnt(0)"
          : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]),
            "=&v"(b0[0]), "=&v"(b1[0]), "=&v"(b0[1]), "=&v"(b1[1]), "=&v"(b0[2]), "=&v"(b1[2]), "=&v"(b0[3]),
            "=&v"(b1[3])
          : "v"(ga), "v"(ba0), "v"(ba1)
          : "memory");
    }
    static_assert(MT == 4, "the read statement above covers four 16-row fragments");
    // the NT weight fragments: all reads issued now, consumed in order behind counted waits
    u32x4 a0[NT], a1[NT];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const uint32_t aa = a_lds0 + so + ni * 16 * F8_ROW;
      asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3" : "=&v"(a0[ni]), "=&v"(a1[ni]) : "v"(aa + ch0), "v"(aa + ch1) : "memory");
    }
    i32x8 bx[MT];
    if constexpr (SE) {
      float gs[32];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        gs[4 * i] = q[i][0];
        gs[4 * i + 1] = q[i][1];
        gs[4 * i + 2] = q[i][2];
        gs[4 * i + 3] = q[i][3];
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int d[8] = {(int)b0[mi][0], (int)b0[mi][1], (int)b0[mi][2], (int)b0[mi][3],
                          (int)b1[mi][0], (int)b1[mi][1], (int)b1[mi][2], (int)b1[mi][3]};
#pragma unroll
        for (int i = 0; i < 8; ++i) bx[mi][i] = gate4(d[i], gs + 4 * i);
      }
    } else {  // the activation reads were issued before the NT weight reads: 2 NT younger reads
      asm volatile("s_waitcnt lgkmcnt(%8)"
                   : "+v"(b0[0]), "+v"(b1[0]), "+v"(b0[1]), "+v"(b1[1]), "+v"(b0[2]), "+v"(b1[2]), "+v"(b0[3]), "+v"(b1[3])
                   : "n"(2 * NT > 15 ? 15 : 2 * NT));
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        bx[mi] = i32x8{(int)b0[mi][0], (int)b0[mi][1], (int)b0[mi][2], (int)b0[mi][3],
                       (int)b1[mi][0], (int)b1[mi][1], (int)b1[mi][2], (int)b1[mi][3]};
    }
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a0[ni]), "+v"(a1[ni]) : "n"(2 * (NT - 1 - ni)));
      const i32x8 af = {(int)a0[ni][0], (int)a0[ni][1], (int)a0[ni][2], (int)a0[ni][3],
                        (int)a1[ni][0], (int)a1[ni][1], (int)a1[ni][2], (int)a1[ni][3]};
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
        acc[ni][mi] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bx[mi], acc[ni][mi], 0, 0, 0, E8M0_ONE, 0,
                                                                       E8M0_ONE);
    }
  };

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nsteps) issue(s, s);
  for (int st = 0; st < nsteps; ++st) {
    const int younger = min(S - 2, nsteps - 1 - st);  // stages issued after st and still in flight
    if (younger >= 2)
      wait_vm<2 * PER>();
    else if (younger == 1)
      wait_vm<PER>();
    else
      wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // stage st landed everywhere; slot (st - 1) % S is free
    if (st + S - 1 < nsteps) issue(st + S - 1, (st + S - 1) % S);
    compute(st, st % S);
  }

  // ---- epilogue: lane = 4 consecutive output channels of one position ------------------------------
  // the skip operand is fetched for the whole tile first (one wait), not load -> wait -> store per piece
  const bf16_t* __restrict__ R = a.res;
  bf16_t* __restrict__ Y = a.y;
  constexpr int RP = SP ? 2 : 1;  // planes of the residual / output rows
  uint2 rv[MT][NT][RP];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int m = m0 + wm * 64 + mi * 16 + r16, n4 = n0 + wn * NT * 16 + ni * 16 + 4 * g;
#pragma unroll
      for (int h = 0; h < RP; ++h)
        rv[mi][ni][h] = (R && m < a.M && n4 < a.cs_out)
                            ? *reinterpret_cast<const uint2*>(R + (size_t)m * a.cs_out * RP + h * a.cs_out + n4)
                            : make_uint2(0u, 0u);
    }
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const int m = m0 + wm * 64 + mi * 16 + r16;
    if (m >= a.M) continue;
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int n4 = n0 + wn * NT * 16 + ni * 16 + 4 * g;
      if (n4 >= a.cs_out) continue;
      const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
      float r[4];
      unpack_bf16x4(rv[mi][ni][0], r);
      if constexpr (SP) {
        float rl[4];
        unpack_bf16x4(rv[mi][ni][RP - 1], rl);
        const float v[4] = {acc[ni][mi][0] + bb.x + (r[0] + rl[0]), acc[ni][mi][1] + bb.y + (r[1] + rl[1]),
                            acc[ni][mi][2] + bb.z + (r[2] + rl[2]), acc[ni][mi][3] + bb.w + (r[3] + rl[3])};
        uint2 hi, lo;
        split4(v, hi, lo);
        bf16_t* yo = Y + (size_t)m * a.cs_out * 2 + n4;
        *reinterpret_cast<uint2*>(yo) = hi;
        *reinterpret_cast<uint2*>(yo + a.cs_out) = lo;
        continue;
      }
      const float4 ws = *reinterpret_cast<const float4*>(a.wscale + n4);
      float v[4] = {fmaf(acc[ni][mi][0], ws.x, bb.x) + r[0], fmaf(acc[ni][mi][1], ws.y, bb.y) + r[1],
                    fmaf(acc[ni][mi][2], ws.z, bb.z) + r[2], fmaf(acc[ni][mi][3], ws.w, bb.w) + r[3]};
      const size_t o = (size_t)m * a.cs_out + n4;
      if (!SE && a.accum) {  // MRF sum of the resblocks in order (models.py:119-125)
        float p[4];
        unpack_bf16x4(*reinterpret_cast<const uint2*>(Y + o), p);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = a.accum == 2 ? (p[j] + v[j]) / a.accum_div : p[j] + v[j];
      }
      const uint2 yb = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      if (SE || Y) *reinterpret_cast<uint2*>(Y + o) = yb;
      // the next IR block's e4m3 expand operand: e4m3 of the STORED bf16 values (one rounding chain, the bytes
      // launch_rows_e4m3 gives when no producer writes them; test_fp8_se_y8_e4m3_handoff_is_exact)
      if (SE && a.y8) *reinterpret_cast<uint32_t*>(a.y8 + (size_t)m * a.ld8 + n4) = e4m3x4_bf16(yb);
      if (!SE && a.y8) {  // the next conv's operand: e4m3(lrelu(v))
        float l[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) l[j] = v[j] > 0.f ? v[j] : v[j] * a.slope8;
        l[4] = l[5] = l[6] = l[7] = 0.f;
        *reinterpret_cast<uint32_t*>(a.y8 + o) = e4m3x8(l).x;
      }
    }
  }
}

template <int KIND, int WM, int WN, int NT, int S = 3>
void launch_tile(G128Args& a, hipStream_t s, double flops, double bytes) {
  constexpr int BM = 64 * WM, BN = 16 * NT * WN;
  const void* fn = reinterpret_cast<const void*>(&gemm128_kernel<KIND, WM, WN, NT, S>);
  allow_lds(fn);
  a.n_tiles = ceil_div(a.cs_out, BN);
  const bool se = KIND != KIND_F8_C1D;
  a.nimg = !se ? 0 : BM % a.P == 0 ? BM / a.P : 1;  // SE: P % BM == 0 otherwise (checked)
  const size_t lds = (size_t)S * (BN + BM) * F8_ROW + (size_t)a.nimg * a.kp * sizeof(float);
  M2S_CHECK(lds <= 160 * 1024, "gemm128: LDS budget");
  M2S_CHECK(!se || BM % a.P == 0 || a.P % BM == 0, "gemm128 SE: tile rows vs image size");
  const dim3 grid(ceil_div(a.M, BM) * a.n_tiles);
  char name[64];
  snprintf(name, sizeof(name), "gemm128_kernel<%d, %d, %d, %d, %d>", KIND, WM, WN, NT, S);  // rocprof's symbol
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((gemm128_kernel<KIND, WM, WN, NT, S>), grid, dim3(64 * WM * WN), lds, s, a);
  M2S_HIP(hipGetLastError());
}

G128Args g128_args() {
  G128Args a;
  std::memset(&a, 0, sizeof(a));
  a.accum_div = 1.f;
  return a;
}

}  // namespace

bool se_gemm_f8_supported(int P, int cs_in, int cs_out) {
  return P % 64 == 0 && cs_in % 16 == 0 && cs_out % 4 == 0 && cs_out <= 224 && (P % 256 == 0 || 256 % P == 0 || cs_out > 128);
}

void launch_se_gemm_f8(const void* x8, int M, int P, int cs_in, const void* w8, int kp, int n_pad, const float* wscale,
                       const float* bias, const void* gate, const void* res, void* y, int cs_out, hipStream_t s,
                       double flops, double bytes, void* y8, int ld8) {
  M2S_CHECK(se_gemm_f8_supported(P, cs_in, cs_out) && kp % F8_ROW == 0 && kp >= cs_in && M % P == 0,
            "se_gemm_f8: unsupported shape");
  M2S_CHECK(!y8 || (ld8 >= cs_out && ld8 % 16 == 0 && y8 != x8), "se_gemm_f8: e4m3 output rows");
  M2S_CHECK(x8 && w8 && wscale && bias && gate && y && y != res && y != x8, "se_gemm_f8: operand pointers");
  M2S_CHECK((double)M * cs_in < 4294967295.0, "se_gemm_f8: input too large");
  if (M <= 0) return;
  G128Args a = g128_args();
  a.x = static_cast<const uint8_t*>(x8);
  a.w = static_cast<const uint8_t*>(w8);
  a.wscale = wscale;
  a.bias = bias;
  a.gate = static_cast<const bf16_t*>(gate);
  a.res = static_cast<const bf16_t*>(res);
  a.y = static_cast<bf16_t*>(y);
  a.y8 = static_cast<uint8_t*>(y8);
  a.ld8 = ld8;
  a.M = M;
  a.P = P;
  a.cs_in = cs_in;
  a.kp = kp;
  a.cs_out = cs_out;
  if (cs_out <= 128) {
    M2S_CHECK(n_pad >= 128, "se_gemm_f8: weight rows");
    launch_tile<KIND_F8_SE, 4, 1, 8>(a, s, flops, bytes);  // 256 x 128: 16x16 maps (one image per tile)
  } else {
    M2S_CHECK(n_pad >= 224, "se_gemm_f8: weight rows");
    launch_tile<KIND_F8_SE, 2, 2, 7>(a, s, flops, bytes);  // 128 x 224: 8x8 maps (two images per tile)
  }
}

bool conv1d_f8_supported(int C, int k) { return (C == 32 || C == 64 || C == 128 || C == 256) && k >= 1 && k <= 31; }

void launch_conv1d_f8(const void* x8, int B, int L, int C, int k, int dil, const void* w8, const float* wscale,
                      const float* bias, const void* res, void* y, void* y8, float slope8, int accum, float accum_div,
                      hipStream_t s, double flops, double bytes) {
  M2S_CHECK(conv1d_f8_supported(C, k) && dil >= 1 && B >= 1 && L >= 1, "conv1d_f8: unsupported shape");
  M2S_CHECK(x8 && w8 && wscale && bias && (y || y8) && (void*)x8 != y && (void*)x8 != y8 && (!res || (res != y8)),
            "conv1d_f8: operand pointers");
  M2S_CHECK(!accum || y, "conv1d_f8: the MRF sum needs y");
  M2S_CHECK((double)B * L * C < 2147483647.0, "conv1d_f8: input too large");
  G128Args a = g128_args();
  a.x = static_cast<const uint8_t*>(x8);
  a.w = static_cast<const uint8_t*>(w8);
  a.wscale = wscale;
  a.bias = bias;
  a.res = static_cast<const bf16_t*>(res);
  a.y = static_cast<bf16_t*>(y);
  a.y8 = static_cast<uint8_t*>(y8);
  a.M = B * L;
  a.P = L;
  a.cs_in = a.cs_out = C;
  a.kp = round_up(k * C, F8_ROW);  // C < 128: the last K step may end on zero taps
  a.ntap = k;
  a.dil = dil;
  a.pad_left = (k - 1) * dil;
  a.accum = accum;
  a.accum_div = accum_div;
  a.slope8 = slope8;
  if (C == 32)
    launch_tile<KIND_F8_C1D, 4, 1, 2>(a, s, flops, bytes);  // 256 positions x 32 channels
  else if (C == 64)
    launch_tile<KIND_F8_C1D, 4, 1, 4>(a, s, flops, bytes);  // 256 positions x 64 channels
  else if (C == 128)
    launch_tile<KIND_F8_C1D, 4, 1, 8>(a, s, flops, bytes);  // 256 positions x 128 channels
  else
    launch_tile<KIND_F8_C1D, 2, 2, 8>(a, s, flops, bytes);  // 128 positions x 256 channels
}

bool se_gemm_sp_supported(int P, int cs_in, int cs_out) {
  return P % 64 == 0 && cs_in % 32 == 0 && cs_out % 4 == 0 && cs_out <= 224 && (P % 256 == 0 || 256 % P == 0 || cs_out > 128);
}

void launch_se_gemm_sp(const void* x, int M, int P, int cs_in, const void* w, int n_pad, const float* bias,
                       const void* gate, const void* res, void* y, int cs_out, hipStream_t s, double flops, double bytes) {
  M2S_CHECK(se_gemm_sp_supported(P, cs_in, cs_out) && M % P == 0, "se_gemm_sp: unsupported shape");
  M2S_CHECK(x && w && bias && gate && y && y != res && y != x, "se_gemm_sp: operand pointers");
  M2S_CHECK((double)M * cs_in * 4 < 4294967295.0 * 4, "se_gemm_sp: input too large");
  if (M <= 0) return;
  G128Args a = g128_args();
  a.x = static_cast<const uint8_t*>(x);
  a.w = static_cast<const uint8_t*>(w);
  a.bias = bias;
  a.gate = static_cast<const bf16_t*>(gate);
  a.res = static_cast<const bf16_t*>(res);
  a.y = static_cast<bf16_t*>(y);
  a.M = M;
  a.P = P;
  a.cs_in = cs_in;
  a.kp = cs_in;  // weight rows [hi kp | lo kp] with kp = cs_in (conv_gemm's split packing)
  a.cs_out = cs_out;
  static const int waves = [] {
    const char* e = std::getenv("M2S_SE_SP_WAVES");
    return e && std::atoi(e) == 4 ? 4 : 8;
  }();

  if (cs_out <= 128) {
    M2S_CHECK(n_pad >= 128, "se_gemm_sp: weight rows");
    if (waves == 8)  // 256 x 128, two waves per SIMD (each gates its rows' fragments for its 64 columns)
      launch_tile<KIND_SP_SE, 4, 2, 4>(a, s, flops, bytes);
    else
      launch_tile<KIND_SP_SE, 4, 1, 8>(a, s, flops, bytes);  // 256 x 128: 16x16 maps (one image per tile)
  } else if (waves == 8) {
    M2S_CHECK(n_pad >= 256, "se_gemm_sp: weight rows");
    launch_tile<KIND_SP_SE, 2, 4, 4>(a, s, flops, bytes);  // 128 x 256 (224 used), two waves per SIMD
  } else {
    M2S_CHECK(n_pad >= 224, "se_gemm_sp: weight rows");
    launch_tile<KIND_SP_SE, 2, 2, 7>(a, s, flops, bytes);  // 128 x 224: 8x8 maps (two images per tile)
  }
}

}  // namespace m2s
