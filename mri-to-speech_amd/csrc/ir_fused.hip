// Fused InvertedResidual front half for stride-1 blocks on small maps (bf16):
//   conv_pw (1x1 expand, MFMA) + bn1 + SiLU  ->  LDS tile  ->  conv_dw 3x3 + bn2 + SiLU  ->  HBM
//   + the SE squeeze (complete per-image channel means).
// (timm InvertedResidual conv_pw/bn1/conv_dw/bn2/se.mean; mri_acoustic_model.py:28-34.)
//
// One workgroup = G whole images (G*P <= 256 positions, G in {1,2,4}) x one 32-channel slice of the
// expanded width (127 VGPRs, 33 KB LDS: 4 workgroups per CU; a loop over several slices per
// workgroup halves the occupancy and measured slower).  The expanded activation never leaves the CU: the unfused sequence writes
// it to HBM from the GEMM and reads it back in the depthwise (2 x 416..1248 channels x P x 2 B per
// image), which made these blocks the largest HBM consumer of the encoder (profiles/ PMC).
// Per slice:
//   phase 1: D[c][m] = sum_k Wpw[c][k] x[m][k] on v_mfma_f32_16x16x32_bf16 (weights = A, positions
//            = B, fragments loaded straight from L1/L2 with a one-step register prefetch), bias +
//            SiLU, bf16 into the LDS tile.  The tile holds each image with a one-pixel zero halo,
//            rows of 32 channels padded by 16 B, so the depthwise needs no bounds checks.
//   phase 2: 4 channel groups x 64 pixel lanes (split evenly over the G images), 9 ds_read_b128 at
//            constant offsets per pixel, v_dot2_f32_bf16 against (w_c, 0) / (0, w_c+1) weight
//            dwords (no unpacking), SiLU, one v_cvt_pk_bf16_f32 per channel pair, 16-byte stores.
//   squeeze: per-lane channel sums -> fixed xor-shuffle tree within each wave -> per-wave partials
//            in LDS -> the image's waves added in order -> SE mean (deterministic).
// Split fp32 (SP = 1, m2s_common.hpp sp_t): phase 1 loads hi and lo fragments of the weights and the
// input and runs three MFMA terms per product; the LDS tile holds the fp32 expanded activation
// (36-float rows) and phase 2 is an fp32 depthwise with fp32 taps, writing hi/lo pairs.  The fp32
// tile is twice the bf16 one, so SP bounds the haloed rows per workgroup at 324 (one 16x16 image,
// two 8x8 images): 47 KB, three workgroups per CU.
#include <type_traits>

#include "conv_igemm.hpp"
#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int SL = 32;         // expanded channels per slice
constexpr int MROW = SL + 8;   // bf16 LDS row stride in bf16 (80 B)
constexpr int MROWF = SL + 4;  // fp32 (SP) LDS row stride in floats (144 B)
constexpr int NT = SL / 16;    // 16-channel MFMA subtiles
constexpr int CG = SL / 8;     // phase-2 channel groups (8 channels = one 16-byte vector)
constexpr int ROWS_MAX = 400;  // haloed pixel rows per workgroup (4 x 10x10, 1 x 18x18)
constexpr int ROWS_MAX_SP = 400;  // SP: fp32 rows (1 x 18x18, 4 x 10x10)
constexpr int POS_MAX = 256;   // positions per workgroup
// One slice per workgroup: a slice loop per workgroup (more reuse of the input) measured slower,
// occupancy 4 -> 2.
#ifndef IRPW_CG8
#define IRPW_CG8 1  // bf16 / fp8 depthwise on 8 groups of 4 channels (0: 4 groups of 8)
#endif
#ifndef IRPW_F16
#define IRPW_F16 1  // e4m3-output modes: f16 tile + v_pk_fma_f16 depthwise, packed-f32 SiLU (0: the bf16 dot2 form)
#endif

typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot2(uint32_t x, uint32_t w, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, x), __builtin_bit_cast(bf16x2_t, w), acc,
                                         false);
}
// the sigmoid of two values: v_pk_mul_f32 / v_pk_add_f32 around the two transcendentals of each (the file builds
// without SLP packing, so the packed forms are spelled out as vector ops)
__device__ __forceinline__ f32x2 sigmoid2(f32x2 z) {
  const f32x2 t = z * -1.4426950408889634f;
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
  return f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
// a (w_c, 0) / (0, w_c+1) bf16 tap dword pair -> the f16 pair (w_c, w_c+1)
__device__ __forceinline__ h16x2 taps_f16(uint32_t lo, uint32_t hi) {
  return __builtin_convertvector((f32x2{__uint_as_float(lo << 16), __uint_as_float(hi & 0xffff0000u)}), h16x2);
}

// S = depthwise stride.  OH x OW is the conv_pw (input) map; with S = 2 the depthwise writes the
// SOH x SOW map, TF-SAME with top / left pads pad_t / pad_l (the stride-2 blocks.5.0 at 16x16).
// SP = 1: x, wpw (rows [hi kp | lo kp]), y and se_mean are split fp32; wdw2 is then the fp32
// tap-major [9][cs_mid] depthwise weight.
template <int MT, int G, int S, int SPM>
__device__ __forceinline__ void ir_pwdw_body(const bf16_t* __restrict__ x, int cs_in, int kp,
                                                         const bf16_t* __restrict__ wpw, const float* __restrict__ bpw,
                                                         const uint32_t* __restrict__ wdw2,
                                                         const float* __restrict__ bdw, int N, int OH, int OW,
                                                         int cs_mid, bf16_t* __restrict__ y,
                                                         bf16_t* __restrict__ se_mean, int SOH, int SOW, int pad_t,
                                                         int pad_l, const float* __restrict__ wsc = nullptr) {
  constexpr bool SP = SPM == 1;  // split fp32
  constexpr bool F8 = SPM >= 2;  // e4m3 depthwise output (fp8 engines: the e4m3 SE GEMM's operand)
  // SPM = 3: the expand on e4m3 too: x = e4m3 rows of kp bytes (launch_se_*_f8 y8), wpw = e4m3 [rows][kp] with
  // per-channel scales wsc (pack_gemm_f8), one v_mfma_scale_f32_16x16x128_f8f6f4 per 128 k
  constexpr bool F8I = SPM == 3;
  // e4m3 output: the tile holds f16 (11-bit significand against the output's 4), the depthwise accumulates in f16
  // on v_pk_fma_f16 (two channels an instruction instead of one v_dot2 per channel); with 4 channels a lane.
  // One image a workgroup only: same-box A/B (gpurun_out/f16dw) fp8 16x16 363 -> 335 us, 8x8 (G = 4) 227 -> 231 us
  constexpr bool F16 = F8 && IRPW_F16 && IRPW_CG8 && G == 1;
  // the haloed tile: dynamic LDS sized for this launch's G images (ir_tile_bytes)
  extern __shared__ __attribute__((aligned(16))) char tile_raw[];
  bf16_t* tile = reinterpret_cast<bf16_t*>(tile_raw);
  float* tilef = reinterpret_cast<float*>(tile_raw);
  __shared__ uint16_t lut[POS_MAX];
  __shared__ float red[4][SL];
  // this slice's depthwise taps: bf16 in their dword halves, or (SP) fp32
  __shared__ uint4 wdw_lds[9][SL / 4];
  __shared__ float4 bdw_lds[SL / 4];
  constexpr int R = SP ? 2 : 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g16 = lane >> 4, r16 = lane & 15;
  const int P = OH * OW, WR = OW + 2, IR = (OH + 2) * WR;
  const int PO = S == 1 ? P : SOH * SOW;  // depthwise output pixels per image
  // XCD-aware: the workgroups of one image group (its slices) are consecutive in `wid` and share
  // blockIdx % 8, i.e. one XCD, so the image is fetched into one L2 instead of eight.
  const int nsl = (cs_mid + SL - 1) / SL;
  const int nwg = gridDim.x, xq = nwg / 8, xr = nwg % 8, xcd = blockIdx.x % 8;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + blockIdx.x / 8;
  const int grp = wid / nsl, sl = wid - grp * nsl;
  const int n0 = grp * G, gi = min(G, N - n0), MP = gi * P;

  // the slice's depthwise weights and biases, staged once: every pixel lane of a channel group
  // needs the same 9 x 8 taps, and loading them per lane from L1/L2 (80 KB per workgroup) cost
  // more than the whole depthwise
  if (tid < 9 * (SL / 4)) {
    const int t = tid / (SL / 4), k = tid - t * (SL / 4), c = sl * SL + 4 * k;
    if constexpr (SP) {  // 8 fp32 taps per uint4 pair: k covers channels 4k..4k+3
      const float* wf = reinterpret_cast<const float*>(wdw2);
      reinterpret_cast<float4*>(&wdw_lds[t][0])[k] =
          c < cs_mid ? *reinterpret_cast<const float4*>(wf + (size_t)t * cs_mid + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      wdw_lds[t][k] = c < cs_mid ? *reinterpret_cast<const uint4*>(wdw2 + (size_t)t * cs_mid + c) : make_uint4(0, 0, 0, 0);
    }
    if (t == 0) bdw_lds[k] = c < cs_mid ? *reinterpret_cast<const float4*>(bdw + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // ---- position -> haloed tile row; zero the tile (the halo stays zero) ----------------------
  if (tid < G * P) {
    const int g = tid / P, p = tid - g * P, oy = p / OW, ox = p - oy * OW;
    lut[tid] = (uint16_t)(g * IR + (oy + 1) * WR + ox + 1);
  }
  {
    uint4* t4 = reinterpret_cast<uint4*>(tile_raw);
    const int n16 = SP ? G * IR * (MROWF / 4) : G * IR * (MROW / 8);
    for (int i = tid; i < n16; i += 256) t4[i] = make_uint4(0, 0, 0, 0);
  }

  const bf16_t* xi = x + (size_t)n0 * P * cs_in * R;
  const int mw = wave * MT * 16;
  // phase 2: CGX channel groups of NCH channels x PLX pixel lanes.  bf16 tiles (SP = 0): 8 groups of 4 channels
  // (IRPW_CG8=0: 4 x 8), half the taps per lane in registers (36 dwords) and twice the pixel lanes: same-box A/B
  // (gpurun_out/r05ai) fp8 16x16 385 -> 361 us, bf16 16x16 478 -> 474 us, 8x8 within +-2 %; asking the compiler
  // for five workgroups per CU instead of four (96 VGPRs, spills) was no faster for fp8 and 6 % slower for bf16
  constexpr int CGX = (!SP && IRPW_CG8) ? 8 : CG, NCH = SL / CGX, PLX = 256 / CGX;
  const int cg = tid % CGX, pl = tid / CGX;
  const int lpi = PLX / G, g = pl / lpi, q = pl - g * lpi;  // phase-2 image and lane within it
  int off[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) off[t] = ((t / 3 - 1) * WR + (t % 3 - 1)) * (SP ? MROWF : MROW);

  {
    const int c0 = sl * SL;
    // ---- phase 1: expand GEMM, positions [mw, mw + MT*16) x channels [c0, c0 + SL) ------------
    f32x4 acc[NT][MT];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint4 fa[2][NT], fb[2][MT];
    uint4 fal[2][SP ? NT : 1], fbl[2][SP ? MT : 1];  // SP: lo halves
    auto load = [&](int buf, int k0) {
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const bf16_t* w = wpw + (size_t)(c0 + ni * 16 + r16) * kp * R + k0 + 8 * g16;
        fa[buf][ni] = *reinterpret_cast<const uint4*>(w);
        if constexpr (SP) fal[buf][ni] = *reinterpret_cast<const uint4*>(w + kp);
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int m = mw + mi * 16 + r16, k = k0 + 8 * g16;
        const bool ok = m < MP && k < cs_in;
        const bf16_t* xp = xi + (size_t)m * cs_in * R + k;
        fb[buf][mi] = ok ? *reinterpret_cast<const uint4*>(xp) : make_uint4(0, 0, 0, 0);
        if constexpr (SP) fbl[buf][mi] = ok ? *reinterpret_cast<const uint4*>(xp + cs_in) : make_uint4(0, 0, 0, 0);
      }
    };
    auto mma = [&](int buf) {
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          if constexpr (SP) {
            acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fal[buf][ni]),
                                                                  __builtin_bit_cast(bf16x8, fb[buf][mi]), acc[ni][mi],
                                                                  0, 0, 0);
            acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[buf][ni]),
                                                                  __builtin_bit_cast(bf16x8, fbl[buf][mi]), acc[ni][mi],
                                                                  0, 0, 0);
          }
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[buf][ni]),
                                                                __builtin_bit_cast(bf16x8, fb[buf][mi]), acc[ni][mi],
                                                                0, 0, 0);
        }
    };
    // the K loop fully unrolled for the block widths of the backbone (kp = cs_in = 128 / 224): loads
    // from clamped addresses (no exec-masked branch; positions past MP feed only discarded output
    // columns), and sched_barriers pin the one-step prefetch ahead of the MFMAs it must overlap.  The
    // generic loop below made every k-step wait for its own loads (conditional loads end in vmcnt(0)).
    auto load_u = [&](int buf, int k0) {
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const bf16_t* w = wpw + (size_t)(c0 + ni * 16 + r16) * kp * R + k0 + 8 * g16;
        fa[buf][ni] = *reinterpret_cast<const uint4*>(w);
        if constexpr (SP) fal[buf][ni] = *reinterpret_cast<const uint4*>(w + kp);
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const bf16_t* xp = xi + (size_t)min(mw + mi * 16 + r16, MP - 1) * cs_in * R + k0 + 8 * g16;
        fb[buf][mi] = *reinterpret_cast<const uint4*>(xp);
        if constexpr (SP) fbl[buf][mi] = *reinterpret_cast<const uint4*>(xp + cs_in);
      }
    };
    auto unrolled = [&](auto ksn_c) {
      constexpr int KSN = decltype(ksn_c)::value;
      load_u(0, 0);
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks) {
        if (ks + 1 < KSN) load_u((ks + 1) & 1, (ks + 1) * 32);
        __builtin_amdgcn_sched_barrier(0);
        mma(ks & 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if constexpr (F8I) {
      const uint8_t* x8 = reinterpret_cast<const uint8_t*>(x) + (size_t)n0 * P * kp;
      const uint8_t* w8 = reinterpret_cast<const uint8_t*>(wpw);
      for (int k0 = 0; k0 < kp; k0 += 128) {  // lane (r16, g16): 32 consecutive k bytes 32 g16 .. of its row
        i32x8 af[NT], bx[MT];
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const uint4* wp = reinterpret_cast<const uint4*>(w8 + (size_t)(c0 + ni * 16 + r16) * kp + k0 + 32 * g16);
          const uint4 u0 = wp[0], u1 = wp[1];
          af[ni] = i32x8{(int)u0.x, (int)u0.y, (int)u0.z, (int)u0.w, (int)u1.x, (int)u1.y, (int)u1.z, (int)u1.w};
        }
        // the row bytes past cs_in are not read: the buffer's rows are laid out per stage (128 / 256 bytes), so
        // a 256-byte row's pad can hold an earlier stage's bytes, NaN included (0 x NaN would leak it)
        const bool kin = k0 + 32 * g16 < cs_in;
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {  // positions past MP read a clamped row: their columns are discarded
          const uint4* xp = reinterpret_cast<const uint4*>(x8 + (size_t)min(mw + mi * 16 + r16, MP - 1) * kp + k0 + 32 * g16);
          const uint4 u0 = kin ? xp[0] : make_uint4(0u, 0u, 0u, 0u), u1 = kin ? xp[1] : make_uint4(0u, 0u, 0u, 0u);
          bx[mi] = i32x8{(int)u0.x, (int)u0.y, (int)u0.z, (int)u0.w, (int)u1.x, (int)u1.y, (int)u1.z, (int)u1.w};
        }
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
#pragma unroll
          for (int mi = 0; mi < MT; ++mi)
            acc[ni][mi] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[ni], bx[mi], acc[ni][mi], 0, 0, 0,
                                                                           0x7f7f7f7f, 0, 0x7f7f7f7f);
      }
    } else if (kp == 128 && cs_in == 128) {
      unrolled(std::integral_constant<int, 4>());
    } else if (kp == 224 && cs_in == 224) {
      unrolled(std::integral_constant<int, 7>());
    } else {
    load(0, 0);
    for (int k0 = 0;;) {
      if (k0 + 32 < kp) load(1, k0 + 32);
      mma(0);
      if ((k0 += 32) >= kp) break;
      if (k0 + 32 < kp) load(0, k0 + 32);
      mma(1);
      if ((k0 += 32) >= kp) break;
    }
    }
    __syncthreads();  // lut/zeroes visible
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int cl = ni * 16 + 4 * g16;  // slice-local channel of acc[ni][.][0]
      const float4 bb = *reinterpret_cast<const float4*>(bpw + c0 + cl);
      if constexpr (F16) {  // (scale,) bias, SiLU on packed f32, f16 pairs into the tile
        f32x2 sc01 = f32x2{1.f, 1.f}, sc23 = f32x2{1.f, 1.f};
        if constexpr (F8I) {
          const float4 sc = *reinterpret_cast<const float4*>(wsc + c0 + cl);
          sc01 = f32x2{sc.x, sc.y};
          sc23 = f32x2{sc.z, sc.w};
        }
        const f32x2 b01 = f32x2{bb.x, bb.y}, b23 = f32x2{bb.z, bb.w};
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          const int m = mw + mi * 16 + r16;
          if (m >= MP) continue;
          const f32x2 z01 = F8I ? __builtin_elementwise_fma(f32x2{acc[ni][mi][0], acc[ni][mi][1]}, sc01, b01)
                                : f32x2{acc[ni][mi][0], acc[ni][mi][1]} + b01;
          const f32x2 z23 = F8I ? __builtin_elementwise_fma(f32x2{acc[ni][mi][2], acc[ni][mi][3]}, sc23, b23)
                                : f32x2{acc[ni][mi][2], acc[ni][mi][3]} + b23;
          const h16x2 y01 = __builtin_convertvector(z01 * sigmoid2(z01), h16x2);
          const h16x2 y23 = __builtin_convertvector(z23 * sigmoid2(z23), h16x2);
          *reinterpret_cast<uint2*>(tile + lut[m] * MROW + cl) =
              make_uint2(__builtin_bit_cast(uint32_t, y01), __builtin_bit_cast(uint32_t, y23));
        }
        continue;
      }
      if constexpr (F8I) {  // the e4m3 weights' per-channel scales
        const float4 sc = *reinterpret_cast<const float4*>(wsc + c0 + cl);
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          acc[ni][mi][0] *= sc.x;
          acc[ni][mi][1] *= sc.y;
          acc[ni][mi][2] *= sc.z;
          acc[ni][mi][3] *= sc.w;
        }
      }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int m = mw + mi * 16 + r16;
        if (m >= MP) continue;
        if constexpr (SP) {
          *reinterpret_cast<float4*>(tilef + lut[m] * MROWF + cl) =
              make_float4(silu(acc[ni][mi][0] + bb.x), silu(acc[ni][mi][1] + bb.y), silu(acc[ni][mi][2] + bb.z),
                          silu(acc[ni][mi][3] + bb.w));
          continue;
        }
        uint2 u;
        u.x = pack_bf16x2(silu(acc[ni][mi][0] + bb.x), silu(acc[ni][mi][1] + bb.y));
        u.y = pack_bf16x2(silu(acc[ni][mi][2] + bb.z), silu(acc[ni][mi][3] + bb.w));
        *reinterpret_cast<uint2*>(tile + lut[m] * MROW + cl) = u;
      }
    }
    __syncthreads();

    // ---- phase 2: depthwise 3x3 (stride 1, pad 1) from the haloed tile ------------------------
    const int c = c0 + cg * NCH;
    float s[NCH];
#pragma unroll
    for (int j = 0; j < NCH; ++j) s[j] = 0.f;
    if (SP && g < gi && c < cs_mid) {
      float w[9][8], b[8];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4 lo = reinterpret_cast<const float4*>(&wdw_lds[t][0])[2 * cg];
        const float4 hi = reinterpret_cast<const float4*>(&wdw_lds[t][0])[2 * cg + 1];
        w[t][0] = lo.x; w[t][1] = lo.y; w[t][2] = lo.z; w[t][3] = lo.w;
        w[t][4] = hi.x; w[t][5] = hi.y; w[t][6] = hi.z; w[t][7] = hi.w;
      }
      {
        const float4 lo = bdw_lds[2 * cg], hi = bdw_lds[2 * cg + 1];
        b[0] = lo.x; b[1] = lo.y; b[2] = lo.z; b[3] = lo.w;
        b[4] = hi.x; b[5] = hi.y; b[6] = hi.z; b[7] = hi.w;
      }
      sp_t* ys = reinterpret_cast<sp_t*>(y);
      for (int p = q; p < PO; p += lpi) {
        int trow;
        if constexpr (S == 1) {
          trow = lut[g * P + p];
        } else {
          const int oy = p / SOW, ox = p - (p / SOW) * SOW;
          trow = g * IR + (S * oy - pad_t + 2) * WR + S * ox - pad_l + 2;
        }
        const float* base = tilef + trow * MROWF + cg * 8;
        float a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = b[j];
#pragma unroll
        for (int ty = 0; ty < 3; ++ty) {  // one tap row at a time: 24 registers of taps in flight
#pragma unroll
          for (int tx = 0; tx < 3; ++tx) {
            const int t = 3 * ty + tx;
            const float4 u0 = *reinterpret_cast<const float4*>(base + off[t]);
            const float4 u1 = *reinterpret_cast<const float4*>(base + off[t] + 4);
            a[0] += w[t][0] * u0.x; a[1] += w[t][1] * u0.y; a[2] += w[t][2] * u0.z; a[3] += w[t][3] * u0.w;
            a[4] += w[t][4] * u1.x; a[5] += w[t][5] * u1.y; a[6] += w[t][6] * u1.z; a[7] += w[t][7] * u1.w;
          }
          asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] = silu(a[j]);
          s[j] += a[j];
        }
        il_st8(ys, (long)(n0 + g) * PO + p, cs_mid, c, a);  // the SE GEMM's interleaved operand
      }
    } else if (F16 && g < gi && c < cs_mid) {
      static_assert(!F16 || NCH == 4, "f16 depthwise: 4 channels a lane");
      h16x2 w[9][2], b2[2];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const uint4 v = wdw_lds[t][cg];
        w[t][0] = taps_f16(v.x, v.y);
        w[t][1] = taps_f16(v.z, v.w);
      }
      {
        const float4 v = bdw_lds[cg];
        b2[0] = __builtin_convertvector((f32x2{v.x, v.y}), h16x2);
        b2[1] = __builtin_convertvector((f32x2{v.z, v.w}), h16x2);
      }
      f32x2 s01 = f32x2{0.f, 0.f}, s23 = f32x2{0.f, 0.f};
      for (int p = q; p < PO; p += lpi) {
        int trow;  // haloed tile row of the tap-(1, 1) input pixel
        if constexpr (S == 1) {
          trow = lut[g * P + p];
        } else {
          const int oy = p / SOW, ox = p - (p / SOW) * SOW;
          trow = g * IR + (S * oy - pad_t + 2) * WR + S * ox - pad_l + 2;
        }
        const bf16_t* base = tile + trow * MROW + cg * NCH;
        uint2 in[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) in[t] = *reinterpret_cast<const uint2*>(base + off[t]);
        h16x2 a0 = b2[0], a1 = b2[1];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          a0 = __builtin_elementwise_fma(__builtin_bit_cast(h16x2, in[t].x), w[t][0], a0);
          a1 = __builtin_elementwise_fma(__builtin_bit_cast(h16x2, in[t].y), w[t][1], a1);
        }
        const f32x2 x01 = __builtin_convertvector(a0, f32x2), x23 = __builtin_convertvector(a1, f32x2);
        const f32x2 g01 = sigmoid2(x01), g23 = sigmoid2(x23);
        s01 += x01 * g01;  // the squeeze sums the unsaturated values
        s23 += x23 * g23;
        // min(x, 448) * sigmoid(x): saturated for e4m3 (SiLU >= -0.28), a NaN x stays NaN through the sigmoid
        const f32x2 o01 = f32x2{fminf(x01.x, 448.f), fminf(x01.y, 448.f)} * g01;
        const f32x2 o23 = f32x2{fminf(x23.x, 448.f), fminf(x23.y, 448.f)} * g23;
        const int r = __builtin_amdgcn_cvt_pk_fp8_f32(o01.x, o01.y, 0, false);
        uint8_t* y8 = reinterpret_cast<uint8_t*>(y) + ((size_t)(n0 + g) * PO + p) * cs_mid + c;
        reinterpret_cast<uint32_t*>(y8)[0] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(o23.x, o23.y, r, true);
      }
      s[0] = s01.x; s[1] = s01.y; s[2 % NCH] = s23.x; s[3 % NCH] = s23.y;
    } else if (!SP && g < gi && c < cs_mid) {
      constexpr int NW2 = NCH / 2;  // tap dwords per lane and tap: (w_c, 0) / (0, w_c+1) pairs
      uint32_t w[9][NCH];
      float b[NCH];
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int k = 0; k < NCH / 4; ++k) {
          const uint4 v = wdw_lds[t][(NCH / 4) * cg + k];
          w[t][4 * k] = v.x; w[t][4 * k + 1] = v.y; w[t][4 * k + 2] = v.z; w[t][4 * k + 3] = v.w;
        }
#pragma unroll
      for (int k = 0; k < NCH / 4; ++k) {
        const float4 v = bdw_lds[(NCH / 4) * cg + k];
        b[4 * k] = v.x; b[4 * k + 1] = v.y; b[4 * k + 2] = v.z; b[4 * k + 3] = v.w;
      }
      bf16_t* yi = y + (size_t)(n0 + g) * PO * cs_mid + c;
      for (int p = q; p < PO; p += lpi) {
        int trow;  // haloed tile row of the tap-(1, 1) input pixel
        if constexpr (S == 1) {
          trow = lut[g * P + p];
        } else {
          const int oy = p / SOW, ox = p - (p / SOW) * SOW;
          trow = g * IR + (S * oy - pad_t + 2) * WR + S * ox - pad_l + 2;
        }
        const bf16_t* base = tile + trow * MROW + cg * NCH;
        uint32_t in[9][NW2];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          if constexpr (NW2 == 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(base + off[t]);
            in[t][0] = v.x; in[t][NW2 > 1 ? 1 : 0] = v.y; in[t][NW2 > 2 ? 2 : 0] = v.z; in[t][NW2 > 3 ? 3 : 0] = v.w;
          } else {
            const uint2 v = *reinterpret_cast<const uint2*>(base + off[t]);
            in[t][0] = v.x; in[t][NW2 > 1 ? 1 : 0] = v.y;
          }
        }
        float a[NCH];
#pragma unroll
        for (int j = 0; j < NCH; ++j) a[j] = b[j];
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int j = 0; j < NW2; ++j) {
            a[2 * j] = dot2(in[t][j], w[t][2 * j], a[2 * j]);
            a[2 * j + 1] = dot2(in[t][j], w[t][2 * j + 1], a[2 * j + 1]);
          }
        uint8_t* y8 = reinterpret_cast<uint8_t*>(y) + ((size_t)(n0 + g) * PO + p) * cs_mid + c;
        if constexpr (F8) {  // saturated as silu_e4m3: min(x, 448) * sigmoid(x), NaN kept; the squeeze sums x * sigmoid(x)
          float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < NCH; ++j) {
            const float gs = sigmoidf_(a[j]);
            s[j] += a[j] * gs;
            o[j] = fminf(a[j], 448.f) * gs;
          }
          const uint2 q = e4m3x8_nosat(o);  // 8 channels -> 8 bytes at byte (n, p, c) of the e4m3 map; 4 -> the first 4
          if constexpr (NCH == 8)
            reinterpret_cast<uint2*>(y8)[0] = q;
          else
            reinterpret_cast<uint32_t*>(y8)[0] = q.x;
          continue;
        }
        float v[NCH];
        uint32_t ow[NW2];
#pragma unroll
        for (int j = 0; j < NW2; ++j) {
          v[2 * j] = silu(a[2 * j]);
          v[2 * j + 1] = silu(a[2 * j + 1]);
          s[2 * j] += v[2 * j];  // the squeeze sums the unrounded values
          s[2 * j + 1] += v[2 * j + 1];
          ow[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
        }
        if constexpr (NCH == 8) {
          *reinterpret_cast<uint4*>(yi + (size_t)p * cs_mid) = make_uint4(ow[0], ow[NW2 > 1 ? 1 : 0], ow[NW2 > 2 ? 2 : 0], ow[NW2 > 3 ? 3 : 0]);
        } else {
          *reinterpret_cast<uint2*>(yi + (size_t)p * cs_mid) = make_uint2(ow[0], ow[NW2 > 1 ? 1 : 0]);
        }
      }
    }
    // ---- squeeze: the wave's pixel lanes (lane / CGX) share cg = lane % CGX; one image per wave
    // when G = 4, else the image spans 4/G waves.
#pragma unroll
    for (int msk = CGX; msk < 64; msk <<= 1)
#pragma unroll
      for (int j = 0; j < NCH; ++j) s[j] += __shfl_xor(s[j], msk);
    if (lane < CGX)
#pragma unroll
      for (int j = 0; j < NCH; ++j) red[wave][lane * NCH + j] = s[j];
    __syncthreads();
    if (tid < G * SL) {
      const int gg = tid / SL, cl = tid - gg * SL, wpi = 4 / G;
      if (gg < gi && c0 + cl < cs_mid) {
        float t = 0.f;
        for (int wv = gg * wpi; wv < (gg + 1) * wpi; ++wv) t += red[wv][cl];
        if constexpr (SP)
          act_st<sp_t>(reinterpret_cast<sp_t*>(se_mean), n0 + gg, cs_mid, c0 + cl, t / (float)PO);
        else
          se_mean[(size_t)(n0 + gg) * cs_mid + c0 + cl] = f2bf(t / (float)PO);
      }
    }
  }
}

template <int MT, int G, int SP>
__global__ void __launch_bounds__(256, SP == 1 ? (MT >= 4 ? 3 : 4) : 4)
    ir_pwdw_kernel(const bf16_t* __restrict__ x, int cs_in, int kp, const bf16_t* __restrict__ wpw,
                   const float* __restrict__ bpw, const uint32_t* __restrict__ wdw2, const float* __restrict__ bdw, int N,
                   int OH, int OW, int cs_mid, bf16_t* __restrict__ y, bf16_t* __restrict__ se_mean,
                   const float* __restrict__ wsc) {
  ir_pwdw_body<MT, G, 1, SP>(x, cs_in, kp, wpw, bpw, wdw2, bdw, N, OH, OW, cs_mid, y, se_mean, OH, OW, 1, 1, wsc);
}

template <int SP>
__global__ void __launch_bounds__(256, SP == 1 ? 3 : 4)
    ir_pwdw_s2_kernel(const bf16_t* __restrict__ x, int cs_in, int kp, const bf16_t* __restrict__ wpw,
                      const float* __restrict__ bpw, const uint32_t* __restrict__ wdw2, const float* __restrict__ bdw,
                      int N, int IH, int IW, int cs_mid, bf16_t* __restrict__ y, bf16_t* __restrict__ se_mean, int OH,
                      int OW, int pad_t, int pad_l, const float* __restrict__ wsc) {
  ir_pwdw_body<4, 1, 2, SP>(x, cs_in, kp, wpw, bpw, wdw2, bdw, N, IH, IW, cs_mid, y, se_mean, OH, OW, pad_t, pad_l, wsc);
}

// images per workgroup: up to 4 small images (measured on the 8x8 maps of blocks.5 in split fp32:
// 1383 / 970 / 745 us per launch at G = 1 / 2 / 4; the per-workgroup latency chain loads -> MFMA ->
// barrier -> depthwise -> barrier -> squeeze amortises over more positions)
int ir_group(int OH, int OW, bool sp) {
  const int P = OH * OW, rows = (OH + 2) * (OW + 2);
  for (int G = 4; G >= 1; G /= 2)
    if (G * P <= POS_MAX && G * rows <= (sp ? ROWS_MAX_SP : ROWS_MAX)) return G;
  return 0;
}
size_t ir_tile_bytes(int OH, int OW, int G, bool sp) {
  return (size_t)G * (OH + 2) * (OW + 2) * (sp ? MROWF * 4 : MROW * 2);
}

}  // namespace

bool ir_fused_supported(int OH, int OW, int cs_in, int cs_mid, bool split) {
  (void)cs_in;
  return ir_group(OH, OW, split) > 0 && cs_mid % 8 == 0;
}

void launch_ir_pwdw(const void* x, int N, int cs_in, int kp, const void* wpw, const float* bpw, const void* wdw,
                    const float* bdw, int OH, int OW, int cs_mid, void* y, void* se_mean, bool split, double flops,
                    double bytes, hipStream_t s, bool f8_out, const void* x8, const void* w8, const float* wsc, int kp8) {
  M2S_CHECK(ir_fused_supported(OH, OW, cs_in, cs_mid, split), "ir_pwdw: unsupported shape");
  M2S_CHECK(!(split && f8_out), "ir_pwdw: e4m3 output is a bf16-path variant");
  const bool f8_in = x8 != nullptr;
  M2S_CHECK(!f8_in || (f8_out && w8 && wsc && kp8 % 128 == 0 && kp8 >= cs_in), "ir_pwdw: e4m3 expand operands");
  const int mode = split ? 1 : f8_in ? 3 : f8_out ? 2 : 0;
  M2S_CHECK(kp % 32 == 0 && kp >= cs_in, "ir_pwdw: kp");
  if (f8_in) {  // the e4m3 operands replace the bf16 ones
    x = x8;
    wpw = w8;
    kp = kp8;
  }
  const int G = ir_group(OH, OW, split), pos = G * OH * OW;
  const dim3 grid(ceil_div(cs_mid, SL) * ceil_div(N, G));
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  const bf16_t* wb = static_cast<const bf16_t*>(wpw);
  const uint32_t* wd = static_cast<const uint32_t*>(wdw);
  bf16_t* yb = static_cast<bf16_t*>(y);
  bf16_t* mb = static_cast<bf16_t*>(se_mean);
  // MT = 16-position subtiles per wave (pos <= 64 * MT); G = images per workgroup.  Each pair is
  // its own symbol, so rocprofv3 and the event profiler see the same kernel.
#define M2S_IRF(MT_, G_, SP_)                                                                            \
  if (pos <= 64 * MT_ && G == G_ && mode == SP_) {                                                 \
    ProfScope ps("ir_pwdw_kernel<" #MT_ ", " #G_ ", " #SP_ ">", flops, bytes, s);                       \
    hipLaunchKernelGGL((ir_pwdw_kernel<MT_, G_, SP_>), grid, dim3(256), ir_tile_bytes(OH, OW, G, split), s, xb, cs_in, \
                       kp, wb, bpw, wd, bdw, N, OH, OW, cs_mid, yb, mb, wsc);                            \
    M2S_HIP(hipGetLastError());                                                                          \
    return;                                                                                              \
  }
  M2S_IRF(1, 1, 0) M2S_IRF(1, 2, 0) M2S_IRF(1, 4, 0)
  M2S_IRF(2, 1, 0) M2S_IRF(2, 2, 0) M2S_IRF(2, 4, 0)
  M2S_IRF(4, 1, 0) M2S_IRF(4, 2, 0) M2S_IRF(4, 4, 0)
  M2S_IRF(1, 1, 1) M2S_IRF(1, 2, 1) M2S_IRF(1, 4, 1)
  M2S_IRF(2, 1, 1) M2S_IRF(2, 2, 1) M2S_IRF(2, 4, 1)
  M2S_IRF(4, 1, 1) M2S_IRF(4, 2, 1) M2S_IRF(4, 4, 1)
  M2S_IRF(4, 1, 2) M2S_IRF(4, 2, 2) M2S_IRF(4, 4, 2)
  M2S_IRF(4, 1, 3) M2S_IRF(4, 2, 3) M2S_IRF(4, 4, 3)
#undef M2S_IRF
  M2S_CHECK(false, "ir_pwdw: no variant for this shape");
}

__global__ void rows_e4m3_kernel(const uint4* __restrict__ x, long rows, int cs8, uint2* __restrict__ y8, int ld8_8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 8-byte group of one row
  if (i >= rows * ld8_8) return;
  const long r = i / ld8_8;
  const int c = (int)(i - r * ld8_8);
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cs8) {
    const uint4 u = x[r * cs8 + c];
    unpack_bf16x4(make_uint2(u.x, u.y), v);
    unpack_bf16x4(make_uint2(u.z, u.w), v + 4);
  }
  y8[i] = e4m3x8(v);
}

void launch_rows_e4m3(const void* x, long rows, int cs, void* y8, int ld8, hipStream_t s) {
  M2S_CHECK(cs % 8 == 0 && ld8 % 8 == 0 && ld8 >= cs && rows >= 0, "rows_e4m3: shape");
  const long n = rows * (ld8 / 8);
  if (n == 0) return;
  ProfScope ps("rows_e4m3_kernel", 0.0, (double)rows * (2.0 * cs + ld8), s);
  hipLaunchKernelGGL(rows_e4m3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, static_cast<const uint4*>(x), rows,
                     cs / 8, static_cast<uint2*>(y8), ld8 / 8);
  M2S_HIP(hipGetLastError());
}

bool ir_fused_s2_supported(int IH, int IW, int cs_in, int cs_mid, bool split) {
  return IH * IW <= 256 && IH * IW > 192 && (IH + 2) * (IW + 2) <= (split ? ROWS_MAX_SP : ROWS_MAX) &&
         cs_mid % 8 == 0 && cs_in > 0;
}

void launch_ir_pwdw_s2(const void* x, int N, int cs_in, int kp, const void* wpw, const float* bpw, const void* wdw,
                       const float* bdw, int IH, int IW, int OH, int OW, int pad_t, int pad_l, int cs_mid, void* y,
                       void* se_mean, bool split, double flops, double bytes, hipStream_t s, bool f8_out, const void* x8,
                       const void* w8, const float* wsc, int kp8) {
  M2S_CHECK(ir_fused_s2_supported(IH, IW, cs_in, cs_mid, split) && kp % 32 == 0 && kp >= cs_in,
            "ir_pwdw_s2: unsupported shape");
  M2S_CHECK(OH == (IH + 1) / 2 && OW == (IW + 1) / 2 && OH * OW <= 64 && pad_t >= 0 && pad_t <= 1 && pad_l >= 0 &&
                pad_l <= 1,
            "ir_pwdw_s2: geometry");
  M2S_CHECK(!(split && f8_out), "ir_pwdw_s2: e4m3 output is a bf16-path variant");
  const bool f8_in = x8 != nullptr;
  M2S_CHECK(!f8_in || (f8_out && w8 && wsc && kp8 % 128 == 0 && kp8 >= cs_in), "ir_pwdw_s2: e4m3 expand operands");
  if (f8_in) {  // the e4m3 operands replace the bf16 ones
    x = x8;
    wpw = w8;
    kp = kp8;
  }
  const int mode = split ? 1 : f8_in ? 3 : f8_out ? 2 : 0;
  const dim3 grid(ceil_div(cs_mid, SL) * N);
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  const bf16_t* wb = static_cast<const bf16_t*>(wpw);
  const uint32_t* wd = static_cast<const uint32_t*>(wdw);
#define M2S_IRS2(SP_)                                                                                            \
  if (mode == SP_) {                                                                                             \
    ProfScope ps("ir_pwdw_s2_kernel<" #SP_ ">", flops, bytes, s);                                               \
    hipLaunchKernelGGL(ir_pwdw_s2_kernel<SP_>, grid, dim3(256), ir_tile_bytes(IH, IW, 1, split), s, xb, cs_in, kp, wb, \
                       bpw, wd, bdw, N, IH, IW, cs_mid, static_cast<bf16_t*>(y), static_cast<bf16_t*>(se_mean), OH, OW,  \
                       pad_t, pad_l, wsc);                                                                       \
    M2S_HIP(hipGetLastError());                                                                                  \
    return;                                                                                                      \
  }
  M2S_IRS2(0) M2S_IRS2(1) M2S_IRS2(2) M2S_IRS2(3)
#undef M2S_IRS2
}

}  // namespace m2s
