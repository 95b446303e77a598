// Stride-2 InvertedResidual front half on row bands, for blocks.3.0 (56 -> 224, 32x32 -> 16x16):
//   conv_pw (1x1 expand, MFMA) + bn1 + SiLU -> fp32 LDS band -> conv_dw 3x3/s2 (TF-SAME) + bn2 + SiLU -> the
//   SE GEMM's operand, + the SE squeeze's per-band partial sums.
// SP = 1: split fp32 (three-term MFMA on hi/lo input and weights, output the interleaved [hi 32 | lo 32]
// operand); SP = 0: bf16 input / weights / output (the bf16 engine), one MFMA term; SP = 2: the same with the
// depthwise output stored as OCP e4m3 bytes (fp8 engines: the operand of the e4m3 SE GEMM, gemm128 KIND_F8_SE).
// (timm InvertedResidual conv_pw/bn1/conv_dw/bn2/se; mri_acoustic_model.py:28-34.)
//
// Unfused, conv_pw wrote the 224-channel expanded map at 32x32 as hi/lo pairs (1.76 GB per 1920 frames)
// and the stride-2 depthwise read it back; ir_pwdw_s2 keeps a whole image per workgroup, which fits
// 16x16 maps only.  Here a workgroup owns (image, band of SB_BO output rows, 32-channel slice): it expands
// the band's 2 SB_BO + 1 input rows (the one shared row between bands is recomputed: 9/8) into an fp32
// tile with zero halo columns (positions outside the image are stored as zeros: the depthwise's
// padding, not SiLU(bias)), then 64 lanes x 4 channel groups run the depthwise.  The squeeze's partial
// sums go to psum[n][band][c] in the layout of dwconv_kernel's pixel blocks, so se_mean_kernel finishes
// the mean.  Grid = N x bands x slices, ordered so that one image's workgroups share an XCD (its input
// is read by every slice).
#include <algorithm>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

constexpr int SB_SL = 32;                // expanded channels per slice
constexpr int SB_BO = 4;                 // output rows per band
constexpr int SB_ROWS = 2 * SB_BO + 1;   // input rows per band
constexpr int SB_MROW = SB_SL + 8;       // fp32 tile row stride (floats): 160 B = 10 16-byte units
// 16-byte unit u (4 channels) of tile position q is stored at unit u ^ sb_swz(q): with the 10-unit stride, the
// depthwise's ds_read_b128 lane groups (4 channel groups x 4 pixels two positions apart) hit 16 distinct bank
// quads and the expand epilogue's ds_write_b128 groups (8 consecutive positions) 8 distinct ones, at every
// offset (exhaustive search, tools/swizzle_search.py); the plain 9-unit stride had 3-way read conflicts
// (SQ_LDS_BANK_CONFLICT 1.7 per LDS instruction, profiles/r04fin9_sq_mfma.txt)
__device__ __forceinline__ int sb_swz(int q) { return ((q >> 1) ^ ((q >> 2) * 6)) & 7; }
constexpr int SB_IWMAX = 32;             // input width bound (tile 9 x 34 rows: 44 KB)
constexpr int SB_MT = 5;                 // 16-position tiles per wave at most: ceil(9 x 32 / 16 / 4)

size_t sb_tile_bytes(int IW) { return (size_t)SB_ROWS * (IW + 2) * SB_MROW * sizeof(float); }

template <int KSN, int SPM>  // expand k-steps (kp / 32), 0 bf16 / 1 split fp32 / 2 bf16 with e4m3 output
__global__ void __launch_bounds__(256, 3)
    ir_s2band_kernel(const bf16_t* __restrict__ x, int IH, int IW, const bf16_t* __restrict__ wpw,
                     const float* __restrict__ bpw, const float* __restrict__ wdw, const float* __restrict__ bdw,
                     int OH, int OW, int pad_t, int pad_l, int cs_mid, bf16_t* __restrict__ y,
                     float* __restrict__ psum) {
  constexpr bool SP = SPM == 1, F8 = SPM == 2;
  constexpr int CS = KSN * 32;  // input channel stride = expand K
  constexpr int R = SP ? 2 : 1;  // bf16 planes per row (hi, lo)
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [SB_ROWS][IW + 2][SB_MROW]
  __shared__ __attribute__((aligned(16))) float wd[10][SB_SL];  // 9 taps + bias of the slice
  __shared__ float red[4][SB_SL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int TW = IW + 2;
  const int nsl = cs_mid / SB_SL, nb = OH / SB_BO;
  // XCD-aware: the bands and slices of one image are consecutive in wid and share blockIdx % 8
  const int nwg = gridDim.x, xq = nwg / 8, xr = nwg % 8, xcd = blockIdx.x % 8;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + blockIdx.x / 8;
  const int sl = wid % nsl, band = (wid / nsl) % nb, n = wid / (nsl * nb);
  const int c0 = sl * SB_SL, oy0 = band * SB_BO, iy0 = 2 * oy0 - pad_t;

  for (int i = tid; i < 10 * SB_SL; i += 256) {
    const int t = i / SB_SL, c = c0 + i % SB_SL;
    wd[t][i % SB_SL] = t < 9 ? wdw[(size_t)t * cs_mid + c] : bdw[c];
  }
  for (int i = tid; i < SB_ROWS * 2 * (SB_MROW / 4); i += 256) {  // the two halo columns of every row
    const int r = i / (2 * (SB_MROW / 4)), q = i % (2 * (SB_MROW / 4)), side = q / (SB_MROW / 4);
    reinterpret_cast<float4*>(tile + ((size_t)r * TW + (side ? TW - 1 : 0)) * SB_MROW)[q % (SB_MROW / 4)] =
        make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // ---- phase 1: expand the band's SB_ROWS x IW input positions (16-position tiles dealt over the waves)
  bf16x8 ah[2][KSN], al[2][KSN];
  float4 bb[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const bf16_t* w = wpw + (size_t)(c0 + nt * 16 + r16) * CS * R + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      ah[nt][ks] = *reinterpret_cast<const bf16x8*>(w + ks * 32);
      al[nt][ks] = SP ? *reinterpret_cast<const bf16x8*>(w + CS + ks * 32) : bf16x8{};
    }
    bb[nt] = *reinterpret_cast<const float4*>(bpw + c0 + nt * 16 + 4 * g);
  }
  const int MP = SB_ROWS * IW, nmt = (MP + 15) / 16;
  const bf16_t* xn = x + (size_t)n * IH * IW * CS * R;
  // every tile's operand loads issued up front (at most SB_MT tiles a wave), then the MFMAs and stores:
  // one L2 round trip per wave instead of one per tile
  bf16x8 bh[SB_MT][KSN], bl[SB_MT][KSN];
#pragma unroll
  for (int i = 0; i < SB_MT; ++i) {
    const int m = (wave + 4 * i) * 16 + r16, r = m / IW, ix = m - r * IW, iy = iy0 + r;
    const bool inside = m < MP && iy >= 0 && iy < IH;
    const bf16_t* xp = xn + ((size_t)(inside ? iy : 0) * IW + (inside ? ix : 0)) * CS * R + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      bh[i][ks] = *reinterpret_cast<const bf16x8*>(xp + ks * 32);
      bl[i][ks] = SP ? *reinterpret_cast<const bf16x8*>(xp + CS + ks * 32) : bf16x8{};
    }
  }
#pragma unroll
  for (int i = 0; i < SB_MT; ++i) {
    const int mt = wave + 4 * i;
    if (mt >= nmt) break;
    const int m = mt * 16 + r16, r = m / IW, ix = m - r * IW, iy = iy0 + r;
    const bool inside = m < MP && iy >= 0 && iy < IH;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        if constexpr (SP) {
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[nt][ks], bh[i][ks], acc[nt], 0, 0, 0);
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[nt][ks], bl[i][ks], acc[nt], 0, 0, 0);
        }
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[nt][ks], bh[i][ks], acc[nt], 0, 0, 0);
      }
    if (m < MP) {  // lane = channels 4 g .. 4 g + 3 of n-tile nt at position m (unit g + 4 nt, swizzled)
      const int q = r * TW + ix + 1, sq = sb_swz(q);
      float* tp = tile + (size_t)q * SB_MROW;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        *reinterpret_cast<float4*>(tp + ((g + 4 * nt) ^ sq) * 4) =
            inside ? make_float4(silu(acc[nt][0] + bb[nt].x), silu(acc[nt][1] + bb[nt].y), silu(acc[nt][2] + bb[nt].z),
                                 silu(acc[nt][3] + bb[nt].w))
                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();

  // ---- phase 2: SB_BO x OW output pixels x 32 channels; thread = (8-channel group cg, pixel lane pl)
  const int cg = tid & 3, pl = tid >> 2;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    float w[9][8], b[8];
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      const float4 lo = *reinterpret_cast<const float4*>(&wd[t][cg * 8]);
      const float4 hi = *reinterpret_cast<const float4*>(&wd[t][cg * 8 + 4]);
      float* d = t < 9 ? w[t] : b;
      d[0] = lo.x; d[1] = lo.y; d[2] = lo.z; d[3] = lo.w;
      d[4] = hi.x; d[5] = hi.y; d[6] = hi.z; d[7] = hi.w;
    }
    sp_t* ys = reinterpret_cast<sp_t*>(y);
    for (int p = pl; p < SB_BO * OW; p += 64) {
      const int oyl = p / OW, ox = p - oyl * OW;
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = b[j];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int q = (2 * oyl + t / 3) * TW + 2 * ox - pad_l + t % 3 + 1, sq = sb_swz(q);
        const float* tp = tile + (size_t)q * SB_MROW;
        const float4 u0 = *reinterpret_cast<const float4*>(tp + ((2 * cg) ^ sq) * 4);
        const float4 u1 = *reinterpret_cast<const float4*>(tp + ((2 * cg + 1) ^ sq) * 4);
        a[0] += w[t][0] * u0.x; a[1] += w[t][1] * u0.y; a[2] += w[t][2] * u0.z; a[3] += w[t][3] * u0.w;
        a[4] += w[t][4] * u1.x; a[5] += w[t][5] * u1.y; a[6] += w[t][6] * u1.z; a[7] += w[t][7] * u1.w;
      }
      const long pix = ((long)n * OH + oy0 + oyl) * OW + ox;
      if constexpr (F8) {  // 8 channels -> 8 e4m3 bytes at byte (pix, c) of the (N, OH*OW, cs_mid) map
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // saturated as silu_e4m3: min(x, 448) * sigmoid(x), NaN kept
          const float g = sigmoidf_(a[j]);
          s[j] += a[j] * g;  // the squeeze sums the unsaturated values
          o[j] = fminf(a[j], 448.f) * g;
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(y) + pix * cs_mid + c0 + cg * 8) = e4m3x8_nosat(o);
        continue;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = silu(a[j]);
        s[j] += a[j];
      }
      if constexpr (SP) {
        il_st8(ys, pix, cs_mid, c0 + cg * 8, a);
      } else {
        *reinterpret_cast<uint4*>(y + pix * cs_mid + c0 + cg * 8) =
            make_uint4(pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(a[4], a[5]), pack_bf16x2(a[6], a[7]));
      }
    }
  }
  // ---- squeeze partials: the wave's 16 pixel lanes (lane bits 2..5), then the 4 waves in order
#pragma unroll
  for (int msk = 4; msk < 64; msk <<= 1)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += __shfl_xor(s[j], msk);
  if (lane < 4)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][lane * 8 + j] = s[j];
  __syncthreads();
  if (tid < SB_SL) psum[((size_t)n * nb + band) * cs_mid + c0 + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

}  // namespace

int ir_s2band_bands(int OH) { return OH / SB_BO; }

bool ir_s2band_supported(int IH, int IW, int OH, int OW, int cs_in, int kp, int cs_mid) {
  return IW <= SB_IWMAX && IW >= 2 * OW - 1 && IH >= 2 * OH - 1 && OW <= 16 && OH % SB_BO == 0 && OH > 0 &&
         cs_in == kp && (kp == 32 || kp == 64) && cs_mid % SB_SL == 0 && cs_mid > 0;
}

void launch_ir_s2band(const void* x, int N, int IH, int IW, int cs_in, int kp, const void* wpw, const float* bpw,
                      const float* wdw, const float* bdw, int OH, int OW, int pad_t, int pad_l, int cs_mid, void* y,
                      float* psum, bool split, double flops, double bytes, hipStream_t s, bool f8_out) {
  M2S_CHECK(N > 0 && ir_s2band_supported(IH, IW, OH, OW, cs_in, kp, cs_mid), "ir_s2band: unsupported shape");
  M2S_CHECK(!(split && f8_out), "ir_s2band: e4m3 output is a bf16-path variant");
  const int mode = split ? 1 : f8_out ? 2 : 0;
  M2S_CHECK(pad_t >= 0 && pad_t <= 1 && pad_l >= 0 && pad_l <= 1 && 2 * (OW - 1) - pad_l + 2 <= IW &&
                2 * (OH - 1) - pad_t + 2 <= IH,
            "ir_s2band: geometry");
  const dim3 grid((unsigned)N * (OH / SB_BO) * (cs_mid / SB_SL));
  const size_t lds = sb_tile_bytes(IW);
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  const bf16_t* wb = static_cast<const bf16_t*>(wpw);
  bf16_t* yb = static_cast<bf16_t*>(y);
#define M2S_SB(KSN_, SP_)                                                                                   \
  if (kp == KSN_ * 32 && mode == SP_) {                                                                      \
    ProfScope ps("ir_s2band_kernel<" #KSN_ ", " #SP_ ">", flops, bytes, s);                                  \
    hipLaunchKernelGGL((ir_s2band_kernel<KSN_, SP_>), grid, dim3(256), lds, s, xb, IH, IW, wb, bpw, wdw, bdw, OH, OW, \
                       pad_t, pad_l, cs_mid, yb, psum);                                                       \
  }
  M2S_SB(2, 1) M2S_SB(1, 1) M2S_SB(2, 0) M2S_SB(1, 0) M2S_SB(2, 2) M2S_SB(1, 2)
#undef M2S_SB
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
