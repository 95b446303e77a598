// Split-fp32 causal dilated Conv1d for the C = 64 HiFi-GAN MRF stage (models.py:11-49, 114-125:
// ResBlock1 convs1 / convs2, k in {3, 7, 11}, d in {1, 3, 5}; causal padding get_padding = (k-1) d on the
// left, utils.py:33-34), with the input rows staged ONCE per tile.
//
// conv_gemm's implicit GEMM streams the activation tile from L2 again for every tap: a k-tap conv
// moves k copies of its input through L2 -> LDS, plus the weights per tile, which made these convs
// L2-bandwidth bound (about 0.2-0.3 of the MFMA rate).  Here a workgroup owns BM = 128 output rows of
// one clip and DMAs the input rows [t0 - 64, t0 + 128) into LDS once (64 history rows cover
// (k - 1) d <= 64; rows before the clip start are the zero padding), then every tap reads its shifted
// 16-row windows from that image.  Only the weights stream, (tap, 32-channel chunk) stages of
// C x 32 hi/lo bf16 in MFMA fragment order through an LDS-DMA ring (4 slots at C = 64, three stages
// ahead: every workgroup reads the same stage from L2 at about the same time, so its latency is long).
//
// LDS image: 2 x C/8 planes (hi planes, then lo planes) of 16-byte chunks [plane][row][8 channels],
// planes a multiple of 256 B apart, so a B-fragment read (16 consecutive rows x 4 planes, ds_read_b128)
// touches 64 distinct banks for ANY row offset (mrf_fused.hip; the taps shift by arbitrary d).
// MFMA v_mfma_f32_16x16x32_bf16: A = weights (16 outputs x 32 inputs), B = 16 positions x 32 inputs,
// three terms per product (Wl Xh + Wh Xl + Wh Xh).  4 waves at C = 64 (wave w: rows [32 w, 32 w + 32), all
// outputs; two workgroups per CU), 8 at C = 128 (rows [32 (w % 4), +32), outputs [64 (w / 4), +64); the
// 96 KB image leaves room for one workgroup per CU).  Epilogue = conv_gemm's: bias, LeakyReLU, residual stored as lrelu(x) and inverted,
// activation after the residual, MRF accumulation.  grid.z batches up to CONV_BATCH convs of one
// shape (the resblocks of a stage).
#include <cstring>

#include "conv_igemm.hpp"
#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_h1_zero[4];

constexpr int H1_BM = 128;               // output rows per tile
constexpr int H1_HIST = 64;              // history rows: (k - 1) d <= 64
constexpr int H1_ROWS = H1_BM + H1_HIST; // image rows
constexpr int H1_PLANE = H1_ROWS * 16;   // 3072 B = 12 x 256

template <int C>
constexpr int h1_stage() {  // bytes of one (tap, 32-channel chunk) weight stage: hi + lo fragments
  return 2 * (C / 16) * 1024;
}
template <int C>
constexpr int h1_slots() {  // weight ring depth: stages in flight = slots - 1 (C = 64: 80 KB, two workgroups per CU)
  return C <= 64 ? 4 : 3;
}
template <int C>
constexpr int h1_lds() {
  return 2 * (C / 8) * H1_PLANE + h1_slots<C>() * h1_stage<C>();
}

__device__ __forceinline__ void dma16(const void* src, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_wave_base)
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int C>
constexpr int h1_waves() {  // C = 128: 8 waves (two per SIMD in the one workgroup its 144 KB allow)
  return C <= 64 ? 4 : 8;
}

template <int C>
__global__ void __launch_bounds__(64 * h1_waves<C>(), 2) conv1d_halo_sp_kernel(const ConvBatch ab, int tiles) {
  constexpr int NPL = C / 8, NT = C / 16, KC = C / 32;
  constexpr int NW = h1_waves<C>(), NTW = NT * 4 / NW;  // waves; 16-output tiles per wave
  constexpr int STAGE = h1_stage<C>();
  constexpr int PPW = STAGE / 1024 / NW;  // weight DMA pieces per wave per stage
  constexpr int SLOTS = h1_slots<C>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* img = smem;
  char* ring = smem + 2 * NPL * H1_PLANE;
  const ConvArgs a = ab.a[blockIdx.z];  // a copy: fields land in SGPRs once, not re-loaded per stage

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int wr = wave & 3, ntb = (wave >> 2) * NTW;  // the wave's 32 rows and first 16-output tile
  const int clip = blockIdx.x / tiles, tile = blockIdx.x - clip * tiles;
  const int L = a.L_out, t0 = tile * H1_BM;
  const int Q = a.ntaps * KC;  // weight stages
  const bf16_t* __restrict__ X = static_cast<const bf16_t*>(a.x);
  const char* W = static_cast<const char*>(a.w);
  const char* zp = reinterpret_cast<const char*>(g_h1_zero);
  asm volatile("" : "+s"(zp));
  const uint32_t img0 = (uint32_t)(uintptr_t)img, ring0 = (uint32_t)(uintptr_t)ring;

  // ---- the epilogue's residual and MRF-sum operands, fetched first: read at the end of the tile they
  // were a second exposed HBM round trip (c2 launches ran ~30 % longer than c1) ----
  bf16_t* __restrict__ Y = static_cast<bf16_t*>(a.y);
  const bf16_t* __restrict__ Rs = static_cast<const bf16_t*>(a.res);
  uint2 prh[2][NTW], prl[2][NTW], pyh[2][NTW], pyl[2][NTW];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int t = t0 + 32 * wr + 16 * i + r16;
    const size_t orow = ((size_t)clip * L + (t < L ? t : 0)) * a.cs_out * 2;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n4 = (ntb + nt) * 16 + 4 * g;
      prh[i][nt] = prl[i][nt] = pyh[i][nt] = pyl[i][nt] = make_uint2(0u, 0u);
      if (Rs && t < L) {
        prh[i][nt] = *reinterpret_cast<const uint2*>(Rs + orow + n4);
        prl[i][nt] = *reinterpret_cast<const uint2*>(Rs + orow + a.cs_out + n4);
      }
      if (a.accum && t < L) {
        pyh[i][nt] = *reinterpret_cast<const uint2*>(Y + orow + n4);
        pyl[i][nt] = *reinterpret_cast<const uint2*>(Y + orow + a.cs_out + n4);
      }
    }
  }

  // ---- the image: piece (plane p, 64-row block rb) = 64 consecutive rows of one plane ----
  {
    constexpr int PIECES = 2 * NPL * (H1_ROWS / 64);
    const int t = t0 - H1_HIST + lane;  // + 64 rb
    for (int pc = wave; pc < PIECES; pc += NW) {
      const int p = pc / (H1_ROWS / 64), rb = pc - p * (H1_ROWS / 64);
      const int half = p / NPL, ch = p - half * NPL, tt = t + 64 * rb;
      const void* src = tt >= 0 && tt < L
                            ? static_cast<const void*>(X + ((size_t)clip * L + tt) * (2 * a.cs_in) + half * a.cs_in + ch * 8)
                            : static_cast<const void*>(zp);
      dma16(src, __builtin_amdgcn_readfirstlane(img0 + (uint32_t)(p * H1_PLANE + rb * 1024)));
    }
  }
  auto issue = [&](int q) {  // weight stage q -> slot q % SLOTS: this wave's PPW pieces
    const char* src = W + (size_t)q * STAGE + (wave * PPW) * 1024 + lane * 16;
    const uint32_t dst = ring0 + (uint32_t)((q % SLOTS) * STAGE + wave * PPW * 1024);
#pragma unroll
    for (int j = 0; j < PPW; ++j) dma16(q < Q ? static_cast<const void*>(src + j * 1024) : static_cast<const void*>(zp), dst + j * 1024);
  };
#pragma unroll
  for (int q = 0; q < SLOTS - 1; ++q) issue(q);

  f32x4 acc[2][NTW];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  int tap = 0, kc = 0;
  for (int q = 0; q < Q; ++q) {
    // stage q (and, at q = 0, the image) landed for this wave once only stages q + 1 .. q + SLOTS - 2
    // are younger (the tail issues zero-page stages, so the count holds)
    wait_vm<(SLOTS - 2) * PPW>();
    __builtin_amdgcn_s_barrier();  // ... for every wave; slot (q - 1) % SLOTS is free
    asm volatile("" ::: "memory");
    issue(q + SLOTS - 1);
    const char* ws = ring + (q % SLOTS) * STAGE + lane * 16;
    bf16x8 wh[NTW], wl[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      wh[nt] = *reinterpret_cast<const bf16x8*>(ws + (ntb + nt) * 1024);
      wl[nt] = *reinterpret_cast<const bf16x8*>(ws + (NT + ntb + nt) * 1024);
    }
    const int shift = (a.ntaps - 1 - tap) * a.dil;
    const char* ib = img + (kc * 4 + g) * H1_PLANE + (H1_HIST + 32 * wr + r16 - shift) * 16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(ib + i * 256);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(ib + NPL * H1_PLANE + i * 256);
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[nt], bh, acc[i][nt], 0, 0, 0);
        acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[nt], bl, acc[i][nt], 0, 0, 0);
        acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[nt], bh, acc[i][nt], 0, 0, 0);
      }
    }
    if (++kc == KC) {
      kc = 0;
      ++tap;
    }
  }
  wait_vm<0>();  // the zero-page stages issued past the end

  // ---- epilogue (conv_gemm.hip's, split): lane = 4 consecutive outputs of one position ----
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int t = t0 + 32 * wr + 16 * i + r16;
    if (t >= L) continue;
    const size_t orow = ((size_t)clip * L + t) * a.cs_out * 2;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const int n4 = (ntb + nt) * 16 + 4 * g;
      const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
      float v[4] = {acc[i][nt][0] + bb.x, acc[i][nt][1] + bb.y, acc[i][nt][2] + bb.z, acc[i][nt][3] + bb.w};
      auto apply_act = [&]() {
        if (a.act == ACT_LRELU) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * a.act_slope;
        }
      };
      if (!a.act_after_res) apply_act();
      if (Rs) {
        float r[4], rl[4];
        unpack_bf16x4(prh[i][nt], r);
        unpack_bf16x4(prl[i][nt], rl);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          r[j] += rl[j];
          if (a.res_unslope != 0.f) r[j] = r[j] > 0.f ? r[j] : r[j] * a.res_unslope;
          v[j] += r[j];
        }
      }
      if (a.accum) {
        float p[4], pl[4];
        unpack_bf16x4(pyh[i][nt], p);
        unpack_bf16x4(pyl[i][nt], pl);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (p[j] + pl[j]) + v[j];
        if (a.accum == 2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = v[j] / a.accum_div;
        }
      }
      if (a.act_after_res) apply_act();
      uint2 hi, lo;
      split4(v, hi, lo);
      *reinterpret_cast<uint2*>(Y + orow + n4) = hi;
      *reinterpret_cast<uint2*>(Y + orow + a.cs_out + n4) = lo;
    }
  }
}

template <int C>
void launch_c(const ConvBatch& b, int n, int B, int L, hipStream_t s, double flops, double bytes) {
  allow_lds(reinterpret_cast<const void*>(&conv1d_halo_sp_kernel<C>));
  const int tiles = ceil_div(L, H1_BM);
  char name[48];
  snprintf(name, sizeof(name), "conv1d_halo_sp_kernel<%d>", C);
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((conv1d_halo_sp_kernel<C>), dim3(B * tiles, 1, n), dim3(64 * h1_waves<C>()), h1_lds<C>(), s, b, tiles);
  M2S_HIP(hipGetLastError());
}

}  // namespace

// C = 128 (8 waves, one workgroup per CU for its 96 KB image) measured 2.42 ms per step against conv_gemm's
// 2.28 for the stage: only C = 64 is routed here.
bool conv1d_halo_sp_supported(int C, int cs, int k, int dil) {
  return C == 64 && cs == C && k >= 1 && k <= 31 && dil >= 1 && (k - 1) * dil <= H1_HIST;
}
size_t conv1d_halo_frag_elems(int C, int k) { return (size_t)k * (C / 32) * 2 * C * 32; }

void launch_conv1d_halo_sp(const ConvArgs* as, int n, hipStream_t s, double flops, double bytes) {
  M2S_CHECK(n >= 1 && n <= CONV_BATCH, "conv1d_halo: 1..CONV_BATCH convs");
  const ConvArgs& a = as[0];
  ConvBatch b;
  std::memset(&b, 0, sizeof(b));
  for (int i = 0; i < n; ++i) {
    const ConvArgs& c = as[i];
    M2S_CHECK(c.kind == KIND_CONV1D && c.cs_in == a.cs_in && c.cs_out == a.cs_in && c.M == a.M && c.L_in == c.L_out &&
                  c.L_out == a.L_out && c.in_xform == IN_NONE && c.pad_left == (c.ntaps - 1) * c.dil &&
                  conv1d_halo_sp_supported(a.cs_in, c.cs_in, c.ntaps, c.dil),
              "conv1d_halo: causal 1-D convs of one shape, C = 64, (k - 1) d <= 64");
    M2S_CHECK(c.x && c.w && c.bias && c.y && c.y != c.x && c.y != c.res, "conv1d_halo: operand pointers");
    for (int j = 0; j < i; ++j) M2S_CHECK(as[j].y != c.y, "conv1d_halo: two convs write one output");
    b.a[i] = c;
  }
  const int L = a.L_out, B = a.M / L;
  M2S_CHECK(B * L == a.M && L > 0, "conv1d_halo: M = clips x L");
  M2S_CHECK((double)a.M * a.cs_in * 2 < 2147483647.0, "conv1d_halo: 32-bit offsets");
  launch_c<64>(b, n, B, L, s, flops, bytes);
}

}  // namespace m2s
