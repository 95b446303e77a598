// Fused HiFi-GAN ResBlock1 (bf16) for the narrow, long MRF stages (C = 32 and 64 channels):
//   for each (c1, c2) pair:  xt = c2(lrelu(c1(lrelu(x)))) ;  x = xt + x        (models.py:35-49)
// and the MRF running sum over the stage's resblocks, S = (S + x) / num_kernels (models.py:119-125),
// in ONE launch per resblock instead of 2 x pairs conv launches plus their HBM round trips.
//
// The convs are causal (get_padding(k, d) = k*d - d on both sides, output truncated to len(x):
// utils.py:33-34, models.py:43-47), so an output tile [t0, t0 + TOUT) of the resblock depends only
// on inputs [t0 - H, t0 + TOUT) with H = sum_p (k-1)(d_p + 1).  A workgroup owns one such tile of
// one clip: it loads the H + TOUT input rows once, runs every conv of the resblock on the shrinking
// valid window in LDS, and writes only the TOUT final rows.  Rows before the clip start are the
// zero padding of every conv input, so each epilogue stores exact zeros there.
//
// LDS holds two activation images, A = lrelu(x) (the c1 input) and T = lrelu(c1 out) (the c2
// input), as C/8 planes of 16-byte chunks ([chunk][row][8 channels]).  With planes a multiple of
// 256 B apart the MFMA B-fragment read of 16 consecutive rows x 4 chunks (ds_read_b128, lane groups
// {0-3,12-15,20-27}, ...) touches 64 distinct banks for ANY row offset - the dilated taps shift the
// row window by arbitrary amounts, which a row-XOR swizzle cannot follow.  The residual x is not
// stored: it is recovered from A as x = a > 0 ? a : 10a (LeakyReLU slope 0.1 is invertible; the
// recovered value carries one bf16 rounding, as a stored bf16 x would).
//
// MFMA v_mfma_f32_16x16x32_bf16: A operand = weights, B = 16 positions x 32 channels of one tap
// from the planes; each lane ends with 4 consecutive channels of one position.  The weights of
// all 2 x pairs convs stream through a 3-slot LDS ring of 8 KB stages (one 1 KB LDS-DMA piece per
// wave per stage; a stage = TG taps, TG = 4 at C = 32, 1 at C = 64), packed on the host in
// fragment order ([tap][n16][k32][lane][8]) so every fragment read is one contiguous 1 KB
// ds_read_b128.  The ring runs across conv boundaries: the next conv's first weights land while
// the current one finishes.  8 waves; subtile (16 rows) s belongs to wave s % 8 in every conv, so
// a lane's residual rows are the rows it writes.
//
// Split fp32 (SP = 1, m2s_common.hpp sp_t; C = 32): x, S and the LDS images carry hi and lo halves
// (NPL hi planes then NPL lo planes), the weights hi and lo fragments per tap ([tap][hi/lo][n16][k32]
// [lane][8], two taps per 8 KB stage), every product is the three MFMA terms, activations are formed in
// fp32 from hi + lo and re-split when stored; x is recovered from A = lrelu(x) in fp32 (10 a for a < 0).
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "conv_igemm.hpp"
#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

constexpr int RB_MAXP = 4;   // (c1, c2) pairs per resblock
constexpr int RB_HMAX = 128; // history rows a tile may carry (k = 11, d = 1,3,5 needs 120)

struct RbArgs {
  const bf16_t* x;  // stage input (B, L, C)
  bf16_t* s;        // MRF running sum (B, L, C)
  const bf16_t* w1[RB_MAXP];
  const float* b1[RB_MAXP];
  const bf16_t* w2[RB_MAXP];
  const float* b2[RB_MAXP];
  int dil[RB_MAXP];
  int np, kp, L, H, tiles;
  int accum;  // 0: S = x ; 1: S += x ; 2: S = (S + x) / div
  float div;
};

__device__ __forceinline__ float lrelu01(float v) { return v > 0.f ? v : v * 0.1f; }
__device__ __forceinline__ float unlrelu01(float a) { return a > 0.f ? a : a * 10.f; }
__device__ __forceinline__ float lo16(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi16(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t lrelu_pk(uint32_t u) { return pack_bf16x2(lrelu01(lo16(u)), lrelu01(hi16(u))); }

// An epilogue store into a plane: lane (g, r16) holds 8 bytes (4 channels) of row r16, and lane groups g and g ^ 1
// hold the two halves of the same 16-byte row chunk.  Stored as one ds_write_b64 per lane, each 16-lane group put
// 16 rows x 8 bytes at a 16-byte stride: rows r and r + 8 share store banks ((a / 4) mod 32), a 2-way conflict
// on every epilogue store (0.29 / 0.40 / 0.69 conflict cycles per LDS instruction at k = 11 / 7 / 3,
// profiles/r06ev2_sq_mfma.txt).  Here the even groups take their partner's half (v_permlane16_swap: lanes l and
// l + 16) and store whole 16-byte rows: every 8-lane ds_write_b128 group covers 128 contiguous bytes.
// p16: the row chunk's start (16-byte aligned: told to the compiler, else it emits ds_write2_b64).
#ifndef RB1_ROWST
#define RB1_ROWST 0  // 1: row-wide stores (conflict-free, measured 5 % slower: DESIGN §13.2)
#endif
__device__ __forceinline__ void st_row16(char* p16, uint2 v, int g) {
  if (!RB1_ROWST) {
    *reinterpret_cast<uint2*>(p16 + 8 * (g & 1)) = v;
    return;
  }
  const auto sx = __builtin_amdgcn_permlane16_swap(v.x, v.x, false, false);
  const auto sy = __builtin_amdgcn_permlane16_swap(v.y, v.y, false, false);
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));  // (a uint4 store was scalarised into 4 stores)
  if (!(g & 1)) *reinterpret_cast<u32x4_t*>(__builtin_assume_aligned(p16, 16)) = u32x4_t{v.x, v.y, sx[1], sy[1]};
}

enum { PASS_C1 = 0, PASS_C2 = 1, PASS_LAST = 2 };
constexpr int RB_NW = 8;          // waves per workgroup
constexpr int RB_STAGE = 8192;    // bytes per weight stage = one 1 KB piece per wave
constexpr int RB_SLOTS = 3;       // weight ring depth

template <int C, int SP = 0>
constexpr int rb_tg() {  // taps per weight stage
  return RB_STAGE / (C * C * 2 * (SP ? 2 : 1));
}

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct Ring {
  const RbArgs* a;
  char* base;
  int ns, q_total, wave, lane;
  // weight stage q (conv q / ns, local stage q % ns) -> ring slot q % RB_SLOTS
  __device__ __forceinline__ void issue(int q) const {
    const int c = q / ns, ls = q - c * ns;
    const bf16_t* w = (c & 1) ? a->w2[c >> 1] : a->w1[c >> 1];
    const char* src = reinterpret_cast<const char*>(w) + (size_t)ls * RB_STAGE + wave * 1024 + lane * 16;
    dma16(src, base + (q % RB_SLOTS) * RB_STAGE + wave * 1024);
  }
};

template <int C, int K, int TOUT, int PASS, int SP>
__device__ __forceinline__ void conv_pass(const RbArgs& a, const Ring& ring, int conv, const char* in, char* io,
                                          const float* bias_lds, int d, int lo_out, int R, int PLANE, int wave,
                                          int g, int r16, int lane, int clip, int t0) {
  constexpr int NT = C / 16, KC = C / 32, TG = rb_tg<C, SP>(), HR = SP ? 2 : 1, NPL = C / 8;
  constexpr int NS = (K + TG - 1) / TG;
  constexpr int MS = (RB_HMAX + TOUT + 16 * RB_NW - 1) / (16 * RB_NW);  // subtiles per wave at most
  const int s_lo = lo_out >> 4, s_hi = R >> 4;

  f32x4 acc[MS][NT];
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int ls = 0; ls < NS; ++ls) {
    const int q = conv * NS + ls;
    // this wave's piece of stage q has landed once only stage q+1 (if any) is younger
    if (q + 1 < ring.q_total)
      wait_vm<1>();
    else
      wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every piece of stage q landed; slot (q-1) % 3 is free
    if (q + 2 < ring.q_total) ring.issue(q + 2);
    const char* ws = ring.base + (q % RB_SLOTS) * RB_STAGE + lane * 16;
#pragma unroll
    for (int tl = 0; tl < TG; ++tl) {
      const int j = ls * TG + tl;  // tap
      if (j >= K) break;
      bf16x8 wf[NT][KC], wl[SP ? NT : 1][SP ? KC : 1];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          wf[nt][kc] = *reinterpret_cast<const bf16x8*>(ws + (((tl * HR) * NT + nt) * KC + kc) * 1024);
          if constexpr (SP) wl[nt][kc] = *reinterpret_cast<const bf16x8*>(ws + (((tl * HR + 1) * NT + nt) * KC + kc) * 1024);
        }
      const int shift = (K - 1 - j) * d;
#pragma unroll
      for (int i = 0; i < MS; ++i) {
        const int s = wave + RB_NW * i;
        if (s >= s_lo && s < s_hi) {
          const int row = 16 * s + r16 - shift + 16;  // +16: guard rows (zeros) below row 0
#pragma unroll
          for (int kc = 0; kc < KC; ++kc) {
            const bf16x8 b = *reinterpret_cast<const bf16x8*>(in + (kc * 4 + g) * PLANE + row * 16);
            if constexpr (SP) {
              const bf16x8 bl = *reinterpret_cast<const bf16x8*>(in + (NPL + kc * 4 + g) * PLANE + row * 16);
#pragma unroll
              for (int nt = 0; nt < NT; ++nt) {
                acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[nt][kc], b, acc[i][nt], 0, 0, 0);
                acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt][kc], bl, acc[i][nt], 0, 0, 0);
              }
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt][kc], b, acc[i][nt], 0, 0, 0);
          }
        }
      }
    }
  }

  // ---- epilogue: 4 consecutive channels of one position per lane ------------------------------
#pragma unroll
  for (int i = 0; i < MS; ++i) {
    const int s = wave + RB_NW * i;
    if (s < s_lo || s >= s_hi) continue;
    const int r = 16 * s + r16, t = t0 + r;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = nt * 16 + 4 * g;
      const float4 bb = *reinterpret_cast<const float4*>(bias_lds + n);
      char* p16 = io + (n >> 3) * PLANE + (r + 16) * 16;  // the row chunk
      char* p = p16 + (n & 7) * 2;
      float v[4] = {acc[i][nt][0] + bb.x, acc[i][nt][1] + bb.y, acc[i][nt][2] + bb.z, acc[i][nt][3] + bb.w};
      if constexpr (PASS != PASS_C1) {  // residual: x recovered from A = lrelu(x) at this row
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        float x[4] = {lo16(u.x), hi16(u.x), lo16(u.y), hi16(u.y)};
        if constexpr (SP) {
          const uint2 ul = *reinterpret_cast<const uint2*>(p + NPL * PLANE);
          x[0] += lo16(ul.x);
          x[1] += hi16(ul.x);
          x[2] += lo16(ul.y);
          x[3] += hi16(ul.y);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += unlrelu01(x[q]);
      }
      if constexpr (PASS != PASS_LAST) {
        float o[4] = {0.f, 0.f, 0.f, 0.f};
        if (t >= 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = lrelu01(v[q]);
        }
        if constexpr (SP) {
          uint2 oh, ol;
          split4(o, oh, ol);
          st_row16(p16, oh, g);
          st_row16(p16 + NPL * PLANE, ol, g);
        } else {
          st_row16(p16, make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])), g);
        }
      } else if (r >= a.H && t < a.L) {
        bf16_t* sp = a.s + ((size_t)clip * a.L + t) * C * HR + n;
        if (a.accum) {
          const uint2 u = *reinterpret_cast<const uint2*>(sp);
          v[0] += lo16(u.x);
          v[1] += hi16(u.x);
          v[2] += lo16(u.y);
          v[3] += hi16(u.y);
          if constexpr (SP) {
            const uint2 ul = *reinterpret_cast<const uint2*>(sp + C);
            v[0] += lo16(ul.x);
            v[1] += hi16(ul.x);
            v[2] += lo16(ul.y);
            v[3] += hi16(ul.y);
          }
          if (a.accum == 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = v[q] / a.div;
          }
        }
        if constexpr (SP) {
          uint2 oh, ol;
          split4(v, oh, ol);
          *reinterpret_cast<uint2*>(sp) = oh;
          *reinterpret_cast<uint2*>(sp + C) = ol;
        } else {
          *reinterpret_cast<uint2*>(sp) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
      }
    }
  }
}

template <int C, int K, int TOUT, int SP>
__global__ void __launch_bounds__(RB_NW * 64) rb1_fused_kernel(const RbArgs a) {
  constexpr int NPL = C / 8;  // 16-byte planes (per half when split)
  constexpr int HR = SP ? 2 : 1;
  constexpr int TG = rb_tg<C, SP>(), NS = (K + TG - 1) / TG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int R = a.H + TOUT, ROWS = R + 16, PLANE = ROWS * 16;
  char* wring = smem;
  float* bias_lds = reinterpret_cast<float*>(smem + RB_SLOTS * RB_STAGE);  // [2 np][C]
  char* bufA = smem + RB_SLOTS * RB_STAGE + 2 * RB_MAXP * C * 4;
  char* bufT = bufA + HR * NPL * PLANE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifndef RB1_PRIO
#define RB1_PRIO 1
#endif
  // the younger half at static priority (er_sp_fused.hip): same-box A/B -3 % / -1 % at k = 11 / 7, +7 % at k = 3
  if (RB1_PRIO && RB_NW == 8 && K >= 7 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int g = lane >> 4, r16 = lane & 15;
  const int clip = blockIdx.x / a.tiles, tile = blockIdx.x - clip * a.tiles;
  const int t0 = tile * TOUT - a.H;  // time of row 0
  const bf16_t* xc = a.x + (size_t)clip * a.L * C * HR;

  // ---- A = lrelu(x) for rows [-16, R) (guard rows and t outside the clip: zeros); T = 0; biases -
  // 16 consecutive lanes take 16 consecutive rows of one plane (ROWS % 16 == 0: rb_history rounds H to 16), so each
  // ds_write_b128 lane group fills 16 distinct bank slots; with the planes of one row on consecutive lanes (the planes
  // lie a multiple of 256 B apart) every store was 4-way conflicted: 0.7 / 1.0 / 1.6 conflict cycles per LDS
  // instruction at k = 11 / 7 / 3 (profiles/r05fin6_sq_mfma.txt)
  for (int i = tid; i < ROWS * NPL; i += RB_NW * 64) {
    const int pr = (i / (16 * NPL)) * 16 + (i & 15), c = (i >> 4) % NPL, t = t0 + pr - 16;
    if constexpr (SP) {
      uint2 h0 = make_uint2(0u, 0u), l0 = h0, h1 = h0, l1 = h0;
      if (pr >= 16 && t >= 0 && t < a.L) {
        const uint4 uh = *reinterpret_cast<const uint4*>(xc + (size_t)t * 2 * C + c * 8);
        const uint4 ul = *reinterpret_cast<const uint4*>(xc + (size_t)t * 2 * C + C + c * 8);
        float v[8] = {lo16(uh.x) + lo16(ul.x), hi16(uh.x) + hi16(ul.x), lo16(uh.y) + lo16(ul.y),
                      hi16(uh.y) + hi16(ul.y), lo16(uh.z) + lo16(ul.z), hi16(uh.z) + hi16(ul.z),
                      lo16(uh.w) + lo16(ul.w), hi16(uh.w) + hi16(ul.w)};
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = lrelu01(v[q]);
        split4(v, h0, l0);
        split4(v + 4, h1, l1);
      }
      *reinterpret_cast<uint4*>(bufA + c * PLANE + pr * 16) = make_uint4(h0.x, h0.y, h1.x, h1.y);
      *reinterpret_cast<uint4*>(bufA + (NPL + c) * PLANE + pr * 16) = make_uint4(l0.x, l0.y, l1.x, l1.y);
      *reinterpret_cast<uint4*>(bufT + c * PLANE + pr * 16) = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(bufT + (NPL + c) * PLANE + pr * 16) = make_uint4(0u, 0u, 0u, 0u);
    } else {
      uint4 u = make_uint4(0u, 0u, 0u, 0u);
      if (pr >= 16 && t >= 0 && t < a.L) {
        u = *reinterpret_cast<const uint4*>(xc + (size_t)t * C + c * 8);
        u.x = lrelu_pk(u.x);
        u.y = lrelu_pk(u.y);
        u.z = lrelu_pk(u.z);
        u.w = lrelu_pk(u.w);
      }
      *reinterpret_cast<uint4*>(bufA + c * PLANE + pr * 16) = u;
      *reinterpret_cast<uint4*>(bufT + c * PLANE + pr * 16) = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  for (int i = tid; i < 2 * a.np * C; i += RB_NW * 64) {
    const int c = i / C, n = i - c * C;
    bias_lds[i] = ((c & 1) ? a.b2[c >> 1] : a.b1[c >> 1])[n];
  }
  // first two weight stages (the loads above complete first: the compiler waits for them before
  // their LDS stores)
  Ring ring{&a, wring, NS, 2 * a.np * NS, wave, lane};
  __syncthreads();
  ring.issue(0);
  if (ring.q_total > 1) ring.issue(1);

  int tot = 0;  // sum over the remaining pairs of (d + 1)
  for (int p = 0; p < a.np; ++p) tot += a.dil[p] + 1;
  for (int p = 0; p < a.np; ++p) {
    const int d = a.dil[p];
    const int lo_x = a.H - (K - 1) * tot;  // first valid row of this pair's input x
    const int lo_t = lo_x + (K - 1) * d;   // ... of c1's output
    const int lo_y = lo_t + (K - 1);       // ... of c2's output (the next x)
    tot -= d + 1;
    conv_pass<C, K, TOUT, PASS_C1, SP>(a, ring, 2 * p, bufA, bufT, bias_lds + 2 * p * C, d, lo_t, R, PLANE, wave, g, r16,
                                   lane, clip, t0);
    __syncthreads();
    if (p + 1 < a.np) {
      conv_pass<C, K, TOUT, PASS_C2, SP>(a, ring, 2 * p + 1, bufT, bufA, bias_lds + (2 * p + 1) * C, 1, lo_y, R, PLANE,
                                     wave, g, r16, lane, clip, t0);
      __syncthreads();
    } else {
      conv_pass<C, K, TOUT, PASS_LAST, SP>(a, ring, 2 * p + 1, bufT, bufA, bias_lds + (2 * p + 1) * C, 1, lo_y, R, PLANE,
                                       wave, g, r16, lane, clip, t0);
    }
  }
}

template <int C, int K, int TOUT, int SP>
void launch_cfg(const RbArgs& a, int B, hipStream_t s, double flops, double bytes) {
  constexpr int NPL = C / 8, HR = SP ? 2 : 1;
  const size_t lds = RB_SLOTS * RB_STAGE + 2 * RB_MAXP * C * 4 + 2 * (size_t)HR * NPL * (a.H + TOUT + 16) * 16;
  M2S_CHECK(lds <= 160 * 1024, "rb1_fused: LDS budget");
  allow_lds(reinterpret_cast<const void*>(&rb1_fused_kernel<C, K, TOUT, SP>));
  char name[64];
  snprintf(name, sizeof(name), "rb1_fused_kernel<%d, %d, %d, %d>", C, K, TOUT, SP);
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((rb1_fused_kernel<C, K, TOUT, SP>), dim3(B * a.tiles), dim3(RB_NW * 64), lds, s, a);
  M2S_HIP(hipGetLastError());
}

int rb_tg_host(int C, bool split) {
  if (split) return rb_tg<32, 1>();
  return C == 32 ? rb_tg<32>() : rb_tg<64>();
}

int rb_history(int k, const int* dil, int np) {
  int h = 0;
  for (int p = 0; p < np; ++p) h += (k - 1) * (dil[p] + 1);
  return round_up(h, 16);
}

template <int C>
constexpr int rb_tout() {
  return 256;
}

}  // namespace

int rb1_frag_taps(int C, int k, bool split) { return round_up(k, rb_tg_host(C, split)); }

bool rb1_fused_supported(int C, int cs, int k, const int* dil, int np, int kp, bool split) {
  if (!(C == 32 || C == 64) || cs != C || np < 1 || np > RB_MAXP || kp != k * C) return false;
  if (split && C != 32) return false;  // C = 64 split images + ring exceed the LDS budget at TOUT = 256
  if (!(k == 3 || k == 5 || k == 7 || k == 11)) return false;
  for (int p = 0; p < np; ++p)
    if (dil[p] < 1) return false;
  return rb_history(k, dil, np) <= RB_HMAX;
}

void launch_rb1_fused(const bf16_t* x, bf16_t* s, int B, int L, int C, int k, int np, const int* dil,
                      const bf16_t* const* w1, const float* const* b1, const bf16_t* const* w2,
                      const float* const* b2, int kp, int accum, float div, bool split, double flops, double bytes,
                      hipStream_t st) {
  M2S_CHECK(rb1_fused_supported(C, C, k, dil, np, kp, split), "rb1_fused: unsupported resblock");
  M2S_CHECK(B > 0 && L > 0 && (double)B * L * C < 2147483647.0, "rb1_fused: shape");
  RbArgs a;
  std::memset(&a, 0, sizeof(a));
  a.x = x;
  a.s = s;
  for (int p = 0; p < np; ++p) {
    a.w1[p] = w1[p];
    a.b1[p] = b1[p];
    a.w2[p] = w2[p];
    a.b2[p] = b2[p];
    a.dil[p] = dil[p];
  }
  a.np = np;
  a.kp = kp;
  a.L = L;
  a.H = rb_history(k, dil, np);
  a.accum = accum;
  a.div = div;
  if (split) {
    a.tiles = ceil_div(L, rb_tout<32>());
    switch (k) {
      case 3: launch_cfg<32, 3, rb_tout<32>(), 1>(a, B, st, flops, bytes); break;
      case 5: launch_cfg<32, 5, rb_tout<32>(), 1>(a, B, st, flops, bytes); break;
      case 7: launch_cfg<32, 7, rb_tout<32>(), 1>(a, B, st, flops, bytes); break;
      default: launch_cfg<32, 11, rb_tout<32>(), 1>(a, B, st, flops, bytes); break;
    }
  } else if (C == 32) {
    a.tiles = ceil_div(L, rb_tout<32>());
    switch (k) {
      case 3: launch_cfg<32, 3, rb_tout<32>(), 0>(a, B, st, flops, bytes); break;
      case 5: launch_cfg<32, 5, rb_tout<32>(), 0>(a, B, st, flops, bytes); break;
      case 7: launch_cfg<32, 7, rb_tout<32>(), 0>(a, B, st, flops, bytes); break;
      default: launch_cfg<32, 11, rb_tout<32>(), 0>(a, B, st, flops, bytes); break;
    }
  } else {
    a.tiles = ceil_div(L, rb_tout<64>());
    switch (k) {
      case 3: launch_cfg<64, 3, rb_tout<64>(), 0>(a, B, st, flops, bytes); break;
      case 5: launch_cfg<64, 5, rb_tout<64>(), 0>(a, B, st, flops, bytes); break;
      case 7: launch_cfg<64, 7, rb_tout<64>(), 0>(a, B, st, flops, bytes); break;
      default: launch_cfg<64, 11, rb_tout<64>(), 0>(a, B, st, flops, bytes); break;
    }
  }
}

}  // namespace m2s
