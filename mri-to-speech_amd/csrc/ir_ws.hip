// Split-fp32 InvertedResidual front half for the stride-1 blocks on 16x16 and 8x8 maps and the stride-2 block
// at 16x16 (blocks.5.0), as one persistent warp-specialised workgroup per CU:
//   conv_pw (1x1 expand, 3-term MFMA) + bn1 + SiLU -> fp32 LDS tile -> conv_dw 3x3 + bn2 + SiLU -> HBM
//   + the SE squeeze (per-image channel means).
// (timm InvertedResidual conv_pw/bn1/conv_dw/bn2/se.mean; mri_acoustic_model.py:28-34.)  Same outputs
// as ir_pwdw_kernel<.., SP = 1> / ir_pwdw_s2_kernel<1> (ir_fused.hip), which launch one short workgroup per
// (images, 32-channel slice) and spend most of their life waiting on a chain of loads and barriers.
//
// A workgroup (16 waves) owns whole images and walks their (band of 8 input rows, 32-channel slice) steps:
//   waves 0-7 (producers): the band's input rows (+ halo rows) sit in LDS (LDS-DMA once per band); the
//     slice's expand weights and biases stream through a two-slot ring, the depthwise taps through three
//     slots (LDS-DMA one to two slices ahead).  MFMA A = weights (16 channels x 32 k), B = 16 positions x
//     32 k, three terms hi*hi + hi*lo + lo*hi; SiLU(acc + b) -> tile[f % 2].
//   waves 8-15 (consumers): the depthwise of slice f from tile[f % 2] (a lane = 4 channels x 1-2 pixels,
//     fp32 taps in registers, no bounds checks: the tile carries a zero halo), SiLU, split-fp32 stores, and
//     the squeeze: per-wave channel sums added to the image's 32.32 fixed-point sums by LDS atomics.
// No workgroup barrier after the start: the roles hand off through monotonic LDS counters (below), every
// wait bounded (a timeout is reported and NaNs the images' SE means).  Every weight, tap and bias reaches
// LDS by DMA from the producers, so the consumers issue no loads (a load's wait would also drain their
// in-flight stores).  Each SIMD holds two producer and two consumer waves, whose MFMA and VALU interleave.
//
// LDS layouts (reads conflict-free for ds_read_b128's lane groups, MI355X_MICROARCH.md LDS table):
//   x     [pos][hi plane | lo plane], planes padded to 256-byte multiples; 16-byte chunk L of row r
//         stored at (L & ~15) | ((L & 15) ^ h(r)), h(r) = ((r & 3) << 2) | f((r >> 2) & 3), f = [0,2,3,1]
//         (the XOR is applied on the DMA source side: a DMA lane's LDS slot is fixed).
//   W     [k-step][plane][32 rows][4 chunks] with the conv_gemm row swizzle.
//   tile  8 planes of 4 channels x TROWS rows of 16 B; row = (band row + 1) * (W + 2) + col + 1 with a
//         zero halo (columns zeroed once, out-of-image rows written as zeros by the producers);
//         TROWS = 4 (mod 16): a consumer wave's lane groups (8 planes x 2 pixels) then land in 16
//         distinct bank slots (searched exhaustively over plane strides).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_ws_zero[4];  // DMA source of padding chunks

constexpr int WS_SL = 32;  // expanded channels per slice
constexpr int WS_BR = 8;   // output rows per band
constexpr int WS_NP = 8;   // producer waves
constexpr int WS_NC = 8;   // consumer waves
constexpr int WS_UMAX = 3; // producer units per wave (ws_layout bounds the band's subtiles to 12)

__device__ __forceinline__ int swz_f(int x) { return (0x1320 >> (4 * x)) & 3; }
__device__ __forceinline__ int hx_of(int r) { return ((r & 3) << 2) | swz_f((r >> 2) & 3); }
// LDS-DMA in inline asm (cdna_hip_programming.md 'Operands and clobbers', the glds16 recipe): hipcc
// neither sees nor counts it, so it does not drain it with vmcnt(0) before the producer's own LDS
// reads (it did with the builtin: W(i+1)'s DMA waited for at every slice).  Completion: wait_vm0.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_wave_base)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// vmcnt(n) for a wave-uniform n the immediate cannot take: the nearest count <= n (waiting for more is safe)
__device__ __forceinline__ void wait_vm_le(int n) {
  if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

struct WsLayout {
  int XR, TROWS, x_bytes, tile_bytes, w_bytes, total;
};

__host__ __device__ inline int ws_cpp(int cs_in) { return (cs_in * 2 + 255) / 256 * 16; }  // chunks per plane
// S = 2: the tile planes lie TROWS = 5 (mod 16) 16-byte units apart (any odd residue: with the stride-2 consumers'
// pixel order below, conflict-free reads; stride 1 keeps TROWS = 4 (mod 16))
__host__ __device__ inline WsLayout ws_layout(int H, int W, int cs_in, int cs_mid, int S = 1) {
  WsLayout L;
  const int cpp = ws_cpp(cs_in), xp = 2 * cpp * 16;
  L.XR = 0;  // input rows a band needs (its rows and the in-image halo rows)
  for (int r0 = 0; r0 < H; r0 += WS_BR) {
    const int a = r0 > 0 ? r0 - 1 : 0, b = r0 + WS_BR + 1 < H ? r0 + WS_BR + 1 : H;
    L.XR = b - a > L.XR ? b - a : L.XR;
  }
  const int tr = ((H < WS_BR ? H : WS_BR) + 2) * (W + 2);
  L.TROWS = S == 1 ? tr + (20 - tr % 16) % 16 : tr + (21 - tr % 16) % 16;
  L.x_bytes = L.XR * W * xp;
  L.tile_bytes = 2 * 8 * L.TROWS * 16;
  L.w_bytes = 2 * (cs_in / 32) * 4096;
  // taps + biases, the squeeze's fixed-point channel sums [cs_mid] (u64), arrival counts and NaN flags [cs_mid / 32],
  // counters
  L.total = L.x_bytes + L.tile_bytes + L.w_bytes + (3 * 320 + 2 * 32) * 4 + cs_mid * 8 + 2 * (cs_mid / WS_SL) * 4 + 128;
  return L;
}

// Scheduling switches (same results; diagnostic builds set them, tools/build_irws_variants.sh + ab_kern.py):
// HAND_END = the W ring hand-off at the end of a slice, else right after the MFMAs (2: by shape); TAPS_AHEAD =
// slice f + 1's depthwise taps issued at the end of slice f, else at the start of slice f + 1 behind a wait for
// the consumers; PF_DEEP = 2-4 k-steps of MFMA operand reads in flight by unit count, else 2.  Same-box A/B
// (gpurun_out/r05m, us per launch): 16x16 HAND_END 0 682-688 / 1 699-705; 8x8 0 540-553 / 1 531-533; TAPS_AHEAD
// and PF_DEEP within 1-2 %
#ifndef IRWS_HAND_END
#define IRWS_HAND_END 2
#endif
#ifndef IRWS_PF_DEEP
#define IRWS_PF_DEEP 1
#endif
#ifndef IRWS_PAIR
#define IRWS_PAIR 1  // 16x16: a consumer lane's two pixels vertically adjacent (shared tap rows)
#endif
#ifndef IRWS_TAPS_AHEAD
#define IRWS_TAPS_AHEAD 1
#endif
// JOINT (hand-off right after the MFMAs): the wait for every producer's slice-f MFMAs and the wait for the consumers'
// release of the tile buffer poll both counters in one LDS round trip (W(f + 2) is issued as soon as the first is met).
// 1 = the stride-2 kernel only, 2 = every shape.  Same-box A/B (gpurun_out/ab_joint.txt, us per launch): <16,4,2>
// 656-665 -> 632-637, <16,4,1> 642-645 -> 670-673
#ifndef IRWS_JOINT
#define IRWS_JOINT 1
#endif
// PAR = the per-parity W ring hand-off (kernel comment at `par`).  Same-box A/B of the two builds (tools/ab_kern.py,
// three alternating rounds, gpurun_out/r06k/ab_par.txt, us per launch): <16,4,1> 668-676 -> 668-674, <16,4,2> 638-645
// -> 626-637, <8,7,1> 548-554 -> 545-546, CNN 31.80-32.11 -> 31.76-31.87 ms: a small gain, on (-DIRWS_PAR=0: shared)
#ifndef IRWS_PAR
#define IRWS_PAR 1
#endif
// S = depthwise stride.  S = 2 (blocks.5.0, 16x16 -> 8x8, TF-SAME pads pad_t / pad_l): the producers expand the
// same input bands; a band's output rows are its 4 stride-2 rows, one pixel a consumer lane (lanes of consumer
// waves 0-3; waves 4-7 only take part in the hand-offs and the squeeze count).
template <int W, int KS, int S>
__global__ void __launch_bounds__(64 * (WS_NP + WS_NC), 1)
    ir_ws_kernel(const bf16_t* __restrict__ x, int N, int H, int cs_mid, const bf16_t* __restrict__ wpw,
                 const float* __restrict__ bpw, const float* __restrict__ wdw, const float* __restrict__ bdw,
                 bf16_t* __restrict__ y, bf16_t* __restrict__ se_mean, unsigned long long* __restrict__ trace,
                 unsigned spin_max, unsigned* __restrict__ err, int pad_t, int pad_l, int fm32, int n_full, int parts) {
  constexpr int par = IRWS_PAR;
  static_assert(S == 1 || (S == 2 && W == 16), "stride 2: the 16-wide maps");
  constexpr int OWS = W / S;                      // output row width
  constexpr int OPB = (WS_BR / S) * OWS;          // output pixels of a full band
  constexpr bool HAND_END = IRWS_HAND_END == 2 ? W == 8 : IRWS_HAND_END, TAPS_AHEAD = IRWS_TAPS_AHEAD;
  constexpr bool JOINT = IRWS_JOINT && !HAND_END && (IRWS_JOINT == 2 || S == 2);
  constexpr int CS = KS * 32;  // input channel stride = expand K
  constexpr int CPP = (CS * 2 + 255) / 256 * 16;
  constexpr int CPR = 2 * CPP;  // 16-byte chunks per LDS x row
  constexpr int XP = CPR * 16;
  constexpr int WT = W + 2;     // tile row (with the zero halo columns)
  constexpr int WS_PXL = WS_BR * W / 64;  // output pixels per consumer lane per slice
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const WsLayout Lg = ws_layout(H, W, CS, cs_mid, S);
  const int NB = (H + WS_BR - 1) / WS_BR, NS = cs_mid / WS_SL, P = H * W;
  const int PO = S == 1 ? P : ((H + 1) / 2) * OWS;  // output pixels of an image (TF-SAME)
  const int PLT = Lg.TROWS * 16;
  char* xs = smem;
  char* tiles = xs + Lg.x_bytes;
  char* wbuf = tiles + Lg.tile_bytes;
  // [3][9 x 32 taps | 32 depthwise bias]: three slots, so slice f + 1's taps can go out at the end of slice f
  // under the tile buffer's own wait (consumers done with slice f - 2), not a later one
  float* wdl = reinterpret_cast<float*>(wbuf + Lg.w_bytes);
  float* bpl = wdl + 3 * 320;  // [2][32] expand bias
  // the squeeze: per channel the sum of the image's SiLU outputs as 32.32 fixed point, added by every consumer
  // wave of every band with an integer LDS atomic (the same bits in any arrival order); per slice index the
  // number of (band, wave) arrivals, whose last one turns the sums into the slice's SE means
  unsigned long long* sq = reinterpret_cast<unsigned long long*>(bpl + 2 * 32);  // [cs_mid]
  unsigned* sq_n = reinterpret_cast<unsigned*>(sq + cs_mid);                      // [NS]
  unsigned* sq_nan = sq_n + cs_mid / WS_SL;  // [NS] a non-finite partial reached the slice's sums: its means are NaN
  // The hand-offs that replace the per-slice barrier, in LDS.  Producer events are shared monotonic counters
  // (one add per producer wave and event): a producer adds slice f + 1's count only after a wait that needed
  // every producer's slice-f add, so "counter >= NP x k" cannot be met by one wave running ahead.  Consumers are
  // not in lockstep with each other (one may consume slice f + 1 while another is still on f), so a shared count
  // could be met that way: their events are one word per consumer wave, and a wait needs every word >= k.
  unsigned* ctr = reinterpret_cast<unsigned*>(smem + Lg.total - 128);
  unsigned* pdone = ctr + 0;   // producers done with slice f's MFMAs: W(f)'s slot and (band end) the x rows free
  unsigned* wrdy = ctr + 1;    // producers whose pieces of W(f) (+ bias) landed
  unsigned* xrdy = ctr + 2;    // producers whose pieces of a band's x rows landed
  unsigned* tfull = ctr + 3;   // producers done writing tile f (and, waves NP-2 / NP-1, taps f landed)
  // set by a wave whose wait timed out (reported through `err`): the squeeze of every slice finalized from then
  // on stores NaN, so the images of this workgroup come out NaN instead of silently wrong
  unsigned* poison = ctr + 4;
  unsigned* tfree = ctr + 8;   // [WS_NC] slices whose tile and taps consumer wave c is done reading

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const bool prod = wave < WS_NP;
  // par (per-parity W ring): a producer's units all have channel tile wave & 1, so even and odd producer waves DMA and
  // read disjoint halves of a slice's expand weights (rows 0-15 / 16-31) and biases; W(f)'s slot-free and W-ready
  // counts are kept per parity (ctr 0 / 5 and 1 / 6) and a wave waits only for the other waves of its parity.  The
  // x band and the tiles stay shared (a band's x rows are free once both parities are past it)
  const int pw = wave & 1;
  unsigned* const pdone_p = par ? (pw ? ctr + 5 : ctr + 0) : pdone;  // this producer's slot-free count
  unsigned* const wrdy_p = par ? (pw ? ctr + 6 : ctr + 1) : wrdy;    // this producer's W-ready count
  const unsigned NPC = par ? WS_NP / 2 : WS_NP;                        // waves behind each of those counts
  // Work units, dealt round-robin over the workgroups: images 0 .. n_full - 1 whole, then the tail images cut into
  // `parts` slice ranges each (launch_ir_ws: 1920 images on 256 CUs were 7 or 8 images a workgroup, 6 % of the
  // launch idle; 1792 whole + 128 halves are 7.5 each).  Every slice of an image still runs all its bands in one
  // workgroup, so its squeeze stays in that workgroup's LDS.
  const int n_units = n_full + (N - n_full) * parts;
  struct Unit {
    int img, lo, hi;  // image and slice range [lo, hi)
  };
  auto unit_of = [&](int u) {
    if (u < n_full) return Unit{u, 0, NS};
    const int q = u - n_full, pt = q % parts;
    return Unit{n_full + q / parts, pt * NS / parts, (pt + 1) * NS / parts};
  };
  int T = 0;
  for (int u = blockIdx.x; u < n_units; u += gridDim.x) {
    const Unit un = unit_of(u);
    T += NB * (un.hi - un.lo);
  }

  auto TR = [&](int i, int k) {
#ifdef IRWS_TRACE
    if (trace && blockIdx.x == 0 && i < 64) {  // every wave of workgroup 0: slot = wave within its role
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (lane == 0) trace[((i * 2 + (wave >= WS_NP)) * 16 + k) * 64 + (wave & 7)] = t;
    }
#else
    (void)i; (void)k; (void)trace;
#endif
  };
  // (image, band, slice) of a flat step, advanced incrementally (a division only at a unit's end); lo / hi: the
  // unit's slice range, u: the unit
  struct Step {
    int img, band, sl, lo, hi, u;
  };
  auto first_step = [&](int u) {
    const Unit un = unit_of(u);
    return Step{un.img, 0, un.lo, un.lo, un.hi, u};
  };
  auto next_step = [&](Step d) {
    if (++d.sl == d.hi) {
      d.sl = d.lo;
      if (++d.band == NB) d = first_step(d.u + (int)gridDim.x);
    }
    return d;
  };

  if (tid < 32) ctr[tid] = 0u;  // ordered before any use by the kernel's one barrier
  for (int i = tid; i < cs_mid; i += 64 * (WS_NP + WS_NC)) sq[i] = 0ull;
  for (int i = tid; i < 2 * NS; i += 64 * (WS_NP + WS_NC)) sq_n[i] = 0u;  // counts and NaN flags
  // the tiles' halo columns are zero for good (the producers write only interior columns)
  for (int i = tid; i < 2 * 8 * Lg.TROWS; i += 64 * (WS_NP + WS_NC)) {
    const int pl = i / Lg.TROWS, r = i - pl * Lg.TROWS, c = r % WT;
    if (c == 0 || c == WT - 1) *reinterpret_cast<float4*>(tiles + pl * PLT + r * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // counter wait: one lane polls (ds_read + lgkmcnt(0), which also retires this wave's own LDS ops), bounded by
  // spin_max polls; a timeout is reported and poisons the workgroup's squeeze (a wrong hand-off, never a hang)
  auto wait_ge = [&](const unsigned* c, unsigned target) {
    const uint32_t a = (uint32_t)(uintptr_t)c;
    for (unsigned n = 0; n < spin_max; ++n) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
      if (__builtin_amdgcn_readfirstlane(v) >= target) return;
      __builtin_amdgcn_s_sleep(1);
    }
    report_async(err, M2S_ASYNC_WS, lane);
    if (lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)poison), "v"(1u) : "memory");
  };
  // per-consumer words: lanes 0..WS_NC-1 read one word each; done when every word >= target
  auto wait_all = [&](const unsigned* words, unsigned target) {
    const uint32_t a = (uint32_t)(uintptr_t)(words + (lane < WS_NC ? lane : 0));
    for (unsigned n = 0; n < spin_max; ++n) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
      if (__builtin_amdgcn_ballot_w64(lane < WS_NC && v < target) == 0) return;
      __builtin_amdgcn_s_sleep(1);
    }
    report_async(err, M2S_ASYNC_WS, lane);
    if (lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)poison), "v"(1u) : "memory");
  };
  // count this wave in: its LDS writes retire first (lgkmcnt(0)); LDS-DMA data is covered by the caller's vmcnt
  auto bump = [&](unsigned* c) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"((uint32_t)(uintptr_t)c), "v"(1u) : "memory");
  };

  // ---- producer pieces -----------------------------------------------------------------------
  auto issue_w = [&](int f, Step d) {  // the slice's expand weights (4 * KS DMA pieces) + expand bias
    const int sl = d.sl;
    char* base = wbuf + (f & 1) * KS * 4096;
    int ln = lane;  // rebuilt per call (asm barrier): hoisted lane offsets cost registers the consumers need
    asm volatile("" : "+v"(ln));
    if (par ? (wave < 2 && ln < 4) : (wave == 0 && ln < 8))  // (par: each parity's first wave its 16 biases)
      dma16(bpw + (sl * WS_SL + (par ? 16 * wave : 0) + 4 * ln), lds_addr(bpl + (f & 1) * 32 + (par ? 16 * wave : 0)));
    const int q = (ln & 3) ^ swz_f((ln >> 4) & 3);
    for (int j = wave; j < 4 * KS; j += WS_NP) {
      const int ks = j >> 2, plane = (j >> 1) & 1, half = j & 1;
      const int row = sl * WS_SL + half * 16 + (ln >> 2);
      dma16(wpw + (row * CS * 2 + plane * CS + ks * 32 + q * 8), lds_addr(base + ks * 4096 + plane * 2048 + half * 1024));
    }
  };
  auto issue_wd = [&](int f, Step d) {  // the slice's depthwise taps [9][32] + bias: 80 lanes of 16 B
    const int c0 = d.sl * WS_SL;
    float* dst = wdl + (f % 3) * 320;
    // the lane's source offset is rebuilt here each time (asm barrier): hoisted out of the slice loop
    // it became two 64-bit pointers spilled to scratch, and their reload's vmcnt wait drained the
    // weight DMA in flight
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if (wave == WS_NP - 2) {
      dma16(wdw + ((ln >> 3) * cs_mid + c0 + 4 * (ln & 7)), lds_addr(dst));
    } else if (wave == WS_NP - 1 && ln < 16) {
      const float* src = ln < 8 ? wdw + (8 * cs_mid + c0 + 4 * ln) : bdw + (c0 + 4 * (ln - 8));
      dma16(src, lds_addr(dst + 256));
    }
  };
  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_ws_zero;
  asm volatile("" : "+s"(zpage));
  auto issue_x = [&](int img, int band) {  // input rows of the band (+ halo rows), swizzled
    const int r0 = band * WS_BR, xr0 = max(r0 - 1, 0), xr1 = min(r0 + WS_BR + 1, H);
    const int ninstr = (xr1 - xr0) * W * CPR / 64;
    const bf16_t* xi = x + ((size_t)img * P + (size_t)xr0 * W) * CS * 2;
    for (int j = wave; j < ninstr; j += WS_NP) {
      const int id = j * 64 + lane, r = id / CPR, p = id - r * CPR;
      const int L = (p & ~15) | ((p & 15) ^ hx_of(r));
      const int plane = L / CPP, k8 = L - plane * CPP;
      const void* src = k8 * 8 < CS ? static_cast<const void*>(xi + (size_t)r * CS * 2 + plane * CS + k8 * 8)
                                    : zpage;
      dma16(src, lds_addr(xs + j * 1024));
    }
  };
  // W ring (two slots): a producer wave counts itself done with W(f)'s slot right after its MFMAs of slice f
  // (pdone, no wait there).  At the end of slice f, its epilogue stored, it waits for its own W(f + 1) pieces
  // (issued a slice earlier: landed) and counts them in (wrdy), then waits until every producer is done with
  // slice f (by then normally true: the wait is where the slowest wave's MFMAs have long ended, not right
  // after this wave's own) and DMAs its pieces of W(f + 2) into W(f)'s slot.  Slice f + 1 starts once wrdy
  // says W(f + 1) is complete.  (Waiting for pdone right after the MFMAs put the slowest wave's MFMA tail and
  // the hand-off latency, ~800 cycles a slice, on every producer's critical path; in-kernel stamps r05k.)
  const bool tap_wave = wave >= WS_NP - 2;  // issue_wd's two waves
  const int npw = (wave < 4 * KS ? (4 * KS - 1 - wave) / WS_NP + 1 : 0) + ((par ? wave < 2 : wave == 0) ? 1 : 0);  // W pieces a slice
  // (JOINT) every producer done with slice f's MFMAs -> W(f + 2) issued; every consumer done with slice f - 2 -> return.
  // One lane polls pdone and lanes 0..WS_NC-1 the consumer words, one ds_read pair and one lgkmcnt wait a poll
  auto wait_pd_tf = [&](int f, Step d2) {
    const unsigned pd_t = f + 1 < T ? NPC * (unsigned)(f + 1) : 0u, tf_t = f >= 2 ? (unsigned)(f - 1) : 0u;
    bool wdone = !(f + 2 < T);
    const uint32_t ap = (uint32_t)(uintptr_t)pdone_p, at = (uint32_t)(uintptr_t)(tfree + (lane < WS_NC ? lane : 0));
    for (unsigned n = 0; n < spin_max; ++n) {
      unsigned vp, vt;
      asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)" : "=&v"(vp), "=&v"(vt) : "v"(ap), "v"(at) : "memory");
      const bool pok = __builtin_amdgcn_readfirstlane(vp) >= pd_t;
      const bool tok = __builtin_amdgcn_ballot_w64(lane < WS_NC && vt < tf_t) == 0;
      if (pok && !wdone) {
        TR(f, 14);
        issue_w(f + 2, d2);
        wdone = true;
      }
      if (pok && tok) return;
      __builtin_amdgcn_s_sleep(1);
    }
    report_async(err, M2S_ASYNC_WS, lane);
    if (lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)poison), "v"(1u) : "memory");
    if (!wdone) issue_w(f + 2, d2);
  };
  auto after_mfma = [&](int f, Step d2) {
    if (HAND_END) {
      bump(pdone_p);
    } else {  // W(f + 1) of this wave landed (younger: only the tap waves' slice-f taps), then every producer's
      if (tap_wave) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else wait_vm0();
      TR(f, 13);
      bump(pdone_p);
      if (JOINT) {
        wait_pd_tf(f, d2);
        return;
      }
      if (f + 1 < T) wait_ge(pdone_p, NPC * (unsigned)(f + 1));
      TR(f, 14);
      if (f + 2 < T) issue_w(f + 2, d2);
    }
  };
  auto produce = [&](int f, Step d, Step d2) {
    const int r0 = d.band * WS_BR, br = min(WS_BR, H - r0), xr0 = max(r0 - 1, 0), xr1 = min(r0 + WS_BR + 1, H);
    const int PB = (xr1 - xr0) * W, nunit = 2 * ((PB + 15) / 16);
    const char* wb = wbuf + (f & 1) * KS * 4096;
    const int hxl = hx_of(r16);
    // units = (16-position subtile t, 16-channel tile nt), dealt round-robin over the producer waves
    // (9 subtiles x 2 on a 16x16 band: at most 3 units = 36 MFMAs a wave).  The wave's unit count NU is
    // uniform, so each count gets a straight-line body: every fragment of a k-step is read at once and
    // the next k-step's reads are issued before this one's MFMAs (with a runtime `u < nunit` test per
    // unit the loads were issued and waited for unit by unit: the MFMA phase took ~2k cycles a slice
    // for 12-36 MFMAs, in-kernel stamps gpurun_out t4a)
    static_assert(WS_NP % 2 == 0, "unit -> channel tile");
    // every unit of a wave has the same 16-channel tile (u & 1 == wave & 1: WS_NP is even), so the
    // weight fragments are read once per k-step, not once per unit
    const int wrow = (wave & 1) * 16 + r16;
    const int wo = wrow * 64 + ((g ^ swz_f((wrow >> 2) & 3)) << 4);
    const int nu = nunit > wave ? (nunit - wave + WS_NP - 1) / WS_NP : 0;
    char* tb = tiles + (f & 1) * 8 * PLT;
    const int trow0 = xr0 - r0 + 1;  // tile row of x row 0
    // from LDS (staged with the weights): a global load here would make hipcc drain the DMA
    const float4 bb = *reinterpret_cast<const float4*>(bpl + (f & 1) * 32 + (wave & 1) * 16 + 4 * g);
    auto units = [&](auto nuc) {
      constexpr int NU = decltype(nuc)::value;
      f32x4 acc[NU];
#pragma unroll
      for (int k = 0; k < NU; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      // k-steps in flight: the LDS round trip under the consumers' tile reads is several hundred cycles, so a wave
      // with one unit (8x8: 21 MFMAs a slice) keeps 3 k-steps of reads ahead, with 2 units 2, with 3 units 1
      constexpr int D = !IRWS_PF_DEEP ? 2 : NU == 1 ? 4 : NU == 2 ? 3 : 2;
      bf16x8 ah[D], al[D], bh[D][NU], bl[D][NU];
      auto load = [&](int ks, int bsel) {
        const int Lh = ks * 4 + g, Ll = CPP + ks * 4 + g;
        const int ph = ((Lh & ~15) | ((Lh & 15) ^ hxl)) << 4, pl = ((Ll & ~15) | ((Ll & 15) ^ hxl)) << 4;
        ah[bsel] = *reinterpret_cast<const bf16x8*>(wb + ks * 4096 + wo);
        al[bsel] = *reinterpret_cast<const bf16x8*>(wb + ks * 4096 + 2048 + wo);
#pragma unroll
        for (int k = 0; k < NU; ++k) {
          const char* xr = xs + (((wave + WS_NP * k) >> 1) * 16 + r16) * XP;
          bh[bsel][k] = *reinterpret_cast<const bf16x8*>(xr + ph);
          bl[bsel][k] = *reinterpret_cast<const bf16x8*>(xr + pl);
        }
      };
#pragma unroll
      for (int ks = 0; ks < D - 1 && ks < KS; ++ks) load(ks, ks);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int c = ks % D;
        if (ks + D - 1 < KS) load(ks + D - 1, (ks + D - 1) % D);
        // keep the reads where they are: left to itself the scheduler sinks each one to its MFMA (least registers)
        // and every k-step waits out a full LDS round trip
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < NU; ++k) {
          acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[c], bh[c][k], acc[k], 0, 0, 0);
          acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c], bl[c][k], acc[k], 0, 0, 0);
          acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c], bh[c][k], acc[k], 0, 0, 0);
        }
      }
      TR(f, 6);
      after_mfma(f, d2);
      TR(f, 8);
      if (!JOINT && f >= 2) wait_all(tfree, (unsigned)(f - 1));  // every consumer is done with tile f - 2 (same buffer)
      TR(f, 9);
      // bias + SiLU -> tile[f % 2]; lane holds channels 4g..4g+3 (of 16-channel tile nt) of position r16
#pragma unroll
      for (int k = 0; k < NU; ++k) {
        const int u = wave + WS_NP * k, nt = u & 1, m = (u >> 1) * 16 + r16;
        if (m < PB) {
          const int ti = (m / W + trow0) * WT + (m % W) + 1;
          *reinterpret_cast<float4*>(tb + (nt * 4 + g) * PLT + ti * 16) =
              make_float4(silu(acc[k][0] + bb.x), silu(acc[k][1] + bb.y), silu(acc[k][2] + bb.z), silu(acc[k][3] + bb.w));
        }
      }
    };
    static_assert(WS_UMAX == 3, "unit counts 1..3");
    if (nu == 3) units(std::integral_constant<int, 3>());
    else if (nu == 2) units(std::integral_constant<int, 2>());
    else if (nu == 1) units(std::integral_constant<int, 1>());
    else {
      after_mfma(f, d2);
      if (!JOINT && f >= 2) wait_all(tfree, (unsigned)(f - 1));
    }
    // halo rows outside the image (above the first band, below the last) hold zeros
    if (tid < 8 * W) {
      const int pl = tid / W, c = tid - pl * W;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r0 == 0) *reinterpret_cast<float4*>(tb + pl * PLT + (c + 1) * 16) = z;
      if (r0 + br == H) *reinterpret_cast<float4*>(tb + pl * PLT + ((br + 1) * WT + c + 1) * 16) = z;
    }
  };

  // ---- consumer pieces -----------------------------------------------------------------------
  const int ct = tid - 64 * WS_NP, cw = ct >> 6, cg = ct & 7, cpl = ct >> 3;
  // A consumer lane's pixels are cpl + 64 k of the band (k < WS_PXL): in the tile they sit 64 / W rows
  // apart (a compile-time offset from the first), and in the SE GEMM's interleaved operand layout
  // (il_st4: position p, channel c -> element p * 2 cs + 2 (c & ~31) + (c & 31)) 64 positions apart.
  // The byte offset of a store is one 24-bit multiply-add on the band's scalar position base; the
  // per-pixel 64-bit position arithmetic (two v_mul_lo_u32 a pixel) was a fifth of the consumer VALU.
  // S = 2: pixel lane cpl = 4 k + i takes output pixel (oy, ox) of the band's 4 x 8, row 2 (k & 1) + (i & 1), column
  // (c_(i & 1) + 4 (i >> 1)) & 7 with c_0 = (k >> 1) + 4 (k & 1), c_1 = c_0 + 6: the four pixel lanes of a
  // ds_read_b128 lane group then sit at 16-byte offsets (c, c, c + 8, c + 8) mod 16, which with the planes an odd
  // number (mod 16) of units apart fill all 16 bank quads in both lane-group patterns (stride-2 columns in pixel order were 2-way conflicted: 0.36 conflict
  // cycles per LDS instruction, profiles/r05fin2_sq_mfma.txt).  Its window's top-left tile row and column are
  // 2 oy - pad_t + 1 and 2 ox - pad_l + 1 (tile row = input row - r0 + 1, column = input column + 1).
  int cpo = cpl, toff0 = ((cpl / W) * WT + cpl % W) * 16;
  if constexpr (S == 2) {
    const int k = cpl >> 2, i = cpl & 3, c0 = (k >> 1) + 4 * (k & 1);
    const int oy = 2 * (k & 1) + (i & 1), ox = (((i & 1) ? c0 + 6 : c0) + 4 * (i >> 1)) & 7;
    cpo = oy * OWS + ox;
    toff0 = ((2 * oy - pad_t + 1) * WT + 2 * ox - pad_l + 1) * 16;
  }
  auto consume = [&](int f, Step d) {
    const int c0 = d.sl * WS_SL, r0 = d.band * WS_BR, br = min(WS_BR, H - r0);
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    TR(f, 4);
    const uint32_t pbase = (uint32_t)(d.img * PO + (r0 / S) * OWS);  // uniform
    // fm32: plain fp32 rows (channel c at byte 4 c of its position), else the interleaved split layout
    const uint32_t yoffb = __builtin_amdgcn_readfirstlane(4u * (uint32_t)c0) + (fm32 ? 16u : 8u) * (uint32_t)cg +
                           pbase * (4u * (uint32_t)cs_mid);  // launch_ir_ws: < 2^32
    const uint32_t yoff0 = yoffb + (uint32_t)cpo * (4u * (uint32_t)cs_mid);
    // lane = (4-channel plane cg, pixels cpl + 64 k): the plane's 9 taps stay in registers
    const float* wd = wdl + (f % 3) * 320 + 4 * cg;
    float w[9][4], b[4];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 v = *reinterpret_cast<const float4*>(wd + t * 32);
      w[t][0] = v.x; w[t][1] = v.y; w[t][2] = v.z; w[t][3] = v.w;
    }
    {
      const float4 v = *reinterpret_cast<const float4*>(wd + 288);
      b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
    }
    const char* tpl = tiles + (f & 1) * 8 * PLT + cg * PLT;
    auto pixel = [&](int k) {
      const char* tp = tpl + toff0 + k * (64 / W) * WT * 16;
      float a[4] = {b[0], b[1], b[2], b[3]};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4 u = *reinterpret_cast<const float4*>(tp + ((t / 3) * WT + (t % 3)) * 16);
        a[0] += w[t][0] * u.x;
        a[1] += w[t][1] * u.y;
        a[2] += w[t][2] * u.z;
        a[3] += w[t][3] * u.w;
        if (t == 5) asm volatile("" ::: "memory");  // two tap rows of loads in flight (registers)
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = silu(a[j]);
        s[j] += a[j];
      }
      char* u = reinterpret_cast<char*>(y) + (yoff0 + (uint32_t)k * 256u * (uint32_t)cs_mid);
      if (fm32) {
        *reinterpret_cast<float4*>(u) = make_float4(a[0], a[1], a[2], a[3]);
      } else {
        uint2 hi, lo;  // the SE GEMM's interleaved operand: [hi 32 | lo 32] per 32-channel group
        split4(a, hi, lo);
        *reinterpret_cast<uint2*>(u) = hi;
        *reinterpret_cast<uint2*>(u + 64) = lo;
      }
    };
    // W = 16, full band: the lane's two pixels are vertically adjacent, (2 a, c) and (2 a + 1, c) for cpl =
    // 16 a + c, so their windows share two tap rows: 12 tile reads for both instead of 18
    auto pixel_pair = [&]() {
      const int pa = cpl >> 4, pc = cpl & 15;
      const char* tp = tpl + ((2 * pa) * WT + pc) * 16;
      float a0[4] = {b[0], b[1], b[2], b[3]}, a1[4] = {b[0], b[1], b[2], b[3]};
#pragma unroll
      for (int ry = 0; ry < 4; ++ry) {
#pragma unroll
        for (int rx = 0; rx < 3; ++rx) {
          const float4 u = *reinterpret_cast<const float4*>(tp + (ry * WT + rx) * 16);
          if (ry < 3) {
            const int t = ry * 3 + rx;
            a0[0] += w[t][0] * u.x; a0[1] += w[t][1] * u.y; a0[2] += w[t][2] * u.z; a0[3] += w[t][3] * u.w;
          }
          if (ry > 0) {
            const int t = (ry - 1) * 3 + rx;
            a1[0] += w[t][0] * u.x; a1[1] += w[t][1] * u.y; a1[2] += w[t][2] * u.z; a1[3] += w[t][3] * u.w;
          }
        }
        if (ry == 1) asm volatile("" ::: "memory");  // two rows of loads in flight (registers)
      }
      const uint32_t po = (uint32_t)(32 * pa + pc);  // band position of the upper pixel
      auto out = [&](float* a, uint32_t pos) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = silu(a[j]);
          s[j] += a[j];
        }
        char* u = reinterpret_cast<char*>(y) + (yoffb + pos * (4u * (uint32_t)cs_mid));
        if (fm32) {
          *reinterpret_cast<float4*>(u) = make_float4(a[0], a[1], a[2], a[3]);
        } else {
          uint2 hi, lo;
          split4(a, hi, lo);
          *reinterpret_cast<uint2*>(u) = hi;
          *reinterpret_cast<uint2*>(u + 64) = lo;
        }
      };
      out(a0, po);
      out(a1, po + 16u);
    };
    if constexpr (S == 2) {
      if (cpl < OPB) pixel(0);  // (the bands of a 16-row map are full)
    } else if (IRWS_PAIR && W == 16 && br == WS_BR) {
      pixel_pair();
    } else if (br == WS_BR) {  // a full band: every lane's pixels exist, so their chains interleave
#pragma unroll
      for (int k = 0; k < WS_PXL; ++k) pixel(k);
    } else {
#pragma unroll
      for (int k = 0; k < WS_PXL; ++k)
        if (cpl + 64 * k < br * W) pixel(k);
    }
    TR(f, 5);
    bump(tfree + cw);  // every tile and tap read of slice f returned: the producers may refill both buffers
    TR(f, 10);
    // squeeze partials: the wave's 8 pixel lanes of each plane (lane bits 3..5): a DPP row rotation
    // inside each 16-lane row, then gfx950's row / half swaps (v_permlane16_swap, v_permlane32_swap: VALU,
    // no LDS round trip, where two ds_bpermute shuffles were); one row of 32 channels per wave
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, s[j]), 0x128, 0xF, 0xF, false));
      const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(s[j]), __float_as_uint(s[j]), false, false);
      s[j] = __uint_as_float(q[0]) + __uint_as_float(q[1]);
      const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(s[j]), __float_as_uint(s[j]), false, false);
      s[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    TR(f, 11);
    // lane L < 8 holds the wave's partial sums of plane L (channels c0 + 4 L ..): add them to the image's fixed-point
    // sums, then count this (band, wave) in; the last of the NB x WS_NC arrivals writes the slice's SE means and
    // clears the sums and the count for the next image (no wait on the other consumers: the atomics are the sync)
    // (every lane with lane & 7 == L holds them after the shuffles: lane L + 8 j < 32 takes sum j, so one
    // conversion and one atomic a lane cover the slice's 32 channels)
    const int sc = 4 * (lane & 7) + ((lane >> 3) & 3);  // the lane's channel in the slice
    {
      const int j = (lane >> 3) & 3;
      const float v = j == 0 ? s[0] : j == 1 ? s[1] : j == 2 ? s[2] : s[3];
      // a non-finite partial (an upstream NaN, or |v| >= 2^31 where the 32.32 conversion is undefined) cannot be
      // carried in fixed point: it flags the image's slice, whose SE means the last arriver stores as NaN (as the
      // float sum propagated it)
      if (lane < WS_SL && !(__builtin_fabsf(v) < 2147483648.0f))
        asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(uintptr_t)(sq_nan + d.sl)), "v"(1u) : "memory");
      if (lane < WS_SL)
        __hip_atomic_fetch_add(sq + c0 + sc, (unsigned long long)(long long)(__builtin_fabsf(v) < 2147483648.0f ? v * 4294967296.0f : 0.f),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // the arrival count is release (this wave's sum adds and poison write are ordered before it) and acquire (the last
    // arriver sees every other wave's adds before it reads the sums): the memory model's ordering, not LDS's in-order
    // execution of one wave's operations
    unsigned arrived = 0;
    if (lane == 0) arrived = __hip_atomic_fetch_add(sq_n + d.sl, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__builtin_amdgcn_readfirstlane(arrived) == (unsigned)(NB * WS_NC - 1) && lane < WS_SL) {
      const unsigned long long t = __hip_atomic_exchange(sq + c0 + sc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // 32.32 -> float: integer part (arithmetic high word) + fraction (low word)
      const float m = __fmaf_rn((float)(unsigned)t, 2.3283064365386963e-10f, (float)(int)(t >> 32)) / (float)PO;
      act_st<sp_t>(reinterpret_cast<sp_t*>(se_mean), d.img, cs_mid, c0 + sc, (*poison || sq_nan[d.sl]) ? __builtin_nanf("") : m);
      if (lane == 0) {
        sq_n[d.sl] = 0u;
        sq_nan[d.sl] = 0u;
      }
    }
  };

  // ---- the slice pipeline.  No workgroup barrier per slice: each role runs its own loop and the hand-offs are
  // the LDS counters above.  Producers may run up to two slices ahead of the consumers (two tile / tap buffers);
  // W(f + 2) is DMA'd into W(f)'s slot once every producer finished slice f's MFMAs, x rows of a band once every
  // producer finished the last band's.  Consumers wait only for their tiles (the squeeze is atomic).
  __syncthreads();  // the counters and the tiles' zero halo columns
  if (prod) {
    __builtin_amdgcn_s_setprio(2);
    Step cur = first_step(blockIdx.x);
    if (T > 0) issue_w(0, cur);
    if (T > 1) issue_w(1, next_step(cur));
    if (TAPS_AHEAD && T > 0 && tap_wave) issue_wd(0, cur);
    if (T > 0) {  // W(0) landed (W(1) and the taps may stay in flight)
      wait_vm_le((T > 1 ? npw : 0) + (TAPS_AHEAD && tap_wave ? 1 : 0));
      bump(wrdy_p);
      if (!HAND_END) wait_ge(wrdy_p, NPC);
    }
    static_assert(4 * KS <= 4 * WS_NP, "pieces per wave");
    int bands = 0;
    for (int i = 0; i < T; ++i) {
      const Step nxt = next_step(cur), nxt2 = next_step(nxt);
      TR(i, 0);
      if (cur.sl == cur.lo) {  // a new band: its input rows, once every producer is done with the last band's
        if (i > 0) {  // (both parities: every producer reads the whole band)
          wait_ge(pdone_p, NPC * (unsigned)i);
          if (par) wait_ge(pw ? ctr + 0 : ctr + 5, NPC * (unsigned)i);
        }
        issue_x(cur.img, cur.band);
        wait_vm0();
        bump(xrdy);
        wait_ge(xrdy, (unsigned)(WS_NP * ++bands));
      }
      TR(i, 1);
      if (!TAPS_AHEAD && tap_wave) {  // slice i's taps into taps[i % 3], once every consumer is done with slice i - 3
        if (i >= 3) wait_all(tfree, (unsigned)(i - 2));
        issue_wd(i, cur);
      }
      if (HAND_END) wait_ge(wrdy_p, NPC * (unsigned)(i + 1));  // W(i) complete (this parity's half)
      TR(i, 2);
      produce(i, cur, nxt2);
      if (HAND_END) {
        // W(i + 1) and (tap waves) slice i's taps landed: nothing else of this wave's is in flight
        wait_vm0();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tile stores
        if (lane == 0) {
          asm volatile("ds_add_u32 %0, %1" ::"v"((uint32_t)(uintptr_t)wrdy_p), "v"(1u) : "memory");
          asm volatile("ds_add_u32 %0, %1" ::"v"((uint32_t)(uintptr_t)tfull), "v"(1u) : "memory");
        }
        TR(i, 12);
        const bool nw = i + 2 < T, nt = TAPS_AHEAD && tap_wave && i + 1 < T;
        if (nw || nt) {
          // W(i)'s slot is free once every producer is done with slice i.  Slice i + 1's taps go to taps[(i + 1) % 3],
          // which held slice i - 2's: produce(i) waited for every consumer to be done with that slice before its
          // tile stores.  Both land during slice i + 1
          wait_ge(pdone_p, NPC * (unsigned)(i + 1));
          if (nw) issue_w(i + 2, nxt2);
          if (nt) issue_wd(i + 1, nxt);
        }
      } else {
        if (tap_wave) {  // slice i's taps landed; younger: W(i + 2) (after_mfma) and, ahead, slice i + 1's taps
          const bool nt = TAPS_AHEAD && i + 1 < T;
          if (nt) issue_wd(i + 1, nxt);
          wait_vm_le((i + 2 < T ? npw : 0) + (nt ? 1 : 0));
        }
        bump(tfull);
        TR(i, 12);
      }
      TR(i, 3);
      cur = nxt;
    }
  } else {
    Step cur = first_step(blockIdx.x);
    for (int i = 0; i < T; ++i) {
      wait_ge(tfull, (unsigned)(WS_NP * (i + 1)));  // tile i and taps i
      consume(i, cur);
      TR(i, 7);
      cur = next_step(cur);
    }
  }
}

#ifdef IRWS_TRACE
// Diagnostic build only (-DIRWS_TRACE, M2S_IR_WS_TRACE=1): per-phase s_memtime stamps of workgroup 0's
// first producer and consumer waves for the first slices of each launch, printed to stderr.
static void dump_trace(unsigned long long* tr, hipStream_t s, const char* tag) {
  static int calls = 0;
  if (++calls > 40) return;
  std::vector<unsigned long long> h(64 * 2 * 16 * 64);
  M2S_HIP(hipStreamSynchronize(s));
  M2S_HIP(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
  auto at = [&](int i, int c, int k, int w = 0) { return (long long)h[((i * 2 + c) * 16 + k) * 64 + w]; };
  fprintf(stderr, "TRACE %s:", tag);
  for (int i = 2; i < 12; ++i)
    // producer: band x, W wait, MFMAs, tile-free wait, epilogue + counts, W / taps hand-off;
    // consumer: tile wait, pixels, tfree bump, shuffles, atomics (+ SE mean)
    fprintf(stderr, " [P x %lld wr %lld mfma %lld tf %lld epi %lld hand %lld | C wait %lld px %lld bump %lld shf %lld at %lld]",
            at(i, 0, 1) - at(i, 0, 0), at(i, 0, 2) - at(i, 0, 1), at(i, 0, 6) - at(i, 0, 2), at(i, 0, 9) - at(i, 0, 6),
            at(i, 0, 12) - at(i, 0, 9), at(i, 0, 3) - at(i, 0, 12), at(i, 1, 4) - at(i - 1, 1, 7), at(i, 1, 5) - at(i, 1, 4),
            at(i, 1, 10) - at(i, 1, 5), at(i, 1, 11) - at(i, 1, 10), at(i, 1, 7) - at(i, 1, 11));
  fprintf(stderr, "\n");
  // per producer wave, relative to wave 0's slice start: MFMA start / end / done-count bump
  fprintf(stderr, "TRACEW %s:", tag);
  for (int i = 2; i < 4; ++i) {  // start / MFMA start / MFMA end / tiles free / stored + counted / end
    fprintf(stderr, " [s%d", i);
    for (int w = 0; w < 8; ++w) {
      fprintf(stderr, " w%d", w);
      for (int k : {0, 2, 6, 9, 12, 3}) fprintf(stderr, "%c%lld", k ? '/' : ' ', at(i, 0, k, w) - at(i, 0, 0));
    }
    fprintf(stderr, "]");
  }
  fprintf(stderr, "\n");
  // consumer waves' px start / tfree bump / end of slices i - 2 .. i, relative to producer wave 0's slice i start
  fprintf(stderr, "TRACEC %s:", tag);
  for (int i = 4; i < 7; ++i) {
    fprintf(stderr, " [s%d P0 mfma_end %lld vm0 %lld pdone %lld after %lld tf %lld tfull %lld |", i, at(i, 0, 6) - at(i, 0, 0),
            at(i, 0, 13) - at(i, 0, 0), at(i, 0, 14) - at(i, 0, 0), at(i, 0, 8) - at(i, 0, 0), at(i, 0, 9) - at(i, 0, 0),
            at(i, 0, 12) - at(i, 0, 0));
    for (int j = i - 2; j <= i; ++j) {
      fprintf(stderr, " c%d:", j);
      for (int w = 0; w < 8; ++w)
        fprintf(stderr, " %lld/%lld/%lld", at(j, 1, 4, w) - at(i, 0, 0), at(j, 1, 10, w) - at(i, 0, 0), at(j, 1, 7, w) - at(i, 0, 0));
    }
    fprintf(stderr, "]");
  }
  fprintf(stderr, "\n");
  M2S_HIP(hipMemset(tr, 0, h.size() * 8));
}
#endif

}  // namespace

bool ir_ws_s2_supported(int H, int W, int cs_in, int kp, int cs_mid, int OH, int OW, int pad_t, int pad_l) {
  return H == 16 && W == 16 && OH == 8 && OW == 8 && pad_t >= 0 && pad_t <= 1 && pad_l >= 0 && pad_l <= 1 &&
         ir_ws_supported(H, W, cs_in, kp, cs_mid) && ws_layout(H, W, cs_in, cs_mid, 2).total <= 160 * 1024;
}

bool ir_ws_supported(int H, int W, int cs_in, int kp, int cs_mid) {
  if (!((W == 8 && (kp == 128 || kp == 224)) || (W == 16 && kp == 128)) || H < 1 || H > 64 || cs_in != kp) return false;
  // the atomic squeeze keeps one sums / count set per workgroup, reused across bands and images: consumer waves
  // may run two slices apart, so a slice index must not recur within three steps (NS = cs_mid / 32 >= 3)
  if (cs_mid % WS_SL != 0 || cs_mid < 3 * WS_SL) return false;
  const WsLayout L = ws_layout(H, W, cs_in, cs_mid);
  const int cpr = 2 * ws_cpp(cs_in);
  return L.total <= 160 * 1024 && (L.XR * W * cpr) % 64 == 0 && L.XR * W * cpr / 64 / WS_NP + 1 <= 60 &&
         2 * ((L.XR * W + 15) / 16) <= WS_NP * WS_UMAX;
}

void launch_ir_ws(const void* x, int N, int H, int W, int cs_in, int kp, int cs_mid, const void* wpw, const float* bpw,
                  const float* wdw, const float* bdw, void* y, void* se_mean, double flops, double bytes,
                  hipStream_t s, AsyncReport rep, int stride, int OH, int OW, int pad_t, int pad_l, double spill,
                  bool fm32) {
  M2S_CHECK(stride == 1 ? ir_ws_supported(H, W, cs_in, kp, cs_mid)
                        : stride == 2 && ir_ws_s2_supported(H, W, cs_in, kp, cs_mid, OH, OW, pad_t, pad_l),
            "ir_ws: unsupported shape");
  M2S_CHECK(N > 0, "ir_ws: no images");
  M2S_CHECK((double)N * H * W * cs_mid * 4.0 < 4294967296.0, "ir_ws: output map too large for 32-bit offsets");
  const WsLayout L = ws_layout(H, W, cs_in, cs_mid, stride);
  const int n_cu = device_cus();
  const dim3 grid(std::min(N, n_cu));
  // tail balancing (kernel comment): whole images up to a multiple of the grid, the rest in `parts` slice ranges,
  // parts ~ grid / tail images so the units come to a whole number of rounds; a range keeps >= 3 slices (the
  // squeeze's reuse distance; each range of a band reloads the band's input rows)
  const int G = (int)grid.x, NSl = cs_mid / WS_SL;
  const int n_full = N / G * G, rem = N - n_full;
  int parts = rem > 0 ? std::max(1, (G + rem / 2) / rem) : 1;
  parts = std::max(1, std::min(parts, NSl / 3));
  if (const char* e = getenv("M2S_IRWS_PARTS"))  // A/B: n = n ranges (1 = no tail split), 0 = the rule above
    if (atoi(e) > 0) parts = std::min(atoi(e), std::max(1, NSl / 3));
#ifdef IRWS_TRACE
  static unsigned long long* tr = [] {
    unsigned long long* p = nullptr;
    if (getenv("M2S_IR_WS_TRACE")) M2S_HIP(hipMalloc(&p, 64 * 2 * 16 * 64 * 8));
    return p;
  }();
#define M2S_IRWS_DUMP(tag) \
  if (tr) dump_trace(tr, s, tag);
#else
  unsigned long long* tr = nullptr;
#define M2S_IRWS_DUMP(tag)
#endif
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  const bf16_t* wb = static_cast<const bf16_t*>(wpw);
  bf16_t* yb = static_cast<bf16_t*>(y);
  bf16_t* mb = static_cast<bf16_t*>(se_mean);
#define M2S_IRWS(W_, KS_, S_, NAME_)                                                                    \
  if (W == W_ && kp == KS_ * 32 && stride == S_) {                                                      \
    allow_lds(reinterpret_cast<const void*>(&ir_ws_kernel<W_, KS_, S_>));                             \
    ProfScope ps(NAME_, flops, bytes, s, spill);                                                        \
    hipLaunchKernelGGL((ir_ws_kernel<W_, KS_, S_>), grid, dim3(64 * (WS_NP + WS_NC)), L.total, s, xb, N, H, cs_mid, wb, \
                       bpw, wdw, bdw, yb, mb, tr, rep.spin_max, rep.err, pad_t, pad_l, fm32 ? 1 : 0, n_full, parts); \
    M2S_IRWS_DUMP(NAME_)                                                                                \
    M2S_HIP(hipGetLastError());                                                                         \
    return;                                                                                             \
  }
  // (the launch log's names are rocprof's symbols, so the event and PMC records of a kernel share a key)
  M2S_IRWS(8, 4, 1, "ir_ws_kernel<8, 4, 1>") M2S_IRWS(8, 7, 1, "ir_ws_kernel<8, 7, 1>")
  M2S_IRWS(16, 4, 1, "ir_ws_kernel<16, 4, 1>") M2S_IRWS(16, 4, 2, "ir_ws_kernel<16, 4, 2>")
#undef M2S_IRWS
#undef M2S_IRWS_DUMP
  M2S_CHECK(false, "ir_ws: no variant for this shape");
}

}  // namespace m2s
