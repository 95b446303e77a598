// Persistent BiLSTM recurrence: one launch for all T steps of both directions
// (nn.LSTM(208, 640, bidirectional) in BiLSTMSumMerge, mri_acoustic_model.py:57-71; gate order
// i, f, g, o; c' = f*c + i*g, h' = o*tanh(c'); h0 = c0 = 0).
//
// Layout.  Workgroup (dir, ug) owns hidden units [8 ug, 8 ug + 8) of one direction: the 32 W_hh
// rows of their four gates stay in VGPRs for the whole launch (each of the 4 waves holds a 160-wide
// K slice: 80 floats per lane as v_mfma_f32_32x32x2_f32 A fragments), so W_hh (6.5 MB per
// direction, fp32) is read from HBM once per launch instead of once per step.  H = 640 gives
// 2 x 80 = 160 co-resident workgroups (one per CU).
// Per step: every wave loads h_{t-1} for its K slice and 32 sequences per B tile straight into B
// fragments (lane = (k half, sequence); the K order inside the slice is permuted so a lane reads 80
// consecutive floats), runs 80 MFMAs per B tile, the four K-slice partials are summed in LDS, and
// 256 threads apply the cell update for (unit, sequence) pairs.  c stays in LDS; h_t goes to `hs`
// (the layer output) and is published to the direction's other workgroups by a release/acquire
// counter barrier (cdna_hip_programming.md Guideline 16): plain stores -> vmcnt(0) -> barrier ->
// agent release fence -> atomic add; consumers poll relaxed, then one agent acquire fence.
// (spin_max == 0 is fault injection: the first wait times out whatever the tags say, so a test of
// the report does not depend on how late a peer happens to publish.)
// Spins are bounded: on timeout the workgroup sets the error word, poisons its remaining outputs
// with NaN and leaves, so the grid always drains; the engine's pinned host flag (`err_host`) is set
// too, and the C ABI reports it (m2s_acoustic_status; the next forward fails with M2S_E_INTERNAL).
// Products are exact fp32 (MFMA f32); only the summation order differs from torch.  The gate
// activations are the rcp-based sigmoid (v_exp + v_rcp, 1 ulp each) and tanh(x) = 2 sigmoid(2x) - 1
// (absolute error ~1e-7): the cell update is on every step's critical path, and libm's expf + IEEE
// divide and tanhf cost 7.51 against 7.18 us per recurrent step at 8 x 1000 (gpurun_out lstmfa0/1).
#include <algorithm>
#include <cstdlib>

#include "kernels.hpp"

namespace m2s {
namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

__device__ __forceinline__ float lstm_sig(float x) { return sigmoidf_(x); }
__device__ __forceinline__ float lstm_tanh(float x) { return 2.f * sigmoidf_(2.f * x) - 1.f; }

constexpr int LP_H = 640;          // hidden size this kernel is built for
constexpr int LP_U = 8;            // units per workgroup (32 gate rows = one MFMA M tile)
constexpr int LP_KW = LP_H / 4;    // K slice per wave
constexpr int LP_KH = LP_KW / 2;   // floats per lane per B tile (k half = lane / 32)
constexpr int LP_BT = 2;           // 32-sequence B tiles per pass
constexpr int LP_BMAX = 64;        // sequences per launch (c in LDS); larger batches: several launches

struct LstmSync {
  unsigned arrive[2];  // per-direction monotonic arrival counters
  unsigned err;        // set on a barrier timeout
};

__global__ void __launch_bounds__(256, 1) lstm_persistent_kernel(const float* __restrict__ pre,
                                                                 const float* __restrict__ whh, float* hs,
                                                                 int Btot, int b0, int B, int T, LstmSync* sync,
                                                                 unsigned spin_max, unsigned* err_host) {
  __shared__ float red[4][LP_BT][32][33];
  __shared__ float cst[LP_U][LP_BMAX];
  __shared__ int abort_flag;
  const int H = LP_H;
  const int dir = blockIdx.x / (H / LP_U), ug = blockIdx.x - dir * (H / LP_U);
  const int nwg = H / LP_U;  // workgroups per direction
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kk = lane >> 5, l32 = lane & 31;
  const int kbase = wave * LP_KW + kk * LP_KH;  // this lane's 80 consecutive k
  // sequences [b0, b0 + B) of the (Btot, T, ...) tensors
  float* hsd = hs + (size_t)dir * Btot * T * H + (size_t)b0 * T * H;
  pre += (size_t)b0 * T * 8 * H;

  // ---- W_hh rows of this workgroup -> A fragments (resident for the launch) --------------------
  float wa[LP_KH];
  {
    const int r = l32, g = r / LP_U, u = ug * LP_U + (r % LP_U);
    const float* wr = whh + ((size_t)dir * 4 * H + (size_t)g * H + u) * H + kbase;
#pragma unroll
    for (int s = 0; s < LP_KH; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(wr + s);
      wa[s] = v.x;
      wa[s + 1] = v.y;
      wa[s + 2] = v.z;
      wa[s + 3] = v.w;
    }
  }
  for (int i = tid; i < LP_U * LP_BMAX; i += 256) (&cst[0][0])[i] = 0.f;
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  unsigned* arrive = &sync->arrive[dir];
  const int nbt = (B + 31) / 32;
  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    const int tprev = dir == 0 ? t - 1 : t + 1;
    // this thread's gate pre-activations for the cell update (pairs p = tid + 256 k; B <= LP_BMAX = 64, so
    // one B-tile pass), fetched before the barrier wait so their latency hides under it
    float prf[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 256 * k, u = p % LP_U, b = p / LP_U;
      const float* pr = pre + ((size_t)b * T + t) * 8 * H + (size_t)dir * 4 * H + ug * LP_U + u;
#pragma unroll
      for (int q = 0; q < 4; ++q) prf[k][q] = b < B ? pr[q * H] : 0.f;
    }
    if (step > 0) {
      // ---- wait until every workgroup of this direction published h_{t-1} -----------------
      if (tid == 0) {
        const unsigned target = (unsigned)step * nwg;
        unsigned spins = 0;
        while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target || spin_max == 0) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_max ||
              __hip_atomic_load(&sync->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            __hip_atomic_store(&sync->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            abort_flag = 1;
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (abort_flag) {  // barrier timed out: flag the host, poison the remaining outputs, leave
        if (tid == 0 && err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int st = step; st < T; ++st) {
          const int tt = dir == 0 ? st : T - 1 - st;
          for (int p = tid; p < LP_U * B; p += 256)
            hsd[((size_t)(p / LP_U) * T + tt) * H + ug * LP_U + p % LP_U] = __builtin_nanf("");
        }
        return;
      }
    }
    for (int bt0 = 0; bt0 < nbt; bt0 += LP_BT) {
      f32x16 acc[LP_BT];
#pragma unroll
      for (int j = 0; j < LP_BT; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
      if (step > 0) {
        float hb[LP_BT][LP_KH];
#pragma unroll
        for (int j = 0; j < LP_BT; ++j) {
          const int b = (bt0 + j) * 32 + l32;
          const float* hr = hsd + ((size_t)b * T + tprev) * H + kbase;
#pragma unroll
          for (int s = 0; s < LP_KH; s += 4) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (b < B) v = *reinterpret_cast<const float4*>(hr + s);
            hb[j][s] = v.x;
            hb[j][s + 1] = v.y;
            hb[j][s + 2] = v.z;
            hb[j][s + 3] = v.w;
          }
        }
#pragma unroll
        for (int s = 0; s < LP_KH; ++s)
#pragma unroll
          for (int j = 0; j < LP_BT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[s], hb[j][s], acc[j], 0, 0, 0);
      }
      // ---- K-slice partials -> LDS: acc[i] holds row 8(i/4) + 4 kk + i%4, sequence l32 ---------
#pragma unroll
      for (int j = 0; j < LP_BT; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) red[wave][j][8 * (i / 4) + 4 * kk + (i % 4)][l32] = acc[j][i];
      __syncthreads();
      // ---- cell update: thread -> (unit, sequence) pairs of these B tiles ---------------------
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int p = tid + 256 * k;
        const int u = p % LP_U, bl = p / LP_U, j = bl / 32, b = bt0 * 32 + bl;
        if (b >= B) continue;
        float gs[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int r = g * LP_U + u;
          gs[g] = (red[0][j][r][bl % 32] + red[1][j][r][bl % 32]) + (red[2][j][r][bl % 32] + red[3][j][r][bl % 32]);
        }
        const int unit = ug * LP_U + u;
        const float gi = lstm_sig(prf[k][0] + gs[0]);
        const float gf = lstm_sig(prf[k][1] + gs[1]);
        const float gg = lstm_tanh(prf[k][2] + gs[2]);
        const float go = lstm_sig(prf[k][3] + gs[3]);
        const float c = step > 0 ? gf * cst[u][b] + gi * gg : gi * gg;
        cst[u][b] = c;
        hsd[((size_t)b * T + t) * H + unit] = go * lstm_tanh(c);
      }
      __syncthreads();  // red reused by the next B tiles
    }
    // ---- publish h_t: stores drained, then one agent-scope release + arrival ------------------
    if (step + 1 < T) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ---- split fp32 batches (B > 4, up to 64 per launch; the bf16x3 / bf16 / fp8 engines) -----------------
// Measured against lstm_persistent_kernel's 24 us per step at B = 64 (gpurun_out lstm1), three changes:
// * the recurrent products are three bf16 MFMA terms (W_hi h_lo + W_lo h_hi + W_hi h_hi, fp32
//   accumulation; v_mfma_f32_32x32x16_bf16, K = 16 per instruction) over split operands: W_hh is split
//   once per launch into resident hi / lo A fragments, and h_t is PUBLISHED split, [seq][hi 640 | lo 640]
//   bf16, so a consumer loads its B fragments as they are (~0.8 instead of ~4.3 us of f32 MFMA chain).
//   The split is the headline's arithmetic (relative error ~2^-16 per product); the fp32 engine keeps
//   the exact-product kernel.
// * the hand-off is per-workgroup flags with write-through payload instead of a counter barrier with
//   a release and an acquire fence: each workgroup stores its units of h_t as 16-byte sc1
//   (write-through) buffer stores, every wave drains them (vmcnt(0)), then after the workgroup barrier
//   one lane stores the workgroup's flag = step + 1 (relaxed agent store = sc1); a consumer's wave 0
//   polls its 40 producers' flags with sc1 loads, the workgroup barrier follows, and EVERY load of the
//   payload is an sc1 buffer load (MI355X_MICROARCH.md § visibility, Valid forms, table row 1; one
//   workgroup per CU is forced by the launch's LDS size).  No fence either side.
// * a workgroup owns 16 units x 32 sequences (not 8 units x 64): it loads h_{t-1} of its 32 sequences
//   only (82 instead of 164 KB a step; at 164 KB the L2 -> CU delivery to the 20 workgroups of an XCD set
//   the step: 24 -> 12.7 us with the first two changes, 7.8 us at 32 sequences).  8 waves, each a
//   80-wide K slice of both 32-row tiles; the 8 partials are summed in LDS.
// Payload buffers alternate by step parity: a workgroup publishes h_{t+1} only after its producers'
// flags of step t are set, i.e. after every reader of the buffer it overwrites finished loading h_{t-1}.
constexpr int LX_U = 16;                     // units per workgroup (64 gate rows = two MFMA M tiles)
constexpr int LX_S = 32;                     // sequences per workgroup (one MFMA N tile)
constexpr int LX_W = 8;                      // waves
constexpr int LX_KW = LP_H / LX_W;           // K slice per wave (80)
constexpr int LX_KS = LX_KW / 16;            // k-steps of 16 per wave (5)
constexpr int LX_G = LP_H / LX_U;            // unit groups per direction (40)
constexpr int LX_FLAGS = 1024;               // [err word | pad | flags 2 dir x 2 halves x 40] (zeroed per launch)
constexpr int LX_PAD_LDS = 16 * 1024;        // dynamic LDS that keeps the workgroups one per CU

__global__ void __launch_bounds__(64 * LX_W, 1) lstm_x3_kernel(const float* __restrict__ pre, const float* __restrict__ whh,
                                                                float* hs, int Btot, int b0, int B, int T, unsigned* sync,
                                                                bf16_t* hx, unsigned spin_max, unsigned* err_host) {
  __shared__ float red[LX_W][2 * 32][LX_S + 1];
  __shared__ float cst[LX_U][LX_S];
  __shared__ __attribute__((aligned(16))) float hst[LX_S][LX_U];
  __shared__ int abort_flag;
  extern __shared__ char lx_pad[];  // occupancy only (LX_PAD_LDS)
  const int H = LP_H;
  // workgroup -> (direction, sequence half, unit group)
  const int dir = blockIdx.x / (2 * LX_G), sh = (blockIdx.x / LX_G) & 1, ug = blockIdx.x % LX_G;
  const int s0 = sh * LX_S, nb = min(LX_S, B - s0);  // this workgroup's sequences [s0, s0 + nb)
  if (nb <= 0) return;  // no live sequence in this half: nobody waits for this workgroup
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int kw = wave * LX_KW;
  unsigned* err = sync;
  unsigned* flags = sync + 64 + (dir * 2 + sh) * LX_G;  // the 40 producers of this (direction, half)
  float* hsd = hs + (size_t)dir * Btot * T * H + (size_t)(b0 + s0) * T * H;
  pre += (size_t)(b0 + s0) * T * 8 * H;
  if (tid == 0) lx_pad[0] = 0;

  // ---- W_hh rows of this workgroup, split -> resident hi / lo A fragments -------------------------
  // tile m, lane (row 32 m + l32 = gate g x 16 + unit, k half hh): k = kw + 16 s + 8 hh + j
  bf16x8 whi[2][LX_KS], wlo[2][LX_KS];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int r = 32 * m + l32, g = r / LX_U, u = ug * LX_U + (r % LX_U);
    const float* wr = whh + ((size_t)dir * 4 * H + (size_t)g * H + u) * H + kw + 8 * hh;
#pragma unroll
    for (int s = 0; s < LX_KS; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(wr + 16 * s);
      const float4 b = *reinterpret_cast<const float4*>(wr + 16 * s + 4);
      const float v0[4] = {a.x, a.y, a.z, a.w}, v1[4] = {b.x, b.y, b.z, b.w};
      uint2 h0, l0, h1, l1;
      split4(v0, h0, l0);
      split4(v1, h1, l1);
      whi[m][s] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
      wlo[m][s] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
    }
  }
  for (int i = tid; i < LX_U * LX_S; i += 64 * LX_W) (&cst[0][0])[i] = 0.f;
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  constexpr int HXS = 2 * LP_H;               // bf16 per published sequence row [hi | lo]
  const size_t hx_par = (size_t)LP_BMAX * HXS;  // one parity buffer of one direction
  bf16_t* hxd = hx + (size_t)dir * 2 * hx_par;
  const int cu = tid % LX_U, cb = tid / LX_U;  // cell-update pair (unit, sequence) of this thread
  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    // the cell update's gate pre-activations, fetched before the wait (their latency hides under it)
    float prf[4];
    {
      const float* pr = pre + ((size_t)cb * T + t) * 8 * H + (size_t)dir * 4 * H + ug * LX_U + cu;
#pragma unroll
      for (int q = 0; q < 4; ++q) prf[q] = cb < nb ? pr[q * H] : 0.f;
    }
    f32x16 acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][i] = 0.f;
    if (step > 0) {
      // ---- wave 0 polls its 40 producers' flags (sc1 loads) until every one reached `step` ----------
      if (wave == 0) {
        unsigned spins = 0;
        for (;;) {
          const bool ok = lane >= LX_G ||
                          __hip_atomic_load(flags + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)step;
          if (__all(ok) && spin_max != 0) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_max || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            if (lane == 0) {
              __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              abort_flag = 1;
            }
            break;
          }
        }
      }
      __syncthreads();
      if (abort_flag) {  // a peer stopped publishing: flag the host, poison the remaining outputs, leave
        if (tid == 0 && err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int st = step; st < T; ++st) {
          const int tt = dir == 0 ? st : T - 1 - st;
          for (int p = tid; p < LX_U * nb; p += 64 * LX_W)
            hsd[((size_t)(p / LX_U) * T + tt) * H + ug * LX_U + p % LX_U] = __builtin_nanf("");
        }
        return;
      }
      // ---- B fragments of h_{t-1}: sequence s0 + l32, k = kw + 16 s + 8 hh (hi and lo), sc1 loads -------
      // (the descriptor's range ends at the last live sequence: lanes past it read zeros)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          hxd + (size_t)((step - 1) & 1) * hx_par, 0, B * HXS * (int)sizeof(bf16_t), 0x00020000);
      uint4 bh[LX_KS], bl[LX_KS];
      const int o = ((s0 + l32) * HXS + kw + 8 * hh) * (int)sizeof(bf16_t);
#pragma unroll
      for (int s = 0; s < LX_KS; ++s) {
        bh[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 32 * s, 0, 16));
        bl[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 32 * s + 2 * LP_H, 0, 16));
      }
      // three terms per k-step, small ones first; the two row tiles' chains interleave
#pragma unroll
      for (int s = 0; s < LX_KS; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wlo[m][s], __builtin_bit_cast(bf16x8, bh[s]), acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(whi[m][s], __builtin_bit_cast(bf16x8, bl[s]), acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(whi[m][s], __builtin_bit_cast(bf16x8, bh[s]), acc[m], 0, 0, 0);
        }
    }
    // ---- K-slice partials -> LDS: acc[m][i] holds row 32 m + 8(i/4) + 4 hh + i%4, sequence l32 ----------
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[wave][32 * m + 8 * (i / 4) + 4 * hh + (i % 4)][l32] = acc[m][i];
    __syncthreads();
    // ---- cell update: thread -> (unit cu, sequence cb), partials summed in a fixed order ----------------
    if (cb < nb) {
      float gs[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int r = g * LX_U + cu;
        gs[g] = ((red[0][r][cb] + red[1][r][cb]) + (red[2][r][cb] + red[3][r][cb])) +
                ((red[4][r][cb] + red[5][r][cb]) + (red[6][r][cb] + red[7][r][cb]));
      }
      const float gi = lstm_sig(prf[0] + gs[0]);
      const float gf = lstm_sig(prf[1] + gs[1]);
      const float gg = lstm_tanh(prf[2] + gs[2]);
      const float go = lstm_sig(prf[3] + gs[3]);
      const float c = step > 0 ? gf * cst[cu][cb] + gi * gg : gi * gg;
      cst[cu][cb] = c;
      const float h = go * lstm_tanh(c);
      hsd[((size_t)cb * T + t) * H + ug * LX_U + cu] = h;
      hst[cb][cu] = h;
    }
    __syncthreads();  // hst complete; red free for the next step
    // ---- publish h_t split: thread (sequence, plane, 8-unit half) stores 16 B, write-through ----------
    if (step + 1 < T) {
      if (tid < 4 * nb) {
        const int b = tid >> 2, plane = (tid >> 1) & 1, half = tid & 1;
        const float4 v0 = *reinterpret_cast<const float4*>(&hst[b][8 * half]);
        const float4 v1 = *reinterpret_cast<const float4*>(&hst[b][8 * half + 4]);
        const float a0[4] = {v0.x, v0.y, v0.z, v0.w}, a1[4] = {v1.x, v1.y, v1.z, v1.w};
        uint2 h0, l0, h1, l1;
        split4(a0, h0, l0);
        split4(a1, h1, l1);
        const uint4 w = plane ? make_uint4(l0.x, l0.y, l1.x, l1.y) : make_uint4(h0.x, h0.y, h1.x, h1.y);
        const __amdgpu_buffer_rsrc_t rd =
            __builtin_amdgcn_make_buffer_rsrc(hxd + (size_t)(step & 1) * hx_par, 0, (int)(hx_par * sizeof(bf16_t)), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, w), rd,
                                               ((s0 + b) * HXS + plane * LP_H + ug * LX_U + 8 * half) * (int)sizeof(bf16_t),
                                               0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(sync + 64 + (dir * 2 + sh) * LX_G + ug, (unsigned)(step + 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- split fp32, small batches (B <= LG_BMAX: configs[4]'s 8 clips a GPU): lstm_x3 with a granule hand-off ------
// lstm_x3's step is three memory round trips deep besides its arithmetic: the h_t stores drain (vmcnt(0)) before the
// workgroup's flag store, a consumer polls its 40 producers' flags, and only then loads the payload (~3.7 us a step
// at 8 x 1000, 78 % of its wave cycles waiting; verdict r05 item 8).  Here h_t travels as data-tagged granules as in
// lstm_small_kernel: each cell-update thread publishes ONE 8-byte sc1 store {tag = step + 1 | hi bf16 | lo bf16} of
// its (unit, sequence) (cdna_hip_programming.md Guideline 16 R2: the data is the flag; no drain, no flag, no
// fence), and every workgroup of the direction sweeps the nb x 640 granules of h_{t-1} with 16-byte sc1 buffer
// loads (two granules each, every one checked by its own tag; the stale ones re-polled together) into an LDS
// image [sequence][hi 640 | lo 640] bf16 (rows padded by 16 B: the B-fragment reads of 16 sequences fall on
// distinct banks), from which the MFMA B fragments are read.  Everything else is lstm_x3's: W_hh split into resident
// hi / lo A fragments, three v_mfma_f32_32x32x16_bf16 terms, K-slice partials summed in LDS in a fixed order, fp32
// cell state and gate math.  Granules are double-buffered by step parity (no workgroup of a direction can be more
// than one step ahead of another: publishing h_{t+1} needs every h_t).
constexpr int LG_BMAX = 16;                            // sequences (one half of lstm_x3's 32-sequence tile)
constexpr int LG_ROWB = 2 * 2 * LP_H + 16;             // LDS image row bytes: hi 640 | lo 640 bf16 + pad
constexpr int LG_PAIRS = LP_H / 2;                     // 16-byte granule pairs per sequence

__global__ void __launch_bounds__(64 * LX_W, 1) lstm_x3g_kernel(const float* __restrict__ pre, const float* __restrict__ whh,
                                                                 float* hs, int B, int T, unsigned* err,
                                                                 unsigned long long* gran, unsigned spin_max,
                                                                 unsigned* err_host, unsigned ep) {
  __shared__ float red[LX_W][2 * 32][LX_S + 1];
  __shared__ float cst[LX_U][LG_BMAX];
  __shared__ __attribute__((aligned(16))) char hxl[LG_BMAX * LG_ROWB];
  __shared__ int abort_flag;
  extern __shared__ char lx_pad[];  // occupancy only
  const int H = LP_H;
  const int dir = blockIdx.x / LX_G, ug = blockIdx.x % LX_G;
  const int nb = B;  // launch_lstm_x3g: B <= LG_BMAX, one workgroup row of sequences
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hh = lane >> 5, l32 = lane & 31;
  const int kw = wave * LX_KW;
  float* hsd = hs + (size_t)dir * B * T * H;
  unsigned long long* gd = gran + (size_t)dir * 2 * LG_BMAX * H;  // [parity][sequence][unit]
  if (tid == 0) lx_pad[0] = 0;

  bf16x8 whi[2][LX_KS], wlo[2][LX_KS];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int r = 32 * m + l32, g = r / LX_U, u = ug * LX_U + (r % LX_U);
    const float* wr = whh + ((size_t)dir * 4 * H + (size_t)g * H + u) * H + kw + 8 * hh;
#pragma unroll
    for (int s = 0; s < LX_KS; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(wr + 16 * s);
      const float4 b = *reinterpret_cast<const float4*>(wr + 16 * s + 4);
      const float v0[4] = {a.x, a.y, a.z, a.w}, v1[4] = {b.x, b.y, b.z, b.w};
      uint2 h0, l0, h1, l1;
      split4(v0, h0, l0);
      split4(v1, h1, l1);
      whi[m][s] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
      wlo[m][s] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
    }
  }
  for (int i = tid; i < LX_U * LG_BMAX; i += 64 * LX_W) (&cst[0][0])[i] = 0.f;
  for (int i = tid; i < LG_BMAX * LG_ROWB / 16; i += 64 * LX_W)  // rows >= nb stay zero (their B columns unused)
    reinterpret_cast<uint4*>(hxl)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  const int cu = tid % LX_U, cb = tid / LX_U;  // cell-update pair (unit, sequence) of this thread
  const uint32_t hx0 = (uint32_t)(uintptr_t)hxl;
  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    float prf[4];
    {
      const float* pr = pre + ((size_t)cb * T + t) * 8 * H + (size_t)dir * 4 * H + ug * LX_U + cu;
#pragma unroll
      for (int q = 0; q < 4; ++q) prf[q] = cb < nb ? pr[q * H] : 0.f;
    }
    f32x16 acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][i] = 0.f;
    if (step > 0) {
      // ---- sweep h_{t-1}: granule pairs q = tid + 512 j (sequence q / 320, units 2 (q % 320) + {0, 1}), all loads
      // issued first, then the tags checked; the stale pairs re-polled together ----------------------------------
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          gd + (size_t)((step - 1) & 1) * LG_BMAX * H, 0, nb * H * (int)sizeof(unsigned long long), 0x00020000);
      constexpr int PJ = (LG_BMAX * LG_PAIRS + 64 * LX_W - 1) / (64 * LX_W);  // pairs per thread at most (10)
      u32x4_t v[PJ];
#pragma unroll
      for (int j = 0; j < PJ; ++j) {
        const int q = tid + 64 * LX_W * j;
        v[j] = q < nb * LG_PAIRS ? __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, 0, 16) : u32x4_t{0u, 0u, 0u, 0u};
      }
      // stale pairs are re-polled together (one round trip a poll for all of them, not one per granule)
      for (unsigned spins = 0;; ++spins) {
        bool stale = false;
#pragma unroll
        for (int j = 0; j < PJ; ++j) {
          const int q = tid + 64 * LX_W * j;
          stale |= q < nb * LG_PAIRS && (v[j][1] != ep + (unsigned)step || v[j][3] != ep + (unsigned)step);
        }
        if (!stale && spin_max != 0) break;
        if (spins >= spin_max || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ep + 1u) {
          __hip_atomic_store(err, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          abort_flag = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int j = 0; j < PJ; ++j) {
          const int q = tid + 64 * LX_W * j;
          if (q < nb * LG_PAIRS && (v[j][1] != ep + (unsigned)step || v[j][3] != ep + (unsigned)step))
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, 0, 16);
        }
      }
#pragma unroll
      for (int j = 0; j < PJ; ++j) {
        const int q = tid + 64 * LX_W * j;
        if (q >= nb * LG_PAIRS) break;
        // hi halves of the two units -> the sequence row's hi plane, lo halves -> its lo plane (4-byte stores)
        const int sq = q / LG_PAIRS, u2 = 2 * (q - sq * LG_PAIRS);
        const uint32_t hi = (v[j][0] & 0xffffu) | (v[j][2] << 16), lo = (v[j][0] >> 16) | (v[j][2] & 0xffff0000u);
        *reinterpret_cast<uint32_t*>(hxl + sq * LG_ROWB + 2 * u2) = hi;
        *reinterpret_cast<uint32_t*>(hxl + sq * LG_ROWB + 2 * H + 2 * u2) = lo;
      }
      __syncthreads();
      if (abort_flag) {  // a peer stopped publishing: flag the host, poison the remaining outputs, leave
        if (tid == 0 && err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int st = step; st < T; ++st) {
          const int tt = dir == 0 ? st : T - 1 - st;
          for (int p = tid; p < LX_U * nb; p += 64 * LX_W)
            hsd[((size_t)(p / LX_U) * T + tt) * H + ug * LX_U + p % LX_U] = __builtin_nanf("");
        }
        return;
      }
      // ---- B fragments of h_{t-1} from the image: sequence l32, k = kw + 16 s + 8 hh (hi and lo) -------------
      uint4 bh[LX_KS], bl[LX_KS];
      const uint32_t o = hx0 + (uint32_t)(l32 * LG_ROWB + 2 * (kw + 8 * hh));
#pragma unroll
      for (int s = 0; s < LX_KS; ++s) {
        if (l32 < LG_BMAX) {
          bh[s] = *reinterpret_cast<const uint4*>(hxl + (o - hx0) + 32 * s);
          bl[s] = *reinterpret_cast<const uint4*>(hxl + (o - hx0) + 32 * s + 2 * H);
        } else {
          bh[s] = bl[s] = make_uint4(0u, 0u, 0u, 0u);
        }
      }
#pragma unroll
      for (int s = 0; s < LX_KS; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wlo[m][s], __builtin_bit_cast(bf16x8, bh[s]), acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(whi[m][s], __builtin_bit_cast(bf16x8, bl[s]), acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(whi[m][s], __builtin_bit_cast(bf16x8, bh[s]), acc[m], 0, 0, 0);
        }
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[wave][32 * m + 8 * (i / 4) + 4 * hh + (i % 4)][l32] = acc[m][i];
    __syncthreads();
    // ---- cell update (unit cu, sequence cb); h_t published as a granule {step + 1 | hi | lo} -------------------
    if (cb < nb) {
      float gs[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int r = g * LX_U + cu;
        gs[g] = ((red[0][r][cb] + red[1][r][cb]) + (red[2][r][cb] + red[3][r][cb])) +
                ((red[4][r][cb] + red[5][r][cb]) + (red[6][r][cb] + red[7][r][cb]));
      }
      const float gi = lstm_sig(prf[0] + gs[0]);
      const float gf = lstm_sig(prf[1] + gs[1]);
      const float gg = lstm_tanh(prf[2] + gs[2]);
      const float go = lstm_sig(prf[3] + gs[3]);
      const float c = step > 0 ? gf * cst[cu][cb] + gi * gg : gi * gg;
      cst[cu][cb] = c;
      const float h = go * lstm_tanh(c);
      hsd[((size_t)cb * T + t) * H + ug * LX_U + cu] = h;
      if (step + 1 < T) {
        const bf16_t hb = f2bf(h), lb = f2bf(h - bf2f(hb));  // the split of sp_t (17 bits)
        __hip_atomic_store(gd + (size_t)(step & 1) * LG_BMAX * H + (size_t)cb * H + ug * LX_U + cu,
                           ((unsigned long long)(ep + (unsigned)step + 1u) << 32) | ((unsigned)lb << 16) | (unsigned)hb,
                           __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();  // red and the image are rewritten next step
  }
}

// ---- small batches (B <= LS_BMAX: the 1 x 1000-frame configs[4] clip, the 1 x 30 configs[0] clip) -----
// At B = 1 the 32-wide MFMA B tile is 1/32 used and the counter barrier (store drain, agent release,
// atomic, relaxed polls, acquire + L2 refill of h) cost ~20 us a step.  Here h_t travels as data-
// tagged 8-byte granules {tag = step + 1, value = h} written by ONE sc1 atomic store each
// (cdna_hip_programming.md Guideline 16 R2: the data is the flag, no fence, no counter); every
// workgroup of the direction sweeps the B x 640 granules of h_{t-1} with relaxed agent loads until
// every tag matches, into LDS.  Granules are double-buffered by step parity (a workgroup can run at
// most one step ahead of any other: publishing h_{t+1} needs every h_t).  The recurrence products
// run on VALU: lane (wave, k half, row) holds the same 80 W_hh values as above and forms B fp32 dot
// products of 80 terms; the 8 K-slice partials of each gate row are summed in LDS in a fixed order.
constexpr int LS_BMAX = 4;   // default small-batch limit
constexpr int LS_BCAP = 8;   // largest instantiation (M2S_LSTM_SMALL_B = 8 selects it for B <= 8)

template <int LS_BMAX>
__global__ void __launch_bounds__(256, 1) lstm_small_kernel(const float* __restrict__ pre, const float* __restrict__ whh,
                                                            float* hs, int B, int T, unsigned long long* gran,
                                                            unsigned* err, unsigned spin_max, unsigned* err_host,
                                                            unsigned ep) {
  __shared__ __attribute__((aligned(16))) float hsh[LS_BMAX][LP_H];  // h_{t-1}, all units
  __shared__ float red[8][32][LS_BMAX];                              // [K slice][gate row][sequence]
  __shared__ float cst[LP_U][LS_BMAX];
  __shared__ int abort_flag;
  const int H = LP_H;
  const int dir = blockIdx.x / (H / LP_U), ug = blockIdx.x - dir * (H / LP_U);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kk = lane >> 5, l32 = lane & 31;
  const int kbase = wave * LP_KW + kk * LP_KH;
  float* hsd = hs + (size_t)dir * B * T * H;
  unsigned long long* gd = gran + (size_t)dir * 2 * LS_BMAX * H;

  float wa[LP_KH];
  {
    const int r = l32, g = r / LP_U, u = ug * LP_U + (r % LP_U);
    const float* wr = whh + ((size_t)dir * 4 * H + (size_t)g * H + u) * H + kbase;
#pragma unroll
    for (int s = 0; s < LP_KH; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(wr + s);
      wa[s] = v.x;
      wa[s + 1] = v.y;
      wa[s + 2] = v.z;
      wa[s + 3] = v.w;
    }
  }
  if (tid < LP_U * LS_BMAX) (&cst[0][0])[tid] = 0.f;
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    float p[LS_BMAX];
#pragma unroll
    for (int b = 0; b < LS_BMAX; ++b) p[b] = 0.f;
    if (step > 0) {
      // ---- h_{t-1}: sweep the direction's granules (tag == step) into LDS -----------------------
      const unsigned long long* src = gd + (size_t)((step - 1) & 1) * LS_BMAX * H;
      bool ok = true;
      for (int i = tid; i < B * H && ok; i += 256) {
        unsigned spins = 0;
        unsigned long long x;
        while (((x = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != ep + (unsigned)step ||
               spin_max == 0) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_max || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ep + 1u) {
            __hip_atomic_store(err, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            abort_flag = 1;
            ok = false;
            break;
          }
        }
        hsh[i / H][i % H] = __uint_as_float((unsigned)x);
      }
      __syncthreads();
      if (abort_flag) {  // a peer stopped publishing: flag the host, poison the remaining outputs, leave
        if (tid == 0 && err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int st = step; st < T; ++st) {
          const int tt = dir == 0 ? st : T - 1 - st;
          for (int q = tid; q < LP_U * B; q += 256)
            hsd[((size_t)(q / LP_U) * T + tt) * H + ug * LP_U + q % LP_U] = __builtin_nanf("");
        }
        return;
      }
      // ---- this lane's 80-term K-slice dot products for gate row l32 -----------------------------
#pragma unroll
      for (int b = 0; b < LS_BMAX; ++b) {
        if (LS_BMAX <= 4 && b >= B) break;  // (the 8-wide instantiation computes all rows: stale ones unused)
        const float* hb = &hsh[b][kbase];
        float a = 0.f;
#pragma unroll
        for (int s = 0; s < LP_KH; s += 4) {
          const float4 v = *reinterpret_cast<const float4*>(hb + s);
          a += wa[s] * v.x;
          a += wa[s + 1] * v.y;
          a += wa[s + 2] * v.z;
          a += wa[s + 3] * v.w;
        }
        p[b] = a;
      }
    }
#pragma unroll
    for (int b = 0; b < LS_BMAX; ++b) red[wave * 2 + kk][l32][b] = p[b];
    __syncthreads();
    // ---- cell update for (unit, sequence); publish h_t as granules (tag = step + 1) ---------------
    if (tid < LP_U * B) {
      const int u = tid % LP_U, b = tid / LP_U, unit = ug * LP_U + u;
      float gs[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int r = g * LP_U + u;
        gs[g] = ((red[0][r][b] + red[1][r][b]) + (red[2][r][b] + red[3][r][b])) +
                ((red[4][r][b] + red[5][r][b]) + (red[6][r][b] + red[7][r][b]));
      }
      const float* pr = pre + ((size_t)b * T + t) * 8 * H + (size_t)dir * 4 * H;
      const float gi = lstm_sig(pr[unit] + gs[0]);
      const float gf = lstm_sig(pr[H + unit] + gs[1]);
      const float gg = lstm_tanh(pr[2 * H + unit] + gs[2]);
      const float go = lstm_sig(pr[3 * H + unit] + gs[3]);
      const float c = step > 0 ? gf * cst[u][b] + gi * gg : gi * gg;
      cst[u][b] = c;
      const float h = go * lstm_tanh(c);
      hsd[((size_t)b * T + t) * H + unit] = h;
      if (step + 1 < T)
        __hip_atomic_store(gd + (size_t)(step & 1) * LS_BMAX * H + (size_t)b * H + unit,
                           ((unsigned long long)(ep + (unsigned)step + 1u) << 32) | __float_as_uint(h), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // red and hsh are rewritten next step
  }
}

// ---- medium batches (LS_BMAX < B <= LM_BMAX: configs[4]'s 8 x 1000 frames, the bench's 64 clips) -------
// The granule exchange of lstm_small_kernel, scaled to B sequences:
// * 512 threads (two waves per SIMD: one wave alone issues v_fma_f32 every 4 cycles, two every 2);
//   lane (wave w, k half kk, gate row l32) keeps 40 W_hh values (k = 80 w + 40 kk ..) in VGPRs;
// * sequences in chunks of LM_CH: the chunk's h_{t-1} granules (LM_CH x 640 x 8 B) are swept into a
//   double-buffered LDS image, and the sweep of chunk c + 1 is ISSUED (LM_G independent sc1 loads per
//   thread, tags checked afterwards) before the dot products of chunk c, so the exchange latency runs
//   under the arithmetic;
// * per chunk the 16 K-slice partials of every (gate row, sequence) are summed in LDS in a fixed order and
//   128 threads apply the cell update and publish h_t (tag = step + 1), as lstm_small_kernel does.
// Double buffering by step parity stays safe per chunk: a workgroup can publish chunk c of h_{t+1} only
// after every workgroup published chunk c of h_t, i.e. after each of them finished reading chunk c of
// h_{t-1}.  Exact fp32 products; the partial-sum order is fixed.
constexpr int LM_BMAX = 64, LM_THREADS = 512;
constexpr int LM_KL = LP_H / 16;                    // k per lane (16 slices of 40)

template <int LM_CH>
__global__ void __launch_bounds__(LM_THREADS, 1) lstm_mid_kernel(const float* __restrict__ pre,
                                                                 const float* __restrict__ whh, float* hs, int B,
                                                                 int T, unsigned long long* gran, unsigned* err,
                                                                 unsigned spin_max, unsigned* err_host) {
  __shared__ __attribute__((aligned(16))) float hsh[2][LM_CH][LP_H];   // h_{t-1} of two chunks
  __shared__ __attribute__((aligned(16))) float red[16][32][LM_CH];    // [K slice][gate row][sequence]
  __shared__ float cst[LP_U][LM_BMAX];
  __shared__ int abort_flag;
  const int H = LP_H;
  const int dir = blockIdx.x / (H / LP_U), ug = blockIdx.x - dir * (H / LP_U);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kk = lane >> 5, l32 = lane & 31;
  const int slice = wave * 2 + kk, kbase = slice * LM_KL;
  float* hsd = hs + (size_t)dir * B * T * H;
  unsigned long long* gd = gran + (size_t)dir * 2 * LM_BMAX * H;
  const int nch = (B + LM_CH - 1) / LM_CH;
  constexpr int LM_G = LM_CH * LP_H / LM_THREADS;  // granules per thread per chunk

  float wa[LM_KL];
  {
    const int r = l32, g = r / LP_U, u = ug * LP_U + (r % LP_U);
    const float* wr = whh + ((size_t)dir * 4 * H + (size_t)g * H + u) * H + kbase;
#pragma unroll
    for (int s = 0; s < LM_KL; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(wr + s);
      wa[s] = v.x;
      wa[s + 1] = v.y;
      wa[s + 2] = v.z;
      wa[s + 3] = v.w;
    }
  }
  for (int i = tid; i < LP_U * LM_BMAX; i += LM_THREADS) (&cst[0][0])[i] = 0.f;
  if (tid == 0) abort_flag = 0;
  __syncthreads();

  unsigned long long g[LM_G];
  // issue the sweep loads of chunk c of h_{step-1} (relaxed agent loads: sc1, served by L2)
  auto issue = [&](int step, int c) {
    const unsigned long long* src = gd + (size_t)((step - 1) & 1) * LM_BMAX * H + (size_t)c * LM_CH * H;
    const int n = min(LM_CH, B - c * LM_CH) * H;
#pragma unroll
    for (int j = 0; j < LM_G; ++j) {
      const int i = tid + j * LM_THREADS;
      g[j] = i < n ? __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    }
  };
  // tags checked, late granules re-polled (bounded), values -> LDS buffer `buf`; false on timeout
  auto land = [&](int step, int c, int buf) -> bool {
    const unsigned long long* src = gd + (size_t)((step - 1) & 1) * LM_BMAX * H + (size_t)c * LM_CH * H;
    const int n = min(LM_CH, B - c * LM_CH) * H;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < LM_G; ++j) {
      const int i = tid + j * LM_THREADS;
      if (i >= n) continue;
      unsigned long long x = g[j];
      unsigned spins = 0;
      while (ok && ((unsigned)(x >> 32) != (unsigned)step || spin_max == 0)) {
        __builtin_amdgcn_s_sleep(1);
        x = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (++spins > spin_max || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          abort_flag = 1;
          ok = false;
        }
      }
      hsh[buf][i / H][i % H] = __uint_as_float((unsigned)x);
    }
    return ok;
  };

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    if (step > 0) {
      issue(step, 0);
      land(step, 0, 0);
    }
    for (int c = 0; c < nch; ++c) {
      const int nb = min(LM_CH, B - c * LM_CH);
      // cell-update threads fetch their gate pre-activations early (tid = u + 8 b)
      float pr4[4] = {0.f, 0.f, 0.f, 0.f};
      const int cu = tid % LP_U, cb = tid / LP_U;
      if (tid < LP_U * nb) {
        const float* pr = pre + ((size_t)(c * LM_CH + cb) * T + t) * 8 * H + (size_t)dir * 4 * H + ug * LP_U + cu;
#pragma unroll
        for (int q = 0; q < 4; ++q) pr4[q] = pr[q * H];
      }
      __syncthreads();  // chunk c's image complete (and red free)
      if (abort_flag) {  // a peer stopped publishing: flag the host, poison the remaining outputs, leave
        if (tid == 0 && err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int st = step; st < T; ++st) {
          const int tt = dir == 0 ? st : T - 1 - st;
          for (int q = tid; q < LP_U * B; q += LM_THREADS)
            hsd[((size_t)(q / LP_U) * T + tt) * H + ug * LP_U + q % LP_U] = __builtin_nanf("");
        }
        return;
      }
      if (step > 0 && c + 1 < nch) issue(step, c + 1);  // next chunk's exchange under this chunk's math
      // this lane's 40-term dot products for its gate row, one sequence at a time (four interleaved
      // accumulators, summed in a fixed order), straight into the partial-sum image
      const int buf = c & 1;
#pragma unroll 2
      for (int b = 0; b < nb; ++b) {
        float a4[4] = {0.f, 0.f, 0.f, 0.f};
        if (step > 0) {
          const float* hb = &hsh[buf][b][kbase];
#pragma unroll
          for (int s = 0; s < LM_KL; s += 4) {
            const float4 v = *reinterpret_cast<const float4*>(hb + s);
            a4[0] = fmaf(wa[s], v.x, a4[0]);
            a4[1] = fmaf(wa[s + 1], v.y, a4[1]);
            a4[2] = fmaf(wa[s + 2], v.z, a4[2]);
            a4[3] = fmaf(wa[s + 3], v.w, a4[3]);
          }
        }
        red[slice][l32][b] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
      if (step > 0 && c + 1 < nch) land(step, c + 1, (c + 1) & 1);
      __syncthreads();
      if (tid < LP_U * nb) {
        const int unit = ug * LP_U + cu, b = c * LM_CH + cb;
        float gs[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = q * LP_U + cu;
          float s = 0.f;
#pragma unroll
          for (int sl = 0; sl < 16; sl += 4)
            s += (red[sl][r][cb] + red[sl + 1][r][cb]) + (red[sl + 2][r][cb] + red[sl + 3][r][cb]);
          gs[q] = s;
        }
        const float gi = lstm_sig(pr4[0] + gs[0]);
        const float gf = lstm_sig(pr4[1] + gs[1]);
        const float gg = lstm_tanh(pr4[2] + gs[2]);
        const float go = lstm_sig(pr4[3] + gs[3]);
        const float cc = step > 0 ? gf * cst[cu][b] + gi * gg : gi * gg;
        cst[cu][b] = cc;
        const float h = go * lstm_tanh(cc);
        hsd[((size_t)b * T + t) * H + unit] = h;
        if (step + 1 < T)
          __hip_atomic_store(gd + (size_t)(step & 1) * LM_BMAX * H + (size_t)b * H + unit,
                             ((unsigned long long)(step + 1) << 32) | __float_as_uint(h), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

}  // namespace

static int small_cap() {
  static const int cap = [] {
    const char* e = std::getenv("M2S_LSTM_SMALL_B");
    return e && std::atoi(e) == 8 ? 8 : LS_BMAX;
  }();
  return cap;
}

// 4 < B <= 16: above 16 sequences every workgroup's sweep of B x 640 granules per step (sc1 loads, the
// exchange volume grows with B) costs more than the counter barrier's plain loads of h (tools/lstm_bench.py,
// profiles/r03f_lstm_ab.txt: B = 32 20.2 vs 18.3 us, B = 64 40.9 vs 24.7 us per step)
bool lstm_mid_supported(int B, int H) { return H == LP_H && B > small_cap() && B <= 16; }

size_t lstm_mid_sync_bytes() { return 256 + (size_t)2 * 2 * LM_BMAX * LP_H * sizeof(unsigned long long); }

void launch_lstm_mid(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                     unsigned* err_host, hipStream_t s) {
  M2S_CHECK(lstm_mid_supported(B, H) && T > 0, "lstm_mid: unsupported shape");
  const int grid = 2 * (H / LP_U);
  // sequences per chunk: 4 up to B = 8 (two chunks at B = 8: the second one's sweep overlaps the first's
  // dot products; 6.5 us per step vs 8.6 at one chunk of 8), 8 above; env M2S_LSTM_MID_CH for A/B runs
  static const int ch_env = [] {
    const char* e = std::getenv("M2S_LSTM_MID_CH");
    const int v = e ? std::atoi(e) : 0;
    return v == 4 || v == 8 || v == 16 ? v : 0;
  }();
  const int ch = ch_env ? ch_env : (B <= 8 ? 4 : 8);
  const void* fn = ch == 4 ? reinterpret_cast<const void*>(&lstm_mid_kernel<4>)
                   : ch == 16 ? reinterpret_cast<const void*>(&lstm_mid_kernel<16>)
                              : reinterpret_cast<const void*>(&lstm_mid_kernel<8>);
  const int resident = device_resident(fn, LM_THREADS, 0);
  M2S_CHECK(grid <= resident, "lstm_mid: grid not co-resident on this device");
  M2S_HIP(hipMemsetAsync(sync, 0, lstm_mid_sync_bytes(), s));
  unsigned* err = static_cast<unsigned*>(sync);
  unsigned long long* gran = reinterpret_cast<unsigned long long*>(static_cast<char*>(sync) + 256);
  if (ch == 4)
    hipLaunchKernelGGL((lstm_mid_kernel<4>), dim3(grid), dim3(LM_THREADS), 0, s, pre, whh, hs, B, T, gran, err,
                       spin_max, err_host);
  else if (ch == 16)
    hipLaunchKernelGGL((lstm_mid_kernel<16>), dim3(grid), dim3(LM_THREADS), 0, s, pre, whh, hs, B, T, gran, err,
                       spin_max, err_host);
  else
    hipLaunchKernelGGL((lstm_mid_kernel<8>), dim3(grid), dim3(LM_THREADS), 0, s, pre, whh, hs, B, T, gran, err,
                       spin_max, err_host);
  M2S_HIP(hipGetLastError());
}

bool lstm_persistent_supported(int H) { return H == LP_H; }

bool lstm_small_supported(int B, int H) { return H == LP_H && B >= 1 && B <= small_cap(); }

// Epoch tags for the granule hand-off (lstm_small, lstm_x3g): a launch publishes tags ep + step + 1 and waits for
// ep + step, its timeout mark is ep + 1, and the engine's counter advances by T + 1 a launch, so every tag and mark of
// an older launch is below every tag this one waits for: no memset node before each call (a ~4.6 us launch of a
// 30-frame pass's ~1 ms).  The buffer is zeroed (and the count restarted) on first use, near the wrap, and under
// stream capture, whose replays would repeat one epoch.
unsigned lstm_epoch(void* sync, size_t bytes, int T, unsigned* epoch, hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  M2S_HIP(hipStreamIsCapturing(s, &cs));
  if (!epoch || *epoch == 0 || cs != hipStreamCaptureStatusNone || *epoch > 0xF0000000u - (unsigned)T) {
    M2S_HIP(hipMemsetAsync(sync, 0, bytes, s));
    if (epoch) *epoch = (unsigned)T + 1u;
    return 0u;
  }
  const unsigned e = *epoch;
  *epoch += (unsigned)T + 1u;
  return e;
}

size_t lstm_small_sync_bytes() { return 256 + (size_t)2 * 2 * LS_BCAP * LP_H * sizeof(unsigned long long); }

void launch_lstm_small(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                       unsigned* err_host, hipStream_t s, unsigned* epoch) {
  M2S_CHECK(lstm_small_supported(B, H) && T > 0, "lstm_small: unsupported shape");
  const int grid = 2 * (H / LP_U);
  const bool b8 = B > LS_BMAX;  // the 8-sequence instantiation (M2S_LSTM_SMALL_B = 8)
  const void* fn = b8 ? reinterpret_cast<const void*>(&lstm_small_kernel<LS_BCAP>)
                      : reinterpret_cast<const void*>(&lstm_small_kernel<LS_BMAX>);
  const int resident = device_resident(fn, 256, 0);
  M2S_CHECK(grid <= resident, "lstm_small: grid not co-resident on this device");
  // [256 B: error word][granules 2 dir x 2 parity x LS_BMAX x H], epoch-tagged (lstm_epoch)
  const unsigned ep = lstm_epoch(sync, lstm_small_sync_bytes(), T, epoch, s);
  unsigned* err = static_cast<unsigned*>(sync);
  unsigned long long* gran = reinterpret_cast<unsigned long long*>(static_cast<char*>(sync) + 256);
  if (b8)
    hipLaunchKernelGGL(lstm_small_kernel<LS_BCAP>, dim3(grid), dim3(256), 0, s, pre, whh, hs, B, T, gran, err, spin_max,
                       err_host, ep);
  else
    hipLaunchKernelGGL(lstm_small_kernel<LS_BMAX>, dim3(grid), dim3(256), 0, s, pre, whh, hs, B, T, gran, err, spin_max,
                       err_host, ep);
  M2S_HIP(hipGetLastError());
}

size_t lstm_persistent_sync_bytes() { return 256; }

void launch_lstm_persistent(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync,
                            unsigned spin_max, unsigned* err_host, hipStream_t s) {
  M2S_CHECK(lstm_persistent_supported(H) && B > 0 && T > 0, "lstm_persistent: unsupported shape");
  const int grid = 2 * (H / LP_U);
  // Every workgroup must be resident (the step barrier waits on all of them).  The grid is 160
  // workgroups at one per CU; check it against the occupancy query once.  (A plain launch has the
  // same residency as a cooperative one, which only adds this check - and crashes rocprofv3 7.x's
  // kernel tracer at process exit.)
  const int resident = device_resident(reinterpret_cast<const void*>(&lstm_persistent_kernel), 256, 0);
  M2S_CHECK(grid <= resident, "lstm_persistent: grid not co-resident on this device");
  LstmSync* sp = static_cast<LstmSync*>(sync);
  for (int b0 = 0; b0 < B; b0 += LP_BMAX) {  // c lives in LDS: at most LP_BMAX sequences per launch
    const int nb = std::min(LP_BMAX, B - b0);
    M2S_HIP(hipMemsetAsync(sync, 0, lstm_persistent_sync_bytes(), s));
    hipLaunchKernelGGL(lstm_persistent_kernel, dim3(grid), dim3(256), 0, s, pre, whh, hs, B, b0, nb, T, sp, spin_max,
                       err_host);
    M2S_HIP(hipGetLastError());
  }
}

size_t lstm_x3_sync_bytes() { return LX_FLAGS + (size_t)2 * 2 * LP_BMAX * 2 * LP_H * sizeof(bf16_t); }

void launch_lstm_x3(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                    unsigned* err_host, hipStream_t s) {
  M2S_CHECK(lstm_persistent_supported(H) && B > 0 && T > 0, "lstm_x3: unsupported shape");
  const int grid = 2 * 2 * LX_G;  // (direction, sequence half, unit group)
  const int resident = device_resident(reinterpret_cast<const void*>(&lstm_x3_kernel), 64 * LX_W, LX_PAD_LDS);
  M2S_CHECK(grid <= resident, "lstm_x3: grid not co-resident on this device");
  unsigned* sp = static_cast<unsigned*>(sync);
  bf16_t* hx = reinterpret_cast<bf16_t*>(static_cast<char*>(sync) + LX_FLAGS);
  for (int b0 = 0; b0 < B; b0 += LP_BMAX) {  // c lives in LDS: at most LP_BMAX sequences per launch
    const int nb = std::min(LP_BMAX, B - b0);
    M2S_HIP(hipMemsetAsync(sync, 0, LX_FLAGS, s));  // error word + flags: epochs restart at 0 each launch
    hipLaunchKernelGGL(lstm_x3_kernel, dim3(grid), dim3(64 * LX_W), LX_PAD_LDS, s, pre, whh, hs, B, b0, nb, T, sp, hx,
                       spin_max, err_host);
    M2S_HIP(hipGetLastError());
  }
}

size_t lstm_x3g_sync_bytes() { return 256 + (size_t)2 * 2 * LG_BMAX * LP_H * sizeof(unsigned long long); }

bool lstm_x3g_supported(int B, int H) { return H == LP_H && B >= 1 && B <= LG_BMAX; }

void launch_lstm_x3g(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                     unsigned* err_host, hipStream_t s, unsigned* epoch) {
  M2S_CHECK(lstm_x3g_supported(B, H) && T > 0, "lstm_x3g: unsupported shape");
  const int grid = 2 * LX_G;  // (direction, unit group): one row of <= 16 sequences
  const int resident = device_resident(reinterpret_cast<const void*>(&lstm_x3g_kernel), 64 * LX_W, LX_PAD_LDS);
  M2S_CHECK(grid <= resident, "lstm_x3g: grid not co-resident on this device");
  // [256 B: error word][granules 2 dir x 2 parity x LG_BMAX x H], epoch-tagged (lstm_epoch)
  const unsigned ep = lstm_epoch(sync, lstm_x3g_sync_bytes(), T, epoch, s);
  unsigned* err = static_cast<unsigned*>(sync);
  unsigned long long* gran = reinterpret_cast<unsigned long long*>(static_cast<char*>(sync) + 256);
  hipLaunchKernelGGL(lstm_x3g_kernel, dim3(grid), dim3(64 * LX_W), LX_PAD_LDS, s, pre, whh, hs, B, T, err, gran, spin_max,
                     err_host, ep);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
