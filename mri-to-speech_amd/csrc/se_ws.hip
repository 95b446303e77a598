// Split-fp32 SE-gated conv_pwl (+ bn3 + skip) of the stride-1 IR blocks as a persistent, warp-specialised
// GEMM with a flag-synchronised LDS ring (no per-K-step barrier):
//
//   y[m][n] = sum_k W[n][k] * (gate[img(m)][k] * X[m][k]) + bias[n] (+ res[m][n]),  all split fp32
//
// (timm InvertedResidual se.conv_expand gate x conv_pwl + bn3 + skip; mri_acoustic_model.py:28-34,46.)
// Operands as gemm128.hip KIND_SP_SE: X interleaved split [M][cs_in / 32][hi 32 | lo 32] bf16 (ir_ws /
// ir_pwdw il_st8), W split rows [n_pad][hi kp | lo kp] (kp = cs_in), gate split [M / P][hi cs_in | lo cs_in],
// res / y split [M][hi cs_out | lo cs_out].  A K step is 32 channels = one 128-byte LDS row per operand row.
//
// Why.  The barrier-synchronous rings (conv_gemm's in-LDS scaling, gemm128 KIND_SP_SE) stream this operand
// at ~3.2 TB/s while the same access pattern streams at 6.1 TB/s when every wave keeps its own DMAs in
// flight without a barrier (tools/bw_probe.hip): a barrier per K step ties every wave to the
// slowest DMA and every tile starts with an empty ring.  Here one workgroup per CU walks its tiles
// (tile = blockIdx.x + i * gridDim.x) and the ring runs across tile boundaries:
//
//   loader waves (NL): for the flat step s (tile, K step) wait until FREE[s % NS] shows the consumers
//     released the slot's previous use, issue their share of the step's DMAs (weights rows, activation
//     rows; at a tile's first step loader 0 also DMAs the tile's gate rows), then, with step s in flight,
//     wait for step s - 1's DMAs (counted vmcnt) and publish it: FULL[(s - 1) % NS] += 1.
//   consumer waves (WM x WN, 64 x 16 NT each): wait until FULL[s % NS] reached NL x (use + 1), read the
//     step's gate, activation and weight fragments, release the slot (FREE += 1) as soon as the reads
//     returned, gate the activations in fp32 and re-split them (17 bits), three bf16 MFMA terms; after a
//     tile's last step the epilogue (bias, skip, split store) runs while the loaders already fill the next
//     tile's first slots.
//
// Flags are monotonic per-slot counters in LDS (ds_add_u32 by one lane, ds_read polls with s_sleep); every
// wait is bounded: past its poll limit the wave reports the timeout through the engine's host-mapped error
// word (m2s_acoustic_status, as the BiLSTM's barrier waits do), a consumer stores its tiles as NaN from then
// on, and the wave goes on (a reported failure, never a hang).  LDS-DMA data is in
// LDS when the issuing wave's vmcnt retires it, and a consumer reads a slot only after the loader's flag
// update that follows that vmcnt wait, so the flag orders the data.
#include <cstdlib>
#include <cstring>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int ROWB = 128;            // bytes per LDS row: 32 channels [hi 32 | lo 32] bf16

__device__ __attribute__((aligned(16))) uint4 g_se_ws_zero[4];  // DMA source of padding lanes


__device__ __forceinline__ void dma16(const void* src, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_wave_base)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)p; }

// flag poll: one ds_read (all lanes read the same dword), then a scalar copy; bounded by `spin_max` polls
// (0: the wait fails at once, the fault injection of m2s_acoustic_set_ws_spin_limit).  false = timed out
__device__ __forceinline__ bool wait_flag(uint32_t addr, unsigned target, unsigned spin_max) {
  for (unsigned i = 0; i < spin_max; ++i) {
    unsigned v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    if (__builtin_amdgcn_readfirstlane(v) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
__device__ __forceinline__ void bump_flag(uint32_t addr, int lane) {
  if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(addr), "v"(1u) : "memory");
}

struct SeWsArgs {
  const uint8_t* x;       // interleaved split activations; F8: e4m3 [M][cs_in]
  const uint8_t* w;       // split weight rows; F8: e4m3 [n_pad][kp]
  const float* bias;      // [n_pad]
  const float* wscale;    // F8: per-output-channel weight scale [n_pad]
  const uint8_t* gate;    // split gates; F8: bf16 [M / P][cs_in]
  const bf16_t* res;      // split skip or null; F8: bf16 [M][cs_out]
  bf16_t* y;              // split output; F8: bf16 [M][cs_out]
  uint8_t* y8;            // F8: e4m3 copy of y (the next IR block's expand operand, rows of ld8 bytes) or null
  int M, P, cs_in, cs_out, n_tiles_m, kp;  // kp: F8 weight row bytes (cs_in rounded up to 128)
  // tail balancing: tiles >= full_tiles are half tiles of BM / 2 rows (n_tiles_m counts both kinds), launch_cfg
  int full_tiles;
  int ld8;
  unsigned spin_max;  // polls per flag wait before it times out
  unsigned* err;      // host-mapped error word (M2S_ASYNC_WS on a timeout) or null
};

constexpr int E8M0_ONE = 0x7f7f7f7f;  // 2^0 block scale in every byte
typedef int i32x8 __attribute__((ext_vector_type(8)));
// physical 16-byte chunk of logical chunk c in LDS row r: c ^ f(r).  Split rows: a fragment reads chunks g (hi)
// and g + 4 (lo) of row r16, f(r) = r & 6; e4m3 rows (F8): chunks 2g and 2g + 1, f(r) = ((r >> 1) & 1) | (r & 4).
// Both are conflict-free for ds_read_b128's lane groups (gemm128.hip swz128 / f8_swz)
template <bool F8>
__device__ __forceinline__ int swz_k(int r) { return F8 ? (((r >> 1) & 1) | (r & 4)) : (r & 6); }
// 4 e4m3 (one dword) x 4 gates -> 4 e4m3 (gemm128.hip gate4; the gate is in (0, 1): no new saturation)
__device__ __forceinline__ int gate4_f8(int d, const float* s) {
  const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(d, false);
  const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(d, true);
  const int r = __builtin_amdgcn_cvt_pk_fp8_f32(lo[0] * s[0], lo[1] * s[1], 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(hi[0] * s[2], hi[1] * s[3], r, true);
}

// NS ring slots; a loader keeps IF steps in flight behind the one it publishes (IF <= NS - 1).  F8: the fp8
// engines' e4m3 form (K step = 128 e4m3 channels, v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales,
// the gate applied to the e4m3 activation fragments in registers, wscale in the epilogue, bf16 in / out) of
// gemm128.hip KIND_F8_SE, on the same ring.
// XF (split engine only): the activations are plain fp32 rows [M][cs_in] (ir_ws's expanded map, launch_ir_ws fm32):
// a K step's 32 channels are still one 128-byte row, a fragment's 8 channels its chunks 2g, 2g + 1 (the e4m3 rows'
// swizzle), and the gating multiplies the fp32 value before the one split -- no hi + lo sum, and ir_ws's consumers
// store one 16-byte vector per 4 channels instead of splitting them.
template <int WM, int WN, int NT, int NL, int NS, int IF, bool F8, bool XF = false>
__global__ void __launch_bounds__(64 * (WM * WN + NL), 1) se_ws_kernel(const SeWsArgs a) {
  static_assert(!(F8 && XF), "fp32 activations: split engine");
  constexpr int NC = WM * WN;                       // consumer waves
  constexpr int BM = 64 * WM, BN = 16 * NT * WN, MT = 4;
  constexpr int BLK = (BN + BM) / 8;                // 8-row (1 KB) DMA blocks per step: weights, then activations
  static_assert(BLK % NL == 0, "DMA blocks per loader");
  constexpr int PER = BLK / NL;                     // DMAs per loader wave per step
  static_assert((IF + 1) * PER <= 63 && IF >= 1 && IF <= NS - 1, "steps in flight per loader within vmcnt");
  constexpr int SLOT = (BN + BM) * ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nimg = BM / a.P > 0 ? BM / a.P : 1;     // images a tile covers (P % BM == 0 or BM % P == 0)
  const int grow = F8 ? a.cs_in * 2 : a.cs_in * 4;  // bytes of one image's gate row (bf16 / split bf16)
  const int gimg = (grow + 1023) / 1024 * 1024;     // ... in LDS
  char* gbuf = smem + NS * SLOT;                    // [2][nimg][gimg]
  unsigned* flags = reinterpret_cast<unsigned*>(gbuf + 2 * nimg * gimg);  // FULL[NS], FREE[NS]
  const uint32_t full0 = lds_u32(flags), free0 = lds_u32(flags + NS), poison = lds_u32(flags + 2 * NS);
  const int nsteps = F8 ? a.kp / 128 : a.cs_in / 32;
  const int n_tiles = a.n_tiles_m;                  // one n tile: BN covers cs_out
  const int my_tiles = (int)blockIdx.x < n_tiles ? (n_tiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  // tile -> first row and row end: BM rows, or BM / 2 past full_tiles (the last round's tail, split so that the
  // workgroups' tile counts even out: 1920 16x16 images on 256 CUs were 7 or 8 tiles a workgroup)
  auto tile_rows = [&](int tile, int& m0, int& mend) {
    m0 = tile < a.full_tiles ? tile * BM : a.full_tiles * BM + (tile - a.full_tiles) * (BM / 2);
    mend = min(m0 + (tile < a.full_tiles ? BM : BM / 2), a.M);
  };

  if (tid <= 2 * NS) flags[tid] = 0u;  // FULL, FREE and the loaders' poison word
  __syncthreads();  // the only workgroup barrier

  if (wave >= NC) {
    // ---------------------------------------------------------------- loaders
    const int l = wave - NC;
    const char* zp = reinterpret_cast<const char*>(g_se_ws_zero);
    const int lrow = lane >> 3, pch = lane & 7;
    // this loader's blocks b = l + NL j: weight rows (b < BN / 8) or activation rows; a lane's row and
    // logical chunk follow from (b, lane) with a few integer ops per DMA (precomputed per block they were
    // 3 x PER registers, which spilled the consumer role)
    const int wrow_b = F8 ? a.kp : a.cs_in * 4, wlo = a.cs_in * 2, xrow_b = F8 ? a.cs_in : a.cs_in * 4;
    int s = 0;
    for (int it = 0; it < my_tiles; ++it) {
      const int tile = blockIdx.x + it * gridDim.x;
      int m0, mend;
      tile_rows(tile, m0, mend);
      const uint8_t* xt = a.x + (size_t)m0 * xrow_b;
      for (int st = 0; st < nsteps; ++st, ++s) {
        const int slot = s % NS, use = s / NS;
        if (use > 0 && !wait_flag(free0 + 4 * slot, (unsigned)(NC * use), a.spin_max)) {
          // a FREE timeout: the refill below may overwrite a slot a consumer still reads, so the poison word makes
          // every consumer store NaN from its next epilogue on (written and retired before the DMA is issued)
          report_async(a.err, M2S_ASYNC_WS, lane);
          if (lane == 0) asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(poison), "v"(1u) : "memory");
        }
        if (st == 0 && l == 0) {  // the tile's gate rows: nimg x 2 cs_in bf16, 16 B a lane
          const int img0 = m0 / a.P, nb = grow / 16;
          char* gdst = gbuf + (it & 1) * nimg * gimg;
          for (int im = 0; im < nimg; ++im)
            for (int o = 0; o < gimg / 16; o += 64) {
              const int e = o + lane;
              const bool ok = e < nb && (img0 + im) * a.P < a.M;
              const void* src = ok ? static_cast<const void*>(a.gate + ((size_t)(img0 + im) * grow + e * 16))
                                   : static_cast<const void*>(zp);
              dma16(src, lds_u32(gdst + im * gimg + o * 16));
            }
        }
        char* base = smem + slot * SLOT;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
          const int b = l + NL * j, r = b * 8 + lrow;
          const int c = pch ^ ((XF && b >= BN / 8) ? swz_k<true>(r & 15) : swz_k<F8>(r & 15));
          const void* src;
          if (b < BN / 8) {
            src = F8 ? a.w + ((size_t)r * wrow_b + st * ROWB + c * 16)
                     : a.w + ((size_t)r * wrow_b + (c < 4 ? c * 16 : wlo + (c - 4) * 16) + st * 64);
          } else {
            const int m = m0 + r - BN;
            const bool in = m < mend && (!F8 || st * ROWB + c * 16 < a.cs_in);  // F8: zeros past cs_in
            src = in ? static_cast<const void*>(xt + ((r - BN) * xrow_b + c * 16 + st * ROWB)) : static_cast<const void*>(zp);
          }
          dma16(src, lds_u32(base + b * 1024));
        }
        if (s >= IF) {  // step s - IF landed: everything but the IF younger steps' DMAs retired
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IF * PER) : "memory");
          bump_flag(full0 + 4 * ((s - IF) % NS), lane);
        }
      }
    }
    // the last IF steps (fewer if the workgroup had fewer steps), oldest first
#pragma unroll
    for (int k = IF - 1; k >= 0; --k) {
      const int q = s - 1 - k;
      if (q < 0 || q < s - IF) continue;
      if (k == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
      else if (k == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bump_flag(full0 + 4 * (q % NS), lane);
    }
    return;
  }

  // ---------------------------------------------------------------- consumers
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, r16 = lane & 15;
  const int sw = swz_k<F8>(r16);
  // a lane's two 16-byte chunks of a fragment row: split hi g / lo g + 4; F8 e4m3 2g, 2g + 1 (32 consecutive k)
  const uint32_t ch0 = (uint32_t)(((F8 ? 2 * g : g) ^ sw) << 4), ch1 = (uint32_t)(((F8 ? 2 * g + 1 : g + 4) ^ sw) << 4);
  const uint32_t sm0 = lds_u32(smem);
  const uint32_t a_lds0 = sm0 + (uint32_t)((wn * NT * 16 + r16) * ROWB);
  const uint32_t b_lds0 = sm0 + (uint32_t)((BN + wm * 64 + r16) * ROWB);
  // XF: the activation rows' chunks (fp32 rows: chunks 2g, 2g + 1 under the e4m3 rows' swizzle), folded into the row base
  // (one register more than the split form, whose 16 x 16 variant sits at 255)
  const uint32_t bx0 = XF ? b_lds0 + (uint32_t)(((2 * g) ^ swz_k<true>(r16)) << 4) : 0u;
  const uint32_t bx1 = XF ? b_lds0 + (uint32_t)(((2 * g + 1) ^ swz_k<true>(r16)) << 4) : 0u;
  const uint32_t wa0 = XF ? a_lds0 + ch0 : 0u, wa1 = XF ? a_lds0 + ch1 : 0u;  // XF: the weight chunks folded likewise
  const uint32_t g_lds0 = lds_u32(gbuf) + (uint32_t)(g * (F8 ? 64 : 16));
  bool bad = false;  // a FULL wait (or a loader's FREE wait) timed out: this wave's tiles are stored as NaN from then on
  int s = 0;
  for (int it = 0; it < my_tiles; ++it) {
    const int tile = blockIdx.x + it * gridDim.x;
    int m0, mend;
    tile_rows(tile, m0, mend);
    // a half tile's upper waves have no rows: they keep the flag protocol (FULL before their FREE, so no wave gets a
    // step ahead of the ring) and skip the reads, MFMAs and stores
    const bool active = m0 + wm * 64 < mend;
    const int wimg = (min(m0 + wm * 64, a.M - 1)) / a.P - m0 / a.P;  // this wave's image within the tile
    const uint32_t gl = g_lds0 + (uint32_t)(((it & 1) * nimg + wimg) * gimg);
    f32x4 acc[NT][MT];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) acc[ni][mi] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int st = 0; st < nsteps; ++st, ++s) {
      const int slot = s % NS, use = s / NS;
      if (!wait_flag(full0 + 4 * slot, (unsigned)(NL * (use + 1)), a.spin_max)) {
        report_async(a.err, M2S_ASYNC_WS, lane);
        bad = true;
      }
      if (!active) {  // nothing to read: release the slot at once
        bump_flag(free0 + 4 * slot, lane);
        continue;
      }
      const uint32_t so = (uint32_t)(slot * SLOT);
      if constexpr (F8) {
        // the lane's 32 gates k = 128 st + 32 g + j (bf16) and its MT activation fragments (e4m3 chunks 2g,
        // 2g + 1 of a row), then the NT weight fragments; released once every read returned
        u32x4 q[4], b0[MT], b1[MT], a0[NT], a1[NT];
        const uint32_t ga = gl + (uint32_t)(st * 256), ba0 = b_lds0 + so + ch0, ba1 = b_lds0 + so + ch1;
        asm volatile(
            "ds_read_b128 %0, %12\n\tds_read_b128 %1, %12 offset:16\n\tds_read_b128 %2, %12 offset:32\n\t"
            "ds_read_b128 %3, %12 offset:48\n\tds_read_b128 %4, %13\n\tds_read_b128 %5, %14\n\t"
            "ds_read_b128 %6, %13 offset:2048\n\tds_read_b128 %7, %14 offset:2048\n\tds_read_b128 %8, %13 offset:4096\n\t"
            "ds_read_b128 %9, %14 offset:4096\n\tds_read_b128 %10, %13 offset:6144\n\tds_read_b128 %11, %14 offset:6144\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(b0[0]), "=&v"(b1[0]), "=&v"(b0[1]), "=&v"(b1[1]),
              "=&v"(b0[2]), "=&v"(b1[2]), "=&v"(b0[3]), "=&v"(b1[3])
            : "v"(ga), "v"(ba0), "v"(ba1)
            : "memory");
        static_assert(MT == 4, "the read statement above covers four 16-row fragments");
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const uint32_t aa = a_lds0 + so + (uint32_t)(ni * 16 * ROWB);
          asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3" : "=&v"(a0[ni]), "=&v"(a1[ni]) : "v"(aa + ch0), "v"(aa + ch1) : "memory");
        }
        float gs[32];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          unpack_bf16x4(make_uint2(q[i][0], q[i][1]), gs + 8 * i);
          unpack_bf16x4(make_uint2(q[i][2], q[i][3]), gs + 8 * i + 4);
        }
#pragma unroll
        for (int mi = 0; mi < MT; ++mi) {
          i32x8 bx;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            bx[i] = gate4_f8((int)b0[mi][i], gs + 4 * i);
            bx[4 + i] = gate4_f8((int)b1[mi][i], gs + 16 + 4 * i);
          }
          if (mi == 0) {  // every read of the slot returned: release it to the loaders
            static_assert(NT <= 8, "wait operands");
            if constexpr (NT == 4)
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0[0]), "+v"(a1[0]), "+v"(a0[1]), "+v"(a1[1]), "+v"(a0[2]),
                           "+v"(a1[2]), "+v"(a0[3]), "+v"(a1[3])::"memory");
            else
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0[0]), "+v"(a1[0]), "+v"(a0[1]), "+v"(a1[1]), "+v"(a0[2]),
                           "+v"(a1[2]), "+v"(a0[3]), "+v"(a1[3]), "+v"(a0[NT > 4 ? 4 : 0]), "+v"(a1[NT > 4 ? 4 : 0]),
                           "+v"(a0[NT > 5 ? 5 : 0]), "+v"(a1[NT > 5 ? 5 : 0]), "+v"(a0[NT > 6 ? 6 : 0]),
                           "+v"(a1[NT > 6 ? 6 : 0]), "+v"(a0[NT > 7 ? 7 : 0]), "+v"(a1[NT > 7 ? 7 : 0])::"memory");
            bump_flag(free0 + 4 * slot, lane);
          }
#pragma unroll
          for (int ni = 0; ni < NT; ++ni) {
            const i32x8 af = {(int)a0[ni][0], (int)a0[ni][1], (int)a0[ni][2], (int)a0[ni][3],
                              (int)a1[ni][0], (int)a1[ni][1], (int)a1[ni][2], (int)a1[ni][3]};
            acc[ni][mi] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bx, acc[ni][mi], 0, 0, 0, E8M0_ONE, 0,
                                                                           E8M0_ONE);
          }
        }
        continue;
      } else {
      // gates k = 32 st + 8 g + j (hi and lo halves) and the MT activation fragments first; their gating
      // runs while the NT weight fragments are read; the slot is released once those returned too
      u32x4 gh, glo, bh[MT], bl[MT], ah[NT], al[NT];
      const uint32_t ga = gl + (uint32_t)(st * 64), ba0 = XF ? bx0 + so : b_lds0 + so + ch0, ba1 = XF ? bx1 + so : b_lds0 + so + ch1;
      const uint32_t gal = ga + (uint32_t)(a.cs_in * 2);  // the lo halves of the gate row
      asm volatile(
          "ds_read_b128 %0, %10\n\tds_read_b128 %1, %13\n\t"
          "ds_read_b128 %2, %11\n\tds_read_b128 %3, %12\n\tds_read_b128 %4, %11 offset:2048\n\t"
          "ds_read_b128 %5, %12 offset:2048\n\tds_read_b128 %6, %11 offset:4096\n\tds_read_b128 %7, %12 offset:4096\n\t"
          "ds_read_b128 %8, %11 offset:6144\n\tds_read_b128 %9, %12 offset:6144\n\ts_waitcnt lgkmcnt(0)"
          : "=&v"(gh), "=&v"(glo), "=&v"(bh[0]), "=&v"(bl[0]), "=&v"(bh[1]), "=&v"(bl[1]), "=&v"(bh[2]), "=&v"(bl[2]),
            "=&v"(bh[3]), "=&v"(bl[3])
          : "v"(ga), "v"(ba0), "v"(ba1), "v"(gal)
          : "memory");
      static_assert(MT == 4, "the read statement above covers four 16-row fragments");
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const uint32_t aa = (XF ? so : a_lds0 + so) + (uint32_t)(ni * 16 * ROWB);
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3"
                     : "=&v"(ah[ni]), "=&v"(al[ni])
                     : "v"(XF ? wa0 + aa : aa + ch0), "v"(XF ? wa1 + aa : aa + ch1)
                     : "memory");
      }
      // gate hi + lo (fp32), gated activations re-split (17 significant bits kept)
      float gsc[8], gl8[8];
      unpack_bf16x4(make_uint2(gh[0], gh[1]), gsc);
      unpack_bf16x4(make_uint2(gh[2], gh[3]), gsc + 4);
      unpack_bf16x4(make_uint2(glo[0], glo[1]), gl8);
      unpack_bf16x4(make_uint2(glo[2], glo[3]), gl8 + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) gsc[j] += gl8[j];
      // per activation fragment: gate + re-split, then its NT x 3 MFMAs (the next fragment's VALU
      // overlaps them); the slot is released after the first fragment, once the weight reads returned
      auto gate_frag = [&](int mi, bf16x8& xh, bf16x8& xl) {
        float v[8];
        if constexpr (XF) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = __uint_as_float(bh[mi][j]) * gsc[j];
            v[4 + j] = __uint_as_float(bl[mi][j]) * gsc[4 + j];
          }
        } else {
          float w[8];
          unpack_bf16x4(make_uint2(bh[mi][0], bh[mi][1]), v);
          unpack_bf16x4(make_uint2(bh[mi][2], bh[mi][3]), v + 4);
          unpack_bf16x4(make_uint2(bl[mi][0], bl[mi][1]), w);
          unpack_bf16x4(make_uint2(bl[mi][2], bl[mi][3]), w + 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (v[j] + w[j]) * gsc[j];
        }
        uint2 h0, l0, h1, l1;
        split4(v, h0, l0);
        split4(v + 4, h1, l1);
        xh = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
        xl = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
      };
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        bf16x8 xh, xl;
        gate_frag(mi, xh, xl);
        if (mi == 0) {  // every read of the slot returned: release it to the loaders
          static_assert(NT <= 8, "wait operands");
          if constexpr (NT == 4)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ah[0]), "+v"(al[0]), "+v"(ah[1]), "+v"(al[1]), "+v"(ah[2]),
                         "+v"(al[2]), "+v"(ah[3]), "+v"(al[3])::"memory");
          else
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ah[0]), "+v"(al[0]), "+v"(ah[1]), "+v"(al[1]), "+v"(ah[2]),
                         "+v"(al[2]), "+v"(ah[3]), "+v"(al[3]), "+v"(ah[NT > 4 ? 4 : 0]), "+v"(al[NT > 4 ? 4 : 0]),
                         "+v"(ah[NT > 5 ? 5 : 0]), "+v"(al[NT > 5 ? 5 : 0]), "+v"(ah[NT > 6 ? 6 : 0]),
                         "+v"(al[NT > 6 ? 6 : 0]), "+v"(ah[NT > 7 ? 7 : 0]), "+v"(al[NT > 7 ? 7 : 0])::"memory");
          bump_flag(free0 + 4 * slot, lane);
        }
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const bf16x8 wh = __builtin_bit_cast(bf16x8, ah[ni]), wl = __builtin_bit_cast(bf16x8, al[ni]);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh, acc[ni][mi], 0, 0, 0);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl, acc[ni][mi], 0, 0, 0);
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh, acc[ni][mi], 0, 0, 0);
        }
      }
      }
    }
    {  // a loader's FREE wait timed out (its refill may have overwritten a slot this wave read): NaN from here on
      unsigned pz;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(pz) : "v"(poison) : "memory");
      bad = bad || __builtin_amdgcn_readfirstlane(pz) != 0u;
    }

    if constexpr (F8) {  // bf16 out = wscale * acc + bias (+ skip), skip rows fetched first
      uint2 rv[MT][NT];
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const int m = m0 + wm * 64 + mi * 16 + r16, n4 = wn * NT * 16 + ni * 16 + 4 * g;
          rv[mi][ni] = (a.res && m < mend && n4 < a.cs_out) ? *reinterpret_cast<const uint2*>(a.res + (size_t)m * a.cs_out + n4)
                                                           : make_uint2(0u, 0u);
        }
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int m = m0 + wm * 64 + mi * 16 + r16;
        if (m >= mend) continue;
#pragma unroll
        for (int ni = 0; ni < NT; ++ni) {
          const int n4 = wn * NT * 16 + ni * 16 + 4 * g;
          if (n4 >= a.cs_out) continue;
          const float4 bb = *reinterpret_cast<const float4*>(a.bias + n4);
          const float4 ws = *reinterpret_cast<const float4*>(a.wscale + n4);
          float r[4];
          unpack_bf16x4(rv[mi][ni], r);
          float v[4] = {fmaf(acc[ni][mi][0], ws.x, bb.x) + r[0], fmaf(acc[ni][mi][1], ws.y, bb.y) + r[1],
                        fmaf(acc[ni][mi][2], ws.z, bb.z) + r[2], fmaf(acc[ni][mi][3], ws.w, bb.w) + r[3]};
          if (bad) v[0] = v[1] = v[2] = v[3] = __builtin_nanf("");
          const uint2 yb = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
          *reinterpret_cast<uint2*>(a.y + (size_t)m * a.cs_out + n4) = yb;
          // e4m3 of the stored bf16 values: the bytes launch_rows_e4m3 gives (test_fp8_se_y8_e4m3_handoff_is_exact)
          if (a.y8) *reinterpret_cast<uint32_t*>(a.y8 + (size_t)m * a.ld8 + n4) = e4m3x4_bf16(yb);
        }
      }
      continue;
    }
    // ---- epilogue: lane = 4 consecutive output channels of one position.  The skip rows of fragment
    // mi + 1 are fetched while fragment mi is finished (all of them at once spilled the NT = 7 variant)
    const bf16_t* __restrict__ R = a.res;
    bf16_t* __restrict__ Y = a.y;
    float4 bias4[NT];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int n4 = wn * NT * 16 + ni * 16 + 4 * g;
      bias4[ni] = n4 < a.cs_out ? *reinterpret_cast<const float4*>(a.bias + n4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    auto load_res = [&](int mi, uint2 (&rv)[NT][2]) {
      const int m = m0 + wm * 64 + mi * 16 + r16;
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int n4 = wn * NT * 16 + ni * 16 + 4 * g;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          rv[ni][h] = (R && m < mend && n4 < a.cs_out)
                          ? *reinterpret_cast<const uint2*>(R + (size_t)m * a.cs_out * 2 + h * a.cs_out + n4)
                          : make_uint2(0u, 0u);
      }
    };
    uint2 rv[2][NT][2];
    load_res(0, rv[0]);
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) {
      if (mi + 1 < MT) load_res(mi + 1, rv[(mi + 1) & 1]);
      const int m = m0 + wm * 64 + mi * 16 + r16;
      if (m >= mend) continue;
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) {
        const int n4 = wn * NT * 16 + ni * 16 + 4 * g;
        if (n4 >= a.cs_out) continue;
        const float4 bb = bias4[ni];
        float r[4], rl[4];
        unpack_bf16x4(rv[mi & 1][ni][0], r);
        unpack_bf16x4(rv[mi & 1][ni][1], rl);
        float v[4] = {acc[ni][mi][0] + bb.x + (r[0] + rl[0]), acc[ni][mi][1] + bb.y + (r[1] + rl[1]),
                      acc[ni][mi][2] + bb.z + (r[2] + rl[2]), acc[ni][mi][3] + bb.w + (r[3] + rl[3])};
        if (bad) v[0] = v[1] = v[2] = v[3] = __builtin_nanf("");
        uint2 hi, lo;
        split4(v, hi, lo);
        bf16_t* yo = Y + (size_t)m * a.cs_out * 2 + n4;
        *reinterpret_cast<uint2*>(yo) = hi;
        *reinterpret_cast<uint2*>(yo + a.cs_out) = lo;
      }
    }
  }
}

template <int WM, int WN, int NT, int NL, int NS, int IF, bool F8 = false, bool XF = false>
void launch_cfg(SeWsArgs& a, hipStream_t s, double flops, double bytes) {
  static_assert(IF <= 3, "tail waits");
  constexpr int BM = 64 * WM, BN = 16 * NT * WN;
  const void* fn = reinterpret_cast<const void*>(&se_ws_kernel<WM, WN, NT, NL, NS, IF, F8, XF>);
  allow_lds(fn);
  const int nimg = BM / a.P > 0 ? BM / a.P : 1;
  const int gimg = ((F8 ? a.cs_in * 2 : a.cs_in * 4) + 1023) / 1024 * 1024;
  const size_t lds = (size_t)NS * (BN + BM) * ROWB + (size_t)2 * nimg * gimg + (2 * NS + 1) * sizeof(unsigned);
  M2S_CHECK(lds <= 160 * 1024, "se_ws: LDS budget");
  M2S_CHECK(BM % a.P == 0 || a.P % BM == 0, "se_ws: tile rows vs image size");
  M2S_CHECK(a.cs_out <= BN, "se_ws: one n tile covers the outputs");
  M2S_CHECK((F8 ? a.kp / 128 : a.cs_in / 32) >= NS, "se_ws: K steps per tile >= ring slots (gate rows are double-buffered per tile)");
  // tail balancing (M2S_SEWS_HALF=1, off by default): when the last round's tiles would fill at most half the
  // workgroups, they run as twice as many half tiles (BM / 2 rows, still whole 64-row consumer blocks and whole images
  // or halves of one) spread over them.  Parity-green, but a half tile costs about a full one here (the weight rows,
  // the ring and the flag protocol stay; half the consumers idle): same-box CNN 31.36 / 31.68 ms off, 31.54 / 31.51 on
  // (gpurun_out/r06i/ab.txt), unlike ir_ws's slice-range split
  const int tiles = ceil_div(a.M, BM), G = std::min(tiles, device_cus());
  const int full = tiles / G * G, rem = tiles - full;
  const bool halve = rem > 0 && 2 * rem <= G && (BM / 2) % 64 == 0 && ((BM / 2) % a.P == 0 || a.P % (BM / 2) == 0) &&
                     getenv("M2S_SEWS_HALF") && atoi(getenv("M2S_SEWS_HALF")) == 1;
  a.full_tiles = halve ? full : tiles;
  a.n_tiles_m = halve ? full + 2 * rem : tiles;
  const dim3 grid(G);
  char name[72];
  if (XF)
    snprintf(name, sizeof(name), "se_ws_kernel<%d, %d, %d, %d, %d, %d, false, true>", WM, WN, NT, NL, NS, IF);
  else
    snprintf(name, sizeof(name), "se_ws_kernel<%d, %d, %d, %d, %d, %d, %s>", WM, WN, NT, NL, NS, IF,
             F8 ? "true" : "false");  // rocprof's symbol
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((se_ws_kernel<WM, WN, NT, NL, NS, IF, F8, XF>), grid, dim3(64 * (WM * WN + NL)), lds, s, a);
  M2S_HIP(hipGetLastError());
}

}  // namespace

bool se_ws_supported(int P, int cs_in, int cs_out) {
  return cs_in % 32 == 0 && cs_in / 32 >= 5 && ((P % 256 == 0 && cs_out <= 128) || (P == 64 && cs_out > 128 && cs_out <= 224));
}

void launch_se_ws(const void* x, int M, int P, int cs_in, const void* w, int n_pad, const float* bias, const void* gate,
                  const void* res, void* y, int cs_out, hipStream_t s, double flops, double bytes, AsyncReport rep,
                  bool x_f32) {
  M2S_CHECK(se_ws_supported(P, cs_in, cs_out) && M % P == 0 && cs_out % 4 == 0, "se_ws: unsupported shape");
  M2S_CHECK(x && w && bias && gate && y && y != res && y != x, "se_ws: operand pointers");
  M2S_CHECK((double)M * cs_in * 4 < 2147483647.0 * 2, "se_ws: input too large");
  if (M <= 0) return;
  SeWsArgs a;
  std::memset(&a, 0, sizeof(a));
  a.x = static_cast<const uint8_t*>(x);
  a.w = static_cast<const uint8_t*>(w);
  a.bias = bias;
  a.gate = static_cast<const uint8_t*>(gate);
  a.res = static_cast<const bf16_t*>(res);
  a.y = static_cast<bf16_t*>(y);
  a.M = M;
  a.P = P;
  a.cs_in = cs_in;
  a.cs_out = cs_out;
  a.spin_max = rep.spin_max;
  a.err = rep.err;
  // tile / ring variants (M2S_SE_WS_CFG, A/B only; 0 = the default)
  static const int cfg = [] {
    const char* e = std::getenv("M2S_SE_WS_CFG");
    return e ? std::atoi(e) : 0;
  }();
  if (x_f32) {  // fp32 activations (ir_ws fm32): the default tiles only
    if (cs_out <= 128) {
      M2S_CHECK(n_pad >= 128, "se_ws: weight rows");
      return launch_cfg<4, 1, 8, 4, 3, 2, false, true>(a, s, flops, bytes);
    }
    M2S_CHECK(n_pad >= 224, "se_ws: weight rows");
    return launch_cfg<2, 2, 7, 4, 3, 2, false, true>(a, s, flops, bytes);
  }
  if (cs_out <= 128) {
    M2S_CHECK(n_pad >= 128, "se_ws: weight rows");
    switch (cfg) {
      case 1: return launch_cfg<4, 2, 4, 2, 3, 1>(a, s, flops, bytes);  // 256 x 128, 3 slots, 1 step in flight
      case 2: return launch_cfg<2, 2, 4, 4, 4, 2>(a, s, flops, bytes);  // 128 x 128, 4 slots, 2 in flight
      case 3: return launch_cfg<2, 2, 4, 4, 4, 1>(a, s, flops, bytes);  // 128 x 128, 4 slots, 1 in flight
      case 4: return launch_cfg<4, 2, 4, 4, 3, 2>(a, s, flops, bytes);  // 256 x 128, 8 consumers 64 x 64 each
      // 256 x 128 (one 16x16 image), 3 slots, 4 consumers of 64 rows x all 128 columns: each activation
      // fragment is gated and re-split by one wave instead of two (the 8-consumer 64 x 64 form above):
      // 408 -> 389 us per launch, same-box per-process A/B (profiles/r04_se_ws_wn1_kstats.txt)
      default: return launch_cfg<4, 1, 8, 4, 3, 2>(a, s, flops, bytes);
    }
  } else {
    M2S_CHECK(n_pad >= 224, "se_ws: weight rows");
    switch (cfg) {
      case 1: return launch_cfg<2, 2, 7, 2, 3, 1>(a, s, flops, bytes);  // 128 x 224 (two 8x8 images)
      default: return launch_cfg<2, 2, 7, 4, 3, 2>(a, s, flops, bytes);
    }
  }
}

bool se_ws_f8_supported(int P, int cs_in, int cs_out) {
  return cs_in % 16 == 0 && (cs_in + 127) / 128 >= 3 && ((P % 256 == 0 && cs_out <= 128) || (P == 64 && cs_out > 128 && cs_out <= 224));
}

void launch_se_ws_f8(const void* x8, int M, int P, int cs_in, const void* w8, int kp, int n_pad, const float* wscale,
                     const float* bias, const void* gate, const void* res, void* y, int cs_out, hipStream_t s, double flops,
                     double bytes, void* y8, int ld8, AsyncReport rep) {
  M2S_CHECK(se_ws_f8_supported(P, cs_in, cs_out) && kp % 128 == 0 && kp >= cs_in && M % P == 0 && cs_out % 4 == 0,
            "se_ws_f8: unsupported shape");
  M2S_CHECK(!y8 || (ld8 >= cs_out && ld8 % 16 == 0 && y8 != x8), "se_ws_f8: e4m3 output rows");
  M2S_CHECK(x8 && w8 && wscale && bias && gate && y && y != res && y != x8, "se_ws_f8: operand pointers");
  M2S_CHECK((double)M * cs_in < 2147483647.0, "se_ws_f8: input too large");
  if (M <= 0) return;
  SeWsArgs a;
  std::memset(&a, 0, sizeof(a));
  a.x = static_cast<const uint8_t*>(x8);
  a.w = static_cast<const uint8_t*>(w8);
  a.wscale = wscale;
  a.bias = bias;
  a.gate = static_cast<const uint8_t*>(gate);
  a.res = static_cast<const bf16_t*>(res);
  a.y = static_cast<bf16_t*>(y);
  a.M = M;
  a.P = P;
  a.cs_in = cs_in;
  a.cs_out = cs_out;
  a.kp = kp;
  a.y8 = static_cast<uint8_t*>(y8);
  a.ld8 = ld8;
  a.spin_max = rep.spin_max;
  a.err = rep.err;
  if (cs_out <= 128) {
    M2S_CHECK(n_pad >= 128, "se_ws_f8: weight rows");
    // 128 x 128 (half a 16x16 image), 4 consumers + 4 loaders, 4 slots: the 8-consumer 256-row tile of the
    // split form spills here (32 fp32 gates a lane next to e4m3 fragments)
    launch_cfg<2, 2, 4, 4, 4, 2, true>(a, s, flops, bytes);
  } else {
    M2S_CHECK(n_pad >= 224, "se_ws_f8: weight rows");
    launch_cfg<2, 2, 7, 4, 3, 2, true>(a, s, flops, bytes);  // 128 x 224 (two 8x8 images)
  }
}

}  // namespace m2s
