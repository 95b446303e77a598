// Fused EdgeResidual block in split fp32 (bf16x3), stride 1 with skip: timm EdgeResidual conv_exp
// 3x3 + bn1 + SiLU -> conv_pwl 1x1 + bn2 -> + shortcut (tf_efficientnetv2_b2 blocks.1.1/.2: 32 -> 128 ->
// 32 at 64x64, blocks.2.1/.2: 56 -> 224 -> 56 at 32x32; built by mri_acoustic_model.py:28-34).
//
// Unfused, conv_exp writes its mid-channel map as hi/lo pairs (4 B per channel: 4 GB per 1920 frames
// for blocks.1) and conv_pwl reads it back; here it stays in registers, as in er_fused.hip: the
// conv_exp accumulators of one 16-pixel subtile (lane = 4 consecutive mid channels of one pixel) are,
// after bias + SiLU, re-split into the hi and lo B fragments of conv_pwl, whose K the host packs in
// the matching permuted order (k-slot 8g+e of k-step s = channel 32s + 4g + e for e < 4, else
// 32s + 16 + 4g + e - 4).
//
// Split arithmetic: every product is W_hi*X_hi + W_hi*X_lo + W_lo*X_hi.  The weights stream through a
// 3-slot LDS ring in "stages" of NT 1-KB fragments (one MFMA A operand per 16 output channels): for
// each conv_exp k-step (tap, 32 input channels) a W_hi stage (MFMAs against the hi and the lo input
// fragments) and a W_lo stage (against the hi fragments); then conv_pwl's W_hi and W_lo stages.  The
// haloed input tile ((TH+2) x 18 pixels, hi and lo planes of every 8-channel chunk: planar, so a
// B-fragment read of 16 consecutive pixels is bank-conflict free) is double-buffered: the next tile's
// lands while this one computes.  Persistent workgroups of NW waves; wave w computes output rows
// RPW*w .. RPW*w + RPW - 1 of the 16-wide tile; one 8-wave workgroup per CU.  (Measured: blocks.1 as two
// independent 4-wave workgroups per CU on 8-row tiles, so that one's bias + SiLU + re-split phase could
// overlap the other's MFMAs, ran 2.03-2.09 ms per launch against 2.0 for the 8-wave 16-row form.)
//
// Waits are counted `s_waitcnt vmcnt`s over a fixed per-wave issue order: per stage PPW ring pieces,
// at stage 0 the next tile's 6 halo pieces, after the last stage ST output stores (the table in
// begin_stage).
#include <algorithm>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

__device__ __attribute__((aligned(16))) uint4 g_ersp_zero[4];

__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
// LDS read the compiler does not see (an ordinary ds_read after an LDS-DMA gets a conservative
// vmcnt(0), which would drain the ring's prefetch)
__device__ __forceinline__ uint2 lds_u2(const void* p) {
  uint2 r;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_off(p)));
  return r;
}
__device__ __forceinline__ float4 lds_f4(const void* p) {
  float4 r;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_off(p)));
  return r;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ bf16x8 frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct ErSpArgs {
  const bf16_t* x;    // (N, H, W, [hi CSI | lo CSI])
  const bf16_t* wst;  // stage stream [NST][NT][64][8] (er_sp_stream_layout)
  const float* bexp;  // [NT * 16] bn1 bias (zero padded)
  const float* bpwl;  // [ON * 16] bn2 bias (zero padded)
  bf16_t* y;          // (N, H, W, [hi 16 ON | lo 16 ON])
  int N, H, W, tiles_x, tiles_y;
};

// TH: tile rows (tile = TH x 16 output pixels); CSI: input channel stride (32 / 64); NT: mid channels / 16;
// ON: output channel stride / 16 (the skip needs ON * 16 == CSI)
// MRG = 2: one ring slot carries a W_hi stage and its W_lo stage (half the barriers; needs NPS == 1).
template <int TH, int CSI, int NT, int ON, int NW, int MRG>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) er_sp_kernel(const ErSpArgs a) {
  constexpr int TW = 16, HW = TW + 2, HH = TH + 2, HPIX = HH * HW;
  constexpr int HPB = (HPIX + 63) / 64;          // 64-pixel DMA pieces per (plane, chunk)
  constexpr int HPLANE = HPB * 1024;             // bytes per (plane, chunk)
  constexpr int CH = CSI / 8;                    // 16-byte chunks per pixel and plane
  constexpr int HBUF = 2 * CH * HPLANE;          // hi + lo planes
  constexpr int HP = 2 * CH * HPB / NW;          // halo pieces per wave
  static_assert((2 * CH * HPB) % NW == 0, "halo pieces must divide over the waves");
  constexpr int PPW = (MRG * NT + NW - 1) / NW;  // ring pieces per wave per stage
  constexpr int SLOT = PPW * NW * 1024;
  constexpr int KC = CSI / 32, NCE = 9 * KC * 2;  // conv_exp stages (k-step x plane)
  constexpr int MID = NT * 16, KS = MID / 32, PN = ON * KS;
  constexpr int NPS = (PN + NT - 1) / NT;        // conv_pwl stages per plane
  constexpr int NST = (NCE + 2 * NPS) / MRG;     // ring stages per tile
  static_assert(MRG == 1 || (MRG == 2 && NPS == 1 && NCE % 2 == 0), "merged stages");
  constexpr int RPW = TH / NW;                   // output rows (16-pixel subtiles) per wave
  constexpr int ST = RPW * ON * 2;               // output stores per wave per tile
  static_assert(NT % 2 == 0 && ON * 16 == CSI && TH % NW == 0, "er_sp shape");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  char* hbuf = smem + 3 * SLOT;
  float* bexp_l = reinterpret_cast<float*>(hbuf + 2 * HBUF);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int tpi = a.tiles_x * a.tiles_y, ntiles = a.N * tpi;

  // the zero page's address in SGPRs for the whole kernel: named directly in the DMA loops it was re-fetched from the
  // GOT (s_getpc + s_load + s_waitcnt lgkmcnt(0), which also drains the wave's LDS reads) at every piece
  const void* zpage = g_ersp_zero;
  asm volatile("" : "+s"(zpage));
  auto stage_dma = [&](int ls, int slot) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int piece = wave * PPW + j;
      const void* src = piece < MRG * NT ? (const void*)(a.wst + ((size_t)(ls * MRG * NT + piece) * 64 + lane) * 8) : zpage;
      dma16(src, ring + slot * SLOT + piece * 1024);
    }
  };
  auto halo_dma = [&](int tile, char* buf) {
    const int n = tile / tpi, tr = tile - n * tpi;
    const int ty0 = (tr / a.tiles_x) * TH - 1, tx0 = (tr - (tr / a.tiles_x) * a.tiles_x) * TW - 1;
    const bf16_t* xi = a.x + (size_t)n * a.H * a.W * (2 * CSI);
#pragma unroll
    for (int j = 0; j < HP; ++j) {
      const int piece = wave * HP + j, pc = piece / HPB, pb = piece - pc * HPB;  // pc = plane * CH + chunk
      const int p = pb * 64 + lane, hy = p / HW, hx = p - hy * HW;
      const int iy = ty0 + hy, ix = tx0 + hx;
      const void* src = zpage;
      if (p < HPIX && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        src = xi + ((size_t)iy * a.W + ix) * (2 * CSI) + (pc / CH) * CSI + (pc % CH) * 8;
      dma16(src, buf + pc * HPLANE + pb * 1024);
    }
  };

  for (int i = tid; i < MID; i += 64 * NW) bexp_l[i] = a.bexp[i];
  __syncthreads();  // bexp_l is read through lds_f4 (asm: no conservative vmcnt(0) before it)
  float4 bp[ON];
#pragma unroll
  for (int on = 0; on < ON; ++on) bp[on] = *reinterpret_cast<const float4*>(a.bpwl + on * 16 + 4 * g);

#ifndef ERSP_PRIO
#define ERSP_PRIO 1
#endif
  // the second-dispatched half of the waves loses every VALU issue arbitration to the first by age; one
  // static priority for it evens the halves' segments out (MI355X_MICROARCH.md, two waves per SIMD, item 4):
  // same-box A/B -1.7 % on the 16-row blocks.1 form, neutral on blocks.2 (profiles/r04_prio_kstats.txt)
  if (ERSP_PRIO && NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  int q = 0;  // global stage counter: ring slot = q % 3
  if ((int)blockIdx.x < ntiles) {
    stage_dma(0, 0);
    stage_dma(1, 1);
    halo_dma(blockIdx.x, hbuf);
  }
  for (int it = 0, tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    const bool has_next = tile + (int)gridDim.x < ntiles;
    const char* hb = hbuf + (it & 1) * HBUF;
    const int n = tile / tpi, tr = tile - n * tpi;
    const int oy0 = (tr / a.tiles_x) * TH, ox = (tr - (tr / a.tiles_x) * a.tiles_x) * TW + r16;

    // stage ls has landed once only the ops this wave issued after it are outstanding (issue order:
    // ... S(ls+1) ... ; stage 0 issues S2 then H(next); after the last stage the ST stores)
    auto begin_stage = [&](int ls) -> const char* {
      if (ls == 0) {
        if (it == 0) wait_vm<0>();
        else wait_vm<PPW + ST>();  // younger: S1, the last tile's stores
      } else if (ls == 1) {
        if (has_next) wait_vm<ST + PPW + HP>();  // younger: stores, S2, H(next)
        else wait_vm<ST + PPW>();
      } else if (ls == 2) {
        if (has_next) wait_vm<HP + PPW>();  // younger: H(next), S3
        else wait_vm<PPW>();
      } else if (ls + 1 < NST || has_next) {
        wait_vm<PPW>();  // younger: S(ls + 1)
      } else {
        wait_vm<0>();  // the last stage of the last tile
      }
      __builtin_amdgcn_s_barrier();  // every wave's pieces of stage ls landed; slot (q + 2) % 3 is free
      asm volatile("" ::: "memory");
      if (ls + 2 < NST) stage_dma(ls + 2, (q + 2) % 3);
      else if (has_next) stage_dma(ls + 2 - NST, (q + 2) % 3);
      if (ls == 0 && has_next) halo_dma(tile + gridDim.x, hbuf + ((it + 1) & 1) * HBUF);
      const char* ws = ring + (q % 3) * SLOT + lane * 16;
      ++q;
      return ws;
    };

    // ---- conv_exp: 9 taps x KC k-steps, each a W_hi stage and a W_lo stage -------------------------
    f32x4 acc[RPW][NT];
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int ks = 0; ks < 9 * KC; ++ks) {
      const int t = ks / KC, kc = ks - t * KC, ky = t / 3, kx = t - (t / 3) * 3;
      bf16x8 bh[RPW], bl[RPW];
      const char* wsm = MRG == 2 ? begin_stage(ks) : nullptr;  // merged: W_hi pieces [0, NT), W_lo [NT, 2 NT)
      {
        const char* ws = MRG == 2 ? wsm : begin_stage(2 * ks);  // W_hi
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const int pix = (RPW * wave + i + ky) * HW + r16 + kx;
          bh[i] = frag(hb + (kc * 4 + g) * HPLANE + pix * 16);
          bl[i] = frag(hb + (CH + kc * 4 + g) * HPLANE + pix * 16);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const bf16x8 af = frag(ws + nt * 1024);
#pragma unroll
          for (int i = 0; i < RPW; ++i) acc[i][nt] = mfma(af, bl[i], mfma(af, bh[i], acc[i][nt]));
        }
      }
      {
        const char* ws = MRG == 2 ? wsm + NT * 1024 : begin_stage(2 * ks + 1);  // W_lo
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const bf16x8 af = frag(ws + nt * 1024);
#pragma unroll
          for (int i = 0; i < RPW; ++i) acc[i][nt] = mfma(af, bh[i], acc[i][nt]);
        }
      }
    }

    // ---- bn1 bias + SiLU, re-split: n-tiles (2 kk, 2 kk + 1) become conv_pwl's B fragments of k-step kk
    bf16x8 mh[RPW][KS], ml[RPW][KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        float v[8];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int nt = 2 * kk + hh;
          const float4 bb = lds_f4(bexp_l + nt * 16 + 4 * g);
          v[4 * hh + 0] = silu(acc[i][nt][0] + bb.x);
          v[4 * hh + 1] = silu(acc[i][nt][1] + bb.y);
          v[4 * hh + 2] = silu(acc[i][nt][2] + bb.z);
          v[4 * hh + 3] = silu(acc[i][nt][3] + bb.w);
        }
        uint2 h0, l0, h1, l1;
        split4(v, h0, l0);
        split4(v + 4, h1, l1);
        mh[i][kk] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
        ml[i][kk] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
      }

    // ---- conv_pwl: NPS W_hi stages, NPS W_lo stages; piece j of a plane = (k-step j / ON, n16 j % ON)
    f32x4 o[RPW][ON];
#pragma unroll
    for (int i = 0; i < RPW; ++i)
#pragma unroll
      for (int on = 0; on < ON; ++on) o[i][on] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* wpm = MRG == 2 ? begin_stage(NCE / 2) : nullptr;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps) {
        const char* ws = MRG == 2 ? wpm + pl * NT * 1024 : begin_stage(NCE + pl * NPS + ps);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int j = ps * NT + nt;
          if (j >= PN) break;
          const int kk = j / ON, on = j - (j / ON) * ON;
          const bf16x8 af = frag(ws + nt * 1024);
#pragma unroll
          for (int i = 0; i < RPW; ++i) {
            o[i][on] = mfma(af, mh[i][kk], o[i][on]);
            if (pl == 0) o[i][on] = mfma(af, ml[i][kk], o[i][on]);
          }
        }
      }

    // ---- + bn2 bias + shortcut (hi + lo of the halo centre); ST hi/lo stores per wave ----------------
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int ry = RPW * wave + i, oy = oy0 + ry;
      const int cpix = ((ry + 1) * HW + r16 + 1) * 16;
#pragma unroll
      for (int on = 0; on < ON; ++on) {
        const int c4 = on * 16 + 4 * g;
        float rh[4], rl[4];
        unpack_bf16x4(lds_u2(hb + (c4 >> 3) * HPLANE + cpix + (c4 & 7) * 2), rh);
        unpack_bf16x4(lds_u2(hb + (CH + (c4 >> 3)) * HPLANE + cpix + (c4 & 7) * 2), rl);
        const float v[4] = {o[i][on][0] + bp[on].x + rh[0] + rl[0], o[i][on][1] + bp[on].y + rh[1] + rl[1],
                            o[i][on][2] + bp[on].z + rh[2] + rl[2], o[i][on][3] + bp[on].w + rh[3] + rl[3]};
        uint2 h, l;
        split4(v, h, l);
        bf16_t* yo = a.y + (((size_t)n * a.H + oy) * a.W + ox) * (2 * CSI) + c4;
        *reinterpret_cast<uint2*>(yo) = h;
        *reinterpret_cast<uint2*>(yo + CSI) = l;
      }
    }
  }
  wait_vm<0>();
}

template <int TH, int CSI, int NT, int ON, int NW, int MRG>
void launch_t(const ErSpArgs& a, const char* name, double flops, double bytes, hipStream_t s) {
  constexpr int HW = 18, HPB = ((TH + 2) * HW + 63) / 64, CH = CSI / 8, PPW = (MRG * NT + NW - 1) / NW;
  const size_t lds = 3 * (size_t)PPW * NW * 1024 + 2 * (size_t)(2 * CH * HPB * 1024) + NT * 16 * sizeof(float);
  M2S_CHECK(lds <= (NW == 4 ? 80 : 160) * 1024, "er_sp: LDS budget");
  allow_lds(reinterpret_cast<const void*>(&er_sp_kernel<TH, CSI, NT, ON, NW, MRG>));
  const int cus = device_cus();
  const int grid = std::min(a.N * a.tiles_x * a.tiles_y, (NW == 4 ? 2 : 1) * cus);
  ProfScope ps(name, flops, bytes, s);
  hipLaunchKernelGGL((er_sp_kernel<TH, CSI, NT, ON, NW, MRG>), dim3(grid), dim3(64 * NW), lds, s, a);
  M2S_HIP(hipGetLastError());
}

int tile_rows(int cs_in) { return cs_in == 32 ? 16 : 8; }

}  // namespace

bool er_sp_supported(int H, int W, int cs_in, int mid, int cs_out) {
  const bool shape = (cs_in == 32 && mid == 128 && cs_out == 32) || (cs_in == 64 && mid == 224 && cs_out == 64);
  return shape && H > 0 && W > 0 && W % 16 == 0 && H % tile_rows(cs_in) == 0;
}

int er_sp_nt_stages(int cs_in, int mid, int cs_out, int* nt) {
  *nt = mid / 16;
  const int kc = cs_in / 32, pn = (cs_out / 16) * (mid / 32);
  return 9 * kc * 2 + 2 * ((pn + *nt - 1) / *nt);
}

void launch_er_sp(const void* x, int N, int H, int W, int cs_in, int mid, int cs_out, const void* wst, const float* bexp,
                  const float* bpwl, void* y, double flops, double bytes, hipStream_t s, bool merged) {
  M2S_CHECK(er_sp_supported(H, W, cs_in, mid, cs_out) && N > 0, "er_sp: unsupported shape");
  ErSpArgs a;
  a.x = static_cast<const bf16_t*>(x);
  a.wst = static_cast<const bf16_t*>(wst);
  a.bexp = bexp;
  a.bpwl = bpwl;
  a.y = static_cast<bf16_t*>(y);
  a.N = N;
  a.H = H;
  a.W = W;
  a.tiles_x = W / 16;
  a.tiles_y = H / tile_rows(cs_in);
  if (cs_in == 32 && merged)
    launch_t<16, 32, 8, 2, 8, 2>(a, "er_sp_kernel<16, 32, 8, 2, 8, 2>", flops, bytes, s);
  else if (cs_in == 32)
    launch_t<16, 32, 8, 2, 8, 1>(a, "er_sp_kernel<16, 32, 8, 2, 8, 1>", flops, bytes, s);
  else
    launch_t<8, 64, 14, 4, 8, 1>(a, "er_sp_kernel<8, 64, 14, 4, 8, 1>", flops, bytes, s);
}

}  // namespace m2s
