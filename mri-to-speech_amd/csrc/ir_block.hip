// Whole InvertedResidual block in one kernel (bf16), stride 1 on 16x16 maps (tf_efficientnetv2_b2
// blocks.3.1-3 and blocks.4.*): conv_pw 1x1 + bn1 + SiLU -> conv_dw 3x3 + bn2 + SiLU -> SqueezeExcite
// (mean -> conv_reduce + SiLU -> conv_expand + sigmoid -> x gate) -> conv_pwl 1x1 + bn3 (+ shortcut)
// (timm InvertedResidual / SqueezeExcite; mri_acoustic_model.py:28-34 builds the backbone).
//
// One workgroup (8 waves) per image.  The SE gate of a channel needs the whole image's mean of that
// channel before conv_pwl may consume it, so the unfused sequence writes the expanded map (256 pixels x
// up to 736 channels) to HBM and reads it back: 2 x 0.7 GB per block of 1920 frames.  Here the map never
// leaves the CU.  The kernel walks the expanded width twice in 32-channel slices:
//   pass 1: expand (MFMA) -> haloed LDS tile -> depthwise (v_dot2) -> SiLU -> per-channel sums only;
//   SE excitation on the channel means, inside the workgroup (VALU);
//   pass 2: expand -> tile -> depthwise -> SiLU -> x gate -> bf16.  The depthwise lane layout (lane =
//           8-channel group g, pixel r16) is exactly conv_pwl's B fragment, so the values go straight
//           into the conv_pwl MFMAs, which accumulate all 128 output channels of the image in VGPRs.
// Status (profiles/r01j_*): correct, but 0.99 ms per 1920-frame block against 0.8 ms for the unfused
// ir_pwdw + se_excite + SE-scaled GEMM sequence, so it is opt-in (M2S_IR_BLOCK=1).  SQ counters: the
// VALU (depthwise dot2 + SiLU, done twice) is busy ~53 % of the time and the barrier-separated phases
// never overlap MFMA with VALU (MFMA ~9 %); 16 waves per workgroup measured slower (1.19 ms).
// Wave w owns image rows 2w, 2w+1 (two 16-pixel MFMA column tiles) in every phase; its expand B
// fragments (x, 128 channels) stay in VGPRs for the whole kernel.  Per slice, the expand and conv_pwl
// weight fragments, the depthwise taps and the two biases arrive as one 18 KB stage of a 2-slot LDS-DMA
// ring, packed on the host in fragment order (model.cpp, Acoustic ctor):
//   [0, 8K)          expand A fragments, piece 2 ks + nt: W_pw[c0 + 16 nt + row][32 ks + 8 g + e]
//   [8K, 16K)        conv_pwl A fragments, piece on:      W_pwl[16 on + row][c0 + 8 g + e]
//   [16K, +1152)     depthwise taps [9][32] u32, bf16 in the channel's dword half (v_dot2 operand)
//   then bn1 bias [32] f32, bn2 bias [32] f32, zeros to 18K.
#include <algorithm>

#include "kernels.hpp"
#include "prof.hpp"

namespace m2s {
namespace {

#ifndef IB_MODE
#define IB_MODE 0  // ablation hooks for tools/_ibab.sh (0 in the library): 1 no depthwise LDS reads,
                   // 2 no SE excitation, 4 no ring wait, 8 no expand fragment reads, 16 no conv_pwl ones,
                   // 32 SiLU -> identity in the slice loop, 64 no depthwise dot2, 128 no squeeze reduction
#endif
#ifndef IB_WAVES
#define IB_WAVES 8
#endif
constexpr int IB_NW = IB_WAVES;                 // waves
constexpr int IB_RW = 16 / IB_NW;               // image rows per wave
constexpr int IB_NT = IB_NW * 64;               // threads
constexpr int IB_P = 256;                       // pixels (16 x 16)
constexpr int IB_HW = 18;                       // haloed tile width
constexpr int IB_PLANE = IB_HW * IB_HW * 16;    // one 8-channel plane of the haloed slice tile
constexpr int IB_CS = 128;                      // input / output channel stride
constexpr int IB_KS = IB_CS / 32;               // expand k-steps
constexpr int IB_NO = IB_CS / 16;               // conv_pwl n16 tiles
constexpr int IB_STAGE = 18 * 1024;
constexpr int IB_TAPS = 16 * 1024, IB_BEXP = IB_TAPS + 9 * 32 * 4, IB_BDW = IB_BEXP + 32 * 4;
constexpr int IB_CMAX = 736;                    // widest expanded stride (means / gates in LDS)
constexpr int IB_RDMAX = 32;
constexpr size_t IB_LDS = 2 * IB_STAGE + 4 * IB_PLANE + (IB_CMAX + IB_NW * 32 + IB_RDMAX) * sizeof(float);

struct IbArgs {
  const bf16_t* x;     // (N, 256, 128)
  const bf16_t* wst;   // [nsl][IB_STAGE bytes]
  const bf16_t* w1;    // SE conv_reduce [>= rd][kp1]
  const float* b1;     // [rd]
  const bf16_t* w2;    // SE conv_expand [>= cs_mid][32]
  const float* b2;     // [>= cs_mid]
  const float* bpwl;   // [128] (zero past cout)
  bf16_t* y;           // (N, 256, 128)
  int nsl, mid, cs_mid, rd, kp1, skip;
};

// 16 bytes per lane, global -> LDS (wave base in M0), issued as inline asm: the compiler then does not
// see the LDS write, and does not put conservative vmcnt(0)s before every later LDS access of the slice
// while the next stage is in flight.  Its own vmcnt counts stay correct (these ops only add younger or
// older outstanding loads); the kernel waits for the ring itself.
__device__ __forceinline__ void dma16(const void* src, void* lds_wave_base) {
  const uint32_t l = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)lds_wave_base;
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(l) : "memory", "m0");
}
__device__ __forceinline__ float dot2(uint32_t x, uint32_t w, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, x), __builtin_bit_cast(bf16x2_t, w), acc, false);
}
__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float act(float x) { return (IB_MODE & 32) ? x : silu(x); }
__device__ __forceinline__ void lds_barrier() {  // LDS writes visible, then the workgroup barrier
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__global__ void __launch_bounds__(IB_NT, 1) ir_block_kernel(const IbArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  char* tile = smem + 2 * IB_STAGE;
  float* mg = reinterpret_cast<float*>(tile + 4 * IB_PLANE);  // channel means, then gates
  float* red = mg + IB_CMAX;                                   // [IB_NW][32] squeeze partials
  float* hid = red + IB_NW * 32;                               // SE hidden layer
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const size_t img = (size_t)blockIdx.x * IB_P * IB_CS;
  const int nq = 2 * a.nsl;

  // stage q: slice q (pass 1: expand pieces + taps) or q - nsl (pass 2: all 18 pieces) -> slot q & 1
  auto stage_dma = [&](int q) {
    const int sl = q < a.nsl ? q : q - a.nsl;
    const char* src = reinterpret_cast<const char*>(a.wst) + (size_t)sl * IB_STAGE + lane * 16;
    char* dst = ring + (q & 1) * IB_STAGE;
#pragma unroll
    for (int p = wave; p < 18; p += IB_NW)
      if (q >= a.nsl || p < 8 || p >= 16) dma16(src + p * 1024, dst + p * 1024);
  };

  stage_dma(0);
  uint4 xb[IB_RW][IB_KS];  // expand B fragments: x[row 2w + i, col r16][32 ks + 8 g ..]
#pragma unroll
  for (int i = 0; i < IB_RW; ++i)
#pragma unroll
    for (int ks = 0; ks < IB_KS; ++ks)
      xb[i][ks] = *reinterpret_cast<const uint4*>(a.x + img + (size_t)(16 * (IB_RW * wave + i) + r16) * IB_CS + 32 * ks + 8 * g);
  for (int i = tid; i < 4 * IB_PLANE / 16; i += IB_NT) reinterpret_cast<uint4*>(tile)[i] = make_uint4(0u, 0u, 0u, 0u);
  // consume xb here: otherwise the compiler's waits for these loads land inside the slice loop, where
  // the hardware counter also counts the (invisible) ring DMA and they would drain the prefetch
#pragma unroll
  for (int i = 0; i < IB_RW; ++i)
#pragma unroll
    for (int ks = 0; ks < IB_KS; ++ks) asm volatile("" ::"v"(xb[i][ks].x), "v"(xb[i][ks].y), "v"(xb[i][ks].z), "v"(xb[i][ks].w));

  f32x4 po[IB_RW][IB_NO];
#pragma unroll
  for (int i = 0; i < IB_RW; ++i)
#pragma unroll
    for (int on = 0; on < IB_NO; ++on) po[i][on] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int q = 0; q < nq; ++q) {
    const bool p2 = q >= a.nsl;
    const int c0 = (p2 ? q - a.nsl : q) * 32;
    // stage q landed (the only vector-memory ops in flight are its DMA pieces); every wave is done
    // with stage q - 1's slot, the tile and the squeeze partials
    if (!(IB_MODE & 4)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (q + 1 < nq) stage_dma(q + 1);
    if (q > 0 && q <= a.nsl && tid < 32) {  // channel means of the slice pass 1 finished last iteration
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < IB_NW; ++w) t += red[w * 32 + tid];
      mg[(q - 1) * 32 + tid] = t * (1.0f / IB_P);
    }
    if ((IB_MODE & 2) && q == a.nsl) {
      for (int c = tid; c < a.cs_mid; c += IB_NT) mg[c] = 1.0f;
      __syncthreads();
    } else if (q == a.nsl) {
      // ---- SE excitation: conv_reduce + SiLU (16 threads per hidden unit), conv_expand + sigmoid ---
      __syncthreads();
      if (tid < 512) {
        const int r = tid >> 4, part = tid & 15;
        float s = 0.f;
        if (r < a.rd)
          for (int c = 8 * part; c < a.cs_mid; c += 128) {
            const uint4 w = *reinterpret_cast<const uint4*>(a.w1 + (size_t)r * a.kp1 + c);
            const float4 m0 = *reinterpret_cast<const float4*>(mg + c), m1 = *reinterpret_cast<const float4*>(mg + c + 4);
            s += lo_f(w.x) * m0.x + hi_f(w.x) * m0.y + lo_f(w.y) * m0.z + hi_f(w.y) * m0.w + lo_f(w.z) * m1.x +
                 hi_f(w.z) * m1.y + lo_f(w.w) * m1.z + hi_f(w.w) * m1.w;
          }
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) s += __shfl_xor(s, m);
        if (part == 0) hid[r] = r < a.rd ? silu(s + a.b1[r]) : 0.f;
      }
      __syncthreads();
      for (int c = tid; c < a.cs_mid; c += IB_NT) {
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < IB_RDMAX; r += 8) {  // conv_expand rows are 32 wide, zero past rd
          const uint4 w = *reinterpret_cast<const uint4*>(a.w2 + (size_t)c * IB_RDMAX + r);
          s += lo_f(w.x) * hid[r] + hi_f(w.x) * hid[r + 1] + lo_f(w.y) * hid[r + 2] + hi_f(w.y) * hid[r + 3] +
               lo_f(w.z) * hid[r + 4] + hi_f(w.z) * hid[r + 5] + lo_f(w.w) * hid[r + 6] + hi_f(w.w) * hid[r + 7];
        }
        mg[c] = c < a.mid ? sigmoidf_(s + a.b2[c]) : 0.f;
      }
      __syncthreads();
    }
    const char* st = ring + (q & 1) * IB_STAGE;

    // ---- conv_pw + bn1 + SiLU for this slice -> haloed tile (plane = 8-channel group) -------------
    {
      f32x4 ea[IB_RW][2];
#pragma unroll
      for (int i = 0; i < IB_RW; ++i)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) ea[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < IB_KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const bf16x8 af = (IB_MODE & 8) ? __builtin_bit_cast(bf16x8, xb[nt % IB_RW][ks ^ 1])
                                          : *reinterpret_cast<const bf16x8*>(st + (2 * ks + nt) * 1024 + lane * 16);
#pragma unroll
          for (int i = 0; i < IB_RW; ++i)
            ea[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8, xb[i][ks]), ea[i][nt], 0, 0, 0);
        }
      const float* bexp = reinterpret_cast<const float*>(st + IB_BEXP);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const float4 bb = *reinterpret_cast<const float4*>(bexp + 16 * nt + 4 * g);
#pragma unroll
        for (int i = 0; i < IB_RW; ++i) {
          const int hp = (IB_RW * wave + i + 1) * IB_HW + r16 + 1;
          *reinterpret_cast<uint2*>(tile + (2 * nt + (g >> 1)) * IB_PLANE + hp * 16 + (g & 1) * 8) =
              make_uint2(pack_bf16x2(act(ea[i][nt][0] + bb.x), act(ea[i][nt][1] + bb.y)),
                         pack_bf16x2(act(ea[i][nt][2] + bb.z), act(ea[i][nt][3] + bb.w)));
        }
      }
    }
    lds_barrier();

    // ---- conv_dw 3x3 + bn2: lane = (8-channel group g, pixel r16) of rows 2w, 2w + 1 --------------
    float dv[IB_RW][8];
    {
      const float* bdw = reinterpret_cast<const float*>(st + IB_BDW);
      const float4 b0 = *reinterpret_cast<const float4*>(bdw + 8 * g), b1 = *reinterpret_cast<const float4*>(bdw + 8 * g + 4);
#pragma unroll
      for (int i = 0; i < IB_RW; ++i) {
        dv[i][0] = b0.x; dv[i][1] = b0.y; dv[i][2] = b0.z; dv[i][3] = b0.w;
        dv[i][4] = b1.x; dv[i][5] = b1.y; dv[i][6] = b1.z; dv[i][7] = b1.w;
      }
      const uint32_t* taps = reinterpret_cast<const uint32_t*>(st + IB_TAPS);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const uint4 wl = (IB_MODE & 1) ? xb[0][t & 3] : *reinterpret_cast<const uint4*>(taps + t * 32 + 8 * g);
        const uint4 wh = (IB_MODE & 1) ? xb[IB_RW - 1][t & 3] : *reinterpret_cast<const uint4*>(taps + t * 32 + 8 * g + 4);
        const uint32_t w[8] = {wl.x, wl.y, wl.z, wl.w, wh.x, wh.y, wh.z, wh.w};
#pragma unroll
        for (int i = 0; i < IB_RW; ++i) {
          const uint4 in = (IB_MODE & 1) ? xb[i][(t + 1) & 3]
                                         : *reinterpret_cast<const uint4*>(tile + g * IB_PLANE +
                                                                           ((IB_RW * wave + i + t / 3) * IB_HW + r16 + t % 3) * 16);
          const uint32_t u[4] = {in.x, in.y, in.z, in.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (IB_MODE & 64) {
              dv[i][2 * j] += __uint_as_float(u[j] ^ w[2 * j]);
            } else {
              dv[i][2 * j] = dot2(u[j], w[2 * j], dv[i][2 * j]);
              dv[i][2 * j + 1] = dot2(u[j], w[2 * j + 1], dv[i][2 * j + 1]);
            }
          }
        }
      }
    }

    if (!p2) {
      // ---- squeeze: SiLU, sum the wave's 32 pixels per channel (16-lane xor tree) -> red ----------
      float s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] = act(dv[0][j]);
#pragma unroll
        for (int i = 1; i < IB_RW; ++i) s[j] += act(dv[i][j]);
      }
#pragma unroll
      for (int m = 1; m < 16; m <<= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (IB_MODE & 128) ? s[(j + m) & 7] : __shfl_xor(s[j], m);
      if (r16 == 0) {
        *reinterpret_cast<float4*>(red + wave * 32 + 8 * g) = make_float4(s[0], s[1], s[2], s[3]);
        *reinterpret_cast<float4*>(red + wave * 32 + 8 * g + 4) = make_float4(s[4], s[5], s[6], s[7]);
      }
    } else {
      // ---- SiLU x gate -> bf16 B fragment -> conv_pwl (k = this slice's 32 channels) -------------
      const float4 g0 = *reinterpret_cast<const float4*>(mg + c0 + 8 * g), g1 = *reinterpret_cast<const float4*>(mg + c0 + 8 * g + 4);
      const float gt[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      bf16x8 mb[IB_RW];
#pragma unroll
      for (int i = 0; i < IB_RW; ++i) {
        uint32_t u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          u[j] = pack_bf16x2(act(dv[i][2 * j]) * gt[2 * j], act(dv[i][2 * j + 1]) * gt[2 * j + 1]);
        mb[i] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
      }
#pragma unroll
      for (int on = 0; on < IB_NO; ++on) {
        const bf16x8 wf = (IB_MODE & 16) ? __builtin_bit_cast(bf16x8, xb[on % IB_RW][(on >> 1) & 3])
                                         : *reinterpret_cast<const bf16x8*>(st + (8 + on) * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < IB_RW; ++i) po[i][on] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, mb[i], po[i][on], 0, 0, 0);
      }
    }
  }

  // ---- + bn3 bias (+ shortcut) -> y ---------------------------------------------------------------
#pragma unroll
  for (int on = 0; on < IB_NO; ++on) {
    const float4 bb = *reinterpret_cast<const float4*>(a.bpwl + 16 * on + 4 * g);
#pragma unroll
    for (int i = 0; i < IB_RW; ++i) {
      const size_t o = img + (size_t)(16 * (IB_RW * wave + i) + r16) * IB_CS + 16 * on + 4 * g;
      float v0 = po[i][on][0] + bb.x, v1 = po[i][on][1] + bb.y, v2 = po[i][on][2] + bb.z, v3 = po[i][on][3] + bb.w;
      if (a.skip) {
        const uint2 r = *reinterpret_cast<const uint2*>(a.x + o);
        v0 += lo_f(r.x);
        v1 += hi_f(r.x);
        v2 += lo_f(r.y);
        v3 += hi_f(r.y);
      }
      *reinterpret_cast<uint2*>(a.y + o) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    }
  }
}

}  // namespace

bool ir_block_supported(int H, int W, int cs_in, int cs_mid, int cs_out, int rd, int kp1, int kp2) {
  return H == 16 && W == 16 && cs_in == IB_CS && cs_out == IB_CS && cs_mid % 32 == 0 && cs_mid > 0 &&
         cs_mid <= IB_CMAX && rd >= 1 && rd <= IB_RDMAX && kp2 == IB_RDMAX && kp1 >= cs_mid;
}

int ir_block_stage_bytes() { return IB_STAGE; }

void launch_ir_block(const bf16_t* x, int N, const bf16_t* wst, int mid, int cs_mid, const bf16_t* w1, int kp1,
                     const float* b1, int rd, const bf16_t* w2, int kp2, const float* b2, const float* bpwl, bool skip,
                     bf16_t* y, double flops, double bytes, hipStream_t s) {
  M2S_CHECK(N > 0 && ir_block_supported(16, 16, IB_CS, cs_mid, IB_CS, rd, kp1, kp2) && mid <= cs_mid,
            "ir_block: unsupported shape");
  IbArgs a;
  a.x = x;
  a.wst = wst;
  a.w1 = w1;
  a.b1 = b1;
  a.w2 = w2;
  a.b2 = b2;
  a.bpwl = bpwl;
  a.y = y;
  a.nsl = cs_mid / 32;
  a.mid = mid;
  a.cs_mid = cs_mid;
  a.rd = rd;
  a.kp1 = kp1;
  a.skip = skip ? 1 : 0;
  static bool attr = [] {
    M2S_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ir_block_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)IB_LDS));
    return true;
  }();
  (void)attr;
  ProfScope ps("ir_block_kernel", flops, bytes, s);
  hipLaunchKernelGGL(ir_block_kernel, dim3(N), dim3(IB_NT), IB_LDS, s, a);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
