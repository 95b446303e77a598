// Non-GEMM kernels of the hot path: stem, depthwise+SE, GAP, BiLSTM recurrence, head, mel glue,
// vocoder input/output edges.  All are HBM/latency-bound; each reads its input once.
#include <algorithm>

#include "kernels.hpp"

#include <type_traits>

namespace m2s {

namespace {

template <typename T>
__device__ __forceinline__ float act_silu(float v) {
  return sizeof(T) == 4 ? silu_exact(v) : silu(v);
}

// ---------------------------------------------------------------------------------------------
// stem: four lanes per output pixel, 8 channels each, so one wave's stores cover 16 whole pixel
// rows (1 KB contiguous in bf16) instead of 64 partial ones.  A lane keeps its 8 channels' 72
// taps + 8 biases in registers and walks pixels grid-stride (weights from LDS per pixel made the
// kernel LDS-issue bound).  TF-SAME pads passed from the host.
template <typename T>
__global__ void __launch_bounds__(256) stem_kernel(const float* __restrict__ frames, int N, int H, int W, int OH,
                                                   int OW, int pad_t, int pad_l, const float* __restrict__ w9,
                                                   const float* __restrict__ bias, int cout, int cs_out,
                                                   T* __restrict__ y) {
  const int o0 = (threadIdx.x & 3) * 8;
  if (o0 >= cs_out) return;
  float w[8][9], bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool ok = o0 + j < cout;
#pragma unroll
    for (int t = 0; t < 9; ++t) w[j][t] = ok ? w9[(o0 + j) * 9 + t] : 0.f;
    bb[j] = ok ? bias[o0 + j] : 0.f;
  }
  const long total = (long)N * OH * OW;
  const int hw = OH * OW;
  for (long p = ((long)blockIdx.x * 256 + threadIdx.x) >> 2; p < total; p += (long)gridDim.x * 64) {
    const int n = (int)(p / hw);
    const int rem = (int)(p - (long)n * hw);
    const int oy = rem / OW, ox = rem - (rem / OW) * OW;
    float in[9];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = oy * 2 - pad_t + ky, ix = ox * 2 - pad_l + kx;
        in[ky * 3 + kx] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? frames[((long)n * H + iy) * W + ix] : 0.f;
      }
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) acc += w[j][t] * in[t];
      v[j] = act_silu<T>(acc + bb[j]);
    }
    act_st8<T>(y, p, cs_out, o0, v);
  }
}

// stem, bf16 with 32 output channels: one thread per output pixel computes all 32 channels.  The
// 288 weights and 32 biases are wave-uniform, so they come through the scalar cache as SGPR
// operands of the FMAs (no VGPRs, no LDS), the 9 input taps are loaded once per pixel instead of
// once per 8-channel lane group, and a lane stores its pixel's 64 bytes (a wave: 4 KB contiguous).
__global__ void __launch_bounds__(256) stem32_kernel(const float* __restrict__ frames, int N, int H, int W, int OH,
                                                     int OW, int pad_t, int pad_l, const float* __restrict__ w9,
                                                     const float* __restrict__ bias, bf16_t* __restrict__ y) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const int hw = OH * OW;
  if (p >= (long)N * hw) return;
  const int n = (int)(p / hw);
  const int rem = (int)(p - (long)n * hw);
  const int oy = rem / OW, ox = rem - (rem / OW) * OW;
  const float* fr = frames + (long)n * H * W;
  float in[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int iy = oy * 2 - pad_t + ky, ix = ox * 2 - pad_l + kx;
      in[ky * 3 + kx] = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? fr[(long)iy * W + ix] : 0.f;
    }
  uint4* out = reinterpret_cast<uint4*>(y + p * 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float a0 = bias[q * 8 + j], a1 = bias[q * 8 + j + 1];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        a0 += w9[(q * 8 + j) * 9 + t] * in[t];
        a1 += w9[(q * 8 + j + 1) * 9 + t] * in[t];
      }
      o[j / 2] = pack_bf16x2(silu(a0), silu(a1));
    }
    out[q] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ---------------------------------------------------------------------------------------------
// One (image, 64-channel block) per workgroup: lane = channel, the four waves take every fourth position (four
// independent chains each) and their partial sums meet in LDS in a fixed order.  (One image per workgroup walking
// its 22 channel blocks was a 9.6 us launch at 32 frames; one thread per (image, channel) over all P positions 20 us.)
template <typename T>
__global__ void __launch_bounds__(256) gap_kernel(const T* __restrict__ x, int N, int P, int C, int cs,
                                                  float* __restrict__ feats) {
  __shared__ float part[4][64];
  const int n = blockIdx.x, q = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c = blockIdx.y * 64 + l;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int k = q;
    for (; k + 12 < P; k += 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += act_ld<T>(x, (long)n * P + k + 4 * j, cs, c);
    }
    for (; k < P; k += 4) a[0] += act_ld<T>(x, (long)n * P + k, cs, c);
  }
  part[q][l] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (q == 0 && c < C) feats[(long)n * C + c] = ((part[0][l] + part[1][l]) + (part[2][l] + part[3][l])) / (float)P;
}

// ---------------------------------------------------------------------------------------------
// BiLSTM step.  grid (H/8, ceil(B/32), 2); block = 8 hidden units x 32 sequences.  Each thread
// owns the 4 gates of one (unit, sequence); W_hh rows and h_{t-1} are staged through LDS in
// 64-wide K chunks.  Gate order i,f,g,o (PyTorch).
constexpr int LSTM_KCH = 64;
__global__ void __launch_bounds__(256) lstm_step_kernel(const float* __restrict__ pre, const float* __restrict__ whh,
                                                        float* __restrict__ hs, float* __restrict__ cst, int B,
                                                        int T, int H, int step) {
  __shared__ float Ws[32][LSTM_KCH + 1];
  __shared__ float Hs[32][LSTM_KCH + 1];
  const int dir = blockIdx.z;
  const int t = dir == 0 ? step : T - 1 - step;
  const int tprev = dir == 0 ? t - 1 : t + 1;
  const int u0 = blockIdx.x * 8, b0 = blockIdx.y * 32;
  const int ul = threadIdx.x >> 5, bl = threadIdx.x & 31;
  const int u = u0 + ul, b = b0 + bl;
  const float* W = whh + (long)dir * 4 * H * H;
  float* hsd = hs + (long)dir * B * T * H;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (step > 0) {
    for (int k0 = 0; k0 < H; k0 += LSTM_KCH) {
      for (int i = threadIdx.x; i < 32 * LSTM_KCH; i += 256) {
        const int r = i / LSTM_KCH, k = i - r * LSTM_KCH;
        const int g = r >> 3, uu = u0 + (r & 7);
        Ws[r][k] = (k0 + k < H && uu < H) ? W[((long)g * H + uu) * H + k0 + k] : 0.f;
        const int bb = b0 + r;
        Hs[r][k] = (k0 + k < H && bb < B) ? hsd[((long)bb * T + tprev) * H + k0 + k] : 0.f;
      }
      __syncthreads();
#pragma unroll 8
      for (int k = 0; k < LSTM_KCH; ++k) {
        const float h = Hs[bl][k];
        acc[0] += Ws[0 * 8 + ul][k] * h;
        acc[1] += Ws[1 * 8 + ul][k] * h;
        acc[2] += Ws[2 * 8 + ul][k] * h;
        acc[3] += Ws[3 * 8 + ul][k] * h;
      }
      __syncthreads();
    }
  }
  if (b >= B || u >= H) return;
  const float* pr = pre + ((long)b * T + t) * 8 * H + (long)dir * 4 * H;
  const float gi = sigmoid_exact(pr[u] + acc[0]);
  const float gf = sigmoid_exact(pr[H + u] + acc[1]);
  const float gg = tanhf(pr[2 * H + u] + acc[2]);
  const float go = sigmoid_exact(pr[3 * H + u] + acc[3]);
  float* cp = cst + ((long)dir * B + b) * H + u;
  const float c = step > 0 ? gf * (*cp) + gi * gg : gi * gg;
  *cp = c;
  hsd[((long)b * T + t) * H + u] = go * tanhf(c);
}

// ---------------------------------------------------------------------------------------------
constexpr int HEAD_W = 16;  // waves of a mel_head workgroup (the K split)
__global__ void __launch_bounds__(64 * HEAD_W) mel_head_kernel(const float* __restrict__ hs, int rows, int H,
                                                              const float* __restrict__ wt, const float* __restrict__ b,
                                                              int n_mels, float* __restrict__ out) {
  // one output row (frame) per workgroup: y = h_fwd + h_bwd staged in LDS, lane = mel (n_mels <= 64), the 16 waves
  // take a sixteenth of K each with four independent FMA chains, the partials added in a fixed order (four waves
  // made a 32-frame head a 14 us launch of 160-long load chains; a 640-long chain per thread 26 us)
  extern __shared__ float ys[];  // [H] + [HEAD_W][64] partial sums
  float* part = ys + H;
  const int row = blockIdx.x;
  const long plane = (long)rows * H;
  for (int k = threadIdx.x; k < H; k += 64 * HEAD_W) ys[k] = hs[(long)row * H + k] + hs[plane + (long)row * H + k];
  __syncthreads();
  const int q = threadIdx.x >> 6;
  const int k0 = q * H / HEAD_W, k1 = (q + 1) * H / HEAD_W;
  for (int nb = 0; nb < n_mels; nb += 64) {  // 64 mels a pass (the reference's n_mels = 64: one pass)
    const int n = nb + (threadIdx.x & 63);
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < n_mels) {
      int k = k0;
      for (; k + 4 <= k1; k += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = fmaf(ys[k + j], wt[(long)(k + j) * n_mels + n], a[j]);
      }
      for (; k < k1; ++k) a[0] = fmaf(ys[k], wt[(long)k * n_mels + n], a[0]);
    }
    if (nb > 0) __syncthreads();  // the previous pass's partials were read
    part[threadIdx.x] = (a[0] + a[1]) + (a[2] + a[3]);
    __syncthreads();
    const int l = threadIdx.x & 63;
    if (q == 0 && n < n_mels) {
      float t[HEAD_W];
#pragma unroll
      for (int w = 0; w < HEAD_W; ++w) t[w] = part[64 * w + l];
#pragma unroll
      for (int st = 1; st < HEAD_W; st *= 2)  // pairwise, fixed order
#pragma unroll
        for (int w = 0; w < HEAD_W; w += 2 * st) t[w] += t[w + st];
      out[(long)row * n_mels + n] = t[0] + b[n];
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) mel_glue_kernel(const float* __restrict__ x, int rows, int n_mels,
                                                       const float* __restrict__ mean, const float* __restrict__ sd,
                                                       float* db, float* ln, T* ln_t, int cs) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * cs) return;
  const int r = (int)(i / cs), n = (int)(i - (long)(i / cs) * cs);
  if (n >= n_mels) {
    if (ln_t) act_st<T>(ln_t, r, cs, n, 0.f);
    return;
  }
  const long o = (long)r * n_mels + n;
  // run_mri_video_inference.py:160-163: torch rounds the multiply and the add separately
  {
#pragma clang fp contract(off)
    const float d = x[o] * sd[n] + mean[n];
    const float p = powf(10.0f, d / 10.0f);
    const float l = logf(fmaxf(p, 1e-5f));
    if (db) db[o] = d;
    if (ln) ln[o] = l;
    if (ln_t) act_st<T>(ln_t, r, cs, n, l);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) mel_to_nlc_kernel(const float* __restrict__ mel, int B, int C, int Tn,
                                                         int layout, T* __restrict__ y, int cs) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * Tn * cs) return;
  const int c = (int)(i % cs);
  const long bt = i / cs;
  const int b = (int)(bt / Tn), t = (int)(bt - (long)b * Tn);
  float v = 0.f;
  if (c < C) v = layout == 0 ? mel[((long)b * C + c) * Tn + t] : mel[bt * C + c];
  act_st<T>(y, bt, cs, c, v);
}

template <typename T>
__global__ void __launch_bounds__(256) conv_post_kernel(const T* __restrict__ x, int B, int L, int C, int cs,
                                                        const float* __restrict__ w, float bias,
                                                        float* __restrict__ wav) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * L) return;
  const int b = (int)(i / L), t = (int)(i - (long)b * L);
  float acc = 0.f;
  for (int j = 0; j < 7; ++j) {
    if (t + j >= L) break;  // right zero pad of 6 (models.py:127)
    for (int c = 0; c < C; c += 4) {
      float v[4];
      act_ld4<T>(x, (long)b * L + t + j, cs, c, v);
      const float* wj = w + j * C + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += wj[e] * (v[e] > 0.f ? v[e] : 0.01f * v[e]);
    }
  }
  wav[i] = tanhf(acc + bias);
}

// conv_post for narrow inputs (C <= 64): a workgroup stages LeakyReLU(x) of its 256 + 6 rows in LDS
// once (coalesced 4-channel loads, pitch C + 1 floats: conflict-free column reads), then each thread
// reduces its 7 taps x C from LDS.  The per-thread form above re-reads every input row 7 times with
// 8-byte loads 4 x C bytes apart (0.27 ms per 806 K samples, ~10x the HBM time of its bytes).
// Same summation order as conv_post_kernel (tap-major, channels ascending).
constexpr int CP_T = 256;
template <typename T>
__global__ void __launch_bounds__(256) conv_post_tile_kernel(const T* __restrict__ x, int L, int C, int cs,
                                                             const float* __restrict__ w, float bias,
                                                             float* __restrict__ wav, int tiles) {
  extern __shared__ float cps[];  // [CP_T + 6][C + 1]
  const int P = C + 1, b = blockIdx.x / tiles, t0 = (blockIdx.x - b * tiles) * CP_T;
  const int q = C / 4, items = (CP_T + 6) * q;
  for (int i = threadIdx.x; i < items; i += 256) {
    const int r = i / q, c = (i - r * q) * 4, t = t0 + r;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < L) act_ld4<T>(x, (long)b * L + t, cs, c, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) cps[r * P + c + e] = v[e] > 0.f ? v[e] : 0.01f * v[e];
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= L) return;
  float acc = 0.f;
  for (int j = 0; j < 7; ++j) {
    const float* row = cps + (threadIdx.x + j) * P;
    const float* wj = w + j * C;
    for (int c = 0; c < C; ++c) acc += wj[c] * row[c];
  }
  wav[(long)b * L + t] = tanhf(acc + bias);
}

__global__ void __launch_bounds__(256) add2_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                   float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = a[i] + b[i];
}

template <typename T>
__global__ void __launch_bounds__(256) unpad_kernel(const T* __restrict__ x, long rows, int C, int cs,
                                                    float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * C) return;
  const long r = i / C;
  y[i] = act_ld<T>(x, r, cs, (int)(i - r * C));
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

// fp8 engines: y = e4m3(lrelu(x)) for 8 bf16 per thread (the operand of the first e4m3 MRF conv of a stage)
__global__ void __launch_bounds__(256) lrelu_e4m3_kernel(const uint4* __restrict__ x, uint2* __restrict__ y, long n8,
                                                         float slope) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const uint4 u = x[i];
  float v[8];
  unpack_bf16x4(make_uint2(u.x, u.y), v);
  unpack_bf16x4(make_uint2(u.z, u.w), v + 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * slope;
  y[i] = e4m3x8(v);
}

}  // namespace

template <typename T>
void launch_unpad(const T* x, long rows, int C, int cs, float* y, hipStream_t s) {
  hipLaunchKernelGGL(unpad_kernel<T>, dim3(nblk(rows * C)), dim3(256), 0, s, x, rows, C, cs, y);
  M2S_HIP(hipGetLastError());
}

void launch_lrelu_e4m3(const bf16_t* x, uint8_t* y, long n, float slope, hipStream_t s) {
  M2S_CHECK(n % 8 == 0, "lrelu_e4m3: n % 8");
  hipLaunchKernelGGL(lrelu_e4m3_kernel, dim3(nblk(n / 8)), dim3(256), 0, s, reinterpret_cast<const uint4*>(x),
                     reinterpret_cast<uint2*>(y), n / 8, slope);
  M2S_HIP(hipGetLastError());
}

void launch_add2(const float* a, const float* b, float* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(add2_kernel, dim3(nblk(n)), dim3(256), 0, s, a, b, y, n);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_stem(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, const float* w9,
                 const float* bias, int cout, int cs_out, T* y, hipStream_t s) {
  M2S_CHECK(cout <= 32 && cs_out % 8 == 0 && cs_out <= 32, "stem: unsupported channel count");
  if (std::is_same<T, bf16_t>::value && cout == 32 && cs_out == 32) {
    hipLaunchKernelGGL(stem32_kernel, dim3((unsigned)nblk((long)N * OH * OW)), dim3(256), 0, s, frames, N, H, W, OH, OW,
                       pad_t, pad_l, w9, bias, reinterpret_cast<bf16_t*>(y));
    M2S_HIP(hipGetLastError());
    return;
  }
  const long blocks = std::min<long>(nblk(4L * N * OH * OW), 256L * 16);
  hipLaunchKernelGGL(stem_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, frames, N, H, W, OH, OW, pad_t,
                     pad_l, w9, bias, cout, cs_out, y);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_gap(const T* x, int N, int P, int C, int cs, float* feats, hipStream_t s) {
  if (N <= 0) return;
  hipLaunchKernelGGL(gap_kernel<T>, dim3(N, ceil_div(C, 64)), dim3(256), 0, s, x, N, P, C, cs, feats);
  M2S_HIP(hipGetLastError());
}

void launch_lstm_step(const float* pre, const float* whh, float* hs, float* cst, int B, int T, int H, int step,
                      hipStream_t s) {
  M2S_CHECK(H % 8 == 0, "lstm: hidden size must be a multiple of 8");
  hipLaunchKernelGGL(lstm_step_kernel, dim3(H / 8, ceil_div(B, 32), 2), dim3(256), 0, s, pre, whh, hs, cst, B, T, H,
                     step);
  M2S_HIP(hipGetLastError());
}

void launch_mel_head(const float* hs, int rows, int H, const float* wt, const float* b, int n_mels, float* out,
                     hipStream_t s) {
  M2S_CHECK(n_mels >= 1 && H >= 4, "mel_head: shape");
  hipLaunchKernelGGL(mel_head_kernel, dim3(rows), dim3(64 * HEAD_W), (H + HEAD_W * 64) * sizeof(float), s, hs, rows, H, wt, b,
                     n_mels, out);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_mel_glue(const float* x, int rows, int n_mels, const float* mean, const float* std_, float* db, float* ln,
                     T* ln_t, int cs, hipStream_t s) {
  if (!ln_t) cs = n_mels;
  hipLaunchKernelGGL(mel_glue_kernel<T>, dim3(nblk((long)rows * cs)), dim3(256), 0, s, x, rows, n_mels, mean, std_, db,
                     ln, ln_t, cs);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_mel_to_nlc(const float* mel, int B, int C, int Tn, int layout, T* y, int cs, hipStream_t s) {
  hipLaunchKernelGGL(mel_to_nlc_kernel<T>, dim3(nblk((long)B * Tn * cs)), dim3(256), 0, s, mel, B, C, Tn, layout, y,
                     cs);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_conv_post(const T* x, int B, int L, int C, int cs, const float* w, float bias, float* wav, hipStream_t s) {
  M2S_CHECK(C % 4 == 0, "conv_post: C % 4");
  if (C <= 64) {
    const int tiles = (L + CP_T - 1) / CP_T;
    M2S_CHECK((double)B * tiles < 2147483647.0, "conv_post: grid");
    hipLaunchKernelGGL(conv_post_tile_kernel<T>, dim3(B * tiles), dim3(256), (CP_T + 6) * (C + 1) * sizeof(float), s, x,
                       L, C, cs, w, bias, wav, tiles);
  } else {
    hipLaunchKernelGGL(conv_post_kernel<T>, dim3(nblk((long)B * L)), dim3(256), 0, s, x, B, L, C, cs, w, bias, wav);
  }
  M2S_HIP(hipGetLastError());
}

#define M2S_INST(T)                                                                                                  \
  template void launch_stem<T>(const float*, int, int, int, int, int, int, int, const float*, const float*, int, int, \
                               T*, hipStream_t);                                                                     \
  template void launch_gap<T>(const T*, int, int, int, int, float*, hipStream_t);                                    \
  template void launch_mel_glue<T>(const float*, int, int, const float*, const float*, float*, float*, T*, int,      \
                                   hipStream_t);                                                                     \
  template void launch_mel_to_nlc<T>(const float*, int, int, int, int, T*, int, hipStream_t);                        \
  template void launch_conv_post<T>(const T*, int, int, int, int, const float*, float, float*, hipStream_t);        \
  template void launch_unpad<T>(const T*, long, int, int, float*, hipStream_t);
M2S_INST(float)
M2S_INST(bf16_t)
M2S_INST(sp_t)

}  // namespace m2s
