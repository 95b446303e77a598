// Non-GEMM kernels of the hot path: stem, depthwise+SE, GAP, BiLSTM recurrence, head, mel glue,
// vocoder input/output edges.  All are HBM/latency-bound; each reads its input once.
#include "kernels.hpp"

namespace m2s {

namespace {

template <typename T>
__device__ __forceinline__ void st4(T* p, float a, float b, float c, float d) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
  } else {
    uint2 u;
    u.x = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
    u.y = (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  }
}

template <typename T>
__device__ __forceinline__ float4 ld4(const T* p) {
  if constexpr (sizeof(T) == 4) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
}

template <typename T>
__device__ __forceinline__ float act_silu(float v) {
  return sizeof(T) == 4 ? silu_exact(v) : silu(v);
}

// ---------------------------------------------------------------------------------------------
// stem: one thread = one output pixel x 32 channels.  TF-SAME pads passed from the host.
template <typename T>
__global__ void __launch_bounds__(256) stem_kernel(const float* __restrict__ frames, int N, int H, int W, int OH,
                                                   int OW, int pad_t, int pad_l, const float* __restrict__ w9,
                                                   const float* __restrict__ bias, int cout, int cs_out,
                                                   T* __restrict__ y) {
  __shared__ float sw[32 * 9 + 32];
  for (int i = threadIdx.x; i < 32 * 9 + 32; i += 256)
    sw[i] = i < 32 * 9 ? (i / 9 < cout ? w9[i] : 0.f) : (i - 288 < cout ? bias[i - 288] : 0.f);
  __syncthreads();
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)N * OH * OW;
  if (p >= total) return;
  const int hw = OH * OW;
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
  T* out = y + p * cs_out;
#pragma unroll
  for (int o = 0; o < 32; o += 4) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) acc += sw[(o + j) * 9 + t] * in[t];
      v[j] = act_silu<T>(acc + sw[288 + o + j]);
    }
    if (o < cs_out) st4<T>(out + o, v[0], v[1], v[2], v[3]);
  }
}

// ---------------------------------------------------------------------------------------------
// depthwise 3x3 + bias + SiLU + SE squeeze.  grid (ceil(cs/512), N, ceil(OH/4)); a thread owns
// 8 channels (one 16-byte vector) of ONE output row and slides a 3x3 window along it, so each
// input vector is loaded once per row it feeds (3 loads per output at stride 1 instead of 9).
// SE partial sums: the 4 rows of a workgroup are added in a fixed order and written per row
// group (psum[n][row_group][cs]); se_fc adds the groups in order (deterministic).
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* v) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  }
}

template <typename T>
__device__ __forceinline__ void st8(T* p, const float* v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    uint4 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    u.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    u.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = u;
  }
}

template <typename T>
__device__ __forceinline__ void dw_col(const T* xn, int iy0, int ix, int IH, int IW, int cs, float (&c)[3][8]) {
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = iy0 + ky;
    if (iy >= 0 && iy < IH && ix >= 0 && ix < IW) {
      ld8<T>(xn + ((long)iy * IW + ix) * cs, c[ky]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) c[ky][j] = 0.f;
    }
  }
}

template <typename T, int S>
__global__ void __launch_bounds__(256) dwconv_kernel(const T* __restrict__ x, int IH, int IW, int OH, int OW,
                                                     int pad_t, int pad_l, int cs, const float* __restrict__ w9,
                                                     const float* __restrict__ bias, T* __restrict__ y,
                                                     float* __restrict__ sums) {
  __shared__ float red[4][512];
  const int n = blockIdx.y;
  const int cg = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + cg * 8;
  const int oy = blockIdx.z * 4 + rl;
  const bool active = c0 < cs && oy < OH;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    float w[9][8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int t = 0; t < 9; ++t) w[t][j] = w9[(c0 + j) * 9 + t];
      b[j] = bias[c0 + j];
    }
    const T* xn = x + (long)n * IH * IW * cs + c0;
    T* yn = y + (long)n * OH * OW * cs + c0;
    {
      const int iy0 = oy * S - pad_t;
      float c0w[3][8], c1w[3][8], c2w[3][8];
      dw_col<T>(xn, iy0, -pad_l, IH, IW, cs, c0w);
      dw_col<T>(xn, iy0, -pad_l + 1, IH, IW, cs, c1w);
      dw_col<T>(xn, iy0, -pad_l + 2, IH, IW, cs, c2w);
      for (int ox = 0; ox < OW; ++ox) {
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float a = b[j];
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            a += w[ky * 3 + 0][j] * c0w[ky][j];
            a += w[ky * 3 + 1][j] * c1w[ky][j];
            a += w[ky * 3 + 2][j] * c2w[ky][j];
          }
          a = act_silu<T>(a);
          s[j] += a;
          acc[j] = a;
        }
        st8<T>(yn + ((long)oy * OW + ox) * cs, acc);
        const int ixn = (ox + 1) * S - pad_l;  // first input column of the next output
        if (S == 1) {
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              c0w[ky][j] = c1w[ky][j];
              c1w[ky][j] = c2w[ky][j];
            }
          dw_col<T>(xn, iy0, ixn + 2, IH, IW, cs, c2w);
        } else {
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int j = 0; j < 8; ++j) c0w[ky][j] = c2w[ky][j];
          dw_col<T>(xn, iy0, ixn + 1, IH, IW, cs, c1w);
          dw_col<T>(xn, iy0, ixn + 2, IH, IW, cs, c2w);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cg * 8 + j] = s[j];
  __syncthreads();
  if (rl == 0 && c0 < cs) {
    float* ps = sums + ((long)n * gridDim.z + blockIdx.z) * cs + c0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      ps[j] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// SE excitation for SE_G images per workgroup.  psum [n][nrg][cs] (row-group partial sums of
// the depthwise output), w1 [rd][C] (conv_reduce), w2t [rd][C] (conv_expand transposed so
// consecutive threads read consecutive c).  Each wave reduces SE_R rows of w1 per pass with
// independent loads in flight (the loop is latency-, not bandwidth-bound).
constexpr int SE_G = 2, SE_R = 8;
__global__ void __launch_bounds__(256) se_fc_kernel(const float* __restrict__ psum, int nrg, int N, int C, int cs,
                                                    int rd, float inv_count, const float* __restrict__ w1,
                                                    const float* __restrict__ b1, const float* __restrict__ w2t,
                                                    const float* __restrict__ b2, float* __restrict__ scale,
                                                    int exact) {
  __shared__ float m[SE_G][1280];
  __shared__ float z[SE_G][128];
  const int n0 = blockIdx.x * SE_G;
  for (int i = threadIdx.x; i < SE_G * C; i += 256) {
    const int g = i / C, c = i - (i / C) * C;
    float acc = 0.f;
    if (n0 + g < N)
      for (int q = 0; q < nrg; ++q) acc += psum[((long)(n0 + g) * nrg + q) * cs + c];
    m[g][c] = acc * inv_count;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int r0 = wave * SE_R; r0 < rd; r0 += 4 * SE_R) {
    float acc[SE_R][SE_G];
#pragma unroll
    for (int q = 0; q < SE_R; ++q)
#pragma unroll
      for (int g = 0; g < SE_G; ++g) acc[q][g] = 0.f;
#pragma unroll 4
    for (int c = lane; c < C; c += 64) {
      float mv[SE_G];
#pragma unroll
      for (int g = 0; g < SE_G; ++g) mv[g] = m[g][c];
#pragma unroll
      for (int q = 0; q < SE_R; ++q) {
        const float wv = r0 + q < rd ? w1[(long)(r0 + q) * C + c] : 0.f;
#pragma unroll
        for (int g = 0; g < SE_G; ++g) acc[q][g] += wv * mv[g];
      }
    }
#pragma unroll
    for (int q = 0; q < SE_R; ++q)
#pragma unroll
      for (int g = 0; g < SE_G; ++g) {
        float a = acc[q][g];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
        acc[q][g] = a;
      }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < SE_R; ++q) {
        if (r0 + q >= rd) break;
#pragma unroll
        for (int g = 0; g < SE_G; ++g) {
          const float v = acc[q][g] + b1[r0 + q];
          z[g][r0 + q] = exact ? silu_exact(v) : silu(v);
        }
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cs; c += 256) {
    float acc[SE_G];
    const float bb = c < C ? b2[c] : 0.f;
#pragma unroll
    for (int g = 0; g < SE_G; ++g) acc[g] = bb;
    if (c < C) {
#pragma unroll 8
      for (int r = 0; r < rd; ++r) {
        const float wv = w2t[(long)r * C + c];
#pragma unroll
        for (int g = 0; g < SE_G; ++g) acc[g] += wv * z[g][r];
      }
    }
#pragma unroll
    for (int g = 0; g < SE_G; ++g) {
      if (n0 + g >= N) break;
      scale[(long)(n0 + g) * cs + c] = c < C ? (exact ? sigmoid_exact(acc[g]) : sigmoidf_(acc[g])) : 0.f;
    }
  }
}

// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) gap_kernel(const T* __restrict__ x, int N, int P, int C, int cs,
                                                  float* __restrict__ feats) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * C) return;
  const int n = (int)(i / C), c = (int)(i - (long)(i / C) * C);
  const T* p = x + (long)n * P * cs + c;
  float acc = 0.f;
  for (int k = 0; k < P; ++k) acc += Elem<T>::to_f(p[(long)k * cs]);
  feats[i] = acc / (float)P;
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
__global__ void __launch_bounds__(256) mel_head_kernel(const float* __restrict__ hs, int rows, int H,
                                                       const float* __restrict__ wt, const float* __restrict__ b,
                                                       int n_mels, float* __restrict__ out) {
  extern __shared__ float ys[];  // [4][H]
  const int r0 = blockIdx.x * 4;
  const long plane = (long)rows * H;
  for (int i = threadIdx.x; i < 4 * H; i += 256) {
    const int r = i / H, k = i - r * H;
    const int row = r0 + r;
    ys[i] = row < rows ? hs[(long)row * H + k] + hs[plane + (long)row * H + k] : 0.f;
  }
  __syncthreads();
  const int r = threadIdx.x >> 6, nl = threadIdx.x & 63;
  const int row = r0 + r;
  if (row >= rows) return;
  for (int n = nl; n < n_mels; n += 64) {
    float acc = 0.f;
    for (int k = 0; k < H; ++k) acc += ys[r * H + k] * wt[(long)k * n_mels + n];
    out[(long)row * n_mels + n] = acc + b[n];
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
    if (ln_t) ln_t[i] = Elem<T>::from_f(0.f);
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
    if (ln_t) ln_t[i] = Elem<T>::from_f(l);
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
  y[i] = Elem<T>::from_f(v);
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
    const T* row = x + ((long)b * L + t + j) * cs;
    for (int c = 0; c < C; c += 4) {
      const float4 v = ld4<T>(row + c);
      const float* wj = w + j * C + c;
      acc += wj[0] * (v.x > 0.f ? v.x : 0.01f * v.x);
      acc += wj[1] * (v.y > 0.f ? v.y : 0.01f * v.y);
      acc += wj[2] * (v.z > 0.f ? v.z : 0.01f * v.z);
      acc += wj[3] * (v.w > 0.f ? v.w : 0.01f * v.w);
    }
  }
  wav[i] = tanhf(acc + bias);
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
  y[i] = Elem<T>::to_f(x[r * cs + (i - r * C)]);
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

template <typename T>
void launch_unpad(const T* x, long rows, int C, int cs, float* y, hipStream_t s) {
  hipLaunchKernelGGL(unpad_kernel<T>, dim3(nblk(rows * C)), dim3(256), 0, s, x, rows, C, cs, y);
  M2S_HIP(hipGetLastError());
}

void launch_add2(const float* a, const float* b, float* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(add2_kernel, dim3(nblk(n)), dim3(256), 0, s, a, b, y, n);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_stem(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, const float* w9,
                 const float* bias, int cout, int cs_out, T* y, hipStream_t s) {
  M2S_CHECK(cout <= 32 && cs_out % 4 == 0, "stem: unsupported channel count");
  hipLaunchKernelGGL(stem_kernel<T>, dim3(nblk((long)N * OH * OW)), dim3(256), 0, s, frames, N, H, W, OH, OW, pad_t,
                     pad_l, w9, bias, cout, cs_out, y);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_dwconv(const T* x, int N, int IH, int IW, int OH, int OW, int stride, int pad_t, int pad_l, int C, int cs,
                   const float* w9, const float* bias, T* y, float* sums, hipStream_t s) {
  (void)C;
  M2S_CHECK(cs % 8 == 0, "dwconv: cs % 8");
  M2S_CHECK(stride == 1 || stride == 2, "dwconv: stride");
  const dim3 grid(ceil_div(cs, 512), N, dw_row_groups(OH));
  if (stride == 1)
    hipLaunchKernelGGL((dwconv_kernel<T, 1>), grid, dim3(256), 0, s, x, IH, IW, OH, OW, pad_t, pad_l, cs, w9, bias, y,
                       sums);
  else
    hipLaunchKernelGGL((dwconv_kernel<T, 2>), grid, dim3(256), 0, s, x, IH, IW, OH, OW, pad_t, pad_l, cs, w9, bias, y,
                       sums);
  M2S_HIP(hipGetLastError());
}

void launch_se_fc(const float* sums, int nrg, int N, int C, int cs, int rd, float inv_count, const float* w1,
                  const float* b1, const float* w2, const float* b2, float* scale, bool exact, hipStream_t s) {
  M2S_CHECK(C <= 1280 && rd <= 128, "se: too many channels");
  hipLaunchKernelGGL(se_fc_kernel, dim3(ceil_div(N, SE_G)), dim3(256), 0, s, sums, nrg, N, C, cs, rd, inv_count, w1,
                     b1, w2, b2, scale, exact ? 1 : 0);
  M2S_HIP(hipGetLastError());
}

template <typename T>
void launch_gap(const T* x, int N, int P, int C, int cs, float* feats, hipStream_t s) {
  hipLaunchKernelGGL(gap_kernel<T>, dim3(nblk((long)N * C)), dim3(256), 0, s, x, N, P, C, cs, feats);
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
  hipLaunchKernelGGL(mel_head_kernel, dim3(ceil_div(rows, 4)), dim3(256), 4 * H * sizeof(float), s, hs, rows, H, wt, b,
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
  hipLaunchKernelGGL(conv_post_kernel<T>, dim3(nblk((long)B * L)), dim3(256), 0, s, x, B, L, C, cs, w, bias, wav);
  M2S_HIP(hipGetLastError());
}

#define M2S_INST(T)                                                                                                  \
  template void launch_stem<T>(const float*, int, int, int, int, int, int, int, const float*, const float*, int, int, \
                               T*, hipStream_t);                                                                     \
  template void launch_dwconv<T>(const T*, int, int, int, int, int, int, int, int, int, int, const float*,           \
                                 const float*, T*, float*, hipStream_t);                                             \
  template void launch_gap<T>(const T*, int, int, int, int, float*, hipStream_t);                                    \
  template void launch_mel_glue<T>(const float*, int, int, const float*, const float*, float*, float*, T*, int,      \
                                   hipStream_t);                                                                     \
  template void launch_mel_to_nlc<T>(const float*, int, int, int, int, T*, int, hipStream_t);                        \
  template void launch_conv_post<T>(const T*, int, int, int, int, const float*, float, float*, hipStream_t);        \
  template void launch_unpad<T>(const T*, long, int, int, float*, hipStream_t);
M2S_INST(float)
M2S_INST(bf16_t)

}  // namespace m2s
