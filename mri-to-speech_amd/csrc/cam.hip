// Kernels of the Grad-CAM path (cam.hpp): train-mode BatchNorm, raw stem / depthwise convs, the
// BiLSTM forward with saved activations and its backward through time, a strided fp32 GEMM for the
// projections and weight gradients, GAP forward / backward.  Exact fp32 (libm sigmoid / tanh / SiLU);
// every reduction runs in a fixed order, so a launch is deterministic.
#include <algorithm>

#include "cam.hpp"

namespace m2s {

namespace {

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

// ---------------------------------------------------------------------------------------------
// strided GEMM: 64 x 64 output tile per 256-thread workgroup, K in steps of 16 through LDS, each
// thread a 4 x 4 block.  Loads follow whichever operand stride is unit, so both the "NN" and the
// transposed ("TN": weight gradients) forms read coalesced rows.
constexpr int GT = 64, GK = 16;
__global__ void __launch_bounds__(256) gemm_f32_kernel(int M, int N, int K, const float* __restrict__ A, long sam,
                                                       long sak, const float* __restrict__ B, long sbk, long sbn,
                                                       float* __restrict__ C, long ldc, const float* __restrict__ b1,
                                                       const float* __restrict__ b2, int accumulate) {
  __shared__ float As[GK][GT + 4];
  __shared__ float Bs[GK][GT + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += GK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * 256;
      int m, k;
      if (sak == 1) { m = e >> 4; k = e & 15; } else { m = e & 63; k = e >> 6; }
      const int gm = m0 + m, gk = k0 + k;
      As[k][m] = (gm < M && gk < K) ? A[gm * sam + gk * sak] : 0.f;
      int n, kb;
      if (sbn == 1) { n = e & 63; kb = e >> 6; } else { n = e >> 4; kb = e & 15; }
      const int gn = n0 + n, gkb = k0 + kb;
      Bs[kb][n] = (gn < N && gkb < K) ? B[gkb * sbk + gn * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GK; ++k) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = As[k][ty * 4 + i];
        b[i] = Bs[k][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + ty * 4 + i;
    if (gm >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gn = n0 + tx * 4 + j;
      if (gn >= N) continue;
      float v = acc[i][j];
      if (b1) v += b1[gn];
      if (b2) v += b2[gn];
      float* c = C + gm * ldc + gn;
      *c = accumulate ? *c + v : v;
    }
  }
}

__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ x, int rows, int cols, long ld,
                                                     float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += x[r * ld + c];
  out[c] = accumulate ? out[c] + s : s;
}

// ---------------------------------------------------------------------------------------------
// conv_stem (grey repeat folded: w9[o][t] = sum of the three input-channel taps), no bias, no act.
__global__ void __launch_bounds__(256) stem_raw_kernel(const float* __restrict__ frames, int N, int H, int W, int OH,
                                                       int OW, int pad_t, int pad_l, const float* __restrict__ w9,
                                                       float* __restrict__ z) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  const int hw = OH * OW;
  if (p >= (long)N * hw) return;
  const int n = (int)(p / hw), rem = (int)(p - (long)n * hw);
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
  float4* out = reinterpret_cast<float4*>(z + p * 32);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) a = fmaf(w9[(q * 4 + j) * 9 + t], in[t], a);
      v[j] = a;
    }
    out[q] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// depthwise 3x3, TF-SAME pads from the host, no bias / act; one thread per (position, 4 channels)
__global__ void __launch_bounds__(256) dw_raw_kernel(const float* __restrict__ x, int N, int IH, int IW, int OH, int OW,
                                                     int stride, int pad_t, int pad_l, int cs,
                                                     const float* __restrict__ w, float* __restrict__ z) {
  const int q = cs / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * OH * OW * q) return;
  const long p = i / q;
  const int c = (int)(i - p * q) * 4;
  const int hw = OH * OW, n = (int)(p / hw), rem = (int)(p - (long)n * hw);
  const int oy = rem / OW, ox = rem - (rem / OW) * OW;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int iy = oy * stride - pad_t + ky, ix = ox * stride - pad_l + kx;
      if (iy < 0 || iy >= IH || ix < 0 || ix >= IW) continue;
      const float4 v = *reinterpret_cast<const float4*>(x + (((long)n * IH + iy) * IW + ix) * cs + c);
      const float4 k = *reinterpret_cast<const float4*>(w + (ky * 3 + kx) * cs + c);
      a[0] = fmaf(k.x, v.x, a[0]);
      a[1] = fmaf(k.y, v.y, a[1]);
      a[2] = fmaf(k.z, v.z, a[2]);
      a[3] = fmaf(k.w, v.w, a[3]);
    }
  *reinterpret_cast<float4*>(z + p * cs + c) = make_float4(a[0], a[1], a[2], a[3]);
}

// ---------------------------------------------------------------------------------------------
// BatchNorm on batch statistics.  Pass 0 sums x, pass 1 sums (x - mean)^2 (two passes: no
// cancellation).  Partial block: 4 row groups x 64 channels; partials reduced per channel in double.
constexpr int BN_MAX_PARTS = 2048;
__global__ void __launch_bounds__(256) bn_partial_kernel(const float* __restrict__ x, long M, int C, int cs,
                                                         const float* __restrict__ mean, long rows_per,
                                                         float* __restrict__ part) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const long r0 = (long)blockIdx.x * rows_per, r1 = std::min(M, r0 + rows_per);
  float acc = 0.f;
  if (c < C) {
    const float mu = mean ? mean[c] : 0.f;
    for (long r = r0 + rg; r < r1; r += 4) {
      float v = x[r * cs + c];
      if (mean) {
        v -= mu;
        v *= v;
      }
      acc += v;
    }
  }
  red[rg][cl] = acc;
  __syncthreads();
  if (rg == 0 && c < C) part[(long)blockIdx.x * C + c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ part, int nparts, long M, int C,
                                                          int pass, const float* __restrict__ gamma, float eps,
                                                          float* __restrict__ stats, float* __restrict__ coef) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int b = 0; b < nparts; ++b) s += (double)part[(long)b * C + c];
  const float v = (float)(s / (double)M);
  if (pass == 0) {
    stats[c] = v;
  } else {
    stats[C + c] = v;
    coef[c] = gamma[c] / sqrtf(v + eps);
  }
}

__device__ __forceinline__ float cam_act(float v, int act) { return act == 1 ? silu_exact(v) : v; }

__global__ void __launch_bounds__(256) bn_apply_kernel(float* __restrict__ x, long M, int C, int cs,
                                                       const float* __restrict__ stats, const float* __restrict__ coef,
                                                       const float* __restrict__ beta, int act,
                                                       const float* __restrict__ res) {
  const int q = cs / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * q) return;
  const long r = i / q;
  const int c = (int)(i - r * q) * 4;
  float4* px = reinterpret_cast<float4*>(x + r * cs + c);
  float4 v = *px;
  float e[4] = {v.x, v.y, v.z, v.w};
  float rr[4] = {0.f, 0.f, 0.f, 0.f};
  if (res) {
    const float4 t = *reinterpret_cast<const float4*>(res + r * cs + c);
    rr[0] = t.x; rr[1] = t.y; rr[2] = t.z; rr[3] = t.w;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cc = c + j;
    e[j] = cc < C ? cam_act((e[j] - stats[cc]) * coef[cc] + beta[cc], act) + rr[j] : 0.f;
  }
  *px = make_float4(e[0], e[1], e[2], e[3]);
}

__global__ void __launch_bounds__(256) to_nchw_kernel(const float* __restrict__ x, int N, int P, int C, int cs,
                                                      float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * C * P) return;
  const long nc = i / P;
  const int p = (int)(i - nc * P), n = (int)(nc / C), c = (int)(nc - (long)n * C);
  y[i] = x[((long)n * P + p) * cs + c];
}

__global__ void __launch_bounds__(256) gap_nchw_kernel(const float* __restrict__ x, long NC, int P,
                                                       float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= NC) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += x[i * P + p];
  y[i] = s / (float)P;
}

__global__ void __launch_bounds__(256) gap_nchw_bwd_kernel(const float* __restrict__ dy, long NC, int P,
                                                           float* __restrict__ dx) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= NC * P) return;
  dx[i] = dy[i / P] / (float)P;
}

// ---------------------------------------------------------------------------------------------
// BiLSTM forward step with saved activations.  Workgroup = 8 hidden units of one direction: their
// 32 W_hh rows (4 gates x 8 units) stay in LDS; thread (row, k-slice of 8) dots interleaved k.
__global__ void __launch_bounds__(256) lstm_train_step_kernel(const float* __restrict__ pre,
                                                              const float* __restrict__ whh, float* __restrict__ gates,
                                                              float* __restrict__ cells, float* __restrict__ hid, int B,
                                                              int T, int H, int step) {
  extern __shared__ float sw[];  // [32][H] then red[32]
  float* red = sw + 32 * H;
  const int dir = blockIdx.y, u0 = blockIdx.x * 8, tid = threadIdx.x;
  const float* W = whh + (long)dir * 4 * H * H;
  for (int i = tid; i < 32 * H; i += 256) {
    const int r = i / H, k = i - r * H;
    sw[i] = W[((long)(r >> 3) * H + u0 + (r & 7)) * H + k];
  }
  __syncthreads();
  const int t = dir == 0 ? step : T - 1 - step, tp = dir == 0 ? t - 1 : t + 1;
  const int r = tid >> 3, ks = tid & 7;
  for (int b = 0; b < B; ++b) {
    const long bt = (long)dir * B * T + (long)b * T;
    float acc = 0.f;
    if (step > 0) {
      const float* hp = hid + (bt + tp) * H;
      for (int k = ks; k < H; k += 8) acc = fmaf(sw[r * H + k], hp[k], acc);
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (ks == 0) red[r] = acc;
    __syncthreads();
    if (tid < 8) {
      const int u = u0 + tid;
      const float* pr = pre + ((long)b * T + t) * 8 * H + (long)dir * 4 * H;
      const float gi = sigmoid_exact(pr[u] + red[tid]);
      const float gf = sigmoid_exact(pr[H + u] + red[8 + tid]);
      const float gg = tanhf(pr[2 * H + u] + red[16 + tid]);
      const float go = sigmoid_exact(pr[3 * H + u] + red[24 + tid]);
      const float cp = step > 0 ? cells[(bt + tp) * H + u] : 0.f;
      const float c = gf * cp + gi * gg;
      float* gs = gates + (bt + t) * 4 * H;
      gs[u] = gi;
      gs[H + u] = gf;
      gs[2 * H + u] = gg;
      gs[3 * H + u] = go;
      cells[(bt + t) * H + u] = c;
      hid[(bt + t) * H + u] = go * tanhf(c);
    }
    __syncthreads();
  }
}

// BPTT step.  Workgroup = 8 hidden units of one direction: their 8 rows of W_hh^T (4H long) in LDS;
// thread (unit, k-slice of 32) dots the previous step's gate gradients, then 8 lanes apply the cell.
__global__ void __launch_bounds__(256) lstm_bptt_step_kernel(const float* __restrict__ whh_t,
                                                             const float* __restrict__ dy, const float* __restrict__ gates,
                                                             const float* __restrict__ cells, float* __restrict__ dc,
                                                             float* __restrict__ dg, int B, int T, int H, int step) {
  extern __shared__ float sw[];  // [8][4H] then red[8]
  const int G = 4 * H;
  float* red = sw + 8 * G;
  const int dir = blockIdx.y, u0 = blockIdx.x * 8, tid = threadIdx.x;
  const float* WT = whh_t + (long)dir * H * G + (long)u0 * G;
  for (int i = tid; i < 8 * G; i += 256) sw[i] = WT[i];
  __syncthreads();
  const int t = dir == 0 ? T - 1 - step : step;
  const int tn = dir == 0 ? t + 1 : t - 1;  // processed before this step: its gate gradients feed dh
  const int tp = dir == 0 ? t - 1 : t + 1;  // the step whose cell this step consumed
  const int ul = tid >> 5, ks = tid & 31;
  for (int b = 0; b < B; ++b) {
    const long bt = (long)dir * B * T + (long)b * T;
    float acc = 0.f;
    if (step > 0) {
      const float* g = dg + (bt + tn) * G;
      for (int k = ks; k < G; k += 32) acc = fmaf(sw[ul * G + k], g[k], acc);
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    acc += __shfl_xor(acc, 8);
    acc += __shfl_xor(acc, 16);
    if (ks == 0) red[ul] = acc;
    __syncthreads();
    if (tid < 8) {
      const int u = u0 + tid;
      const float* gs = gates + (bt + t) * G;
      const float gi = gs[u], gf = gs[H + u], gg = gs[2 * H + u], go = gs[3 * H + u];
      const float c = cells[(bt + t) * H + u];
      const bool first = dir == 0 ? t == 0 : t == T - 1;
      const float cp = first ? 0.f : cells[(bt + tp) * H + u];
      const float dh = dy[((long)b * T + t) * H + u] + red[tid];
      const float tc = tanhf(c);
      float* dcp = dc + ((long)dir * B + b) * H + u;
      const float dcv = (step > 0 ? *dcp : 0.f) + dh * go * (1.f - tc * tc);
      float* o = dg + (bt + t) * G;
      o[u] = dcv * gg * gi * (1.f - gi);
      o[H + u] = dcv * cp * gf * (1.f - gf);
      o[2 * H + u] = dcv * gi * (1.f - gg * gg);
      o[3 * H + u] = dh * tc * go * (1.f - go);
      *dcp = dcv * gf;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) lstm_hprev_kernel(const float* __restrict__ hid, float* __restrict__ hp, int B,
                                                         int T, int H) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2L * B * T * H) return;
  const int k = (int)(i % H);
  const long row = i / H;
  const int t = (int)(row % T);
  const long db = row / T;
  const int dir = (int)(db / B);
  const int tp = dir == 0 ? t - 1 : t + 1;
  hp[i] = (tp >= 0 && tp < T) ? hid[(db * T + tp) * H + k] : 0.f;
}

__global__ void __launch_bounds__(256) transpose_kernel(const float* __restrict__ x, int rows, int cols,
                                                        float* __restrict__ y) {
  __shared__ float tile[32][33];
  const long plane = (long)blockIdx.z * rows * cols;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int r = r0 + j, c = c0 + tx;
    tile[j][tx] = (r < rows && c < cols) ? x[plane + (long)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int c = c0 + j, r = r0 + tx;
    if (c < cols && r < rows) y[plane + (long)c * rows + r] = tile[tx][j];
  }
}

}  // namespace

void launch_gemm_f32(int M, int N, int K, const float* A, long sam, long sak, const float* B, long sbk, long sbn,
                     float* C, long ldc, const float* bias1, const float* bias2, bool accumulate, hipStream_t s) {
  M2S_CHECK(M >= 0 && N >= 0 && K >= 0, "gemm_f32: negative size");
  if (M == 0 || N == 0) return;
  dim3 grid(ceil_div(N, GT), ceil_div(M, GT));
  M2S_CHECK(grid.y <= 65535, "gemm_f32: too many rows");
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, s, M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, bias1, bias2,
                     accumulate ? 1 : 0);
  M2S_HIP(hipGetLastError());
}

void launch_colsum(const float* x, int rows, int cols, long ld, float* out, bool accumulate, hipStream_t s) {
  if (cols <= 0) return;
  hipLaunchKernelGGL(colsum_kernel, dim3(nblk(cols)), dim3(256), 0, s, x, rows, cols, ld, out, accumulate ? 1 : 0);
  M2S_HIP(hipGetLastError());
}

void launch_stem_raw(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, const float* w9,
                     float* z, hipStream_t s) {
  hipLaunchKernelGGL(stem_raw_kernel, dim3(nblk((long)N * OH * OW)), dim3(256), 0, s, frames, N, H, W, OH, OW, pad_t,
                     pad_l, w9, z);
  M2S_HIP(hipGetLastError());
}

void launch_dw_raw(const float* x, int N, int IH, int IW, int OH, int OW, int stride, int pad_t, int pad_l, int cs,
                   const float* w, float* z, hipStream_t s) {
  M2S_CHECK(cs % 4 == 0, "dw_raw: cs % 4");
  hipLaunchKernelGGL(dw_raw_kernel, dim3(nblk((long)N * OH * OW * (cs / 4))), dim3(256), 0, s, x, N, IH, IW, OH, OW,
                     stride, pad_t, pad_l, cs, w, z);
  M2S_HIP(hipGetLastError());
}

size_t bn_train_scratch_floats(long M, int cs) {
  (void)M;
  return (size_t)BN_MAX_PARTS * cs + cs;
}

void launch_bn_train(float* x, long M, int C, int cs, const float* gamma, const float* beta, float eps, int act,
                     const float* res, float* stats, float* scratch, hipStream_t s) {
  M2S_CHECK(M > 0 && C > 0 && C <= cs && cs % 4 == 0, "bn_train: shape");
  const long rows_per = std::max<long>(256, (M + BN_MAX_PARTS - 1) / BN_MAX_PARTS);
  const int parts = (int)((M + rows_per - 1) / rows_per);
  float* part = scratch;
  float* coef = scratch + (size_t)BN_MAX_PARTS * cs;
  const dim3 pg(parts, ceil_div(C, 64));
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(bn_partial_kernel, pg, dim3(256), 0, s, x, M, C, cs, pass ? stats : nullptr, rows_per, part);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(nblk(C)), dim3(256), 0, s, part, parts, M, C, pass, gamma, eps, stats,
                       coef);
  }
  hipLaunchKernelGGL(bn_apply_kernel, dim3(nblk(M * (cs / 4))), dim3(256), 0, s, x, M, C, cs, stats, coef, beta, act,
                     res);
  M2S_HIP(hipGetLastError());
}

void launch_to_nchw(const float* x, int N, int P, int C, int cs, float* y, hipStream_t s) {
  hipLaunchKernelGGL(to_nchw_kernel, dim3(nblk((long)N * C * P)), dim3(256), 0, s, x, N, P, C, cs, y);
  M2S_HIP(hipGetLastError());
}

void launch_gap_nchw(const float* x, long NC, int P, float* y, hipStream_t s) {
  if (NC <= 0) return;
  hipLaunchKernelGGL(gap_nchw_kernel, dim3(nblk(NC)), dim3(256), 0, s, x, NC, P, y);
  M2S_HIP(hipGetLastError());
}

void launch_gap_nchw_bwd(const float* dy, long NC, int P, float* dx, hipStream_t s) {
  if (NC <= 0) return;
  hipLaunchKernelGGL(gap_nchw_bwd_kernel, dim3(nblk(NC * P)), dim3(256), 0, s, dy, NC, P, dx);
  M2S_HIP(hipGetLastError());
}

void launch_lstm_train_step(const float* pre, const float* whh, float* gates, float* cells, float* hid, int B, int T,
                            int H, int step, hipStream_t s) {
  M2S_CHECK(H % 8 == 0 && (32 * H + 32) * sizeof(float) <= 160 * 1024, "lstm_train: hidden size");
  const size_t lds = (32 * (size_t)H + 32) * sizeof(float);
  allow_lds(reinterpret_cast<const void*>(&lstm_train_step_kernel));
  hipLaunchKernelGGL(lstm_train_step_kernel, dim3(H / 8, 2), dim3(256), lds, s, pre, whh, gates, cells, hid, B, T, H,
                     step);
  M2S_HIP(hipGetLastError());
}

void launch_lstm_bptt_step(const float* whh_t, const float* dy, const float* gates, const float* cells, float* dc,
                           float* dg, int B, int T, int H, int step, hipStream_t s) {
  M2S_CHECK(H % 8 == 0 && (32 * (size_t)H + 8) * sizeof(float) <= 160 * 1024, "lstm_bptt: hidden size");
  const size_t lds = (32 * (size_t)H + 8) * sizeof(float);
  allow_lds(reinterpret_cast<const void*>(&lstm_bptt_step_kernel));
  hipLaunchKernelGGL(lstm_bptt_step_kernel, dim3(H / 8, 2), dim3(256), lds, s, whh_t, dy, gates, cells, dc, dg, B, T, H,
                     step);
  M2S_HIP(hipGetLastError());
}

void launch_lstm_hprev(const float* hid, float* hp, int B, int T, int H, hipStream_t s) {
  hipLaunchKernelGGL(lstm_hprev_kernel, dim3(nblk(2L * B * T * H)), dim3(256), 0, s, hid, hp, B, T, H);
  M2S_HIP(hipGetLastError());
}

void launch_transpose(const float* x, int planes, int rows, int cols, float* y, hipStream_t s) {
  hipLaunchKernelGGL(transpose_kernel, dim3(ceil_div(cols, 32), ceil_div(rows, 32), planes), dim3(256), 0, s, x, rows,
                     cols, y);
  M2S_HIP(hipGetLastError());
}

}  // namespace m2s
