// Implicit-GEMM convolution on MFMA (the workhorse of both the CNN encoder and the vocoder).
//
// One kernel family covers every dense conv of the hot path, channel-last layouts:
//   KIND_CONV2D : NHWC 2-D conv, square kernel ks, stride, TF-SAME pads (pad_t, pad_l)
//                 (timm conv_stem/conv/conv_exp/conv_pw/conv_pwl, mri_acoustic_model.py:28-34)
//   KIND_CONV1D : NLC 1-D conv, taps ks, dilation, left pad (causal MRF convs, conv_pre;
//                 models.py:11-49,94,114-115)
//   KIND_CONVT  : one output phase r of a ConvTranspose1d (stride u) as a 1-D conv over the
//                 input with reversed taps (models.py:98-101,117-118); grid.z = phase
//   KIND_GEMM   : plain row GEMM (1x1 conv at stride 1, LSTM input projection)
//
// GEMM view: D[n][m] = sum_k W[n][k] * X[m][k], n = output channel, m = output position,
// k = (tap, input channel).  The MFMA A operand is the weight tile, B is the activation
// tile, so each lane ends up holding 4 consecutive output channels of ONE position and
// the epilogue stores 8/16 contiguous bytes (channel-last) per lane.
#pragma once

#include "m2s_common.hpp"

namespace m2s {

enum ConvKind { KIND_CONV2D = 0, KIND_CONV1D = 1, KIND_CONVT = 2, KIND_GEMM = 3 };
enum Act { ACT_NONE = 0, ACT_SILU = 1, ACT_LRELU = 2, ACT_SIGMOID = 3 };
enum InXform { IN_NONE = 0, IN_LRELU = 1, IN_SE_SCALE = 2 };

struct ConvArgs {
  const void* x;        // input activations, channel-last, channel stride cs_in
  const void* w;        // packed weights [phase][n_pad][kp]  (T)
  const float* bias;    // [n_pad] fp32 (zero padded)
  const void* res;      // residual, same layout as y (or null)
  void* y;              // output, channel-last, channel stride cs_out
  const void* in_scale; // IN_SE_SCALE: [img][cs_in] in the compute dtype (SE gates)
  const float* wscale;  // fp8 operands (M2S_DT_FP8): [n_pad] per-output-channel weight scales, else null
  int kind;
  int M;                // GEMM rows (output positions per phase)
  int cs_in, cs_out;    // channel strides
  int n_pad;            // weight rows per phase (>= grid.y * N tile)
  int kp;               // weight row length
  int ntaps;            // taps (ks*ks for 2-D)
  int tpc;              // taps per K chunk (KC / cs_in if cs_in < KC else 1)
  // 2-D
  int IH, IW, OH, OW, ks, stride, pad_t, pad_l;
  // 1-D / transposed
  int L_in, L_out, dil, pad_left;
  int ct_u, ct_pad, ct_k;  // transposed conv: stride, padding, kernel size
  // epilogue
  int act; float act_slope;
  int in_xform; float in_slope;
  int accum;            // 0: y = v ; 1: y = y_prev + v ; 2: y = (y_prev + v) / accum_div
  float accum_div;
  // split conv_gemm only (the pre-activated MRF chain, model.cpp Vocoder::run_t):
  float res_unslope;    // != 0: res holds lrelu(x); x = r > 0 ? r : r * res_unslope (slope 0.1 -> 10)
  int act_after_res;    // act applied after the residual add (y = lrelu(v + x)) instead of before it
  // fp32 conv_igemm only: the four waves of a workgroup split the K chunks of one wave's rows (the BiLSTM input
  // projection of a small pass, model.cpp)
  int kwave;
};

// Up to CONV_BATCH 1-D convs of one shape (same kind, M, cs_in, cs_out, n_pad; own x / w / bias / res
// / y / taps / dilation) in ONE launch, grid.z = batch index: the independent resblocks of an MRF
// stage (models.py:119-125) share a launch so their tiles fill the chip together.
constexpr int CONV_BATCH = 3;
struct ConvBatch {
  ConvArgs a[CONV_BATCH];
};

// flops / bytes: algorithmic work of this launch, recorded by the profiler (m2s_prof_*).
// bf16 and split fp32 (sp_t) run the LDS-DMA pipelined kernel (conv_gemm.hip); fp32 (the exact
// f32-MFMA parity path) runs the direct-load kernel of conv_igemm.hip.
template <typename T>
void launch_conv(const ConvArgs& a, hipStream_t s, double flops = 0.0, double bytes = 0.0);
// split: x, w, res, y and in_scale hold [hi | lo] rows (m2s_common.hpp sp_t); w rows are 2 * kp long.
// a.wscale set (bf16 storage only): e4m3 operands - w holds e4m3-grid values (exact in bf16) of
// w / wscale[n], the activation fragments are rounded to e4m3 after the LDS read, the products run
// on v_mfma_f32_16x16x32_fp8_fp8 and the epilogue multiplies by wscale[n].
void launch_conv_gemm(const ConvArgs& a, bool split, hipStream_t s, double flops, double bytes);
// n (1..CONV_BATCH) split-fp32 KIND_CONV1D convs of one shape in one launch; put the longest K first
// (blocks dispatch in z order, so the longest tiles start first and the short ones fill the tail).
void launch_conv_gemm_batch(const ConvArgs* a, int n, hipStream_t s, double flops, double bytes);
// bf16 3x3 stride-1 convs with cs_in in {32, 64}: persistent LDS-resident-weight kernel
// (conv_halo.hip); launch_conv_gemm routes them there.
bool conv_halo_supported(const ConvArgs& a);
void launch_conv_halo(const ConvArgs& a, hipStream_t s, double flops, double bytes);

// Host-side helpers shared by the packers.
inline int conv_tpc(int cs_in, int kc) { return cs_in < kc ? kc / cs_in : 1; }
inline int conv_kp(int ntaps, int cs_in, int kc) {
  int tpc = conv_tpc(cs_in, kc);
  return round_up(ntaps, tpc) * cs_in;
}

}  // namespace m2s
