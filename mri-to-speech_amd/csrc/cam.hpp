// Grad-CAM path of the acoustic model (the reference's scripts/mri_gradcam_formant.py:128-279):
// a train-mode backbone forward (BatchNorm on batch statistics, timm / torch semantics) and the
// autograd kernels behind the feature-map gradient: BiLSTM forward with saved activations and its
// backward through time, the head Linear, GAP.  Exact fp32 throughout (the reference runs fp32).
#pragma once

#include <vector>

#include "conv_igemm.hpp"
#include "model.hpp"

namespace m2s {

// ---- kernels (cam.hip) ------------------------------------------------------------------------
// C[m][n] (accumulate ? += : =) sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] (+ bias1[n] + bias2[n]);
// C row-major with leading dimension ldc.  fp32 FMA, k ascending per output.
void launch_gemm_f32(int M, int N, int K, const float* A, long sam, long sak, const float* B, long sbk, long sbn,
                     float* C, long ldc, const float* bias1, const float* bias2, bool accumulate, hipStream_t s);
// out[c] (+)= sum over rows of x[r*ld + c], c < cols (rows ascending)
void launch_colsum(const float* x, int rows, int cols, long ld, float* out, bool accumulate, hipStream_t s);
// conv_stem without bias / activation: frames (N,H,W) -> z (N,OH,OW,32) with w9 [32][9] (RGB repeat folded)
void launch_stem_raw(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, const float* w9,
                     float* z, hipStream_t s);
// depthwise 3x3 without bias / activation: x (N,IH,IW,cs) -> z (N,OH,OW,cs), w tap-major [9][cs]
void launch_dw_raw(const float* x, int N, int IH, int IW, int OH, int OW, int stride, int pad_t, int pad_l, int cs,
                   const float* w, float* z, hipStream_t s);
// BatchNorm with batch statistics over rows x (M, cs), C real channels:
//   stats[0:C] = mean, stats[C:2C] = biased variance (two passes, partial sums reduced in double);
//   x <- act((x - mean) * gamma / sqrt(var + eps) + beta) (+ res), pad channels zero.
size_t bn_train_scratch_floats(long M, int cs);
void launch_bn_train(float* x, long M, int C, int cs, const float* gamma, const float* beta, float eps, int act,
                     const float* res, float* stats, float* scratch, hipStream_t s);
// (N,P,cs) channel-last -> (N,C,P) dense
void launch_to_nchw(const float* x, int N, int P, int C, int cs, float* y, hipStream_t s);
// GAP of NCHW maps and its backward: y (N*C) = mean over P; dx (N*C*P) = dy / P
void launch_gap_nchw(const float* x, long NC, int P, float* y, hipStream_t s);
void launch_gap_nchw_bwd(const float* dy, long NC, int P, float* dx, hipStream_t s);
// BiLSTM with saved activations, both directions, one launch per time step (grid: H/8 unit groups x 2).
//   pre (B,T,8H) = x W_ih^T + b_ih + b_hh for [fwd 4H | bwd 4H]; whh (2,4H,H);
//   gates (2,B,T,4H) post-activation i,f,g,o; cells, hid (2,B,T,H)
void launch_lstm_train_step(const float* pre, const float* whh, float* gates, float* cells, float* hid, int B, int T,
                            int H, int step, hipStream_t s);
// backward step (reverse of the forward order per direction): whh_t (2,H,4H) = W_hh^T, dy (B,T,H) (the
// sum merge sends the same dy to both directions), dc (2,B,H) carried cell gradient, dg (2,B,T,4H) out
void launch_lstm_bptt_step(const float* whh_t, const float* dy, const float* gates, const float* cells, float* dc,
                           float* dg, int B, int T, int H, int step, hipStream_t s);
// hp (2,B,T,H): the hidden state each step consumed (fwd: h[t-1], bwd: h[t+1], zero at the ends)
void launch_lstm_hprev(const float* hid, float* hp, int B, int T, int H, hipStream_t s);
// (rows, cols) -> (cols, rows), for `planes` consecutive matrices
void launch_transpose(const float* x, int planes, int rows, int cols, float* y, hipStream_t s);

// ---- BiLSTM (nn.LSTM 1 layer, bidirectional, batch_first, sum merge) and Linear with autograd ------
// x (B,T,C); weights in nn.LSTM layout per direction d (0 fwd, 1 reverse): w_ih (4H,C), w_hh (4H,H),
// b_ih / b_hh (4H).  forward: y (B,T,H) = h_fwd + h_bwd, saved gates (2,B,T,4H), cells / hid (2,B,T,H).
// backward: dy (B,T,H) -> dx (B,T,C), dw_ih / dw_hh / db (= d b_ih = d b_hh) per direction; any output
// pointer may be null.
size_t bilstm_train_workspace_bytes(int B, int T, int C, int H);
void bilstm_train_forward(const float* x, int B, int T, int C, int H, const float* const w_ih[2],
                          const float* const w_hh[2], const float* const b_ih[2], const float* const b_hh[2], float* y,
                          float* gates, float* cells, float* hid, void* ws, size_t wsb, hipStream_t s);
void bilstm_train_backward(const float* x, const float* dy, int B, int T, int C, int H, const float* const w_ih[2],
                           const float* const w_hh[2], const float* gates, const float* cells, const float* hid,
                           float* dx, float* const dw_ih[2], float* const dw_hh[2], float* const db[2], void* ws,
                           size_t wsb, hipStream_t s);
// y (rows,out) = x (rows,in) W^T + b ; backward dx = dy W, dw = dy^T x, db = column sums of dy
void linear_forward(const float* x, int rows, int in, int out, const float* w, const float* b, float* y, hipStream_t s);
void linear_backward(const float* dy, const float* x, int rows, int in, int out, const float* w, float* dx, float* dw,
                     float* db, hipStream_t s);

// ---- the train-mode backbone ---------------------------------------------------------------------
class CamBackbone {
 public:
  CamBackbone(const StateDict& sd, int device);
  int device() const { return device_; }
  // BatchNorm layers in state-dict order (conv_stem's bn1, then per block bn1 / bn2 / bn3); stats layout
  // per layer [mean C | var C]
  int bn_layers() const { return (int)bn_.size(); }
  int bn_channels(int i) const { return bn_[i].C; }
  int bn_stats_floats() const;
  size_t workspace_bytes(int N, int H, int W) const;
  // frames (N,H,W) -> the five timm feature maps (taps[i]: (N,C,OH,OW) fp32 dense, shapes as
  // effnet_features), bn_stats: batch mean / biased var of every BN layer
  void forward(const float* frames, int N, int H, int W, float* const taps[5], float* bn_stats, void* ws, size_t wsb,
               hipStream_t s);

 private:
  struct BNp {
    int C = 0;
    size_t g = 0, b = 0;  // gamma, beta (arena offsets)
  };
  struct Blk {
    int type = 0, stride = 1, cin = 0, cout = 0, mid = 0, rd = 0;
    bool skip = false;
    PConv c1, c2, se1, se2;
    size_t dw = 0;
    int bn[3] = {-1, -1, -1};
  };
  int device_;
  Arena arena_;
  size_t stem_w_ = 0;
  int stem_bn_ = 0;
  std::vector<BNp> bn_;
  std::vector<Blk> blocks_;
};

}  // namespace m2s
