// Launchers for the non-GEMM kernels of the hot path.
#pragma once

#include "m2s_common.hpp"

namespace m2s {

// Asynchronous failure report of the persistent kernels' bounded waits (LDS flag rings, grid hand-offs): the
// engine's host-mapped error word takes one of these codes; m2s_acoustic_status turns it into an error.
enum AsyncCode : unsigned { M2S_ASYNC_LSTM = 1u, M2S_ASYNC_WS = 2u };
struct AsyncReport {
  unsigned spin_max = 1u << 20;  // polls per LDS flag wait (each ~1 s_sleep) before it counts as timed out
  unsigned* err = nullptr;       // host-mapped error word, or null (no report)
};
// one lane of the wave stores `code` to the host-mapped word (system scope: the host reads it after a sync)
__device__ __forceinline__ void report_async(unsigned* err, unsigned code, int lane) {
  if (err && lane == 0) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// conv_stem (3x3 s2 TF-SAME, grey repeat folded: w[o][9]) + bn1 + SiLU.  frames fp32 (N,H,W)
// -> y (N,OH,OW,cs_out) T.  timm conv_stem/bn1, mri_acoustic_model.py:41-46.
template <typename T>
void launch_stem(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l,
                 const float* w9, const float* bias, int cout, int cs_out, T* y, hipStream_t s);

// conv_dw (3x3 depthwise, stride 1/2, TF-SAME) + bn2 + SiLU, plus per-(image, pixel block, channel)
// partial sums of the output (SE squeeze).  x (N,IH,IW,cs) -> y (N,OH,OW,cs),
// sums (N, dw_pixel_blocks(OH, OW), cs) fp32.  (dwse.hip)
int dw_pixel_blocks(int OH, int OW);
template <typename T>
void launch_dwconv(const T* x, int N, int IH, int IW, int OH, int OW, int stride, int pad_t, int pad_l,
                   int C, int cs, const float* w9, const float* bias, T* y, float* sums, hipStream_t s);

// SE squeeze: mean (N, cs) in the compute dtype from the depthwise partial sums (N, npb, cs).
// (The excitation conv_reduce -> SiLU -> conv_expand -> sigmoid then runs as two MFMA GEMMs.)
template <typename T>
void launch_se_mean(const float* psum, int N, int npb, int cs, float inv_count, T* mean, hipStream_t s);

// Fused conv_pw + bn1 + SiLU + conv_dw (stride 1) + bn2 + SiLU + SE squeeze for maps whose
// haloed tile fits a workgroup ((OH+2)(OW+2) <= 400 bf16 / 324 split, OH*OW <= 256): x (N,P,cs_in) ->
// y (N,P,cs_mid), se_mean (N,cs_mid).  wpw packed [>=ceil64(cs_mid)][kp], bpw likewise padded.
// bf16: x/y/se_mean bf16, wdw = tap-major [9][cs_mid] bf16 weights in the dword half of their channel
// (uint32).  split (bf16x3): x/y/se_mean sp_t, wpw rows [hi kp | lo kp], wdw = fp32 [9][cs_mid].
// (ir_fused.hip)
bool ir_fused_supported(int OH, int OW, int cs_in, int cs_mid, bool split);
void launch_ir_pwdw(const void* x, int N, int cs_in, int kp, const void* wpw, const float* bpw, const void* wdw,
                    const float* bdw, int OH, int OW, int cs_mid, void* y, void* se_mean, bool split, double flops,
                    double bytes, hipStream_t s, bool f8_out = false, const void* x8 = nullptr,
                    const void* w8 = nullptr, const float* wsc = nullptr, int kp8 = 0);
// f8_out (bf16 inputs and weights): the depthwise output y is stored as OCP e4m3 bytes [N][P][cs_mid]
// (saturated to +-448), the operand of launch_se_gemm_f8; the SE means stay bf16 (exact sums).
// x8 (with f8_out): the expand runs on e4m3 too: x8 = the block input as e4m3 rows of kp8 bytes (kp8 = cs_in
// rounded up to 128, zero past cs_in; launch_se_*_f8 y8 / launch_rows_e4m3), w8 = e4m3 [rows][kp8] with
// per-channel scales wsc (pack_gemm_f8), one block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 per 128 k.
// bf16 (N*P, cs) rows -> e4m3 rows of ld8 bytes (zeros past cs): an e4m3 expand operand for a block input
// no e4m3 producer wrote.
void launch_rows_e4m3(const void* x, long rows, int cs, void* y8, int ld8, hipStream_t s);

// fp8 engines: the SE-gated conv_pwl (+ bn3 + skip) of a stride-1 IR block on v_mfma_scale_f32_16x16x128_f8f6f4:
// y (M, cs_out) bf16 = wscale[n] * sum_k w8[n][k] e4m3(gate[m / P][k] x8[m][k]) + bias[n] (+ res (M, cs_out) bf16).
// x8: e4m3 (M, cs_in) (launch_ir_pwdw f8_out); w8: e4m3 [n_pad][kp], kp = cs_in rounded up to 128, zero
// padded (pack_gemm_f8); gate: bf16 (M / P, cs_in).  P % 64 == 0, cs_out <= 224.  (gemm128.hip)
// y8 (optional): an e4m3 copy of y, rows of ld8 bytes (the next IR block's expand operand).
bool se_gemm_f8_supported(int P, int cs_in, int cs_out);
void launch_se_gemm_f8(const void* x8, int M, int P, int cs_in, const void* w8, int kp, int n_pad, const float* wscale,
                       const float* bias, const void* gate, const void* res, void* y, int cs_out, hipStream_t s,
                       double flops, double bytes, void* y8 = nullptr, int ld8 = 0);

// bf16x3 engines: the same SE-gated conv_pwl (+ bn3 + skip) in split fp32 on gemm128.hip: x interleaved split
// (M, cs_in / 32, [hi 32 | lo 32]) (il_st8), w split rows [hi cs_in | lo cs_in] (conv_gemm packing, n_pad rows),
// gate split (M / P, [hi cs_in | lo cs_in]), res / y split (M, [hi cs_out | lo cs_out]).  P % 64 == 0.
bool se_gemm_sp_supported(int P, int cs_in, int cs_out);
void launch_se_gemm_sp(const void* x, int M, int P, int cs_in, const void* w, int n_pad, const float* bias,
                       const void* gate, const void* res, void* y, int cs_out, hipStream_t s, double flops, double bytes);

// The same split SE-gated conv_pwl as a persistent warp-specialised GEMM: loader waves fill a 3-slot LDS
// ring by LDS-DMA and consumer waves compute, synchronised by per-slot FULL / FREE counters in LDS (no
// per-K-step barrier; the ring runs across tiles).  Same operands as launch_se_gemm_sp; P % 256 == 0 with
// cs_out <= 128 (16x16 maps) or P == 64 with 128 < cs_out <= 224 (8x8 maps).  (se_ws.hip)
bool se_ws_supported(int P, int cs_in, int cs_out);
// Every FULL / FREE wait is bounded by rep.spin_max polls; a timeout is reported through rep.err and the
// consumer's tiles from then on are stored as NaN.
// x_f32: x holds plain fp32 rows [M][cs_in] (ir_ws's fm32 output) instead of the interleaved split layout.
void launch_se_ws(const void* x, int M, int P, int cs_in, const void* w, int n_pad, const float* bias, const void* gate,
                  const void* res, void* y, int cs_out, hipStream_t s, double flops, double bytes, AsyncReport rep = {},
                  bool x_f32 = false);

// fp8 engines: launch_se_gemm_f8's operation (e4m3 x8 / w8, bf16 gate / res / y) on the same warp-specialised
// flag ring.  (se_ws.hip)
bool se_ws_f8_supported(int P, int cs_in, int cs_out);
// y8 (optional): an e4m3 copy of y, rows of ld8 bytes (the next IR block's e4m3 expand operand, launch_ir_pwdw x8)
void launch_se_ws_f8(const void* x8, int M, int P, int cs_in, const void* w8, int kp, int n_pad, const float* wscale,
                     const float* bias, const void* gate, const void* res, void* y, int cs_out, hipStream_t s, double flops,
                     double bytes, void* y8 = nullptr, int ld8 = 0, AsyncReport rep = {});

// The same for a stride-2 depthwise (TF-SAME, top / left pads pad_t / pad_l) on an IH x IW <= 256-pixel
// conv_pw map: y (N, OH*OW, cs_mid), se_mean over the OH x OW output.  (ir_fused.hip)
// Split-fp32 IR front half (conv_pw + bn1 + SiLU + conv_dw + bn2 + SiLU + SE squeeze) on W = 8 / 16 maps as
// one persistent warp-specialised workgroup per CU; same outputs as launch_ir_pwdw(split = true) (stride 1) and
// launch_ir_pwdw_s2(split = true) (stride 2: 16x16 -> 8x8, TF-SAME pads pad_t / pad_l; y is the OH x OW map).
// wdw: fp32 tap-major [9][cs_mid].  (ir_ws.hip)
bool ir_ws_supported(int H, int W, int cs_in, int kp, int cs_mid);
bool ir_ws_s2_supported(int H, int W, int cs_in, int kp, int cs_mid, int OH, int OW, int pad_t, int pad_l);
// The hand-off waits are bounded by rep.spin_max polls; a timeout is reported through rep.err and the images of
// that workgroup get NaN SE means (their block output is NaN).
void launch_ir_ws(const void* x, int N, int H, int W, int cs_in, int kp, int cs_mid, const void* wpw, const float* bpw,
                  const float* wdw, const float* bdw, void* y, void* se_mean, double flops, double bytes,
                  hipStream_t s, AsyncReport rep = {}, int stride = 1, int OH = 0, int OW = 0, int pad_t = 0,
                  int pad_l = 0, double spill = 0.0, bool fm32 = false);
// fm32: y is stored as plain fp32 rows [N * OH * OW][cs_mid] (for launch_se_ws(x_f32 = true)) instead of the
// interleaved split layout: one 16-byte store per 4 channels, no split in the consumers.
// Stride-2 IR front half on bands of 4 output rows (blocks.3.0: 32x32 -> 16x16), split fp32 or bf16: y =
// the SE GEMM's operand (N, OH*OW, cs_mid; split: interleaved hi/lo), psum = squeeze partial sums
// (N, OH / 4, cs_mid) for launch_se_mean.  wdw: fp32 tap-major [9][cs_mid].  (ir_s2band.hip)
int ir_s2band_bands(int OH);
bool ir_s2band_supported(int IH, int IW, int OH, int OW, int cs_in, int kp, int cs_mid);
void launch_ir_s2band(const void* x, int N, int IH, int IW, int cs_in, int kp, const void* wpw, const float* bpw,
                      const float* wdw, const float* bdw, int OH, int OW, int pad_t, int pad_l, int cs_mid, void* y,
                      float* psum, bool split, double flops, double bytes, hipStream_t s, bool f8_out = false);
bool ir_fused_s2_supported(int IH, int IW, int cs_in, int cs_mid, bool split);
void launch_ir_pwdw_s2(const void* x, int N, int cs_in, int kp, const void* wpw, const float* bpw, const void* wdw,
                       const float* bdw, int IH, int IW, int OH, int OW, int pad_t, int pad_l, int cs_mid, void* y,
                       void* se_mean, bool split, double flops, double bytes, hipStream_t s, bool f8_out = false,
                       const void* x8 = nullptr, const void* w8 = nullptr, const float* wsc = nullptr, int kp8 = 0);

// Fused HiFi-GAN ResBlock1 (all (c1, c2) pairs of one resblock + the MRF running sum), bf16 for C in
// {32, 64} or split fp32 (split: x, S as [hi C | lo C] per position) for C = 32:
// x (B, L, C) -> S (B, L, C) with S = x' (accum 0), S += x' (1), S = (S + x') / div (2).  (mrf_fused.hip)
// Split-fp32 causal dilated Conv1d with the tile's input rows staged once in LDS (conv1d_halo.hip), for the
// C = 64 MRF convs; a[i].w in fragment order [tap][C/32][hi/lo][C/16][64 lanes][8] bf16
// (conv1d_halo_frag_elems), n batched convs of one shape (grid.z).
bool conv1d_halo_sp_supported(int C, int cs, int k, int dil);
size_t conv1d_halo_frag_elems(int C, int k);
void launch_conv1d_halo_sp(const struct ConvArgs* a, int n, hipStream_t s, double flops, double bytes);
// w1/w2 are in fragment order: [rb1_frag_taps(C, k, split)][hi/lo if split][C/16][C/32][64 lanes][8] bf16,
// element (tap t, n16, k32, lane, e) = W[n16*16 + lane%16][k32*32 + 8*(lane/16) + e][t] (zero taps past k).
bool rb1_fused_supported(int C, int cs, int k, const int* dil, int np, int kp, bool split);
int rb1_frag_taps(int C, int k, bool split);
void launch_rb1_fused(const bf16_t* x, bf16_t* s, int B, int L, int C, int k, int np, const int* dil,
                      const bf16_t* const* w1, const float* const* b1, const bf16_t* const* w2,
                      const float* const* b2, int kp, int accum, float div, bool split, double flops, double bytes,
                      hipStream_t st);

// conv_stem + bn1 + SiLU + blocks.0.0 (3x3 32->16 + SiLU) + blocks.0.1 (3x3 16->16 + SiLU + skip) in
// one kernel: frames (N,H,W) fp32 -> y (N,OH,OW,16).  w0/w1: packed conv rows (kp 288 / 160); bf16, or
// split fp32 (`split`: [hi | lo] weight rows, y in sp_t layout).  (stem_b0.hip)
void launch_stem_b0(const float* frames, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, const float* w9,
                    const float* b9, const void* w0, const float* b0, int kp0, const void* w1, const float* b1,
                    int kp1, void* y, bool split, double flops, double bytes, hipStream_t s);

// SqueezeExcite excitation (bf16, or split fp32 with split = true): gate (N, cs_mid) =
// sigmoid(W2 · SiLU(W1 · mean + b1) + b2), mean (N, cs_mid) from the squeeze; w1 packed [>= rd][kp1],
// w2 packed [>= mid][kp2] (split: rows [hi kp | lo kp]).  (se_excite.hip)
bool se_excite_supported(int rd, int kp2, int cs_mid);
void launch_se_excite(const void* mean, int N, int mid, int cs_mid, const void* w1, int kp1, const float* b1,
                      int rd, const void* w2, int kp2, const float* b2, void* gate, bool split, hipStream_t s);

// bf16 EdgeResidual (stride 1, skip) 32 -> 128 -> 32: conv_exp 3x3 + SiLU, conv_pwl 1x1, + x in one
// persistent kernel; x, y (N,H,W,32); wexp / wpwl in the kernel's fragment orders.  (er_fused.hip)
bool er_fused_supported(int H, int W, int cin, int mid, int cout, int kp_exp, int kp_pwl);
void launch_er_fused(const bf16_t* x, int N, int H, int W, const bf16_t* wexp, const float* bexp, const bf16_t* wpwl,
                     const float* bpwl, bf16_t* y, double flops, double bytes, hipStream_t s);

// fp8 engines: er_fused's block on e4m3 operands (v_mfma_scale_f32_16x16x128_f8f6f4): wexp e4m3 [3][8][2][64][16]
// (tap groups of four, per-channel scales sexp), wpwl e4m3 [2][2][64][16] (permuted K, scales spwl); x, y bf16
// (N,H,W,32); x8 (optional): the input as e4m3 bytes (N,H,W,32) from the producer (ers2_fused / er8_fused y8),
// y8 (optional, needs x8): e4m3 bytes of y for the next er8 block.  (er8_fused.hip)
bool er8_fused_supported(int H, int W, int cin, int mid, int cout);
void launch_er8_fused(const bf16_t* x, int N, int H, int W, const uint8_t* wexp, const float* sexp, const float* bexp,
                      const uint8_t* wpwl, const float* spwl, const float* bpwl, bf16_t* y, double flops, double bytes,
                      hipStream_t s, const uint8_t* x8 = nullptr, uint8_t* y8 = nullptr);

// bf16 EdgeResidual (stride 1, skip) 56 -> 224 -> 56 (channel strides 64 / 224 / 64): same fusion with the
// weights streamed through an LDS ring; wst = er2_stage_elems() bf16 in the kernel's stage order.
// (er2_fused.hip)
bool er2_fused_supported(int H, int W, int cs_in, int mid, int cout, int kp_exp, int kp_pwl);
int er2_stage_elems();
// fp8 engines: the same block (56 -> 224 -> 56, 32x32, skip) on e4m3 operands (er8w_fused.hip): x8 = the input as
// e4m3 bytes (N, H, W, 64) written by the producer block, wst = the e4m3 stage stream (er8w_stream_bytes(); conv_exp
// 5 K steps of [16 n16][2][64][16 B], then conv_pwl [4][2][2][64][16 B] with the permuted K), per-channel scales
// sexp [224] / spwl [64]; y8 (optional) = e4m3 of y for the next such block.
bool er8w_fused_supported(int H, int W, int cs_in, int mid, int cout);
size_t er8w_stream_bytes();
void launch_er8w_fused(const bf16_t* x, const uint8_t* x8, int N, int H, int W, const uint8_t* wst, const float* sexp,
                       const float* bexp, const float* spwl, const float* bpwl, bf16_t* y, uint8_t* y8, double flops,
                       double bytes, hipStream_t s);
void launch_er2_fused(const bf16_t* x, int N, int H, int W, const bf16_t* wst, const float* bexp, const float* bpwl,
                      bf16_t* y, double flops, double bytes, hipStream_t s);

// Split-fp32 EdgeResidual (stride 1, skip), (cs_in, mid, cs_out) in {(32, 128, 32), (64, 224, 64)}: conv_exp
// 3x3 + SiLU -> conv_pwl + x with the three-term products, weights streamed in W_hi / W_lo stages of
// `nt` = mid / 16 fragments; x, y in sp_t layout; wst = er_sp_nt_stages() stages of nt x [64][8] bf16.
// (er_sp_fused.hip)
bool er_sp_supported(int H, int W, int cs_in, int mid, int cs_out);
int er_sp_nt_stages(int cs_in, int mid, int cs_out, int* nt);
// merged: blocks.1's W_hi and W_lo stages share one ring slot (half the barriers, same MFMA order).
void launch_er_sp(const void* x, int N, int H, int W, int cs_in, int mid, int cs_out, const void* wst, const float* bexp,
                  const float* bpwl, void* y, double flops, double bytes, hipStream_t s, bool merged = true);

// bf16 stride-2 EdgeResidual (no skip), (cs_in, mid, cs_out) in {(16, 64, 32), (32, 128, 64)}: conv_exp
// 3x3/s2 TF-SAME + SiLU -> conv_pwl; x (N,H,W,cs_in) -> y (N,OH,OW,cs_out); wexp ers2_exp_elems() bf16 in
// the kernel's fragment order, wpwl [cs_out/16][mid/32][64][8] with er_fused.hip's K permutation.
// (ers2_fused.hip)
bool ers2_fused_supported(int OH, int OW, int cs_in, int mid, int cs_out, int kp_exp, int kp_pwl);
int ers2_exp_elems(int cs_in, int mid);
// split fp32 blocks.1.0 (16 -> 64 -> 32): wexp [hi/lo][k-step][n16][lane][8], wpwl [hi/lo][n16][k-step][lane][8]
bool ers2_sp_supported(int OH, int OW, int cs_in, int mid, int cs_out);
void launch_ers2_sp(const void* x, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, int cs_in, int mid,
                    int cs_out, const void* wexp, const float* bexp, const void* wpwl, const float* bpwl, void* y,
                    double flops, double bytes, hipStream_t s);
void launch_ers2_fused(const bf16_t* x, int N, int H, int W, int OH, int OW, int pad_t, int pad_l, int cs_in, int mid,
                       int cs_out, const bf16_t* wexp, const float* bexp, const bf16_t* wpwl, const float* bpwl,
                       bf16_t* y, double flops, double bytes, hipStream_t s, uint8_t* y8 = nullptr);

// Decoded frames -> model input: uint8 (N,H,W) grey or (N,H,W,3) BGR -> fp32 (N,H,W) in [0, 1]
// (_preprocess_frame, run_mri_video_inference.py:34-54, minus the host-side resize).  (preprocess.hip)
void launch_preprocess(const uint8_t* frames, int N, int H, int W, int channels, float* out, hipStream_t s);

// Global average pool: x (N,P,cs) T -> feats (N,C) fp32 (dense, row stride C).
template <typename T>
void launch_gap(const T* x, int N, int P, int C, int cs, float* feats, hipStream_t s);

// One BiLSTM time step for both directions (step s: fwd t = s, bwd t = T-1-s).
// pre (B,T,8H) fp32 = x W_ih^T + b_ih + b_hh for [fwd | bwd]; whh (2,4H,H); hs (2,B,T,H); cst (2,B,H).
void launch_lstm_step(const float* pre, const float* whh, float* hs, float* cst, int B, int T, int H,
                      int step, hipStream_t s);

// The same recurrence for all T steps in ONE persistent launch (lstm_persistent.hip): W_hh resident
// in VGPRs across 160 workgroups, a release/acquire counter barrier per step.  H = 640 only.
// `sync` = lstm_persistent_sync_bytes() of device memory (reset by the launcher).
bool lstm_persistent_supported(int H);
size_t lstm_persistent_sync_bytes();
// `spin_max` bounds each barrier wait (polls with s_sleep 1); on a timeout the kernel stores 1 to
// `err_host` (pinned, host-mapped) and writes NaN to the rest of the outputs.
// Small batches (B <= 4): the same recurrence with h exchanged as data-tagged granules instead of a
// counter barrier, VALU dot products (lstm_persistent.hip).  `sync` = lstm_small_sync_bytes().
bool lstm_small_supported(int B, int H);
size_t lstm_small_sync_bytes();
// epoch: the engine's epoch count for a sync buffer of its own (tags continue across calls, no memset; null = zero
// the buffer every call)
void launch_lstm_small(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                       unsigned* err_host, hipStream_t s, unsigned* epoch = nullptr);
constexpr unsigned LSTM_SPIN_MAX = 1u << 24;
// 4 < B <= 64: the same granule exchange with 512-thread workgroups, sequences in chunks of 16 whose
// sweep overlaps the previous chunk's dot products (lstm_persistent.hip).  `sync` = lstm_mid_sync_bytes().
bool lstm_mid_supported(int B, int H);
size_t lstm_mid_sync_bytes();
void launch_lstm_mid(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                     unsigned* err_host, hipStream_t s);
void launch_lstm_persistent(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync,
                            unsigned spin_max, unsigned* err_host, hipStream_t s);
// B > 4 in split fp32 (the bf16x3 / bf16 / fp8 engines): three bf16 MFMA terms over W_hh and h_t split
// hi / lo, h_t published split by write-through stores behind per-workgroup flags (no fences).
// Split engines, 5..16 sequences: lstm_x3's arithmetic with the h_t hand-off as data-tagged granules (no flag round
// trip, no store drain); `sync` = lstm_x3g_sync_bytes() (epoch-tagged, see launch_lstm_small).  (lstm_persistent.hip)
bool lstm_x3g_supported(int B, int H);
size_t lstm_x3g_sync_bytes();
void launch_lstm_x3g(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                     unsigned* err_host, hipStream_t s, unsigned* epoch = nullptr);
// `sync` = lstm_x3_sync_bytes() (flags reset by the launcher).
size_t lstm_x3_sync_bytes();
void launch_lstm_x3(const float* pre, const float* whh, float* hs, int B, int T, int H, void* sync, unsigned spin_max,
                    unsigned* err_host, hipStream_t s);

// head: y = hs[0] + hs[1] (sum merge); out = y W^T + b.  wt (H, n_mels) transposed weight.
void launch_mel_head(const float* hs, int rows, int H, const float* wt, const float* b, int n_mels,
                     float* out, hipStream_t s);

// mel glue: db = x*std + mean; ln = log(clamp(10^(db/10), 1e-5)).  Any output may be null.
// ln_t (rows, cs) T channel-last copy feeds the vocoder.
template <typename T>
void launch_mel_glue(const float* x, int rows, int n_mels, const float* mean, const float* std_,
                     float* db, float* ln, T* ln_t, int cs, hipStream_t s);

// mel (B,C,T) fp32 [layout 0] or (B,T,C) fp32 [layout 1] -> (B,T,cs) T.
template <typename T>
void launch_mel_to_nlc(const float* mel, int B, int C, int Tn, int layout, T* y, int cs, hipStream_t s);

// conv_post: leaky_relu(0.01) -> right pad 6 -> Conv1d(C,1,7) -> tanh.  x (B,L,cs) T -> wav (B,L) fp32.
template <typename T>
void launch_conv_post(const T* x, int B, int L, int C, int cs, const float* w /*[7][C]*/, float bias,
                      float* wav, hipStream_t s);

// y = a + b (fp32, n elements)
void launch_add2(const float* a, const float* b, float* y, long n, hipStream_t s);
// fp8 engines: y (n bytes, e4m3) = lrelu(x) for bf16 x, n % 8 == 0  (kernels.hip)
void launch_lrelu_e4m3(const bf16_t* x, uint8_t* y, long n, float slope, hipStream_t s);
// fp8 engines, HiFi-GAN MRF conv at C in {128, 256} (models.py:11-49, causal left pad (k - 1) dil): x8 e4m3
// (B, L, C) already LeakyReLU'd; w8 e4m3 [C][k C] tap-major (pack_gemm_f8), per-channel scales; v = conv + bias
// (+ res bf16); y bf16 = v, or with accum 1 / 2 the MRF running sum y + v / (y + v) / accum_div; y8 (e4m3) =
// lrelu(v, slope8).  Either output may be null.  (gemm128.hip)
bool conv1d_f8_supported(int C, int k);
void launch_conv1d_f8(const void* x8, int B, int L, int C, int k, int dil, const void* w8, const float* wscale,
                      const float* bias, const void* res, void* y, void* y8, float slope8, int accum, float accum_div,
                      hipStream_t s, double flops, double bytes);

// (rows, cs) T -> (rows, C) fp32 dense (debug taps)
template <typename T>
void launch_unpad(const T* x, long rows, int C, int cs, float* y, hipStream_t s);

}  // namespace m2s
