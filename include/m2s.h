/*
 * m2s.h - C ABI of libm2s, the MI355X (gfx950) implementation of the rtMRI video -> mel ->
 * waveform inference hot path of YamaneKoyo/mri-to-speech.
 *
 * Plain pointers and sizes only.  Every device pointer is a HIP device allocation on the
 * object's device; `stream` is a hipStream_t (NULL = default stream).  Every call is
 * asynchronous on `stream` unless stated otherwise.  Functions return M2S_OK or an error
 * code; m2s_last_error() gives a thread-local message.  Nothing here falls back to the CPU:
 * without a gfx950 device the create calls fail with M2S_E_NODEV.
 *
 * Reference interfaces replaced (paths inside the reference repository):
 *   m2s_acoustic_*      OTNLikeCNNBiLSTM built by build_acoustic_model(**kw) and loaded with
 *                       load_state_dict(strict=False)   mri2speech_code/mri_acoustic_model.py:74-156,
 *                       scripts/run_mri_video_inference.py:119-148
 *   m2s_acoustic_forward   OTNLikeCNNBiLSTM.forward (eval)   mri_acoustic_model.py:116-136
 *   m2s_effnet_forward     EffNetV2B2Backbone.forward + GlobalAvgPool   mri_acoustic_model.py:15-18,39-48
 *   m2s_bilstm_summerge    BiLSTMSumMerge.forward + head Linear   mri_acoustic_model.py:67-72,135
 *   m2s_mel_glue           denormalize_mel + dB -> ln-power   run_mri_video_inference.py:160-163,227-233
 *   m2s_vocoder_*          Generator(h) + load_state_dict(ckpt['generator']) + weight-norm removal
 *                          models.py:88-109, run_mri_video_inference.py:89-116
 *   m2s_vocoder_forward    Generator.forward   models.py:113-131
 *   m2s_pipeline_forward   the no_grad section of main()   run_mri_video_inference.py:222-242
 *   m2s_cam_*              the train-mode backbone forward of compute_gradcam (model.train(): BatchNorm
 *                          on batch statistics)   scripts/mri_gradcam_formant.py:153-160,221-225
 *   m2s_bilstm_train_*     BiLSTMSumMerge forward + autograd backward   mri_acoustic_model.py:50-72,
 *                          scripts/mri_gradcam_formant.py:162-164,247-248
 *   m2s_linear_*           nn.Linear head forward + backward   mri_acoustic_model.py:103,135,
 *                          scripts/mri_gradcam_formant.py:165
 *   m2s_gap_*              GlobalAvgPool / feats.mean((2,3)) forward + backward
 *                          mri_acoustic_model.py:15-18, scripts/mri_gradcam_formant.py:162
 */
#ifndef M2S_H_
#define M2S_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define M2S_ABI_VERSION 6

enum m2s_status { M2S_OK = 0, M2S_E_ARG = 1, M2S_E_HIP = 2, M2S_E_STATE = 3, M2S_E_NODEV = 4, M2S_E_INTERNAL = 5 };
/* compute dtype of the convolution stacks.  The BiLSTM input projection, head and glue run in fp32 in every
 * dtype; the BiLSTM recurrence runs exact-f32 products in M2S_DT_F32 and for B <= 4 (lstm_small_kernel), and
 * split three-term bf16x3 products (W_hh and h_t as hi + lo bf16 pairs, fp32 cell state and gates;
 * lstm_x3_kernel) for B > 4 in the BF16, BF16X3 and FP8 engines:
 *   M2S_DT_F32    exact f32 MFMA products (v_mfma_f32_16x16x4_f32), fp32 storage
 *   M2S_DT_BF16   bf16 storage and operands, fp32 accumulation
 *   M2S_DT_BF16X3 split fp32: every activation / weight is a bf16 pair hi + lo (17 significant
 *                 bits), products are the three bf16 MFMA terms hi*hi + hi*lo + lo*hi with fp32
 *                 accumulation; meets the fp32 tolerances of the parity tests
 *   M2S_DT_FP8    configs[4]: OCP e4m3 storage and block-scaled e4m3 MFMA
 *                 (v_mfma_scale_f32_16x16x128_f8f6f4, unit E8M0 block scales, per-output-channel
 *                 fp32 weight scales applied in the epilogue) for: the IR blocks' conv_pw expand
 *                 (stride 1 and blocks.5.0), expanded maps and SE-gated conv_pwl GEMMs (every IR
 *                 block, blocks.3.0 / 5.0 included); the EdgeResidual blocks.1.1/.2 and blocks.2.1/.2
 *                 (conv_exp + conv_pwl); the C = 128 / 256 MRF convs (C = 64 / 32 on request:
 *                 M2S_F8_MRF64 / M2S_F8_MRF32, slower than the fused bf16 ResBlock1).  The stem, the
 *                 stride-2 EdgeResidual blocks.1.0 / 2.0, the blocks.3.0 expand, the IR depthwise convs
 *                 (f16 or fp32 accumulation of a 16-bit tile), the C = 32 / 64 MRF convs and the
 *                 upsamplers run the bf16 path */
enum m2s_dtype { M2S_DT_F32 = 0, M2S_DT_BF16 = 1, M2S_DT_BF16X3 = 2, M2S_DT_FP8 = 3 };
/* host tensor element types */
enum m2s_elem { M2S_ELEM_F32 = 0, M2S_ELEM_I64 = 1 };

int m2s_abi_version(void);
const char* m2s_last_error(void);
/* M2S_OK if HIP device `device` exists and is gfx950 (synchronous). */
int m2s_device_check(int device);

/* One state-dict entry, reference key name, contiguous row-major HOST memory. */
typedef struct m2s_tensor {
  const char* name;
  const void* data;
  int elem; /* m2s_elem */
  int ndim;
  int64_t shape[4];
} m2s_tensor;

/* ------------------------------------------------------------------ acoustic model ---- */
typedef struct m2s_acoustic m2s_acoustic;

/* Packs a reference-format state dict (keys of OTNLikeCNNBiLSTM.state_dict(): cnn.backbone.*,
 * rnn.lstm.*, head.*) for `device`: BatchNorm folded, grey->RGB repeat folded into conv_stem,
 * layouts converted.  Unknown keys are ignored (strict=False); a missing required key is
 * M2S_E_ARG naming the key.  Synchronous. */
int m2s_acoustic_create(const m2s_tensor* sd, int n, int n_mels, int rnn_hidden, int dtype, int device,
                        m2s_acoustic** out);
void m2s_acoustic_destroy(m2s_acoustic* m);
/* frames per CNN pass (bounds the CNN workspace); default 1920 (= m2s.config.CNN_CHUNK, the size bench.py times).
 * A pass may hold up to chunk + chunk / 16 frames where one pass fewer then covers N (no short tail pass), so
 * the workspace and the kernels' size checks see up to ~6 % more frames than `frames`. */
int m2s_acoustic_set_chunk(m2s_acoustic* m, int frames);
/* Asynchronous failure report.  The persistent BiLSTM waits at a grid barrier once per time step, and
 * the persistent CNN kernels (ir_ws, se_ws) at LDS flags between their producer and consumer waves;
 * a wait that exceeds its poll limit poisons the affected outputs with NaN and raises a host-visible flag.  This call returns M2S_E_INTERNAL (and clears the flag) when such a
 * launch has happened: call it after synchronising the stream.  The next forward / bilstm /
 * pipeline call on the engine fails the same way.  Synchronous, host only. */
int m2s_acoustic_status(m2s_acoustic* m);
/* Fault injection for tests: polls per BiLSTM barrier wait before it times out (default 2^24); 0 makes
 * the first wait time out unconditionally. */
int m2s_acoustic_set_lstm_spin_limit(m2s_acoustic* m, unsigned polls);
/* Fault injection for tests: polls per LDS flag-ring wait of the persistent CNN kernels (ir_ws producers'
 * weight-slot wait, se_ws FULL / FREE waits; default 2^20) before it times out; 0 makes every such wait time out.
 * A timeout poisons the affected outputs with NaN and is reported by m2s_acoustic_status. */
int m2s_acoustic_set_ws_spin_limit(m2s_acoustic* m, unsigned polls);
size_t m2s_acoustic_workspace_bytes(const m2s_acoustic* m, int B, int T, int H, int W);
/* frames (B,T,H,W) fp32 in [0,1] -> mel_norm (B,T,n_mels) fp32. */
int m2s_acoustic_forward(m2s_acoustic* m, const float* frames, int B, int T, int H, int W, float* mel_norm,
                         void* ws, size_t ws_bytes, void* stream);
/* frames (N,H,W) -> feats (N,208) fp32 (GAP of the last timm feature map). */
int m2s_effnet_forward(m2s_acoustic* m, const float* frames, int N, int H, int W, float* feats, void* ws,
                       size_t ws_bytes, void* stream);
/* Debug tap: feature map after `n_blocks` timm blocks (0 = after conv_stem/bn1), written as
 * (N,OH,OW,C) fp32 dense to `out`; returns OH, OW, C through the pointers. */
int m2s_effnet_probe(m2s_acoustic* m, const float* frames, int N, int H, int W, int n_blocks, float* out,
                     int* oh, int* ow, int* oc, void* ws, size_t ws_bytes, void* stream);
/* feats (B,T,208) -> y (B,T,rnn_hidden) sum-merged BiLSTM output (may be NULL) and
 * mel_norm (B,T,n_mels) head output (may be NULL). */
int m2s_bilstm_summerge(m2s_acoustic* m, const float* feats, int B, int T, float* y, float* mel_norm, void* ws,
                        size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------- mel glue ---- */
/* mel_db = x*std + mean; mel_log = ln(clamp(10^(mel_db/10), 1e-5)); x (rows,n_mels).
 * mean/std are DEVICE fp32 arrays of n_mels; either output may be NULL. */
int m2s_mel_glue(const float* mel_norm, int rows, int n_mels, const float* mean, const float* std, float* mel_db,
                 float* mel_log, void* stream);

/* ----------------------------------------------------------------------- vocoder ---- */
typedef struct m2s_hifigan_h {
  int resblock; /* 1 or 2 (h.resblock "1"/"2") */
  int num_mels;
  int upsample_initial_channel;
  int n_up;
  int upsample_rates[8];
  int upsample_kernel_sizes[8];
  int n_kernels;
  int resblock_kernel_sizes[8];
  int n_dilations[8];
  int resblock_dilation_sizes[8][8];
} m2s_hifigan_h;

typedef struct m2s_vocoder m2s_vocoder;

/* Frame preprocessing after the host decode (replaces _preprocess_frame,
 * run_mri_video_inference.py:34-54, except the cv2.resize): frames uint8 (n,h,w) grey
 * (channels = 1) or (n,h,w,3) BGR (channels = 3) -> out (n,h,w) fp32, per frame z-score then
 * min-max to [0, 1]; a constant frame gives zeros.  Device pointers, stream-ordered. */
int m2s_preprocess_frames(const uint8_t* frames, int n, int h, int w, int channels, float* out, void* stream);

/* Packs a Generator state dict (weight_g/weight_v or plain weight after remove_weight_norm).
 * Strict like load_state_dict(ckpt['generator']): a missing key is M2S_E_ARG.  Synchronous. */
int m2s_vocoder_create(const m2s_tensor* sd, int n, const m2s_hifigan_h* h, int dtype, int device, m2s_vocoder** out);
void m2s_vocoder_destroy(m2s_vocoder* v);
size_t m2s_vocoder_workspace_bytes(const m2s_vocoder* v, int B, int T);
/* mel fp32, layout 0 = (B,num_mels,T) as Generator.forward takes it, 1 = (B,T,num_mels);
 * wav (B, T*prod(upsample_rates)) fp32. */
int m2s_vocoder_forward(m2s_vocoder* v, const float* mel, int mel_layout, int B, int T, float* wav, void* ws,
                        size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------- end to end ---- */
size_t m2s_pipeline_workspace_bytes(const m2s_acoustic* m, const m2s_vocoder* v, int B, int T, int H, int W);
/* frames (B,T,H,W) -> mel_norm, mel_db, mel_log (B,T,n_mels) and wav (B,T*hop).  mel_* may be NULL. */
int m2s_pipeline_forward(m2s_acoustic* m, m2s_vocoder* v, const float* frames, int B, int T, int H, int W,
                         const float* mean, const float* std, float* mel_norm, float* mel_db, float* mel_log,
                         float* wav, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------- Grad-CAM (autograd) path ---- */
/* compute_gradcam (scripts/mri_gradcam_formant.py:203-279) runs the model in train() and back-
 * propagates a mel-band power to the last feature map.  These entry points are that path, exact
 * fp32; every pointer is a device pointer on the current HIP device unless stated otherwise. */
typedef struct m2s_cam m2s_cam;
/* Packs the backbone part of an acoustic state dict (cnn.backbone.*) with unfolded BatchNorms:
 * raw conv weights, BN gamma / beta.  Synchronous. */
int m2s_cam_create(const m2s_tensor* sd, int n, int device, m2s_cam** out);
void m2s_cam_destroy(m2s_cam* c);
/* BatchNorm layers in state-dict order (conv_stem's bn1, then bn1 / bn2 / bn3 of every block) and
 * their channel counts: m2s_cam_backbone writes [mean C | biased var C] per layer, in that order. */
int m2s_cam_bn_layers(const m2s_cam* c);
int m2s_cam_bn_channels(const m2s_cam* c, int layer);
size_t m2s_cam_workspace_bytes(const m2s_cam* c, int N, int H, int W);
/* frames (N,H,W) fp32 -> the five timm feature maps with train-mode BatchNorm (statistics of the N
 * frames), taps[i] (N,C_i,OH_i,OW_i) fp32 (C = 16, 32, 56, 120, 208 at strides 2..32; a NULL entry
 * is skipped), and every BN layer's batch statistics into bn_stats. */
int m2s_cam_backbone(m2s_cam* c, const float* frames, int N, int H, int W, float* const* taps, float* bn_stats,
                     void* ws, size_t ws_bytes, void* stream);
/* nn.LSTM(C, H, bidirectional, batch_first) + sum merge with saved activations.  w[8] = w_ih, w_hh,
 * b_ih, b_hh of the forward direction, then of the reverse one (nn.LSTM layouts).  x (B,T,C) ->
 * y (B,T,H); gates (2,B,T,4H) post-activation i,f,g,o, cells / hid (2,B,T,H) kept for the backward. */
size_t m2s_bilstm_train_workspace_bytes(int B, int T, int C, int H);
int m2s_bilstm_train_forward(const float* x, int B, int T, int C, int H, const float* const* w, float* y,
                             float* gates, float* cells, float* hid, void* ws, size_t ws_bytes, void* stream);
/* Backward through time: dy (B,T,H) -> dx (B,T,C) and grads[6] = d w_ih, d w_hh, d bias (= d b_ih =
 * d b_hh) of the forward direction, then of the reverse one; any output may be NULL. */
int m2s_bilstm_train_backward(const float* x, const float* dy, int B, int T, int C, int H, const float* const* w,
                              const float* gates, const float* cells, const float* hid, float* dx, float* const* grads,
                              void* ws, size_t ws_bytes, void* stream);
/* y (rows,out) = x (rows,in) w^T + b (b may be NULL); backward dx = dy w, dw = dy^T x, db = sum dy. */
int m2s_linear_forward(const float* x, int rows, int in, int out, const float* w, const float* b, float* y,
                       void* stream);
int m2s_linear_backward(const float* dy, const float* x, int rows, int in, int out, const float* w, float* dx,
                        float* dw, float* db, void* stream);
/* mean over the last P elements of nc rows (NCHW maps: nc = N*C, P = H*W) and its backward. */
int m2s_gap_forward(const float* x, int64_t nc, int p, float* y, void* stream);
int m2s_gap_backward(const float* dy, int64_t nc, int p, float* dx, void* stream);

/* -------------------------------------------------------------------- profiling ---- */
/* While enabled, every kernel launch is bracketed by HIP events on its own stream. */
typedef struct m2s_prof_stat {
  char name[96];     /* kernel symbol family, e.g. "conv_igemm<bf16,conv2d,2x4>" */
  int64_t launches;
  double ms;         /* summed event time */
  double flops;      /* summed algorithmic FLOPs */
  double bytes;      /* summed algorithmic HBM bytes (compulsory in + out + weights) */
} m2s_prof_stat;
int m2s_prof_enable(int on);
/* Synchronises on the recorded events, writes up to `max` stats, clears the record. */
int m2s_prof_collect(m2s_prof_stat* out, int max, int* n_out);
/* One recorded launch, in launch order: its kernel name, the stage of the path it belongs to
 * ("cnn", "bilstm", "head", "glue", "voc_pre", "ups_c<C>", "mrf_c<C>", "voc_post"; bench.py's
 * roofline.stages), event time, algorithmic FLOPs and bytes (compulsory in + out + weights of the
 * operation the kernel implements), and spill_bytes: an intermediate map the kernel writes only for a
 * later kernel of the same operation to read back (ir_ws: the IR block's expanded depthwise map, which
 * the SE-gated conv_pwl reads; ABI 6), counted once, not part of `bytes`. */
typedef struct m2s_prof_launch {
  char name[96];
  char stage[24];
  double ms;
  double flops;
  double bytes;
  double spill_bytes;
} m2s_prof_launch;
/* Synchronises on the recorded events, writes up to `max` launches in launch order (*n_out = all of
 * them), clears the record.  out == NULL: *n_out = the number recorded, the record stays. */
int m2s_prof_launches(m2s_prof_launch* out, int max, int* n_out);

#ifdef __cplusplus
}
#endif

#endif /* M2S_H_ */
