// PyTorch-ROCm custom ops over the libm2s C ABI (include/m2s.h): torch.ops.m2s.*.
//
// The ops take the packed model as an opaque int handle (an m2s_acoustic* / m2s_vocoder* created
// through the C ABI and owned by the Python engine object), allocate their outputs and workspace
// through the torch caching allocator on the CURRENT HIP stream (so concurrent streams get separate,
// stream-ordered workspaces) and launch there.  Fake (meta) kernels for torch.compile / FakeTensor
// tracing live in m2s/ops.py.  Errors: TORCH_CHECK -> RuntimeError with m2s_last_error().
//
// Reference interfaces (mri2speech_code/mri_acoustic_model.py, models.py, scripts/run_mri_video_inference.py):
//   acoustic_forward   OTNLikeCNNBiLSTM.forward (eval)                 mri_acoustic_model.py:116-136
//   effnet_forward     EffNetV2B2Backbone.forward + GlobalAvgPool      mri_acoustic_model.py:15-18,39-48
//   effnet_features    the timm feature maps (Grad-CAM tap)           mri_gradcam_formant.py:155-158
//   bilstm_summerge    BiLSTMSumMerge.forward + head Linear            mri_acoustic_model.py:67-72,135
//   mel_glue           denormalize_mel + dB -> ln-power                run_mri_video_inference.py:160-163,227-233
//   hifigan_forward    Generator.forward                               models.py:113-131
//   pipeline_forward   the no_grad section of main()                   run_mri_video_inference.py:222-242
//   preprocess_frames  _preprocess_frame after the host decode         run_mri_video_inference.py:34-54
//   cam_backbone       backbone(x) in train() (batch-statistics BN)    mri_gradcam_formant.py:153-160,221-225
//   bilstm_train_*     model.rnn(seq) forward / autograd backward      mri_gradcam_formant.py:162-164,247-248
//   linear_*           model.head(...) forward / autograd backward     mri_gradcam_formant.py:165
//   gap_*              feats.mean(dim=(2,3)) forward / backward        mri_gradcam_formant.py:162
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <tuple>
#include <vector>

#include "../../include/m2s.h"

namespace {

void ok(int rc, const char* what) { TORCH_CHECK(rc == M2S_OK, "libm2s ", what, " failed (", rc, "): ", m2s_last_error()); }

// PyTorch-ROCm exposes HIP devices as DeviceType::CUDA ("masquerading"); torch.cuda.current_stream()
// is this stream
void* S() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using Guard = c10::hip::HIPGuardMasqueradingAsCUDA;

at::Tensor f32_on_device(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP (cuda) tensor; libm2s has no CPU path");
  return t.to(at::kFloat).contiguous();
}

at::Tensor workspace(size_t bytes, const at::Tensor& like) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 256)}, like.options().dtype(at::kByte));
}

m2s_acoustic* A(int64_t h) {
  TORCH_CHECK(h != 0, "null acoustic handle");
  return reinterpret_cast<m2s_acoustic*>(h);
}
m2s_vocoder* V(int64_t h) {
  TORCH_CHECK(h != 0, "null vocoder handle");
  return reinterpret_cast<m2s_vocoder*>(h);
}

// frames (B,T,H,W) -> mel_norm (B,T,n_mels)
at::Tensor acoustic_forward(int64_t h, const at::Tensor& frames, int64_t n_mels) {
  TORCH_CHECK(frames.dim() == 4, "acoustic_forward: frames must be (B,T,H,W)");
  const Guard g(frames.device());
  const at::Tensor x = f32_on_device(frames, "frames");
  const int B = x.size(0), T = x.size(1), H = x.size(2), W = x.size(3);
  at::Tensor out = at::empty({B, T, n_mels}, x.options());
  if (B * T == 0) return out;
  at::Tensor ws = workspace(m2s_acoustic_workspace_bytes(A(h), B, T, H, W), x);
  ok(m2s_acoustic_forward(A(h), x.data_ptr<float>(), B, T, H, W, out.data_ptr<float>(), ws.data_ptr(), ws.numel(), S()),
     "acoustic_forward");
  return out;
}

// frames (N,H,W) -> feats (N,208)
at::Tensor effnet_forward(int64_t h, const at::Tensor& frames) {
  TORCH_CHECK(frames.dim() == 3, "effnet_forward: frames must be (N,H,W)");
  const Guard g(frames.device());
  const at::Tensor x = f32_on_device(frames, "frames");
  const int N = x.size(0), H = x.size(1), W = x.size(2);
  at::Tensor out = at::empty({N, 208}, x.options());
  if (N == 0) return out;
  at::Tensor ws = workspace(m2s_acoustic_workspace_bytes(A(h), N, 1, H, W), x);
  ok(m2s_effnet_forward(A(h), x.data_ptr<float>(), N, H, W, out.data_ptr<float>(), ws.data_ptr(), ws.numel(), S()),
     "effnet_forward");
  return out;
}

// frames (N,H,W) -> feature map after `n_blocks` timm blocks (0 = stem), (N,C,OH,OW)
at::Tensor effnet_features(int64_t h, const at::Tensor& frames, int64_t n_blocks) {
  TORCH_CHECK(frames.dim() == 3, "effnet_features: frames must be (N,H,W)");
  const Guard g(frames.device());
  const at::Tensor x = f32_on_device(frames, "frames");
  const int N = x.size(0), H = x.size(1), W = x.size(2);
  // the stem output (32 channels at H/2 x W/2) is the largest map of the network
  at::Tensor buf = at::empty({(int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * 32}, x.options());
  at::Tensor ws = workspace(m2s_acoustic_workspace_bytes(A(h), N, 1, H, W), x);
  int oh = 0, ow = 0, oc = 0;
  ok(m2s_effnet_probe(A(h), x.data_ptr<float>(), N, H, W, (int)n_blocks, buf.data_ptr<float>(), &oh, &ow, &oc,
                      ws.data_ptr(), ws.numel(), S()),
     "effnet_features");
  return buf.narrow(0, 0, (int64_t)N * oh * ow * oc).view({N, oh, ow, oc}).permute({0, 3, 1, 2}).contiguous();
}

// feats (B,T,208) -> (y (B,T,hidden) sum-merged BiLSTM output, mel_norm (B,T,n_mels) head output)
std::tuple<at::Tensor, at::Tensor> bilstm_summerge(int64_t h, const at::Tensor& feats, int64_t hidden, int64_t n_mels) {
  TORCH_CHECK(feats.dim() == 3 && feats.size(2) == 208, "bilstm_summerge: feats must be (B,T,208)");
  const Guard g(feats.device());
  const at::Tensor x = f32_on_device(feats, "feats");
  const int B = x.size(0), T = x.size(1);
  at::Tensor y = at::empty({B, T, hidden}, x.options());
  at::Tensor m = at::empty({B, T, n_mels}, x.options());
  if (B * T == 0) return {y, m};
  at::Tensor ws = workspace(m2s_acoustic_workspace_bytes(A(h), B, T, 64, 64), x);
  ok(m2s_bilstm_summerge(A(h), x.data_ptr<float>(), B, T, y.data_ptr<float>(), m.data_ptr<float>(), ws.data_ptr(),
                         ws.numel(), S()),
     "bilstm_summerge");
  return {y, m};
}

// mel_norm (..., n_mels), mean/std (n_mels) -> (mel_db, mel_log), same shape
std::tuple<at::Tensor, at::Tensor> mel_glue(const at::Tensor& mel_norm, const at::Tensor& mean, const at::Tensor& std_) {
  const Guard g(mel_norm.device());
  const at::Tensor x = f32_on_device(mel_norm, "mel_norm");
  const int nm = x.size(-1);
  TORCH_CHECK(mean.numel() == nm && std_.numel() == nm, "mel_glue: mean/std must have n_mels entries");
  const at::Tensor mu = mean.to(x.device(), at::kFloat).contiguous(), sd = std_.to(x.device(), at::kFloat).contiguous();
  at::Tensor db = at::empty_like(x), ln = at::empty_like(x);
  ok(m2s_mel_glue(x.data_ptr<float>(), (int)(x.numel() / nm), nm, mu.data_ptr<float>(), sd.data_ptr<float>(),
                  db.data_ptr<float>(), ln.data_ptr<float>(), S()),
     "mel_glue");
  return {db, ln};
}

// mel (B,num_mels,T) [layout 0] or (B,T,num_mels) [layout 1] -> wav (B,1,T*hop)
at::Tensor hifigan_forward(int64_t v, const at::Tensor& mel, int64_t layout, int64_t hop) {
  TORCH_CHECK(mel.dim() == 3 && (layout == 0 || layout == 1), "hifigan_forward: mel must be 3-D, layout 0 or 1");
  const Guard g(mel.device());
  const at::Tensor x = f32_on_device(mel, "mel");
  const int B = x.size(0), T = layout == 0 ? x.size(2) : x.size(1);
  at::Tensor wav = at::empty({B, 1, (int64_t)T * hop}, x.options());
  if (B * T == 0) return wav;
  at::Tensor ws = workspace(m2s_vocoder_workspace_bytes(V(v), B, T), x);
  ok(m2s_vocoder_forward(V(v), x.data_ptr<float>(), (int)layout, B, T, wav.data_ptr<float>(), ws.data_ptr(), ws.numel(),
                         S()),
     "hifigan_forward");
  return wav;
}

// frames (B,T,H,W) -> (mel_norm, mel_db, mel_log (B,T,n_mels), wav (B,T*hop))
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> pipeline_forward(int64_t h, int64_t v, const at::Tensor& frames,
                                                                            const at::Tensor& mean, const at::Tensor& std_,
                                                                            int64_t n_mels, int64_t hop) {
  TORCH_CHECK(frames.dim() == 4, "pipeline_forward: frames must be (B,T,H,W)");
  const Guard g(frames.device());
  const at::Tensor x = f32_on_device(frames, "frames");
  const int B = x.size(0), T = x.size(1), H = x.size(2), W = x.size(3);
  const at::Tensor mu = mean.to(x.device(), at::kFloat).contiguous(), sd = std_.to(x.device(), at::kFloat).contiguous();
  TORCH_CHECK(mu.numel() == n_mels && sd.numel() == n_mels, "pipeline_forward: mean/std must have n_mels entries");
  at::Tensor mn = at::empty({B, T, n_mels}, x.options()), db = at::empty_like(mn), ln = at::empty_like(mn);
  at::Tensor wav = at::empty({B, (int64_t)T * hop}, x.options());
  if (B * T == 0) return {mn, db, ln, wav};
  at::Tensor ws = workspace(m2s_pipeline_workspace_bytes(A(h), V(v), B, T, H, W), x);
  ok(m2s_pipeline_forward(A(h), V(v), x.data_ptr<float>(), B, T, H, W, mu.data_ptr<float>(), sd.data_ptr<float>(),
                          mn.data_ptr<float>(), db.data_ptr<float>(), ln.data_ptr<float>(), wav.data_ptr<float>(),
                          ws.data_ptr(), ws.numel(), S()),
     "pipeline_forward");
  return {mn, db, ln, wav};
}

// decoded frames uint8 (T,H,W) grey or (T,H,W,3) BGR -> (T,H,W) fp32 in [0,1]
at::Tensor preprocess_frames(const at::Tensor& frames) {
  TORCH_CHECK(frames.is_cuda() && frames.scalar_type() == at::kByte, "preprocess_frames: uint8 HIP tensor expected");
  TORCH_CHECK(frames.dim() == 3 || (frames.dim() == 4 && frames.size(3) == 3), "preprocess_frames: (T,H,W[,3])");
  const Guard g(frames.device());
  const at::Tensor x = frames.contiguous();
  const int n = x.size(0), hh = x.size(1), ww = x.size(2), ch = x.dim() == 4 ? 3 : 1;
  at::Tensor out = at::empty({n, hh, ww}, x.options().dtype(at::kFloat));
  ok(m2s_preprocess_frames(x.data_ptr<uint8_t>(), n, hh, ww, ch, out.data_ptr<float>(), S()), "preprocess_frames");
  return out;
}

m2s_cam* Cm(int64_t h) {
  TORCH_CHECK(h != 0, "null cam handle");
  return reinterpret_cast<m2s_cam*>(h);
}

std::vector<const float*> f32_ptrs(const std::vector<at::Tensor>& ts, size_t n, const char* what) {
  TORCH_CHECK(ts.size() == n, what, ": expected ", n, " tensors");
  std::vector<const float*> p;
  for (const auto& t : ts) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), what, ": contiguous fp32 HIP tensors");
    p.push_back(t.data_ptr<float>());
  }
  return p;
}

// frames (N,H,W) -> five train-mode feature maps (N,C,OH,OW) + BN batch statistics (flat)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> cam_backbone(int64_t h,
                                                                                                const at::Tensor& frames) {
  TORCH_CHECK(frames.dim() == 3, "cam_backbone: frames must be (N,H,W)");
  const Guard g(frames.device());
  const at::Tensor x = f32_on_device(frames, "frames");
  const int N = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(N > 0, "cam_backbone: empty batch");
  static const int ch[5] = {16, 32, 56, 120, 208}, red[5] = {2, 4, 8, 16, 32};
  std::vector<at::Tensor> taps;
  std::vector<float*> tp;
  for (int i = 0; i < 5; ++i) {
    int oh = H, ow = W;
    for (int r = 1; r < red[i]; r *= 2) oh = (oh + 1) / 2, ow = (ow + 1) / 2;
    taps.push_back(at::empty({N, ch[i], oh, ow}, x.options()));
    tp.push_back(taps.back().data_ptr<float>());
  }
  int64_t nst = 0;
  for (int l = 0; l < m2s_cam_bn_layers(Cm(h)); ++l) nst += 2 * m2s_cam_bn_channels(Cm(h), l);
  at::Tensor stats = at::empty({nst}, x.options());
  at::Tensor ws = workspace(m2s_cam_workspace_bytes(Cm(h), N, H, W), x);
  ok(m2s_cam_backbone(Cm(h), x.data_ptr<float>(), N, H, W, tp.data(), stats.data_ptr<float>(), ws.data_ptr(),
                      ws.numel(), S()),
     "cam_backbone");
  return {taps[0], taps[1], taps[2], taps[3], taps[4], stats};
}

// x (B,T,C), w = [w_ih, w_hh, b_ih, b_hh] x (fwd, reverse) -> y (B,T,H), gates (2,B,T,4H), cells, hid (2,B,T,H)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bilstm_train_forward(const at::Tensor& x_,
                                                                                const std::vector<at::Tensor>& w) {
  TORCH_CHECK(x_.dim() == 3, "bilstm_train_forward: x must be (B,T,C)");
  const Guard g(x_.device());
  const at::Tensor x = f32_on_device(x_, "x");
  std::vector<at::Tensor> wc;
  for (const auto& t : w) wc.push_back(f32_on_device(t, "lstm weight"));
  const auto p = f32_ptrs(wc, 8, "bilstm_train_forward");
  const int B = x.size(0), T = x.size(1), C = x.size(2), Hd = wc[1].size(1);
  TORCH_CHECK(wc[0].size(0) == 4 * Hd && wc[0].size(1) == C && wc[1].size(0) == 4 * Hd, "bilstm_train_forward: weight shapes");
  at::Tensor y = at::empty({B, T, Hd}, x.options());
  at::Tensor gates = at::empty({2, B, T, 4 * Hd}, x.options());
  at::Tensor cells = at::empty({2, B, T, Hd}, x.options()), hid = at::empty({2, B, T, Hd}, x.options());
  if (B * T == 0) return {y, gates, cells, hid};
  at::Tensor ws = workspace(m2s_bilstm_train_workspace_bytes(B, T, C, Hd), x);
  ok(m2s_bilstm_train_forward(x.data_ptr<float>(), B, T, C, Hd, p.data(), y.data_ptr<float>(), gates.data_ptr<float>(),
                              cells.data_ptr<float>(), hid.data_ptr<float>(), ws.data_ptr(), ws.numel(), S()),
     "bilstm_train_forward");
  return {y, gates, cells, hid};
}

// -> dx (B,T,C), [d w_ih, d w_hh, d bias] x (fwd, reverse)
std::tuple<at::Tensor, std::vector<at::Tensor>> bilstm_train_backward(const at::Tensor& dy_, const at::Tensor& x_,
                                                                      const std::vector<at::Tensor>& w,
                                                                      const at::Tensor& gates, const at::Tensor& cells,
                                                                      const at::Tensor& hid) {
  const Guard g(x_.device());
  const at::Tensor x = f32_on_device(x_, "x"), dy = f32_on_device(dy_, "dy");
  std::vector<at::Tensor> wc;
  for (const auto& t : w) wc.push_back(f32_on_device(t, "lstm weight"));
  const auto p = f32_ptrs(wc, 8, "bilstm_train_backward");
  const int B = x.size(0), T = x.size(1), C = x.size(2), Hd = wc[1].size(1);
  TORCH_CHECK(dy.sizes() == at::IntArrayRef({B, T, Hd}), "bilstm_train_backward: dy shape");
  const at::Tensor gs = f32_on_device(gates, "gates"), cs = f32_on_device(cells, "cells"), hs = f32_on_device(hid, "hid");
  at::Tensor dx = at::zeros_like(x);
  std::vector<at::Tensor> grads;
  for (int d = 0; d < 2; ++d) {
    grads.push_back(at::zeros_like(wc[4 * d]));
    grads.push_back(at::zeros_like(wc[4 * d + 1]));
    grads.push_back(at::zeros_like(wc[4 * d + 2]));
  }
  if (B * T == 0) return {dx, grads};
  std::vector<float*> gp;
  for (auto& t : grads) gp.push_back(t.data_ptr<float>());
  at::Tensor ws = workspace(m2s_bilstm_train_workspace_bytes(B, T, C, Hd), x);
  ok(m2s_bilstm_train_backward(x.data_ptr<float>(), dy.data_ptr<float>(), B, T, C, Hd, p.data(), gs.data_ptr<float>(),
                               cs.data_ptr<float>(), hs.data_ptr<float>(), dx.data_ptr<float>(), gp.data(),
                               ws.data_ptr(), ws.numel(), S()),
     "bilstm_train_backward");
  return {dx, grads};
}

// x (..., in), w (out, in), b (out) -> y (..., out)
at::Tensor linear_forward(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& b_) {
  const Guard g(x_.device());
  const at::Tensor x = f32_on_device(x_, "x"), w = f32_on_device(w_, "weight");
  TORCH_CHECK(w.dim() == 2 && x.size(-1) == w.size(1), "linear_forward: shapes");
  at::Tensor b;
  if (b_.has_value()) b = f32_on_device(*b_, "bias");
  const int in = w.size(1), out = w.size(0), rows = x.numel() / in;
  auto shape = x.sizes().vec();
  shape.back() = out;
  at::Tensor y = at::empty(shape, x.options());
  if (rows == 0) return y;
  ok(m2s_linear_forward(x.data_ptr<float>(), rows, in, out, w.data_ptr<float>(), b.defined() ? b.data_ptr<float>() : nullptr,
                        y.data_ptr<float>(), S()),
     "linear_forward");
  return y;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> linear_backward(const at::Tensor& dy_, const at::Tensor& x_,
                                                               const at::Tensor& w_) {
  const Guard g(x_.device());
  const at::Tensor x = f32_on_device(x_, "x"), w = f32_on_device(w_, "weight"), dy = f32_on_device(dy_, "dy");
  const int in = w.size(1), out = w.size(0), rows = x.numel() / in;
  TORCH_CHECK(dy.numel() == (int64_t)rows * out, "linear_backward: dy shape");
  at::Tensor dx = at::empty_like(x), dw = at::zeros_like(w), db = at::zeros({out}, w.options());
  if (rows == 0) return {dx, dw, db};
  ok(m2s_linear_backward(dy.data_ptr<float>(), x.data_ptr<float>(), rows, in, out, w.data_ptr<float>(),
                         dx.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(), S()),
     "linear_backward");
  return {dx, dw, db};
}

// (N,C,H,W) -> (N,C) mean over H,W ; backward (N,C) -> (N,C,H,W)
at::Tensor gap_forward(const at::Tensor& x_) {
  TORCH_CHECK(x_.dim() == 4, "gap_forward: (N,C,H,W)");
  const Guard g(x_.device());
  const at::Tensor x = f32_on_device(x_, "x");
  at::Tensor y = at::empty({x.size(0), x.size(1)}, x.options());
  ok(m2s_gap_forward(x.data_ptr<float>(), x.size(0) * x.size(1), (int)(x.size(2) * x.size(3)), y.data_ptr<float>(), S()),
     "gap_forward");
  return y;
}

at::Tensor gap_backward(const at::Tensor& dy_, int64_t h, int64_t w) {
  TORCH_CHECK(dy_.dim() == 2, "gap_backward: dy (N,C)");
  const Guard g(dy_.device());
  const at::Tensor dy = f32_on_device(dy_, "dy");
  at::Tensor dx = at::empty({dy.size(0), dy.size(1), h, w}, dy.options());
  ok(m2s_gap_backward(dy.data_ptr<float>(), dy.numel(), (int)(h * w), dx.data_ptr<float>(), S()), "gap_backward");
  return dx;
}

}  // namespace

TORCH_LIBRARY(m2s, m) {
  m.def("acoustic_forward(int handle, Tensor frames, int n_mels) -> Tensor");
  m.def("effnet_forward(int handle, Tensor frames) -> Tensor");
  m.def("effnet_features(int handle, Tensor frames, int n_blocks) -> Tensor");
  m.def("bilstm_summerge(int handle, Tensor feats, int hidden, int n_mels) -> (Tensor, Tensor)");
  m.def("mel_glue(Tensor mel_norm, Tensor mean, Tensor std) -> (Tensor, Tensor)");
  m.def("hifigan_forward(int handle, Tensor mel, int layout, int hop) -> Tensor");
  m.def("pipeline_forward(int acoustic, int vocoder, Tensor frames, Tensor mean, Tensor std, int n_mels, int hop)"
        " -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("preprocess_frames(Tensor frames) -> Tensor");
  m.def("cam_backbone(int handle, Tensor frames) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("bilstm_train_forward(Tensor x, Tensor[] weights) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("bilstm_train_backward(Tensor dy, Tensor x, Tensor[] weights, Tensor gates, Tensor cells, Tensor hid)"
        " -> (Tensor, Tensor[])");
  m.def("linear_forward(Tensor x, Tensor weight, Tensor? bias) -> Tensor");
  m.def("linear_backward(Tensor dy, Tensor x, Tensor weight) -> (Tensor, Tensor, Tensor)");
  m.def("gap_forward(Tensor x) -> Tensor");
  m.def("gap_backward(Tensor dy, int h, int w) -> Tensor");
}

TORCH_LIBRARY_IMPL(m2s, CUDA, m) {  // CUDA = the HIP device key of PyTorch-ROCm
  m.impl("acoustic_forward", &acoustic_forward);
  m.impl("effnet_forward", &effnet_forward);
  m.impl("effnet_features", &effnet_features);
  m.impl("bilstm_summerge", &bilstm_summerge);
  m.impl("mel_glue", &mel_glue);
  m.impl("hifigan_forward", &hifigan_forward);
  m.impl("pipeline_forward", &pipeline_forward);
  m.impl("preprocess_frames", &preprocess_frames);
  m.impl("cam_backbone", &cam_backbone);
  m.impl("bilstm_train_forward", &bilstm_train_forward);
  m.impl("bilstm_train_backward", &bilstm_train_backward);
  m.impl("linear_forward", &linear_forward);
  m.impl("linear_backward", &linear_backward);
  m.impl("gap_forward", &gap_forward);
  m.impl("gap_backward", &gap_backward);
}
