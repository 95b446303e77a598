// extern "C" surface of libm2s (include/m2s.h): argument checks, device guards, and the
// exception -> status-code boundary.  No CPU fallback exists behind any of these entry points.
#include <cstring>
#include <string>

#include "../../include/m2s.h"
#include "cam.hpp"
#include "model.hpp"

struct m2s_acoustic {
  m2s::Acoustic impl;
};
struct m2s_vocoder {
  m2s::Vocoder impl;
};
struct m2s_cam {
  m2s::CamBackbone impl;
};

extern "C" int m2s_prof_enable_impl(int on);
extern "C" int m2s_prof_collect_impl(m2s_prof_stat* out, int max, int* n_out);
extern "C" int m2s_prof_launches_impl(m2s_prof_launch* out, int max, int* n_out);

namespace {

thread_local std::string g_err;

class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    M2S_HIP(hipGetDevice(&prev_));
    if (prev_ != dev) M2S_HIP(hipSetDevice(dev));
    dev_ = dev;
  }
  ~DeviceGuard() {
    if (prev_ != dev_) (void)hipSetDevice(prev_);
  }

 private:
  int prev_ = 0, dev_ = 0;
};

template <class F>
int guarded(F f) {
  try {
    f();
    return M2S_OK;
  } catch (const m2s::Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_err = e.what();
    return M2S_E_INTERNAL;
  } catch (...) {
    g_err = "unknown error";
    return M2S_E_INTERNAL;
  }
}

void check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw m2s::Error(M2S_E_NODEV, "no HIP device visible");
  if (device < 0 || device >= n) throw m2s::Error(M2S_E_NODEV, "device index out of range");
  hipDeviceProp_t p;
  M2S_HIP(hipGetDeviceProperties(&p, device));
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    throw m2s::Error(M2S_E_NODEV, std::string("libm2s is built for gfx950, device is ") + p.gcnArchName);
}

hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

// an earlier launch of this engine hit a BiLSTM barrier timeout (its outputs hold NaN): fail loudly
void no_pending_error(m2s::Acoustic& a) {
  const unsigned e = a.take_async_error();
  if (e == m2s::M2S_ASYNC_WS)
    throw m2s::Error(M2S_E_INTERNAL, "a previous CNN launch timed out at an LDS flag-ring wait (ir_ws / se_ws "
                                     "producer-consumer hand-off); the affected outputs were poisoned with NaN");
  if (e != 0)
    throw m2s::Error(M2S_E_INTERNAL, "a previous BiLSTM launch timed out at its grid barrier (workgroups not "
                                     "co-resident?); its outputs were poisoned with NaN");
}

}  // namespace

extern "C" {

int m2s_abi_version(void) { return M2S_ABI_VERSION; }
const char* m2s_last_error(void) { return g_err.c_str(); }

int m2s_device_check(int device) {
  return guarded([&] { check_device(device); });
}

int m2s_acoustic_create(const m2s_tensor* sd, int n, int n_mels, int rnn_hidden, int dtype, int device,
                        m2s_acoustic** out) {
  return guarded([&] {
    M2S_CHECK(out && (sd || n == 0), "null argument");
    check_device(device);
    DeviceGuard g(device);
    *out = new m2s_acoustic{m2s::Acoustic(m2s::make_state_dict(sd, n), n_mels, rnn_hidden, dtype, device)};
  });
}

void m2s_acoustic_destroy(m2s_acoustic* m) { delete m; }

int m2s_acoustic_set_chunk(m2s_acoustic* m, int frames) {
  return guarded([&] {
    M2S_CHECK(m && frames > 0, "bad argument");
    m->impl.chunk = frames;
  });
}

int m2s_acoustic_status(m2s_acoustic* m) {
  return guarded([&] {
    M2S_CHECK(m, "null argument");
    no_pending_error(m->impl);
  });
}

int m2s_acoustic_set_lstm_spin_limit(m2s_acoustic* m, unsigned polls) {
  return guarded([&] {
    M2S_CHECK(m, "bad argument");
    m->impl.lstm_spin_max_ = polls;
  });
}

int m2s_acoustic_set_ws_spin_limit(m2s_acoustic* m, unsigned polls) {
  return guarded([&] {
    M2S_CHECK(m, "bad argument");
    m->impl.ws_spin_max_ = polls;
  });
}

size_t m2s_acoustic_workspace_bytes(const m2s_acoustic* m, int B, int T, int H, int W) {
  size_t r = 0;
  guarded([&] { r = m->impl.workspace_bytes(B, T, H, W); });
  return r;
}

int m2s_acoustic_forward(m2s_acoustic* m, const float* frames, int B, int T, int H, int W, float* mel_norm, void* ws,
                         size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(m && frames && mel_norm && ws, "null argument");
    no_pending_error(m->impl);
    DeviceGuard g(m->impl.device());
    m->impl.forward(frames, B, T, H, W, mel_norm, ws, ws_bytes, S(stream));
  });
}

int m2s_effnet_forward(m2s_acoustic* m, const float* frames, int N, int H, int W, float* feats, void* ws,
                       size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(m && frames && feats && ws, "null argument");
    DeviceGuard g(m->impl.device());
    m2s::Workspace w(ws, ws_bytes);
    m->impl.effnet(frames, N, H, W, feats, -1, nullptr, nullptr, w, S(stream));
  });
}

int m2s_effnet_probe(m2s_acoustic* m, const float* frames, int N, int H, int W, int n_blocks, float* out, int* oh,
                     int* ow, int* oc, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(m && frames && ws, "null argument");
    M2S_CHECK(n_blocks >= 0 && n_blocks <= 28, "n_blocks out of range");
    DeviceGuard g(m->impl.device());
    m2s::Workspace w(ws, ws_bytes);
    int dims[3] = {0, 0, 0};
    m->impl.effnet(frames, N, H, W, nullptr, n_blocks, out, dims, w, S(stream));
    if (oh) *oh = dims[0];
    if (ow) *ow = dims[1];
    if (oc) *oc = dims[2];
  });
}

int m2s_bilstm_summerge(m2s_acoustic* m, const float* feats, int B, int T, float* y, float* mel_norm, void* ws,
                        size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(m && feats && ws, "null argument");
    no_pending_error(m->impl);
    DeviceGuard g(m->impl.device());
    m2s::Workspace w(ws, ws_bytes);
    m->impl.bilstm(feats, B, T, y, mel_norm, w, S(stream));
  });
}

int m2s_mel_glue(const float* mel_norm, int rows, int n_mels, const float* mean, const float* std, float* mel_db,
                 float* mel_log, void* stream) {
  return guarded([&] {
    M2S_CHECK(mel_norm && mean && std && rows >= 0 && n_mels > 0, "bad argument");
    if (rows == 0) return;
    m2s::launch_mel_glue<float>(mel_norm, rows, n_mels, mean, std, mel_db, mel_log, nullptr, n_mels, S(stream));
  });
}

int m2s_preprocess_frames(const uint8_t* frames, int n, int h, int w, int channels, float* out, void* stream) {
  return guarded([&] {
    M2S_CHECK(frames && out && n >= 0 && h > 0 && w > 0 && (channels == 1 || channels == 3), "bad argument");
    m2s::launch_preprocess(frames, n, h, w, channels, out, S(stream));
  });
}

int m2s_vocoder_create(const m2s_tensor* sd, int n, const m2s_hifigan_h* h, int dtype, int device, m2s_vocoder** out) {
  return guarded([&] {
    M2S_CHECK(out && h && (sd || n == 0), "null argument");
    check_device(device);
    DeviceGuard g(device);
    *out = new m2s_vocoder{m2s::Vocoder(m2s::make_state_dict(sd, n), *h, dtype, device)};
  });
}

void m2s_vocoder_destroy(m2s_vocoder* v) { delete v; }

size_t m2s_vocoder_workspace_bytes(const m2s_vocoder* v, int B, int T) {
  size_t r = 0;
  guarded([&] { r = v->impl.workspace_bytes(B, T); });
  return r;
}

int m2s_vocoder_forward(m2s_vocoder* v, const float* mel, int mel_layout, int B, int T, float* wav, void* ws,
                        size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(v && mel && wav && ws, "null argument");
    M2S_CHECK(mel_layout == 0 || mel_layout == 1, "mel_layout must be 0 or 1");
    DeviceGuard g(v->impl.device());
    m2s::Workspace w(ws, ws_bytes);
    v->impl.forward(mel, mel_layout, B, T, wav, w, S(stream));
  });
}

size_t m2s_pipeline_workspace_bytes(const m2s_acoustic* m, const m2s_vocoder* v, int B, int T, int H, int W) {
  size_t r = 0;
  guarded([&] {
    const size_t rows = (size_t)B * T;
    m2s::Workspace w(nullptr, 0);
    w.take<float>(rows * m->impl.n_mels());
    w.take<char>(rows * m2s::chan_stride(m->impl.n_mels()) * 4);
    w.take<char>(std::max(m->impl.workspace_bytes(B, T, H, W), v->impl.workspace_bytes(B, T)));
    r = w.used();
  });
  return r;
}

int m2s_pipeline_forward(m2s_acoustic* m, m2s_vocoder* v, const float* frames, int B, int T, int H, int W,
                         const float* mean, const float* std, float* mel_norm, float* mel_db, float* mel_log,
                         float* wav, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(m && v && frames && mean && std && wav && ws, "null argument");
    M2S_CHECK(m->impl.device() == v->impl.device(), "acoustic model and vocoder on different devices");
    M2S_CHECK(m->impl.n_mels() == v->impl.num_mels(), "n_mels mismatch between acoustic model and vocoder");
    no_pending_error(m->impl);
    DeviceGuard g(m->impl.device());
    const size_t rows = (size_t)B * T;
    const int nm = m->impl.n_mels(), cs = m2s::chan_stride(nm);
    m2s::Workspace w(ws, ws_bytes);
    float* mn = w.take<float>(rows * nm);
    void* ln_t = w.take<char>(rows * cs * 4);
    char* rest = w.take<char>(0);
    const size_t rest_bytes = ws_bytes - (size_t)(rest - static_cast<char*>(ws));
    // acoustic scratch is dead once mel_norm is written; the vocoder reuses it
    m->impl.forward(frames, B, T, H, W, mn, rest, rest_bytes, S(stream));
    if (mel_norm) M2S_HIP(hipMemcpyAsync(mel_norm, mn, rows * nm * sizeof(float), hipMemcpyDeviceToDevice, S(stream)));
    m2s::Workspace vw(rest, rest_bytes);
    v->impl.forward_from_norm(mn, mean, std, B, T, mel_db, mel_log, ln_t, wav, vw, S(stream));
  });
}

int m2s_cam_create(const m2s_tensor* sd, int n, int device, m2s_cam** out) {
  return guarded([&] {
    M2S_CHECK(out && (sd || n == 0), "null argument");
    check_device(device);
    DeviceGuard g(device);
    *out = new m2s_cam{m2s::CamBackbone(m2s::make_state_dict(sd, n), device)};
  });
}

void m2s_cam_destroy(m2s_cam* c) { delete c; }

int m2s_cam_bn_layers(const m2s_cam* c) { return c ? c->impl.bn_layers() : 0; }

int m2s_cam_bn_channels(const m2s_cam* c, int layer) {
  return c && layer >= 0 && layer < c->impl.bn_layers() ? c->impl.bn_channels(layer) : 0;
}

size_t m2s_cam_workspace_bytes(const m2s_cam* c, int N, int H, int W) {
  size_t r = 0;
  if (!c) return 0;  // like the other size queries: 0 for a null handle
  guarded([&] { r = c->impl.workspace_bytes(N, H, W); });
  return r;
}

int m2s_cam_backbone(m2s_cam* c, const float* frames, int N, int H, int W, float* const* taps, float* bn_stats,
                     void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(c && frames && taps && bn_stats && ws, "null argument");
    DeviceGuard g(c->impl.device());
    c->impl.forward(frames, N, H, W, taps, bn_stats, ws, ws_bytes, S(stream));
  });
}

size_t m2s_bilstm_train_workspace_bytes(int B, int T, int C, int H) {
  size_t r = 0;
  guarded([&] { r = m2s::bilstm_train_workspace_bytes(B, T, C, H); });
  return r;
}

int m2s_bilstm_train_forward(const float* x, int B, int T, int C, int H, const float* const* w, float* y,
                             float* gates, float* cells, float* hid, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(x && w && y && gates && cells && hid && ws, "null argument");
    for (int i = 0; i < 8; ++i) M2S_CHECK(w[i], "null LSTM weight");
    const float* wih[2] = {w[0], w[4]};
    const float* whh[2] = {w[1], w[5]};
    const float* bih[2] = {w[2], w[6]};
    const float* bhh[2] = {w[3], w[7]};
    m2s::bilstm_train_forward(x, B, T, C, H, wih, whh, bih, bhh, y, gates, cells, hid, ws, ws_bytes, S(stream));
  });
}

int m2s_bilstm_train_backward(const float* x, const float* dy, int B, int T, int C, int H, const float* const* w,
                              const float* gates, const float* cells, const float* hid, float* dx, float* const* grads,
                              void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    M2S_CHECK(x && dy && w && gates && cells && hid && ws, "null argument");
    const float* wih[2] = {w[0], w[4]};
    const float* whh[2] = {w[1], w[5]};
    M2S_CHECK(wih[0] && wih[1] && whh[0] && whh[1], "null LSTM weight");
    float* dwih[2] = {grads ? grads[0] : nullptr, grads ? grads[3] : nullptr};
    float* dwhh[2] = {grads ? grads[1] : nullptr, grads ? grads[4] : nullptr};
    float* db[2] = {grads ? grads[2] : nullptr, grads ? grads[5] : nullptr};
    m2s::bilstm_train_backward(x, dy, B, T, C, H, wih, whh, gates, cells, hid, dx, dwih, dwhh, db, ws, ws_bytes,
                               S(stream));
  });
}

int m2s_linear_forward(const float* x, int rows, int in, int out, const float* w, const float* b, float* y,
                       void* stream) {
  return guarded([&] {
    M2S_CHECK(x && w && y && rows >= 0 && in > 0 && out > 0, "bad argument");
    m2s::linear_forward(x, rows, in, out, w, b, y, S(stream));
  });
}

int m2s_linear_backward(const float* dy, const float* x, int rows, int in, int out, const float* w, float* dx,
                        float* dw, float* db, void* stream) {
  return guarded([&] {
    M2S_CHECK(dy && x && w && rows >= 0 && in > 0 && out > 0, "bad argument");
    m2s::linear_backward(dy, x, rows, in, out, w, dx, dw, db, S(stream));
  });
}

int m2s_gap_forward(const float* x, int64_t nc, int p, float* y, void* stream) {
  return guarded([&] {
    M2S_CHECK(x && y && nc >= 0 && p > 0, "bad argument");
    m2s::launch_gap_nchw(x, nc, p, y, S(stream));
  });
}

int m2s_gap_backward(const float* dy, int64_t nc, int p, float* dx, void* stream) {
  return guarded([&] {
    M2S_CHECK(dy && dx && nc >= 0 && p > 0, "bad argument");
    m2s::launch_gap_nchw_bwd(dy, nc, p, dx, S(stream));
  });
}

int m2s_prof_enable(int on) { return m2s_prof_enable_impl(on); }

int m2s_prof_collect(m2s_prof_stat* out, int max, int* n_out) {
  return guarded([&] { m2s_prof_collect_impl(out, max, n_out); });
}

}  // extern "C"

int m2s_prof_launches(m2s_prof_launch* out, int max, int* n_out) {
  return guarded([&] { m2s_prof_launches_impl(out, max, n_out); });
}
