// Packed models and their execution plans (host side of libm2s).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "../../include/m2s.h"
#include "conv_igemm.hpp"
#include "kernels.hpp"

namespace m2s {

struct HostTensor {
  const float* data = nullptr;
  std::vector<int64_t> shape;
  size_t numel() const {
    size_t n = 1;
    for (auto d : shape) n *= (size_t)d;
    return n;
  }
};
using StateDict = std::map<std::string, HostTensor>;
StateDict make_state_dict(const m2s_tensor* t, int n);

// Host staging of every packed array; one device allocation per model.
class Arena {
 public:
  size_t add(const void* p, size_t bytes);
  template <class V>
  size_t add_vec(const std::vector<V>& v) {
    return add(v.data(), v.size() * sizeof(V));
  }
  void upload(int device);
  void* ptr(size_t off) const { return static_cast<char*>(dev_) + off; }
  size_t bytes() const { return host_.size(); }
  ~Arena();

 private:
  std::vector<uint8_t> host_;
  void* dev_ = nullptr;
};

// One packed dense conv layer (rows = output channels [x phases], k = tap * cs_in + c).
struct PConv {
  int kind = KIND_GEMM;
  int cin = 0, cout = 0, cs_in = 0, cs_out = 0;
  int ntaps = 1, ks = 1, stride = 1, kp = 0, n_pad = 0, tpc = 1, phases = 1;
  int dil = 1, pad_left = 0;
  int ct_u = 1, ct_pad = 0, ct_k = 1;
  double macs_per_row = 0;  // algorithmic MACs per output position (all phases)
  size_t w_off = 0, b_off = 0, ws_off = 0;
  bool fp8 = false;                // M2S_DT_FP8: e4m3-grid weights (bf16 storage) + per-channel scales
  const void* w = nullptr;
  const float* b = nullptr;
  const float* wscale = nullptr;   // [n_pad] when fp8
  void resolve(const Arena& a) {
    w = a.ptr(w_off);
    b = static_cast<const float*>(a.ptr(b_off));
    wscale = fp8 ? static_cast<const float*>(a.ptr(ws_off)) : nullptr;
  }
};

class Workspace {  // bump allocator over a caller-provided device buffer
 public:
  Workspace(void* base, size_t bytes) : base_(static_cast<char*>(base)), cap_(bytes) {}
  template <class T>
  T* take(size_t n) {
    size_t off = (used_ + 255) & ~size_t(255);
    used_ = off + n * sizeof(T);
    if (base_ && used_ > cap_) throw Error(M2S_E_ARG, "workspace too small");
    return base_ ? reinterpret_cast<T*>(base_ + off) : nullptr;
  }
  size_t used() const { return (used_ + 255) & ~size_t(255); }

 private:
  char* base_;
  size_t cap_;
  size_t used_ = 0;
};

class Acoustic {
 public:
  Acoustic(const StateDict& sd, int n_mels, int hidden, int dtype, int device);
  ~Acoustic();
  Acoustic(const Acoustic&) = delete;
  Acoustic& operator=(const Acoustic&) = delete;
  // M2S_E_INTERNAL (and clears the flag) if a BiLSTM barrier of an earlier launch timed out
  unsigned take_async_error();
  unsigned lstm_spin_max_ = LSTM_SPIN_MAX;  // fault injection: m2s_acoustic_set_lstm_spin_limit
  unsigned ws_spin_max_ = 1u << 20;        // LDS flag-ring waits of ir_ws / se_ws; m2s_acoustic_set_ws_spin_limit
  AsyncReport ws_report() const {
    AsyncReport r;
    r.spin_max = ws_spin_max_;
    r.err = err_dev_;
    return r;
  }
  int device() const { return device_; }
  int n_mels() const { return n_mels_; }
  int chunk = 1920;  // = m2s.config.CNN_CHUNK (the benched pass size)
  bool ir_fused_ = true;  // bf16: fused conv_pw + conv_dw + SE squeeze (env M2S_IR_FUSED=0 disables)
  bool ir_ws_ = true;     // split fp32: the persistent warp-specialised form of it (env M2S_IR_WS=0 disables)
  bool ir_ws_s2_ = true;  // ... also for the stride-2 block at 16x16 (env M2S_IR_WS_S2=0: ir_pwdw_s2)
  // Small passes (the reference CLI's one clip, configs[1]'s 8 x 4): the persistent one-workgroup-per-image (ir_ws)
  // and one-tile-per-CU (se_ws) kernels fill a few dozen CUs there, so below these sizes the pass runs the grid forms
  // (ir_pwdw / ir_pwdw_s2, the split-K conv_gemm SE GEMM).  Env M2S_IRWS_MIN (images per pass) / M2S_SEWS_MIN (se_ws
  // tiles, in CUs: 1 = one full round) override.
  int irws_min_ = 512;
  // ir_ws -> se_ws hand-off of the expanded map as plain fp32 rows instead of split pairs (env M2S_IRWS_F32=0: split)
  bool irws_f32_ = true;
  int sews_min_cus_ = 1;
  bool stem_fused_ = true;  // bf16: stem + blocks.0 in one kernel (env M2S_STEM_FUSED=0 disables)
  bool f8_er_ = true;            // fp8: EdgeResidual blocks.1.1/.2 on e4m3 (env M2S_F8_ER=0: bf16 er_fused)
  bool se_y8_ = true;            // fp8: the SE GEMM also stores the next expand's e4m3 operand (env M2S_SE_Y8=0:
                                 // launch_rows_e4m3 converts it; the same bytes, test_fp8_se_y8_e4m3_handoff_is_exact)
  bool f8_er2_ = true;           // fp8: EdgeResidual blocks.2.1/.2 on e4m3 (er8w_fused; env M2S_F8_ER2=0: bf16 er2_fused)
  bool er8_x8_ = true;           // ... their input as e4m3 bytes from the producer (env M2S_ER8_X8=0: converted
                                 // in er8_fused; the same bytes, test_fp8_er8_e4m3_handoff_is_exact)
  bool f8_expand_ = true;        // fp8: the stride-1 IR expand on e4m3 (env M2S_F8_EXPAND=0: bf16 expand)
  bool f8_s2_ = true;            // fp8: the stride-2 IR blocks (blocks.3.0 ir_s2band, blocks.5.0 ir_pwdw_s2) with e4m3
                                 // depthwise output + e4m3 SE GEMM (env M2S_F8_S2=0: bf16)
  bool se_fused_ = true;    // bf16: SE excitation in one kernel (env M2S_SE_FUSED=0: two GEMMs)
  bool er_fused_ = true;    // bf16: EdgeResidual 32->128->32 in one kernel (env M2S_ER_FUSED=0 disables)
  bool se_sp_ = false;      // split: SE-gated conv_pwl on gemm128.hip (env M2S_SE_SP=1; default conv_gemm's in-LDS
                            // scaling: the two measured equal, 7.85 vs 7.88 ms per step, profiles/r03o_se_sp_ab.txt)
  bool se_ws_ = true;      // split: SE-gated conv_pwl on the warp-specialised flag ring (se_ws.hip; env M2S_SE_WS=0:
                            // conv_gemm's barrier ring; 8.03 -> 7.17 ms per step, gpurun_out s4a)
  bool er_mrg_ = true;      // split EdgeResidual blocks.1: merged W_hi / W_lo ring stages (env M2S_ER_MRG=0: one per
                            // slot; 2088 vs 2164 us per launch, gpurun_out r03er)
  bool ir_s2band_ = true;   // blocks.3.0: fused banded conv_pw + stride-2 depthwise (env M2S_IR_S2BAND=0: unfused)
  bool lstm_persistent_ = true;  // one-launch BiLSTM recurrence (env M2S_LSTM_PERSISTENT=0: a launch per step)
  bool lstm_mid_ = true;         // 4 < B <= 16: granule-exchange recurrence (env M2S_LSTM_MID=0: counter barrier)
  bool lstm_x3_ = true;          // B > 4, non-fp32 engines: split-bf16 MFMA recurrence (env M2S_LSTM_X3=0: lstm_mid / f32)
  bool lstm_x3g_ = true;   // ... and for 5..16 sequences its granule hand-off form (env M2S_LSTM_X3G=0: lstm_x3)
  // (the M2S_* switches are read once, when the engine is created: A/B tests of fused vs unfused)

  size_t workspace_bytes(int B, int T, int H, int W) const;
  void forward(const float* frames, int B, int T, int H, int W, float* mel_norm, void* ws, size_t wsb, hipStream_t s);
  void effnet(const float* frames, int N, int H, int W, float* feats, int stop_after, float* probe, int* probe_dims,
              Workspace& ws, hipStream_t s);
  void bilstm(const float* feats, int B, int T, float* y, float* mel_norm, Workspace& ws, hipStream_t s);

 private:
  struct Block {
    int type = 0;  // 0 cn, 1 er, 2 ir
    int stride = 1, cin = 0, cout = 0, mid = 0, rd = 0;
    bool skip = false;
    PConv c1, c2;              // cn: c1 ; er: conv_exp, conv_pwl ; ir: conv_pw, conv_pwl
    size_t dw_w = 0, dw_b = 0;  // ir depthwise, tap-major (9 x cs_mid) and (cs_mid), fp32
    size_t dw_w2 = 0;           // bf16 engines: the same taps as bf16 in the channel's dword half
    PConv se1, se2;             // ir SE: conv_reduce (mid -> rd, SiLU), conv_expand (rd -> mid, sigmoid)
    size_t er_wexp = 0, er_wpwl = 0;  // bf16 er 32 -> 128 -> 32 stride 1: fused-kernel fragment orders
    bool er_frag = false;
    // fp8 engines, er 32 -> 128 -> 32 stride 1 on e4m3 (er8_fused.hip): fragments, per-channel scales
    size_t er8_wexp = 0, er8_sexp = 0, er8_wpwl = 0, er8_spwl = 0;
    bool er8 = false;
    // fp8 engines, er 56 -> 224 -> 56 stride 1 on e4m3 (er8w_fused.hip): stage stream, per-channel scales
    size_t er8w_w = 0, er8w_sexp = 0, er8w_spwl = 0;
    bool er8w = false;
    size_t er_sp_w = 0;  // split fp32 er stride 1: er_sp_fused.hip stage stream
    bool er_sp = false;
    bool ers_sp = false;  // split fp32 er stride 2 (blocks.1.0): er_wexp / er_wpwl in [hi/lo] fragment order
    // fp8 engines, ir conv_pwl: e4m3 bytes [f8_npad][f8_kp] of W / scale, per-channel scales, bias
    size_t f8_w = 0, f8_s = 0, f8_b = 0;
    int f8_kp = 0, f8_npad = 0;
    bool f8_pwl = false;
    // fp8 engines, ir conv_pw (stride 1): e4m3 bytes [round_up(cs_mid, 32)][f8x_kp] of W / scale, scales
    size_t f8x_w = 0, f8x_s = 0;
    int f8x_kp = 0;
    bool f8_pw = false;
  };
  template <typename T>
  void effnet_t(const float* frames, int N, int H, int W, float* feats, int stop_after, float* probe, int* probe_dims,
                Workspace& ws, hipStream_t s);
  size_t effnet_ws(int N, int H, int W) const;
  int pass_frames(int N) const;
  size_t effnet_x8(int H, int W) const;  // fp8 engines: bytes per image of an e4m3 expand-operand buffer
  void effnet_dims(int H, int W, size_t* io_elems, size_t* mid_elems, size_t* se_elems) const;

  int dtype_, device_, n_mels_, hidden_;
  Arena arena_;
  size_t stem_w_ = 0, stem_b_ = 0;
  std::vector<Block> blocks_;
  PConv lstm_ih_;
  size_t whh_ = 0, head_wt_ = 0, head_b_ = 0;
  int max_mid_cs_ = 0;
  unsigned* err_host_ = nullptr;  // pinned, host-mapped: set by lstm_persistent_kernel on a barrier timeout
  unsigned* err_dev_ = nullptr;
  // the granule BiLSTM kernels' sync buffer (lstm_small / lstm_x3g), zeroed once, and its epoch count
  // (lstm_persistent.hip lstm_epoch)
  void* gsync_ = nullptr;
  unsigned gsync_epoch_ = 0;
};

class Vocoder {
 public:
  Vocoder(const StateDict& sd, const m2s_hifigan_h& h, int dtype, int device);
  int device() const { return device_; }
  int hop() const { return hop_; }
  int num_mels() const { return h_.num_mels; }
  size_t workspace_bytes(int B, int T) const;
  void forward(const float* mel, int layout, int B, int T, float* wav, Workspace& ws, hipStream_t s);
  // pipeline entry: mel glue (dB, ln-power; run_mri_video_inference.py:227-233) fused with the
  // cast to the channel-last vocoder input (ln_buf: rows x cs(num_mels) x 4 bytes), then the generator.
  void forward_from_norm(const float* mel_norm, const float* mean, const float* std_, int B, int T, float* mel_db,
                         float* mel_log, void* ln_buf, float* wav, Workspace& ws, hipStream_t s);
  size_t act_elems(int B, int T) const;
  bool mrf_fused_ = true;
  bool mrf_halo_ = true;   // split: C = 64 MRF convs with once-staged input rows (env M2S_MRF_HALO=0: conv_gemm)
  // fp8: the C = 64 / 32 MRF convs on e4m3 (conv1d_f8, 128 / C taps a K step; env M2S_F8_MRF64=1 / M2S_F8_MRF32=1).
  // Off: the fused bf16 ResBlock1 keeps a resblock's intermediates on chip and is faster at configs[4] (8 x 1000
  // frames, same box, gpurun_out/f8s2: fp8 step 74.8 ms with both fused, 79.7 with C = 64 on e4m3, 85.1 with both)
  bool f8_mrf64_ = false;
  bool f8_mrf32_ = false;
  bool mrf_batch_ = true;  // split: resblocks of a conv_gemm MRF stage batched per launch (env M2S_MRF_BATCH=0 disables)  // bf16: fused ResBlock1 kernel for C in {32, 64} (env M2S_MRF_FUSED=0 disables)

 private:
  template <typename T>
  void run_t(const void* mel_nlc, int B, int Tn, float* wav, Workspace& ws, hipStream_t s);
  template <typename T>
  void mrf_stage_batched(int i, const T* X, T* S, T* const (*Bt)[3], int B, int L, bool act_out, hipStream_t s);
  int act_buffers() const;  // activation buffers of act_elems() each in the workspace
  struct RB {
    int k = 3;
    std::vector<int> dil;
    std::vector<PConv> c1, c2;  // resblock "1": c1 (dilated) + c2 ; "2": c1 only
    // bf16 resblock "1" at C in {32, 64}: the same weights in the fused kernel's fragment order
    std::vector<size_t> f1_off, f2_off;
    std::vector<const bf16_t*> f1, f2;
    // split resblock "1" at C in {64, 128}: conv1d_halo.hip fragment order
    std::vector<size_t> h1_off, h2_off;
    std::vector<const bf16_t*> h1, h2;
    // fp8 resblock "1" at C in {128, 256}: e4m3 [C][k C] weights, scales, biases (conv1d_f8)
    struct F8 {
      size_t w = 0, s = 0, b = 0;
      const void* wp = nullptr;
      const float* sp = nullptr;
      const float* bp = nullptr;
    };
    std::vector<F8> q1, q2;
  };
  m2s_hifigan_h h_;
  int dtype_, device_, hop_ = 1;
  Arena arena_;
  PConv pre_;
  std::vector<PConv> ups_;
  std::vector<RB> rbs_;
  size_t post_w_ = 0;
  float post_b_ = 0.f;
  int post_c_ = 0;
};

}  // namespace m2s
