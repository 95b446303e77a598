// Weight packing and execution plans for the acoustic model (CNN + BiLSTM + head) and the
// HiFi-GAN generator.  Packing mirrors what the reference does at load time and folds what is
// constant at inference:
//   * BatchNorm (eps 1e-3, torch's alpha = w / sqrt(var + eps), beta = b - mean * alpha) into
//     the preceding conv (timm BatchNormAct2d);
//   * the grey -> RGB repeat (mri_acoustic_model.py:43-44) into conv_stem (sum over in-channels);
//   * weight norm w = g * v / ||v|| (models.py:94-108; run_mri_video_inference.py:99-115);
//   * LSTM b_ih + b_hh.
#include "model.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "pack.hpp"
#include "prof.hpp"

namespace m2s {

// ------------------------------------------------------------------------------------------
StateDict make_state_dict(const m2s_tensor* t, int n) {
  StateDict sd;
  for (int i = 0; i < n; ++i) {
    M2S_CHECK(t[i].name != nullptr, "state dict entry without a name");
    if (t[i].elem != M2S_ELEM_F32) continue;  // num_batches_tracked etc.
    M2S_CHECK(t[i].ndim >= 0 && t[i].ndim <= 4, std::string("bad ndim for ") + t[i].name);
    HostTensor h;
    h.data = static_cast<const float*>(t[i].data);
    for (int d = 0; d < t[i].ndim; ++d) h.shape.push_back(t[i].shape[d]);
    sd[t[i].name] = h;
  }
  return sd;
}


size_t Arena::add(const void* p, size_t bytes) {
  size_t off = (host_.size() + 255) & ~size_t(255);
  host_.resize(off + bytes);
  if (bytes) std::memcpy(host_.data() + off, p, bytes);
  return off;
}

void Arena::upload(int device) {
  M2S_HIP(hipSetDevice(device));
  M2S_HIP(hipMalloc(&dev_, host_.size() + 256));
  M2S_HIP(hipMemcpy(dev_, host_.data(), host_.size(), hipMemcpyHostToDevice));
  std::vector<uint8_t>().swap(host_);
}

Arena::~Arena() {
  if (dev_) (void)hipFree(dev_);
}


// ------------------------------------------------------------------------------------------
// Acoustic model

struct BN {
  std::vector<float> a, b;
};
static BN fold_bn(const StateDict& sd, const std::string& p, int c) {
  const float* w = need(sd, p + ".weight", {c}).data;
  const float* bb = need(sd, p + ".bias", {c}).data;
  const float* m = need(sd, p + ".running_mean", {c}).data;
  const float* v = need(sd, p + ".running_var", {c}).data;
  BN r;
  r.a.resize(c);
  r.b.resize(c);
  for (int i = 0; i < c; ++i) {
    const float invstd = 1.0f / std::sqrt(v[i] + 1e-3f);
    r.a[i] = invstd * w[i];
    r.b[i] = bb[i] - m[i] * r.a[i];
  }
  return r;
}

Acoustic::Acoustic(const StateDict& sd, int n_mels, int hidden, int dtype, int device)
    : dtype_(dtype), device_(device), n_mels_(n_mels), hidden_(hidden) {
  M2S_CHECK(dtype == M2S_DT_F32 || dtype == M2S_DT_BF16 || dtype == M2S_DT_BF16X3 || dtype == M2S_DT_FP8, "bad dtype");
  M2S_CHECK(n_mels > 0 && hidden > 0 && hidden % 8 == 0, "bad n_mels / rnn_hidden");
  if (const char* e = std::getenv("M2S_IR_FUSED")) ir_fused_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_IR_WS")) ir_ws_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_IR_WS_S2")) ir_ws_s2_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_IRWS_MIN")) irws_min_ = std::atoi(e);
  if (const char* e = std::getenv("M2S_IRWS_F32")) irws_f32_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_SEWS_MIN")) sews_min_cus_ = std::atoi(e);
  if (const char* e = std::getenv("M2S_STEM_FUSED")) stem_fused_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_F8_EXPAND")) f8_expand_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_F8_S2")) f8_s2_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_F8_ER")) f8_er_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_ER8_X8")) er8_x8_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_F8_ER2")) f8_er2_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_SE_Y8")) se_y8_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_SE_FUSED")) se_fused_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_ER_FUSED")) er_fused_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_SE_SP")) se_sp_ = std::strcmp(e, "0") != 0;  // A/B only
  if (const char* e = std::getenv("M2S_SE_WS")) se_ws_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_ER_MRG")) er_mrg_ = std::strcmp(e, "0") != 0;  // A/B and tests only
  if (const char* e = std::getenv("M2S_IR_S2BAND")) ir_s2band_ = std::strcmp(e, "0") != 0;  // A/B and tests only
  if (const char* e = std::getenv("M2S_LSTM_PERSISTENT")) lstm_persistent_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_LSTM_MID")) lstm_mid_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_LSTM_X3")) lstm_x3_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_LSTM_X3G")) lstm_x3g_ = std::strcmp(e, "0") != 0;
  const std::string P = "cnn.backbone.";
  {  // stem: fold repeat(1,3,1,1) by summing the 3 input channels; then BN
    const float* w = need(sd, P + "conv_stem.weight", {EFF_STEM, 3, 3, 3}).data;
    BN bn = fold_bn(sd, P + "bn1", EFF_STEM);
    std::vector<float> w9(EFF_STEM * 9);
    for (int o = 0; o < EFF_STEM; ++o)
      for (int t = 0; t < 9; ++t)
        w9[o * 9 + t] = (w[(o * 3 + 0) * 9 + t] + w[(o * 3 + 1) * 9 + t] + w[(o * 3 + 2) * 9 + t]) * bn.a[o];
    stem_w_ = arena_.add_vec(w9);
    stem_b_ = arena_.add_vec(bn.b);
  }
  // fp8 engines run the bf16 kernels (and bf16 packings) except the stride-1 IR blocks' SE-gated conv_pwl,
  // which gets an e4m3 copy for the block-scaled MFMA (gemm128.hip) below
  const int pdt = dtype == M2S_DT_FP8 ? M2S_DT_BF16 : dtype;
  int cin = EFF_STEM;
  for (int s = 0; s < 6; ++s) {
    const StageDef& sdf = kStages[s];
    for (int r = 0; r < sdf.reps; ++r) {
      Block b;
      b.type = sdf.type;
      b.stride = r == 0 ? sdf.stride : 1;
      b.cin = cin;
      b.cout = sdf.cout;
      b.skip = b.stride == 1 && cin == sdf.cout;
      const std::string q = P + "blocks." + std::to_string(s) + "." + std::to_string(r) + ".";
      const int k = sdf.k;
      auto conv2d_kxk = [&](PConv& pc, const std::string& wk, int ci, int co, const BN& bn) {
        const float* w = need(sd, wk, {co, ci, k, k}).data;
        pc = make_pconv(KIND_CONV2D, ci, co, k * k, pdt);
        pc.ks = k;
        pc.stride = b.stride;
        pc.macs_per_row = (double)co * ci * k * k;
        pack_conv(arena_, pdt, pc, [&](int, int n, int t, int c) { return w[((size_t)n * ci + c) * k * k + t] * bn.a[n]; },
                  [&](int n) { return bn.b[n]; });
      };
      auto conv1x1 = [&](PConv& pc, const std::string& wk, int ci, int co, const BN& bn) {
        const float* w = need(sd, wk, {co, ci, 1, 1}).data;
        pc = make_pconv(KIND_GEMM, ci, co, 1, pdt);
        pc.macs_per_row = (double)co * ci;
        pack_conv(arena_, pdt, pc, [&](int, int n, int, int c) { return w[(size_t)n * ci + c] * bn.a[n]; },
                  [&](int n) { return bn.b[n]; });
      };
      if (b.type == 0) {
        conv2d_kxk(b.c1, q + "conv.weight", cin, b.cout, fold_bn(sd, q + "bn1", b.cout));
      } else if (b.type == 1) {
        b.mid = make_divisible(cin * (double)sdf.exp);
        conv2d_kxk(b.c1, q + "conv_exp.weight", cin, b.mid, fold_bn(sd, q + "bn1", b.mid));
        conv1x1(b.c2, q + "conv_pwl.weight", b.mid, b.cout, fold_bn(sd, q + "bn2", b.cout));
        if (dtype == M2S_DT_BF16X3 && b.stride == 1 && b.skip && k == 3 &&
            er_sp_supported(32, 32, b.c1.cs_in, b.mid, chan_stride(b.cout))) {
          // er_sp_fused.hip stage stream: per conv_exp k-step (tap, 32 input channels) a W_hi and a W_lo
          // stage of nt fragments [n16][lane][8]; then conv_pwl's W_hi stages and W_lo stages, piece
          // j = (k-step j / ON, n16 j % ON), K permuted as in er_fused.hip
          int nt = 0;
          const int csi = b.c1.cs_in, cso = chan_stride(b.cout), nst = er_sp_nt_stages(csi, b.mid, cso, &nt);
          const int kc = csi / 32, nce = 9 * kc * 2, on_n = cso / 16, pn = on_n * (b.mid / 32), nps = (pn + nt - 1) / nt;
          const float* we = need(sd, q + "conv_exp.weight", {b.mid, cin, 3, 3}).data;
          const float* wq = need(sd, q + "conv_pwl.weight", {b.cout, b.mid, 1, 1}).data;
          const BN e1 = fold_bn(sd, q + "bn1", b.mid), e2 = fold_bn(sd, q + "bn2", b.cout);
          std::vector<uint16_t> st((size_t)nst * nt * 64 * 8, 0);
          for (int sg = 0; sg < nst; ++sg)
            for (int pc = 0; pc < nt; ++pc)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int row = ln & 15, g8 = ln >> 4;
                  float v = 0.f;
                  int plane;
                  if (sg < nce) {
                    plane = sg & 1;
                    const int ks = sg >> 1, t = ks / kc, c = (ks % kc) * 32 + 8 * g8 + e, n = 16 * pc + row;
                    if (c < cin) v = we[((size_t)n * cin + c) * 9 + t] * e1.a[n];
                  } else {
                    plane = (sg - nce) / nps;
                    const int j = ((sg - nce) % nps) * nt + pc;
                    if (j >= pn) continue;
                    const int kk = j / on_n, on = j % on_n, o = on * 16 + row;
                    const int c = 32 * kk + (e < 4 ? 4 * g8 + e : 16 + 4 * g8 + e - 4);
                    if (o < b.cout) v = wq[(size_t)o * b.mid + c] * e2.a[o];
                  }
                  uint16_t hi, lo;
                  split_host(v, &hi, &lo);
                  st[(((size_t)sg * nt + pc) * 64 + ln) * 8 + e] = plane == 0 ? hi : lo;
                }
          b.er_sp_w = arena_.add_vec(st);
          b.er_sp = true;
        } else if (dtype == M2S_DT_BF16X3 && b.stride == 2 && k == 3 &&
                   ers2_sp_supported(8, 16, b.c1.cs_in, b.mid, chan_stride(b.cout))) {
          // ers2_sp_kernel (ers2_fused.hip): conv_exp [hi/lo][k-step][n16][lane][8] (lane groups 0-1:
          // tap 2s, 2-3: tap 2s + 1), conv_pwl [hi/lo][n16][k-step][lane][8] with the permuted K
          const int csi = b.c1.cs_in, cso = chan_stride(b.cout), ks_n = (9 * csi + 31) / 32, ntn = b.mid / 16;
          const int onn = cso / 16, pkn = b.mid / 32;
          const float* we = need(sd, q + "conv_exp.weight", {b.mid, cin, 3, 3}).data;
          const float* wq = need(sd, q + "conv_pwl.weight", {b.cout, b.mid, 1, 1}).data;
          const BN e1 = fold_bn(sd, q + "bn1", b.mid), e2 = fold_bn(sd, q + "bn2", b.cout);
          const size_t fe_half = (size_t)ks_n * ntn * 64 * 8, fp_half = (size_t)onn * pkn * 64 * 8;
          std::vector<uint16_t> fe(2 * fe_half, 0), fp(2 * fp_half, 0);
          for (int s2 = 0; s2 < ks_n; ++s2)
            for (int nt = 0; nt < ntn; ++nt)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int g8 = ln >> 4, n = nt * 16 + (ln & 15), t = 2 * s2 + (g8 >> 1), c = 8 * (g8 & 1) + e;
                  const float v = t < 9 && c < cin ? we[((size_t)n * cin + c) * 9 + t] * e1.a[n] : 0.f;
                  const size_t i = (((size_t)s2 * ntn + nt) * 64 + ln) * 8 + e;
                  split_host(v, &fe[i], &fe[fe_half + i]);
                }
          for (int on = 0; on < onn; ++on)
            for (int ks = 0; ks < pkn; ++ks)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int n = on * 16 + (ln & 15), g4 = 4 * (ln >> 4);
                  const int c = 32 * ks + (e < 4 ? g4 + e : 16 + g4 + e - 4);
                  const float v = n < b.cout ? wq[(size_t)n * b.mid + c] * e2.a[n] : 0.f;
                  const size_t i = (((size_t)on * pkn + ks) * 64 + ln) * 8 + e;
                  split_host(v, &fp[i], &fp[fp_half + i]);
                }
          b.er_wexp = arena_.add_vec(fe);
          b.er_wpwl = arena_.add_vec(fp);
          b.ers_sp = true;
        } else if (pdt == M2S_DT_BF16 && b.stride == 1 && b.skip && k == 3 &&
            er_fused_supported(64, 64, cin, b.mid, b.cout, b.c1.kp, b.c2.kp)) {
          // er_fused.hip operand orders: conv_exp [tap][n16][lane][8] (lane = (k8 group, row));
          // conv_pwl [n16][k-step][lane][8] with the k-slot permutation of the kernel's header
          const float* we = need(sd, q + "conv_exp.weight", {b.mid, cin, 3, 3}).data;
          const float* wq = need(sd, q + "conv_pwl.weight", {b.cout, b.mid, 1, 1}).data;
          const BN e1 = fold_bn(sd, q + "bn1", b.mid), e2 = fold_bn(sd, q + "bn2", b.cout);
          std::vector<uint16_t> fe((size_t)9 * 8 * 64 * 8), fp((size_t)2 * 4 * 64 * 8);
          for (int t = 0; t < 9; ++t)
            for (int nt = 0; nt < 8; ++nt)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int n = nt * 16 + (ln & 15), c = 8 * (ln >> 4) + e;
                  fe[(((size_t)t * 8 + nt) * 64 + ln) * 8 + e] = f2bf_host(we[((size_t)n * cin + c) * 9 + t] * e1.a[n]);
                }
          for (int on = 0; on < 2; ++on)
            for (int ks = 0; ks < 4; ++ks)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int n = on * 16 + (ln & 15), g4 = 4 * (ln >> 4);
                  const int c = 32 * ks + (e < 4 ? g4 + e : 16 + g4 + e - 4);
                  fp[(((size_t)on * 4 + ks) * 64 + ln) * 8 + e] = f2bf_host(wq[(size_t)n * b.mid + c] * e2.a[n]);
                }
          b.er_wexp = arena_.add_vec(fe);
          b.er_wpwl = arena_.add_vec(fp);
          b.er_frag = true;
          if (dtype == M2S_DT_FP8) {
            // er8_fused.hip: conv_exp [q][nt][half][lane][16 B], byte 16 half + j of lane (r16, g) = tap 4q + g
            // (zero past tap 8), input channel 16 half + j of output channel 16 nt + r16; conv_pwl
            // [on][half][lane][16 B], byte b = 4 nt + e of lane (r16, g) = mid channel 16 nt + 4 g + e
            std::vector<float> s1(128, 1.f), s2(32, 1.f);
            auto wexp_at = [&](int n, int c, int t) { return we[((size_t)n * cin + c) * 9 + t] * e1.a[n]; };
            for (int n = 0; n < 128; ++n) {
              float amax = 0.f;
              for (int c = 0; c < 32; ++c)
                for (int t = 0; t < 9; ++t) amax = std::max(amax, std::fabs(wexp_at(n, c, t)));
              if (amax > 0.f) s1[n] = amax / 448.f;
            }
            for (int o = 0; o < 32; ++o) {
              float amax = 0.f;
              for (int c = 0; c < 128; ++c) amax = std::max(amax, std::fabs(wq[(size_t)o * b.mid + c] * e2.a[o]));
              if (amax > 0.f) s2[o] = amax / 448.f;
            }
            std::vector<uint8_t> f8e((size_t)3 * 8 * 2 * 64 * 16, 0), f8p((size_t)2 * 2 * 64 * 16, 0);
            for (int q4 = 0; q4 < 3; ++q4)
              for (int nt = 0; nt < 8; ++nt)
                for (int h = 0; h < 2; ++h)
                  for (int ln = 0; ln < 64; ++ln)
                    for (int j = 0; j < 16; ++j) {
                      const int t = 4 * q4 + (ln >> 4), n = nt * 16 + (ln & 15), c = 16 * h + j;
                      if (t < 9)
                        f8e[((((size_t)q4 * 8 + nt) * 2 + h) * 64 + ln) * 16 + j] =
                            e4m3_bits_host(e4m3_host(wexp_at(n, c, t) / s1[n]));
                    }
            for (int on = 0; on < 2; ++on)
              for (int h = 0; h < 2; ++h)
                for (int ln = 0; ln < 64; ++ln)
                  for (int j = 0; j < 16; ++j) {
                    const int o = on * 16 + (ln & 15), bb = 16 * h + j, c = 16 * (bb >> 2) + 4 * (ln >> 4) + (bb & 3);
                    f8p[(((size_t)on * 2 + h) * 64 + ln) * 16 + j] =
                        e4m3_bits_host(e4m3_host(wq[(size_t)o * b.mid + c] * e2.a[o] / s2[o]));
                  }
            b.er8_wexp = arena_.add_vec(f8e);
            b.er8_sexp = arena_.add_vec(s1);
            b.er8_wpwl = arena_.add_vec(f8p);
            b.er8_spwl = arena_.add_vec(s2);
            b.er8 = true;
          }
        } else if (pdt == M2S_DT_BF16 && b.stride == 1 && b.skip && k == 3 &&
                   er2_fused_supported(32, 32, b.c1.cs_in, b.mid, b.cout, b.c1.kp, b.c2.kp)) {
          // er2_fused.hip stage stream [20][16 pieces][lane][8]: stages 0..17 = conv_exp k-step s (tap
          // s / 2, input channels 32 (s % 2) ..), piece = n16; stages 18 / 19 = conv_pwl k-steps 0..3 /
          // 4..6, piece = local k-step * 4 + n16, with er_fused.hip's k-slot permutation
          const float* we = need(sd, q + "conv_exp.weight", {b.mid, cin, 3, 3}).data;
          const float* wq = need(sd, q + "conv_pwl.weight", {b.cout, b.mid, 1, 1}).data;
          const BN e1 = fold_bn(sd, q + "bn1", b.mid), e2 = fold_bn(sd, q + "bn2", b.cout);
          std::vector<uint16_t> st((size_t)er2_stage_elems(), 0);
          for (int sg = 0; sg < 20; ++sg)
            for (int pc = 0; pc < 16; ++pc)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int row = ln & 15, g8 = ln >> 4;
                  float v = 0.f;
                  if (sg < 18) {
                    const int n = 16 * pc + row, c = (sg & 1) * 32 + 8 * g8 + e, t = sg >> 1;
                    if (pc < 14 && c < cin) v = we[((size_t)n * cin + c) * 9 + t] * e1.a[n];
                  } else {
                    const int kk = pc >> 2, n = 16 * (pc & 3) + row, ks = (sg == 18 ? 0 : 4) + kk;
                    const int c = 32 * ks + (e < 4 ? 4 * g8 + e : 16 + 4 * g8 + e - 4);
                    if ((sg == 18 || kk < 3) && n < b.cout) v = wq[(size_t)n * b.mid + c] * e2.a[n];
                  }
                  st[(((size_t)sg * 16 + pc) * 64 + ln) * 8 + e] = f2bf_host(v);
                }
          b.er_wexp = arena_.add_vec(st);
          b.er_frag = true;
          if (dtype == M2S_DT_FP8 && er8w_fused_supported(32, 32, b.c1.cs_in, b.mid, b.cout)) {
            // er8w_fused.hip stage stream: conv_exp K step q = [nt 0..15][half][lane (r16, g)][16 B], byte 16 half + j =
            // tap 2q + (g >> 1), input channel 32 (g & 1) + 16 half + j of output channel 16 nt + r16 (zero past tap 8,
            // channel 55, mid channel 223); conv_pwl [on][kq][half][lane][16 B], byte b = 16 half + j = mid channel
            // 16 (8 kq + b / 4) + 4 g + (b & 3) of output channel 16 on + r16.  Weights / per-channel scale s = amax / 448
            const int mid = b.mid, co = b.cout;
            std::vector<float> s1(mid, 1.f), s2(64, 1.f);
            auto wexp_at = [&](int n, int c, int t) { return we[((size_t)n * cin + c) * 9 + t] * e1.a[n]; };
            for (int n = 0; n < mid; ++n) {
              float amax = 0.f;
              for (int c = 0; c < cin; ++c)
                for (int t = 0; t < 9; ++t) amax = std::max(amax, std::fabs(wexp_at(n, c, t)));
              if (amax > 0.f) s1[n] = amax / 448.f;
            }
            for (int o = 0; o < co; ++o) {
              float amax = 0.f;
              for (int c = 0; c < mid; ++c) amax = std::max(amax, std::fabs(wq[(size_t)o * mid + c] * e2.a[o]));
              if (amax > 0.f) s2[o] = amax / 448.f;
            }
            std::vector<uint8_t> w8(er8w_stream_bytes(), 0);
            for (int q2 = 0; q2 < 5; ++q2)
              for (int nt = 0; nt < 16; ++nt)
                for (int h = 0; h < 2; ++h)
                  for (int ln = 0; ln < 64; ++ln)
                    for (int j = 0; j < 16; ++j) {
                      const int g4 = ln >> 4, t = 2 * q2 + (g4 >> 1), c = 32 * (g4 & 1) + 16 * h + j, n = 16 * nt + (ln & 15);
                      if (t < 9 && c < cin && n < mid)
                        w8[(((((size_t)q2 * 16 + nt) * 2 + h) * 64 + ln) * 16) + j] = e4m3_bits_host(e4m3_host(wexp_at(n, c, t) / s1[n]));
                    }
            const size_t pw0 = (size_t)5 * 32 * 1024;
            for (int on = 0; on < 4; ++on)
              for (int kq = 0; kq < 2; ++kq)
                for (int h = 0; h < 2; ++h)
                  for (int ln = 0; ln < 64; ++ln)
                    for (int j = 0; j < 16; ++j) {
                      const int o = 16 * on + (ln & 15), bb = 16 * h + j, ntp = 8 * kq + (bb >> 2);
                      const int c = 16 * ntp + 4 * (ln >> 4) + (bb & 3);
                      if (o < co && ntp < mid / 16)
                        w8[pw0 + (((((size_t)on * 2 + kq) * 2 + h) * 64 + ln) * 16) + j] =
                            e4m3_bits_host(e4m3_host(wq[(size_t)o * mid + c] * e2.a[o] / s2[o]));
                    }
            b.er8w_w = arena_.add_vec(w8);
            b.er8w_sexp = arena_.add_vec(s1);
            b.er8w_spwl = arena_.add_vec(s2);
            b.er8w = true;
          }
        } else if (pdt == M2S_DT_BF16 && b.stride == 2 && k == 3 &&
                   ers2_fused_supported(8, 16, b.c1.cs_in, b.mid, chan_stride(b.cout), b.c1.kp, b.c2.kp)) {
          // ers2_fused.hip: conv_exp [k-step][n16][lane][8] (CIN 16: lane groups 0-1 tap 2s, 2-3 tap
          // 2s + 1; CIN 32: tap s), conv_pwl [n16][k-step][lane][8] with the permuted K
          const int csi = b.c1.cs_in, cso = chan_stride(b.cout), ks_n = (9 * csi + 31) / 32;
          const float* we = need(sd, q + "conv_exp.weight", {b.mid, cin, 3, 3}).data;
          const float* wq = need(sd, q + "conv_pwl.weight", {b.cout, b.mid, 1, 1}).data;
          const BN e1 = fold_bn(sd, q + "bn1", b.mid), e2 = fold_bn(sd, q + "bn2", b.cout);
          std::vector<uint16_t> fe((size_t)ers2_exp_elems(csi, b.mid), 0), fp((size_t)cso * b.mid, 0);
          for (int s2 = 0; s2 < ks_n; ++s2)
            for (int nt = 0; nt < b.mid / 16; ++nt)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int g8 = ln >> 4, n = nt * 16 + (ln & 15);
                  const int t = csi == 16 ? 2 * s2 + (g8 >> 1) : s2, c = csi == 16 ? 8 * (g8 & 1) + e : 8 * g8 + e;
                  const float v = t < 9 && c < cin ? we[((size_t)n * cin + c) * 9 + t] * e1.a[n] : 0.f;
                  fe[(((size_t)s2 * (b.mid / 16) + nt) * 64 + ln) * 8 + e] = f2bf_host(v);
                }
          for (int on = 0; on < cso / 16; ++on)
            for (int ks = 0; ks < b.mid / 32; ++ks)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int n = on * 16 + (ln & 15), g4 = 4 * (ln >> 4);
                  const int c = 32 * ks + (e < 4 ? g4 + e : 16 + g4 + e - 4);
                  const float v = n < b.cout ? wq[(size_t)n * b.mid + c] * e2.a[n] : 0.f;
                  fp[(((size_t)on * (b.mid / 32) + ks) * 64 + ln) * 8 + e] = f2bf_host(v);
                }
          b.er_wexp = arena_.add_vec(fe);
          b.er_wpwl = arena_.add_vec(fp);
          b.er_frag = true;
        }
      } else {
        b.mid = make_divisible(cin * (double)sdf.exp);
        b.rd = (int)std::lround(b.mid * (sdf.se / sdf.exp));
        const int m = b.mid, cs = chan_stride(m);
        max_mid_cs_ = std::max(max_mid_cs_, cs);
        conv1x1(b.c1, q + "conv_pw.weight", cin, m, fold_bn(sd, q + "bn1", m));
        // the e4m3 expand (ir_pwdw / ir_pwdw_s2 x8; the stride-2 blocks' copy is used where ir_pwdw_s2 runs, blocks.5.0)
        if (dtype == M2S_DT_FP8 && chan_stride(cin) <= 256) {
          const float* wq = need(sd, q + "conv_pw.weight", {m, cin, 1, 1}).data;
          const BN bn1 = fold_bn(sd, q + "bn1", m);
          size_t boff = 0;
          b.f8x_kp = round_up(chan_stride(cin), 128);
          pack_gemm_f8(arena_, cin, m, round_up(cs, 32), b.f8x_kp, [&](int n, int c) { return wq[(size_t)n * cin + c] * bn1.a[n]; },
                       [&](int n) { return bn1.b[n]; }, &b.f8x_w, &b.f8x_s, &boff);
          b.f8_pw = true;
        }
        const float* wd = need(sd, q + "conv_dw.weight", {m, 1, k, k}).data;
        BN bn2 = fold_bn(sd, q + "bn2", m);
        std::vector<float> w9((size_t)cs * 9, 0.f), bd(cs, 0.f);
        for (int c = 0; c < m; ++c) {
          for (int t = 0; t < 9; ++t) w9[(size_t)t * cs + c] = wd[(size_t)c * 9 + t] * bn2.a[c];  // tap-major
          bd[c] = bn2.b[c];
        }
        b.dw_w = arena_.add_vec(w9);
        b.dw_b = arena_.add_vec(bd);
        if (pdt == M2S_DT_BF16) {  // fused kernel: bf16 weight in the half matching the channel
          std::vector<uint32_t> w2(w9.size());  // (v_dot2 against a (c, c+1) activation dword)
          for (size_t i = 0; i < w9.size(); ++i) {
            const uint32_t h = f2bf_host(w9[i]);
            w2[i] = (i % cs) % 2 == 0 ? h : h << 16;
          }
          b.dw_w2 = arena_.add_vec(w2);
        }
        const float* w1 = need(sd, q + "se.conv_reduce.weight", {b.rd, m, 1, 1}).data;
        const float* b1 = need(sd, q + "se.conv_reduce.bias", {b.rd}).data;
        const float* w2 = need(sd, q + "se.conv_expand.weight", {m, b.rd, 1, 1}).data;
        const float* b2 = need(sd, q + "se.conv_expand.bias", {m}).data;
        // SE excitation as two GEMMs over all images: (N x mid) . W1^T -> SiLU -> . W2^T -> sigmoid
        const int rd = b.rd;
        // (fp8 engines keep the SE excitation in bf16: a gate error scales the whole block output)
        const int se_dt = dtype == M2S_DT_FP8 ? M2S_DT_BF16 : dtype;
        b.se1 = make_pconv(KIND_GEMM, m, rd, 1, se_dt);
        b.se1.macs_per_row = (double)m * rd;
        pack_conv(arena_, se_dt, b.se1, [&](int, int n, int, int c) { return w1[(size_t)n * m + c]; },
                  [&](int n) { return b1[n]; });
        b.se2 = make_pconv(KIND_GEMM, rd, m, 1, se_dt);
        b.se2.macs_per_row = (double)m * rd;
        pack_conv(arena_, se_dt, b.se2, [&](int, int n, int, int c) { return w2[(size_t)n * rd + c]; },
                  [&](int n) { return b2[n]; });
        conv1x1(b.c2, q + "conv_pwl.weight", m, b.cout, fold_bn(sd, q + "bn3", b.cout));
        if (dtype == M2S_DT_FP8 && chan_stride(b.cout) <= 224) {  // (stride 2: used with ir_pwdw_s2's e4m3 output)
          const float* wq = need(sd, q + "conv_pwl.weight", {b.cout, m, 1, 1}).data;
          const BN bn3 = fold_bn(sd, q + "bn3", b.cout);
          b.f8_kp = round_up(cs, 128);
          b.f8_npad = std::max(round_up(chan_stride(b.cout), 64), chan_stride(b.cout) > 128 ? 224 : 128);
          pack_gemm_f8(arena_, m, b.cout, b.f8_npad, b.f8_kp, [&](int n, int c) { return wq[(size_t)n * m + c] * bn3.a[n]; },
                       [&](int n) { return bn3.b[n]; }, &b.f8_w, &b.f8_s, &b.f8_b);
          b.f8_pwl = true;
        }
      }
      blocks_.push_back(b);
      cin = sdf.cout;
    }
  }
  // BiLSTM: input projection of both directions as one fp32 GEMM (rows [fwd 4H | bwd 4H]).
  const int H = hidden_;
  const float* wih[2] = {need(sd, "rnn.lstm.weight_ih_l0", {4 * H, EFF_OUT}).data,
                         need(sd, "rnn.lstm.weight_ih_l0_reverse", {4 * H, EFF_OUT}).data};
  const float* bih[2] = {need(sd, "rnn.lstm.bias_ih_l0", {4 * H}).data, need(sd, "rnn.lstm.bias_ih_l0_reverse", {4 * H}).data};
  const float* bhh[2] = {need(sd, "rnn.lstm.bias_hh_l0", {4 * H}).data, need(sd, "rnn.lstm.bias_hh_l0_reverse", {4 * H}).data};
  const float* whh[2] = {need(sd, "rnn.lstm.weight_hh_l0", {4 * H, H}).data,
                         need(sd, "rnn.lstm.weight_hh_l0_reverse", {4 * H, H}).data};
  lstm_ih_ = make_pconv(KIND_GEMM, EFF_OUT, 8 * H, 1, M2S_DT_F32);
  lstm_ih_.cs_in = EFF_OUT;  // 208 = 13 x 16: valid fp32 K chunking without padding
  lstm_ih_.tpc = 1;
  lstm_ih_.kp = EFF_OUT;
  lstm_ih_.cs_out = 8 * H;
  lstm_ih_.n_pad = round_up(8 * H, 64);
  lstm_ih_.macs_per_row = 8.0 * H * EFF_OUT;
  pack_conv(arena_, M2S_DT_F32, lstm_ih_,
            [&](int, int n, int, int c) { return wih[n / (4 * H)][(size_t)(n % (4 * H)) * EFF_OUT + c]; },
            [&](int n) { return bih[n / (4 * H)][n % (4 * H)] + bhh[n / (4 * H)][n % (4 * H)]; });
  std::vector<float> wh((size_t)2 * 4 * H * H);
  std::memcpy(wh.data(), whh[0], sizeof(float) * 4 * H * H);
  std::memcpy(wh.data() + (size_t)4 * H * H, whh[1], sizeof(float) * 4 * H * H);
  whh_ = arena_.add_vec(wh);
  const float* hw = need(sd, "head.weight", {n_mels, H}).data;
  const float* hb = need(sd, "head.bias", {n_mels}).data;
  std::vector<float> wt((size_t)H * n_mels);
  for (int n = 0; n < n_mels; ++n)
    for (int k = 0; k < H; ++k) wt[(size_t)k * n_mels + n] = hw[(size_t)n * H + k];
  head_wt_ = arena_.add_vec(wt);
  head_b_ = arena_.add(hb, sizeof(float) * n_mels);

  arena_.upload(device);
  M2S_HIP(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
  *err_host_ = 0;
  M2S_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0));
  M2S_HIP(hipMalloc(&gsync_, std::max(lstm_small_sync_bytes(), lstm_x3g_sync_bytes())));
  for (auto& b : blocks_) {
    b.c1.resolve(arena_);
    if (b.type != 0) b.c2.resolve(arena_);
    if (b.type == 2) {
      b.se1.resolve(arena_);
      b.se2.resolve(arena_);
    }
  }
  lstm_ih_.resolve(arena_);
}

Acoustic::~Acoustic() {
  if (err_host_) (void)hipHostFree(err_host_);
  if (gsync_) (void)hipFree(gsync_);
}

unsigned Acoustic::take_async_error() { return __atomic_exchange_n(err_host_, 0u, __ATOMIC_ACQ_REL); }

void Acoustic::effnet_dims(int H, int W, size_t* io, size_t* mid, size_t* se) const {
  int oh, ow, ph, pw;
  same_pad(H, 3, 2, &oh, &ph);
  same_pad(W, 3, 2, &ow, &pw);
  size_t mio = (size_t)oh * ow * chan_stride(EFF_STEM), mmid = 0, mse = 0;
  for (const Block& b : blocks_) {
    int nh, nw;
    same_pad(oh, 3, b.stride, &nh, &ph);
    same_pad(ow, 3, b.stride, &nw, &pw);
    if (b.type == 1) mmid = std::max(mmid, (size_t)nh * nw * chan_stride(b.mid));
    if (b.type == 2) {
      mmid = std::max(mmid, (size_t)oh * ow * chan_stride(b.mid));
      mse = std::max(mse, (size_t)dw_pixel_blocks(nh, nw) * chan_stride(b.mid));
      if (b.stride == 2 && nh % 4 == 0) mse = std::max(mse, (size_t)ir_s2band_bands(nh) * chan_stride(b.mid));
    }
    mio = std::max(mio, (size_t)nh * nw * chan_stride(b.cout));
    oh = nh;
    ow = nw;
  }
  *io = mio;
  *mid = mmid;
  *se = mse;
}

size_t Acoustic::effnet_x8(int H, int W) const {
  if (dtype_ != M2S_DT_FP8 || (!f8_expand_ && !f8_er_)) return 0;
  int oh, ow, ph, pw;
  same_pad(H, 3, 2, &oh, &ph);
  same_pad(W, 3, 2, &ow, &pw);
  size_t mx = 0;
  for (const Block& b : blocks_) {
    int nh, nw;
    same_pad(oh, 3, b.stride, &nh, &ph);
    same_pad(ow, 3, b.stride, &nw, &pw);
    if (b.f8_pw && f8_expand_) mx = std::max(mx, (size_t)oh * ow * b.f8x_kp);  // the block input's map
    if (b.er8 && f8_er_) mx = std::max(mx, (size_t)nh * nw * 32);              // er8_fused x8 / y8 (N, H, W, 32)
    if (b.er8w && f8_er_) mx = std::max(mx, (size_t)nh * nw * 64);             // er8w_fused x8 / y8 (N, H, W, 64)
    oh = nh;
    ow = nw;
  }
  return round_up((int)mx, 256);
}

// Frames per CNN pass: `chunk`, or, where one pass fewer of at most chunk + chunk / 16 frames covers N, that
// (8 x 1000 frames: 4 passes of 2000 instead of 4 x 1920 + a 320-frame tail, which fills the persistent
// kernels' one-workgroup-per-CU grids for under two of their rounds).  Every pass is exact (per-frame work), so
// the split never changes a result (test_effnet_chunking_is_exact).
int Acoustic::pass_frames(int N) const {
  if (N <= chunk) return N;
  const int n = ceil_div(N, chunk), even = ceil_div(N, n - 1);
  return even <= chunk + chunk / 16 ? even : chunk;
}

size_t Acoustic::effnet_ws(int N, int H, int W) const {
  size_t io, mid, se;
  effnet_dims(H, W, &io, &mid, &se);
  const size_t es = act_bytes(dtype_);
  const size_t nc = pass_frames(N);
  Workspace ws(nullptr, 0);
  ws.take<char>(nc * io * es);
  ws.take<char>(nc * io * es);
  ws.take<char>(nc * mid * es);
  ws.take<char>(nc * mid * es);
  ws.take<float>(nc * se);
  ws.take<char>(nc * max_mid_cs_ * es);   // SE means
  ws.take<char>(nc * SE_RD_MAX * es);     // SE hidden (rd <= 64)
  ws.take<char>(nc * max_mid_cs_ * es);   // SE gates
  ws.take<char>(nc * effnet_x8(H, W));    // fp8: e4m3 expand operands, two buffers
  ws.take<char>(nc * effnet_x8(H, W));
  return ws.used();
}

size_t Acoustic::workspace_bytes(int B, int T, int H, int W) const {
  const size_t BT = (size_t)B * T;
  Workspace ws(nullptr, 0);
  ws.take<float>(BT * EFF_OUT);
  ws.take<char>(effnet_ws(B * T, H, W));
  ws.take<float>(BT * 8 * hidden_);
  ws.take<float>(2 * BT * hidden_);
  ws.take<float>((size_t)2 * B * hidden_);
  ws.take<char>(std::max({lstm_persistent_sync_bytes(), lstm_small_sync_bytes(), lstm_mid_sync_bytes(), lstm_x3_sync_bytes(), lstm_x3g_sync_bytes()}));
  return ws.used();
}

void Acoustic::effnet(const float* frames, int N, int H, int W, float* feats, int stop_after, float* probe,
                      int* probe_dims, Workspace& ws, hipStream_t s) {
  StageTag tag("cnn");
  if (dtype_ == M2S_DT_BF16 || dtype_ == M2S_DT_FP8)
    effnet_t<bf16_t>(frames, N, H, W, feats, stop_after, probe, probe_dims, ws, s);
  else if (dtype_ == M2S_DT_BF16X3)
    effnet_t<sp_t>(frames, N, H, W, feats, stop_after, probe, probe_dims, ws, s);
  else
    effnet_t<float>(frames, N, H, W, feats, stop_after, probe, probe_dims, ws, s);
}

template <typename T>
void Acoustic::effnet_t(const float* frames, int N, int H, int W, float* feats, int stop_after, float* probe,
                        int* probe_dims, Workspace& ws, hipStream_t s) {
  M2S_CHECK(N > 0 && H >= 32 && W >= 32, "effnet: bad input size");
  size_t io, mid, se;
  effnet_dims(H, W, &io, &mid, &se);
  const int nc_max = pass_frames(N);
  constexpr int R = Elem<T>::R;  // split fp32: hi + lo planes
  T* A = ws.take<T>((size_t)nc_max * io * R);
  T* Bb = ws.take<T>((size_t)nc_max * io * R);
  T* M = ws.take<T>((size_t)nc_max * mid * R);
  T* M2 = ws.take<T>((size_t)nc_max * mid * R);
  float* sums = ws.take<float>((size_t)nc_max * se);
  T* se_mean = ws.take<T>((size_t)nc_max * max_mid_cs_ * R);
  T* se_hid = ws.take<T>((size_t)nc_max * SE_RD_MAX * R);
  T* scale = ws.take<T>((size_t)nc_max * max_mid_cs_ * R);
  // fp8: e4m3 copies of IR block inputs (the e4m3 expand's operand), written by the previous block's SE GEMM
  // (y8) or converted (the expand reads no byte past cs_in of a row)
  const size_t x8b = effnet_x8(H, W);
  uint8_t* X8[2] = {x8b ? ws.take<uint8_t>((size_t)nc_max * x8b) : nullptr, x8b ? ws.take<uint8_t>((size_t)nc_max * x8b) : nullptr};

  for (int n0 = 0; n0 < N; n0 += nc_max) {
    const int nc = std::min(nc_max, N - n0);
    int oh, ow, pt, pl;
    same_pad(H, 3, 2, &oh, &pt);
    same_pad(W, 3, 2, &ow, &pl);
    // stem + blocks.0 (two 3x3 ConvBnAct at stride 1: 32 -> 16, 16 -> 16 + skip) in one kernel
    constexpr bool SPL = std::is_same<T, sp_t>::value;
    const bool front = ((std::is_same<T, bf16_t>::value && (dtype_ == M2S_DT_BF16 || dtype_ == M2S_DT_FP8)) || SPL) && stem_fused_ && !(probe && stop_after >= 0 && stop_after < 2) &&
                       blocks_.size() >= 2 && blocks_[0].type == 0 && blocks_[0].stride == 1 && !blocks_[0].skip &&
                       blocks_[0].cout == 16 && blocks_[0].c1.cs_in == 32 && blocks_[0].c1.kp == 288 &&
                       blocks_[1].type == 0 && blocks_[1].stride == 1 && blocks_[1].skip && blocks_[1].cout == 16 &&
                       blocks_[1].c1.cs_in == 16 && blocks_[1].c1.kp == 160 && chan_stride(16) == 16;
    T* cur = A;
    T* nxt = Bb;
    int cc = EFF_STEM;
    int bi = 0;
    if (front) {
      const double px = (double)nc * oh * ow;
      launch_stem_b0(frames + (size_t)n0 * H * W, nc, H, W, oh, ow, pt, pl, static_cast<const float*>(arena_.ptr(stem_w_)),
                     static_cast<const float*>(arena_.ptr(stem_b_)), blocks_[0].c1.w, blocks_[0].c1.b, blocks_[0].c1.kp,
                     blocks_[1].c1.w, blocks_[1].c1.b, blocks_[1].c1.kp, A, SPL,
                     2.0 * px * (EFF_STEM * 9 + 16 * 9 * 32 + 16 * 9 * 16), 4.0 * nc * H * W + (SPL ? 4.0 : 2.0) * px * 16, s);
      cc = 16;
      bi = 2;
    } else {
      ProfScope ps(std::is_same<T, bf16_t>::value ? std::string("stem32_kernel") : tname<T>("stem_kernel"), 2.0 * nc * oh * ow * EFF_STEM * 27, 4.0 * nc * H * W + (sizeof(T) * Elem<T>::R) * (double)nc * oh * ow * 32, s);
      launch_stem<T>(frames + (size_t)n0 * H * W, nc, H, W, oh, ow, pt, pl, static_cast<const float*>(arena_.ptr(stem_w_)),
                     static_cast<const float*>(arena_.ptr(stem_b_)), EFF_STEM, chan_stride(EFF_STEM), A, s);
    }
    auto tap = [&](int done) {
      if (stop_after == done && probe) {
        launch_unpad<T>(cur, (long)nc * oh * ow, cc, chan_stride(cc), probe + (size_t)n0 * oh * ow * cc, s);
        if (probe_dims) {
          probe_dims[0] = oh;
          probe_dims[1] = ow;
          probe_dims[2] = cc;
        }
        return true;
      }
      return false;
    };
    if (tap(bi)) continue;  // bi = 0, or 2 after the fused front
    bool stopped = false;
    uint8_t* cur8 = nullptr;  // fp8: the e4m3 copy of cur in X8[0] / X8[1], when one was written
    for (size_t k = front ? 2 : 0; k < blocks_.size(); ++k) {
      const Block& b = blocks_[k];
      uint8_t* next8 = nullptr;  // the e4m3 copy of this block's output, if its SE GEMM wrote one
      int nh, nw, qt, ql;
      same_pad(oh, 3, b.stride, &nh, &qt);
      same_pad(ow, 3, b.stride, &nw, &ql);
      // the next block takes an e4m3 expand operand (fp8 engines: stride-1 IR blocks, and the stride-2 one on
      // ir_pwdw_s2, whose input map is this block's nh x nw output)
      const bool want8 = X8[0] && f8_expand_ && k + 1 < blocks_.size() && blocks_[k + 1].f8_pw &&
                         (blocks_[k + 1].stride == 1 ||
                          (f8_s2_ && ir_fused_s2_supported(nh, nw, blocks_[k + 1].c1.cs_in, chan_stride(blocks_[k + 1].mid), false)));
      // the next block is an e4m3 EdgeResidual (er8_fused): this block also stores its output as e4m3 bytes
      // (er8w_fused, blocks.2.1/.2, always takes its e4m3 operand from the producer; M2S_ER8_X8=0 switches only
      // er8_fused to its in-kernel conversion)
      uint8_t* const er8_next = X8[0] && f8_er_ && k + 1 < blocks_.size() &&
                                        ((er8_x8_ && blocks_[k + 1].er8) || (f8_er2_ && blocks_[k + 1].er8w))
                                    ? (cur8 == X8[0] ? X8[1] : X8[0])
                                    : nullptr;
      auto a2d = [&](const PConv& pc, const void* x, void* y) {
        ConvArgs a = conv_args(pc);
        a.x = x;
        a.y = y;
        a.IH = oh;
        a.IW = ow;
        a.OH = nh;
        a.OW = nw;
        a.pad_t = qt;
        a.pad_l = ql;
        a.M = nc * nh * nw;
        return a;
      };
      if (b.type == 0) {
        ConvArgs a = a2d(b.c1, cur, nxt);
        a.act = ACT_SILU;
        a.res = b.skip ? cur : nullptr;
        run_conv<T>(a, b.c1, s);
      } else if (b.type == 1 && std::is_same<T, sp_t>::value && er_fused_ && b.er_sp &&
                 er_sp_supported(nh, nw, b.c1.cs_in, b.mid, chan_stride(b.cout))) {
        const double px = (double)nc * nh * nw;
        launch_er_sp(cur, nc, nh, nw, b.c1.cs_in, b.mid, chan_stride(b.cout), arena_.ptr(b.er_sp_w), b.c1.b, b.c2.b, nxt,
                     2.0 * px * b.mid * (9.0 * b.cin + b.cout), 4.0 * px * (b.c1.cs_in + chan_stride(b.cout)), s, er_mrg_);
      } else if (b.type == 1 && std::is_same<T, sp_t>::value && er_fused_ && b.ers_sp && b.stride == 2 &&
                 ers2_sp_supported(nh, nw, b.c1.cs_in, b.mid, chan_stride(b.cout))) {
        const double px = (double)nc * nh * nw;
        launch_ers2_sp(cur, nc, oh, ow, nh, nw, qt, ql, b.c1.cs_in, b.mid, chan_stride(b.cout), arena_.ptr(b.er_wexp),
                       b.c1.b, arena_.ptr(b.er_wpwl), b.c2.b, nxt, 2.0 * px * b.mid * (9.0 * b.cin + b.cout),
                       4.0 * ((double)nc * oh * ow * b.c1.cs_in + px * chan_stride(b.cout)), s);
      } else if (b.type == 1 && std::is_same<T, bf16_t>::value && er_fused_ && f8_er_ && b.er8 &&
                 er8_fused_supported(nh, nw, b.cin, b.mid, b.cout)) {
        const double px = (double)nc * nh * nw;
        uint8_t* y8 = cur8 && er8_next && er8_fused_supported(nh, nw, b.cout, b.mid, b.cout) ? er8_next : nullptr;
        launch_er8_fused(reinterpret_cast<const bf16_t*>(cur), nc, nh, nw, static_cast<const uint8_t*>(arena_.ptr(b.er8_wexp)),
                         static_cast<const float*>(arena_.ptr(b.er8_sexp)), b.c1.b,
                         static_cast<const uint8_t*>(arena_.ptr(b.er8_wpwl)), static_cast<const float*>(arena_.ptr(b.er8_spwl)),
                         b.c2.b, reinterpret_cast<bf16_t*>(nxt), 2.0 * px * b.mid * (9.0 * b.cin + b.cout),
                         2.0 * px * (2.0 * b.cin) + (3.0 * 8 * 2048 + 2 * 2048), s, cur8, y8);
        next8 = y8;
      } else if (b.type == 1 && std::is_same<T, bf16_t>::value && er_fused_ && b.er_frag &&
                 er_fused_supported(nh, nw, b.cin, b.mid, b.cout, b.c1.kp, b.c2.kp)) {
        const double px = (double)nc * nh * nw;
        launch_er_fused(reinterpret_cast<const bf16_t*>(cur), nc, nh, nw,
                        static_cast<const bf16_t*>(arena_.ptr(b.er_wexp)), b.c1.b,
                        static_cast<const bf16_t*>(arena_.ptr(b.er_wpwl)), b.c2.b, reinterpret_cast<bf16_t*>(nxt),
                        2.0 * px * b.mid * (9.0 * b.cin + b.cout), 2.0 * px * (2.0 * b.cin) + 2.0 * (9.0 * 32 * 128 + 128 * 32), s);
      } else if (b.type == 1 && std::is_same<T, bf16_t>::value && er_fused_ && f8_er_ && f8_er2_ && b.er8w && cur8 &&
                 er8w_fused_supported(nh, nw, b.c1.cs_in, b.mid, b.cout)) {
        const double px = (double)nc * nh * nw;
        uint8_t* y8 = er8_next && blocks_[k + 1].er8w ? er8_next : nullptr;
        launch_er8w_fused(reinterpret_cast<const bf16_t*>(cur), cur8, nc, nh, nw, static_cast<const uint8_t*>(arena_.ptr(b.er8w_w)),
                          static_cast<const float*>(arena_.ptr(b.er8w_sexp)), b.c1.b,
                          static_cast<const float*>(arena_.ptr(b.er8w_spwl)), b.c2.b, reinterpret_cast<bf16_t*>(nxt), y8,
                          2.0 * px * b.mid * (9.0 * b.cin + b.cout),
                          // e4m3 input + bf16 shortcut + bf16 output (+ its e4m3 copy) + the weights once
                          px * (b.cin + 2.0 * b.cin + 2.0 * b.cout + (y8 ? b.cout : 0.0)) + (9.0 * b.cin + b.cout) * b.mid, s);
        next8 = y8;
      } else if (b.type == 1 && std::is_same<T, bf16_t>::value && er_fused_ && b.er_frag &&
                 er2_fused_supported(nh, nw, b.c1.cs_in, b.mid, b.cout, b.c1.kp, b.c2.kp)) {
        const double px = (double)nc * nh * nw;
        launch_er2_fused(reinterpret_cast<const bf16_t*>(cur), nc, nh, nw, static_cast<const bf16_t*>(arena_.ptr(b.er_wexp)),
                         b.c1.b, b.c2.b, reinterpret_cast<bf16_t*>(nxt), 2.0 * px * b.mid * (9.0 * b.cin + b.cout),
                         2.0 * px * (2.0 * b.c1.cs_in) + 2.0 * er2_stage_elems(), s);
      } else if (b.type == 1 && std::is_same<T, bf16_t>::value && er_fused_ && b.er_frag && b.stride == 2 &&
                 ers2_fused_supported(nh, nw, b.c1.cs_in, b.mid, chan_stride(b.cout), b.c1.kp, b.c2.kp)) {
        const double px = (double)nc * nh * nw;
        // fp8: an e4m3 copy of the output for an er8_fused next block (the copy is (N, OH, OW, cs_out) bytes)
        uint8_t* y8 = er8_next && ((chan_stride(b.cout) == 32 && blocks_[k + 1].er8 && er8_fused_supported(nh, nw, 32, 128, 32)) ||
                                   (chan_stride(b.cout) == 64 && blocks_[k + 1].er8w && er8w_fused_supported(nh, nw, 64, 224, b.cout)))
                          ? er8_next
                          : nullptr;
        launch_ers2_fused(reinterpret_cast<const bf16_t*>(cur), nc, oh, ow, nh, nw, qt, ql, b.c1.cs_in, b.mid,
                          chan_stride(b.cout), static_cast<const bf16_t*>(arena_.ptr(b.er_wexp)), b.c1.b,
                          static_cast<const bf16_t*>(arena_.ptr(b.er_wpwl)), b.c2.b, reinterpret_cast<bf16_t*>(nxt),
                          2.0 * px * b.mid * (9.0 * b.cin + b.cout),
                          2.0 * ((double)nc * oh * ow * b.c1.cs_in + px * chan_stride(b.cout)) + (y8 ? px * 32 : 0.0), s, y8);
        next8 = y8;
      } else if (b.type == 1) {
        ConvArgs a = a2d(b.c1, cur, M);
        a.act = ACT_SILU;
        run_conv<T>(a, b.c1, s);
        ConvArgs p = conv_args(b.c2);
        p.x = M;
        p.y = nxt;
        p.M = nc * nh * nw;
        p.OH = nh * nw;
        p.res = b.skip ? cur : nullptr;
        run_conv<T>(p, b.c2, s);
      } else {
        const int cs = chan_stride(b.mid);
        constexpr bool SPL = std::is_same<T, sp_t>::value;
        const bool FUSABLE = (std::is_same<T, bf16_t>::value && (dtype_ == M2S_DT_BF16 || dtype_ == M2S_DT_FP8)) || SPL;
        bool f8 = false;  // fp8 engine: e4m3 depthwise output -> the e4m3 SE GEMM
        // bf16 feeds the fused kernel bf16 depthwise taps (dword halves), split fp32 the fp32 taps
        const void* wdw = arena_.ptr(SPL ? b.dw_w : b.dw_w2);
        const bool big = nc >= irws_min_;  // persistent ir_ws only where its one-image workgroups fill the chip
        // the SE-gated conv_pwl runs on se_ws (below): then ir_ws hands it the expanded map as plain fp32 rows
        // (one 16-byte store per 4 channels, no split; se_ws gates the fp32 value before its one split)
        const bool sews = SPL && se_ws_ && se_ws_supported(nh * nw, cs, chan_stride(b.cout)) &&
                          // se_ws runs one persistent workgroup per tile (256 rows; 128 at 8 x 8) up to one per CU:
                          // below a full round of tiles the split-K conv_gemm SE GEMM fills the chip instead
                          ceil_div(nc * nh * nw, nh * nw == 64 ? 128 : 256) >= sews_min_cus_ * device_cus();
        bool mid_f32 = false;
        if (SPL && b.stride == 1 && ir_fused_ && ir_ws_ && big && ir_ws_supported(nh, nw, b.c1.cs_in, b.c1.kp, cs)) {
          const double P = (double)nh * nw;
          launch_ir_ws(cur, nc, nh, nw, b.c1.cs_in, b.c1.kp, cs, b.c1.w, b.c1.b, static_cast<const float*>(arena_.ptr(b.dw_w)),
                       static_cast<const float*>(arena_.ptr(b.dw_b)), M2, se_mean, 2.0 * nc * P * b.mid * (b.c1.cin + 9),
                       // algorithmic bytes on the real channel counts (split fp32: 4 B an element): compulsory = the
                       // block input, the split expand weights, taps and biases, the SE means out; the depthwise output
                       // map is a spill (written here only for the SE-gated conv_pwl to read back: m2s.h spill_bytes)
                       4.0 * nc * P * b.c1.cin + 4.0 * b.mid * (b.c1.cin + 11.0) + 4.0 * nc * b.mid, s, ws_report(), 1, 0, 0,
                       0, 0, 4.0 * nc * P * b.mid, mid_f32 = sews && irws_f32_);
        } else if (FUSABLE && b.stride == 1 && ir_fused_ && ir_fused_supported(nh, nw, b.c1.cs_in, cs, SPL)) {
          const double P = (double)nh * nw, es = SPL ? 4.0 : 2.0;
          f8 = b.f8_pwl && se_gemm_f8_supported(nh * nw, cs, chan_stride(b.cout));
          const bool f8x = f8 && f8_expand_ && b.f8_pw && X8[0];  // the expand on e4m3 (x8 of the block input)
          if (f8x && !cur8) {  // no e4m3 producer wrote this input: convert it
            cur8 = X8[0];
            launch_rows_e4m3(cur, (long)nc * nh * nw, b.c1.cs_in, cur8, b.f8x_kp, s);
          }
          launch_ir_pwdw(cur, nc, b.c1.cs_in, b.c1.kp, b.c1.w, b.c1.b, wdw, static_cast<const float*>(arena_.ptr(b.dw_b)),
                         nh, nw, cs, M2, se_mean, SPL, 2.0 * nc * P * b.mid * (b.c1.cin + 9),
                         nc * P * ((f8x ? 1.0 : es) * b.c1.cin + (f8 ? 1.0 : es) * b.mid), s, f8, f8x ? cur8 : nullptr,
                         f8x ? arena_.ptr(b.f8x_w) : nullptr, f8x ? static_cast<const float*>(arena_.ptr(b.f8x_s)) : nullptr,
                         b.f8x_kp);
        } else if (SPL && b.stride == 2 && ir_fused_ && ir_ws_ && ir_ws_s2_ && big &&
                   ir_ws_s2_supported(oh, ow, b.c1.cs_in, b.c1.kp, cs, nh, nw, qt, ql)) {
          const double Pi = (double)oh * ow, Po = (double)nh * nw;
          launch_ir_ws(cur, nc, oh, ow, b.c1.cs_in, b.c1.kp, cs, b.c1.w, b.c1.b, static_cast<const float*>(arena_.ptr(b.dw_w)),
                       static_cast<const float*>(arena_.ptr(b.dw_b)), M2, se_mean, 2.0 * nc * b.mid * (Pi * b.c1.cin + Po * 9),
                       4.0 * nc * Pi * b.c1.cin + 4.0 * b.mid * (b.c1.cin + 11.0) + 4.0 * nc * b.mid, s, ws_report(), 2, nh, nw,
                       qt, ql, 4.0 * nc * Po * b.mid, mid_f32 = sews && irws_f32_);
        } else if (FUSABLE && b.stride == 2 && ir_fused_ && ir_fused_s2_supported(oh, ow, b.c1.cs_in, cs, SPL) &&
                   nh * nw <= 64) {
          const double Pi = (double)oh * ow, Po = (double)nh * nw, es = SPL ? 4.0 : 2.0;
          // fp8 engines (blocks.5.0): e4m3 depthwise output for the e4m3 SE GEMM, the expand on e4m3 as for stride 1
          f8 = f8_s2_ && b.f8_pwl && se_gemm_f8_supported(nh * nw, cs, chan_stride(b.cout));
          const bool f8x = f8 && f8_expand_ && b.f8_pw && X8[0];
          if (f8x && !cur8) {  // no e4m3 producer wrote this input: convert it
            cur8 = X8[0];
            launch_rows_e4m3(cur, (long)nc * oh * ow, b.c1.cs_in, cur8, b.f8x_kp, s);
          }
          launch_ir_pwdw_s2(cur, nc, b.c1.cs_in, b.c1.kp, b.c1.w, b.c1.b, wdw, static_cast<const float*>(arena_.ptr(b.dw_b)),
                            oh, ow, nh, nw, qt, ql, cs, M2, se_mean, SPL, 2.0 * nc * b.mid * (Pi * b.c1.cin + Po * 9),
                            nc * ((f8x ? 1.0 : es) * Pi * b.c1.cin + (f8 ? 1.0 : es) * Po * b.mid), s, f8,
                            f8x ? cur8 : nullptr, f8x ? arena_.ptr(b.f8x_w) : nullptr,
                            f8x ? static_cast<const float*>(arena_.ptr(b.f8x_s)) : nullptr, b.f8x_kp);
        } else if (FUSABLE && b.stride == 2 && ir_fused_ && ir_s2band_ &&
                   ir_s2band_supported(oh, ow, nh, nw, b.c1.cs_in, b.c1.kp, cs)) {
          const double Pi = (double)oh * ow, Po = (double)nh * nw, es = SPL ? 4.0 : 2.0;
          // fp8 engines (blocks.3.0): e4m3 depthwise output for the e4m3 SE GEMM (the expand stays bf16)
          f8 = f8_s2_ && b.f8_pwl && se_gemm_f8_supported(nh * nw, cs, chan_stride(b.cout));
          launch_ir_s2band(cur, nc, oh, ow, b.c1.cs_in, b.c1.kp, b.c1.w, b.c1.b, static_cast<const float*>(arena_.ptr(b.dw_w)),
                           static_cast<const float*>(arena_.ptr(b.dw_b)), nh, nw, qt, ql, cs, M2, sums, SPL,
                           2.0 * nc * b.mid * (Pi * 1.125 * b.c1.cin + Po * 9),
                           nc * (es * Pi * b.c1.cs_in + (f8 ? 1.0 : es) * Po * cs), s, f8);
          ProfScope ps(tname<T>("se_mean_kernel"), 0.0, 4.0 * nc * cs * ir_s2band_bands(nh) + es * nc * cs, s);
          launch_se_mean<T>(sums, nc, ir_s2band_bands(nh), cs, 1.0f / (float)(nh * nw), se_mean, s);
        } else {
        ConvArgs e = conv_args(b.c1);
        e.x = cur;
        e.y = M;
        e.M = nc * oh * ow;
        e.OH = oh * ow;
        e.act = ACT_SILU;
        run_conv<T>(e, b.c1, s);
        {
          ProfScope ps(b.stride == 2 ? tname<T>("dwconv_kernel", ", 2") : tname<T>("dwconv_kernel", ", 1"), 2.0 * nc * nh * nw * b.mid * 9,
                       (sizeof(T) * Elem<T>::R) * (double)nc * (oh * ow + nh * nw) * b.mid, s);
          launch_dwconv<T>(M, nc, oh, ow, nh, nw, b.stride, qt, ql, b.mid, cs,
                           static_cast<const float*>(arena_.ptr(b.dw_w)), static_cast<const float*>(arena_.ptr(b.dw_b)),
                           M2, sums, s);
        }
        {
          ProfScope ps(tname<T>("se_mean_kernel"), 0.0, 4.0 * nc * cs * dw_pixel_blocks(nh, nw) + (sizeof(T) * Elem<T>::R) * (double)nc * cs, s);
          launch_se_mean<T>(sums, nc, dw_pixel_blocks(nh, nw), cs, 1.0f / (float)(nh * nw), se_mean, s);
        }
        }
        if (FUSABLE && se_fused_ && se_excite_supported(b.rd, b.se2.kp, cs)) {
          launch_se_excite(se_mean, nc, b.mid, cs, b.se1.w, b.se1.kp, b.se1.b, b.rd, b.se2.w, b.se2.kp, b.se2.b, scale,
                           SPL, s);
        } else {
        ConvArgs r1 = conv_args(b.se1);  // conv_reduce + SiLU, all images of the chunk at once
        r1.x = se_mean;
        r1.y = se_hid;
        r1.M = nc;
        r1.act = ACT_SILU;
        run_conv<T>(r1, b.se1, s);
        ConvArgs r2 = conv_args(b.se2);  // conv_expand + sigmoid -> per-(image, channel) gates
        r2.x = se_hid;
        r2.y = scale;
        r2.M = nc;
        r2.act = ACT_SIGMOID;
        run_conv<T>(r2, b.se2, s);
        }
        // fp8: an e4m3 copy of the output for the next block's expand, into the buffer cur8 does not hold
        const int ld8 = want8 ? blocks_[k + 1].f8x_kp : 0;
        if (f8 && want8 && se_y8_) next8 = cur8 == X8[0] ? X8[1] : X8[0];
        if (f8 && se_ws_ && se_ws_f8_supported(nh * nw, cs, chan_stride(b.cout))) {
          const double rows = (double)nc * nh * nw;
          launch_se_ws_f8(M2, nc * nh * nw, nh * nw, cs, arena_.ptr(b.f8_w), b.f8_kp, b.f8_npad,
                          static_cast<const float*>(arena_.ptr(b.f8_s)), static_cast<const float*>(arena_.ptr(b.f8_b)),
                          scale, b.skip ? cur : nullptr, nxt, chan_stride(b.cout), s, 2.0 * rows * b.mid * b.cout,
                          rows * b.mid + 2.0 * rows * b.cout * (b.skip ? 2.0 : 1.0) + (double)b.cout * b.mid + 2.0 * nc * b.mid +
                              (next8 ? rows * b.cout : 0.0),
                          next8, ld8, ws_report());
        } else if (f8) {
          const double rows = (double)nc * nh * nw, co = chan_stride(b.cout);
          launch_se_gemm_f8(M2, nc * nh * nw, nh * nw, cs, arena_.ptr(b.f8_w), b.f8_kp, b.f8_npad,
                            static_cast<const float*>(arena_.ptr(b.f8_s)), static_cast<const float*>(arena_.ptr(b.f8_b)),
                            scale, b.skip ? cur : nullptr, nxt, chan_stride(b.cout), s, 2.0 * rows * b.mid * b.cout,
                            rows * cs + 2.0 * rows * co * (b.skip ? 2.0 : 1.0) + (double)b.f8_npad * b.f8_kp +
                                2.0 * nc * cs + (next8 ? rows * ld8 : 0.0),
                            next8, ld8);
        } else if (sews) {
          const double rows = (double)nc * nh * nw;
          launch_se_ws(M2, nc * nh * nw, nh * nw, cs, b.c2.w, b.c2.n_pad, b.c2.b, scale, b.skip ? cur : nullptr, nxt,
                       chan_stride(b.cout), s, 2.0 * rows * b.mid * b.cout,
                       4.0 * rows * b.mid + 4.0 * rows * b.cout * (b.skip ? 2.0 : 1.0) + 4.0 * b.cout * b.mid + 4.0 * nc * b.mid,
                       ws_report(), mid_f32);
        } else if (SPL && se_sp_ && se_gemm_sp_supported(nh * nw, cs, chan_stride(b.cout))) {
          const double rows = (double)nc * nh * nw, co = chan_stride(b.cout);
          launch_se_gemm_sp(M2, nc * nh * nw, nh * nw, cs, b.c2.w, b.c2.n_pad, b.c2.b, scale, b.skip ? cur : nullptr, nxt,
                            chan_stride(b.cout), s, 2.0 * rows * b.mid * b.cout,
                            4.0 * rows * cs + 4.0 * rows * co * (b.skip ? 2.0 : 1.0) + 4.0 * b.c2.n_pad * b.c2.kp +
                                4.0 * nc * cs);
        } else {
        ConvArgs p = conv_args(b.c2);
        p.x = M2;
        p.y = nxt;
        p.M = nc * nh * nw;
        p.OH = nh * nw;
        p.in_xform = IN_SE_SCALE;
        p.in_scale = scale;
        p.res = b.skip ? cur : nullptr;
        run_conv<T>(p, b.c2, s);
        }
      }
      std::swap(cur, nxt);
      cur8 = next8;
      oh = nh;
      ow = nw;
      cc = b.cout;
      ++bi;
      if (tap(bi)) {
        stopped = true;
        break;
      }
    }
    if (stopped || !feats) continue;
    ProfScope ps(tname<T>("gap_kernel"), (double)nc * oh * ow * cc, (sizeof(T) * Elem<T>::R) * (double)nc * oh * ow * cc, s);
    launch_gap<T>(cur, nc, oh * ow, cc, chan_stride(cc), feats + (size_t)n0 * EFF_OUT, s);
  }
}

void Acoustic::bilstm(const float* feats, int B, int T, float* y, float* mel_norm, Workspace& ws, hipStream_t s) {
  M2S_CHECK(B > 0 && T > 0, "bilstm: empty input");
  const int H = hidden_;
  const size_t BT = (size_t)B * T;
  float* pre = ws.take<float>(BT * 8 * H);
  float* hs = ws.take<float>(2 * BT * H);
  float* cst = ws.take<float>((size_t)2 * B * H);
  StageTag tag("bilstm");
  ConvArgs a = conv_args(lstm_ih_);
  a.x = feats;
  a.y = pre;
  a.M = (int)BT;
  // small passes (<= 64 frames): the four waves of a row tile split K (one 30-frame clip: 20 -> 12 us); larger passes
  // keep four row groups a workgroup sharing the weight tile (K split there: the 1920-frame step's projection
  // 0.13 ms slower).  The K summation order therefore differs between the two size classes (fp32 rounding only).
  a.kwave = BT <= 64 ? 1 : 0;
  run_conv<float>(a, lstm_ih_, s);
  void* sync = ws.take<char>(std::max({lstm_persistent_sync_bytes(), lstm_small_sync_bytes(), lstm_mid_sync_bytes(), lstm_x3_sync_bytes(), lstm_x3g_sync_bytes()}));
  if (lstm_persistent_ && lstm_small_supported(B, H)) {
    ProfScope ps("lstm_small_kernel", 2.0 * 2 * B * 4.0 * H * H * (T - 1), 4.0 * 2 * 4 * H * H + 4.0 * BT * (8.0 * H + 2.0 * H), s);
    launch_lstm_small(pre, static_cast<const float*>(arena_.ptr(whh_)), hs, B, T, H, gsync_, lstm_spin_max_, err_dev_, s,
                      &gsync_epoch_);
  } else if (lstm_persistent_ && lstm_x3_ && lstm_x3g_ && dtype_ != M2S_DT_F32 && lstm_x3g_supported(B, H)) {
    // 5..16 sequences (configs[4]'s 8 clips a GPU): the granule hand-off (lstm_persistent.hip lstm_x3g_kernel)
    ProfScope ps("lstm_x3g_kernel", 3.0 * 2 * B * 4.0 * H * H * (T - 1), 4.0 * 2 * 4 * H * H + 4.0 * BT * (8.0 * H + 2.0 * H), s);
    launch_lstm_x3g(pre, static_cast<const float*>(arena_.ptr(whh_)), hs, B, T, H, gsync_, lstm_spin_max_, err_dev_, s,
                    &gsync_epoch_);
  } else if (lstm_persistent_ && lstm_x3_ && dtype_ != M2S_DT_F32 && lstm_persistent_supported(H)) {
    // split engines above the small-batch kernel: 4.1 / 5.2 / 9.9 us per step at B = 8 / 16 / 64 against
    // lstm_mid's 7.2 / 11.9 and the f32 counter-barrier kernel's 24 (gpurun_out lstm2, lstm3_x3small)
    ProfScope ps("lstm_x3_kernel", 3.0 * 2 * B * 4.0 * H * H * (T - 1), 4.0 * 2 * 4 * H * H + 4.0 * BT * (8.0 * H + 2.0 * H), s);
    launch_lstm_x3(pre, static_cast<const float*>(arena_.ptr(whh_)), hs, B, T, H, sync, lstm_spin_max_, err_dev_, s);
  } else if (lstm_persistent_ && lstm_mid_ && lstm_mid_supported(B, H)) {
    ProfScope ps("lstm_mid_kernel", 2.0 * 2 * B * 4.0 * H * H * (T - 1), 4.0 * 2 * 4 * H * H + 4.0 * BT * (8.0 * H + 2.0 * H), s);
    launch_lstm_mid(pre, static_cast<const float*>(arena_.ptr(whh_)), hs, B, T, H, sync, lstm_spin_max_, err_dev_, s);
  } else if (lstm_persistent_ && lstm_persistent_supported(H)) {
    // algorithmic bytes: W_hh of both directions once, gate pre-activations in, h out
    ProfScope ps("lstm_persistent_kernel", 2.0 * 2 * B * 4.0 * H * H * (T - 1),
                 4.0 * 2 * 4 * H * H + 4.0 * BT * (8.0 * H + 2.0 * H), s);
    launch_lstm_persistent(pre, static_cast<const float*>(arena_.ptr(whh_)), hs, B, T, H, sync, lstm_spin_max_,
                           err_dev_, s);
  } else {
    for (int st = 0; st < T; ++st) {
      ProfScope ps("lstm_step_kernel", 2.0 * 2 * B * 4.0 * H * H, 4.0 * 2 * 4 * H * H, s);
      launch_lstm_step(pre, static_cast<const float*>(arena_.ptr(whh_)), hs, cst, B, T, H, st, s);
    }
  }
  if (mel_norm) {
    StageTag head("head");
    ProfScope ps("mel_head_kernel", 2.0 * BT * H * n_mels_, 4.0 * BT * (2 * H + n_mels_), s);
    launch_mel_head(hs, (int)BT, H, static_cast<const float*>(arena_.ptr(head_wt_)),
                    static_cast<const float*>(arena_.ptr(head_b_)), n_mels_, mel_norm, s);
  }
  if (y) launch_add2(hs, hs + BT * H, y, (long)(BT * H), s);
}

void Acoustic::forward(const float* frames, int B, int T, int H, int W, float* mel_norm, void* wsp, size_t wsb,
                       hipStream_t s) {
  M2S_CHECK(B > 0 && T > 0, "acoustic: empty input");
  Workspace ws(wsp, wsb);
  float* feats = ws.take<float>((size_t)B * T * EFF_OUT);
  effnet(frames, B * T, H, W, feats, -1, nullptr, nullptr, ws, s);
  bilstm(feats, B, T, nullptr, mel_norm, ws, s);
}

// ------------------------------------------------------------------------------------------
// Vocoder
static std::vector<float> fold_wn(const StateDict& sd, const std::string& p, std::vector<int64_t> shape) {
  auto it = sd.find(p + ".weight");
  if (it != sd.end()) {
    const HostTensor& t = need(sd, p + ".weight", shape);
    return std::vector<float>(t.data, t.data + t.numel());
  }
  std::vector<int64_t> gs(shape.size(), 1);
  gs[0] = shape[0];
  const HostTensor& g = need(sd, p + ".weight_g", gs);
  const HostTensor& v = need(sd, p + ".weight_v", shape);
  const size_t inner = v.numel() / shape[0];
  std::vector<float> w(v.numel());
  for (int64_t i = 0; i < shape[0]; ++i) {
    double acc = 0.0;
    for (size_t j = 0; j < inner; ++j) acc += (double)v.data[i * inner + j] * v.data[i * inner + j];
    const float sc = g.data[i] / (float)std::sqrt(acc);
    for (size_t j = 0; j < inner; ++j) w[i * inner + j] = v.data[i * inner + j] * sc;
  }
  return w;
}

Vocoder::Vocoder(const StateDict& sd, const m2s_hifigan_h& h, int dtype, int device)
    : h_(h), dtype_(dtype), device_(device) {
  M2S_CHECK(dtype == M2S_DT_F32 || dtype == M2S_DT_BF16 || dtype == M2S_DT_BF16X3 || dtype == M2S_DT_FP8, "bad dtype");
  M2S_CHECK(h.resblock == 1 || h.resblock == 2, "resblock must be 1 or 2");
  // fp8 engines: e4m3 resblock (MRF) convs at C = 64 / 128 / 256; conv_pre, the upsamplers and the fused
  // C = 32 ResBlock1 kernel stay bf16
  const int io_dt = dtype == M2S_DT_FP8 ? M2S_DT_BF16 : dtype;
  if (const char* e = std::getenv("M2S_MRF_FUSED")) mrf_fused_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_MRF_BATCH")) mrf_batch_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_MRF_HALO")) mrf_halo_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_F8_MRF64")) f8_mrf64_ = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("M2S_F8_MRF32")) f8_mrf32_ = std::strcmp(e, "0") != 0;
  M2S_CHECK(h.n_up >= 1 && h.n_up <= 8 && h.n_kernels >= 1 && h.n_kernels <= 8, "bad generator config");
  const int c0 = h.upsample_initial_channel;
  {  // conv_pre: Conv1d(num_mels, c0, 7), no weight norm (models.py:94)
    const HostTensor& w = need(sd, "conv_pre.weight", {c0, h.num_mels, 7});
    const HostTensor& b = need(sd, "conv_pre.bias", {c0});
    pre_ = make_pconv(KIND_CONV1D, h.num_mels, c0, 7, io_dt);
    pre_.ks = 7;
    pre_.pad_left = 0;  // F.pad(x, (0, 6)): look-ahead of 6 frames, zeros past the end
    pre_.macs_per_row = (double)c0 * h.num_mels * 7;
    const int ci = h.num_mels;
    pack_conv(arena_, io_dt, pre_, [&](int, int n, int t, int c) { return w.data[((size_t)n * ci + c) * 7 + t]; },
              [&](int n) { return b.data[n]; });
  }
  hop_ = 1;
  for (int i = 0; i < h.n_up; ++i) {
    const int u = h.upsample_rates[i], k = h.upsample_kernel_sizes[i];
    const int ci = c0 >> i, co = c0 >> (i + 1);
    M2S_CHECK(co >= 4, "generator too narrow");
    // ConvTranspose1d(k, u, padding (k-u)/2) (models.py:98-101) gives L*u outputs only when k - u is
    // even and non-negative; the polyphase packing and conv_post's look-ahead assume exactly L*u
    M2S_CHECK(u >= 1 && k >= u && (k - u) % 2 == 0,
              "upsample kernel " + std::to_string(k) + " / rate " + std::to_string(u) +
                  ": k - u must be even and >= 0 (output length L*u)");
    hop_ *= u;
    const std::string p = "ups." + std::to_string(i);
    std::vector<float> w = fold_wn(sd, p, {ci, co, k});  // ConvTranspose1d weight (in, out, k)
    const HostTensor& b = need(sd, p + ".bias", {co});
    PConv pc = make_pconv(KIND_CONVT, ci, co, (k + u - 1) / u, io_dt);
    pc.phases = u;
    pc.ct_u = u;
    pc.ct_pad = (k - u) / 2;
    pc.ct_k = k;
    pc.macs_per_row = (double)ci * co * k / u;  // per output position, averaged over phases
    const int pad = pc.ct_pad;
    pack_conv(arena_, io_dt, pc,
              [&](int ph, int n, int t, int c) {
                const int j = (ph + pad) % u + t * u;  // tap t of phase ph uses kernel index j
                return j < k ? w[((size_t)c * co + n) * k + j] : 0.f;
              },
              [&](int n) { return b.data[n]; });
    ups_.push_back(pc);
    for (int j = 0; j < h.n_kernels; ++j) {
      RB rb;
      rb.k = h.resblock_kernel_sizes[j];
      const int kk = rb.k;
      M2S_CHECK(h.n_dilations[j] >= 1 && h.n_dilations[j] <= 8, "resblock dilations: 1..8 per kernel size");
      for (int d = 0; d < h.n_dilations[j]; ++d) rb.dil.push_back(h.resblock_dilation_sizes[j][d]);
      const std::string q = "resblocks." + std::to_string(i * h.n_kernels + j);
      auto mk = [&](const std::string& name, int dil) {
        std::vector<float> wv = fold_wn(sd, name, {co, co, kk});
        const HostTensor& bv = need(sd, name + ".bias", {co});
        PConv c = make_pconv(KIND_CONV1D, co, co, kk, dtype);
        c.ks = kk;
        c.dil = dil;
        c.pad_left = (kk - 1) * dil;  // get_padding(k, d) = k*d - d, then truncation: causal (utils.py:33-34)
        c.macs_per_row = (double)co * co * kk;
        pack_conv(arena_, dtype, c, [&](int, int n, int t, int cc) { return wv[((size_t)n * co + cc) * kk + t]; },
                  [&](int n) { return bv.data[n]; });
        return c;
      };
      const bool fsplit = dtype == M2S_DT_BF16X3;
      // (fp8 engines: the fused bf16 ResBlock1 at C = 32 / 64, e4m3 convs at the wider stages)
      const bool frag = (dtype == M2S_DT_BF16 || dtype == M2S_DT_FP8 || fsplit) && h.resblock == 1 &&
                        rb1_fused_supported(co, chan_stride(co), kk, rb.dil.data(), (int)rb.dil.size(), kk * co, fsplit);
      auto mk_frag = [&](const std::string& name) {  // fragment order of mrf_fused.hip
        std::vector<float> wv = fold_wn(sd, name, {co, co, kk});
        const int taps = rb1_frag_taps(co, kk, fsplit), nt16 = co / 16, k32 = co / 32, hr = fsplit ? 2 : 1;
        std::vector<uint16_t> f((size_t)taps * hr * nt16 * k32 * 64 * 8);
        size_t o = 0;
        for (int t = 0; t < taps; ++t)
          for (int half = 0; half < hr; ++half)
            for (int nt = 0; nt < nt16; ++nt)
              for (int kc = 0; kc < k32; ++kc)
                for (int ln = 0; ln < 64; ++ln)
                  for (int e = 0; e < 8; ++e) {
                    const int n = nt * 16 + (ln & 15), c = kc * 32 + 8 * (ln >> 4) + e;
                    const float w = t < kk ? wv[((size_t)n * co + c) * kk + t] : 0.f;
                    if (fsplit) {
                      uint16_t hi, lo;
                      split_host(w, &hi, &lo);
                      f[o++] = half ? lo : hi;
                    } else {
                      f[o++] = f2bf_host(w);
                    }
                  }
        return arena_.add_vec(f);
      };
      // fp8: the C = 128 / 256 (and, f8_mrf64_, C = 64) resblock convs as e4m3 bytes for conv1d_f8 (K = 128
      // block-scaled MFMA; C = 64: two taps a K step)
      const bool q8 = dtype == M2S_DT_FP8 && h.resblock == 1 &&
                      ((co >= 128 && !frag) || (co == 64 && f8_mrf64_) || (co == 32 && f8_mrf32_)) &&
                      conv1d_f8_supported(co, kk);
      auto mk_q8 = [&](const std::string& name) {
        std::vector<float> wv = fold_wn(sd, name, {co, co, kk});
        const HostTensor& bv = need(sd, name + ".bias", {co});
        RB::F8 f;
        pack_gemm_f8(
            arena_, kk * co, co, co, round_up(kk * co, 128),
            [&](int n, int kx) { return wv[((size_t)n * co + kx % co) * kk + kx / co]; },  // K = tap-major t C + c
            [&](int n) { return bv.data[n]; }, &f.w, &f.s, &f.b);
        return f;
      };
      bool halo = fsplit && h.resblock == 1 && !frag;
      for (size_t d = 0; d < rb.dil.size(); ++d) halo = halo && conv1d_halo_sp_supported(co, chan_stride(co), kk, rb.dil[d]);
      auto mk_halo = [&](const std::string& name) {  // fragment order of conv1d_halo.hip
        std::vector<float> wv = fold_wn(sd, name, {co, co, kk});
        std::vector<uint16_t> f(conv1d_halo_frag_elems(co, kk));
        size_t o = 0;
        for (int t = 0; t < kk; ++t)
          for (int kc = 0; kc < co / 32; ++kc)
            for (int half = 0; half < 2; ++half)
              for (int nt = 0; nt < co / 16; ++nt)
                for (int ln = 0; ln < 64; ++ln)
                  for (int e = 0; e < 8; ++e) {
                    const int n = nt * 16 + (ln & 15), c = kc * 32 + 8 * (ln >> 4) + e;
                    uint16_t hi, lo;
                    split_host(wv[((size_t)n * co + c) * kk + t], &hi, &lo);
                    f[o++] = half ? lo : hi;
                  }
        return arena_.add_vec(f);
      };
      for (size_t d = 0; d < rb.dil.size(); ++d) {
        if (h.resblock == 1) {
          rb.c1.push_back(mk(q + ".convs1." + std::to_string(d), rb.dil[d]));
          rb.c2.push_back(mk(q + ".convs2." + std::to_string(d), 1));
          if (frag) {
            rb.f1_off.push_back(mk_frag(q + ".convs1." + std::to_string(d)));
            rb.f2_off.push_back(mk_frag(q + ".convs2." + std::to_string(d)));
          }
          if (halo) {
            rb.h1_off.push_back(mk_halo(q + ".convs1." + std::to_string(d)));
            rb.h2_off.push_back(mk_halo(q + ".convs2." + std::to_string(d)));
          }
          if (q8) {
            rb.q1.push_back(mk_q8(q + ".convs1." + std::to_string(d)));
            rb.q2.push_back(mk_q8(q + ".convs2." + std::to_string(d)));
          }
        } else {
          rb.c1.push_back(mk(q + ".convs." + std::to_string(d), rb.dil[d]));
        }
      }
      rbs_.push_back(rb);
    }
  }
  post_c_ = c0 >> h.n_up;
  {
    std::vector<float> w = fold_wn(sd, "conv_post", {1, post_c_, 7});
    const HostTensor& b = need(sd, "conv_post.bias", {1});
    std::vector<float> wt((size_t)7 * post_c_);
    for (int c = 0; c < post_c_; ++c)
      for (int t = 0; t < 7; ++t) wt[(size_t)t * post_c_ + c] = w[(size_t)c * 7 + t];
    post_w_ = arena_.add_vec(wt);
    post_b_ = b.data[0];
  }
  arena_.upload(device);
  pre_.resolve(arena_);
  for (auto& u : ups_) u.resolve(arena_);
  for (auto& rb : rbs_) {
    for (auto& c : rb.c1) c.resolve(arena_);
    for (auto& c : rb.c2) c.resolve(arena_);
    for (size_t o : rb.f1_off) rb.f1.push_back(static_cast<const bf16_t*>(arena_.ptr(o)));
    for (size_t o : rb.f2_off) rb.f2.push_back(static_cast<const bf16_t*>(arena_.ptr(o)));
    for (size_t o : rb.h1_off) rb.h1.push_back(static_cast<const bf16_t*>(arena_.ptr(o)));
    for (size_t o : rb.h2_off) rb.h2.push_back(static_cast<const bf16_t*>(arena_.ptr(o)));
    for (auto* qv : {&rb.q1, &rb.q2})
      for (RB::F8& f : *qv) {
        f.wp = arena_.ptr(f.w);
        f.sp = static_cast<const float*>(arena_.ptr(f.s));
        f.bp = static_cast<const float*>(arena_.ptr(f.b));
      }
  }
}

size_t Vocoder::act_elems(int B, int T) const {
  size_t m = (size_t)B * T * chan_stride(h_.upsample_initial_channel);
  size_t L = T;
  for (int i = 0; i < h_.n_up; ++i) {
    L *= h_.upsample_rates[i];
    m = std::max(m, (size_t)B * L * chan_stride(h_.upsample_initial_channel >> (i + 1)));
  }
  return m;
}

size_t Vocoder::workspace_bytes(int B, int T) const {
  const size_t es = act_bytes(dtype_);
  Workspace ws(nullptr, 0);
  ws.take<char>((size_t)B * T * chan_stride(h_.num_mels) * es);
  for (int i = 0; i < act_buffers(); ++i) ws.take<char>(act_elems(B, T) * es);
  return ws.used();
}

void Vocoder::forward(const float* mel, int layout, int B, int T, float* wav, Workspace& ws, hipStream_t s) {
  M2S_CHECK(B > 0 && T > 0, "vocoder: empty input");
  const int cs = chan_stride(h_.num_mels);
  if (dtype_ == M2S_DT_BF16 || dtype_ == M2S_DT_FP8) {
    bf16_t* mn = ws.take<bf16_t>((size_t)B * T * cs);
    launch_mel_to_nlc<bf16_t>(mel, B, h_.num_mels, T, layout, mn, cs, s);
    run_t<bf16_t>(mn, B, T, wav, ws, s);
  } else if (dtype_ == M2S_DT_BF16X3) {
    sp_t* mn = ws.take<sp_t>((size_t)B * T * cs * 2);
    launch_mel_to_nlc<sp_t>(mel, B, h_.num_mels, T, layout, mn, cs, s);
    run_t<sp_t>(mn, B, T, wav, ws, s);
  } else {
    float* mn = ws.take<float>((size_t)B * T * cs);
    launch_mel_to_nlc<float>(mel, B, h_.num_mels, T, layout, mn, cs, s);
    run_t<float>(mn, B, T, wav, ws, s);
  }
}

void Vocoder::forward_from_norm(const float* mel_norm, const float* mean, const float* std_, int B, int T,
                                float* mel_db, float* mel_log, void* ln_buf, float* wav, Workspace& ws, hipStream_t s) {
  M2S_CHECK(B > 0 && T > 0, "vocoder: empty input");
  const int nm = h_.num_mels, cs = chan_stride(nm);
  ws.take<char>((size_t)B * T * cs * act_bytes(dtype_));  // same carve as forward()
  StageTag tag("glue");
  if (dtype_ == M2S_DT_BF16 || dtype_ == M2S_DT_FP8) {
    ProfScope ps("mel_glue_kernel<unsigned short>", 0.0, 4.0 * B * T * nm * 4, s);
    launch_mel_glue<bf16_t>(mel_norm, B * T, nm, mean, std_, mel_db, mel_log, static_cast<bf16_t*>(ln_buf), cs, s);
  } else if (dtype_ == M2S_DT_BF16X3) {
    ProfScope ps("mel_glue_kernel<m2s::sp_t>", 0.0, 4.0 * B * T * nm * 4, s);
    launch_mel_glue<sp_t>(mel_norm, B * T, nm, mean, std_, mel_db, mel_log, static_cast<sp_t*>(ln_buf), cs, s);
  } else {
    ProfScope ps("mel_glue_kernel<float>", 0.0, 4.0 * B * T * nm * 4, s);
    launch_mel_glue<float>(mel_norm, B * T, nm, mean, std_, mel_db, mel_log, static_cast<float*>(ln_buf), cs, s);
  }
  if (dtype_ == M2S_DT_BF16 || dtype_ == M2S_DT_FP8)
    run_t<bf16_t>(ln_buf, B, T, wav, ws, s);
  else if (dtype_ == M2S_DT_BF16X3)
    run_t<sp_t>(ln_buf, B, T, wav, ws, s);
  else
    run_t<float>(ln_buf, B, T, wav, ws, s);
}

// split: + the batched stages' per-resblock buffers; fp8: + one for the e4m3 pair outputs (run_t)
int Vocoder::act_buffers() const { return dtype_ == M2S_DT_BF16X3 ? 5 + 3 * CONV_BATCH : dtype_ == M2S_DT_FP8 ? 6 : 5; }

// Split-fp32 ResBlock1 stage with the resblocks batched (conv_gemm batch launches, grid.z = resblock):
// X holds a0 = lrelu(x) (the upsampler's epilogue applied it), so no conv re-applies LeakyReLU to its
// operand fragments per K step; each c2 recovers its residual x from lrelu(x) (slope 0.1 is
// invertible: x = a > 0 ? a : 10 a) and stores lrelu(xt + x) for the next pair's c1.  Per pair:
// one launch for the c1 of every resblock, one for the c2 (the last pair's c2 accumulates the MRF
// sum S = (x_0 + x_1 + ...) / num_kernels in resblock order, models.py:119-125, so it stays serial).
template <typename T>
void Vocoder::mrf_stage_batched(int i, const T* X, T* S, T* const (*Bt)[3], int B, int L, bool act_out,
                                hipStream_t s) {
  const int nk = h_.n_kernels, np = (int)rbs_[i * nk].dil.size();
  int ord[CONV_BATCH];
  for (int j = 0; j < nk; ++j) ord[j] = j;
  std::sort(ord, ord + nk, [&](int x, int y) { return rbs_[i * nk + x].c1[0].kp > rbs_[i * nk + y].c1[0].kp; });
  auto a_in = [&](int j, int p) -> const T* { return p == 0 ? X : Bt[j][1 + ((p - 1) & 1)]; };  // lrelu(x) of pair p
  bool halo = mrf_halo_;  // input rows staged once per tile (conv1d_halo.hip) where the stage has the weights for it
  for (int j = 0; j < nk; ++j) halo = halo && !rbs_[i * nk + j].h1.empty();
  auto launch_batch = [&](ConvArgs* cs, int n, double fl, double by) {
    if (halo)
      launch_conv1d_halo_sp(cs, n, s, fl, by);
    else
      launch_conv_gemm_batch(cs, n, s, fl, by);
  };
  for (int p = 0; p < np; ++p) {
    ConvArgs cs[CONV_BATCH];
    double fl = 0.0, by = 0.0, f, b;
    for (int jj = 0; jj < nk; ++jj) {
      const int j = ord[jj];
      const RB& rb = rbs_[i * nk + j];
      ConvArgs c = conv_args(rb.c1[p]);
      if (halo) c.w = rb.h1[p];
      c.x = a_in(j, p);
      c.y = Bt[j][0];
      c.L_in = c.L_out = L;
      c.M = B * L;
      c.act = ACT_LRELU;
      c.act_slope = 0.1f;
      conv_cost<T>(c, rb.c1[p], &f, &b);
      fl += f;
      by += b;
      cs[jj] = c;
    }
    launch_batch(cs, nk, fl, by);
    fl = by = 0.0;
    for (int jj = 0; jj < nk; ++jj) {
      const int j = p + 1 < np ? ord[jj] : jj;
      const RB& rb = rbs_[i * nk + j];
      ConvArgs c = conv_args(rb.c2[p]);
      if (halo) c.w = rb.h2[p];
      c.x = Bt[j][0];
      c.res = a_in(j, p);
      c.res_unslope = 10.f;
      c.L_in = c.L_out = L;
      c.M = B * L;
      if (p + 1 < np) {  // a_{p+1} = lrelu(xt + x)
        c.y = Bt[j][1 + (p & 1)];
        c.act = ACT_LRELU;
        c.act_slope = 0.1f;
        c.act_after_res = 1;
        conv_cost<T>(c, rb.c2[p], &f, &b);
        fl += f;
        by += b;
        cs[jj] = c;
      } else {  // xs = sum_j resblock_j(x); x = xs / num_kernels
        c.y = S;
        c.accum = j == 0 ? 0 : (j == nk - 1 ? 2 : 1);
        c.accum_div = (float)nk;
        if (act_out && j == nk - 1) {  // S = lrelu(xs / num_kernels) for the next upsampler
          c.act = ACT_LRELU;
          c.act_slope = 0.1f;
          c.act_after_res = 1;
        }
        if (halo) {
          conv_cost<T>(c, rb.c2[p], &f, &b);
          launch_conv1d_halo_sp(&c, 1, s, f, b);
        } else {
          run_conv<T>(c, rb.c2[p], s);
        }
      }
    }
    if (p + 1 < np) launch_batch(cs, nk, fl, by);
  }
}

template <typename T>
void Vocoder::run_t(const void* mel_nlc, int B, int Tn, float* wav, Workspace& ws, hipStream_t s) {
  constexpr bool SPL = std::is_same<T, sp_t>::value;
  const size_t n = act_elems(B, Tn) * Elem<T>::R;
  T* X = ws.take<T>(n);
  T* Hb[2] = {ws.take<T>(n), ws.take<T>(n)};
  T* T1 = ws.take<T>(n);
  T* S = ws.take<T>(n);
  T* E8 = dtype_ == M2S_DT_FP8 ? ws.take<T>(n) : nullptr;  // fp8: e4m3 outputs of the C = 128 / 256 MRF pairs
  T* Bt[CONV_BATCH][3] = {};  // split: per resblock, c1 output and the pair outputs (ping-pong)
  if (SPL)
    for (int j = 0; j < CONV_BATCH; ++j)
      for (int q = 0; q < 3; ++q) Bt[j][q] = ws.take<T>(n);
  int L = Tn;
  const int nk = h_.n_kernels;
  auto is_batched = [&](int i) {  // stage i's MRF runs as batched split launches (mrf_stage_batched)
    const PConv& up = ups_[i];
    const bool fused = (std::is_same<T, bf16_t>::value || SPL) && mrf_fused_ && !rbs_[i * nk].f1.empty();
    bool b = SPL && mrf_batch_ && !fused && h_.resblock == 1 && nk <= CONV_BATCH && up.cout >= 32 && up.cout % 32 == 0;
    for (int j = 0; j < nk; ++j) b = b && rbs_[i * nk + j].dil.size() == rbs_[i * nk].dil.size();
    return b;
  };
  // split: the upsampler's input S may already hold lrelu(x) (slope 0.1, models.py:116-117), written so
  // by its producer's epilogue (conv_pre, or a batched stage's final MRF accumulation), so the
  // upsampler does not re-apply LeakyReLU to its operand fragments every K step
  bool s_act = SPL;
  {
    StageTag tag("voc_pre");
    ConvArgs a = conv_args(pre_);
    a.x = mel_nlc;
    a.y = S;
    a.L_in = L;
    a.L_out = L;
    a.M = B * L;
    if (s_act) {
      a.act = ACT_LRELU;
      a.act_slope = 0.1f;
    }
    run_conv<T>(a, pre_, s);
  }
  for (int i = 0; i < h_.n_up; ++i) {
    const PConv& up = ups_[i];
    const bool batched = is_batched(i);
    StageTag tag("ups_c" + std::to_string(up.cout));
    ConvArgs a = conv_args(up);
    a.x = S;
    a.y = X;
    a.L_in = L;
    a.L_out = L * up.ct_u;
    a.M = B * L;  // rows per phase
    if (!s_act) {
      a.in_xform = IN_LRELU;
      a.in_slope = 0.1f;
    }
    if (batched) {  // X = lrelu(upsampled x): the MRF convs read it as is (mrf_stage_batched)
      a.act = ACT_LRELU;
      a.act_slope = 0.1f;
    }
    run_conv<T>(a, up, s);
    L *= up.ct_u;
    StageTag mrf("mrf_c" + std::to_string(up.cout));  // the stage's MRF (ResBlocks + sum), models.py:119-125
    if (batched) {
      // the last accumulation stores lrelu(S) when the next consumer is an upsampler (conv_post
      // takes F.leaky_relu's default slope 0.01 on the raw S)
      s_act = i + 1 < h_.n_up;
      mrf_stage_batched<T>(i, X, S, Bt, B, L, s_act, s);
      continue;
    }
    s_act = false;
    // every resblock of the stage must carry e4m3 weights (q8 is decided per resblock: k <= 31)
    bool stage_f8 = std::is_same<T, bf16_t>::value;
    for (int j = 0; j < nk && stage_f8; ++j) {
      const RB& rb = rbs_[i * nk + j];
      stage_f8 = rb.q1.size() == rb.dil.size() && rb.q2.size() == rb.dil.size() && !rb.dil.empty();
    }
    if (stage_f8) {
      // fp8 stage (C = 128 / 256): e4m3 operands.  X8 = e4m3(lrelu(x)) once; per pair, c1 stores only
      // e4m3(lrelu(xt)) (its sole consumer is c2), c2 adds the bf16 residual and stores x (bf16, the next
      // residual) and e4m3(lrelu(x)) (the next c1's operand); the last c2 accumulates the MRF sum in S.
      const int C = up.cout;
      const long nel = (long)B * L * C;
      uint8_t* X8 = reinterpret_cast<uint8_t*>(T1);  // T1 (2 bytes / element) holds X8 and T8
      uint8_t* T8 = X8 + nel;
      uint8_t* H8[2] = {reinterpret_cast<uint8_t*>(E8), reinterpret_cast<uint8_t*>(E8) + nel};
      {
        ProfScope ps("lrelu_e4m3_kernel", 0.0, 3.0 * nel, s);
        launch_lrelu_e4m3(reinterpret_cast<const bf16_t*>(X), X8, nel, 0.1f, s);
      }
      const double rows = (double)B * L;
      for (int j = 0; j < nk; ++j) {
        const RB& rb = rbs_[i * nk + j];
        const int np = (int)rb.dil.size();
        const bf16_t* cur = reinterpret_cast<const bf16_t*>(X);
        const uint8_t* cur8 = X8;
        for (int p = 0; p < np; ++p) {
          const double fl = 2.0 * rows * C * C * rb.k, wb = (double)C * C * rb.k;
          launch_conv1d_f8(cur8, B, L, C, rb.k, rb.dil[p], rb.q1[p].wp, rb.q1[p].sp, rb.q1[p].bp, nullptr, nullptr, T8,
                           0.1f, 0, 1.f, s, fl, 2.0 * nel + wb);
          if (p == np - 1) {
            const int accum = j == 0 ? 0 : (j == nk - 1 ? 2 : 1);
            launch_conv1d_f8(T8, B, L, C, rb.k, 1, rb.q2[p].wp, rb.q2[p].sp, rb.q2[p].bp, cur, S, nullptr, 0.f, accum,
                             (float)nk, s, fl, nel * (1.0 + 2.0 + 2.0 + (accum ? 2.0 : 0.0)) + wb);
          } else {
            bf16_t* xo = reinterpret_cast<bf16_t*>(Hb[p & 1]);
            launch_conv1d_f8(T8, B, L, C, rb.k, 1, rb.q2[p].wp, rb.q2[p].sp, rb.q2[p].bp, cur, xo, H8[p & 1], 0.1f, 0,
                             1.f, s, fl, nel * (1.0 + 2.0 + 2.0 + 1.0) + wb);
            cur = xo;
            cur8 = H8[p & 1];
          }
        }
      }
      continue;
    }
    for (int j = 0; j < nk; ++j) {
      const RB& rb = rbs_[i * nk + j];
      const T* hcur = X;
      const int np = (int)rb.dil.size();
      const int accum = j == 0 ? 0 : (j == nk - 1 ? 2 : 1);
      if ((std::is_same<T, bf16_t>::value || SPL) && mrf_fused_ && !rb.f1.empty()) {
        // one launch for the whole resblock + MRF sum (mrf_fused.hip)
        const bf16_t* w1[8];
        const bf16_t* w2[8];
        const float* b1[8];
        const float* b2[8];
        double macs = 0.0;
        for (int p = 0; p < np; ++p) {
          w1[p] = rb.f1[p];
          w2[p] = rb.f2[p];
          b1[p] = rb.c1[p].b;
          b2[p] = rb.c2[p].b;
          macs += rb.c1[p].macs_per_row + rb.c2[p].macs_per_row;
        }
        const int C = rb.c1[0].cout;
        const double rows = (double)B * L;
        const double bytes = (SPL ? 2.0 : 1.0) * (2.0 * rows * C * (2 + (accum ? 1 : 0)) + 2.0 * np * 2 * C * C * rb.k);
        launch_rb1_fused(reinterpret_cast<const bf16_t*>(X), reinterpret_cast<bf16_t*>(S), B, L, C, rb.k, np,
                         rb.dil.data(), w1, b1, w2, b2, rb.c1[0].kp, accum, (float)nk, SPL, 2.0 * macs * rows, bytes,
                         s);
        continue;
      }
      for (int p = 0; p < np; ++p) {
        const bool last = p == np - 1;
        T* out = last ? S : Hb[p & 1];
        ConvArgs c = conv_args(rb.c1[p]);
        c.x = hcur;
        c.L_in = L;
        c.L_out = L;
        c.M = B * L;
        c.in_xform = IN_LRELU;
        c.in_slope = 0.1f;
        if (h_.resblock == 1) {  // xt = c2(lrelu(c1(lrelu(x)))) ; x = xt + x
          c.y = T1;
          c.act = ACT_LRELU;
          c.act_slope = 0.1f;
          run_conv<T>(c, rb.c1[p], s);
          c = conv_args(rb.c2[p]);
          c.x = T1;
          c.L_in = L;
          c.L_out = L;
          c.M = B * L;
        }
        c.y = out;
        c.res = hcur;
        if (last) {  // xs = sum_j resblock_j(x); x = xs / num_kernels (models.py:119-125)
          c.accum = j == 0 ? 0 : (j == nk - 1 ? 2 : 1);
          c.accum_div = (float)nk;
        }
        run_conv<T>(c, h_.resblock == 1 ? rb.c2[p] : rb.c1[p], s);
        hcur = out;
      }
    }
  }
  StageTag tag("voc_post");
  ProfScope ps(tname<T>(post_c_ <= 64 ? "conv_post_tile_kernel" : "conv_post_kernel"), 2.0 * B * L * post_c_ * 7, (sizeof(T) * Elem<T>::R) * (double)B * L * post_c_ + 4.0 * B * L, s);
  launch_conv_post<T>(S, B, L, post_c_, chan_stride(post_c_), static_cast<const float*>(arena_.ptr(post_w_)), post_b_,
                      wav, s);
}

}  // namespace m2s
