// Grad-CAM path host code (cam.hpp): the train-mode backbone plan and the BiLSTM / Linear autograd
// entry points.
//
// Reference behaviour (scripts/mri_gradcam_formant.py): compute_gradcam puts the model in train()
// (:223), so the backbone's BatchNorms normalise with the statistics of the B*T frames of the call and
// update their running statistics (timm BatchNormAct2d = torch BatchNorm2d, momentum 0.1, eps 1e-3);
// the last feature map is made a gradient leaf (:155-160), pooled, run through rnn and head
// (:162-165), and the band power's gradient is read back at feats.grad (:247-248).  Nothing needs the
// backbone's own backward, so the backbone here is a forward with batch statistics only.
#include "cam.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "pack.hpp"

namespace m2s {

namespace {

const int kTaps[5] = {2, 5, 8, 18, 28};  // timm features_only taps: blocks run (mri_gradcam_formant.py:155-158)

}  // namespace

CamBackbone::CamBackbone(const StateDict& sd, int device) : device_(device) {
  const std::string P = "cnn.backbone.";
  auto add_bn = [&](const std::string& p, int c) {
    BNp b;
    b.C = c;
    b.g = arena_.add(need(sd, p + ".weight", {c}).data, sizeof(float) * c);
    b.b = arena_.add(need(sd, p + ".bias", {c}).data, sizeof(float) * c);
    bn_.push_back(b);
    return (int)bn_.size() - 1;
  };
  {  // grey repeated to RGB: the three input-channel taps of conv_stem summed
    const float* w = need(sd, P + "conv_stem.weight", {EFF_STEM, 3, 3, 3}).data;
    std::vector<float> w9(EFF_STEM * 9);
    for (int o = 0; o < EFF_STEM; ++o)
      for (int t = 0; t < 9; ++t) w9[o * 9 + t] = w[(o * 3 + 0) * 9 + t] + w[(o * 3 + 1) * 9 + t] + w[(o * 3 + 2) * 9 + t];
    stem_w_ = arena_.add_vec(w9);
    stem_bn_ = add_bn(P + "bn1", EFF_STEM);
  }
  auto zero = [](int) { return 0.f; };
  int cin = EFF_STEM;
  for (int s = 0; s < 6; ++s) {
    const StageDef& sdf = kStages[s];
    for (int r = 0; r < sdf.reps; ++r) {
      Blk b;
      b.type = sdf.type;
      b.stride = r == 0 ? sdf.stride : 1;
      b.cin = cin;
      b.cout = sdf.cout;
      b.skip = b.stride == 1 && cin == sdf.cout;
      const std::string q = P + "blocks." + std::to_string(s) + "." + std::to_string(r) + ".";
      auto conv3 = [&](PConv& pc, const std::string& wk, int ci, int co) {
        const float* w = need(sd, wk, {co, ci, 3, 3}).data;
        pc = make_pconv(KIND_CONV2D, ci, co, 9, M2S_DT_F32);
        pc.ks = 3;
        pc.stride = b.stride;
        pc.macs_per_row = 9.0 * co * ci;
        pack_conv(arena_, M2S_DT_F32, pc, [&](int, int n, int t, int c) { return w[((size_t)n * ci + c) * 9 + t]; }, zero);
      };
      auto conv1 = [&](PConv& pc, const std::string& wk, int ci, int co) {
        const float* w = need(sd, wk, {co, ci, 1, 1}).data;
        pc = make_pconv(KIND_GEMM, ci, co, 1, M2S_DT_F32);
        pc.macs_per_row = (double)co * ci;
        pack_conv(arena_, M2S_DT_F32, pc, [&](int, int n, int, int c) { return w[(size_t)n * ci + c]; }, zero);
      };
      if (b.type == 0) {
        conv3(b.c1, q + "conv.weight", cin, b.cout);
        b.bn[0] = add_bn(q + "bn1", b.cout);
      } else if (b.type == 1) {
        b.mid = make_divisible(cin * (double)sdf.exp);
        conv3(b.c1, q + "conv_exp.weight", cin, b.mid);
        b.bn[0] = add_bn(q + "bn1", b.mid);
        conv1(b.c2, q + "conv_pwl.weight", b.mid, b.cout);
        b.bn[1] = add_bn(q + "bn2", b.cout);
      } else {
        b.mid = make_divisible(cin * (double)sdf.exp);
        b.rd = (int)std::lround(b.mid * (sdf.se / sdf.exp));
        const int m = b.mid, cs = chan_stride(m), rd = b.rd;
        conv1(b.c1, q + "conv_pw.weight", cin, m);
        b.bn[0] = add_bn(q + "bn1", m);
        const float* wd = need(sd, q + "conv_dw.weight", {m, 1, 3, 3}).data;
        std::vector<float> w9((size_t)cs * 9, 0.f);
        for (int c = 0; c < m; ++c)
          for (int t = 0; t < 9; ++t) w9[(size_t)t * cs + c] = wd[(size_t)c * 9 + t];
        b.dw = arena_.add_vec(w9);
        b.bn[1] = add_bn(q + "bn2", m);
        const float* w1 = need(sd, q + "se.conv_reduce.weight", {rd, m, 1, 1}).data;
        const float* b1 = need(sd, q + "se.conv_reduce.bias", {rd}).data;
        const float* w2 = need(sd, q + "se.conv_expand.weight", {m, rd, 1, 1}).data;
        const float* b2 = need(sd, q + "se.conv_expand.bias", {m}).data;
        b.se1 = make_pconv(KIND_GEMM, m, rd, 1, M2S_DT_F32);
        b.se1.macs_per_row = (double)m * rd;
        pack_conv(arena_, M2S_DT_F32, b.se1, [&](int, int n, int, int c) { return w1[(size_t)n * m + c]; },
                  [&](int n) { return b1[n]; });
        b.se2 = make_pconv(KIND_GEMM, rd, m, 1, M2S_DT_F32);
        b.se2.macs_per_row = (double)m * rd;
        pack_conv(arena_, M2S_DT_F32, b.se2, [&](int, int n, int, int c) { return w2[(size_t)n * rd + c]; },
                  [&](int n) { return b2[n]; });
        conv1(b.c2, q + "conv_pwl.weight", m, b.cout);
        b.bn[2] = add_bn(q + "bn3", b.cout);
      }
      blocks_.push_back(b);
      cin = sdf.cout;
    }
  }
  arena_.upload(device);
  for (auto& b : blocks_) {
    b.c1.resolve(arena_);
    if (b.type != 0) b.c2.resolve(arena_);
    if (b.type == 2) {
      b.se1.resolve(arena_);
      b.se2.resolve(arena_);
    }
  }
}

int CamBackbone::bn_stats_floats() const {
  int n = 0;
  for (const BNp& b : bn_) n += 2 * b.C;
  return n;
}

namespace {
struct CamDims {
  size_t io = 0, mid = 0;  // per-frame floats of the block outputs / expanded maps
  int cs_mid = 0;
};
}  // namespace

static CamDims cam_dims(int H, int W) {
  CamDims d;
  int oh, ow, p;
  same_pad(H, 3, 2, &oh, &p);
  same_pad(W, 3, 2, &ow, &p);
  d.io = (size_t)oh * ow * chan_stride(EFF_STEM);
  int cin = EFF_STEM;
  for (int s = 0; s < 6; ++s)
    for (int r = 0; r < kStages[s].reps; ++r) {
      const int st = r == 0 ? kStages[s].stride : 1;
      int nh, nw;
      same_pad(oh, 3, st, &nh, &p);
      same_pad(ow, 3, st, &nw, &p);
      if (kStages[s].type != 0) {
        const int cs = chan_stride(make_divisible(cin * (double)kStages[s].exp));
        d.mid = std::max(d.mid, (size_t)(kStages[s].type == 2 ? oh * ow : nh * nw) * cs);
        d.cs_mid = std::max(d.cs_mid, cs);
      }
      d.io = std::max(d.io, (size_t)nh * nw * chan_stride(kStages[s].cout));
      cin = kStages[s].cout;
      oh = nh;
      ow = nw;
    }
  return d;
}

size_t CamBackbone::workspace_bytes(int N, int H, int W) const {
  const CamDims d = cam_dims(H, W);
  Workspace w(nullptr, 0);
  w.take<float>((size_t)N * d.io);
  w.take<float>((size_t)N * d.io);
  w.take<float>((size_t)N * d.mid);
  w.take<float>((size_t)N * d.mid);
  w.take<float>((size_t)N * d.cs_mid);
  w.take<float>((size_t)N * SE_RD_MAX);
  w.take<float>((size_t)N * d.cs_mid);
  w.take<float>(bn_train_scratch_floats(0, std::max(d.cs_mid, 256)));
  return w.used();
}

void CamBackbone::forward(const float* frames, int N, int H, int W, float* const taps[5], float* bn_stats, void* ws,
                          size_t wsb, hipStream_t s) {
  M2S_CHECK(N > 0 && H >= 32 && W >= 32, "cam backbone: bad input size");
  const CamDims d = cam_dims(H, W);
  Workspace w(ws, wsb);
  float* A = w.take<float>((size_t)N * d.io);
  float* Bf = w.take<float>((size_t)N * d.io);
  float* M = w.take<float>((size_t)N * d.mid);
  float* M2 = w.take<float>((size_t)N * d.mid);
  float* sem = w.take<float>((size_t)N * d.cs_mid);
  float* hid = w.take<float>((size_t)N * SE_RD_MAX);
  float* gate = w.take<float>((size_t)N * d.cs_mid);
  float* scr = w.take<float>(bn_train_scratch_floats(0, std::max(d.cs_mid, 256)));
  // the conv kernels index their inputs with 32-bit offsets: run them over frame chunks
  const int fc = (int)std::max<size_t>(1, std::min<size_t>(N, 2147483647ull / std::max(d.io, d.mid)));
  std::vector<size_t> st_off(bn_.size());
  {
    size_t o = 0;
    for (size_t i = 0; i < bn_.size(); ++i) {
      st_off[i] = o;
      o += 2 * (size_t)bn_[i].C;
    }
  }
  auto bn = [&](float* x, long rows, int layer, int cs, int act, const float* res) {
    const BNp& p = bn_[layer];
    launch_bn_train(x, rows, p.C, cs, static_cast<const float*>(arena_.ptr(p.g)),
                    static_cast<const float*>(arena_.ptr(p.b)), 1e-3f, act, res, bn_stats + st_off[layer], scr, s);
  };
  int oh, ow, pt, pl;
  same_pad(H, 3, 2, &oh, &pt);
  same_pad(W, 3, 2, &ow, &pl);
  launch_stem_raw(frames, N, H, W, oh, ow, pt, pl, static_cast<const float*>(arena_.ptr(stem_w_)), A, s);
  bn(A, (long)N * oh * ow, stem_bn_, chan_stride(EFF_STEM), 1, nullptr);
  float* cur = A;
  float* nxt = Bf;
  int ti = 0;
  for (size_t k = 0; k < blocks_.size(); ++k) {
    const Blk& b = blocks_[k];
    int nh, nw, qt, ql;
    same_pad(oh, 3, b.stride, &nh, &qt);
    same_pad(ow, 3, b.stride, &nw, &ql);
    const int cso = chan_stride(b.cout), csm = b.mid ? chan_stride(b.mid) : 0;
    // one conv over all frames, chunked; in / out per-frame strides in floats
    auto conv = [&](const PConv& pc, const float* x, size_t xs, float* y, size_t ys, int IH, int IW, int OH, int OW,
                    const float* scale) {
      for (int n0 = 0; n0 < N; n0 += fc) {
        const int nc = std::min(fc, N - n0);
        ConvArgs a = conv_args(pc);
        a.x = x + (size_t)n0 * xs;
        a.y = y + (size_t)n0 * ys;
        a.M = nc * OH * OW;
        if (pc.kind == KIND_CONV2D) {
          a.IH = IH;
          a.IW = IW;
          a.OH = OH;
          a.OW = OW;
          a.pad_t = qt;
          a.pad_l = ql;
        } else {
          a.OH = OH * OW;  // rows per image (the SE gate table is per image)
        }
        if (scale) {
          a.in_xform = IN_SE_SCALE;
          a.in_scale = scale + (size_t)n0 * pc.cs_in;
        }
        run_conv<float>(a, pc, s);
      }
    };
    const size_t pin = (size_t)oh * ow, pout = (size_t)nh * nw;
    if (b.type == 0) {
      conv(b.c1, cur, pin * b.c1.cs_in, nxt, pout * cso, oh, ow, nh, nw, nullptr);
      bn(nxt, (long)N * pout, b.bn[0], cso, 1, b.skip ? cur : nullptr);
    } else if (b.type == 1) {
      conv(b.c1, cur, pin * b.c1.cs_in, M, pout * csm, oh, ow, nh, nw, nullptr);
      bn(M, (long)N * pout, b.bn[0], csm, 1, nullptr);
      conv(b.c2, M, pout * csm, nxt, pout * cso, nh, nw, nh, nw, nullptr);
      bn(nxt, (long)N * pout, b.bn[1], cso, 0, b.skip ? cur : nullptr);
    } else {
      conv(b.c1, cur, pin * b.c1.cs_in, M, pin * csm, oh, ow, oh, ow, nullptr);
      bn(M, (long)N * pin, b.bn[0], csm, 1, nullptr);
      launch_dw_raw(M, N, oh, ow, nh, nw, b.stride, qt, ql, csm, static_cast<const float*>(arena_.ptr(b.dw)), M2, s);
      bn(M2, (long)N * pout, b.bn[1], csm, 1, nullptr);
      launch_gap<float>(M2, N, (int)pout, csm, csm, sem, s);  // SE squeeze, (N, cs_mid)
      ConvArgs r1 = conv_args(b.se1);                        // conv_reduce + SiLU
      r1.x = sem;
      r1.y = hid;
      r1.M = N;
      r1.act = ACT_SILU;
      run_conv<float>(r1, b.se1, s);
      ConvArgs r2 = conv_args(b.se2);  // conv_expand + sigmoid -> gates
      r2.x = hid;
      r2.y = gate;
      r2.M = N;
      r2.act = ACT_SIGMOID;
      run_conv<float>(r2, b.se2, s);
      conv(b.c2, M2, pout * csm, nxt, pout * cso, nh, nw, nh, nw, gate);
      bn(nxt, (long)N * pout, b.bn[2], cso, 0, b.skip ? cur : nullptr);
    }
    std::swap(cur, nxt);
    oh = nh;
    ow = nw;
    if (ti < 5 && (int)k + 1 == kTaps[ti]) {
      if (taps && taps[ti]) launch_to_nchw(cur, N, oh * ow, b.cout, cso, taps[ti], s);
      ++ti;
    }
  }
}

// ---- BiLSTM / Linear autograd entry points -------------------------------------------------------
size_t bilstm_train_workspace_bytes(int B, int T, int C, int H) {
  const size_t BT = (size_t)B * T;
  Workspace w(nullptr, 0);
  w.take<float>(std::max(BT * 8 * H, (size_t)2 * BT * 4 * H));  // fwd: gate pre-activations; bwd: dG
  w.take<float>((size_t)2 * 4 * H * H);                         // W_hh of both directions (or W_hh^T)
  w.take<float>(std::max((size_t)2 * B * H, (size_t)2 * BT * H));  // bwd: dc, then h_prev
  w.take<float>((size_t)2 * B * H);
  (void)C;
  return w.used();
}

void bilstm_train_forward(const float* x, int B, int T, int C, int H, const float* const w_ih[2],
                          const float* const w_hh[2], const float* const b_ih[2], const float* const b_hh[2], float* y,
                          float* gates, float* cells, float* hid, void* ws, size_t wsb, hipStream_t s) {
  M2S_CHECK(B > 0 && T > 0 && C > 0 && H > 0 && H % 8 == 0, "bilstm_train: shape");
  const long BT = (long)B * T;
  Workspace w(ws, wsb);
  float* pre = w.take<float>(std::max(BT * 8 * H, 2 * BT * 4 * (long)H));
  float* whh = w.take<float>((size_t)2 * 4 * H * H);
  for (int d = 0; d < 2; ++d) {
    // pre[bt][d*4H + n] = sum_c x[bt][c] W_ih[n][c] + b_ih[n] + b_hh[n]
    launch_gemm_f32((int)BT, 4 * H, C, x, C, 1, w_ih[d], 1, C, pre + (size_t)d * 4 * H, 8L * H, b_ih[d], b_hh[d], false, s);
    M2S_HIP(hipMemcpyAsync(whh + (size_t)d * 4 * H * H, w_hh[d], sizeof(float) * 4 * H * H, hipMemcpyDeviceToDevice, s));
  }
  for (int st = 0; st < T; ++st) launch_lstm_train_step(pre, whh, gates, cells, hid, B, T, H, st, s);
  launch_add2(hid, hid + BT * H, y, BT * H, s);
}

void bilstm_train_backward(const float* x, const float* dy, int B, int T, int C, int H, const float* const w_ih[2],
                           const float* const w_hh[2], const float* gates, const float* cells, const float* hid,
                           float* dx, float* const dw_ih[2], float* const dw_hh[2], float* const db[2], void* ws,
                           size_t wsb, hipStream_t s) {
  M2S_CHECK(B > 0 && T > 0 && C > 0 && H > 0 && H % 8 == 0, "bilstm_train: shape");
  const long BT = (long)B * T;
  const int G = 4 * H;
  Workspace w(ws, wsb);
  float* dg = w.take<float>(std::max(BT * 8 * H, 2 * BT * (long)G));
  float* wt = w.take<float>((size_t)2 * G * H);
  float* hp = w.take<float>(std::max((size_t)2 * B * H, (size_t)2 * BT * H));
  float* dc = w.take<float>((size_t)2 * B * H);
  for (int d = 0; d < 2; ++d) launch_transpose(w_hh[d], 1, G, H, wt + (size_t)d * G * H, s);
  for (int st = 0; st < T; ++st) launch_lstm_bptt_step(wt, dy, gates, cells, dc, dg, B, T, H, st, s);
  launch_lstm_hprev(hid, hp, B, T, H, s);
  for (int d = 0; d < 2; ++d) {
    const float* g = dg + (size_t)d * BT * G;
    if (dx)  // dx[bt][c] (+)= sum_n dG[bt][n] W_ih[n][c]
      launch_gemm_f32((int)BT, C, G, g, G, 1, w_ih[d], C, 1, dx, C, nullptr, nullptr, d == 1, s);
    if (dw_ih && dw_ih[d])  // dW_ih[n][c] = sum_bt dG[bt][n] x[bt][c]
      launch_gemm_f32(G, C, (int)BT, g, 1, G, x, C, 1, dw_ih[d], C, nullptr, nullptr, false, s);
    if (dw_hh && dw_hh[d])  // dW_hh[n][k] = sum_bt dG[bt][n] h_prev[bt][k]
      launch_gemm_f32(G, H, (int)BT, g, 1, G, hp + (size_t)d * BT * H, H, 1, dw_hh[d], H, nullptr, nullptr, false, s);
    if (db && db[d]) launch_colsum(g, (int)BT, G, G, db[d], false, s);
  }
}

void linear_forward(const float* x, int rows, int in, int out, const float* w, const float* b, float* y, hipStream_t s) {
  launch_gemm_f32(rows, out, in, x, in, 1, w, 1, in, y, out, b, nullptr, false, s);
}

void linear_backward(const float* dy, const float* x, int rows, int in, int out, const float* w, float* dx, float* dw,
                     float* db, hipStream_t s) {
  if (dx) launch_gemm_f32(rows, in, out, dy, out, 1, w, in, 1, dx, in, nullptr, nullptr, false, s);
  if (dw) launch_gemm_f32(out, in, rows, dy, 1, out, x, in, 1, dw, in, nullptr, nullptr, false, s);
  if (db) launch_colsum(dy, rows, out, out, db, false, s);
}

}  // namespace m2s
