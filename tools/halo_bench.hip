// Microbenchmark of the halo 3x3 conv (conv_halo.hip) at the encoder's stride-1 shapes, one
// executable per HALO_MODE variant (1 no MFMA, 4 no stores, 8 no halo prefetch): microseconds
// per launch for 1920 images.
#include "../mri-to-speech_amd/csrc/conv_halo.hip"

#include <cstring>
#include <vector>

using namespace m2s;

static void run(const char* name, int H, int cs_in, int cout, int act, bool res = false) {
  const int N = 1920, kp = (cs_in == 16 ? 10 : 9) * cs_in, npad = (cout + 63) / 64 * 64;
  std::vector<uint16_t> hx((size_t)N * H * H * cs_in), hw((size_t)npad * kp);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = 0x3c00 + (i * 7 % 64);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0x3a00 + (i * 5 % 64);
  std::vector<float> hb(npad, 0.01f);
  bf16_t *x, *w, *y;
  float* b;
  hipMalloc(&x, hx.size() * 2);
  hipMalloc(&w, hw.size() * 2);
  hipMalloc(&y, (size_t)N * H * H * cout * 2);
  hipMalloc(&b, npad * 4);
  hipMemcpy(x, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(b, hb.data(), npad * 4, hipMemcpyHostToDevice);
  ConvArgs a;
  std::memset(&a, 0, sizeof(a));
  a.x = x; a.w = w; a.bias = b; a.y = y;
  a.kind = KIND_CONV2D; a.M = N * H * H; a.cs_in = cs_in; a.cs_out = cout; a.n_pad = npad; a.kp = kp;
  a.ntaps = 9; a.tpc = 1; a.IH = a.IW = a.OH = a.OW = H; a.ks = 3; a.stride = 1; a.pad_t = a.pad_l = 1;
  a.act = act; a.accum_div = 1.f;
  if (res) a.res = x;
  if (!conv_halo_supported(a)) { std::printf("%s: not a halo shape\n", name); return; }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) launch_conv_halo(a, nullptr, 0, 0);
  const int iters = 10;
  hipEventRecord(e0, nullptr);
  for (int i = 0; i < iters; ++i) launch_conv_halo(a, nullptr, 0, 0);
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / iters;
  const double tf = 2.0 * N * H * H * cout * 9.0 * cs_in / us / 1e6;
  const double gbs = 2.0 * N * H * H * (cs_in + cout) / us / 1e3;
  std::printf("mode=%d %-26s us=%8.1f TF/s=%6.1f GB/s=%6.0f\n", HALO_MODE, name, us, tf, gbs);
  hipFree(x); hipFree(w); hipFree(y); hipFree(b);
}

int main() {
  run("b0 128x128 32->16 silu", 128, 32, 16, ACT_SILU);
  run("b0.1 128x128 16->16 silu+res", 128, 16, 16, ACT_SILU, true);
  run("b1 64x64 32->128 silu", 64, 32, 128, ACT_SILU);
  run("b2 32x32 64->224 silu", 32, 64, 224, ACT_SILU);
  run("b1 64x64 32->128 none", 64, 32, 128, ACT_NONE);
  return 0;
}
