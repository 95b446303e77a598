// Microbenchmark of the fused IR kernel (ir_fused.hip) at the encoder's shapes, one executable per
// IRF_MODE variant (see tools/irf_bench.sh): 0 full, 1 no expand GEMM, 2 no depthwise, 4 no y
// stores.  Prints microseconds per launch for the b4 (16x16, 120->720) and b5 (8x8, 208->1248)
// shapes at 1920 images.
#include "../mri-to-speech_amd/csrc/ir_fused.hip"

#include <cstdio>
#include <vector>

using namespace m2s;

static void run(const char* name, int N, int H, int cs_in, int cs_mid) {
  const int P = H * H, npad = (cs_mid + 63) / 64 * 64;
  std::vector<uint16_t> hx((size_t)N * P * cs_in), hw((size_t)npad * cs_in);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = 0x3c00 + (i * 7 % 64);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0x3a00 + (i * 5 % 64);
  std::vector<float> hb(npad, 0.01f), hdb(cs_mid, 0.02f);
  std::vector<uint32_t> hd2((size_t)9 * cs_mid, 0x3c00u);
  bf16_t *x, *w, *y, *se;
  float *b, *db;
  uint32_t* d2;
  hipMalloc(&x, hx.size() * 2);
  hipMalloc(&w, hw.size() * 2);
  hipMalloc(&y, (size_t)N * P * cs_mid * 2);
  hipMalloc(&se, (size_t)N * cs_mid * 2);
  hipMalloc(&b, npad * 4);
  hipMalloc(&db, cs_mid * 4);
  hipMalloc(&d2, hd2.size() * 4);
  hipMemcpy(x, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(b, hb.data(), npad * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, hdb.data(), cs_mid * 4, hipMemcpyHostToDevice);
  hipMemcpy(d2, hd2.data(), hd2.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i)
    launch_ir_pwdw(x, N, cs_in, cs_in, w, b, d2, db, H, H, cs_mid, y, se, 0, 0, nullptr);
  const int iters = 20;
  hipEventRecord(e0, nullptr);
  for (int i = 0; i < iters; ++i)
    launch_ir_pwdw(x, N, cs_in, cs_in, w, b, d2, db, H, H, cs_mid, y, se, 0, 0, nullptr);
  hipEventRecord(e1, nullptr);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / iters;
  const double ybytes = 2.0 * N * P * cs_mid;
  std::printf("mode=%d %s us=%.1f  y-write GB/s=%.0f\n", IRF_MODE, name, us, ybytes / us / 1e3);
  hipFree(x); hipFree(w); hipFree(y); hipFree(se); hipFree(b); hipFree(db); hipFree(d2);
}

int main() {
  run("b4 16x16 128->736", 1920, 16, 128, 736);
  run("b5 8x8 224->1248", 1920, 8, 224, 1248);
  return 0;
}
