// Microbenchmark of the fused stem + blocks.0 kernel (stem_b0.hip), one executable per SB_MODE
// variant: 0 full, 1 no stem, 2 no blocks.0.0 MFMA, 4 no blocks.0.1 MFMA.  1920 frames of 256x256.
#include "../mri-to-speech_amd/csrc/stem_b0.hip"

#include <cstdio>
#include <vector>

using namespace m2s;

int main() {
  const int N = 1920, H = 256, W = 256, OH = 128, OW = 128;
  std::vector<float> hf((size_t)N * H * W), hw9(32 * 9, 0.05f), hb(64, 0.01f);
  for (size_t i = 0; i < hf.size(); ++i) hf[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
  std::vector<uint16_t> hw0(64 * 288, 0x3c00), hw1(64 * 160, 0x3c00);
  float *fr, *w9, *b;
  bf16_t *w0, *w1, *y;
  (void)hipMalloc(&fr, hf.size() * 4);
  (void)hipMalloc(&w9, hw9.size() * 4);
  (void)hipMalloc(&b, hb.size() * 4);
  (void)hipMalloc(&w0, hw0.size() * 2);
  (void)hipMalloc(&w1, hw1.size() * 2);
  (void)hipMalloc(&y, (size_t)N * OH * OW * 16 * 2);
  (void)hipMemcpy(fr, hf.data(), hf.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(w9, hw9.data(), hw9.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(w0, hw0.data(), hw0.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(w1, hw1.data(), hw1.size() * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&] { launch_stem_b0(fr, N, H, W, OH, OW, 0, 0, w9, b, w0, b, 288, w1, b, 160, y, 0, 0, nullptr); };
  for (int i = 0; i < 3; ++i) run();
  const int iters = 10;
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < iters; ++i) run();
  (void)hipEventRecord(e1, nullptr);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::printf("SB_MODE=%d us=%.1f\n", SB_MODE, 1000.0 * ms / iters);
  return 0;
}
