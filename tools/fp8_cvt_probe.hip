// Probe (measurement tool, not product code): what v_cvt_pk_fp8_f32 returns for out-of-range and NaN
// inputs (OCP e4m3fn: max finite 448 = 0x7e, NaN = 0x7f; the assembler takes no clamp bit on it), and
// v_cvt_scalef32_pk_fp8_f32 with a unit scale.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fp8_cvt_probe.hip -o tools/fp8_cvt_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void probe(const float* x, unsigned* plain, unsigned* clamped, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  plain[i] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(x[i], x[i], 0, false);
  clamped[i] = __builtin_bit_cast(unsigned,
      __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(__builtin_bit_cast(__attribute__((ext_vector_type(2))) short, (int)0), x[i], x[i], 1.0f, false)) ;
}

int main() {
  const float v[] = {0.5f, -0.2785f, 447.f, 448.f, 449.f, 463.f, 464.f, 479.f, 480.f, 500.f, 1000.f, 1e30f,
                     INFINITY, -INFINITY, NAN, -NAN, -448.f, -500.f, -1e30f, 1e-9f};
  const int n = sizeof(v) / sizeof(v[0]);
  float* dx;
  unsigned *dp, *dc;
  hipMalloc(&dx, sizeof(v));
  hipMalloc(&dp, n * 4);
  hipMalloc(&dc, n * 4);
  hipMemcpy(dx, v, sizeof(v), hipMemcpyHostToDevice);
  probe<<<1, 64>>>(dx, dp, dc, n);
  unsigned p[64], c[64];
  hipMemcpy(p, dp, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(c, dc, n * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("%12g  cvt_pk 0x%02x  scalef32 0x%02x\n", v[i], p[i] & 0xff, c[i] & 0xff);
  return 0;
}
