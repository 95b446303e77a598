"""Library reference point: torch.matmul (hipBLASLt/rocBLAS) on the encoder's 1x1-conv GEMM shapes,
bf16, for comparison with conv_gemm (tools/kstats.py).  GPU box only."""
import time

import torch

dev = torch.device("cuda", 0)
shapes = [("b4 conv_pwl", 491520, 736, 128), ("b5 conv_pwl", 122880, 1248, 224), ("b3 conv_pwl", 491520, 416, 128),
          ("b1 conv_pwl", 7864320, 128, 32), ("b2 conv_pwl", 1966080, 224, 64), ("b4 conv_pw", 491520, 128, 736)]
for name, M, K, N in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    it = 20
    t0 = time.perf_counter()
    for _ in range(it):
        c = a @ b
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / it * 1e6
    gb = 2 * (M * K + K * N + M * N) / 1e9
    print(f"{name:12s} M={M} K={K} N={N}: {us:8.1f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s  {gb / us * 1e6 / 1e3:6.2f} TB/s")
