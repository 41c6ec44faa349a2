"""hipBLASLt (torch.matmul, bf16) reference throughput at the conv-GEMM shapes,
for calibrating the hand-written MFMA engine against the vendor library."""
import torch

dev = torch.device("cuda", 0)
shapes = [(65536, 512, 4608), (262144, 256, 2304), (1048576, 128, 1152), (4194304, 64, 576),
          (8192, 8192, 8192), (256, 2304, 262144), (128, 1152, 1048576)]
for M, N, K in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for _ in range(it):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    print(f"M={M} N={N} K={K}: {us:9.1f} us {2.0 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)
    del a, b, c
