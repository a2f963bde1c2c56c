"""Throughput of the vendor bf16 GEMM (torch.matmul -> hipBLASLt) at the c2 FC
shapes, plain K and with K x 6 (the six bf16x6 products as one K-concatenated
GEMM), against the same shapes in fp32 (rocBLAS / hipBLASLt sgemm).  Tells how
far the MFMA pipe runs under the board's power limit for a library kernel."""
import time

import torch


def bench(m, n, k, dtype, reps=20):
    a = torch.randn(m, k, device="cuda", dtype=dtype)
    b = torch.randn(k, n, device="cuda", dtype=dtype)
    for _ in range(3):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return dt * 1e6, 2.0 * m * n * k / dt / 1e12


for name, (m, n, k) in {"fc_fwd": (4096, 1024, 11616), "fc_dgrad": (4096, 11616, 1024),
                        "fc_wgrad": (1024, 11616, 4096)}.items():
    for dt, kk in ((torch.float32, k), (torch.bfloat16, k), (torch.bfloat16, 6 * k)):
        us, tf = bench(m, n, kk, dt)
        print(f"{name} {str(dt):15s} K={kk:6d}: {us:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)
