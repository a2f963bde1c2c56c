"""Library f16 GEMM rates at c2's FC shapes with K' = 3K (the f16x3 products
as one concatenated-K f16 GEMM, fp32 out), beside fp32 sgemm: what a
pre-split operand layout could reach through the vendor library."""
import torch

SHAPES = [("fwd", 4096, 1024, 11616), ("dgrad", 4096, 11616, 1024), ("wgrad", 1024, 11616, 4096)]


def bench(fn, calls=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(calls):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / calls


for name, m, n, k in SHAPES:
    a = torch.randn(m, 3 * k, device="cuda", dtype=torch.float16)
    b = torch.randn(3 * k, n, device="cuda", dtype=torch.float16)
    bt = b.t().contiguous().t()
    fl = 2 * m * n * k
    for lab, bb in (("nn", b), ("nt", bt)):
        try:
            us = bench(lambda: torch.ops.aten.mm.dtype(a, bb, torch.float32))
            print(f"{name} f16 3K fp32-out {lab}: {us:.1f} us, {fl / us / 1e6:.0f} fp32-eq TF/s", flush=True)
        except Exception as ex:
            print(name, lab, "mm.dtype failed:", str(ex)[:200], flush=True)
    us = bench(lambda: torch.mm(a, b))
    print(f"{name} f16 3K f16-out: {us:.1f} us, {fl / us / 1e6:.0f} fp32-eq TF/s", flush=True)
    a32 = torch.randn(m, k, device="cuda")
    b32 = torch.randn(k, n, device="cuda")
    us = bench(lambda: torch.mm(a32, b32))
    print(f"{name} sgemm: {us:.1f} us, {fl / us / 1e6:.0f} TF/s", flush=True)
