"""Probe: fp32 GEMM as an exact 3-way bf16 split (bf16x6 / bf16x9) on the bf16
MFMA path, against rocBLAS/hipBLASLt fp32 sgemm, at the c2 FC shapes.

x = h + m + l exactly (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m)); a product
a*b is the sum of the nine h/m/l cross products, each exact in fp32.  bf16x6 keeps
the six down to 2^-16 relative (hh, hm, mh, mm, hl, lh); the dropped ones are
< 2^-24 relative.  Error is measured against fp64 with the dot-product scale
S = |A| |B| (tests/_util.py's bound)."""
import time
import torch

torch.manual_seed(0)
dev = "cuda"


def split3(x):
    h = x.bfloat16()
    r = x - h.float()
    m = r.bfloat16()
    l = (r - m.float()).bfloat16()
    return h, m, l


PAIRS = {"x6": [(0, 0), (0, 1), (1, 0), (1, 1), (0, 2), (2, 0)],
         "x9": [(i, j) for i in range(3) for j in range(3)],
         "x3": [(0, 0), (0, 1), (1, 0)]}


def kcat(a3, b3, pairs):
    A = torch.cat([a3[i] for i, _ in pairs], dim=1).contiguous()
    B = torch.cat([b3[j] for _, j in pairs], dim=1).contiguous()
    return A, B


def timeit(f, n=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def err(c, a, b):
    t = a.double() @ b.double().t()
    S = a.double().abs() @ b.double().abs().t()
    e = (c.double() - t).abs()
    return float((e / S.clamp_min(1e-300)).max()), float(e.norm() / t.norm())


# (name, M, N, K): C[M x N] = A[M x K] B[N x K]^T  (the three c2 FC GEMMs)
SHAPES = [("fwd", 4096, 1024, 11616), ("dgrad", 4096, 11616, 1024),
          ("wgrad", 1024, 11616, 4096)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev)
    b = torch.randn(N, K, device=dev) * 0.01
    flop = 2 * M * N * K
    c32 = a @ b.t()
    t32 = timeit(lambda: a @ b.t())
    rows = min(M, 256)
    e32 = err(c32[:rows], a[:rows], b)
    print(f"{name:6s} f32 sgemm   {t32*1e3:7.3f} ms {flop/t32/1e12:7.1f} TF/s  "
          f"max e/S {e32[0]:.2e}  norm {e32[1]:.2e}", flush=True)
    a3, b3 = split3(a), split3(b)
    ts = timeit(lambda: (split3(a), split3(b)))
    for mode, pairs in PAIRS.items():
        A, B = kcat(a3, b3, pairs)
        c = torch.mm(A, B.t(), out_dtype=torch.float32)
        t = timeit(lambda: torch.mm(A, B.t(), out_dtype=torch.float32))
        e = err(c[:rows], a[:rows], b)
        print(f"{name:6s} bf16{mode:3s}    {t*1e3:7.3f} ms {flop/t/1e12:7.1f} TF/s equiv "
              f"({len(pairs)*flop/t/1e12:7.1f} bf16 TF/s)  split {ts*1e3:.3f} ms  "
              f"max e/S {e[0]:.2e}  norm {e[1]:.2e}", flush=True)
        del A, B, c
    del a3, b3
    torch.cuda.empty_cache()
