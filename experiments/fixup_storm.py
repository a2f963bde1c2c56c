"""Time the f16x3 GEMM on c2's weight-gradient shape (1024 x 11616 x 4096,
op(A) transposed: split K, op(B) row-contiguous) with 0, 2, 32 and 128 spread
rows of op(A) whose every output the store's check rejects (the construction of
test_gemm_f16x3_intra_group_range), and c2's forward shape (op(B) K-contiguous)
with 0 and 2: the split-K sum defers those rows to gemm_f16x3_fixup_kernel."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch, kcnn

kcnn.init(0)
kcnn.set_gemm_mode(2)
g = torch.Generator(device="cuda")
for name, m, n, k, ta, tb, rows in (("wgrad", 1024, 11616, 4096, True, False, (0, 2, 32, 128)),
                                    ("fwd", 4096, 1024, 11616, False, True, (0, 2, 16))):
    for nr in rows:
        g.manual_seed(5)
        a = torch.randn((k, m) if ta else (m, k), generator=g, device="cuda")
        b = torch.randn((n, k) if tb else (k, n), generator=g, device="cuda")
        A = a.t() if ta else a
        B = b.t() if tb else b
        k0 = k // 3
        for i in range(nr):
            i0 = (i * 997 + 5) % m
            A[i0] = torch.randn(k, generator=g, device="cuda") * 2.0 ** -28
            A[i0, k0] = 1.0
        if nr:
            B[k0, :] = 0.0
        c = torch.empty((m, n), device="cuda")
        for _ in range(3):
            kcnn.gemm(a, b, c, ta, tb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            kcnn.gemm(a, b, c, ta, tb)
        e1.record()
        torch.cuda.synchronize()
        ref = (A.double() @ B.double())
        err = float(((c.double() - ref).abs()).max() / ref.abs().max())
        print(f"{name} spread rows {nr}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per GEMM "
              f"(with statistics), max err / max |C| {err:.2e}", flush=True)
