"""Normwise and worst elementwise (err / S) error of CuMatrixBase::AddMatMat
at the c2 FC shapes, per engine: rocBLAS sgemm (gemm mode 0), bf16x6 (1),
f16x3 (2), against torch's fp64 product of the same operands, and the ratio
of each to sgemm's (the allowance tests/test_gpu_gemm.py states)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch
import kcnn

kcnn.init(0)
SHAPES = [("fwd", 4096, 1024, 11616, False, True), ("dgrad", 4096, 11616, 1024, False, False),
          ("wgrad", 1024, 11616, 4096, True, False)]
for seed in (1, 2):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    for name, m, n, k, ta, tb in SHAPES:
        a = torch.randn((k, m) if ta else (m, k), device="cuda", generator=g)
        b = torch.randn((n, k) if tb else (k, n), device="cuda", generator=g) * 0.01
        A = (a.t() if ta else a).double()
        B = (b.t() if tb else b).double()
        t = A @ B
        s = A.abs() @ B.abs()
        res = {}
        for mode in (0, 1, 2):
            kcnn.set_gemm_mode(mode)
            c = torch.zeros(m, n, device="cuda")
            kcnn.gemm(a, b, c, ta, tb)
            torch.cuda.synchronize()
            d = c.double() - t
            res[mode] = (float(d.norm() / t.norm()), float((d.abs() / s).max()))
        r0 = res[0][0]
        print(f"seed {seed} {name:6s} " + "  ".join(
            f"mode {md}: norm {v[0]:.3e} ({v[0] / r0:.2f}x sgemm) worst {v[1]:.2e}"
            for md, v in res.items()), flush=True)
kcnn.set_gemm_mode(2)
