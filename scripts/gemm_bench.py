"""Time CuMatrixBase::AddMatMat (kcnn_gemm) at the c2 FC shapes in gemm mode 0
(rocBLAS sgemm) and 1 (bf16x6 split kernel)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch
import kcnn

kcnn.init(0)
SHAPES = [("fwd", 4096, 1024, 11616, False, True), ("dgrad", 4096, 11616, 1024, False, False),
          ("wgrad", 1024, 11616, 4096, True, False)]
if len(sys.argv) > 1:
    SHAPES = [s for s in SHAPES if s[0] in sys.argv[1:]]
for name, m, n, k, ta, tb in SHAPES:
    a = torch.randn((k, m) if ta else (m, k), device="cuda")
    b = torch.randn((n, k) if tb else (k, n), device="cuda") * 0.01
    c = torch.zeros(m, n, device="cuda")
    if "p" in os.environ.get("GEMM_MODES", "0,1"):
        ap, bp = kcnn.split_planes(a), kcnn.split_planes(b)
        for _ in range(3):
            kcnn.gemm_planes(ap, bp, c, k, ta, tb)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            kcnn.gemm_planes(ap, bp, c, k, ta, tb)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 20
        t = time.perf_counter()
        for _ in range(20):
            kcnn.split_planes(a)
        torch.cuda.synchronize()
        ds = (time.perf_counter() - t) / 20
        print(f"{name:6s} planes: {dt*1e3:7.3f} ms  {2*m*n*k/dt/1e12:7.1f} TF/s (fp32-equivalent); "
              f"split of A {ds*1e3:.3f} ms (incl. alloc)", flush=True)
    for mode in [int(x) for x in os.environ.get("GEMM_MODES", "0,1").split(",") if x != "p"]:
        kcnn.set_gemm_mode(mode)
        for _ in range(3):
            kcnn.gemm(a, b, c, ta, tb)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            kcnn.gemm(a, b, c, ta, tb)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 20
        print(f"{name:6s} mode {mode}: {dt*1e3:7.3f} ms  {2*m*n*k/dt/1e12:7.1f} TF/s (fp32-equivalent)",
              flush=True)
