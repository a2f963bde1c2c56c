"""r06 diagnostic: normwise error of AddMatMat over long K (the weight
gradient's reduction over frames) per engine, against float64, beside torch's
fp32 matmul.  Operand pattern of a weight gradient: op(A) = dY^T, op(B) = X."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch
import kcnn as kc
kc.init(0)
torch.backends.cuda.matmul.allow_tf32 = False
g = torch.Generator(device="cuda"); g.manual_seed(1)
M, N = 512, 1024
for K in (4096, 16384, 65536, 262144):
    dy = torch.randn((K, M), generator=g, device="cuda") * 1e-2
    x = torch.randn((K, N), generator=g, device="cuda")
    t = dy.double().t() @ x.double()
    res = []
    for mode in (2, 1, 0):
        kc.set_gemm_mode(mode)
        c = torch.zeros((M, N), device="cuda")
        kc.gemm(dy, x, c, True, False, 1.0, 0.0)
        torch.cuda.synchronize()
        res.append(float((c.double() - t).norm() / t.norm()))
    kc.set_gemm_mode(2)
    c32 = dy.t() @ x
    e32 = float((c32.double() - t).norm() / t.norm())
    print(f"K {K:7d}: f16x3 {res[0]:.2e}  bf16x6 {res[1]:.2e}  rocBLAS {res[2]:.2e}  torch fp32 {e32:.2e}", flush=True)
