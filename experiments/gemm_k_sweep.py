"""The f16x3 GEMM's per-tile overhead: c2's data-gradient shape (M 4096, N
11616, B row-contiguous) at several K, 20 calls each, under a kernel trace
(the main loop's time per tile is a + b * K steps; a is the prologue +
epilogue).  Prints nothing itself; read the trace."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch
import kcnn

kcnn.init(0)
kcnn.set_gemm_mode(2)
for k in (256, 512, 1024, 2048):
    a = torch.randn((4096, k), device="cuda")
    b = torch.randn((k, 11616), device="cuda") * 0.01
    c = torch.zeros(4096, 11616, device="cuda")
    for _ in range(20):
        kcnn.gemm(a, b, c, False, False)
    torch.cuda.synchronize()
    print("K", k, "done", flush=True)
