"""f16x3 GEMM time against K around nnet.config's last FC dX (M = N = 4096,
K = 3454 is not a multiple of the 32-deep K step): a ragged K's cost.
Prints one line per (K, layout)."""
import sys
import torch
sys.path.insert(0, "kaldi-cnn_amd")
import kcnn

kcnn.init(0)
kcnn.set_gemm_mode(2)
for K, pitch in ((3454, 0), (3454, 2), (3456, 0), (4096, 0)):
    for name, ta, tb in (("dX", False, False), ("fwd", False, True)):
        m = n = 4096
        a = torch.randn(m, K + pitch, device="cuda")[:, :K]
        b = (torch.randn(n, K + pitch, device="cuda")[:, :K] if tb
             else torch.randn(K, n, device="cuda")) * 0.01
        c = torch.empty(m, n, device="cuda")
        for _ in range(3):
            kcnn.gemm(a, b, c, ta, tb, 1.0, 0.0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            kcnn.gemm(a, b, c, ta, tb, 1.0, 0.0)
        e1.record()
        torch.cuda.synchronize()
        print(f"K={K} pitch+{pitch} {name}: {e0.elapsed_time(e1) / 10 * 1000:.1f} us per call (stats included)",
              flush=True)
