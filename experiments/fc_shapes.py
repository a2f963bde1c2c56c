"""c2's three FC GEMM shapes (forward, data gradient, weight gradient), N
calls each through kcnn_gemm (statistics launches included), timed by HIP
events on the library's stream; run under a kernel trace for per-kernel
times.  KCNN_LIB picks the library build.
  python experiments/fc_shapes.py [calls]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch
import kcnn

SHAPES = [("fwd", 4096, 1024, 11616, False, True),
          ("dgrad", 4096, 11616, 1024, False, False),
          ("wgrad", 1024, 11616, 4096, True, False)]


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    kcnn.init(0)
    kcnn.set_gemm_mode(2)
    g = torch.Generator(device="cuda").manual_seed(5)
    for name, m, n, k, ta, tb in SHAPES:
        a = torch.randn((k, m) if ta else (m, k), device="cuda", generator=g)
        b = torch.randn((n, k) if tb else (k, n), device="cuda", generator=g) * 0.01
        c = torch.zeros(m, n, device="cuda")
        for _ in range(3):
            kcnn.gemm(a, b, c, ta, tb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(calls):
            kcnn.gemm(a, b, c, ta, tb)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / calls
        print(f"{name} {m}x{n}x{k}: {us:.1f} us per call, "
              f"{2 * m * n * k / us / 1e6:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
