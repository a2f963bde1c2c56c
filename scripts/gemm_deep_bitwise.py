"""Bitwise comparison of FC GEMM kernel generations: run the c2 FC products
(and ragged shapes) once per value of an experiment switch in the
experiment build (libkcnn_timing.so), each in its own process, and compare
the outputs bit for bit.  Default: KCNN_X6_DEEP=0/1 on the bf16x6 engine
(gemm_x6_kernel vs gemm_x6d_kernel); VAR=KCNN_F16X3_FAST GEMM=2 compares
the f16x3 two-phase and fast kernels.

  python scripts/gemm_deep_bitwise.py            # driver: both runs + compare
  python scripts/gemm_deep_bitwise.py run OUT    # one run (env selects the kernel)
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SHAPES = [  # (name, trans_a, trans_b, m, n, k): c2 FC forward, dgrad, wgrad; ragged
    ("fc_fwd", False, True, 4096, 1024, 11616),
    ("fc_dgrad", False, False, 4096, 11616, 1024),
    ("fc_wgrad", True, False, 1024, 11616, 4096),
    ("ragged", False, False, 1000, 1000, 512),
    ("ragged_k", False, True, 1000, 520, 1003),
    ("ragged_t", True, False, 520, 1000, 2021),
]


def run(out):
    sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
    import torch
    import kcnn
    kcnn.set_gemm_mode(int(os.environ.get("GEMM", "1")))
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    res = {}
    for name, ta, tb, m, n, k in SHAPES:
        a = torch.randn((k, m) if ta else (m, k), generator=g, device="cuda")
        b = torch.randn((n, k) if tb else (k, n), generator=g, device="cuda")
        c = torch.empty((m, n), device="cuda")
        kcnn.gemm(a, b, c, trans_a=ta, trans_b=tb)
        torch.cuda.synchronize()
        res[name] = c.cpu().numpy()
    np.savez(out, **res)


def main():
    lib = os.path.join(ROOT, "kaldi-cnn_amd", "libkcnn_timing.so")
    outs = []
    for v in (0, 1):
        out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gemm_deep{v}.npz")
        env = dict(os.environ, KCNN_LIB=lib)
        env[os.environ.get("VAR", "KCNN_X6_DEEP")] = str(v)
        subprocess.run([sys.executable, __file__, "run", out], env=env, check=True, timeout=300)
        outs.append(np.load(out))
    bad = 0
    for name, *_ in SHAPES:
        x, y = outs[0][name], outs[1][name]
        same = np.array_equal(x.view(np.uint32), y.view(np.uint32))
        bad += not same
        print(f"{name}: {'bitwise equal' if same else 'DIFFERENT'} {x.shape}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        main()
