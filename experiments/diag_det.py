"""Determinism of the frame forward: the same Propagate repeated, diffs located
by (frame, filter, position) -- diagnostic for a nondeterministic result."""
import sys, os
for d in ("tests", "kaldi-cnn_amd", "oracle"):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", d))
import numpy as np
import kcnn as kc
from _util import dev, host, randn, rng
from test_gpu_components import make_pair

SH = {"halfB": (34, 10, 2, 3, 2, 96, 0, 0), "c2": (40, 11, 3, 8, 1, 128, 0, 0),
      "k4g64": (9, 5, 1, 2, 2, 64, 0, 0)}
for name, cfg in SH.items():
    H, W, C, kh, kw, G, _, _ = cfg
    oh, ow = H - kh + 1, W - kw + 1
    P = oh * ow
    for fam in (2, 1):
        kc.set_kernel_family("fwd_x6", fam)
        comp, oc = make_pair(kc, cfg, seed=5)
        x = dev(randn(rng(6), (601, H * W * C)))
        ref = host(comp.Propagate(x))
        bad = 0
        for rep in range(30):
            y = host(comp.Propagate(x))
            d = y != ref
            if d.any():
                bad += 1
                fr, col = np.nonzero(d)
                g, p = col // P, col % P
                if bad <= 4:
                    print(f"{name} fam {fam} rep {rep}: {d.sum()} diffs; frames {sorted(set(fr.tolist()))[:8]} "
                          f"filters {sorted(set(g.tolist()))[:16]} pos {sorted(set(p.tolist()))[:16]} "
                          f"max|d| {np.abs(y - ref)[d].max():.3e} ref {ref[d][:3]} y {y[d][:3]}", flush=True)
        print(f"{name} fam {fam}: {bad} of 30 reps differ", flush=True)
