"""Fused vs unfused at 601 frames on one stack: which outputs / derivs differ,
and in which frames (diagnostic for test_pooled_backward_across_frames)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kaldi-cnn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np
import kcnn as kc
from test_gpu_nnet import STACKS, run

name = sys.argv[1] if len(sys.argv) > 1 else "halfB_G96_2x1x4"
for fam in (2, 1):
    kc.set_kernel_family("fwd_x6", fam)
    for rep in range(2):
        a = run(kc, STACKS[name], fused=True, N=601)
        b = run(kc, STACKS[name], fused=False, N=601)
        msg = []
        for grp, (A, B) in (("out", (a[0], b[0])), ("deriv", (a[1], b[1])), ("param", (a[2], b[2]))):
            for k, (u, v) in enumerate(zip(A, B)):
                d = ~((u == v) | (np.isnan(u) & np.isnan(v)))
                if d.any():
                    rows = np.unique(np.nonzero(d)[0]) if d.ndim == 2 else []
                    msg.append(f"{grp}{k}: {d.sum()} diff, frames {list(rows[:12])}")
        print(f"fwd_x6={fam} rep {rep}:", "; ".join(msg) or "all equal", flush=True)
