"""Error events of the frame forward over repeated Propagate calls against a
3-call majority (nondeterminism hunt).  KCNN_LIB picks the library."""
import sys, os
for d in ("tests", "kaldi-cnn_amd", "oracle"):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", d))
import numpy as np
import kcnn as kc
from _util import dev, host, randn, rng
from test_gpu_components import make_pair

SH = {"halfB": (34, 10, 2, 3, 2, 96, 0, 0), "c2": (40, 11, 3, 8, 1, 128, 0, 0),
      "k4g64": (9, 5, 1, 2, 2, 64, 0, 0), "g40": (10, 6, 2, 3, 2, 40, 0, 0)}
cfg = SH[os.environ.get("SHAPE", "halfB")]
H, W, C, kh, kw, G, _, _ = cfg
P = (H - kh + 1) * (W - kw + 1)
REPS = int(os.environ.get("REPS", "40"))
fam = int(os.environ.get("FAM", "2"))
kc.set_kernel_family("fwd_x6", fam)
comp, oc = make_pair(kc, cfg, seed=5)
x = dev(randn(rng(6), (601, H * W * C)))
a, b, c = (host(comp.Propagate(x)) for _ in range(3))
ref = np.where(a == b, a, c)
events = 0; elems = 0; where = []
for rep in range(REPS):
    y = host(comp.Propagate(x))
    d = y != ref
    if d.any():
        events += 1; elems += int(d.sum())
        fr, col = np.nonzero(d)
        where.append((int(fr[0]), int(col[0] // P), int(col[0] % P), int(d.sum())))
print(f"{os.environ.get('SHAPE', 'halfB')} {os.path.basename(os.environ.get('KCNN_LIB', 'libkcnn.so'))} fam {fam}: {events}/{REPS} calls with errors, "
      f"{elems} elements; first: {where[:6]}", flush=True)
