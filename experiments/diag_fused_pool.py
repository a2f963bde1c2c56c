"""Repeated Conv -> Maxpool forwards of one test_gpu_nnet stack at 601 frames:
fused (pooled in the conv kernel) vs unfused (conv, then the pool kernel),
each against a 3-call majority of itself, and fused vs unfused; counts the
calls whose outputs differ (nondeterminism hunt).  STACK, REPS, KCNN_LIB."""
import os, sys
for d in ("tests", "kaldi-cnn_amd", "oracle"):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", d))
import numpy as np
import kcnn as kc
from _util import dev, host, randn, rng
from test_gpu_nnet import STACKS, build

name = os.environ.get("STACK", "halfB_G96_2x1x4")
REPS = int(os.environ.get("REPS", "30"))
kc.init(0)
cfg = STACKS[name]
x = None
res = {}
for fused in (1, 0):
    kc.set_fusion(fused)
    net = build(kc, cfg, seed=11)
    if x is None:
        x = dev(randn(rng(3), (601, net.components[0].InputDim())))
    outs = []
    for _ in range(REPS + 3):
        net.Propagate(x)
        outs.append(host(net.Output(1)))  # the pooled output
    ref = np.where(outs[0] == outs[1], outs[0], outs[2])
    bad = [int((o != ref).sum()) for o in outs[3:]]
    res[fused] = ref
    print(f"{name} fusion {fused}: {sum(b > 0 for b in bad)}/{REPS} calls differ "
          f"from the majority, elements {sum(bad)}", flush=True)
kc.set_fusion(1)
d = res[1] != res[0]
print(f"{name} fused vs unfused majority: {int(d.sum())} elements differ; first "
      f"{np.argwhere(d)[:4].tolist()}", flush=True)
