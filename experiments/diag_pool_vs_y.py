"""The check of test_pooled_backward_across_frames repeated: a fused Conv ->
Maxpool forward at 601 frames, its pooled output against the oracle's
maxpool of the conv output (mode 1: the output recomputed by the unfused
conv; mode 2: stored by the fused kernel itself).  STACK, REPS, MODE."""
import os, sys
for d in ("tests", "kaldi-cnn_amd", "oracle"):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", d))
import numpy as np
import kcnn as kc
import oracle as O
from _util import dev, host, randn, rng
from test_gpu_nnet import STACKS, build

name = os.environ.get("STACK", "halfB_G96_2x1x4")
REPS = int(os.environ.get("REPS", "40"))
mode = int(os.environ.get("MODE", "1"))
kc.init(0)
cfg = STACKS[name]
H, W, C, kh, kw, G, pc, fo, ph, pw = cfg[:10]
qh, qw = (cfg[10], cfg[11]) if len(cfg) > 10 else (1, 1)
oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
kc.set_fusion(mode)
net = build(kc, cfg, seed=11)
x = dev(randn(rng(3), (601, net.components[0].InputDim())))
events = 0
for rep in range(REPS):
    net.Propagate(x)
    p = host(net.Output(1))
    y = host(net.Output(0))
    ref = O.maxpool_prop(y, oh, ow, qh, qw, pc, p.shape[1])
    d = p != ref
    if d.any():
        events += 1
        fr, col = np.nonzero(d)
        print(f"rep {rep}: {int(d.sum())} differ, first (frame, col) {list(zip(fr[:4].tolist(), col[:4].tolist()))}", flush=True)
kc.set_fusion(1)
print(f"{name} mode {mode}: {events}/{REPS} calls with pooled != maxpool(Y)", flush=True)
