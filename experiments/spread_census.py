"""Which scale groups of the c2 bench step are spread (f16-split.h): conv W
(one group), the FC operands' rows / columns, from the bench's own initial
parameters and synthetic data (numpy on the host copies)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch, kcnn, bench

kcnn.init(0); kcnn.set_randn_seed(20261015)
net = kcnn.Nnet(bench.stack_config())
conv, pool, fc = net.components
def ebits(b):
    b = b.astype(np.int64)
    return np.where(b >= 0x00800000, (b >> 23) - 127, np.floor(np.log2(np.maximum(b, 1))) - 149)
def spread_frac(x, axis):
    a = np.abs(x).view(np.uint32) if x.dtype == np.float32 else None
    bits = np.abs(x).astype(np.float32).view(np.uint32)
    mx = bits.max(axis=axis)
    nz = np.where(bits > 0, bits, np.uint32(0xffffffff)).min(axis=axis)
    sp = (nz != 0xffffffff) & (ebits(nz) < ebits(mx) - 20)
    return int(sp.sum()), sp.size
W = conv.LinearParams().cpu().numpy()
print("conv W spread:", spread_frac(W.ravel(), 0))
Wf = fc.LinearParams().cpu().numpy()
print("fc W rows (fwd op(B) cols):", spread_frac(Wf, 1), " fc W cols (dgrad op(B)):", spread_frac(Wf, 0))
g = torch.Generator(device="cuda"); g.manual_seed(20261015)
x = torch.randn((4096, 1320), generator=g, device="cuda")
net.Propagate(x)
P = net.Output(1).cpu().numpy()
print("P rows:", spread_frac(P, 1), " P cols:", spread_frac(P, 0))
