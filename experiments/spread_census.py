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
# r05: pool_count_kernel's suspect frames (row min below 2^(E - 17), E the
# largest value's binade) and the small elements they hold per column
bits = np.abs(P).view(np.uint32).astype(np.int64)
gm = bits.max()
eg = int(ebits(np.array([max(gm, 0x7fffff)]))[0]) - 17
rmin = np.where(bits > 0, bits, 0xffffffff).min(1)
sus = (rmin != 0xffffffff) & (ebits(rmin) < eg)
ecol = ebits(((bits >> 23).max(0) << 23) | 0x7fffff)
small = (bits != 0) & (ebits(np.maximum(bits, 1)) < ecol[None, :] - 17)
print("suspect frames:", int(sus.sum()), "of", P.shape[0], " small elements:", int(small.sum()),
      " columns with one:", int(small.any(0).sum()), " E:", eg + 17)
U = P.shape[1] // 363
segmin = np.where(bits > 0, bits, 0xffffffff).reshape(P.shape[0], U, 363).min(2)
ecolU = ecol.reshape(U, 363).max(1)
print("suspect (frame, channel) segments:", int(((segmin != 0xffffffff) & (ebits(segmin) < ecolU[None, :] - 17)).sum()),
      "of", P.shape[0] * U)
