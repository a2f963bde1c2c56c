"""Generate the committed golden fixtures under tests/golden/ (test data).

  python scripts/make_golden.py

Each fixture holds seeded inputs and the oracle's outputs (oracle/, the CPU
restatement of the reference's CPU branches) in three forms:
  *_f32    the reference's own fp32 evaluation order (accum mode 0),
  *_truth  fp64-accumulated ("truth", accum mode 1),
  *_scale  sum of |terms| of every output (the dot-product error scale S).
The fixtures were cross-checked against an independent PyTorch float64
formulation (tests/torch_ref.py) when generated (see tests/test_oracle.py,
which re-checks them on every CPU test run).  Shapes: SURVEY Appendix A.11
(both Backprop branches, padding, 3-D pooling), N <= 8 frames.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# name: (H, W, C, kh, kw, G, pad_h, pad_w, N)
CONV = {
    "conv_c2": (40, 11, 3, 8, 1, 128, 0, 0, 1),          # BASELINE c2, flip branch
    "conv_nnet_cfg_l1": (40, 21, 1, 40, 4, 16, 0, 0, 3),  # pad-kernel branch
    "conv_c5_C3_pad": (8, 9, 16, 3, 3, 8, 1, 1, 2),      # padded input
    "conv_c5_C4": (4, 9, 8, 4, 3, 16, 0, 0, 3),          # pad-kernel branch
    "conv_small_pad": (5, 6, 2, 3, 3, 5, 1, 2, 4),
    "conv_tiny": (3, 4, 1, 2, 2, 3, 0, 0, 8),
}
# name: (H, W, C, ph, pw, pc, overlap, overlap2D, N)
POOL = {
    "pool_c2": (33, 11, 128, 1, 1, 4, False, False, 2),
    "pool_c5_P1": (33, 11, 16, 3, 1, 4, False, False, 2),
    "pool_c5_P2": (8, 9, 16, 2, 1, 4, False, False, 3),
    "pool_overlap": (4, 3, 6, 1, 1, 3, True, False, 3),
    "pool_overlap2D": (2, 3, 16, 1, 1, 2, False, True, 3),
}


def triple(fn):
    out = []
    for mode in (0, 1, 2):
        with O.accum(mode):
            out.append(fn())
    return out


def conv_case(name, cfg, seed):
    H, W, C, kh, kw, G, ph, pw, N = cfg
    r = np.random.default_rng(seed)
    f32 = lambda shape, s=1.0: (r.standard_normal(shape) * s).astype(np.float32)  # noqa: E731
    oc = O.Conv(H, W, C, kh, kw, G, in_pad_height=ph, in_pad_width=pw)
    oc.W, oc.b, oc.prev = f32((kh * kw * C, G), 0.1), f32(G, 0.5), f32((kh * kw * C, G), 0.01)
    W0, b0, p0 = oc.W.copy(), oc.b.copy(), oc.prev.copy()
    x = f32((N, H * W * C))
    y = triple(lambda: oc.propagate(x))
    dy = f32(y[0].shape)
    dx = triple(lambda: oc.backprop(x, dy, update=False))
    gr = triple(lambda: oc.gradient(x, dy))
    with O.accum(1):
        oc.backprop(x, dy, update=True)
    d = dict(cfg=np.array(cfg[:8], np.int32), flip_branch=np.int32(oc.flip_branch()),
             x=x, W=W0, b=b0, prev=p0, dy=dy,
             W_upd=oc.W, b_upd=oc.b, prev_upd=oc.prev)
    for key, (a32, at, asc) in (("y", y), ("dx", dx)):
        d[f"{key}_f32"], d[f"{key}_truth"], d[f"{key}_scale"] = a32, at.astype(np.float64), asc
    d["gW_f32"], d["gW_truth"], d["gW_scale"] = gr[0][0], gr[1][0].astype(np.float64), gr[2][0]
    d["gb_f32"], d["gb_truth"], d["gb_scale"] = gr[0][1], gr[1][1].astype(np.float64), gr[2][1]
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)


def pool_case(name, cfg, seed):
    H, W, C, ph, pw, pc, ov, ov2, N = cfg
    r = np.random.default_rng(seed)
    op = O.Pool(H, W, C, ph, pw, pc, overlap=ov, overlap2D=ov2)
    x = (r.integers(-7, 8, size=(N, H * W * C)) * 0.25).astype(np.float32)  # ties
    y = op.propagate(x)
    dp = r.standard_normal(y.shape).astype(np.float32)
    dx = op.backprop(x, y, dp)
    np.savez_compressed(os.path.join(OUT, name + ".npz"),
                        cfg=np.array(cfg[:6] + (int(ov), int(ov2)), np.int32),
                        x=x, y=y, dp=dp, dx=dx)


def main():
    os.makedirs(OUT, exist_ok=True)
    for i, (name, cfg) in enumerate(CONV.items()):
        conv_case(name, cfg, 1000 + i)
    for i, (name, cfg) in enumerate(POOL.items()):
        pool_case(name, cfg, 2000 + i)
    total = sum(os.path.getsize(os.path.join(OUT, f)) for f in os.listdir(OUT))
    print(f"wrote {len(CONV) + len(POOL)} fixtures, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
