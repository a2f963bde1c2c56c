"""CPU tests of the oracle (oracle/, the CPU restatement of the reference's
CPU branches) -- SURVEY 8(c): it is pinned here by
  (i)   hand-derivable known-answer tests,
  (ii)  the committed golden fixtures (tests/golden/, scripts/make_golden.py),
        re-checked against an independent PyTorch float64 formulation
        (tests/torch_ref.py, written from the layout spec, not the loops),
  (iii) the reference's own finite-difference gradient pattern
        (nnet-conv-test.cc:60-210), and
  (iv)  numpy restatements of the reshape helpers.
The reference holds no golden vectors of its own and cannot be built here
(SURVEY 8c), so these are the pins; "parity unpinned" against the reference's
binaries is recorded in DESIGN.md.
"""
import glob
import os

import numpy as np
import pytest

import oracle as O
import torch_ref as T
from _util import assert_bound, assert_same, randn, rng, triple

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---------------------------------------------------------------------------
# (i) known answers

def test_kat_conv2d_single_channel():
    # H=3 x W=2 map, col = h + w*H, values 1..6; kernel 2x1: rows ky=0 -> 10,
    # ky=1 -> 100 (row = c*kh*kw + kx*kh + ky); p = px*oh + py.
    x = np.arange(1, 7, dtype=np.float32).reshape(1, 6)
    k = np.array([[10.0], [100.0]], np.float32)
    y = O.conv2d(x, k, 3, 2, 1, 2, 1, 1)
    assert_same(y, np.array([[210, 320, 540, 650]], np.float32), "conv KAT 1")
    # concat=false: rows p*R + n, one column per group
    y2 = O.conv2d(x, k, 3, 2, 1, 2, 1, 1, concat=False)
    assert_same(y2, np.array([[210], [320], [540], [650]], np.float32), "conv KAT 1 (M)")


def test_kat_conv2d_two_channels_two_groups():
    # H=1, W=3, C=2: x(c,w) = [[1,2,3],[4,5,6]]; kernel 1x2, rows c*2 + kx.
    x = np.array([[1, 2, 3, 4, 5, 6]], np.float32)
    k = np.array([[1, 0], [0, 1], [1, 1], [2, 0]], np.float32)
    y = O.conv2d(x, k, 1, 3, 2, 1, 2, 2)
    assert_same(y, np.array([[15, 19, 6, 8]], np.float32), "conv KAT 2")


def test_kat_conv_component_bias_and_padding():
    # 1x1 kernel with pad 1 on a 2x2 map: the padded ring gives bias only.
    oc = O.Conv(2, 2, 1, 1, 1, 1, in_pad_height=1, in_pad_width=1)
    oc.W = np.array([[2.0]], np.float32)
    oc.b = np.array([0.5], np.float32)
    y = oc.propagate(np.array([[1, 2, 3, 4]], np.float32))
    # 4x4 output, col = py + px*4; interior (1..2, 1..2) = 2*x + 0.5
    exp = np.full((4, 4), 0.5, np.float32)           # [px][py]
    exp[1, 1], exp[1, 2], exp[2, 1], exp[2, 2] = 2.5, 4.5, 6.5, 8.5
    assert_same(y, exp.reshape(1, 16), "conv KAT pad+bias")


def test_kat_maxpool_ties_and_routing():
    # H=2, W=2, C=2, pool 2x1x1: windows (h0,h1) at each (c, w)
    x = np.array([[3, 3, 1, 5, 7, 2, 2, 2]], np.float32)
    y = O.maxpool_prop(x, 2, 2, 2, 1, 1, 4)
    assert_same(y, np.array([[3, 5, 7, 2]], np.float32), "maxpool KAT")
    dp = np.array([[10, 20, 30, 40]], np.float32)
    dx = O.maxpool_backprop(x, y, dp, 2, 2, 2, 1, 1)
    # every tied maximum receives the full derivative (A.9)
    assert_same(dx, np.array([[10, 10, 0, 20, 30, 0, 40, 40]], np.float32), "maxpool bwd KAT")
    # 4-way tie across 2 channels x 2 columns
    x4 = np.ones((1, 4), np.float32)
    y4 = O.maxpool_prop(x4, 1, 2, 1, 2, 2, 1)
    dx4 = O.maxpool_backprop(x4, y4, np.array([[7]], np.float32), 1, 2, 1, 2, 2)
    assert_same(dx4, np.full((1, 4), 7, np.float32), "4-way tie")


def test_kat_maxpool_special_values():
    # A.8: val = -1e20; NaN never wins (val < NaN is false); all below -1e20
    # gives -1e20.
    x = np.array([[np.nan, 2.0, -1e30, -1e25, np.inf, 1.0]], np.float32)
    y = O.maxpool_prop(x, 2, 3, 2, 1, 1, 3)
    assert_same(y, np.array([[2.0, -1e20, np.inf]], np.float32), "maxpool special")


# ---------------------------------------------------------------------------
# (iv) reshape helpers against numpy restatements of Appendix A

def test_reshape_helpers_match_appendix_a():
    r = rng(5)
    kh, kw, C, G, R = 3, 2, 4, 5, 3
    ks = kh * kw
    Wm = randn(r, (ks * C, G))
    flip = O.flip_mat(Wm, kh, kw, C, G)                       # A.3
    exp = np.zeros((ks * G, C), np.float32)
    for g in range(G):
        for rr in range(ks):
            for c in range(C):
                exp[g * ks + rr, c] = Wm[c * ks + (ks - 1 - rr), g]
    assert_same(flip, exp, "FlipMat")

    H0, W0 = 4, 3
    X = randn(r, (R, H0 * W0 * C))
    pad = O.padding_zero(X, H0, W0, C, kh, kw)                # A.4
    PH, PW = H0 + 2 * (kh - 1), W0 + 2 * (kw - 1)
    exp = np.zeros((R, PH * PW * C), np.float32)
    for c in range(C):
        for J in range(PW):
            for I in range(PH):
                if kh - 1 <= I < kh - 1 + H0 and kw - 1 <= J < kw - 1 + W0:
                    exp[:, c * PH * PW + J * PH + I] = X[:, (I - kh + 1) + (J - kw + 1) * H0 + c * H0 * W0]
    assert_same(pad, exp, "PaddingZero")

    bs = 6
    M = randn(r, (R, bs * C))
    tb = O.tp_block(M, C, bs)                                 # A.5
    exp = np.array([[M[j // bs, i * bs + j % bs] for j in range(R * bs)] for i in range(C)],
                   np.float32)
    assert_same(tb, exp, "TpBlock")

    M = randn(r, (R, bs * G))
    tib = O.tp_inside_block(M, G, bs)                         # A.6
    exp = np.array([[M[i // bs, j * bs + i % bs] for j in range(G)] for i in range(bs * R)],
                   np.float32)
    assert_same(tib, exp, "TpInsideBlock")

    M = randn(r, (C * bs, G))
    mp = O.mod_permute_row(M, C, bs)                          # A.7
    exp = np.zeros_like(M)
    for i in range(C * bs):
        exp[(i % C) * bs + i // C] = M[i]
    assert_same(mp, exp, "ModPermuteRow")

    H0, W0, K = 3, 2, 3                                        # conv2D.cc:706-725
    comp = randn(r, (R, C * H0 * W0))
    cont = randn(r, (R, K * C * H0 * W0))
    exp = cont.copy()
    for j in range(C * H0 * W0):
        exp[:, ((j // (H0 * W0)) * K + 1) * H0 * W0 + j % (H0 * W0)] = comp[:, j]
    assert_same(O.mod_permute_channel(comp, 1, K, H0, W0, cont.copy(), True), exp,
                "ModPermuteChannel to container")
    back = O.mod_permute_channel(np.zeros_like(comp), 1, K, H0, W0, exp, False)
    assert_same(back, comp, "ModPermuteChannel from container")

    M = randn(r, (R, G * bs))
    v = randn(r, (G,))
    exp = M + np.repeat(v, bs)[None, :]                        # A.2
    assert_same(O.add_mat_rep_vec(M.copy(), v, bs), exp, "AddMatRepVec")


# ---------------------------------------------------------------------------
# (ii) golden fixtures

CONV_FIX = sorted(glob.glob(os.path.join(GOLDEN, "conv_*.npz")))
POOL_FIX = sorted(glob.glob(os.path.join(GOLDEN, "pool_*.npz")))


def test_golden_present():
    assert len(CONV_FIX) >= 6 and len(POOL_FIX) >= 5, "run scripts/make_golden.py"


def _conv_from(f):
    H, W, C, kh, kw, G, ph, pw = (int(v) for v in f["cfg"])
    oc = O.Conv(H, W, C, kh, kw, G, in_pad_height=ph, in_pad_width=pw)
    oc.W, oc.b, oc.prev = f["W"].copy(), f["b"].copy(), f["prev"].copy()
    return oc, (H, W, C, kh, kw, G, ph, pw)


@pytest.mark.parametrize("path", CONV_FIX, ids=[os.path.basename(p)[:-4] for p in CONV_FIX])
def test_golden_conv_oracle_reproduces(path):
    """The oracle reproduces its fixtures (fp32 bitwise, truth and scale
    to fp64 rounding) and the reference's branch choice (:489-497)."""
    f = np.load(path)
    oc, _ = _conv_from(f)
    assert oc.flip_branch() == bool(f["flip_branch"])
    x, dy = f["x"], f["dy"]
    y = triple(lambda: oc.propagate(x))
    dx = triple(lambda: oc.backprop(x, dy, update=False))
    gr = triple(lambda: oc.gradient(x, dy))
    for key, got in (("y", y), ("dx", dx), ("gW", [g[0] for g in gr]), ("gb", [g[1] for g in gr])):
        assert_same(got[0], f[f"{key}_f32"], f"{key} f32")
        np.testing.assert_allclose(got[1], f[f"{key}_truth"], rtol=1e-6, atol=1e-30)
        np.testing.assert_allclose(got[2], f[f"{key}_scale"], rtol=1e-6, atol=1e-30)
    with O.accum(1):
        oc.backprop(x, dy, update=True)
    np.testing.assert_allclose(oc.W, f["W_upd"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(oc.b, f["b_upd"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(oc.prev, f["prev_upd"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("path", CONV_FIX, ids=[os.path.basename(p)[:-4] for p in CONV_FIX])
def test_golden_conv_against_torch_fp64(path):
    """The fixtures against an independent float64 formulation: truth (fp64
    accumulation, stored as fp32) to a few fp32 ulps of the error scale, fp32
    to the 1e-5 * S parity bound."""
    f = np.load(path)
    H, W, C, kh, kw, G, ph, pw = (int(v) for v in f["cfg"])
    y_t = T.conv_fwd(f["x"], f["W"], f["b"], H, W, C, kh, kw, G, ph, pw)
    dx_t, gW_t, gb_t = T.conv_grads(f["x"], f["W"], f["dy"], H, W, C, kh, kw, G, ph, pw)
    for key, ref in (("y", y_t), ("dx", dx_t), ("gW", gW_t), ("gb", gb_t)):
        assert_bound(f[f"{key}_truth"], ref, f[f"{key}_scale"], rtol=3e-7, what=f"{key} truth")
        assert_bound(f[f"{key}_f32"], ref, f[f"{key}_scale"], rtol=1e-5, what=f"{key} f32")


def test_golden_conv_update_formula():
    """A.12: prev' = m*prev - lr'*wd*W + lr'*gW; W' = W + prev'; b' = b + lr'*gb
    with lr' = lr / N (the reference divides by the local row count)."""
    for path in CONV_FIX:
        f = np.load(path)
        N = f["x"].shape[0]
        lr = 0.02 / N
        prev = 0.9 * f["prev"].astype(np.float64) - lr * 0.0002 * f["W"] + lr * f["gW_truth"]
        np.testing.assert_allclose(f["prev_upd"], prev, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(f["W_upd"], f["W"] + prev, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(f["b_upd"], f["b"] + lr * f["gb_truth"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("path", POOL_FIX, ids=[os.path.basename(p)[:-4] for p in POOL_FIX])
def test_golden_pool(path):
    f = np.load(path)
    H, W, C, ph, pw, pc, ov, ov2 = (int(v) for v in f["cfg"])
    op = O.Pool(H, W, C, ph, pw, pc, overlap=bool(ov), overlap2D=bool(ov2))
    y = op.propagate(f["x"])
    assert_same(y, f["y"], "maxpool fwd")
    assert_same(op.backprop(f["x"], y, f["dp"]), f["dx"], "maxpool bwd")
    if not ov and not ov2:  # torch's max_pool3d has the same non-overlap windows
        assert_same(T.maxpool_fwd(f["x"], H, W, C, ph, pw, pc).astype(np.float32), y, "torch")
    assert (np.abs(f["dx"]).sum(axis=1) > 0).all()


# ---------------------------------------------------------------------------
# (iii) finite differences (the reference's test pattern, nnet-conv-test.cc)

@pytest.mark.parametrize("cfg", [(5, 6, 2, 3, 3, 4, 1, 1), (8, 5, 1, 4, 2, 3, 0, 0),
                                 (40, 11, 3, 8, 1, 8, 0, 0)])
def test_fd_gradients(cfg):
    H, W, C, kh, kw, G, ph, pw = cfg
    r = rng(sum(cfg))
    oc = O.Conv(H, W, C, kh, kw, G, in_pad_height=ph, in_pad_width=pw)
    oc.W, oc.b = randn(r, (kh * kw * C, G), 0.3), randn(r, (G,), 0.5)
    x = randn(r, (2, H * W * C))
    Rw = randn(r, (2, oc.output_dim))                         # objf = sum(y * Rw)

    def objf(xx, WW):
        o2 = O.Conv(H, W, C, kh, kw, G, in_pad_height=ph, in_pad_width=pw)
        o2.W, o2.b = WW, oc.b
        with O.accum(1):
            return float((o2.propagate(xx).astype(np.float64) * Rw).sum())

    with O.accum(1):
        dx = oc.backprop(x, Rw, update=False)
        gW, gb = oc.gradient(x, Rw)
    for _ in range(3):
        dxp = randn(r, x.shape, 1e-3)
        pred = float((dx.astype(np.float64) * dxp).sum())
        obs = objf(x + dxp, oc.W) - objf(x, oc.W)
        assert abs(pred - obs) <= 0.15 * abs(pred + obs) / 2 or abs(pred - obs) < 1e-6
        dWp = randn(r, oc.W.shape, 1e-3)
        pred = float((gW.astype(np.float64) * dWp).sum())
        obs = objf(x, oc.W + dWp) - objf(x, oc.W)
        assert abs(pred - obs) <= 0.05 * abs(pred + obs) / 2 or abs(pred - obs) < 1e-6
    np.testing.assert_allclose(gb, Rw.reshape(2, G, -1).sum(axis=(0, 2)), rtol=1e-5, atol=1e-5)


def test_both_dgrad_branches_agree():
    """A.11: the pad-kernel and flip branches compute the same dX; the
    oracle runs whichever the heuristic picks, so compare two shapes that
    straddle it against torch at fp64 truth."""
    for cfg in [(40, 21, 1, 40, 4, 4, 0, 0), (40, 11, 3, 8, 1, 4, 0, 0)]:
        H, W, C, kh, kw, G, ph, pw = cfg
        r = rng(9)
        oc = O.Conv(H, W, C, kh, kw, G)
        oc.W = randn(r, (kh * kw * C, G), 0.1)
        x = randn(r, (2, H * W * C))
        dy = randn(r, (2, oc.output_dim))
        _, dxt, dxs = triple(lambda: oc.backprop(x, dy, update=False))
        dx_ref, _, _ = T.conv_grads(x, oc.W, dy, H, W, C, kh, kw, G)
        assert_bound(dxt, dx_ref, dxs, rtol=3e-7, what=f"branch flip={oc.flip_branch()}")


def test_fc_oracle_against_numpy():
    r = rng(4)
    fc = O.FC(7, 5)
    fc.W, fc.b = randn(r, (5, 7)), randn(r, (5,))
    x = randn(r, (3, 7))
    with O.accum(1):
        y = fc.propagate(x)
        dy = randn(r, (3, 5))
        dx = fc.backprop(x, dy, update=False)
        gW, gb = fc.gradient(x, dy)
    x64, W64 = x.astype(np.float64), fc.W.astype(np.float64)
    np.testing.assert_allclose(y, x64 @ W64.T + fc.b, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(dx, dy.astype(np.float64) @ W64, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gW, dy.astype(np.float64).T @ x64, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gb, dy.sum(axis=0), rtol=1e-6, atol=1e-6)
