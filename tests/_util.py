"""Shared helpers for the parity tests."""
import numpy as np

import oracle as O


def rng(seed=0):
    return np.random.default_rng(seed)


def randn(r, shape, scale=1.0):
    return (r.standard_normal(shape) * scale).astype(np.float32)


def with_ties(r, shape, levels=7):
    """Inputs quantised to a few levels so max-pool windows contain ties."""
    return (r.integers(-levels, levels + 1, size=shape) * 0.25).astype(np.float32)


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.detach().float().cpu().numpy()


def padded(a, extra_cols=5):
    """Device copy of `a` with a row stride larger than its width (a pitched
    matrix, as Kaldi's CuMatrix allocates), returned as a column-range view."""
    import torch
    r, c = a.shape
    base = torch.full((r, c + extra_cols), float("nan"), dtype=torch.float32, device="cuda")
    base[:, :c] = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return base[:, :c]


def triple(fn):
    """Run an oracle computation in fp32 (reference order), fp64-accumulated
    ("truth") and |.|-accumulated (error scale S) mode."""
    out = []
    for mode in (0, 1, 2):
        with O.accum(mode):
            out.append(fn())
    return out


def assert_bound(actual, truth, scale, rtol=1e-5, what="", norm_rtol=None):
    """Parity criterion of SURVEY 8(d): |a - t| <= rtol * S elementwise (S =
    sum of |terms|, the dot-product error scale) and normwise
    ||a - t|| / ||t|| <= rtol (norm_rtol when given)."""
    a = np.asarray(actual, np.float64)
    t = np.asarray(truth, np.float64)
    s = np.asarray(scale, np.float64)
    assert a.shape == t.shape, (a.shape, t.shape)
    assert np.isfinite(a).all(), f"{what}: non-finite output"
    err = np.abs(a - t)
    lim = rtol * s + 1e-30
    bad = err > lim
    assert not bad.any(), (
        f"{what}: {bad.sum()} / {bad.size} elements exceed {rtol}*S; "
        f"worst err/S = {(err / np.maximum(s, 1e-30)).max():.3e}")
    nt = np.linalg.norm(t)
    if nt > 0:
        rel = np.linalg.norm(a - t) / nt
        lim_n = rtol if norm_rtol is None else norm_rtol
        assert rel <= lim_n, f"{what}: normwise rel err {rel:.3e} > {lim_n}"


def assert_same(actual, expected, what=""):
    """Bit-exact (value) equality, NaN-aware."""
    a = np.asarray(actual)
    e = np.asarray(expected)
    assert a.shape == e.shape, (what, a.shape, e.shape)
    eq = (a == e) | (np.isnan(a) & np.isnan(e))
    assert eq.all(), f"{what}: {(~eq).sum()} of {eq.size} elements differ"
