"""The bf16x6 kernels over the whole finite fp32 range.

bf16x6 splits each fp32 operand into three bf16 parts (x6-util.h).  Two
corners of fp32 are where such a split can fail:
  * |x| near FLT_MAX: a rounding split makes h = bf16(x) overflow to Inf for
    finite |x| >= 3.3961e38 and the product becomes NaN; the truncating split
    (|h| <= |x|) cannot;
  * |x| below 2^-110: the residual parts m, l fall under bf16's subnormal
    range (its least subnormal is 2^-133, fp32's 2^-149), so the split keeps
    fewer than 24 significant bits (about 13 at 2^-120).
Each case below feeds such operands to the conv forward, the fused backward
(dX and gradient), the implicit GEMM / long weight gradient and the FC GEMM.
Huge operands meet the full parity bar (elementwise 1e-5 * S and normwise
1e-5).  Tiny operands meet the elementwise bound on the bf16x6 kernels (the
normwise error of a cancelling sum is up to ~1e-4 there: DESIGN.md §4, the
bf16x6 contract) and the full bar on the fp32-MFMA kernel families
(kcnn.set_kernel_family(..., 0)), which is what a caller with operands that
small selects.
"""
import numpy as np
import pytest

import oracle as O
from _util import assert_bound, dev, host, randn, rng, triple
import _util
from test_gpu_components import make_pair

pytestmark = pytest.mark.gpu

SHAPES = {
    "c2": (40, 11, 3, 8, 1, 128, 0, 0),          # frame kernels (forward, fused backward)
    "c5_C3": (8, 9, 256, 3, 3, 256, 1, 1),       # implicit GEMM, wide weight gradient
    "c5_C4": (4, 9, 64, 4, 3, 256, 0, 0),        # pad-kernel dX branch
}

HUGE = 3.4e38          # > 3.3961e38: a rounding split of this overflows
TINY = 2.0 ** -120     # residuals below bf16's normal range


def scaled_inputs(kind, r, N, in_dim, out_dim, groups=1):
    """X and dY with one operand at the edge of the range.  Scales keep every
    exact product and sum finite and normal, so the fp32 reference stays
    within its own bound: a huge dY value sits in a different output column
    (map) for every row, so no bias-gradient sum meets two of them."""
    x = randn(r, (N, in_dim))
    dy = randn(r, (N, out_dim))
    if kind == "huge_x":
        x *= 1e-3
        idx = r.integers(0, in_dim, size=(N, 3))
        for n in range(N):
            x[n, idx[n]] = np.float32(HUGE) * np.sign(x[n, idx[n]] + 1e-30)
        dy *= 1e-6
    elif kind == "huge_dy":
        per = out_dim // groups
        for n in range(N):
            col = ((n * 37) % groups) * per + (n * 11) % per
            dy[n, col] = np.float32(HUGE) * (1 if n % 2 else -1)
        x *= 1e-6
    elif kind == "tiny_x":
        x = (x * TINY).astype(np.float32)
    elif kind == "tiny_dy":
        dy = (dy * TINY).astype(np.float32)
    return x, dy


FAMILIES = ("fwd_x6", "bwd_x6", "igemm_x6", "wgrad_x6", "gemm")
CASES = [("huge_x", "x6"), ("huge_dy", "x6"), ("tiny_x", "x6"), ("tiny_dy", "x6"),
         ("tiny_x", "fp32"), ("tiny_dy", "fp32")]


@pytest.fixture
def engine(kc, request):
    """x6: the default kernels; fp32: every family on the fp32-input MFMA."""
    kind, eng = request.param
    old = {f: kc.get_kernel_family(f) for f in FAMILIES}
    if eng == "fp32":
        for f in FAMILIES:
            kc.set_kernel_family(f, 0)
    bound = assert_bound
    if kind.startswith("tiny") and eng == "x6":
        # the bf16x6 contract for operands below 2^-110: elementwise 1e-5 * S,
        # normwise 1e-4
        def bound(a, t, s, rtol=1e-5, what=""):
            _util.assert_bound(a, t, s, rtol=rtol, what=what, norm_rtol=1e-4)
    yield kind, bound
    for f, v in old.items():
        kc.set_kernel_family(f, v)


@pytest.mark.parametrize("engine", CASES, indirect=True, ids=[f"{k}-{e}" for k, e in CASES])
@pytest.mark.parametrize("name", list(SHAPES))
def test_conv_x6_range(kc, name, engine):
    kind, assert_bound = engine
    cfg = SHAPES[name]
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=3)
    if kind.startswith("huge"):
        # weights small so that W * HUGE stays far from overflow in every sum
        oc.W = (oc.W * 1e-3).astype(np.float32)
        comp.SetParam(kc.PARAM_LINEAR, dev(oc.W))
    r = rng(41)
    N = 5
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    x, dy = scaled_inputs(kind, r, N, H * W * C, oh * ow * G, G)
    if kind in ("huge_x", "tiny_x"):
        _, y_t, y_s = triple(lambda: oc.propagate(x))
        assert np.isfinite(y_t).all()
        assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"{name} {kind} Propagate")
    _, dx_t, dx_s = triple(lambda: oc.backprop(x, dy, update=False))
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: oc.gradient(x, dy))
    assert np.isfinite(dx_t).all() and np.isfinite(gW_t).all()
    dx, g = comp.BackpropGradient(dev(x), dev(dy))
    g = host(g)
    kd = kh * kw * C
    assert_bound(host(dx), dx_t, dx_s, what=f"{name} {kind} dX")
    assert_bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{name} {kind} gW")
    assert_bound(g[kd * G:], gb_t, gb_s, what=f"{name} {kind} gb")


@pytest.mark.parametrize("engine", CASES, indirect=True, ids=[f"{k}-{e}" for k, e in CASES])
def test_fc_x6_range(kc, engine):
    kind, assert_bound = engine
    I, Od, N = 2048, 96, 64
    comp = kc.Component.NewFromString(
        f"FullyConnectedComponent input-dim={I} output-dim={Od} learning-rate=0.02 "
        f"param-stddev=0.01 bias-stddev=1 weight-decay=0.0002 momentum=0.9")
    r = rng(5)
    of = O.FC(I, Od)
    of.W = randn(r, (Od, I), 0.05 if not kind.startswith("huge") else 1e-5)
    of.b = randn(r, (Od,), 0.5)
    of.prev = np.zeros((Od, I), np.float32)
    for which, v in ((0, of.W), (1, of.b), (2, of.prev)):
        comp.SetParam(which, dev(v))
    x, dy = scaled_inputs(kind, r, N, I, Od, Od)
    if kind in ("huge_x", "tiny_x"):
        _, y_t, y_s = triple(lambda: of.propagate(x))
        assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"FC {kind} Propagate")
    _, dx_t, dx_s = triple(lambda: of.backprop(x, dy, update=False))
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: of.gradient(x, dy))
    g = host(comp.ComputeGradient(dev(x), dev(dy)))
    assert_bound(g[:Od * I].reshape(Od, I), gW_t, gW_s, what=f"FC {kind} gW")
    assert_bound(g[Od * I:], gb_t, gb_s, what=f"FC {kind} gb")
    dx = comp.Backprop(dev(x), None, dev(dy), update=False)
    assert_bound(host(dx), dx_t, dx_s, what=f"FC {kind} dX")
