"""The kernel-family selectors (kcnn.set_kernel_family, include/kcnn.h;
kaldi-lite/kcnn-knobs.h) against the oracle: every family switched to its
fp32-MFMA implementation (and the weight gradient's 128-wide bf16x6 kernel,
the implicit GEMM's bf16x6 form beside its f16x3 default)
must meet the same parity bar as the default kernels (and the forward's
bf16x6 form beside its f16x3 default), on shapes that reach each family (c2, c5 layers, nnet.config layer 1, the FC GEMM)."""
import numpy as np
import pytest

import oracle as O
from _util import assert_bound, dev, host, randn, rng, triple
from test_gpu_components import make_pair

pytestmark = pytest.mark.gpu

FAMILY_SHAPES = {
    # family, value: shapes (H, W, C, kh, kw, G, pad_h, pad_w) that reach it
    ("fwd_x6", 0): [(40, 11, 3, 8, 1, 128, 0, 0)],
    ("fwd_x6", 1): [(40, 11, 3, 8, 1, 128, 0, 0), (9, 5, 1, 2, 2, 64, 0, 0)],
    ("bwd_x6", 0): [(40, 11, 3, 8, 1, 128, 0, 0), (40, 11, 3, 8, 1, 256, 0, 0)],
    ("igemm_x6", 0): [(8, 9, 256, 3, 3, 256, 1, 1), (40, 21, 1, 40, 4, 128, 0, 0)],
    ("igemm_x6", 1): [(8, 9, 256, 3, 3, 256, 1, 1), (40, 21, 1, 40, 4, 128, 0, 0)],
    ("wgrad_x6", 0): [(8, 9, 256, 3, 3, 256, 1, 1), (4, 9, 64, 4, 3, 256, 0, 0)],
    ("wgrad_x6", 1): [(8, 9, 256, 3, 3, 256, 1, 1), (11, 11, 64, 4, 3, 256, 0, 0)],
}


@pytest.fixture
def family(kc, request):
    name, value = request.param
    old = kc.get_kernel_family(name)
    kc.set_kernel_family(name, value)
    yield name, value
    kc.set_kernel_family(name, old)


@pytest.mark.parametrize("family,cfg", [(f, c) for f, cs in FAMILY_SHAPES.items() for c in cs],
                         indirect=["family"])
def test_conv_family(kc, family, cfg):
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=G + kh)
    r = rng(17 + C)
    N = 11
    x = randn(r, (N, H * W * C))
    _, y_t, y_s = triple(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"{family} Propagate")
    dy = randn(r, y_t.shape)
    _, dx_t, dx_s = triple(lambda: oc.backprop(x, dy, update=False))
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: oc.gradient(x, dy))
    dx, g = comp.BackpropGradient(dev(x), dev(dy))
    g = host(g)
    kd = kh * kw * C
    assert_bound(host(dx), dx_t, dx_s, what=f"{family} dX")
    assert_bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{family} gW")
    assert_bound(g[kd * G:], gb_t, gb_s, what=f"{family} gb")
    g2 = host(comp.ComputeGradient(dev(x), dev(dy)))
    assert_bound(g2[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{family} gW (gradient only)")


@pytest.mark.parametrize("family", [("gemm", 0)], indirect=True)
def test_fc_family(kc, family):
    I, Od, N = 1000, 130, 300
    comp = kc.Component.NewFromString(
        f"FullyConnectedComponent input-dim={I} output-dim={Od} learning-rate=0.02 "
        f"param-stddev=0.01 bias-stddev=1 weight-decay=0.0002 momentum=0.9")
    r = rng(23)
    of = O.FC(I, Od)
    of.W = randn(r, (Od, I), 0.05)
    of.b = randn(r, (Od,), 0.5)
    of.prev = np.zeros((Od, I), np.float32)
    for which, v in ((0, of.W), (1, of.b), (2, of.prev)):
        comp.SetParam(which, dev(v))
    x = randn(r, (N, I))
    _, y_t, y_s = triple(lambda: of.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what="FC Propagate (sgemm)")
    dy = randn(r, (N, Od))
    _, dx_t, dx_s = triple(lambda: of.backprop(x, dy, update=False))
    _, (gW_t, _), (gW_s, _) = triple(lambda: of.gradient(x, dy))
    g = host(comp.ComputeGradient(dev(x), dev(dy)))
    assert_bound(g[:Od * I].reshape(Od, I), gW_t, gW_s, what="FC gW (sgemm)")
    dx = comp.Backprop(dev(x), None, dev(dy), update=False)
    assert_bound(host(dx), dx_t, dx_s, what="FC dX (sgemm)")
