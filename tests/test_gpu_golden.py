"""The HIP path against the committed golden fixtures (tests/golden/, made by
scripts/make_golden.py from the oracle and cross-checked against torch fp64
on the CPU side, tests/test_oracle.py).  No oracle call at run time: these
compare the GPU results with stored truth + error scale only."""
import glob
import os

import numpy as np
import pytest

from _util import assert_bound, assert_same, dev, host

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONV_FIX = sorted(glob.glob(os.path.join(GOLDEN, "conv_*.npz")))
POOL_FIX = sorted(glob.glob(os.path.join(GOLDEN, "pool_*.npz")))


def _conv_line(H, W, C, kh, kw, G, ph, pw):
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    return (f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} "
            f"in-pad-height={ph} in-pad-width={pw} kernel-height={kh} "
            f"kernel-width={kw} stride=1 group={G} out-height={oh} out-width={ow} "
            f"learning-rate=0.02")


@pytest.mark.parametrize("literal", [False, True], ids=["fused", "literal"])
@pytest.mark.parametrize("path", CONV_FIX, ids=[os.path.basename(p)[:-4] for p in CONV_FIX])
def test_conv_golden(kc, path, literal):
    f = np.load(path)
    cfg = tuple(int(v) for v in f["cfg"])
    kc.set_literal_path(literal)
    try:
        comp = kc.Component.NewFromString(_conv_line(*cfg))
        assert comp.FlipKernelBranch() == bool(f["flip_branch"])
        comp.SetParam(kc.PARAM_LINEAR, dev(f["W"]))
        comp.SetParam(kc.PARAM_BIAS, dev(f["b"]))
        comp.SetParam(kc.PARAM_PREV_GRAD, dev(f["prev"]))
        x, dy = dev(f["x"]), dev(f["dy"])
        assert_bound(host(comp.Propagate(x)), f["y_truth"], f["y_scale"], what="y")
        assert_bound(host(comp.Backprop(x, None, dy, update=False)), f["dx_truth"],
                     f["dx_scale"], what="dX")
        kd, G = f["W"].shape
        g = host(comp.ComputeGradient(x, dy))
        assert_bound(g[:kd * G].reshape(kd, G), f["gW_truth"], f["gW_scale"], what="gW")
        assert_bound(g[kd * G:], f["gb_truth"], f["gb_scale"], what="gb")
        comp.Backprop(x, None, dy, update=True)
        lr = 0.02 / f["x"].shape[0]
        sW = np.abs(f["W"]) + np.abs(f["prev"]) + lr * f["gW_scale"] + 1e-30
        assert_bound(host(comp.LinearParams()), f["W_upd"], sW, what="W'")
        assert_bound(host(comp.BiasParams()), f["b_upd"], np.abs(f["b"]) + lr * f["gb_scale"],
                     what="b'")
    finally:
        kc.set_literal_path(False)


@pytest.mark.parametrize("path", POOL_FIX, ids=[os.path.basename(p)[:-4] for p in POOL_FIX])
def test_pool_golden(kc, path):
    f = np.load(path)
    H, W, C, ph, pw, pc, ov, ov2 = (int(v) for v in f["cfg"])
    line = (f"MaxpoolComponent in-height={H} in-width={W} in-channel={C} "
            f"pool-height-dim={ph} pool-width-dim={pw} pool-channel-dim={pc}"
            + (" overlap=true" if ov else "") + (" overlap2D=true" if ov2 else ""))
    comp = kc.Component.NewFromString(line)
    x = dev(f["x"])
    y = comp.Propagate(x)
    assert_same(host(y), f["y"], "maxpool fwd")
    assert_same(host(comp.Backprop(x, y, dev(f["dp"]))), f["dx"], "maxpool bwd")
