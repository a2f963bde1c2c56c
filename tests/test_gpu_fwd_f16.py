"""The f16x3 frame-resident conv forward (cnsl-conv-frame.hip, AR = 2) over the
corners of fp32: Inf / NaN operands, operands far below or above 1, and a
dynamic range of 2^120 inside one frame.

The kernel scales W by one power of two and each output position's im2col
column by its own (f16-split.h), so every case below must meet the full
parity bar (elementwise 1e-5 * S and normwise 1e-5) where the
reference's fp32 result is finite, and reproduce the reference's IEEE
pattern (+Inf, -Inf, NaN) where it is not: the frames of such a wave run
plain fp32 sums (fwd_item_fp32).  The Conv -> Maxpool fusion must stay
bit-identical to the unfused pair on the same data.
"""
import numpy as np
import pytest

import oracle as O
from _util import assert_bound, assert_same, dev, host, randn, rng, triple
from test_gpu_components import make_pair
from test_gpu_nnet import build

pytestmark = pytest.mark.gpu

C2 = (40, 11, 3, 8, 1, 128, 0, 0)
K4_G64 = (9, 5, 1, 2, 2, 64, 0, 0)     # Kdim 4: one k16 step, two filter groups
K12_G40 = (10, 6, 2, 3, 2, 40, 0, 0)   # a partial filter group


@pytest.fixture
def f16(kc):
    old = kc.get_kernel_family("fwd_x6")
    kc.set_kernel_family("fwd_x6", 2)
    yield
    kc.set_kernel_family("fwd_x6", old)


def check_pattern(y, y_ref, y_t, y_s, what):
    """Non-finite entries: the reference's exact pattern; the rest: the bound."""
    nan_r, nan = np.isnan(y_ref), np.isnan(y)
    assert (nan == nan_r).all(), f"{what}: NaN pattern differs at {np.argwhere(nan != nan_r)[:5]}"
    inf_r = np.isinf(y_ref)
    assert (np.isinf(y) == inf_r).all(), f"{what}: Inf pattern differs"
    assert (np.sign(y[inf_r]) == np.sign(y_ref[inf_r])).all(), f"{what}: Inf signs differ"
    fin = np.isfinite(y_ref)
    assert_bound(y[fin], y_t[fin], y_s[fin], what=what)


def nonfinite_inputs(r, N, dim):
    x = randn(r, (N, dim))
    x[1, 100] = np.inf                 # one +Inf
    x[2, 700] = -np.inf                # one -Inf
    x[3, 333] = np.nan                 # NaN propagates through the products
    x[4, 40] = np.inf                  # +Inf and -Inf under one output column
    x[4, 41] = -np.inf
    x[5, :] = 0.0                      # Inf * 0 = NaN below
    x[5, 7] = np.inf
    return x


@pytest.mark.parametrize("name", ["c2", "k4_g64", "k12_g40"])
def test_fwd_nonfinite_inputs(kc, f16, name):
    cfg = {"c2": C2, "k4_g64": K4_G64, "k12_g40": K12_G40}[name]
    comp, oc = make_pair(kc, cfg, seed=7)
    H, W, C = cfg[:3]
    r = rng(8)
    x = nonfinite_inputs(r, 7, H * W * C) if name == "c2" else randn(r, (7, H * W * C))
    if name != "c2":
        x[2, 3] = np.inf
        x[4, 5] = np.nan
        x[5, 20] = -np.inf
    with np.errstate(invalid="ignore", over="ignore"):
        y_ref = oc.propagate(x)
        _, y_t, y_s = triple(lambda: oc.propagate(x))
    y = host(comp.Propagate(dev(x)))
    check_pattern(y, y_ref, y_t, y_s, f"{name} Inf/NaN X")


def test_fwd_nonfinite_weights(kc, f16):
    comp, oc = make_pair(kc, C2, seed=9)
    oc.W = oc.W.copy()
    oc.W[3, 5] = np.inf                # every position meets it (filter 5)
    oc.W[10, 77] = -np.inf
    comp.SetParam(kc.PARAM_LINEAR, dev(oc.W))
    r = rng(10)
    x = randn(r, (5, 40 * 11 * 3))
    x[2, 50:60] = 0.0                  # some positions: -Inf * 0 = NaN
    with np.errstate(invalid="ignore", over="ignore"):
        y_ref = oc.propagate(x)
        _, y_t, y_s = triple(lambda: oc.propagate(x))
    y = host(comp.Propagate(dev(x)))
    check_pattern(y, y_ref, y_t, y_s, "c2 Inf W")


@pytest.mark.parametrize("scale", [2.0 ** -120, 2.0 ** -60, 2.0 ** 60, 3.0e36])
def test_fwd_scaled_inputs_zero_bias(kc, f16, scale):
    """With b = 0 the output is the conv sum alone, so a lost low part would
    show; the full bar (normwise 1e-5) applies."""
    comp, oc = make_pair(kc, C2, seed=11)
    oc.b = np.zeros_like(oc.b)
    comp.SetParam(kc.PARAM_BIAS, dev(oc.b))
    r = rng(12)
    x = (randn(r, (6, 40 * 11 * 3)) * np.float32(scale)).astype(np.float32)
    _, y_t, y_s = triple(lambda: oc.propagate(x))
    assert np.isfinite(y_t).all()
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"c2 x * {scale:g}")


def test_fwd_frame_dynamic_range(kc, f16):
    """Positions of one frame 2^120 apart: each column carries its own scale."""
    comp, oc = make_pair(kc, C2, seed=13)
    r = rng(14)
    x = randn(r, (4, 40 * 11 * 3))
    ramp = np.float32(2.0) ** np.linspace(-60, 60, 40).round().astype(np.float32)
    x = (x.reshape(4, 3, 11, 40) * ramp[None, None, None, :]).reshape(4, -1).astype(np.float32)
    _, y_t, y_s = triple(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what="c2 2^+-60 ramp")


@pytest.mark.parametrize("fusion", [1, 2])
def test_fused_forward_nonfinite_is_exact(kc, f16, fusion):
    """Conv -> Maxpool fused (mask from registers) vs unfused on frames whose
    waves take the fp32 items: the same Y, so the same pool and mask."""
    from test_gpu_nnet import STACKS
    outs = {}
    for fused in (fusion, 0):
        kc.set_fusion(fused)
        try:
            net = build(kc, STACKS["c2"], seed=21)
            x = nonfinite_inputs(rng(22), 9, net.components[0].InputDim())
            x[6:] = randn(rng(23), (3, x.shape[1]))   # frames 6..8 all finite
            net.Propagate(dev(x))
            outs[fused] = [host(net.Output(i)) for i in range(2)]
        finally:
            kc.set_fusion(1)
    for k in range(2):
        assert_same(outs[fusion][k], outs[0][k], f"fusion {fusion} output {k}")
    # the finite frames are untouched by their neighbours' Inf
    y = outs[0][0]
    assert np.isfinite(y[6:]).all() and np.isfinite(y[0]).all()


@pytest.mark.parametrize("group", ["W", "position"])
@pytest.mark.parametrize("spread", [24, 28, 32])
def test_fwd_intra_group_range(kc, f16, group, spread):
    """The forward's scale groups (one for all of W, one per output
    position's im2col column) with their largest element meeting zeros in
    the other operand and every other element 2^-spread below it; bias 0, so
    the small elements carry all of S.  group "W": W's
    channel-0 rows are 1, the rest N(0,1) * 2^-spread, X's channel 0 is 0;
    "position": X's channel 0 is 1 (each position's largest taps), channels
    1-2 N(0,1) * 2^-spread, W's channel-0 rows 0."""
    comp, oc = make_pair(kc, C2, seed=41)
    r = rng(42 + spread)
    x = randn(r, (6, 40 * 11 * 3)).reshape(6, 3, 11 * 40)
    Wm = randn(r, (24, 128), 0.01)
    if group == "W":
        Wm[:8] = 1.0                      # channel 0's 8 taps (row c*8 + ky)
        Wm[8:] *= np.float32(2.0 ** -spread)
        x[:, 0] = 0.0
    else:
        Wm[:8] = 0.0
        x[:, 0] = 1.0
        x[:, 1:] *= np.float32(2.0 ** -spread)
    x = x.reshape(6, -1).astype(np.float32)
    oc.W = Wm.astype(np.float32)
    oc.b = np.zeros_like(oc.b)
    comp.SetParam(kc.PARAM_LINEAR, dev(oc.W))
    comp.SetParam(kc.PARAM_BIAS, dev(oc.b))
    _, y_t, y_s = triple(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"{group} spread 2^{spread}")


@pytest.mark.parametrize("cfg", [(34, 10, 2, 3, 2, 96, 0, 0), C2], ids=["G96_k12", "c2"])
def test_fwd_repeat_bitwise(kc, f16, cfg):
    """Repeated forwards of one 601-frame input are bitwise equal (DESIGN §3,
    the r04 nondeterminism: one accumulator register of 16 lanes wrong in
    about one call in four with the column max through v_permlane32_swap and
    the split's v_fma_mix as inline asm; the product build takes ds_bpermute
    and a compiler-visible split)."""
    comp, _ = make_pair(kc, cfg, seed=5)
    H, W, C = cfg[:3]
    x = dev(randn(rng(6), (601, H * W * C)))
    y0 = host(comp.Propagate(x))
    for rep in range(12):
        assert_same(host(comp.Propagate(x)), y0, f"repeat {rep}")
