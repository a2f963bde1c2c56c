"""GPU parity of the nnet0 components (reference nnet0/nnet-component-nnet0.cc)
against the CPU oracle: Propagate, Backprop (data gradient, both of the
reference's branches), Update (weight/bias gradient + momentum/decay step),
the FC layer, Read/Write round trips and a finite-difference gradient check
(the reference's own test pattern, nnet0/nnet-conv-test.cc:60-210).

Both execution paths of the product are checked: the fused MI355X kernels
(default) and the literal replay of the reference's CuMatrixBase call
sequence (kcnn.set_literal_path(True)).
"""
import os

import numpy as np
import pytest

import oracle as O
from _util import assert_bound, assert_same, dev, host, randn, rng, triple, with_ties

pytestmark = pytest.mark.gpu

CONVS = {
    # name: (H, W, C, kh, kw, G, pad_h, pad_w)
    "c2": (40, 11, 3, 8, 1, 128, 0, 0),                 # BASELINE c2 (flip branch)
    "nnet_cfg_l1": (40, 21, 1, 40, 4, 128, 0, 0),       # nnet.config:2 (pad-kernel branch)
    "nnet_cfg_l2": (1, 18, 128, 1, 3, 128, 0, 0),       # nnet.config:4
    "c5_C3_pad": (8, 9, 256, 3, 3, 32, 1, 1),           # padded (c5 C3, fewer groups)
    "c5_C4": (4, 9, 64, 4, 3, 256, 0, 0),               # pad-kernel branch
    "small_pad": (5, 6, 2, 3, 3, 5, 1, 2),
    "tiny": (3, 4, 1, 2, 2, 3, 0, 0),
    "c5_C1_G256": (40, 11, 3, 8, 1, 256, 0, 0),         # c5 C1: 128-filter chunks
    # long-kernel weight gradient (conv_wgrad2_kernel): chunks of 32 positions
    "c5_C3": (8, 9, 256, 3, 3, 256, 1, 1),              # P = 72: 3 chunks, padded
    "c5_C2": (11, 11, 64, 4, 3, 256, 0, 0),             # P = 72, no padding
    "nch2_pad": (7, 8, 16, 3, 3, 128, 1, 1),            # P = 56: 2 chunks; Kdim 144
    "fpc2_pad": (4, 4, 32, 3, 3, 128, 1, 1),            # P = 16: 2 frames per chunk
    # implicit-GEMM v2 with its im2col-row table: Kdim not a multiple of 16
    "ig2_tail_g64": (6, 7, 9, 3, 3, 64, 1, 1),          # Kdim 81, one 64-filter tile
    "ig2_tail_g128": (5, 6, 11, 3, 3, 128, 1, 0),       # Kdim 99, pad on one axis
    # scatter-form data gradient (HW >= 1.25 P) on a padded map
    "scatter_pad": (12, 10, 4, 5, 5, 32, 1, 1),          # HW 120, P 80, Kdim 100
    # bf16x6 implicit GEMM / weight gradient edges: partial filter tiles of
    # both tile shapes, Kdim off the 32-step, 5x5 taps on a padded map, P = 2
    "x6_g320_pad": (6, 7, 8, 3, 3, 320, 1, 1),          # 256 + 64 filters, Kdim 72
    "x6_g96_k75": (9, 10, 5, 3, 5, 96, 0, 0),           # 128-row tile, 96 used
    "x6_5x5_pad2": (7, 7, 4, 5, 5, 64, 2, 2),           # 25 taps, pad 2
    "x6_p2": (1, 4, 40, 1, 3, 64, 0, 0),                # P = 2, Kdim 120
}


def conv_line(H, W, C, kh, kw, G, ph, pw, lr=0.02):
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    return (f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} "
            f"in-pad-height={ph} in-pad-width={pw} kernel-height={kh} "
            f"kernel-width={kw} stride=1 group={G} out-height={oh} out-width={ow} "
            f"learning-rate={lr} param-stddev=0.1 bias-stddev=0.5")


def make_pair(kc, cfg, seed):
    H, W, C, kh, kw, G, ph, pw = cfg
    comp = kc.Component.NewFromString(conv_line(*cfg))
    r = rng(seed)
    oc = O.Conv(H, W, C, kh, kw, G, in_pad_height=ph, in_pad_width=pw)
    oc.W = randn(r, (kh * kw * C, G), 0.1)
    oc.b = randn(r, (G,), 0.5)
    oc.prev = randn(r, (kh * kw * C, G), 0.01)  # nonzero momentum state
    comp.SetParam(kc.PARAM_LINEAR, dev(oc.W))
    comp.SetParam(kc.PARAM_BIAS, dev(oc.b))
    comp.SetParam(kc.PARAM_PREV_GRAD, dev(oc.prev))
    return comp, oc


@pytest.fixture(params=["fused", "literal"])
def path(request, kc):
    kc.set_literal_path(request.param == "literal")
    yield request.param
    kc.set_literal_path(False)


@pytest.mark.parametrize("name", list(CONVS))
def test_conv_component(kc, path, name):
    cfg = CONVS[name]
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=len(name))
    assert comp.FlipKernelBranch() == oc.flip_branch()
    N = 9
    r = rng(100 + len(name))
    x = randn(r, (N, H * W * C))
    # Propagate (:423-446)
    f32, y_t, y_s = triple(lambda: oc.propagate(x))
    y = comp.Propagate(dev(x))
    assert_bound(host(y), y_t, y_s, what=f"{name} Propagate")
    # Backprop data gradient (:461-540), no update
    dy = randn(r, y_t.shape)
    _, dx_t, dx_s = triple(lambda: oc.backprop(x, dy, update=False))
    dx = comp.Backprop(dev(x), None, dev(dy), update=False)
    assert_bound(host(dx), dx_t, dx_s, what=f"{name} Backprop dX")
    # Update (:738-777): compare the gradient, then the updated parameters
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: oc.gradient(x, dy))
    g = host(comp.ComputeGradient(dev(x), dev(dy)))
    kd = kh * kw * C
    assert_bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{name} gW")
    assert_bound(g[kd * G:], gb_t, gb_s, what=f"{name} gb")
    W0, b0, p0 = oc.W.copy(), oc.b.copy(), oc.prev.copy()
    with O.accum(1):
        oc.backprop(x, dy, update=True)
    comp.Backprop(dev(x), None, dev(dy), update=True)
    lr = 0.02 / N
    # bound: the update is W + m*prev - lr*wd*W + lr*gW; its rounding error
    # is a few ulps of each term plus lr * (gradient error <= 1e-5 * S).
    scale_W = np.abs(W0) + np.abs(p0) + lr * gW_s + 1e-30
    assert_bound(host(comp.LinearParams()), oc.W, scale_W, what=f"{name} W'")
    assert_bound(host(comp.PrevGrad()), oc.prev, np.abs(p0) + lr * gW_s + 1e-6 * np.abs(W0),
                 what=f"{name} prev'")
    assert_bound(host(comp.BiasParams()), oc.b, np.abs(b0) + lr * gb_s, what=f"{name} b'")


FUSED_BWD = {
    # shapes in the fused single-pass backward's range (kh*kw*C <= 31,
    # group in {32, 64, 96, 128}, 16 <= oh*ow <= 512) and at its edges
    "c2_grid_stride": ((40, 11, 3, 8, 1, 128, 0, 0), 300),  # R > grid
    "even_P": ((41, 11, 1, 8, 3, 64, 0, 0), 7),              # P = 306
    "padded": ((12, 10, 2, 3, 3, 32, 1, 1), 5),              # P = 120, pad 1
    "K31_G96": ((40, 5, 1, 31, 1, 96, 0, 0), 6),             # ones row = 31
    "P512": ((35, 16, 1, 4, 1, 32, 0, 0), 3),                # max positions
    "P16": ((5, 5, 2, 2, 2, 128, 0, 0), 4),                  # min positions
    "oh1": ((8, 40, 1, 8, 3, 64, 0, 0), 5),                  # oh = 1
    "c5_C1_G256": ((40, 11, 3, 8, 1, 256, 0, 0), 6),         # 2 chunks of 128 filters
    "G224": ((9, 7, 2, 2, 3, 224, 0, 0), 5),                 # chunks 128 + 96
}


@pytest.mark.parametrize("name", list(FUSED_BWD))
def test_conv_backprop_gradient(kc, name):
    """BackpropGradient: dX and [gW | gb] from one pass over dY (fused
    kernel) against the oracle's Backprop (:461-540) and Update gradient
    (:738-765); also the gradient-only form and Backprop(update=True)."""
    cfg, N = FUSED_BWD[name]
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=7 + len(name))
    r = rng(200 + len(name))
    x = randn(r, (N, H * W * C))
    f32, y_t, y_s = triple(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"{name} Propagate")
    dy = randn(r, y_t.shape)
    _, dx_t, dx_s = triple(lambda: oc.backprop(x, dy, update=False))
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: oc.gradient(x, dy))
    kd = kh * kw * C
    dx, g = comp.BackpropGradient(dev(x), dev(dy))
    g = host(g)
    assert_bound(host(dx), dx_t, dx_s, what=f"{name} dX")
    assert_bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{name} gW")
    assert_bound(g[kd * G:], gb_t, gb_s, what=f"{name} gb")
    _, g2 = comp.BackpropGradient(dev(x), dev(dy), want_in_deriv=False)
    assert_same(host(g2), g, what=f"{name} gradient-only == fused")  # deterministic
    W0, b0, p0 = oc.W.copy(), oc.b.copy(), oc.prev.copy()
    with O.accum(1):
        oc.backprop(x, dy, update=True)
    dx2 = comp.Backprop(dev(x), None, dev(dy), update=True)
    assert_same(host(dx2), host(dx), what=f"{name} Backprop(update) dX")
    lr = 0.02 / N
    scale_W = np.abs(W0) + np.abs(p0) + lr * gW_s + 1e-30
    assert_bound(host(comp.LinearParams()), oc.W, scale_W, what=f"{name} W'")
    assert_bound(host(comp.BiasParams()), oc.b, np.abs(b0) + lr * gb_s, what=f"{name} b'")


@pytest.mark.parametrize("cfg,N", [
    ((8, 9, 256, 3, 3, 256, 1, 1), 70),    # c5 C3: several frames per split
    ((4, 9, 64, 4, 3, 256, 0, 0), 61),     # c5 C4: P = 7, 4 frames per chunk, ragged tail
])
def test_conv_wgrad_long(kc, cfg, N):
    """Weight/bias gradient of long kernels (conv_wgrad2_kernel: frame-range
    splits, fixed-order reduction) against the oracle's Update gradient
    (nnet-component-nnet0.cc:738-765); deterministic across calls."""
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=N)
    r = rng(300 + N)
    x = randn(r, (N, H * W * C))
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    dy = randn(r, (N, oh * ow * G))
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: oc.gradient(x, dy))
    g = host(comp.ComputeGradient(dev(x), dev(dy)))
    kd = kh * kw * C
    assert_bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{cfg} gW")
    assert_bound(g[kd * G:], gb_t, gb_s, what=f"{cfg} gb")
    assert_same(host(comp.ComputeGradient(dev(x), dev(dy))), g, what="repeat")


def test_conv_backprop_gradient_special_values(kc):
    """Inf in the last map's tail must not leak into other columns: the
    fused kernel reads row tails past oh*ow (masked to exact zeros)."""
    cfg = (40, 11, 3, 8, 1, 128, 0, 0)
    comp, oc = make_pair(kc, cfg, seed=11)
    r = rng(11)
    N = 3
    x = randn(r, (N, 40 * 11 * 3))
    dy = randn(r, (N, 363 * 128))
    dy[1, 5 * 363 + 0] = np.inf      # start of map 5: adjacent to map 4's tail
    dy[2, 127 * 363 + 362] = -np.inf  # very last element of the frame
    with O.accum(1):
        gW_t, gb_t = oc.gradient(x, dy)
        dx_t = oc.backprop(x, dy, update=False)
    dx, g = comp.BackpropGradient(dev(x), dev(dy))
    g = host(g)
    kd = 24
    gW = g[:kd * 128].reshape(kd, 128)
    # non-finite pattern identical to the reference's
    np.testing.assert_array_equal(np.isfinite(gW), np.isfinite(gW_t))
    np.testing.assert_array_equal(np.isfinite(g[kd * 128:]), np.isfinite(gb_t))
    np.testing.assert_array_equal(np.isfinite(host(dx)), np.isfinite(dx_t))


def test_conv_update_divides_by_local_rows(kc):
    # B10: Update divides the learning rate by in_value.NumRows() (:767).
    cfg = CONVS["tiny"]
    comp, oc = make_pair(kc, cfg, 3)
    r = rng(3)
    x = randn(r, (4, 12))
    dy = randn(r, (4, 2 * 3 * 3))
    gW, gb = oc.gradient(x, dy)
    comp.Backprop(dev(x), None, dev(dy), update=True)
    oc.apply(gW, gb, 4)
    assert_bound(host(comp.LinearParams()), oc.W, np.abs(oc.W) + 1e-3, what="W")


@pytest.mark.parametrize("cfg", [
    (33, 11, 128, 1, 1, 4, False, False),
    (8, 9, 256, 2, 1, 4, False, False),
    (4, 3, 6, 1, 1, 3, True, False),
    (2, 3, 16, 1, 1, 2, False, True),
    (33, 11, 256, 3, 1, 4, False, False),   # c5 P1 (3-D window, 16-B gather kernel)
    (3, 2, 8, 3, 2, 2, False, False),       # 4-element groups wrap h -> w -> c
    (6, 5, 3, 2, 5, 3, False, False),       # row length 90: not a multiple of 4
    (9, 5, 12, 3, 5, 6, False, False),      # plane kernel, 270-float runs (no 16-B)
    (33, 11, 128, 1, 1, 4, True, False),    # intermap overlap on c2's maps (channel streams)
    (33, 11, 256, 1, 1, 2, False, True),    # overlap2D, 16 x 16 channel grid
    (3, 5, 49, 1, 1, 4, False, True),       # overlap2D pc 4, 7 x 7 grid
    (4, 4, 9, 1, 1, 2, True, False),        # overlap pc 2
])
def test_maxpool_component(kc, path, cfg):
    H, W, C, ph, pw, pc, ov, ov2 = cfg
    line = (f"MaxpoolComponent in-height={H} in-width={W} in-channel={C} "
            f"pool-height-dim={ph} pool-width-dim={pw} pool-channel-dim={pc} "
            f"overlap={'true' if ov else 'false'} overlap2D={'true' if ov2 else 'false'}")
    comp = kc.Component.NewFromString(line)
    op = O.Pool(H, W, C, ph, pw, pc, ov, ov2)
    assert comp.OutputDim() == op.output_dim
    r = rng(sum(cfg[:6]))
    x = with_ties(r, (7, H * W * C))
    y = op.propagate(x)
    yg = comp.Propagate(dev(x))
    assert_same(host(yg), y, "Maxpool Propagate")
    dy = randn(r, y.shape)
    dx = op.backprop(x, y, dy)
    dxg = comp.Backprop(dev(x), dev(y), dev(dy))
    assert_same(host(dxg), dx, "Maxpool Backprop")


@pytest.mark.parametrize("I,Od,N", [(300, 70, 33), (8192, 64, 40)])  # 2nd: split-K GEMM
def test_fc_component(kc, path, I, Od, N):
    comp = kc.Component.NewFromString(
        f"FullyConnectedComponent input-dim={I} output-dim={Od} learning-rate=0.02 "
        f"param-stddev=0.01 bias-stddev=1 weight-decay=0.0002 momentum=0.9")
    r = rng(5)
    of = O.FC(I, Od)
    of.W = randn(r, (Od, I), 0.05)
    of.b = randn(r, (Od,), 0.5)
    of.prev = randn(r, (Od, I), 0.01)
    for which, v in ((0, of.W), (1, of.b), (2, of.prev)):
        comp.SetParam(which, dev(v))
    x = randn(r, (N, I))
    _, y_t, y_s = triple(lambda: of.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what="FC Propagate")
    dy = randn(r, (N, Od))
    _, dx_t, dx_s = triple(lambda: of.backprop(x, dy, update=False))
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: of.gradient(x, dy))
    W0, p0, b0 = of.W.copy(), of.prev.copy(), of.b.copy()
    with O.accum(1):
        of.backprop(x, dy, update=True)
    dx = comp.Backprop(dev(x), None, dev(dy), update=True)
    assert_bound(host(dx), dx_t, dx_s, what="FC dX")
    lr = 0.02 / N
    assert_bound(host(comp.LinearParams()), of.W,
                 np.abs(W0) + np.abs(p0) + lr * gW_s, what="FC W'")
    assert_bound(host(comp.BiasParams()), of.b, np.abs(b0) + lr * gb_s, what="FC b'")


@pytest.mark.parametrize("I,Od,N", [(300, 70, 33), (8192, 64, 40), (2048, 1024, 300)])
def test_fc_bias_in_gemm_store(kc, I, Od, N):
    """FC Propagate adds the bias in the f16x3 GEMM's own store (one split or
    the split-K sum): the bits of the reference's two calls, out =
    CopyRowsFromVec(bias) then AddMatMat(1, in, W^T, beta = 1)."""
    import torch
    comp = kc.Component.NewFromString(
        f"FullyConnectedComponent input-dim={I} output-dim={Od} learning-rate=0.02 "
        f"param-stddev=0.01 bias-stddev=1")
    r = rng(I + Od)
    W = randn(r, (Od, I), 0.05)
    b = randn(r, (Od,), 0.5)
    comp.SetParam(0, dev(W))
    comp.SetParam(1, dev(b))
    x = randn(r, (N, I))
    y = host(comp.Propagate(dev(x)))
    c = dev(np.broadcast_to(b, (N, Od)).copy())
    kc.gemm(dev(x), dev(W), c, False, True, 1.0, 1.0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(y, host(c))


@pytest.mark.parametrize("I,Od,N,spread", [(512, 256, 2048, False), (300, 70, 33, False),
                                           (1000, 130, 4100, False), (11616, 1024, 4096, False),
                                           (512, 256, 2048, True), (11616, 1024, 4096, True)])
def test_fc_update_equals_gradient_then_apply(kc, I, Od, N, spread):
    """The update inside Backprop (UpdateSimple, nnet-component-nnet0.cc:1133-1150)
    must give the bits of ComputeGradient + ApplyGradient, the split the DP
    step uses.  Under f16x3 UpdateSimple applies the momentum update in the
    gradient GEMM's own store (kl_gemm_f16x3_momentum); the other path writes
    the gradient and runs hipF_momentum_update.  The first, third and c2
    shapes split the gradient GEMM's K (N >= 2048 frames), the second does
    not (its tile epilogue applies the update).  `spread`: two output units'
    derivatives are N(0,1) * 2^-28 but for one frame whose input is 0, so
    every element of those two gradient rows fails the store's check and is
    recomputed (split K: by gemm_f16x3_fixup_kernel), with the update applied
    there."""
    line = (f"FullyConnectedComponent input-dim={I} output-dim={Od} learning-rate=0.02 "
            f"param-stddev=0.01 bias-stddev=1 weight-decay=0.0002 momentum=0.9")
    r = rng(9)
    params = [randn(r, (Od, I), 0.05), randn(r, (Od,), 0.5), randn(r, (Od, I), 0.01)]
    xh, dyh = randn(r, (N, I)), randn(r, (N, Od), 0.1)
    if spread:
        k0 = N // 3
        for j0 in (3, Od - 2):
            dyh[:, j0] = randn(r, (N,), 2.0 ** -28)
            dyh[k0, j0] = 1.0
        xh[k0, :] = 0.0
    x, dy = dev(xh), dev(dyh)
    out = []
    for fused in (True, False):
        comp = kc.Component.NewFromString(line)
        for which, v in enumerate(params):
            comp.SetParam(which, dev(v))
        if fused:
            comp.Backprop(x, None, dy, update=True)
        else:
            comp.ApplyGradient(comp.ComputeGradient(x, dy), N)
        out.append([host(comp.GetParam(w)) for w in range(3)])
    for k in range(3):
        assert_same(out[0][k], out[1][k], f"FC param {k}")


@pytest.mark.parametrize("name,N", [("c2", 600), ("nnet_cfg_l1", 2048), ("nnet_cfg_l2", 2048),
                                    ("c5_C3_pad", 1024), ("c5_C4", 1024)])
def test_conv_update_equals_gradient_then_apply(kc, name, N):
    """ConvolutionComponent's update inside Backprop (:738-777) gives the
    bits of BackpropGradient + ApplyGradient (the DP step's split), and the
    same data gradient (taken with the pre-update kernel).  The frame kernels
    and the long-kernel weight gradients (nnet.config's and c5's layers:
    kcnn_reduce_splits_wgrad) apply the momentum step in their gradient
    reduction (conv-update.h); the other paths run ApplyGradient."""
    H, W, C, kh, kw, G, ph, pw = CONVS[name]
    line = conv_line(H, W, C, kh, kw, G, ph, pw) + " weight-decay=0.0005 momentum=0.9"
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    r = rng(21)
    params = [randn(r, (kh * kw * C, G), 0.05), randn(r, (G,), 0.5),
              randn(r, (kh * kw * C, G), 0.01)]
    x, dy = dev(randn(r, (N, H * W * C))), dev(randn(r, (N, oh * ow * G), 0.1))
    out = []
    for fused in (True, False):
        comp = kc.Component.NewFromString(line)
        for which, v in enumerate(params):
            comp.SetParam(which, dev(v))
        if fused:
            dx = comp.Backprop(x, None, dy, update=True)
        else:
            dx, g = comp.BackpropGradient(x, dy)
            comp.ApplyGradient(g, N)
        out.append([host(dx)] + [host(comp.GetParam(w)) for w in range(3)])
    for k, what in enumerate(["dX", "W", "b", "prev_grad"]):
        assert_same(out[0][k], out[1][k], f"conv {name} {what}")


@pytest.mark.parametrize("binary", [True, False])
def test_read_write_roundtrip(kc, tmp_path, binary):
    comps = [
        kc.Component.NewFromString(conv_line(*CONVS["small_pad"])),
        kc.Component.NewFromString(
            "MaxpoolComponent in-height=6 in-width=4 in-channel=8 pool-height-dim=2 "
            "pool-width-dim=2 pool-channel-dim=2"),
        kc.Component.NewFromString(
            "FullyConnectedComponent input-dim=20 output-dim=7 learning-rate=0.01 "
            "weight-decay=0.0005 momentum=0.5"),
    ]
    for c in comps:
        p = tmp_path / f"{c.Type()}.{'bin' if binary else 'txt'}"
        c.Write(p, binary)
        c2 = kc.Component.ReadNew(p)
        assert c2.Type() == c.Type() and c2.Info() == c.Info()
        if c.Type() != "MaxpoolComponent":
            for which in (0, 1, 2):
                assert_same(host(c2.GetParam(which)), host(c.GetParam(which)),
                            f"{c.Type()} param {which}")
            assert c2.LearningRate() == c.LearningRate()


def test_fd_gradient_check(kc):
    """nnet-conv-test.cc:60-210 pattern: objective = sum(out * objf_vec);
    predicted change tr(delta^T dX) vs observed change under a small input
    perturbation; the same for a parameter perturbation via DotProduct."""
    cfg = (6, 5, 2, 3, 2, 4, 0, 0)
    comp, _ = make_pair(kc, cfg, 11)
    import torch
    r = rng(12)
    x = dev(randn(r, (4, 60)).astype(np.float64).astype(np.float32))
    y = comp.Propagate(x)
    w = dev(randn(r, tuple(y.shape)))
    dx = comp.Backprop(x, None, w, update=False)
    obj = lambda xx: float((comp.Propagate(xx).double() * w.double()).sum())
    base = obj(x)
    for _ in range(3):
        delta = dev(randn(r, tuple(x.shape), 1e-3))
        pred = float((delta.double() * dx.double()).sum())
        obs = obj(x + delta) - base
        assert abs(pred - obs) <= 0.15 * abs(pred + obs) / 2 + 1e-4, (pred, obs)
    # parameter gradient: grad component via SetZero(true) + Update on it
    grad_comp = comp.Copy()
    grad_comp.SetZero(True)
    g = comp.ComputeGradient(x, w)
    kd = 3 * 2 * 2
    Wd = dev(randn(r, (kd, 4), 1e-3))
    perturbed = comp.Copy()
    perturbed.SetParam(kc.PARAM_LINEAR, comp.LinearParams() + Wd)
    pred = float((Wd.double().flatten() * g[:kd * 4].double()).sum())
    obs = float((perturbed.Propagate(x).double() * w.double()).sum()) - base
    assert abs(pred - obs) <= 0.05 * abs(pred + obs) / 2 + 1e-4, (pred, obs)


def test_init_from_string_quirks(kc):
    # B5: learning-rate is effectively mandatory
    with pytest.raises(kc.KcnnError):
        kc.Component.NewFromString(
            "ConvolutionComponent in-height=4 in-width=4 in-channel=1 kernel-height=2 "
            "kernel-width=2 stride=1 group=2 out-height=3 out-width=3")
    # B6: stride != 1 rejected
    with pytest.raises(kc.KcnnError):
        kc.Component.NewFromString(conv_line(4, 4, 1, 2, 2, 2, 0, 0).replace("stride=1", "stride=2"))
    # B4: weight-decay/momentum from the config are ignored (0.0002 / 0.9)
    c = kc.Component.NewFromString(conv_line(4, 4, 1, 2, 2, 2, 0, 0) +
                                   " weight-decay=0.5 momentum=0.1")
    assert "weight-decay=0.0002" in c.Info() and "momentum=0.9" in c.Info()
    # unknown option
    with pytest.raises(kc.KcnnError):
        kc.Component.NewFromString(conv_line(4, 4, 1, 2, 2, 2, 0, 0) + " foo=1")
    # bad geometry
    with pytest.raises(kc.KcnnError):
        kc.Component.NewFromString(conv_line(4, 4, 1, 2, 2, 2, 0, 0).replace("out-height=3", "out-height=4"))
    # Maxpool: window must tile the map
    with pytest.raises(kc.KcnnError):
        kc.Component.NewFromString("MaxpoolComponent in-height=5 in-width=4 in-channel=2 "
                                   "pool-height-dim=2 pool-width-dim=1 pool-channel-dim=1")
