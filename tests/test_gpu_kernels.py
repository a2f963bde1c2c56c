"""GPU parity of the CuMatrixBase extension methods (reference
cudamatrix/cu-matrix.h:451-480, bodies cnslmat/conv2D.cc) against the CPU
oracle, called through libkcnn.so's C-ABI.

Integer/index work (every reshape helper, max pooling and its routing) must be
bit-exact; the convolution contraction is checked against the fp64-accumulated
oracle with the dot-product error bound |a - t| <= 1e-5 * sum|x_k w_k|
(north_star: fp32 within 1e-5 relative).
"""
import numpy as np
import pytest

import oracle as O
from _util import (assert_bound, assert_same, dev, host, padded, randn, rng,
                   triple, with_ties)

pytestmark = pytest.mark.gpu

# (H, W, C, kh, kw, G): BASELINE c2, nnet.config layer 1 and 2, c5 layers,
# small odd shapes, a 1x1 kernel, kernel == input.
CONV_SHAPES = [
    (40, 11, 3, 8, 1, 128),
    (40, 21, 1, 40, 4, 128),
    (1, 18, 128, 1, 3, 128),
    (11, 11, 64, 4, 3, 256),
    (4, 9, 64, 4, 3, 256),
    (6, 5, 2, 3, 2, 4),
    (7, 3, 5, 1, 1, 9),
    (5, 4, 3, 5, 4, 17),
    (9, 8, 3, 2, 3, 3),
    (12, 7, 2, 3, 3, 1),
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("concat", [True, False])
def test_conv2d(kc, shape, concat):
    H, W, C, kh, kw, G = shape
    r = rng(hash(shape) & 0xffff)
    N = 5
    x = randn(r, (N, H * W * C))
    k = randn(r, (kh * kw * C, G))
    f32, truth, S = triple(lambda: O.conv2d(x, k, H, W, C, kh, kw, G, concat))
    out = kc.Conv2D(padded(x), dev(k), H, W, C, kh, kw, G, concat=concat)
    assert_bound(host(out), truth, S, what=f"Conv2D{shape} concat={concat}")
    # the fp32 oracle itself is also within the bound at these sizes
    assert_bound(f32, truth, S, rtol=2e-5, what="oracle fp32")


def test_conv2d_splitk_long_reduction(kc):
    # The shape ConvolutionComponent::Update feeds Conv2D (:763): rows = C,
    # "channels" = samples, kernel = TpInsideBlock(dY): K = oh*ow*N is long,
    # M*G small -> the split-K + fixed-order reduce path.
    H, W, C, kh, kw, G, N = 40, 11, 3, 8, 1, 128, 64
    oh, ow = H - kh + 1, W - kw + 1
    r = rng(7)
    x = randn(r, (N, H * W * C))
    dy = randn(r, (N, oh * ow * G))
    xt = O.tp_block(x, C, H * W)
    dyt = O.tp_inside_block(dy, G, oh * ow)
    f32, truth, S = triple(lambda: O.conv2d(xt, dyt, H, W, N, oh, ow, G, False))
    out = kc.Conv2D(dev(xt), dev(dyt), H, W, N, oh, ow, G, concat=False)
    assert_bound(host(out), truth, S, what="Conv2D split-K")


@pytest.mark.parametrize("rep,shape", [(363, (7, 363 * 128)), (3, (4, 12)), (1, (3, 5))])
def test_add_mat_rep_vec(kc, rep, shape):
    r = rng(rep)
    m = randn(r, shape)
    v = randn(r, (shape[1] // rep,))
    exp = O.add_mat_rep_vec(m.copy(), v, rep)
    d = padded(m)
    kc.AddMatRepVec(d, dev(v), rep)
    assert_same(host(d), exp, "AddMatRepVec")


@pytest.mark.parametrize("kh,kw,C,G", [(8, 1, 3, 128), (3, 2, 4, 5), (1, 1, 2, 3), (40, 4, 1, 7)])
def test_flip_mat(kc, kh, kw, C, G):
    r = rng(kh * 100 + G)
    m = randn(r, (kh * kw * C, G))
    assert_same(host(kc.FlipMat(padded(m), kh, kw, C, G)), O.flip_mat(m, kh, kw, C, G), "FlipMat")


@pytest.mark.parametrize("H,W,C,kh,kw", [(33, 11, 128, 8, 1), (4, 6, 2, 3, 2), (1, 18, 3, 1, 3), (5, 5, 1, 1, 1)])
def test_padding_zero(kc, H, W, C, kh, kw):
    r = rng(H * W + kh)
    m = randn(r, (3, H * W * C))
    assert_same(host(kc.PaddingZero(padded(m), H, W, C, kh, kw)),
                O.padding_zero(m, H, W, C, kh, kw), "PaddingZero")


@pytest.mark.parametrize("C,bs,R", [(3, 440, 6), (2, 4, 5), (1, 7, 3), (128, 24, 3)])
def test_tp_block(kc, C, bs, R):
    r = rng(C * bs)
    m = randn(r, (R, C * bs))
    assert_same(host(kc.TpBlock(padded(m), C, bs)), O.tp_block(m, C, bs), "TpBlock")


@pytest.mark.parametrize("G,bs,R", [(128, 363, 4), (3, 5, 7), (1, 4, 2)])
def test_tp_inside_block(kc, G, bs, R):
    r = rng(G * bs + R)
    m = randn(r, (R, G * bs))
    assert_same(host(kc.TpInsideBlock(padded(m), G, bs)),
                O.tp_inside_block(m, G, bs), "TpInsideBlock")


@pytest.mark.parametrize("C,bs,cols", [(3, 8, 128), (2, 5, 3), (1, 4, 6)])
def test_mod_permute_row(kc, C, bs, cols):
    r = rng(C + bs)
    m = randn(r, (C * bs, cols))
    assert_same(host(kc.ModPermuteRow(padded(m), C, bs)),
                O.mod_permute_row(m, C, bs), "ModPermuteRow")


@pytest.mark.parametrize("H,W,C,K,R", [(33, 11, 4, 2, 5), (2, 3, 1, 3, 7), (1, 1, 5, 4, 2)])
def test_mod_permute_channel(kc, H, W, C, K, R):
    r = rng(H + W + C + K)
    comp = randn(r, (R, C * H * W))
    cont = randn(r, (R, K * C * H * W))
    for k in range(K):
        exp = O.mod_permute_channel(comp, k, K, H, W, cont.copy(), True)
        got = kc.ModPermuteChannel(padded(comp), k, K, H, W, padded(cont), True)
        assert_same(host(got), exp, "ModPermuteChannel to container")
        back = kc.ModPermuteChannel(padded(np.zeros_like(comp)), k, K, H, W,
                                    padded(exp), False)
        assert_same(host(back), comp, "ModPermuteChannel from container")


POOLS = [  # (H, W, C, ph, pw, pc, overlap, overlap2D)
    (33, 11, 128, 1, 1, 4, False, False),   # BASELINE c2: 1x1x4 intermap pool
    (8, 9, 256, 2, 1, 4, False, False),     # c5 P2
    (1, 12, 256, 1, 2, 1, False, False),    # nnet.config maxpool
    (6, 4, 8, 2, 2, 2, False, False),
    (3, 5, 6, 3, 5, 3, False, False),
    (5, 3, 12, 1, 1, 3, False, False),      # channel-only pc=3 (direct kernel)
    (7, 2, 8, 1, 1, 2, False, False),       # channel-only pc=2
    (3, 3, 16, 1, 1, 8, False, False),      # channel-only pc=8 (group kernel)
    (4, 3, 6, 1, 1, 3, True, False),        # overlap (1-D channel sliding)
    (2, 3, 16, 1, 1, 2, False, True),       # overlap2D (4x4 map, 2x2 window)
    (3, 2, 25, 1, 1, 3, False, True),
]


def _pool_out_dim(H, W, C, ph, pw, pc, ov, ov2):
    return O.Pool(H, W, C, ph, pw, pc, ov, ov2).output_dim


@pytest.mark.parametrize("cfg", POOLS)
def test_maxpool_prop_backprop(kc, cfg):
    H, W, C, ph, pw, pc, ov, ov2 = cfg
    r = rng(sum(cfg[:6]))
    N = 6
    x = with_ties(r, (N, H * W * C))  # ties in most windows
    od = _pool_out_dim(*cfg)
    y = O.maxpool_prop(x, H, W, ph, pw, pc, od, ov, ov2)
    yg = kc.Maxpool_prop(padded(x), H, W, ph, pw, pc, ov, ov2, kc.zeros(N, od))
    assert_same(host(yg), y, f"Maxpool_prop{cfg}")
    dy = randn(r, (N, od))
    dx = O.maxpool_backprop(x, y, dy, H, W, ph, pw, pc, ov, ov2)
    dxg = kc.Maxpool_backprop(dev(x), dev(y), padded(dy), kc.zeros(N, H * W * C),
                              H, W, ph, pw, pc, ov, ov2)
    assert_same(host(dxg), dx, f"Maxpool_backprop{cfg}")
    # every tied maximum receives the full derivative (not "first argmax")
    if not (ov or ov2):
        assert (dx != 0).sum() > N * od


def test_maxpool_special_values(kc):
    # NaN never wins (`val < x` is false), all-below -1e20 gives -1e20,
    # +/-inf propagate -- reference cnsl-cu-kernels.cu:251-260.
    H, W, C, pc = 2, 1, 4, 4
    x = np.array([[np.nan, 1.0, 2.0, np.nan, 0.0, np.nan, -3.0, np.inf],
                  [-np.inf, -1e30, -1e25, -5e20, -1e21, -2e30, -3e22, -1e29]],
                 np.float32)
    y = O.maxpool_prop(x, H, W, 1, 1, pc, 2)
    yg = kc.Maxpool_prop(dev(x), H, W, 1, 1, pc, False, False, kc.zeros(2, 2))
    assert_same(host(yg), y, "special values")
    assert y[0, 0] == 2.0 and y[0, 1] == np.inf
    assert (y[1] == np.float32(-1e20)).all()
