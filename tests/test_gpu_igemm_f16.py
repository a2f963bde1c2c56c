"""The f16x3 implicit GEMM (cnsl-conv-igemm-x6.hip; igemm_x6 family 2, the
default, takes it for convolutions of at least 2^34 flop -- c5's C2 / C3
forward and data gradients -- and family 3, set here, for every shape).

Scale groups (f16-split.h): one per filter (a column of W over every k) and
one per frame of the input (every im2col column reads one frame).  A tile
whose groups hold Inf / NaN, or one of whose products the store check cannot
clear (a spread group's small elements carrying the sum), is recomputed as
fp32 dot products by conv_igemm_fixup_kernel, so:
  * ordinary data meets the parity bar (1e-5 * S elementwise,
    1e-5 normwise) against the oracle;
  * a group spread over 2^24 ... 2^32 whose largest element meets zeros
    still meets the elementwise bar (the f16x3 products alone miss it by
    up to 50x: VERDICT r04 item 1's model);
  * frames with Inf / NaN give the reference's IEEE pattern (the listed
    tiles are recomputed as fp32 dot products).
Reference: CuMatrixBase::Conv2D (src/cnslmat/conv2D.cc:43-201) and
ConvolutionComponent::Propagate / Backprop (src/nnet0/nnet-component-nnet0.cc:
423-446, 461-544).
"""
import numpy as np
import pytest

from _util import assert_bound, assert_same, dev, host, randn, rng, triple
from test_gpu_components import conv_line, make_pair
from test_gpu_fwd_f16 import check_pattern, nonfinite_inputs

pytestmark = pytest.mark.gpu

C5_C2 = (11, 11, 64, 4, 3, 256, 0, 0)
C5_C3 = (8, 9, 256, 3, 3, 256, 1, 1)
C5_C4 = (4, 9, 64, 4, 3, 256, 0, 0)
NNET_L2 = (1, 18, 128, 1, 4, 128, 0, 0)   # a G = 128 (128 x 256 tile) shape


@pytest.fixture
def fam(kc):
    old = kc.get_kernel_family("igemm_x6")

    def set_(v):
        kc.set_kernel_family("igemm_x6", v)
    yield set_
    kc.set_kernel_family("igemm_x6", old)


@pytest.mark.parametrize("cfg", [C5_C2, C5_C3, C5_C4, NNET_L2],
                         ids=["c5_C2", "c5_C3", "c5_C4", "G128"])
def test_igemm_f16_parity(kc, fam, cfg):
    fam(3)
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=7 + C)
    r = rng(3 + G)
    N = 37
    x = randn(r, (N, H * W * C))
    _, y_t, y_s = triple(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what="f16x3 Propagate")
    dy = randn(r, y_t.shape)
    _, dx_t, dx_s = triple(lambda: oc.backprop(x, dy, update=False))
    dx = comp.Backprop(dev(x), None, dev(dy), update=False)
    assert_bound(host(dx), dx_t, dx_s, what="f16x3 dX")


@pytest.mark.parametrize("spread", [24, 28, 32])
@pytest.mark.parametrize("group", ["filter", "frame"])
def test_igemm_intra_group_range(kc, fam, group, spread):
    """A scale group's largest elements meet zeros in the other operand and
    every other element sits 2^-spread below them, bias 0: the small elements
    carry all of S.  "filter": W's channel-0 taps are 1 and the rest
    N(0,1) * 2^-spread, X's channel 0 is 0; "frame": X's channel 0 is 1 (the
    frame's largest values), the other channels N(0,1) * 2^-spread, W's
    channel-0 taps 0."""
    fam(3)
    H, W, C, kh, kw, G, ph, pw = C5_C3
    comp, oc = make_pair(kc, C5_C3, seed=43)
    r = rng(44 + spread)
    N = 6
    x = randn(r, (N, C, W * H))
    Wm = randn(r, (kh * kw * C, G), 0.01)
    taps = kh * kw
    if group == "filter":
        Wm[:taps] = 1.0
        Wm[taps:] *= np.float32(2.0 ** -spread)
        x[:, 0] = 0.0
    else:
        Wm[:taps] = 0.0
        x[:, 0] = 1.0
        x[:, 1:] *= np.float32(2.0 ** -spread)
    x = x.reshape(N, -1).astype(np.float32)
    oc.W = Wm.astype(np.float32)
    oc.b = np.zeros_like(oc.b)
    comp.SetParam(kc.PARAM_LINEAR, dev(oc.W))
    comp.SetParam(kc.PARAM_BIAS, dev(oc.b))
    _, y_t, y_s = triple(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"{group} spread 2^{spread}")


@pytest.mark.parametrize("cfg", [C5_C3, C5_C2], ids=["c5_C3", "c5_C2"])
def test_igemm_nonfinite_frames(kc, fam, cfg):
    """Frames holding Inf / NaN have no scale: their tiles are recomputed as
    fp32 dot products (conv_igemm_fixup_kernel), which gives the reference's
    IEEE pattern (+Inf, -Inf, NaN) where its result is not finite and the bar
    elsewhere; the Conv -> Maxpool fusion (c5 C3 -> P2) goes through the same
    fixup's pooling."""
    fam(3)
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=5)
    r = rng(9)
    x = nonfinite_inputs(r, 8, H * W * C)
    y_ref, y_t, y_s = triple(lambda: oc.propagate(x))
    check_pattern(host(comp.Propagate(dev(x))), y_ref, y_t, y_s, "igemm f16x3 non-finite")


def test_igemm_nonfinite_pooled(kc, fam):
    """c5's C3 with its P2 pool in the implicit GEMM's epilogue (and the
    fixup's pooling) against the unfused pair on non-finite frames: bitwise."""
    fam(3)
    H, W, C, kh, kw, G, ph, pw = C5_C3
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    cfg = "\n".join([conv_line(*C5_C3),
                     f"MaxpoolComponent in-height={oh} in-width={ow} in-channel={G} "
                     f"pool-height-dim=2 pool-width-dim=1 pool-channel-dim=4"])
    x = dev(nonfinite_inputs(rng(10), 8, H * W * C))
    outs = []
    for fuse in (True, False):
        kc.set_fusion(fuse)
        try:
            net = kc.Nnet(cfg)
            conv = net.components[0]
            conv.SetParam(kc.PARAM_LINEAR, dev(randn(rng(11), (kh * kw * C, G), 0.05)))
            conv.SetParam(kc.PARAM_BIAS, dev(randn(rng(12), (G,), 0.5)))
            net.Propagate(x)
            outs.append(host(net.Output()))
        finally:
            kc.set_fusion(True)
    assert_same(outs[0], outs[1], "fused vs unfused")


def test_igemm_f16_repeat_bitwise(kc, fam):
    """Repeated calls on one input give the same bits (tile list, fixup)."""
    fam(3)
    comp, _ = make_pair(kc, C5_C3, seed=11)
    H, W, C = C5_C3[:3]
    x = dev(randn(rng(12), (301, H * W * C)))
    y0 = host(comp.Propagate(x))
    for rep in range(4):
        assert_same(host(comp.Propagate(x)), y0, f"repeat {rep}")


@pytest.mark.parametrize("kind", ["huge_x", "huge_dy", "tiny_x", "tiny_dy"])
def test_igemm_f16_fp32_range(kc, fam, kind):
    """The edges of fp32 (test_gpu_x6_range's operands: values up to 3.4e38,
    or scaled by 2^-120) through the f16x3 forward and data gradient at the
    full bar: the scales put every group into f16's range, and the frames
    whose spread the check cannot clear are recomputed in fp32."""
    from test_gpu_x6_range import scaled_inputs
    fam(3)
    H, W, C, kh, kw, G, ph, pw = C5_C3
    comp, oc = make_pair(kc, C5_C3, seed=3)
    if kind.startswith("huge"):
        oc.W = (oc.W * 1e-3).astype(np.float32)
        comp.SetParam(kc.PARAM_LINEAR, dev(oc.W))
    r = rng(41)
    N = 5
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    x, dy = scaled_inputs(kind, r, N, H * W * C, oh * ow * G, G)
    if kind in ("huge_x", "tiny_x"):
        _, y_t, y_s = triple(lambda: oc.propagate(x))
        assert_bound(host(comp.Propagate(dev(x))), y_t, y_s, what=f"{kind} Propagate")
    _, dx_t, dx_s = triple(lambda: oc.backprop(x, dy, update=False))
    dx = comp.Backprop(dev(x), None, dev(dy), update=False)
    assert_bound(host(dx), dx_t, dx_s, what=f"{kind} dX")


# ---------------------------------------------------------------------------
# The weight gradient's f16x3 form (conv_wgrad_x6w_kernel<P, true>, wgrad_x6
# family 3; not the default): scale groups over the whole batch (a filter of dY, an input channel
# of X), rejected partials recomputed in fp32, flagged blocks on bf16x6.
# Reference: ConvolutionComponent::Update's gradient (src/nnet0/
# nnet-component-nnet0.cc:738-765).

@pytest.fixture
def wfam(kc):
    old = kc.get_kernel_family("wgrad_x6")

    def set_(v):
        kc.set_kernel_family("wgrad_x6", v)
    yield set_
    kc.set_kernel_family("wgrad_x6", old)


def _grad_check(kc, comp, oc, x, dy, what, bound=assert_bound):
    _, (gW_t, gb_t), (gW_s, gb_s) = triple(lambda: oc.gradient(x, dy))
    g = host(comp.ComputeGradient(dev(x), dev(dy)))
    kd = gW_t.shape[0]
    G = gW_t.shape[1]
    bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what=f"{what} gW")
    bound(g[kd * G:], gb_t, gb_s, what=f"{what} gb")


@pytest.mark.parametrize("cfg", [C5_C3, C5_C2, C5_C4], ids=["c5_C3", "c5_C2", "c5_C4"])
def test_wgrad_f16_parity(kc, wfam, cfg):
    wfam(3)
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=17 + C)
    r = rng(5 + G)
    N = 41
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    x = randn(r, (N, H * W * C))
    dy = randn(r, (N, oh * ow * G))
    _grad_check(kc, comp, oc, x, dy, "f16x3")


@pytest.mark.parametrize("spread", [24, 32])
@pytest.mark.parametrize("group", ["filter", "channel"])
def test_wgrad_intra_group_range(kc, wfam, group, spread):
    """A group's largest values meet zeros and the rest sit 2^-spread below:
    "filter": dY's filter-0 maps are 1 on frame 0 and N(0,1) 2^-spread on the
    other frames, X zero on frame 0; "channel": X's channel 0 is 1 on frame
    0 and the rest of the batch N(0,1) 2^-spread, dY zero on frame 0."""
    wfam(3)
    H, W, C, kh, kw, G, ph, pw = C5_C3
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    P = oh * ow
    comp, oc = make_pair(kc, C5_C3, seed=47)
    r = rng(48 + spread)
    N = 9
    x = randn(r, (N, C, H * W))
    dy = randn(r, (N, G, P))
    sc = np.float32(2.0 ** -spread)
    if group == "filter":
        dy[1:] *= sc
        dy[0] = 0.0
        dy[0, 0] = 1.0
        x[0] = 0.0
    else:
        x[1:] *= sc
        x[0] = 0.0
        x[0, 0] = 1.0
        dy[0] = 0.0
    _grad_check(kc, comp, oc, x.reshape(N, -1).astype(np.float32),
                dy.reshape(N, -1).astype(np.float32), f"{group} spread 2^{spread}")


@pytest.mark.parametrize("kind", ["huge_x", "huge_dy", "tiny_x", "tiny_dy"])
def test_wgrad_f16_fp32_range(kc, wfam, kind):
    """test_gpu_x6_range's operands through the f16x3 weight gradient: the
    full bar for huge ones; tiny ones at the bf16x6 contract where a block
    falls back to it (elementwise 1e-5 S, normwise 1e-4)."""
    from test_gpu_x6_range import scaled_inputs
    import _util
    wfam(3)
    H, W, C, kh, kw, G, ph, pw = C5_C3
    comp, oc = make_pair(kc, C5_C3, seed=3)
    r = rng(41)
    N = 5
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    x, dy = scaled_inputs(kind, r, N, H * W * C, oh * ow * G, G)

    def bound(a, t, s, rtol=1e-5, what=""):
        _util.assert_bound(a, t, s, rtol=rtol, what=what, norm_rtol=1e-4)
    _grad_check(kc, comp, oc, x, dy, kind, bound if kind.startswith("tiny") else assert_bound)


def test_wgrad_f16_nonfinite_blocks(kc, wfam):
    """A frame with Inf / NaN flags the blocks of its split; they run on the
    bf16x6 form: the non-finite entries are those of the bf16x6 kernel."""
    H, W, C, kh, kw, G, ph, pw = C5_C3
    comp, _ = make_pair(kc, C5_C3, seed=9)
    r = rng(10)
    N = 7
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    x = randn(r, (N, H * W * C))
    x[2, 77] = np.inf
    dy = randn(r, (N, oh * ow * G))
    outs = []
    for fam_v in (1, 3):
        wfam(fam_v)
        outs.append(host(comp.ComputeGradient(dev(x), dev(dy))))
    # family 1 is the 128-wide bf16x6 kernel: same non-finite positions
    assert (np.isfinite(outs[0]) == np.isfinite(outs[1])).all()
