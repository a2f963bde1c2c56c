"""The f16x3 implicit GEMM (cnsl-conv-igemm-x6.hip, igemm_x6 family 2, the
default for the long-kernel convolutions: c5 C2-C4 forward and data
gradient, nnet.config's convolutions).

Scale groups (f16-split.h): one per filter (a column of W over every k) and
one per frame of the input (every im2col column reads one frame).  A tile
whose groups hold Inf / NaN, or one of whose products the store check cannot
clear (a spread group's small elements carrying the sum), is recomputed by
the bf16x6 form of the same kernel, so:
  * ordinary data meets the parity bar (1e-5 * S elementwise,
    1e-5 normwise) against the oracle;
  * a group spread over 2^24 ... 2^32 whose largest element meets zeros
    still meets the elementwise bar (the f16x3 products alone miss it by
    up to 50x: VERDICT r04 item 1's model);
  * frames with Inf / NaN give the bf16x6 kernel's bits.
Reference: CuMatrixBase::Conv2D (src/cnslmat/conv2D.cc:43-201) and
ConvolutionComponent::Propagate / Backprop (src/nnet0/nnet-component-nnet0.cc:
423-446, 461-544).
"""
import numpy as np
import pytest

from _util import assert_bound, assert_same, dev, host, randn, rng, triple
from test_gpu_components import make_pair

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
    fam(2)
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
    fam(2)
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


def test_igemm_nonfinite_frames_take_bf16x6(kc, fam):
    """Frames holding Inf / NaN have no scale: their tiles are recomputed by
    the bf16x6 form, so those frames' outputs are bitwise the bf16x6 kernel's
    (family 1), and the other frames stay within the bar."""
    H, W, C, kh, kw, G, ph, pw = C5_C3
    comp, oc = make_pair(kc, C5_C3, seed=5)
    r = rng(9)
    N = 12
    x = randn(r, (N, H * W * C))
    x[3, 100] = np.inf
    x[7, 5000] = np.nan
    xd = dev(x)
    fam(1)
    y1 = host(comp.Propagate(xd))
    fam(2)
    y2 = host(comp.Propagate(xd))
    for n in (3, 7):
        assert_same(y2[n], y1[n], f"frame {n}")
    ok = [n for n in range(N) if n not in (3, 7)]
    _, y_t, y_s = triple(lambda: oc.propagate(x[ok]))
    assert_bound(y2[ok], y_t, y_s, what="finite frames")


def test_igemm_f16_repeat_bitwise(kc, fam):
    """Repeated calls on one input give the same bits (tile flags, redo)."""
    fam(2)
    comp, _ = make_pair(kc, C5_C3, seed=11)
    H, W, C = C5_C3[:3]
    x = dev(randn(rng(12), (301, H * W * C)))
    y0 = host(comp.Propagate(x))
    for rep in range(4):
        assert_same(host(comp.Propagate(x)), y0, f"repeat {rep}")
