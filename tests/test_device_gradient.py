"""tests/_stack.device_gradient (the float64 gradient the full-size GPU tests
check updates against, F.unfold + einsum on the tensors' device) against
the oracle's fp64-accumulated gradient on small CPU cases: padded and
unpadded convolutions, a pitched input view, and the FC layer."""
import numpy as np
import pytest

import oracle as O
from _stack import device_gradient, truth
from _util import rng


@pytest.mark.parametrize("cfg", [(8, 9, 5, 3, 3, 6, 1, 1), (11, 7, 3, 4, 2, 4, 0, 0),
                                 (40, 11, 3, 8, 1, 8, 0, 0), (6, 5, 4, 3, 3, 3, 1, 2)])
def test_device_gradient_conv(cfg):
    import torch
    H, W, C, kh, kw, G, ph, pw = cfg
    oc = O.Conv(H, W, C, kh, kw, G, in_pad_height=ph, in_pad_width=pw)
    r = rng(3)
    N = 7
    x = r.standard_normal((N, H * W * C)).astype(np.float32)
    dy = r.standard_normal((N, oc.output_dim)).astype(np.float32)
    oc.W = r.standard_normal((kh * kw * C, G)).astype(np.float32)
    (gW_t, gb_t), (gW_s, gb_s) = truth(lambda: oc.gradient(x, dy))
    xt = torch.zeros((N, H * W * C + 5))
    xt[:, :H * W * C] = torch.from_numpy(x)
    (gW, gb), (sW, sb) = device_gradient(oc, xt[:, :H * W * C], torch.from_numpy(dy), chunk=3)
    np.testing.assert_allclose(gW, gW_t, rtol=1e-6, atol=1e-6 * float(np.abs(gW_s).max()))
    np.testing.assert_allclose(gb, gb_t, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(sW, gW_s, rtol=1e-5)
    np.testing.assert_allclose(sb, gb_s, rtol=1e-5)


def test_device_gradient_fc():
    import torch
    oc = O.FC(37, 11)
    r = rng(4)
    x = r.standard_normal((50, 37)).astype(np.float32)
    dy = r.standard_normal((50, 11)).astype(np.float32)
    oc.W = r.standard_normal((11, 37)).astype(np.float32)
    (gW_t, gb_t), (gW_s, gb_s) = truth(lambda: oc.gradient(x, dy))
    (gW, gb), (sW, sb) = device_gradient(oc, torch.from_numpy(x), torch.from_numpy(dy), chunk=4)
    np.testing.assert_allclose(gW, gW_t, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gb, gb_t, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(sW, gW_s, rtol=1e-5)
    np.testing.assert_allclose(sb, gb_s, rtol=1e-5)
