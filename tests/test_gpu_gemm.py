"""CuMatrixBase::AddMatMat on the GPU: the bf16x6 split kernel (gemm mode 1,
kaldi-lite/cu-gemm-x6.hip) and rocBLAS sgemm (mode 0) against a float64
product, with the dot-product error bound of SURVEY 8(d):
|c - t| <= 1e-5 * (|alpha| |op(A)| |op(B)| + |beta| |C0|) elementwise and
||c - t|| / ||t|| <= 1e-5.  The float64 truth is torch's fp64 matmul on the
same device (a plain PyTorch reference of the op, as for every float kernel).
"""
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _mats(torch, m, n, k, ta, tb, seed, scale_b=0.01, pitch=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)

    def mk(r, c, s):
        base = torch.randn((r, c + pitch), generator=g, device="cuda") * s
        return base[:, :c]

    a = mk(k, m, 1.0) if ta else mk(m, k, 1.0)
    b = mk(n, k, scale_b) if tb else mk(k, n, scale_b)
    c = mk(m, n, 1.0)
    return a, b, c


def _check(torch, kc, m, n, k, ta, tb, alpha=1.0, beta=0.0, mode=1, seed=1, pitch=0):
    a, b, c0 = _mats(torch, m, n, k, ta, tb, seed, pitch=pitch)
    c = c0.clone()
    kc.set_gemm_mode(mode)
    try:
        kc.gemm(a, b, c, ta, tb, alpha, beta)
    finally:
        kc.set_gemm_mode(1)
    torch.cuda.synchronize()
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    t = alpha * (A @ B) + beta * c0.double()
    s = abs(alpha) * (A.abs() @ B.abs()) + abs(beta) * c0.double().abs()
    err = (c.double() - t).abs()
    assert torch.isfinite(c).all()
    worst = float((err / s.clamp_min(1e-30)).max())
    assert worst <= RTOL, f"max err/S {worst:.3e}"
    rel = float((c.double() - t).norm() / t.norm())
    assert rel <= RTOL, f"normwise {rel:.3e}"
    return c, worst, rel


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(1, 1, 1), (7, 5, 3), (33, 17, 40), (300, 129, 77),
                                   (257, 260, 1000), (64, 11616, 96)])
def test_gemm_x6_small_and_ragged(kc, ta, tb, shape):
    import torch
    m, n, k = shape
    _check(torch, kc, m, n, k, ta, tb)


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
def test_gemm_x6_alpha_beta_pitched(kc, ta, tb):
    import torch
    _check(torch, kc, 130, 70, 200, ta, tb, alpha=0.37, beta=1.0, pitch=12)
    _check(torch, kc, 130, 70, 200, ta, tb, alpha=-2.0, beta=0.5, pitch=4)


def test_gemm_x6_split_k_is_deterministic(kc):
    """Thin output, long K: the K split over workgroups with the fixed-order
    partial sum; bitwise equal across runs."""
    import torch
    c1, _, _ = _check(torch, kc, 256, 256, 9000, False, True, beta=1.0)
    c2, _, _ = _check(torch, kc, 256, 256, 9000, False, True, beta=1.0)
    assert torch.equal(c1, c2)


def test_gemm_x6_beta_zero_ignores_nan(kc):
    import torch
    a = torch.randn(40, 50, device="cuda")
    b = torch.randn(50, 30, device="cuda")
    c = torch.full((40, 30), float("nan"), device="cuda")
    kc.gemm(a, b, c)
    torch.cuda.synchronize()
    assert torch.isfinite(c).all()


@pytest.mark.parametrize("name,m,n,k,ta,tb", [
    ("fc_fwd", 4096, 1024, 11616, False, True),     # out = in W^T
    ("fc_dgrad", 4096, 11616, 1024, False, False),  # in_deriv = out_deriv W
    ("fc_wgrad", 1024, 11616, 4096, True, False),   # gW = out_deriv^T in
    # nnet.config's last FC dX: out_deriv has 3454 columns and that pitch, so
    # its rows are not 16-B aligned; AddMatMat copies it to a padded pitch
    ("nnet_fc3_dgrad", 4096, 4096, 3454, False, False),
])
def test_gemm_c2_fc_shapes(kc, name, m, n, k, ta, tb):
    """The c2 stack's three FC GEMMs at full size: the split kernel meets the
    bound, and its error is no worse than rocBLAS sgemm's (x 1.5)."""
    import torch
    _, w6, r6 = _check(torch, kc, m, n, k, ta, tb, mode=1)
    _, w0, r0 = _check(torch, kc, m, n, k, ta, tb, mode=0)
    assert w6 <= 1.5 * w0 + 1e-8 and r6 <= 1.5 * r0 + 1e-8, (w6, w0, r6, r0)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape,pitch", [((4, 4, 32), 0), ((260, 132, 64), 4),
                                         ((300, 1000, 2048), 0), ((256, 256, 9024), 8),
                                         ((1028, 516, 96), 0)])
def test_gemm_x6_fast_path_shapes(kc, ta, tb, shape, pitch):
    """Shapes the one-block-per-K-step kernel takes (K a multiple of 32, rows
    multiples of 4, 16-B aligned pitches): partial tiles read 0 past M / N
    through the buffer range, split K, both operand layouts."""
    import torch
    m, n, k = shape
    _check(torch, kc, m, n, k, ta, tb, pitch=pitch)
    _check(torch, kc, m, n, k, ta, tb, alpha=0.5, beta=1.0, pitch=pitch)


def _check_planes(torch, kc, m, n, k, ta, tb, alpha=1.0, beta=0.0, seed=3):
    a, b, c0 = _mats(torch, m, n, k, ta, tb, seed)
    ap, bp = kc.split_planes(a), kc.split_planes(b)
    # the planes are an exact encoding: h + m + l == x
    for x, xp in ((a, ap), (b, bp)):
        f = (xp.to(torch.int32) << 16).view(torch.float32)[..., :x.shape[1]]
        assert torch.equal(f[0] + f[1] + f[2], x)
    c = c0.clone()
    kc.gemm_planes(ap, bp, c, k, ta, tb, alpha, beta)
    torch.cuda.synchronize()
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    t = alpha * (A @ B) + beta * c0.double()
    s = abs(alpha) * (A.abs() @ B.abs()) + abs(beta) * c0.double().abs()
    worst = float(((c.double() - t).abs() / s.clamp_min(1e-30)).max())
    rel = float((c.double() - t).norm() / t.norm())
    assert worst <= RTOL and rel <= RTOL, (worst, rel)
    return c


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(8, 8, 32), (264, 136, 64), (1024, 1000, 2048),
                                   (256, 256, 9024)])
def test_gemm_planes(kc, ta, tb, shape):
    """The plane GEMM (LDS-DMA of pre-split operands) against float64, with
    partial tiles, split K and both operand layouts; bitwise equal to the
    in-kernel split path's product is not required (different kernels), the
    bound is."""
    import torch
    m, n, k = shape
    _check_planes(torch, kc, m, n, k, ta, tb)
    _check_planes(torch, kc, m, n, k, ta, tb, alpha=0.5, beta=1.0)
