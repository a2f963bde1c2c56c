"""CuMatrixBase::AddMatMat on the GPU: the f16x3 split kernel (gemm mode 2,
the default, kaldi-lite/cu-gemm-f16x3.hip), the bf16x6 split kernel (mode 1,
cu-gemm-x6.hip) and rocBLAS sgemm (mode 0) against a float64 product, with
the dot-product error bound of SURVEY 8(d):
|c - t| <= 1e-5 * (|alpha| |op(A)| |op(B)| + |beta| |C0|) elementwise and
||c - t|| / ||t|| <= 1e-5.  The float64 truth is torch's fp64 matmul on the
same device (a plain PyTorch reference of the op, as for every float kernel).
"""
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-5
SPLIT_MODES = [2, 1]   # f16x3, bf16x6


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


def _gemm_mode(kc, mode, fn):
    old = kc.get_kernel_family("gemm")
    kc.set_gemm_mode(mode)
    try:
        return fn()
    finally:
        kc.set_gemm_mode(old)


def _bound(torch, a, b, c0, c, ta, tb, alpha, beta):
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    t = alpha * (A @ B) + beta * c0.double()
    s = abs(alpha) * (A.abs() @ B.abs()) + abs(beta) * c0.double().abs()
    err = (c.double() - t).abs()
    assert torch.isfinite(c).all()
    worst = float((err / s.clamp_min(1e-300)).max())
    assert worst <= RTOL, f"max err/S {worst:.3e}"
    rel = float((c.double() - t).norm() / t.norm().clamp_min(1e-300))
    assert rel <= RTOL, f"normwise {rel:.3e}"
    return worst, rel


def _check(torch, kc, m, n, k, ta, tb, alpha=1.0, beta=0.0, mode=2, seed=1, pitch=0):
    a, b, c0 = _mats(torch, m, n, k, ta, tb, seed, pitch=pitch)
    c = c0.clone()
    _gemm_mode(kc, mode, lambda: kc.gemm(a, b, c, ta, tb, alpha, beta))
    torch.cuda.synchronize()
    worst, rel = _bound(torch, a, b, c0, c, ta, tb, alpha, beta)
    return c, worst, rel


@pytest.mark.parametrize("mode", SPLIT_MODES)
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(1, 1, 1), (7, 5, 3), (33, 17, 40), (300, 129, 77),
                                   (257, 260, 1000), (64, 11616, 96), (129, 70, 4133)])
def test_gemm_x6_small_and_ragged(kc, mode, ta, tb, shape):
    import torch
    m, n, k = shape
    _check(torch, kc, m, n, k, ta, tb, mode=mode)


@pytest.mark.parametrize("mode", SPLIT_MODES)
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
def test_gemm_x6_alpha_beta_pitched(kc, mode, ta, tb):
    import torch
    _check(torch, kc, 130, 70, 200, ta, tb, alpha=0.37, beta=1.0, pitch=12, mode=mode)
    _check(torch, kc, 130, 70, 200, ta, tb, alpha=-2.0, beta=0.5, pitch=4, mode=mode)


@pytest.mark.parametrize("mode", SPLIT_MODES)
def test_gemm_x6_split_k_is_deterministic(kc, mode):
    """Thin output, long K: the K split over workgroups with the fixed-order
    partial sum; bitwise equal across runs."""
    import torch
    c1, _, _ = _check(torch, kc, 256, 256, 9000, False, True, beta=1.0, mode=mode)
    c2, _, _ = _check(torch, kc, 256, 256, 9000, False, True, beta=1.0, mode=mode)
    assert torch.equal(c1, c2)


@pytest.mark.parametrize("mode", SPLIT_MODES)
def test_gemm_x6_beta_zero_ignores_nan(kc, mode):
    import torch
    a = torch.randn(40, 50, device="cuda")
    b = torch.randn(50, 30, device="cuda")
    c = torch.full((40, 30), float("nan"), device="cuda")
    _gemm_mode(kc, mode, lambda: kc.gemm(a, b, c))
    torch.cuda.synchronize()
    assert torch.isfinite(c).all()


@pytest.mark.parametrize("case", ["spread", "subnormal_a", "huge_a"])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape", [(300, 200, 1000), (256, 256, 9024)])
def test_gemm_f16x3_row_scales(kc, case, ta, tb, shape):
    """f16x3 scales each row of op(A) and column of op(B) by its own power of
    two, so operands anywhere in fp32's range meet the full bar: rows spread
    over 2^-60..2^60 and columns over 2^-30..2^30 with zero rows / columns and
    a single-element row; all of A fp32 subnormals (2^-140, B at 2^110); all
    of A near FLT_MAX / 2 (2^126, B at 2^-120)."""
    import torch
    m, n, k = shape
    a, b, c0 = _mats(torch, m, n, k, ta, tb, seed=7)
    A = a.t() if ta else a          # views: scaling them scales the stored data
    B = b.t() if tb else b
    if case == "spread":
        g = torch.Generator(device="cuda")
        g.manual_seed(11)
        A.mul_(torch.exp2(torch.randint(-60, 61, (m, 1), generator=g, device="cuda").float()))
        B.mul_(torch.exp2(torch.randint(-30, 31, (1, n), generator=g, device="cuda").float()))
        A[3].zero_()
        B[:, 5].zero_()
        A[7].zero_()
        A[7, k // 2] = 1.5
    elif case == "subnormal_a":
        A.mul_(2.0 ** -140)
        B.mul_(2.0 ** 110)
        assert float(A.abs().max()) < 2.0 ** -126   # every element subnormal
    else:
        A.mul_(2.0 ** 125)
        B.mul_(2.0 ** -120)
    c = c0.clone()
    kc.gemm(a, b, c, ta, tb, 1.0, 0.0)
    torch.cuda.synchronize()
    _bound(torch, a, b, c0, c, ta, tb, 1.0, 0.0)


@pytest.mark.parametrize("mode", [2, 0])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("shape", [(260, 140, 300), (300, 260, 4500), (1024, 11616, 2048)])
def test_gemm_nonfinite_pattern(kc, mode, ta, tb, shape):
    """Inf and NaN operands give sgemm's IEEE pattern (+Inf, -Inf, NaN, and
    the finite elements elsewhere within the bound): f16x3 computes the rows
    and columns they touch as fp32 dot products; rocBLAS for comparison.
    The second shape splits K over workgroups (in-kernel reduction); the
    third runs 256 of its 364 tiles whole and splits the other 108 (the
    split-K cost model's mixed grid, block_tile), with Inf / NaN rows in
    both parts."""
    import torch
    m, n, k = shape
    a, b, c0 = _mats(torch, m, n, k, ta, tb, seed=5)
    A = a.t() if ta else a
    B = b.t() if tb else b
    A[4, 10] = float("inf")
    A[9, 11] = float("-inf")
    A[20, 0] = float("nan")
    A[30, 12] = float("inf"); A[30, 13] = float("-inf")
    B[12, 7] = float("inf")
    B[:, 100] = 0.0; B[50, 100] = float("-inf")
    B[0, 60] = 0.0                     # Inf * 0 in row 20? (NaN anyway)
    B[10, 3] = 0.0                     # row 4's Inf meets a zero: NaN
    c = c0.clone()
    beta = 0.5
    _gemm_mode(kc, mode, lambda: kc.gemm(a, b, c, ta, tb, 1.0, beta))
    torch.cuda.synchronize()
    t = A.double() @ B.double() + beta * c0.double()
    fin = torch.isfinite(t)
    assert torch.equal(torch.isnan(c), torch.isnan(t))
    assert torch.equal(torch.isposinf(c), torch.isposinf(t))
    assert torch.equal(torch.isneginf(c), torch.isneginf(t))
    s = A.double().abs().nan_to_num(posinf=0) @ B.double().abs().nan_to_num(posinf=0) + \
        beta * c0.double().abs()
    err = (c.double() - t).abs()[fin]
    assert float((err / s[fin].clamp_min(1e-300)).max()) <= RTOL


@pytest.mark.parametrize("name,m,n,k,ta,tb", [
    ("fc_fwd", 4096, 1024, 11616, False, True),     # out = in W^T
    ("fc_dgrad", 4096, 11616, 1024, False, False),  # in_deriv = out_deriv W
    ("fc_wgrad", 1024, 11616, 4096, True, False),   # gW = out_deriv^T in
    # nnet.config's last FC dX: out_deriv has 3454 columns and that pitch, so
    # its rows are not 16-B aligned; AddMatMat copies it to a padded pitch
    ("nnet_fc3_dgrad", 4096, 4096, 3454, False, False),
])
def test_gemm_c2_fc_shapes(kc, name, m, n, k, ta, tb):
    """The c2 stack's three FC GEMMs at full size: both split kernels meet the
    bound; bf16x6's error is no worse than rocBLAS sgemm's (x 1.5), f16x3's
    within 2x of it normwise and 2e-6 * S elementwise (measured r05,
    scripts/gemm_error_ratio.py: f16x3 0.44-0.89x sgemm's normwise error,
    bf16x6 0.62-1.31x)."""
    import torch
    _, w3, r3 = _check(torch, kc, m, n, k, ta, tb, mode=2)
    _, w6, r6 = _check(torch, kc, m, n, k, ta, tb, mode=1)
    _, w0, r0 = _check(torch, kc, m, n, k, ta, tb, mode=0)
    assert w6 <= 1.5 * w0 + 1e-8 and r6 <= 1.5 * r0 + 1e-8, (w6, w0, r6, r0)
    # f16x3: 22-23 of fp32's 24 bits per operand and 3 accumulator roundings
    # per 16 products (sgemm: one per product)
    assert w3 <= 2e-6 and r3 <= 2 * r0 + 1e-8, (w3, w0, r3, r0)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape,pitch", [((4, 4, 32), 0), ((260, 132, 64), 4),
                                         ((300, 1000, 2048), 0), ((256, 256, 9024), 8),
                                         ((1028, 516, 96), 0)])
def test_gemm_x6_fast_path_shapes(kc, ta, tb, shape, pitch):
    """(run on the default engine, f16x3, and on bf16x6)"""
    """Shapes the one-block-per-K-step kernel takes (K a multiple of 32, rows
    multiples of 4, 16-B aligned pitches): partial tiles read 0 past M / N
    through the buffer range, split K, both operand layouts."""
    import torch
    m, n, k = shape
    for mode in SPLIT_MODES:
        _check(torch, kc, m, n, k, ta, tb, pitch=pitch, mode=mode)
        _check(torch, kc, m, n, k, ta, tb, alpha=0.5, beta=1.0, pitch=pitch, mode=mode)


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


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("shape,pitch", [((258, 130, 300), 2), ((258, 130, 4500), 2),
                                         ((3454, 64, 1024), 2), ((130, 70, 200), 12)])
def test_gemm_f16x3_ragged_rows(kc, ta, tb, shape, pitch):
    """M and N not multiples of 4: a row-contiguous operand with a 16-B pitch
    takes the 16-B transposed loads, whose last quad runs into the pitch's
    padding (those rows / columns of C are not stored); an odd pitch is
    copied to a padded one first; split K sums slabs of a padded pitch."""
    import torch
    m, n, k = shape
    for alpha, beta in ((1.0, 0.0), (0.5, 1.0)):
        a, b, c0 = _mats(torch, m, n, k, ta, tb, 9, pitch=pitch)
        for x in (a, b):  # NaN in the pitch's padding: never reaches a stored C
            torch.as_strided(x, (x.shape[0], pitch), (x.stride(0), 1), x.shape[1]).fill_(
                float("nan"))
        c = c0.clone()
        _gemm_mode(kc, 2, lambda: kc.gemm(a, b, c, ta, tb, alpha, beta))
        torch.cuda.synchronize()
        _bound(torch, a, b, c0, c, ta, tb, alpha, beta)


C2_FC = [("fc_fwd", 4096, 1024, 11616, False, True),
         ("fc_dgrad", 4096, 11616, 1024, False, False),
         ("fc_wgrad", 1024, 11616, 4096, True, False)]


@pytest.mark.parametrize("name,m,n,k,ta,tb", C2_FC, ids=[c[0] for c in C2_FC])
@pytest.mark.parametrize("side", ["row", "col"])
@pytest.mark.parametrize("spread", [24, 28, 32])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_f16x3_intra_group_range(kc, name, m, n, k, ta, tb, side, spread, beta):
    """The f16x3 scale is one power of two per row of op(A) / column of
    op(B), set by the group's largest element; elements far below it lose
    their low part (an f16 subnormal).  Here one row of op(A) (side "row") or
    one column of op(B) ("col") is N(0,1) * 2^-spread except one element of
    size 1 whose partner in the other operand is 0 for every output: the
    small elements carry all of S, and the elementwise 1e-5 * S bar must
    hold.  c2's FC shapes, all three transposes; beta 1
    as in the nnet2 AffineComponent update (the staged epilogue
    of a one-split tile once applied beta twice to a rejected element)."""
    import torch
    a, b, c0 = _mats(torch, m, n, k, ta, tb, seed=31)
    A = a.t() if ta else a
    B = b.t() if tb else b
    g = torch.Generator(device="cuda")
    g.manual_seed(32 + spread)
    k0 = k // 3
    if side == "row":
        for i0 in (5, m - 2):
            A[i0] = torch.randn(k, generator=g, device="cuda") * 2.0 ** -spread
            A[i0, k0] = 1.0
        B[k0, :] = 0.0
    else:
        for j0 in (7, n - 3):
            B[:, j0] = torch.randn(k, generator=g, device="cuda") * (0.01 * 2.0 ** -spread)
            B[k0, j0] = -0.01
        A[:, k0] = 0.0
    # an all-zero column of op(B) / row of op(A) beside the spread groups: its
    # products are exactly 0 and are not checked (weight -inf in the sum)
    if side == "row":
        B[:, 1] = 0.0
    else:
        A[2, :] = 0.0
    c = c0.clone()
    _gemm_mode(kc, 2, lambda: kc.gemm(a, b, c, ta, tb, 1.0, beta))
    torch.cuda.synchronize()
    _bound(torch, a, b, c0, c, ta, tb, 1.0, beta)
    zero = c[:, 1] if side == "row" else c[2, :]
    want = (c0[:, 1] if side == "row" else c0[2, :]) * beta
    assert torch.equal(zero, want), zero
