"""The pooled output's operand statistics from the register-pooled conv +
maxpool forward (pool-stats.h; cnsl-conv-frame.hip: the RP kernel's row
maxima / minima, pool_colmax_kernel, pool_count_kernel), checked bit for bit
against the same statistics computed here from the pooled output the kernel
wrote: per frame the exact max |value| bits, the exact min nonzero bits and,
for a spread frame, the count of its small elements; per pooled column the
max's binade bound, the min over the column's small elements and their
count, spread or not (f16-split.h's definitions; a count in a column that
is not spread only adds GEMM checks).  The FC GEMMs take
these blocks as their f16x3 scales and check thresholds, so a wrong count
would let a spread product through unchecked.

c2's first layer (40 x 11 x 3 maps, 8 x 1 kernel, 128 filters, pool 4 over
channels: P = 363, 11616 pooled columns) through the C-ABI entry point
kcnn_conv2d_maxpool_stats.  Spread groups are made by frames whose maps are
zero (their conv output is the bias alone) and one pool group whose biases
are 2^-30: that group's pooled value is 2^-30 in those frames and O(1) in
the others.
"""
import ctypes

import numpy as np
import pytest

from _util import dev, randn, rng

pytestmark = pytest.mark.gpu

H, W, C, KH, KW, G, PC = 40, 11, 3, 8, 1, 128, 4
P = (H - KH + 1) * (W - KW + 1)
NPOOL = G // PC * P
NONFINITE = 0x7F800000


class PoolStatsOut(ctypes.Structure):
    _fields_ = [("rowmax", ctypes.c_void_p), ("colmax", ctypes.c_void_p),
                ("partials", ctypes.c_void_p), ("partial_words", ctypes.c_size_t),
                ("produced", ctypes.c_int)]


def ebits(b):
    """f16-split.h ebits over an array of nonzero |x| bit patterns."""
    b = b.astype(np.int64)
    sub = np.floor(np.log2(np.maximum(b, 1))).astype(np.int64) - 149
    return np.where(b >= 0x00800000, (b >> 23) - 127, sub)


def expected(Pm):
    a = np.abs(Pm).view(np.uint32).astype(np.int64)
    R = a.shape[0]
    # rows: exact max, exact min nonzero, spread count
    rmax = a.max(1)
    nz = np.where(a == 0, 0xFFFFFFFF, a)
    rmin = nz.min(1)
    rmin = np.where(rmin == 0xFFFFFFFF, 0, rmin)
    e_r = ebits(rmax)
    rspread = (rmin != 0) & (rmax < NONFINITE) & (ebits(np.maximum(rmin, 1)) < e_r - 20)
    small_r = (a != 0) & (ebits(np.maximum(a, 1)) < (e_r - 17)[:, None])
    rcnt = np.where(rspread, small_r.sum(1), 0)
    # columns: the max's binade bound, the min over the small elements
    byte = (a >> 23).max(0)
    cmax = (byte << 23) | 0x7FFFFF
    e_c = ebits(cmax)
    small_c = (a != 0) & (ebits(np.maximum(a, 1)) < (e_c - 17)[None, :]) & (cmax < NONFINITE)[None, :]
    cmin = np.where(small_c, a, 0xFFFFFFFF).min(0)
    cspread = (cmin != 0xFFFFFFFF) & (ebits(np.minimum(cmin, 0x7FFFFFFF)) < e_c - 20)
    ccnt = small_c.sum(0)  # every small element, spread or not (pool_count_kernel)
    row = np.concatenate([rmax, rmin, rcnt]).astype(np.uint32)
    col = np.concatenate([cmax, cmin, ccnt]).astype(np.uint32)
    return row, col, int(rspread.sum()), int(cspread.sum())


def run_stats(kc, x, Wm, b):
    import torch
    L = kc.lib()
    R = x.shape[0]
    X, K, B = dev(x), dev(Wm), dev(b)
    pool = torch.empty((R, NPOOL), dtype=torch.float32, device="cuda")
    mask = torch.empty((R, NPOOL), dtype=torch.uint8, device="cuda")
    L.kcnn_conv2d_maxpool_stats_words.restype = ctypes.c_size_t
    pw = L.kcnn_conv2d_maxpool_stats_words(R, H, W, C, KH, KW, G, PC)
    assert pw > 0
    rows = torch.full((3 * R,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    cols = torch.full((3 * NPOOL,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    part = torch.full((pw,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    st = PoolStatsOut(rows.data_ptr(), cols.data_ptr(), part.data_ptr(), pw, 0)
    D = kc.MatrixDim
    rc = L.kcnn_conv2d_maxpool_stats(
        ctypes.c_void_p(X.data_ptr()), D(R, H * W * C, H * W * C), H, W, C, 0, 0,
        ctypes.c_void_p(K.data_ptr()), D(KH * KW * C, G, G), KH, KW, G,
        ctypes.c_void_p(B.data_ptr()), None, D(R, P * G, P * G),
        ctypes.c_void_p(pool.data_ptr()), D(R, NPOOL, NPOOL),
        ctypes.c_void_p(mask.data_ptr()), NPOOL, PC,
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), ctypes.byref(st))
    torch.cuda.synchronize()
    assert rc == 0
    assert st.produced == 1, "the register-pooled kernel did not run (no statistics)"
    u = lambda t: t.cpu().numpy().view(np.uint32)
    return pool.cpu().numpy(), u(rows), u(cols)


@pytest.fixture
def f16(kc):
    old = kc.get_kernel_family("fwd_x6")
    kc.set_kernel_family("fwd_x6", 2)
    yield
    kc.set_kernel_family("fwd_x6", old)


@pytest.mark.parametrize("case", ["plain", "spread", "spread_many"])
def test_pool_stats_exact(kc, f16, case):
    r = rng({"plain": 3, "spread": 4, "spread_many": 5}[case])
    R = 300
    x = randn(r, (R, H * W * C))
    Wm = randn(r, (KH * KW * C, G), 0.1)
    b = randn(r, (G,))
    if case != "plain":
        b[5 * PC:6 * PC] = np.float32(2.0 ** -30)      # pool group 5: tiny biases
        b[9 * PC:10 * PC] = np.float32(2.0 ** -19)     # pool group 9: small, not spread
        zero = [10, 11, 299] if case == "spread" else list(range(0, R, 7))
        x[zero] = 0.0
        x[50] *= np.float32(2.0 ** -25)                # conv sum far under the biases
    Pm, rows, cols = run_stats(kc, x, Wm, b)
    row_e, col_e, nrs, ncs = expected(Pm)
    if case != "plain":
        assert nrs > 0 and ncs > 0, (nrs, ncs)         # the case makes spread groups
    for name, got, exp, n in (("row", rows, row_e, R), ("col", cols, col_e, NPOOL)):
        for k, part in enumerate(("max", "min", "cnt")):
            g_, e_ = got[k * n:(k + 1) * n], exp[k * n:(k + 1) * n]
            bad = np.flatnonzero(g_ != e_)
            assert bad.size == 0, (f"{case}: {name} {part} differs at {bad[:5]}: "
                                   f"got {g_[bad[:5]]} want {e_[bad[:5]]}")
