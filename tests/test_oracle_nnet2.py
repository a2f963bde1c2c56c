"""CPU tests of the oracle's upstream nnet2 components either side of the
CNN path: RectifiedLinearComponent and SpliceComponent
(reference src/nnet2/nnet-component.cc:799-827, :2638-2819).  Pinned by
hand-derived known answers (including the reference's non-finite semantics:
ApplyFloor keeps NaN, the backprop is a product so 0 * inf = NaN) and by an
independent numpy formulation of the splice index maps."""
import numpy as np

import oracle as O
from _util import assert_same, randn, rng


def test_relu_known_answers():
    x = np.array([[-1.5, 0.0, 2.0, np.nan], [-0.0, 3.0, -np.inf, np.inf]], np.float32)
    y = O.ReLU(4).propagate(x)
    assert_same(y, np.array([[0, 0, 2, np.nan], [-0.0, 3, 0, np.inf]], np.float32), "relu fwd")
    assert np.signbit(y[1, 0])  # -0.0 is not < 0: kept (ApplyFloor)
    dy = np.array([[5.0, 6.0, 7.0, 8.0], [np.inf, 1.0, 2.0, 3.0]], np.float32)
    r = O.ReLU(4)
    dx = r.backprop(y, dy, update=True)
    # Heaviside(y) = [[0,0,1,0],[0,1,0,1]]; 0 * inf = nan at [1,0]
    assert_same(dx, np.array([[0, 0, 7, 0], [np.nan, 1, 0, 3]], np.float32), "relu bwd")
    assert r.count == 2
    np.testing.assert_array_equal(r.deriv_sum, [0, 1, 1, 1])
    assert r.value_sum[1] == 3.0 and r.value_sum[2] == 2.0 and np.isnan(r.value_sum[3])


def test_relu_stats_accumulate():
    r = rng(5)
    relu = O.ReLU(6)
    tv, td, n = np.zeros(6), np.zeros(6), 0
    for rows in (3, 7):
        y = relu.propagate(randn(r, (rows, 6)))
        relu.backprop(y, randn(r, (rows, 6)), update=True)
        tv += y.astype(np.float64).sum(0)
        td += (y > 0).sum(0)
        n += rows
    np.testing.assert_allclose(relu.value_sum, tv, rtol=1e-6)
    np.testing.assert_array_equal(relu.deriv_sum, td)
    assert relu.count == n
    # update=False leaves the stats alone (to_update == NULL)
    relu.backprop(relu.propagate(randn(r, (2, 6))), randn(r, (2, 6)), update=False)
    assert relu.count == n


def _splice_ref(x, context, const_dim, out_cs):
    """numpy formulation: output frame t of a chunk concatenates input frames
    t + c - context[0] (c in context), then the const tail of frame t."""
    ctx = list(context)
    in_cs = out_cs + ctx[-1] - ctx[0]
    dim = x.shape[1] - const_dim
    n = x.shape[0] // in_cs
    xs = x.reshape(n, in_cs, -1)
    out = []
    for t in range(out_cs):
        parts = [xs[:, t + c - ctx[0], :dim] for c in ctx]
        if const_dim:
            parts.append(xs[:, t, dim:])
        out.append(np.concatenate(parts, axis=1))
    return np.stack(out, 1).reshape(n * out_cs, -1)


def test_splice_known_answer():
    # two chunks of 3 one-dimensional frames, context -1..1: one output frame each
    x = np.arange(6, dtype=np.float32).reshape(6, 1)
    s = O.Splice(1, (-1, 0, 1))
    assert_same(s.propagate(x), np.array([[0, 1, 2], [3, 4, 5]], np.float32), "splice KAT")
    dy = np.array([[1, 10, 100], [2, 20, 200]], np.float32)
    assert_same(s.backprop(dy), np.array([[1], [10], [100], [2], [20], [200]], np.float32),
                "splice bwd KAT")


def test_splice_matches_numpy_with_const_and_overlap():
    r = rng(9)
    ctx, const, out_cs, n = (-2, -1, 0, 1, 2, 3), 2, 3, 4
    in_cs = out_cs + 5
    x = randn(r, (n * in_cs, 7))
    s = O.Splice(7, ctx, const)
    y = s.propagate(x, num_chunks=n, out_cs=out_cs)
    assert_same(y, _splice_ref(x, ctx, const, out_cs), "splice fwd")
    # backprop = transpose of the index map: sum over every use, in order c
    dy = randn(r, y.shape)
    dx = s.backprop(dy, num_chunks=n, out_cs=out_cs)
    exp = np.zeros_like(x)
    dim = 7 - const
    for k in range(n):
        for t in range(out_cs):
            for ci, c in enumerate(ctx):
                exp[k * in_cs + t + c - ctx[0], :dim] += dy[k * out_cs + t, ci * dim:(ci + 1) * dim]
            exp[k * in_cs + t, dim:] = dy[k * out_cs + t, len(ctx) * dim:]
    np.testing.assert_allclose(dx, exp, rtol=1e-6, atol=1e-6)


def test_chunk_offsets_and_gapped_splice():
    """Upstream Nnet::ComputeChunkInfo restated (oracle.chunk_offsets) and the
    offset-list splice against a direct numpy gather (SpliceComponent::
    Propagate's index vectors, nnet-component.cc:2670-2681)."""
    import numpy as np
    offs = O.chunk_offsets([[-2, -1, 0, 1, 2], [0], [-3, 0, 3], [0]])
    assert offs == [list(range(11)), [2, 5, 8], [2, 5, 8], [5], [5]]
    assert O.chunk_offsets([list(range(-10, 11))]) == [list(range(21)), [10]]
    r = np.random.default_rng(4)
    N, D = 3, 5
    sp = O.Splice(D, (-3, 0, 3))
    x = r.standard_normal((N * 3, D)).astype(np.float32)          # offsets 2, 5, 8
    y = sp.propagate_offsets(x, [2, 5, 8], [5], N)
    want = np.concatenate([x.reshape(N, 3, D)[:, i] for i in range(3)], axis=1)
    np.testing.assert_array_equal(y, want)
    dx = sp.backprop_offsets(y, [2, 5, 8], [5], N)
    np.testing.assert_array_equal(dx, x)                          # one reader per row
    # contiguous offsets: the offset-list form equals the range form
    sp2 = O.Splice(D, (-1, 0, 1))
    x2 = r.standard_normal((N * 4, D)).astype(np.float32)
    np.testing.assert_array_equal(sp2.propagate_offsets(x2, [0, 1, 2, 3], [1, 2], N),
                                  sp2.propagate(x2, N, out_cs=2))
