"""GPU parity of the upstream nnet2 components either side of the CNN path
(reference src/nnet2/nnet-component.cc): SpliceComponent
(:2524-2866) feeding the first convolution and RectifiedLinearComponent
(:799-827) after it, against the oracle (oracle/).  Both are copies /
element-wise maps, so outputs and derivatives are bit-exact; the ReLU's fp64
diagnostic stats (UpdateStats :337-363) match to fp32 column-sum order.  The
kcnn_nnet runtime is checked on the first layers of the reference's own
egs/exp/nnet/nnet.config (Splice -> Conv -> ReLU -> Conv -> ReLU -> Maxpool
-> FC), parameters after one update included."""
import numpy as np
import pytest

import oracle as O
from _util import assert_same, dev, host, randn, rng

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dim", [2304, 2303])  # 16-B lanes; the one-column kernels
def test_relu_component(kc, dim):
    r = rng(1)
    N = 70  # two 64-row stats parts, the second ragged
    comp = kc.Component.NewFromString(f"RectifiedLinearComponent dim={dim}")
    assert comp.Type() == "RectifiedLinearComponent" and comp.InputDim() == dim
    assert not comp.BackpropNeedsInput() and comp.BackpropNeedsOutput()
    x = randn(r, (N, dim))
    x[0, :4] = [np.nan, -np.inf, np.inf, -0.0]
    ref = O.ReLU(dim)
    y = ref.propagate(x)
    yg = comp.Propagate(dev(x))
    assert_same(host(yg), y, "ReLU Propagate")
    dy = randn(r, (N, dim))
    dy[1, 7] = np.inf   # where y <= 0 the reference's product gives NaN
    for upd in (False, True, True):
        dx = ref.backprop(y, dy, update=upd)
        dxg = comp.Backprop(None, yg, dev(dy), update=upd)
        assert_same(host(dxg), dx, f"ReLU Backprop update={upd}")
    vs, ds, cnt = comp.NonlinearStats()
    assert cnt == ref.count == 2 * N
    np.testing.assert_array_equal(ds, ref.deriv_sum)
    fin = np.isfinite(ref.value_sum)
    np.testing.assert_array_equal(np.isfinite(vs), fin)
    np.testing.assert_allclose(vs[fin], ref.value_sum[fin], rtol=2e-6, atol=1e-5)


@pytest.mark.parametrize("ctx,const,out_cs,n", [
    ((-10, 10), 0, 1, 33),     # nnet.config:1 (input-dim=40, left/right 10)
    ((-2, 3), 3, 4, 5),        # const tail, several output frames per chunk
    ((0, 0), 0, 2, 6),         # context {0}: identity layout
])
def test_splice_component(kc, ctx, const, out_cs, n):
    lo, hi = ctx
    idim = 40 if const == 0 else 11
    line = f"SpliceComponent input-dim={idim} left-context={-lo} right-context={hi}"
    if const:
        line += f" const-component-dim={const}"
    comp = kc.Component.NewFromString(line)
    context = tuple(range(lo, hi + 1))
    assert comp.Context() == list(context)
    s = O.Splice(idim, context, const)
    assert comp.OutputDim() == s.output_dim
    assert not comp.BackpropNeedsInput() and not comp.BackpropNeedsOutput()
    in_cs = out_cs + hi - lo
    r = rng(len(context) + n)
    x = randn(r, (n * in_cs, idim))
    y = s.propagate(x, num_chunks=n, out_cs=out_cs)
    yg = comp.Propagate(dev(x), num_chunks=n)
    assert_same(host(yg), y, "Splice Propagate")
    dy = randn(r, y.shape)
    dx = s.backprop(dy, num_chunks=n, out_cs=out_cs)
    dxg = comp.Backprop(None, None, dev(dy), num_chunks=n)
    assert host(dxg).shape == dx.shape
    assert_same(host(dxg), dx, "Splice Backprop")


@pytest.mark.parametrize("binary", [True, False])
def test_nnet2_read_write_roundtrip(kc, tmp_path, binary):
    relu = kc.Component.NewFromString("RectifiedLinearComponent dim=12")
    r = rng(3)
    y = relu.Propagate(dev(randn(r, (5, 12))))
    relu.Backprop(None, y, dev(randn(r, (5, 12))), update=True)  # stats
    comps = [relu,
             kc.Component.NewFromString("SpliceComponent input-dim=13 left-context=2 "
                                        "right-context=1 const-component-dim=3"),
             kc.Component.NewFromString("SpliceComponent input-dim=4 context=-3:0:2")]
    for c in comps:
        p = tmp_path / f"{c.Type()}.{'bin' if binary else 'txt'}"
        c.Write(p, binary)
        c2 = kc.Component.ReadNew(p)
        assert c2.Type() == c.Type() and c2.Info() == c.Info()
        assert c2.InputDim() == c.InputDim() and c2.OutputDim() == c.OutputDim()
        if c.Type() == "SpliceComponent":
            assert c2.Context() == c.Context()
        else:
            a, b = c.NonlinearStats(), c2.NonlinearStats()
            assert a[2] == b[2] == 5.0
            if binary:
                np.testing.assert_array_equal(a[0], b[0])
            else:
                np.testing.assert_allclose(a[0], b[0], rtol=1e-15)
            np.testing.assert_array_equal(a[1], b[1])


NNET_CFG_PREFIX = """SpliceComponent input-dim=40 left-context=10 right-context=10 const-component-dim=0
ConvolutionComponent in-height=40 in-width=21 in-channel=1 kernel-height=40 kernel-width=4 stride=1 group=128 out-height=1 out-width=18 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=2304
ConvolutionComponent in-height=1 in-width=18 in-channel=128 kernel-height=1 kernel-width=3 stride=1 group=128 out-height=1 out-width=16 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=2048
MaxpoolComponent in-height=1 in-width=16 in-channel=128 pool-height-dim=1 pool-width-dim=2 pool-channel-dim=1
FullyConnectedComponent input-dim=1024 output-dim=64 learning-rate=0.02 param-stddev=0.01 bias-stddev=1 weight-decay=0.0005 momentum=0.9"""


def test_nnet_config_prefix(kc):
    """nnet.config:1-5 + a pool and an FC through the kcnn_nnet runtime (chunk
    infos from the Splice context: 21 input frames per output frame) against
    the oracle chain, including every parameter after the in-Backprop update."""
    kc.set_randn_seed(5)
    net = kc.Nnet(NNET_CFG_PREFIX)
    sp, c1, r1, c2, r2, mp, fc = net.components
    N = 24
    r = rng(17)
    x = randn(r, (N * 21, 40))
    dy = randn(r, (N, 64), 0.05)

    def conv_oracle(c, H, W, C, kh, kw, G):
        oc = O.Conv(H, W, C, kh, kw, G)
        oc.W = host(c.LinearParams()); oc.b = host(c.BiasParams()); oc.prev = host(c.PrevGrad())
        return oc
    o1 = conv_oracle(c1, 40, 21, 1, 40, 4, 128)
    o2 = conv_oracle(c2, 1, 18, 128, 1, 3, 128)
    of = O.FC(1024, 64, weight_decay=0.0005)
    of.W = host(fc.LinearParams()); of.b = host(fc.BiasParams()); of.prev = host(fc.PrevGrad())
    osp, orl1, orl2 = O.Splice(40, tuple(range(-10, 11))), O.ReLU(2304), O.ReLU(2048)
    opl = O.Pool(1, 16, 128, 1, 2, 1)

    net.Propagate(dev(x))
    net.Backprop(dev(dy))
    with O.accum(1):
        a0 = osp.propagate(x)
        a1 = o1.propagate(a0); a2 = orl1.propagate(a1)
        a3 = o2.propagate(a2); a4 = orl2.propagate(a3)
        a5 = opl.propagate(a4); of.propagate(a5)
        d5 = of.backprop(a5, dy, update=True)
        d4 = opl.backprop(a4, a5, d5)
        d3 = orl2.backprop(a4, d4)
        d2 = o2.backprop(a2, d3, update=True)
        d1 = orl1.backprop(a2, d2)
        o1.backprop(a0, d1, update=True)
    assert_same(host(net.Output(0)), a0, "Splice output")
    np.testing.assert_allclose(host(net.Output(2)), a2, rtol=1e-5, atol=1e-5)
    for name, got, exp in (("conv1 W", c1.LinearParams(), o1.W), ("conv1 b", c1.BiasParams(), o1.b),
                           ("conv2 W", c2.LinearParams(), o2.W), ("conv2 b", c2.BiasParams(), o2.b),
                           ("fc W", fc.LinearParams(), of.W), ("fc b", fc.BiasParams(), of.b)):
        g = host(got)
        err = np.abs(g - exp).max() / max(np.abs(exp).max(), 1e-30)
        assert err < 1e-5, f"{name}: rel err {err:.2e}"
    # ReLU stats accumulated by the in-Backprop UpdateStats of each ReLU
    vs, ds, cnt = r1.NonlinearStats()
    assert cnt == N
    np.testing.assert_array_equal(ds, orl1.deriv_sum)


GAPPED_CFG = """SpliceComponent input-dim=8 context=-2:-1:0:1:2 const-component-dim=0
RectifiedLinearComponent dim=40
SpliceComponent input-dim=40 context=-3:0:3 const-component-dim=0
FullyConnectedComponent input-dim=120 output-dim=16 learning-rate=0.02 param-stddev=0.05 bias-stddev=1 weight-decay=0.0002 momentum=0.9"""


def test_gapped_splice_stack(kc):
    """A gapped context deeper in the stack (upstream Nnet::ComputeChunkInfo:
    the second Splice's context -3:0:3 leaves the first Splice's output and
    the ReLU with chunk offsets {2, 5, 8}, not a contiguous range) against the
    oracle's offset-list splices (oracle.chunk_offsets); the input chunk is
    contiguous (11 frames per output frame)."""
    kc.set_randn_seed(3)
    net = kc.Nnet(GAPPED_CFG)
    s1, rl, s2, fc = net.components
    offs = O.chunk_offsets([s1.Context(), rl.Context(), s2.Context(), fc.Context()])
    assert offs[1] == [2, 5, 8] and len(offs[0]) == 11
    N = 13
    r = rng(29)
    x = randn(r, (N * len(offs[0]), 8))
    dy = randn(r, (N, 16), 0.1)
    net.Propagate(dev(x))
    outs = [host(net.Output(i)) for i in range(4)]
    o1, orl, o2 = O.Splice(8, tuple(s1.Context())), O.ReLU(40), O.Splice(40, tuple(s2.Context()))
    of = O.FC(120, 16)
    of.W = host(fc.LinearParams()); of.b = host(fc.BiasParams()); of.prev = host(fc.PrevGrad())
    a0 = o1.propagate_offsets(x, offs[0], offs[1], N)
    a1 = orl.propagate(a0)
    a2 = o2.propagate_offsets(a1, offs[2], offs[3], N)
    assert_same(outs[0], a0, "Splice 1 (gapped chunk offsets)")
    assert_same(outs[1], a1, "ReLU")
    assert_same(outs[2], a2, "Splice 2")
    # known answer, derived by hand (independent of oracle.chunk_offsets):
    # 11 input frames 0..10 per chunk; the first splice (-2..2) produces the
    # frames at offsets 2, 5, 8, i.e. output row 3n + j is input rows
    # 11n + 3j + 0..4 side by side; the second (-3, 0, 3) reads those three
    # rows of its chunk for its one output frame (offset 5)
    kat1 = np.stack([np.concatenate([x[11 * n + 3 * j + c] for c in range(5)])
                     for n in range(N) for j in range(3)])
    assert_same(outs[0], kat1, "Splice 1 known answer")
    kat2 = np.stack([np.concatenate([outs[1][3 * n + j] for j in range(3)]) for n in range(N)])
    assert_same(outs[2], kat2, "Splice 2 known answer")
    with O.accum(1):
        y_t = of.propagate(a2)
    np.testing.assert_allclose(outs[3], y_t, rtol=1e-5, atol=1e-6)
    net.Backprop(dev(dy))
    with O.accum(1):
        d3 = of.backprop(a2, dy, update=True)
    d2 = o2.backprop_offsets(d3, offs[2], offs[3], N)
    d1 = orl.backprop(a1, d2)
    d0 = o1.backprop_offsets(d1, offs[0], offs[1], N)
    np.testing.assert_allclose(host(net.InputDeriv(3)), d3, rtol=1e-5, atol=1e-6)
    # splice backprops and the ReLU backprop on the GPU's own derivatives
    g3 = host(net.InputDeriv(3))
    assert_same(host(net.InputDeriv(2)), o2.backprop_offsets(g3, offs[2], offs[3], N), "Splice 2 dX")
    g2 = host(net.InputDeriv(2))
    assert_same(host(net.InputDeriv(1)), orl.backprop(a1, g2, update=False), "ReLU dX")
    g1 = host(net.InputDeriv(1))
    assert_same(host(net.InputDeriv(0)), o1.backprop_offsets(g1, offs[0], offs[1], N), "Splice 1 dX")
    np.testing.assert_allclose(host(net.InputDeriv(0)), d0, rtol=1e-5, atol=1e-6)
    err = np.abs(host(fc.LinearParams()) - of.W).max() / np.abs(of.W).max()
    assert err < 1e-5, err
