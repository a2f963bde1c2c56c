"""Parity at BASELINE.json's sizes (the configurations the bench lines are
measured on), layer by layer against the oracle (tests/_stack.py):

  * c1 (configs[0]): the Conv -> Maxpool forward at its 256 frames;
  * c2 (configs[1]): the exact bench.py step -- its stack, its parameters
    (kcnn_set_randn_seed 20261015), its inputs, 4096 frames, fusion mode 1,
    the default kernels -- with every output, input derivative and updated
    parameter checked;
  * c3 (configs[2]): the same stack at 65536 frames, with the conv output
    stored (fusion mode 0: Y has 3.04e9 elements, past 2^31) and
    in the default mode, on sampled rows including the last ones and those
    on both sides of element 2^31;
  * c5 (configs[4]): the whole deep stack end to end at a small batch;
  * the host guards' fallbacks: shapes and strides past the limits of the
    fast kernels' 32-bit addressing (a conv input over 2 GB, pools with more
    than 2^31 outputs / 2^33 inputs) run the general kernels, which must
    give the same results.
"""
import numpy as np
import pytest

import bench
import oracle as O
from _stack import check_step, oracle_layers, truth
from _util import assert_bound, assert_same, host, rng

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _inputs(B, in_cols, out_cols, seed=20261015):
    import torch
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    x = torch.randn((B, in_cols), generator=gen, device="cuda")
    dy = torch.randn((B, out_cols), generator=gen, device="cuda") * 1e-2
    return x, dy


@pytest.mark.parametrize("fusion", [0, 1])
def test_c1_forward(kc, fusion):
    """BASELINE configs[0]: Conv(40x11x3, 8x1, 128) -> Maxpool(1x1x4), forward
    only, 256 frames (the reference's --use-gpu=no case, here on the GPU)."""
    kc.set_fusion(fusion)
    try:
        kc.set_randn_seed(20261015)
        cfg = "\n".join(bench.stack_config().splitlines()[:2])
        net = kc.Nnet(cfg)
        x, _ = _inputs(256, bench.H * bench.W * bench.C, 1)
        conv, pool = oracle_layers(cfg, net, kc)
        net.Propagate(x)
        y, p = host(net.Output(0)), host(net.Output(1))
        xh = host(x)
        y_t, y_s = truth(lambda: conv.propagate(xh))
        assert_bound(y, y_t, y_s, what="c1 conv Propagate")
        assert_same(p, pool.propagate(y), "c1 maxpool Propagate")
    finally:
        kc.set_fusion(1)


def test_c2_bench_step(kc):
    """The step bench.py times (BASELINE configs[1]), checked whole."""
    kc.set_fusion(1)
    kc.set_randn_seed(20261015)
    cfg = bench.stack_config()
    net = kc.Nnet(cfg)
    x, dy = _inputs(4096, bench.H * bench.W * bench.C, bench.FC_OUT)
    check_step(kc, cfg, net, x, dy, what="c2@4096")


def _c3_rows(B, row_elems):
    """64 rows: spread over the batch, the last rows, and the rows around
    element 2^31 of the conv output."""
    r = np.linspace(0, B - 1, 56).astype(np.int64)
    edge = (1 << 31) // row_elems
    extra = [edge - 1, edge, edge + 1, B - 3, B - 2, B - 1, 1, 0]
    return np.unique(np.concatenate([r, extra]))


@pytest.mark.parametrize("fusion", [0, 1])
def test_c3_sampled_rows(kc, fusion):
    """BASELINE configs[2]: 65536 frames on one GPU.  Row-local outputs and
    input derivatives of every layer on sampled rows."""
    import torch
    B = 65536
    y_elems = bench.P * bench.G
    assert B * y_elems > (1 << 31)
    kc.set_fusion(fusion)
    try:
        kc.set_randn_seed(20261015)
        cfg = bench.stack_config()
        net = kc.Nnet(cfg)
        x, dy = _inputs(B, bench.H * bench.W * bench.C, bench.FC_OUT, seed=3)
        rows = _c3_rows(B, y_elems)
        check_step(kc, cfg, net, x, dy, rows=rows, what=f"c3 fusion {fusion}")
    finally:
        kc.set_fusion(1)
        del net
        torch.cuda.empty_cache()


def test_c5_whole_stack(kc):
    """BASELINE configs[4]: the deep stack end to end (fusion mode 1: C1's
    3x1x4 pool and C3's 2x1x4 pool fused), every layer and update."""
    kc.set_fusion(1)
    kc.set_randn_seed(5)
    cfg, _, _ = bench.c5_config()
    net = kc.Nnet(cfg)
    x, dy = _inputs(40, 40 * 11 * 3, bench.FC_OUT, seed=9)
    check_step(kc, cfg, net, x, dy, what="c5")


# ---- host-guard fallbacks ------------------------------------------------------

def _huge_stride_view(a, stride):
    """Device copy of `a` [R x c] as a view with row stride `stride` floats."""
    import torch
    R, c = a.shape
    base = torch.zeros((R, stride), dtype=torch.float32, device="cuda")
    base[:, :c] = torch.from_numpy(a).cuda()
    return base[:, :c]


def test_conv_input_over_2gb_fallback(kc):
    """A long-kernel conv whose input rows span more than 2^31 bytes (row
    stride 60 M floats): the bf16x6 implicit GEMM and the fp32 implicit GEMM
    v2 decline (32-bit buffer offsets, cnsl-conv-igemm-x6.hip
    igemm_x6_blocks, cnsl-conv-mfma.hip conv2d_impl) and the general
    implicit-GEMM kernel runs; the backward's kernels take their own
    fallbacks.  Results equal the oracle's."""
    import torch
    from test_gpu_components import make_pair
    cfg = (8, 9, 16, 3, 3, 64, 1, 1)            # Kdim 144: the implicit-GEMM family
    H, W, C, kh, kw, G, ph, pw = cfg
    comp, oc = make_pair(kc, cfg, seed=4)
    r = rng(8)
    N = 9
    stride = 60 * (1 << 20)
    assert N * stride * 4 >= (1 << 31)
    x = (r.standard_normal((N, H * W * C))).astype(np.float32)
    xv = _huge_stride_view(x, stride)
    y_t, y_s = truth(lambda: oc.propagate(x))
    assert_bound(host(comp.Propagate(xv)), y_t, y_s, what="Propagate, 2 GB input")
    dy = r.standard_normal(y_t.shape).astype(np.float32)
    dyv = _huge_stride_view(dy, stride)
    dx_t, dx_s = truth(lambda: oc.backprop(x, dy, update=False))
    (gW_t, gb_t), (gW_s, gb_s) = truth(lambda: oc.gradient(x, dy))
    dx, g = comp.BackpropGradient(xv, dyv)
    g = host(g)
    kd = kh * kw * C
    assert_bound(host(dx), dx_t, dx_s, what="dX, 2 GB input")
    assert_bound(g[:kd * G].reshape(kd, G), gW_t, gW_s, what="gW, 2 GB input")
    assert_bound(g[kd * G:], gb_t, gb_s, what="gb, 2 GB input")
    del xv, dyv
    torch.cuda.empty_cache()


def _tied_rows(shape, seed):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(-7, 8, shape, generator=g, dtype=torch.float32,
                         device="cuda").mul_(0.25)


@pytest.mark.parametrize("case", ["channel_1x1x4_2^31_outputs", "window_3x1x4_2^33_inputs"])
def test_maxpool_fallbacks_past_32_bits(kc, case):
    """Maxpool shapes past the direct kernels' limits (hipF_maxpool_prop /
    hipF_maxpool_backprop: more than 2^31 pooled values; the 16-B window
    backprop: 2^33 inputs or more) run the element-wise gather kernels with
    64-bit offsets.  Bit-exact on sampled rows, ties included."""
    import torch
    if case.startswith("channel"):
        H, W, C, ph, pw, pc = 33, 11, 128, 1, 1, 4
        rows = (1 << 31) // (H * W * C // pc) + 5
    else:
        H, W, C, ph, pw, pc = 33, 11, 256, 3, 1, 4
        rows = (1 << 33) // (H * W * C) + 5
    comp = kc.Component.NewFromString(
        f"MaxpoolComponent in-height={H} in-width={W} in-channel={C} "
        f"pool-height-dim={ph} pool-width-dim={pw} pool-channel-dim={pc}")
    op = O.Pool(H, W, C, ph, pw, pc)
    x = _tied_rows((rows, H * W * C), 1)
    y = comp.Propagate(x)
    if case.startswith("channel"):
        assert y.numel() >= (1 << 31)
    else:
        assert x.numel() >= (1 << 33)
    dy = _tied_rows(tuple(y.shape), 2)
    dx = comp.Backprop(x, y, dy)
    sample = np.unique(np.concatenate([np.linspace(0, rows - 1, 24).astype(np.int64),
                                       [rows - 2, rows - 1]]))
    idx = torch.as_tensor(sample, device="cuda")
    xs, ys, dys, dxs = (host(t.index_select(0, idx)) for t in (x, y, dy, dx))
    assert_same(ys, op.propagate(xs), f"{case} Propagate")
    assert_same(dxs, op.backprop(xs, ys, dys), f"{case} Backprop")
    del x, y, dy, dx
    torch.cuda.empty_cache()
