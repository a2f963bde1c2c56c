"""GPU tests of the kcnn_nnet runtime (the NnetUpdater-style component stack,
include/kcnn.h kcnn_nnet_*), in particular its Conv -> Maxpool fusion:
ConvolutionComponent::PropagateMaxpool writes the pooled output and the pool's
routing mask in one pass (Y too in fusion mode 2), and the pool's Backprop
runs from the mask (MaxpoolComponent::BackpropFromMask), or for 1x1x4 / 1x1x8
pools and ph x 1 x pc windows (ph in {2, 3}, ph * pc <= 16) inside the conv's
backward (ConvolutionComponent::BackpropPooled).

The fusion is an exact transformation, so every output, input derivative and
updated parameter must be bit-identical with fusion on and off; the pool
output and the routed derivative are also checked bitwise against the oracle
(A.8 / A.9) applied to the GPU's own Y.
"""
import numpy as np
import pytest

import oracle as O
from _util import assert_same, dev, host, randn, rng

pytestmark = pytest.mark.gpu


def stack(H, W, C, kh, kw, G, pc, fc_out, ph=0, pw=0, qh=1, qw=1):
    """qh x qw x pc: the pool window (1 x 1 x pc: channel-only)."""
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    return "\n".join([
        f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} "
        f"in-pad-height={ph} in-pad-width={pw} kernel-height={kh} kernel-width={kw} "
        f"stride=1 group={G} out-height={oh} out-width={ow} learning-rate=0.02 "
        f"param-stddev=0.1 bias-stddev=0.5",
        f"MaxpoolComponent in-height={oh} in-width={ow} in-channel={G} "
        f"pool-height-dim={qh} pool-width-dim={qw} pool-channel-dim={pc}",
        f"FullyConnectedComponent input-dim={oh * ow * G // (pc * qh * qw)} output-dim={fc_out} "
        f"learning-rate=0.02 param-stddev=0.05 bias-stddev=1",
    ]), (oh, ow)


STACKS = {
    # name: (H, W, C, kh, kw, G, pc, fc_out, pad_h, pad_w)
    "c2": (40, 11, 3, 8, 1, 128, 4, 64, 0, 0),      # BASELINE c2 shape
    "pc2_G96": (12, 7, 2, 3, 2, 96, 2, 32, 0, 0),
    "pc8_G64": (9, 5, 1, 2, 2, 64, 8, 16, 0, 0),
    "G48_pad": (6, 5, 2, 3, 3, 48, 4, 8, 1, 1),     # last filter group of 16 maps
    "G40_pc4": (10, 6, 2, 3, 2, 40, 4, 8, 0, 0),    # bf16x6 forward: pooled rows past G
    "pc3_unfused": (8, 6, 1, 3, 1, 30, 3, 8, 0, 0),  # not fusable: plain path
    "G256_pc4": (12, 6, 2, 4, 2, 256, 4, 16, 0, 0),  # 2 filter chunks of 128
    # G = 128, pc = 4 with 10 and 11 position tiles (P 300, 352): the f16x3
    # forward's register-pooled statistics form needs all 12, so these take
    # the generic item loop; the FC GEMM's scales from the fused forward's
    # statistics must equal the unfused statistics pass's (bitwise FC output)
    "G128_P300": (32, 10, 3, 3, 1, 128, 4, 16, 0, 0),
    "G128_P352": (39, 11, 3, 8, 1, 128, 4, 16, 0, 0),
    # 3-D windows (qh x qw x pc, 16-bit routing mask): (..., pad_h, pad_w, qh, qw)
    "c5_P1_3x1x4": (40, 11, 3, 8, 1, 256, 4, 16, 0, 0, 3, 1),
    "win_2x2x2": (9, 8, 2, 2, 1, 64, 2, 8, 0, 0, 2, 2),
    "win_2x1x8_pad": (6, 6, 1, 3, 3, 32, 8, 8, 1, 1, 2, 1),
    "win_2x1x4_G96": (10, 6, 2, 3, 2, 96, 4, 8, 0, 0, 2, 1),
    # the position-half pooled backward (conv_bwd_x6q_kernel) with a B half
    # (P > 256) at 2 and 3 slabs per frame, PCM = 8 and a 2 x 1 x 4 window
    "halfB_G64_pc8": (40, 9, 1, 8, 1, 64, 8, 8, 0, 0),
    "halfB_G96_2x1x4": (34, 10, 2, 3, 2, 96, 4, 8, 0, 0, 2, 1),
    # long kernels (implicit GEMM, the pool in its epilogue): c5's C3 -> P2
    # shape class, nnet.config's conv4 -> Maxpool(1x2x1), and pc = 2
    "long_2x1x4_pad": (8, 9, 16, 3, 3, 256, 4, 8, 1, 1, 2, 1),
    "long_1x2x1": (1, 14, 32, 1, 3, 64, 1, 8, 0, 0, 1, 2),
    "long_2x1x2_G96": (6, 5, 8, 3, 3, 96, 2, 8, 0, 0, 2, 1),
}
LONG_POOLED = ["long_2x1x4_pad", "long_1x2x1", "long_2x1x2_G96"]


def build(kc, cfg, seed, ties=False):
    H, W, C, kh, kw, G, pc, fo, ph, pw = cfg[:10]
    text, _ = stack(*cfg)
    net = kc.Nnet(text)
    conv, pool, fc = net.components
    r = rng(seed)
    Wc = randn(r, (kh * kw * C, G), 0.1)
    bc = randn(r, (G,), 0.5)
    if ties:  # the maps of every pool group identical: 4-way (pc-way) ties
        for j in range(G // pc):
            Wc[:, j * pc:(j + 1) * pc] = Wc[:, j * pc:j * pc + 1]
            bc[j * pc:(j + 1) * pc] = bc[j * pc]
    conv.SetParam(kc.PARAM_LINEAR, dev(Wc))
    conv.SetParam(kc.PARAM_BIAS, dev(bc))
    conv.SetParam(kc.PARAM_PREV_GRAD, dev(randn(r, (kh * kw * C, G), 0.01)))
    fc.SetParam(kc.PARAM_LINEAR, dev(randn(r, (fo, fc.InputDim()), 0.05)))
    return net


def run(kc, cfg, fused, ties=False, N=37, mode=0):
    kc.set_fusion(fused)
    try:
        net = build(kc, cfg, seed=11, ties=ties)
        r = rng(3)
        x = dev(randn(r, (N, net.components[0].InputDim())))
        dy = dev(randn(r, (N, net.components[2].OutputDim()), 0.1))
        net.Propagate(x)
        outs = [host(net.Output(i)) for i in range(3)]
        grads = None
        if mode == 0:
            net.Backprop(dy)
        else:
            import torch
            grads = [torch.zeros(c.NumGradientParams(), device="cuda")
                     if k != 1 else None for k, c in enumerate(net.components)]
            for i in (2, 1, 0):
                net.BackpropComponent(i, dy, mode=1, grad=grads[i], skip_first_dx=False)
            grads = [host(g[None, :]) if g is not None else None for g in grads]
        derivs = [host(net.InputDeriv(i)) for i in range(3)]
        params = [host(c.GetParam(w)) for c in (net.components[0], net.components[2])
                  for w in (kc.PARAM_LINEAR, kc.PARAM_BIAS)]
        return outs, derivs, params, grads
    finally:
        kc.set_fusion(1)


@pytest.mark.parametrize("name", sorted(STACKS))
@pytest.mark.parametrize("ties", [False, True])
def test_fusion_is_exact(kc, name, ties):
    cfg = STACKS[name]
    a = run(kc, cfg, fused=True, ties=ties)
    b = run(kc, cfg, fused=False, ties=ties)
    for k, (u, v) in enumerate(zip(a[0], b[0])):
        assert_same(u, v, f"{name} output {k}")
    for k, (u, v) in enumerate(zip(a[1], b[1])):
        assert_same(u, v, f"{name} input deriv {k}")
    for k, (u, v) in enumerate(zip(a[2], b[2])):
        assert_same(u, v, f"{name} param {k}")


@pytest.mark.parametrize("name", ["c2", "c5_P1_3x1x4", "long_2x1x4_pad", "long_1x2x1"])
def test_fusion_storing_conv_output(kc, name):
    """Mode 2 stores Y in the fused pass; mode 1 recomputes it on request."""
    a = run(kc, STACKS[name], fused=2)
    b = run(kc, STACKS[name], fused=1)
    for k in range(3):
        for i in range(3 if k < 2 else 4):
            assert_same(a[k][i], b[k][i], f"{name} {k}/{i}")


def test_unstored_conv_output_after_backprop(kc):
    """Mode 1: the conv output of a fused pair is gone once its backprop ran."""
    cfg = STACKS["c2"]
    for mode in (1, 2):
        kc.set_fusion(mode)
        try:
            net = build(kc, cfg, seed=11)
            r = rng(3)
            x = dev(randn(r, (8, net.components[0].InputDim())))
            net.Propagate(x)
            net.Backprop(dev(randn(r, (8, net.components[2].OutputDim()), 0.1)))
            if mode == 1:
                with pytest.raises(Exception, match="not stored"):
                    net.Output(0)
            else:
                assert host(net.Output(0)).shape == (8, net.components[0].OutputDim())
        finally:
            kc.set_fusion(1)


@pytest.mark.parametrize("name", ["c2", "pc2_G96", "pc8_G64", "c5_P1_3x1x4", "win_2x1x8_pad",
                                  "halfB_G64_pc8", "halfB_G96_2x1x4"])
def test_fusion_exact_gradient_mode(kc, name):
    a = run(kc, STACKS[name], fused=True, mode=1)
    b = run(kc, STACKS[name], fused=False, mode=1)
    for k, (u, v) in enumerate(zip(a[3], b[3])):
        if u is not None:
            assert_same(u, v, f"{name} grad {k}")
    assert_same(a[1][0], b[1][0], f"{name} conv input deriv")


def _calls(kc, key):
    """Calls of one profile scope so far (the profile accumulates)."""
    for line in kc.profile_string().splitlines():
        parts = line.split("\t")
        if parts[0] == key:
            return int(parts[2].split()[0])
    return 0


@pytest.mark.parametrize("name,pooled", [("c2", True), ("pc8_G64", True), ("G256_pc4", True),
                                         ("c5_P1_3x1x4", True), ("win_2x1x8_pad", True),
                                         ("win_2x1x4_G96", True), ("pc2_G96", False),
                                         ("G48_pad", False), ("win_2x2x2", False)])
def test_pooled_backward_path(kc, name, pooled):
    """Fusion mode 1 runs a 1x1x4 / 1x1x8 pool's Backprop (and a 3x1x4, 2x1x4,
    2x1x8 window's) inside the conv's
    (ConvolutionComponent::BackpropPooled); other shapes fall back to
    BackpropFromMask + the conv's own Backprop (the exactness tests above
    cover both routes)."""
    key = "ConvolutionComponent::BackpropPooled"
    kc.set_profiling(True)
    try:
        before = _calls(kc, key)
        run(kc, STACKS[name], fused=1)
        after = _calls(kc, key)
    finally:
        kc.set_profiling(False)
    assert (after > before) == pooled


@pytest.mark.parametrize("name", ["c2", "c5_P1_3x1x4", "win_2x1x8_pad", "win_2x1x4_G96",
                                  "halfB_G64_pc8", "halfB_G96_2x1x4"] + LONG_POOLED)
@pytest.mark.parametrize("ties", [False, True])
def test_fused_pool_matches_oracle(kc, name, ties):
    cfg = STACKS[name]
    H, W, C, kh, kw, G, pc, fo, ph, pw = cfg[:10]
    qh, qw = (cfg[10], cfg[11]) if len(cfg) > 10 else (1, 1)
    outs, derivs, _, _ = run(kc, cfg, fused=True, ties=ties)
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    y, p = outs[0], outs[1]
    assert_same(p, O.maxpool_prop(y, oh, ow, qh, qw, pc, p.shape[1]), "fused Maxpool_prop")
    dp = derivs[2]
    assert_same(derivs[1], O.maxpool_backprop(y, p, dp, oh, ow, qh, qw, pc),
                "mask-routed Maxpool_backprop")
    if ties and qh * qw == 1:  # every map of a group is a maximum: all get the derivative
        assert (derivs[1] != 0).mean() > 0.99 * (dp != 0).mean()


@pytest.mark.parametrize("name,fused", [("c2", True), ("c5_P1_3x1x4", True),
                                        ("long_2x1x4_pad", True), ("long_1x2x1", True),
                                        ("long_2x1x2_G96", True), ("pc3_unfused", False)])
def test_fused_forward_path(kc, name, fused):
    """The conv + pool forward runs as one pass (PropagateMaxpool) for the
    frame kernels' pools and for two-position windows after long kernels
    (the implicit GEMM's pooled epilogue); other pools run unfused."""
    key = "ConvolutionComponent::PropagateMaxpool"
    kc.set_profiling(True)
    try:
        before = _calls(kc, key)
        run(kc, STACKS[name], fused=1)
        after = _calls(kc, key)
    finally:
        kc.set_profiling(False)
    assert (after > before) == fused


# Conv -> RectifiedLinearComponent: fusion mode 1 runs the ReLU in the conv's
# forward epilogue (ConvolutionComponent::PropagateRelu, implicit-GEMM shapes)
RELU_STACKS = {
    # name: (H, W, C, kh, kw, G, pad, fused)
    "ig2": (9, 8, 8, 3, 3, 64, 0, True),        # kh*kw*C = 72: implicit GEMM v2
    "ig2_pad": (8, 9, 8, 3, 3, 128, 1, True),   # padded, 2 filter groups per block
    "c2_frame": (40, 11, 3, 8, 1, 128, 0, False),  # frame kernels: ReLU runs separately
    "nnet_conv2": (1, 18, 128, 1, 3, 128, 0, True),  # nnet.config's second conv
    "direct_g8": (8, 8, 8, 3, 3, 8, 0, False),   # G <= 8: direct kernel, ReLU separate
}


def relu_stack(H, W, C, kh, kw, G, pad):
    oh, ow = H + 2 * pad - kh + 1, W + 2 * pad - kw + 1
    return "\n".join([
        f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} "
        f"in-pad-height={pad} in-pad-width={pad} kernel-height={kh} kernel-width={kw} "
        f"stride=1 group={G} out-height={oh} out-width={ow} learning-rate=0.02 "
        f"param-stddev=0.1 bias-stddev=0.5",
        f"RectifiedLinearComponent dim={oh * ow * G}",
        f"FullyConnectedComponent input-dim={oh * ow * G} output-dim=16 "
        f"learning-rate=0.02 param-stddev=0.05 bias-stddev=1",
    ])


def run_relu(kc, cfg, mode, N=33):
    kc.set_fusion(mode)
    try:
        net = kc.Nnet(relu_stack(*cfg[:7]))
        conv, _, fc = net.components
        r = rng(5)
        conv.SetParam(kc.PARAM_LINEAR, dev(randn(r, (cfg[3] * cfg[4] * cfg[2], cfg[5]), 0.1)))
        conv.SetParam(kc.PARAM_BIAS, dev(randn(r, (cfg[5],), 0.5)))
        fc.SetParam(kc.PARAM_LINEAR, dev(randn(r, (16, fc.InputDim()), 0.05)))
        x = dev(randn(r, (N, net.components[0].InputDim())))
        dy = dev(randn(r, (N, 16), 0.1))
        net.Propagate(x)
        outs = [host(net.Output(i)) for i in range(3)]
        net.Backprop(dy)
        derivs = [host(net.InputDeriv(i)) for i in range(3)]
        params = [host(c.GetParam(w)) for c in (net.components[0], net.components[2])
                  for w in (kc.PARAM_LINEAR, kc.PARAM_BIAS)]
        vs, ds, cnt = net.components[1].NonlinearStats()
        return outs, derivs, params, (np.asarray(vs), np.asarray(ds), cnt)
    finally:
        kc.set_fusion(1)


@pytest.mark.parametrize("name", sorted(RELU_STACKS))
def test_conv_relu_fusion_is_exact(kc, name):
    cfg = RELU_STACKS[name]
    key = "ConvolutionComponent::PropagateRelu"
    kc.set_profiling(True)
    try:
        before = _calls(kc, key)
        a = run_relu(kc, cfg, 1)
        after = _calls(kc, key)
    finally:
        kc.set_profiling(False)
    assert (after > before) == cfg[7]
    b = run_relu(kc, cfg, 0)
    for k in range(3):
        for i, (u, v) in enumerate(zip(a[k], b[k])):
            assert_same(u, v, f"{name} {k}/{i}")
    assert np.array_equal(a[3][0], b[3][0]) and np.array_equal(a[3][1], b[3][1])
    assert a[3][2] == b[3][2]
    assert (a[0][1] >= 0).all()


# The pooled backward (conv_bwd_x6q_kernel) carries state from one frame to
# the next inside a workgroup (the next frame's im2col gather in the last
# slab's P_A, the previous frame's col2im spread over P_A, n1/n2 wrap-around);
# that loop runs only when the frames outnumber the grid (256 workgroups).
# 601 frames (not a multiple of 256, more than 2 frames per workgroup) run
# every variant through it: fusion on/off bitwise (the unfused backward is a
# different kernel, conv_bwd_x6_kernel, also grid-striding) and the whole step
# (outputs, input derivatives, the update) against the oracle.
CROSS_FRAME = ["halfB_G64_pc8", "halfB_G96_2x1x4", "win_2x1x4_G96", "c5_P1_3x1x4", "pc8_G64"]


@pytest.mark.parametrize("name", CROSS_FRAME)
def test_pooled_backward_across_frames(kc, name):
    from _stack import check_step
    cfg = STACKS[name]
    N = 601
    a = run(kc, cfg, fused=True, N=N)
    b = run(kc, cfg, fused=False, N=N)
    for k, (u, v) in enumerate(zip(a[1], b[1])):
        assert_same(u, v, f"{name} input deriv {k} at {N} frames")
    for k, (u, v) in enumerate(zip(a[2], b[2])):
        assert_same(u, v, f"{name} param {k} at {N} frames")
    kc.set_fusion(1)
    net = build(kc, cfg, seed=11)
    r = rng(3)
    x = dev(randn(r, (N, net.components[0].InputDim())))
    dy = dev(randn(r, (N, net.components[2].OutputDim()), 0.1))
    check_step(kc, stack(*cfg)[0], net, x, dy, what=f"{name} N={N}")
