"""c5 (BASELINE configs[4]) at the bench's size with the default kernel
families.

The f16x3 implicit GEMM (igemm_x6 family 2) takes a convolution only when it
is worth >= 2^34 flop (cnsl-conv-igemm-x6.hip use_f16): at c5 that is C2's
and C3's forward, C3's data gradient and C2's 1x1 data gradient once a call
holds more than ~200 frames, so the 40-frame whole-stack test
(test_gpu_fullsize.py) never reaches it.  Here:

  * test_c5_sampled_rows: the whole c5 step at 4096 frames, exactly as
    `bench.py --config c5` runs it: every layer's outputs and input
    derivatives on 64 sampled rows (the oracle on the GPU's own inputs of
    each layer, tests/_stack.py), every update against a float64 gradient of
    the whole batch (device_gradient), and kcnn_conv_fix_counts showing the
    f16x3 implicit GEMM ran;
  * test_c3_pool_adversarial: C3 -> P2 (fused: the pool in the implicit
    GEMM's epilogue) at 4096 frames with frames whose values span 2^28: some
    with a few channels far under the rest (a handful of outputs fail the
    store check and are recomputed one by one, conv_igemm_efix_kernel, which
    re-pools their windows) and one whose every value but one is tiny (every
    tile touching it is recomputed, conv_igemm_fixup_kernel).  Both lists are
    asserted non-empty through the C-ABI's counters, and the sampled rows
    (the adversarial frames among them) and the update are checked as above.

Reference: nnet-component-nnet0.cc:423-446 (Propagate), :461-544
(Backprop), :738-777 (Update), :869-892 (Maxpool); conv2D.cc:43-201.
"""
import numpy as np
import pytest

import bench
from _stack import check_step

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

B = 4096


def _sample_rows(extra=()):
    r = np.linspace(0, B - 1, 56).astype(np.int64)
    return np.unique(np.concatenate([r, np.array([0, 1, B - 3, B - 2, B - 1] + list(extra),
                                                  dtype=np.int64)]))


def test_c5_sampled_rows(kc):
    import torch
    kc.set_fusion(1)
    kc.set_randn_seed(20261015)
    cfg, _, _ = bench.c5_config()
    net = kc.Nnet(cfg)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(20261015)
    x = torch.randn((B, 40 * 11 * 3), generator=gen, device="cuda")
    dy = torch.randn((B, bench.FC_OUT), generator=gen, device="cuda") * 1e-2
    kc.conv_fix_counts(reset=True)
    try:
        check_step(kc, cfg, net, x, dy, rows=_sample_rows(), what="c5@4096")
        calls, tiles, elems = kc.conv_fix_counts()
        print(f"\nc5@4096: {calls} f16x3 calls, {tiles} tiles and {elems} elements "
              "recomputed in fp32")
        # C2, C3 forward, C3 data gradient, C2's 1x1 data gradient (plus the
        # outputs recomputed on request for the check)
        assert calls >= 4, (calls, tiles, elems)
    finally:
        del net
        torch.cuda.empty_cache()


# C3 (8x9x256, 3x3, pad 1, 256 filters) -> P2 (2x1x4), as in c5
def _c3_p2_config():
    h, w, c, kh, kw, g, pad = bench.C5_LAYERS[3][1]
    ph, pw, pc = bench.C5_LAYERS[4][1]
    oh, ow = h + 2 * pad - kh + 1, w + 2 * pad - kw + 1
    return "\n".join([
        f"ConvolutionComponent in-height={h} in-width={w} in-channel={c} "
        f"in-pad-height={pad} in-pad-width={pad} kernel-height={kh} kernel-width={kw} "
        f"stride=1 group={g} out-height={oh} out-width={ow} learning-rate=0.02 "
        f"param-stddev=0.01 bias-stddev=0.5",
        f"MaxpoolComponent in-height={oh} in-width={ow} in-channel={g} "
        f"pool-height-dim={ph} pool-width-dim={pw} pool-channel-dim={pc}"]), (h, w, c, oh, ow, g,
                                                                               ph, pw, pc)


def test_c3_pool_adversarial(kc):
    import torch
    cfg, (h, w, c, oh, ow, g, ph, pw, pc) = _c3_p2_config()
    hw = h * w
    kc.set_fusion(1)
    kc.set_randn_seed(7)
    net = kc.Nnet(cfg)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(77)
    x = torch.randn((B, hw * c), generator=gen, device="cuda")
    out_dim = (oh // ph) * (ow // pw) * (g // pc)
    dp = torch.randn((B, out_dim), generator=gen, device="cuda") * 1e-2
    # element-level frames: 8 of the 256 channels (channel c is the run
    # [c*HW, (c+1)*HW) of a row) 2^28 under the rest -- the frame's scale
    # group is spread and its small elements few, so only outputs that come
    # out near zero fail the check (simulated: ~4 per frame, at most 4 in any
    # wave's 64 x 64 block, below the 8 a wave lists); one frame in 64, so two
    # never share a wave.  The same frames' pooled derivatives: 16 of the 64
    # pooled channels 2^28 under the rest (the data gradient's groups)
    spread_frames = list(range(5, B, 64))
    sf = torch.as_tensor(spread_frames, device="cuda")
    x[sf, :8 * hw] *= 2.0 ** -28
    pq = (oh // ph) * (ow // pw)
    dp[sf, :16 * pq] *= 2.0 ** -28
    # a tile-level frame: one value 1, every other 2^-28 of N(0,1)
    ft = B // 2 + 3
    x[ft] *= 2.0 ** -28
    x[ft, 100] = 1.0
    kc.conv_fix_counts(reset=True)
    rows = _sample_rows(spread_frames[::8] + [spread_frames[-1], ft, ft - 1, ft + 1])
    try:
        check_step(kc, cfg, net, x, dp, rows=rows, what="C3->P2 adversarial")
        calls, tiles, elems = kc.conv_fix_counts()
        print(f"\nC3->P2 adversarial: {calls} f16x3 calls, {tiles} tiles and {elems} "
              "elements recomputed in fp32")
        assert calls >= 2, (calls, tiles, elems)      # forward and data gradient
        assert tiles > 0, (calls, tiles, elems)       # conv_igemm_fixup_kernel
        assert elems > 0, (calls, tiles, elems)       # conv_igemm_efix_kernel
    finally:
        del net
        torch.cuda.empty_cache()
