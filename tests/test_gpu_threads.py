"""Re-entrancy of the const component API (SURVEY 8(b) Threading).

The reference's Propagate / Backprop are const (nnet-component-nnet0.h:23-191)
and upstream's nnet-train-parallel calls them from several host threads on
one model (egs/steps/nnet0/train_conv_dropout.sh:205-208).  Here 4 host
threads share one Conv, one Maxpool and one FC component and each runs
Propagate and Backprop(to_update = NULL) on its own inputs, several times,
through the C-ABI (ctypes releases the GIL, so the calls overlap on the
host).  Every thread's outputs and input derivatives must match the oracle,
bit-exact for the pool, and the shared parameters must be unchanged.
"""
import threading

import numpy as np
import pytest

import oracle as O
from _util import assert_bound, assert_same, dev, host, randn, rng, triple

pytestmark = pytest.mark.gpu

H, W, C, KH, KW, G, PC, F = 40, 11, 3, 8, 1, 128, 4, 96
OH, OW = H - KH + 1, W - KW + 1
NTHREADS, REPS = 4, 3


def _components(kc):
    conv = kc.Component.NewFromString(
        f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} kernel-height={KH} "
        f"kernel-width={KW} stride=1 group={G} out-height={OH} out-width={OW} "
        f"learning-rate=0.02 param-stddev=0.1 bias-stddev=0.5")
    pool = kc.Component.NewFromString(
        f"MaxpoolComponent in-height={OH} in-width={OW} in-channel={G} pool-height-dim=1 "
        f"pool-width-dim=1 pool-channel-dim={PC}")
    I = OH * OW * G // PC
    fc = kc.Component.NewFromString(
        f"FullyConnectedComponent input-dim={I} output-dim={F} learning-rate=0.02 "
        f"param-stddev=0.01 bias-stddev=1 weight-decay=0.0002 momentum=0.9")
    r = rng(17)
    oc = O.Conv(H, W, C, KH, KW, G)
    oc.W = randn(r, (KH * KW * C, G), 0.1)
    oc.b = randn(r, (G,), 0.5)
    oc.prev = randn(r, (KH * KW * C, G), 0.01)
    for which, v in ((kc.PARAM_LINEAR, oc.W), (kc.PARAM_BIAS, oc.b),
                     (kc.PARAM_PREV_GRAD, oc.prev)):
        conv.SetParam(which, dev(v))
    of = O.FC(I, F)
    of.W = randn(r, (F, I), 0.02)
    of.b = randn(r, (F,), 0.5)
    of.prev = randn(r, (F, I), 0.01)
    for which, v in ((0, of.W), (1, of.b), (2, of.prev)):
        fc.SetParam(which, dev(v))
    op = O.Pool(OH, OW, G, 1, 1, PC)
    return (conv, pool, fc), (oc, op, of)


def _params(comps):
    conv, _, fc = comps
    return [host(t).copy() for t in (conv.LinearParams(), conv.BiasParams(), conv.PrevGrad(),
                                     fc.LinearParams(), fc.BiasParams(), fc.PrevGrad())]


@pytest.mark.parametrize("frames", [37, 300])
def test_const_api_reentrant_across_threads(kc, frames):
    import torch
    comps, orc = _components(kc)
    conv, pool, fc = comps
    oc, op, of = orc
    before = _params(comps)
    inputs = []
    for t in range(NTHREADS):
        r = rng(100 + t)
        inputs.append((randn(r, (frames, H * W * C)), randn(r, (frames, F), 1e-2)))

    results = [None] * NTHREADS
    errors = []
    start = threading.Barrier(NTHREADS)

    def work(t):
        try:
            x, dy = inputs[t]
            xd, dyd = dev(x), dev(dy)
            torch.cuda.synchronize()
            start.wait()
            for _ in range(REPS):
                y = conv.Propagate(xd)
                p = pool.Propagate(y)
                z = fc.Propagate(p)
                dp = fc.Backprop(p, None, dyd, update=False)
                dyc = pool.Backprop(y, p, dp, update=False)
                dx = conv.Backprop(xd, None, dyc, update=False)
            torch.cuda.synchronize()
            results[t] = tuple(host(a) for a in (y, p, z, dp, dyc, dx))
        except Exception as e:  # noqa: BLE001 -- reported on the main thread
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(NTHREADS)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads), "a thread did not finish"
    assert not errors, errors

    for t in range(NTHREADS):
        x, dy = inputs[t]
        y, p, z, dp, dyc, dx = results[t]
        _, y_t, y_s = triple(lambda: oc.propagate(x))
        assert_bound(y, y_t, y_s, what=f"thread {t} conv Propagate")
        # the pool's routing is checked bit-exact on the GPU's own conv output
        assert_same(p, op.propagate(y), f"thread {t} Maxpool Propagate")
        _, z_t, z_s = triple(lambda: of.propagate(p))
        assert_bound(z, z_t, z_s, what=f"thread {t} FC Propagate")
        _, dp_t, dp_s = triple(lambda: of.backprop(p, dy, update=False))
        assert_bound(dp, dp_t, dp_s, what=f"thread {t} FC dX")
        assert_same(dyc, op.backprop(y, p, dp), f"thread {t} Maxpool Backprop")
        _, dx_t, dx_s = triple(lambda: oc.backprop(x, dyc, update=False))
        assert_bound(dx, dx_t, dx_s, what=f"thread {t} conv dX")

    after = _params(comps)
    for b, a, name in zip(before, after, ("conv W", "conv b", "conv prev", "FC W", "FC b",
                                          "FC prev")):
        assert_same(a, b, f"{name} changed by Backprop(to_update = NULL)")
