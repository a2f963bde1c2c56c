"""Data-parallel step (kaldi-cnn_amd/kcnn_dp.py) on CPU: two gloo
ranks, each backpropagating its own row shard through a CPU stand-in of the
component stack (the oracle, oracle/), must end with exactly the parameters
of one process that trained on the whole batch -- the sum all-reduce plus
the update with the GLOBAL frame count reproduces the single-process math
(the reference divides by its local row count, nnet-component-nnet0.cc:767).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

import oracle as O
import kcnn_dp

CONV = (12, 5, 2, 3, 2, 4)        # H, W, C, kh, kw, G
POOL = (1, 1, 2)                   # ph, pw, pc
FC_OUT = 6
N_GLOBAL, STEPS = 8, 2


class _Comp:
    def __init__(self, oc):
        self.oc = oc

    def NumGradientParams(self):
        if isinstance(self.oc, O.Pool):
            return 0
        return self.oc.W.size + self.oc.b.size

    def ApplyGradient(self, grad, n):
        g = grad.numpy()
        nw = self.oc.W.size
        with O.accum(1):
            self.oc.apply(g[:nw].reshape(self.oc.W.shape).copy(), g[nw:].copy(), n)


class OracleNet:
    """kcnn.Nnet's host interface over the CPU oracle (test stand-in)."""

    def __init__(self, seed):
        H, W, C, kh, kw, G = CONV
        r = np.random.default_rng(seed)
        conv = O.Conv(H, W, C, kh, kw, G)
        conv.W = (r.standard_normal((kh * kw * C, G)) * 0.1).astype(np.float32)
        conv.b = (r.standard_normal(G) * 0.5).astype(np.float32)
        pool = O.Pool(conv.out_height, conv.out_width, G, *POOL)
        fc = O.FC(pool.output_dim, FC_OUT)
        fc.W = (r.standard_normal((FC_OUT, pool.output_dim)) * 0.1).astype(np.float32)
        fc.b = np.ones(FC_OUT, np.float32)
        self.components = [_Comp(conv), _Comp(pool), _Comp(fc)]

    def NumComponents(self):
        return 3

    def Propagate(self, x):
        self.fwd = [x.numpy()]
        with O.accum(1):
            for c in self.components:
                self.fwd.append(c.oc.propagate(self.fwd[-1]))
        self.deriv = [None] * 4

    def BackpropComponent(self, i, out_deriv, mode, grad=None, skip_first_dx=True):
        od = out_deriv.numpy() if i == 2 else self.deriv[i + 1]
        oc = self.components[i].oc
        with O.accum(1):
            if isinstance(oc, O.Pool):
                self.deriv[i] = oc.backprop(self.fwd[i], self.fwd[i + 1], od)
                return
            if mode != 3:  # mode 3: the gradient only
                self.deriv[i] = oc.backprop(self.fwd[i], od, update=False)
            if mode in (1, 3):
                gW, gb = oc.gradient(self.fwd[i], od)
                grad.copy_(torch.from_numpy(np.concatenate([gW.ravel(), gb])))


    def BackpropSplit(self, i, out_deriv, grad, skip_first_dx, between):
        """kcnn_nnet_backprop_split: mode 3, between(), mode 2."""
        self.BackpropComponent(i, out_deriv, 3, grad, skip_first_dx)
        between()
        self.BackpropComponent(i, out_deriv, 2, None, skip_first_dx)


def _data():
    H, W, C = CONV[:3]
    r = np.random.default_rng(77)
    xs = [r.standard_normal((N_GLOBAL, H * W * C)).astype(np.float32) for _ in range(STEPS)]
    dys = [(r.standard_normal((N_GLOBAL, FC_OUT)) * 0.1).astype(np.float32) for _ in range(STEPS)]
    return xs, dys


def _params(net):
    return [np.concatenate([c.oc.W.ravel(), c.oc.b]) for c in net.components
            if not isinstance(c.oc, O.Pool)]


def _worker(rank, world, port, q, split):
    kcnn_dp.SPLIT_GRADIENT_PARAMS = split
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    net = OracleNet(seed=5)                              # identical replicas
    grads = kcnn_dp.gradient_buffers(net, lambda n: torch.empty(n))
    xs, dys = _data()
    per = N_GLOBAL // world
    for x, dy in zip(xs, dys):
        sl = slice(rank * per, (rank + 1) * per)         # this rank's row shard
        kcnn_dp.dp_train_step(net, torch.from_numpy(x[sl]), torch.from_numpy(dy[sl]),
                              grads, tdist, N_GLOBAL)
    q.put((rank, _params(net)))
    tdist.barrier()
    tdist.destroy_process_group()


class _LocalDist:
    """world_size 1: the all-reduce is the identity (counted)."""
    class _W:
        def wait(self):
            pass

    def __init__(self):
        self.sizes = []

    def all_reduce(self, t, async_op=False):
        self.sizes.append(t.numel())
        return self._W()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("split", [1 << 20, 1, 100])
def test_dp_two_ranks_equal_one_process(split, monkeypatch):
    """split = 1 << 20: both gradients in the flat bucket (one all-reduce);
    split = 1: every gradient on its own (mode 3) with its all-reduce
    started before the layer's data gradient (mode 2); split = 100: the FC
    gradient (486 values) on its own, the conv's (52) in the bucket."""
    monkeypatch.setattr(kcnn_dp, "SPLIT_GRADIENT_PARAMS", split)
    ref = OracleNet(seed=5)
    grads = kcnn_dp.gradient_buffers(ref, lambda n: torch.empty(n))
    for x, dy in zip(*_data()):
        kcnn_dp.dp_train_step(ref, torch.from_numpy(x), torch.from_numpy(dy), grads,
                              _LocalDist(), N_GLOBAL)
    want = _params(ref)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, split)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        for a, b in zip(got[r], want):
            # same math up to the fp32 rounding of a 2-way split of each sum
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(got[0], got[1]):
        np.testing.assert_array_equal(a, b)             # replicas stay identical


def test_dp_update_uses_global_count():
    """With the per-rank (local) count the result differs: the DP step must
    divide by N_global, not by the shard's rows."""
    a, b = OracleNet(seed=5), OracleNet(seed=5)
    x, dy = (t[0] for t in _data())
    for net, n in ((a, N_GLOBAL), (b, N_GLOBAL // 2)):
        g = kcnn_dp.gradient_buffers(net, lambda k: torch.empty(k))
        kcnn_dp.dp_train_step(net, torch.from_numpy(x), torch.from_numpy(dy), g,
                              _LocalDist(), n)
    assert not np.allclose(_params(a)[0], _params(b)[0])


@pytest.mark.parametrize("split,want", [(1 << 20, [52 + 486]), (1, [486, 52]), (100, [486, 52])])
def test_dp_collectives_per_step(split, want, monkeypatch):
    """The step issues one all-reduce per large gradient, in backprop order,
    then one for the flat bucket of all the others (the conv's
    filter and bias gradients in a single all-reduce)."""
    monkeypatch.setattr(kcnn_dp, "SPLIT_GRADIENT_PARAMS", split)
    net = OracleNet(seed=5)
    grads = kcnn_dp.gradient_buffers(net, lambda n: torch.zeros(n))
    assert grads.num_collectives() == len(want)
    d = _LocalDist()
    x, dy = (t[0] for t in _data())
    marks = []
    kcnn_dp.dp_train_step(net, torch.from_numpy(x), torch.from_numpy(dy), grads, d,
                          N_GLOBAL, mark=marks.append)
    assert d.sizes == want
    assert marks == ["wait_begin", "wait_end"]
    if grads.bucket is not None:
        # the bucket's views alias one contiguous buffer
        assert sum(grads[i].numel() for i in grads.small) == grads.bucket.numel()
        assert grads[grads.small[0]].data_ptr() == grads.bucket.data_ptr()
