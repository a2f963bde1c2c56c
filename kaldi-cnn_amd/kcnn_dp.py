"""Data-parallel training step for a kcnn component stack.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm): the
minibatch is row-sharded -- frames are independent through Conv, Maxpool and
FC -- and every rank holds a full replica of the parameters.  The only
exchange is the parameter gradient, summed (fp32) by as few all-reduces as
the overlap allows:

  * every gradient shorter than SPLIT_GRADIENT_PARAMS values -- all the
    convolutions' filter and bias gradients (c2: 3,200 values; c5: four
    layers, 1.2 M) -- lives in ONE flat bucket and is reduced by one
    all-reduce once the last of them exists (north_star's single all-reduce
    of the filter/bias gradients);
  * a gradient at least that long (an FC layer's: 11.9 M values, 47.6 MB at
    c2) gets its own all-reduce, started as soon as that gradient is
    computed (kcnn_nnet_backprop_component mode 3) and before the layer's
    data gradient (mode 2), so it runs over xGMI beside the FC dX GEMM and
    the conv/maxpool backward below it.

So the c2 and c5 steps issue two collectives, nnet.config four (three FC
layers + the bucket).  Every replica then applies the reference's update
step (nnet-component-nnet0.cc:767-775) with the GLOBAL frame count, which
reproduces the single-GPU math at the same global batch (the reference
itself divides by its local row count, :767).

`net` is duck-typed: anything with NumComponents(), components[i]
(NumGradientParams, ApplyGradient), Propagate(x),
BackpropComponent(i, out_deriv, mode, grad) and BackpropSplit(i, out_deriv,
grad, skip_first_dx, between) -- kcnn.Nnet on the GPU; the tests drive the
same function with a CPU stand-in over gloo.
"""
from __future__ import annotations

import os

# gradients at least this long get their own all-reduce, started before the
# layer's data gradient; shorter ones share the flat bucket
SPLIT_GRADIENT_PARAMS = int(os.environ.get("KCNN_DP_SPLIT_PARAMS", 1 << 20))


class GradientBuffers:
    """A replica's gradient storage: {component index: flat [linear | bias]
    buffer}.  Components with fewer than `own` gradient values get views into
    one contiguous bucket (in component order); the others own a buffer."""

    def __init__(self, net, alloc, own=None):
        own = SPLIT_GRADIENT_PARAMS if own is None else own
        sizes = {i: c.NumGradientParams() for i, c in enumerate(net.components)
                 if c.NumGradientParams() > 0}
        self.large = sorted(i for i, n in sizes.items() if n >= own)
        self.small = sorted(i for i in sizes if i not in self.large)
        total = sum(sizes[i] for i in self.small)
        self.bucket = alloc(total) if total else None
        self.bufs = {}
        off = 0
        for i in self.small:
            self.bufs[i] = self.bucket[off:off + sizes[i]]
            off += sizes[i]
        for i in self.large:
            self.bufs[i] = alloc(sizes[i])

    def __contains__(self, i):
        return i in self.bufs

    def __getitem__(self, i):
        return self.bufs[i]

    def num_collectives(self):
        return len(self.large) + (1 if self.bucket is not None else 0)

    def bytes_per_step(self):
        return sum(b.numel() for b in self.bufs.values()) * 4


def gradient_buffers(net, alloc, own=None):
    return GradientBuffers(net, alloc, own)


def dp_train_step(net, x, out_deriv, grads, dist, frames_global, mark=None):
    """Propagate + backprop + all-reduced update of one row shard.

    mode 1 = data gradient and parameter gradient (no update), mode 2 = data
    gradient only, mode 3 = parameter gradient only
    (kcnn_nnet_backprop_component).  The first layer's input derivative is
    computed too, as upstream NnetUpdater does and as the 1-GPU step
    (Nnet.Backprop) does, so N=1 and N>1 do the same work.

    mark(name), when given, is called on the host at "wait_begin" (all
    collectives issued, the backward queued) and "wait_end" (the compute
    stream now waits for every collective): bench.py records stream events
    there to measure the all-reduce time the step did not hide."""
    net.Propagate(x)
    pending = []
    for i in reversed(range(net.NumComponents())):
        if i in grads.large and getattr(net.components[i], "SplitGradient", lambda: True)():
            # the gradient, its all-reduce started, then the data gradient
            # (one library call: both GEMMs' statistics from one pass)
            def start(i=i):
                pending.append(([i], dist.all_reduce(grads[i], async_op=True)))
            net.BackpropSplit(i, out_deriv, grads[i], False, start)
        elif i in grads.large:
            net.BackpropComponent(i, out_deriv, mode=1, grad=grads[i], skip_first_dx=False)
            pending.append(([i], dist.all_reduce(grads[i], async_op=True)))
        elif i in grads:
            net.BackpropComponent(i, out_deriv, mode=1, grad=grads[i], skip_first_dx=False)
        else:
            net.BackpropComponent(i, out_deriv, mode=2, skip_first_dx=False)
    if grads.bucket is not None:
        pending.append((grads.small, dist.all_reduce(grads.bucket, async_op=True)))
    if mark:
        mark("wait_begin")
    # NCCL (RCCL) runs a process group's collectives in order on one stream,
    # so the compute stream waits for the last one alone: each stream wait
    # (and the event behind it) cost the c2 step 20-50 us of GPU idle at
    # world size 1 (rocprofv3 trace); other backends wait for each
    backend = getattr(dist, "get_backend", lambda: None)()
    waits = pending[-1:] if backend == "nccl" else pending
    for _, work in waits:
        work.wait()
    if mark:
        mark("wait_end")
    for ids, _ in pending:
        for i in ids:
            net.components[i].ApplyGradient(grads[i], frames_global)
