"""Data-parallel training step for a kcnn component stack.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm): the
minibatch is row-sharded -- frames are independent through Conv, Maxpool and
FC -- and every rank holds a full replica of the parameters.  The only
exchange is the parameter gradient: each updatable component's flat gradient
[linear | bias] is all-reduced (sum, fp32) as soon as that component's
backward is done, so the reduction of the 47.6 MB FC gradient overlaps the
conv/maxpool backward below it.  Every replica then applies the reference's
update step (nnet-component-nnet0.cc:767-775) with the GLOBAL frame count,
which reproduces the single-GPU math at the same global batch (the reference
itself divides by its local row count, :767).

`net` is duck-typed: anything with NumComponents(), components[i]
(NumGradientParams, ApplyGradient), Propagate(x) and
BackpropComponent(i, out_deriv, mode, grad) -- kcnn.Nnet on the GPU; the
tests drive the same function with a CPU stand-in over gloo.
"""
from __future__ import annotations

import os


def gradient_buffers(net, alloc):
    """{component index: flat gradient buffer} for the updatable components."""
    return {i: alloc(c.NumGradientParams()) for i, c in enumerate(net.components)
            if c.NumGradientParams() > 0}


# gradients at least this long are computed on their own (mode 3) and their
# all-reduce starts before the layer's data gradient: the FC layer's 47.6 MB
# then reduces beside its dX GEMM as well as the conv backward
SPLIT_GRADIENT_PARAMS = int(os.environ.get("KCNN_DP_SPLIT_PARAMS", 1 << 20))


def dp_train_step(net, x, out_deriv, grads, dist, frames_global):
    """Propagate + backprop + all-reduced update of one row shard.

    mode 1 = data gradient and parameter gradient (no update), mode 2 = data
    gradient only, mode 3 = parameter gradient only
    (kcnn_nnet_backprop_component).  The first layer's input derivative is
    computed too, as upstream NnetUpdater does and as the 1-GPU step
    (Nnet.Backprop) does, so N=1 and N>1 do the same work."""
    net.Propagate(x)
    pending = []
    for i in reversed(range(net.NumComponents())):
        if i in grads and grads[i].numel() >= SPLIT_GRADIENT_PARAMS and \
                getattr(net.components[i], "SplitGradient", lambda: True)():
            net.BackpropComponent(i, out_deriv, mode=3, grad=grads[i], skip_first_dx=False)
            pending.append((i, dist.all_reduce(grads[i], async_op=True)))
            net.BackpropComponent(i, out_deriv, mode=2, skip_first_dx=False)
        elif i in grads:
            net.BackpropComponent(i, out_deriv, mode=1, grad=grads[i], skip_first_dx=False)
            pending.append((i, dist.all_reduce(grads[i], async_op=True)))
        else:
            net.BackpropComponent(i, out_deriv, mode=2, skip_first_dx=False)
    for i, work in pending:
        work.wait()
        net.components[i].ApplyGradient(grads[i], frames_global)
