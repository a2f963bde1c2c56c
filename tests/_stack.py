"""Layer-by-layer parity of a whole kcnn_nnet training step against the oracle.

One Propagate + Backprop (update in Backprop, the bench's step) of a
Conv / Maxpool / FC stack runs on the GPU through libkcnn.so.  Every layer is
then checked against the oracle applied to the GPU's own inputs of that
layer -- the previous layer's GPU output going forward, the next layer's GPU
input derivative going back -- so a check sees exactly one component's
arithmetic (no rounding carried in from other layers, and max-pool routing
decided by the same values on both sides):

  Conv / FC Propagate        1e-5 * S bound       (nnet-component-nnet0.cc:423-446, 1133)
  Maxpool Propagate/Backprop bit-exact            (A.8 / A.9)
  Conv / FC Backprop (dX)    1e-5 * S bound       (:461-544)
  Conv / FC update           bound on W', b', prev' (:738-777, :1133-1150)

`rows` restricts the row-local checks (outputs and input derivatives) to a
sample of rows; the parameter update, a sum over all rows, is then checked
against a float64 gradient of the whole batch computed with torch on the
same device (`device_gradient`: im2col by F.unfold and fp64 contractions,
written from the layout spec) unless `update=False`.
"""
import numpy as np

import oracle as O
from _util import assert_bound, assert_same, host


def truth(fn):
    """fn in the oracle's fp64-accumulated mode (truth) and |.|-accumulated
    mode (the error scale S)."""
    out = []
    for mode in (1, 2):
        with O.accum(mode):
            out.append(fn())
    return out


def oracle_layers(config, net, kc):
    """Oracle objects for the stack's config lines, with the GPU stack's
    current parameters."""
    layers = []
    for line, c in zip(config.strip().splitlines(), net.components):
        t, *kvs = line.split()
        info = dict(kv.split("=", 1) for kv in kvs)
        g = lambda k, d=None: int(info.get(k, d))
        assert t == c.Type(), (t, c.Type())
        if t == "ConvolutionComponent":
            # B4: weight-decay / momentum from the config line are ignored
            oc = O.Conv(g("in-height"), g("in-width"), g("in-channel"), g("kernel-height"),
                        g("kernel-width"), g("group"), in_pad_height=g("in-pad-height", 0),
                        in_pad_width=g("in-pad-width", 0),
                        learning_rate=float(info["learning-rate"]))
        elif t == "MaxpoolComponent":
            oc = O.Pool(g("in-height"), g("in-width"), g("in-channel"), g("pool-height-dim"),
                        g("pool-width-dim"), g("pool-channel-dim"),
                        info.get("overlap", "false") == "true",
                        info.get("overlap2D", "false") == "true")
        elif t == "FullyConnectedComponent":
            oc = O.FC(c.InputDim(), c.OutputDim(),
                      learning_rate=float(info["learning-rate"]),
                      weight_decay=float(info.get("weight-decay", 0.0002)),
                      momentum=float(info.get("momentum", 0.9)))
        else:
            raise ValueError(t)
        if t != "MaxpoolComponent":
            oc.W = host(c.GetParam(kc.PARAM_LINEAR))
            oc.b = host(c.GetParam(kc.PARAM_BIAS)).ravel().copy()
            oc.prev = host(c.GetParam(kc.PARAM_PREV_GRAD))
        layers.append(oc)
    return layers


def device_gradient(oc, a, d, chunk=256, dtype=None):
    """The float64 gradient of a Conv / FC layer over every row of its input
    `a` and output derivative `d` (torch tensors, any device, row-strided
    views allowed): ((gW, gb) rounded to fp32, (S_W, S_b) the sums of
    |terms|), in the oracle's layouts -- conv gW[c*kh*kw + kx*kh + ky][g]
    (cnsl-cu-kernels.cu:26-30), FC gW[out][in] (nnet-component-nnet0.cc:1141).
    Chunked over rows so the fp64 im2col stays a few hundred MB.  With
    dtype=torch.float32 the same contraction in fp32 (an sgemm's accumulation:
    the error an fp32 reference itself carries over a long reduction)."""
    import torch
    import torch.nn.functional as F
    N = a.shape[0]
    dt = torch.float64 if dtype is None else dtype
    if isinstance(oc, O.FC):
        gW = gS = gb = bS = 0
        for n0 in range(0, N, 4 * chunk):
            x = a[n0:n0 + 4 * chunk].to(dt)
            y = d[n0:n0 + 4 * chunk].to(dt)
            gW = gW + y.t() @ x
            gS = gS + y.abs().t() @ x.abs()
            gb = gb + y.sum(0)
            bS = bS + y.abs().sum(0)
    else:
        H, W, C = oc.in_height, oc.in_width, oc.in_channel
        kh, kw, G = oc.kernel_height, oc.kernel_width, oc.group
        oh, ow = oc.out_height, oc.out_width
        gW = gS = gb = bS = 0
        for n0 in range(0, N, chunk):
            xs = a[n0:n0 + chunk].to(dt)
            n = xs.shape[0]
            # row col = h + w*H + c*H*W  ->  [n, C, H, W]
            xt = xs.reshape(n, C, W, H).transpose(2, 3)
            u = F.unfold(xt, (kh, kw), padding=(oc.in_pad_height, oc.in_pad_width))
            # output col = g*P + px*oh + py  ->  [n, G, oh*ow] in unfold's order
            y = d[n0:n0 + chunk].to(dt).reshape(n, G, ow, oh).transpose(2, 3).reshape(
                n, G, oh * ow)
            gW = gW + torch.einsum("nkl,ngl->kg", u, y)
            gS = gS + torch.einsum("nkl,ngl->kg", u.abs(), y.abs())
            gb = gb + y.sum((0, 2))
            bS = bS + y.abs().sum((0, 2))
        # unfold's k = c*kh*kw + ky*kw + kx  ->  the kernel matrix's c*kh*kw + kx*kh + ky
        def kmat(t):
            return t.reshape(C, kh, kw, G).permute(0, 2, 1, 3).reshape(C * kw * kh, G)
        gW, gS = kmat(gW), kmat(gS)
    out = [t.double().cpu().numpy() for t in (gW, gb, gS, bS)]
    return (out[0].astype(np.float32), out[1].astype(np.float32)), (out[2], out[3])


def fp32_gradient_error(oc, a, d, gW_t):
    """Normwise relative error of the same gradient accumulated in fp32 on
    the device (device_gradient with float32; no reduced-precision matmul)
    against the float64 one: what an fp32 sgemm reaches on this reduction."""
    import torch
    torch.backends.cuda.matmul.allow_tf32 = False
    (g32, _), _ = device_gradient(oc, a, d, dtype=torch.float32)
    t = np.asarray(gW_t, np.float64)
    return float(np.linalg.norm(g32.astype(np.float64) - t) / max(np.linalg.norm(t), 1e-300))


def _rows(t, rows):
    if rows is None:
        return host(t)
    import torch
    idx = torch.as_tensor(rows, device=t.device)
    return host(t.index_select(0, idx))


def run_step(kc, config, net, x, dy, rows=None, keep=False):
    """The training step on the GPU; returns the oracle layers (parameters
    before the step), the layers' outputs and input derivatives (sampled
    rows), the parameters after and, with `keep`, device copies of every
    layer's whole output and input derivative."""
    n = net.NumComponents()
    before = oracle_layers(config, net, kc)
    net.Propagate(x)
    # outputs first: a fused conv's output is recomputed on request, which is
    # possible until its backprop runs
    full_o = [net.Output(i).clone() for i in range(n)] if keep else None
    outs = [_rows(net.Output(i), rows) for i in range(n)]
    net.Backprop(dy)
    full_d = [net.InputDeriv(i).clone() for i in range(n)] if keep else None
    derivs = [_rows(net.InputDeriv(i), rows) for i in range(n)]
    after = [[host(c.GetParam(w)) for w in (kc.PARAM_LINEAR, kc.PARAM_BIAS, kc.PARAM_PREV_GRAD)]
             if c.NumGradientParams() > 0 else None for c in net.components]
    return before, outs, derivs, after, (full_o, full_d)


def check_step(kc, config, net, x, dy, rows=None, what="", update=True):
    """One step checked layer by layer; with `rows`, the row-local checks on
    those rows and (update=True) the updates against device_gradient."""
    keep = rows is not None and update
    layers, outs, derivs, after, (full_o, full_d) = run_step(kc, config, net, x, dy, rows,
                                                            keep=keep)
    xin = _rows(x, rows)
    dout = _rows(dy, rows)
    ins = [xin] + outs[:-1]
    d_next = derivs[1:] + [dout]
    N = x.shape[0]
    for i, oc in enumerate(layers):
        tag = f"{what} layer {i} {type(oc).__name__}"
        a, y = ins[i], outs[i]
        if isinstance(oc, O.Pool):
            assert_same(y, oc.propagate(a), f"{tag} Propagate")
            assert_same(derivs[i], oc.backprop(a, y, d_next[i]), f"{tag} Backprop")
            continue
        y_t, y_s = truth(lambda: oc.propagate(a))
        assert_bound(y, y_t, y_s, what=f"{tag} Propagate")
        dx_t, dx_s = truth(lambda: oc.backprop(a, d_next[i], update=False))
        assert_bound(derivs[i], dx_t, dx_s, what=f"{tag} dX")
        if rows is not None and not update:
            continue
        # the update: W' = W + m*prev - lr*wd*W + lr*gW (bias: b + lr*gb), lr
        # divided by the rows of the step (B10)
        if rows is None:
            (gW_t, gb_t), (gW_s, gb_s) = truth(lambda: oc.gradient(a, d_next[i]))
        else:
            a_full = x if i == 0 else full_o[i - 1]
            d_full = dy if i == len(layers) - 1 else full_d[i + 1]
            (gW_t, gb_t), (gW_s, gb_s) = device_gradient(oc, a_full, d_full)
            # over a whole large batch (c3: 23.8 M terms per conv gradient
            # element) fp32 accumulation alone can pass 1e-5 normwise on a
            # gradient with cancellation; the normwise bar of prev' (the
            # gradient's image) is then 2x what the fp32 contraction reaches
            # (as the FC GEMM test's 2x sgemm), the elementwise 1e-5 * S bar
            # unchanged
            e32 = fp32_gradient_error(oc, a_full, d_full, gW_t)
            norm_prev = max(1e-5, 2 * e32)
        W0, b0, p0 = oc.W.copy(), oc.b.copy(), oc.prev.copy()
        with O.accum(1):
            oc.apply(gW_t, gb_t, N)
        lr = oc.learning_rate / N
        W1, b1, p1 = after[i]
        assert_bound(W1, oc.W, np.abs(W0) + np.abs(p0) + lr * gW_s + 1e-30, what=f"{tag} W'")
        assert_bound(b1.ravel(), oc.b, np.abs(b0) + lr * gb_s, what=f"{tag} b'")
        assert_bound(p1, oc.prev, np.abs(p0) + lr * gW_s + 1e-6 * np.abs(W0),
                     what=f"{tag} prev' (fp32 contraction's normwise error "
                          f"{e32 if rows is not None else 0:.2e})",
                     norm_rtol=norm_prev if rows is not None else None)
