"""The nnet.config bench model's FC GEMM operands over training steps: per
GEMM (forward, data gradient, weight gradient of each FullyConnectedComponent)
the spread groups of op(A) / op(B) (f16-split.h), their small-element counts
and how many C elements the store's check rejects (|C| under 2^9 (cnt_r +
cnt_c) 2^-(s_r + s_c), C in float64 on the GPU).  Same model, data and
seeds as `bench.py --config nnet`."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd")); sys.path.insert(0, ROOT)
import torch, kcnn, bench

kcnn.init(0)
kcnn.set_fusion(1)
kcnn.set_randn_seed(20261015)
net = kcnn.Nnet(bench.NNET_CONFIG)
B = 4096
gen = torch.Generator(device="cuda"); gen.manual_seed(20261015)
x = torch.randn((21 * B, 40), generator=gen, device="cuda")
dy = torch.randn((B, 3456), generator=gen, device="cuda").mul_(1e-2)[:, :3454]
FC = [(14, 13, 15), (16, 15, 17), (18, 17, None)]  # (fc index, input comp, next comp)


def group_stats(X, per_row):
    """(spread mask, count, scale exponent) per row (per_row) or column."""
    ax = 1 if per_row else 0
    a = X.abs().double()
    mx = a.amax(dim=ax)
    nz = torch.where(a > 0, a, torch.full_like(a, float("inf")))
    mn = nz.amin(dim=ax)
    e = torch.floor(torch.log2(mx.clamp_min(1e-300)))
    emn = torch.floor(torch.log2(mn.clamp_min(1e-300)))
    spread = torch.isfinite(mn) & (emn < e - 20) & (mx > 0)
    bound = torch.pow(2.0, e - 17)
    small = (a > 0) & (a < bound.unsqueeze(ax))
    cnt = torch.where(spread, small.sum(dim=ax).double(), torch.zeros_like(e))
    s = 14 - e
    return spread, cnt, s


def census(name, A, Bm):
    """C = A @ Bm (A: M x K rows, Bm: K x N columns), torch fp32 inputs."""
    sa, ca, ea = group_stats(A, True)
    sb, cb, eb = group_stats(Bm, False)
    C = A.double() @ Bm.double()
    thr = 512.0 * (1 + 1 / 1024) * (ca.unsqueeze(1) + cb.unsqueeze(0)) * torch.pow(
        2.0, -(ea.unsqueeze(1) + eb.unsqueeze(0)))
    rej = ((ca.unsqueeze(1) + cb.unsqueeze(0)) > 0) & ~(C.abs() >= thr)
    print(f"  {name}: A rows spread {int(sa.sum())}/{A.shape[0]} (cnt max {int(ca.max())}, "
          f"sum {int(ca.sum())}); B cols spread {int(sb.sum())}/{Bm.shape[1]} (cnt max "
          f"{int(cb.max())}, sum {int(cb.sum())}); rejected {int(rej.sum())} of {C.numel()}",
          flush=True)


for step in range(41):
    net.Propagate(x)
    if step in (0, 5, 20, 40):
        print(f"step {step}", flush=True)
        for fi, ii, ni in FC:
            X = net.Output(ii).float()
            W = net.components[fi].LinearParams().float()
            census(f"FC{fi} fwd", X, W.t())
    net.Backprop(dy)
    if step in (0, 5, 20, 40):
        for fi, ii, ni in FC:
            X = net.Output(ii).float()
            W = net.components[fi].LinearParams().float()
            dZ = dy.float() if ni is None else net.InputDeriv(ni).float()
            census(f"FC{fi} dgrad", dZ, W)
            census(f"FC{fi} wgrad", dZ.t().contiguous(), X)
