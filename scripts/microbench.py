"""Per-kernel timing of the c2 hot path (HIP events on the launch stream).

  python scripts/microbench.py [--frames 4096] [--reps 20] [--only fwd,dgrad,...]

Times ConvolutionComponent Propagate / data gradient / weight gradient and
MaxpoolComponent Propagate / Backprop in isolation, and reports GB/s against
the algorithmic bytes.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import kcnn  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    kcnn.init(0)
    B = a.frames
    cfg = bench.stack_config().split("\n")
    conv = kcnn.Component.NewFromString(cfg[0])
    pool = kcnn.Component.NewFromString(cfg[1])
    x = torch.randn(B, conv.InputDim(), device="cuda")
    y = conv.Propagate(x)
    p = pool.Propagate(y)
    dp = torch.randn_like(p)
    dy = torch.randn_like(y)
    dx = torch.empty_like(x)
    dyp = torch.empty_like(y)
    grad = torch.empty(conv.NumGradientParams(), device="cuda")
    pool_ov = kcnn.Component.NewFromString(
        f"MaxpoolComponent in-height={bench.OH} in-width={bench.OW} in-channel={bench.G} "
        f"pool-height-dim=1 pool-width-dim=1 pool-channel-dim={bench.PC} overlap=true")
    p_ov = pool_ov.Propagate(y)
    dp_ov = torch.randn_like(p_ov)
    pool_2d = kcnn.Component.NewFromString(
        f"MaxpoolComponent in-height={bench.OH} in-width={bench.OW} in-channel=256 "
        f"pool-height-dim=1 pool-width-dim=1 pool-channel-dim=2 overlap2D=true")
    y2 = torch.randn(B, bench.OH * bench.OW * 256, device="cuda")
    p_2d = pool_2d.Propagate(y2)
    dp_2d = torch.randn_like(p_2d)
    dy2 = torch.empty_like(y2)
    conv_b = bench.CONV_BYTES_PER_PASS * B
    tests = {
        "fwd": (lambda: conv.Propagate(x, y), conv_b),
        "dgrad": (lambda: conv.Backprop(x, None, dy, dx, update=False), conv_b),
        "wgrad": (lambda: conv.ComputeGradient(x, dy, grad), conv_b),
        "bwd_fused": (lambda: conv.BackpropGradient(x, dy, dx, grad), conv_b + x.numel() * 4),
        "bwd_fused_nodx": (lambda: conv.BackpropGradient(x, dy, None, grad, want_in_deriv=False),
                           conv_b),
        "pool_fwd": (lambda: pool.Propagate(y, p), bench.POOL_FWD_BYTES * B),
        "pool_bwd": (lambda: pool.Backprop(y, p, dp, dyp), bench.POOL_BWD_BYTES * B),
        # intermap pooling variants: overlapping channel
        # windows on Y, and overlap2D on a 16 x 16 map grid (256 channels)
        "pool_ov_fwd": (lambda: pool_ov.Propagate(y, p_ov), (y.numel() + p_ov.numel()) * 4),
        "pool_ov_bwd": (lambda: pool_ov.Backprop(y, p_ov, dp_ov, dyp),
                        (2 * y.numel() + 2 * p_ov.numel()) * 4),
        "pool_ov2d_fwd": (lambda: pool_2d.Propagate(y2, p_2d), (y2.numel() + p_2d.numel()) * 4),
        "pool_ov2d_bwd": (lambda: pool_2d.Backprop(y2, p_2d, dp_2d, dy2),
                          (2 * y2.numel() + 2 * p_2d.numel()) * 4),
        # HBM reference points of the same size (torch kernels)
        "fill_y": (lambda: dyp.fill_(1.0), dyp.numel() * 4),
        "copy_y": (lambda: dyp.copy_(y), 2 * dyp.numel() * 4),
        "sum_y": (lambda: y.sum(), y.numel() * 4),
    }
    only = [t for t in a.only.split(",") if t]
    for name, (fn, byts) in tests.items():
        if only and name not in only:
            continue
        ms = timeit(fn, a.reps)
        print(f"{name:10s} {ms * 1e3:9.1f} us  {byts / ms / 1e6:8.1f} GB/s "
              f"({byts / ms / 1e6 / bench.PEAK_HBM_GBS * 100:5.1f}% of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
