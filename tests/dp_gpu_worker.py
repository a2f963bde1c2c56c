"""Worker of tests/test_gpu_dp.py, run under torch.distributed.run: the
bench's data-parallel step (kcnn_dp.dp_train_step) through libkcnn.so on the
GPU, with gloo ranks sharing the device.  Every rank trains on its own row
shard of one global batch; rank 0 then also trains a fresh replica on the
whole batch in one process.  Parameters go to <out>/rank<r>.npz and
<out>/single.npz for the test to compare."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import kcnn      # noqa: E402
import kcnn_dp   # noqa: E402

H, W, C, KH, KW, G, PC, F = 40, 11, 3, 8, 1, 32, 4, 64
OH, OW = H - KH + 1, W - KW + 1
CFG = "\n".join([
    f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} kernel-height={KH} "
    f"kernel-width={KW} stride=1 group={G} out-height={OH} out-width={OW} "
    f"learning-rate=0.02 param-stddev=0.05 bias-stddev=0.5",
    f"MaxpoolComponent in-height={OH} in-width={OW} in-channel={G} pool-height-dim=1 "
    f"pool-width-dim=1 pool-channel-dim={PC}",
    f"FullyConnectedComponent input-dim={OH * OW * G // PC} output-dim={F} learning-rate=0.02 "
    f"param-stddev=0.05 bias-stddev=1 weight-decay=0.0002 momentum=0.9",
])


# a long-kernel stack (implicit-GEMM v2 forward, wgrad v2, scatter dgrad,
# 3-D pool) -- the c5 code paths through the same DP step
CFG_LONG = "\n".join([
    "ConvolutionComponent in-height=8 in-width=9 in-channel=16 in-pad-height=1 in-pad-width=1 "
    "kernel-height=3 kernel-width=3 stride=1 group=128 out-height=8 out-width=9 "
    "learning-rate=0.02 param-stddev=0.05 bias-stddev=0.5",
    "MaxpoolComponent in-height=8 in-width=9 in-channel=128 pool-height-dim=2 "
    "pool-width-dim=1 pool-channel-dim=4",
    "ConvolutionComponent in-height=4 in-width=9 in-channel=32 kernel-height=3 kernel-width=3 "
    "stride=1 group=128 out-height=2 out-width=7 learning-rate=0.02 param-stddev=0.05 "
    "bias-stddev=0.5",
    f"FullyConnectedComponent input-dim={2 * 7 * 128} output-dim={F} learning-rate=0.02 "
    f"param-stddev=0.05 bias-stddev=1 weight-decay=0.0002 momentum=0.9",
])
CONFIGS = {"c2": (CFG, H * W * C), "long": (CFG_LONG, 8 * 9 * 16)}


def params(net):
    out = {}
    for i, c in enumerate(net.components):
        if c.NumGradientParams() > 0:
            out[f"W{i}"] = c.LinearParams().cpu().numpy()
            out[f"b{i}"] = c.BiasParams().cpu().numpy()
            out[f"p{i}"] = c.PrevGrad().cpu().numpy()
    return out


def main():
    out_dir, steps, n_global = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    cfg, in_dim = CONFIGS[sys.argv[4] if len(sys.argv) > 4 else "c2"]
    backend = sys.argv[5] if len(sys.argv) > 5 else "gloo"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if backend == "nccl":
        # RCCL: one GPU per rank (the one-GPU test box runs world size 1)
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{rank}"))
        kcnn.init(rank)
    else:
        dist.init_process_group("gloo")
        kcnn.init(0)
    kcnn.set_randn_seed(7)
    net = kcnn.Nnet(cfg)
    r = np.random.default_rng(11)
    xs = [r.standard_normal((n_global, in_dim)).astype(np.float32) for _ in range(steps)]
    dys = [(r.standard_normal((n_global, F)) * 0.05).astype(np.float32) for _ in range(steps)]
    per = n_global // world
    grads = kcnn_dp.gradient_buffers(net, lambda n: torch.empty(n, device="cuda"))
    for s in range(steps):
        x = torch.from_numpy(xs[s][rank * per:(rank + 1) * per]).cuda()
        dy = torch.from_numpy(dys[s][rank * per:(rank + 1) * per]).cuda()
        kcnn_dp.dp_train_step(net, x, dy, grads, dist, n_global)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **params(net))
    if rank == 0:
        kcnn.set_randn_seed(7)
        ref = kcnn.Nnet(cfg)
        for s in range(steps):
            ref.Propagate(torch.from_numpy(xs[s]).cuda())
            ref.Backprop(torch.from_numpy(dys[s]).cuda())  # update with N = n_global
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, "single.npz"), **params(ref))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
