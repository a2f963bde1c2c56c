"""Data-parallel training step on the GPU (bench.py --gpus N):
two ranks (gloo, sharing the one GPU of the test box -- RCCL needs a GPU
per rank) run kcnn_dp.dp_train_step through libkcnn.so on their shards of a
global batch.  The replicas must stay bitwise identical, and must match one
process that trained on the whole batch (the reference's update with the
global frame count, nnet-component-nnet0.cc:767) to the fp32 reduction-order
tolerance."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("stack,n_params,split,backend,nproc", [
    ("c2", 6, None, "gloo", 2), ("long", 9, None, "gloo", 2), ("c2", 6, "1", "gloo", 2),
    ("long", 9, None, "nccl", 1)])
def test_dp_two_ranks_match_single_process(tmp_path, stack, n_params, split, backend, nproc):
    """split "1": every non-conv gradient computed on its own (mode 3) and
    all-reduced while the layer's data gradient (mode 2) runs.  backend
    "nccl": the RCCL communicator and its async all-reduces (world size 1 on
    the one-GPU test box; RCCL takes one GPU per rank)."""
    steps, n_global = 2, 48
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "dp_gpu_worker.py"), str(tmp_path), str(steps), str(n_global),
           stack, backend]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    if split:
        env["KCNN_DP_SPLIT_PARAMS"] = split
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    a = np.load(tmp_path / "rank0.npz")
    b = np.load(tmp_path / f"rank{nproc - 1}.npz")
    single = np.load(tmp_path / "single.npz")
    assert sorted(a.files) == sorted(single.files) and len(a.files) == n_params
    for k in a.files:
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"replicas differ: {k}")
        ref = single[k]
        err = np.abs(a[k] - ref).max() / max(np.abs(ref).max(), 1e-30)
        assert err < 1e-5, f"{k}: DP vs single-process relative error {err:.2e}"


def test_bench_gpus_n_launches_n_ranks():
    """`python bench.py --gpus 2` (no launcher in the environment) starts the
    two ranks itself and reports a two-GPU line (gloo: both ranks share the
    test box's one GPU)."""
    import json
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--steps", "2", "--warmup", "1",
                        "--frames-per-gpu", "256", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["dp"]["ranks_seen"] == 2
    assert res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 512


@pytest.mark.parametrize("name,N", [("c2", 4096), ("c2", 37), ("long_2x1x4_pad", 64)])
def test_backprop_split_equals_mode3_then_mode2(kc, name, N):
    """kcnn_nnet_backprop_split (the FC layer's gradient, the caller's
    callback, its data gradient; one statistics pass) gives the bits of the
    mode-3 and mode-2 calls, and calls back once, between the two."""
    import torch
    from _util import dev, host, randn, rng
    from test_gpu_nnet import STACKS, build

    def run(split):
        net = build(kc, STACKS[name], seed=11)
        r = rng(3)
        x = dev(randn(r, (N, net.components[0].InputDim())))
        dy = dev(randn(r, (N, net.components[2].OutputDim()), 0.1))
        fc = net.components[2]
        grad = torch.zeros(fc.NumGradientParams(), device="cuda")
        net.Propagate(x)
        calls = []
        if split:
            net.BackpropSplit(2, dy, grad, False,
                              lambda: calls.append(host(grad[None, :]).copy()))
        else:
            net.BackpropComponent(2, dy, mode=3, grad=grad, skip_first_dx=False)
            calls.append(host(grad[None, :]).copy())
            net.BackpropComponent(2, dy, mode=2, skip_first_dx=False)
        return calls, host(grad[None, :]), host(net.InputDeriv(2))

    a, b = run(True), run(False)
    assert len(a[0]) == 1
    for u, v, what in ((a[0][0], b[0][0], "grad at the callback"), (a[1], b[1], "grad"),
                       (a[2], b[2], "input derivative")):
        np.testing.assert_array_equal(u, v, err_msg=f"{name} N={N}: {what}")


def test_backprop_split_callback_error(kc):
    """An exception in the callback reaches the caller."""
    import torch
    from _util import dev, randn, rng
    from test_gpu_nnet import STACKS, build
    net = build(kc, STACKS["c2"], seed=11)
    r = rng(3)
    x = dev(randn(r, (8, net.components[0].InputDim())))
    dy = dev(randn(r, (8, net.components[2].OutputDim()), 0.1))
    grad = torch.zeros(net.components[2].NumGradientParams(), device="cuda")
    net.Propagate(x)

    def boom():
        raise RuntimeError("callback failed")
    with pytest.raises(RuntimeError, match="callback failed"):
        net.BackpropSplit(2, dy, grad, False, boom)
