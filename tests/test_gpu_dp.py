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
