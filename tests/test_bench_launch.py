"""bench.py's self-launch (no GPU): `python bench.py --gpus N` without a
launcher in the environment runs itself under torch.distributed.run with N
ranks on 127.0.0.1 and passes the child's exit status on (VERDICT r04 item 2;
the GPU run of the same path is tests/test_gpu_dp.py)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launch_ranks_command(monkeypatch):
    import bench
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    assert bench.launch_ranks(8) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3"][-4:]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launch_ranks_failure_is_nonzero(monkeypatch):
    import bench

    class R:
        returncode = -9   # a rank killed by a signal

    monkeypatch.setattr(subprocess, "run", lambda cmd, env=None: R())
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.launch_ranks(2) != 0


def test_main_relaunches_without_world_size(monkeypatch):
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    calls = []
    monkeypatch.setattr(bench, "launch_ranks", lambda n: calls.append(n) or 3)
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 3
    assert calls == [4]
