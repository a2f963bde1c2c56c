"""Host time to issue one c2 step (no synchronisation inside) against the
GPU's time per step: if issuing takes as long as executing, the host (not the
GPU) sets the step time and the trace's gaps are the host catching up."""
import sys
import time

import torch

sys.path.insert(0, "kaldi-cnn_amd")
sys.path.insert(0, ".")
import kcnn  # noqa: E402
import bench  # noqa: E402

kcnn.init(0)
kcnn.set_fusion(1)
net = kcnn.Nnet(bench.stack_config())
B = 4096
x = torch.randn((B, bench.H * bench.W * bench.C), device="cuda")
dy = torch.randn((B, bench.FC_OUT), device="cuda") * 1e-2
for _ in range(5):
    net.Propagate(x)
    net.Backprop(dy)
torch.cuda.synchronize()
for trial in range(3):
    t0 = time.perf_counter()
    marks = []
    for _ in range(20):
        a = time.perf_counter()
        net.Propagate(x)
        b = time.perf_counter()
        net.Backprop(dy)
        c = time.perf_counter()
        marks.append((b - a, c - b))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    prop = sum(m[0] for m in marks) / 20 * 1e6
    back = sum(m[1] for m in marks) / 20 * 1e6
    print(f"trial {trial}: issue {1e3 * (t1 - t0) / 20:.3f} ms/step (Propagate {prop:.0f} us, "
          f"Backprop {back:.0f} us), issue + drain {1e3 * (t2 - t0) / 20:.3f} ms/step",
          flush=True)
