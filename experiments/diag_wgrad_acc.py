"""r06 diagnostic: normwise error of the conv weight gradient (through the
update's prev') against float64, by batch size, backward family and fusion
mode, beside an fp32 contraction's error (tests/_stack.device_gradient)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "kaldi-cnn_amd", "tests", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch
import bench
import kcnn as kc
from _stack import oracle_layers, device_gradient, fp32_gradient_error
from _util import host

kc.init(0)
for B in [int(b) for b in sys.argv[1].split(",")]:
    for fam in (1, 0):
        for fusion in (0, 1):
            kc.set_kernel_family("bwd_x6", fam)
            kc.set_fusion(fusion)
            kc.set_randn_seed(20261015)
            cfg = bench.stack_config()
            net = kc.Nnet(cfg)
            gen = torch.Generator(device="cuda"); gen.manual_seed(3)
            x = torch.randn((B, bench.H * bench.W * bench.C), generator=gen, device="cuda")
            dy = torch.randn((B, bench.FC_OUT), generator=gen, device="cuda") * 1e-2
            oc = oracle_layers(cfg, net, kc)[0]
            net.Propagate(x)
            net.Backprop(dy)
            d = net.InputDeriv(1).clone()
            p1 = host(net.components[0].GetParam(kc.PARAM_PREV_GRAD))
            (gW, gb), (gS, bS) = device_gradient(oc, x, d)
            lr = oc.learning_rate / B
            t = lr * gW.astype(np.float64)
            e = np.linalg.norm(p1 - t) / np.linalg.norm(t)
            e32 = fp32_gradient_error(oc, x, d, gW)
            worst = float((np.abs(p1 - t) / (lr * gS + 1e-30)).max())
            print(f"B {B:6d} bwd_x6 {fam} fusion {fusion}: prev' normwise {e:.2e}  "
                  f"elementwise err/S {worst:.2e}  fp32 contraction {e32:.2e}  "
                  f"S/|t| median {np.median(gS / np.maximum(np.abs(gW), 1e-30)):.1f}", flush=True)
            del net, d
            torch.cuda.empty_cache()
kc.set_kernel_family("bwd_x6", 1)
