"""Repeat one GEMM shape and report the worst error per run and where the
bad elements are (tile rows / columns), to locate a nondeterministic fault."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))
import torch
import kcnn

kcnn.init(0)
m, n, k, ta, tb = [int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (4096, 11616, 1024, 0, 0))]
g = torch.Generator(device="cuda"); g.manual_seed(1)
a = torch.randn((k, m) if ta else (m, k), generator=g, device="cuda")
b = torch.randn((n, k) if tb else (k, n), generator=g, device="cuda") * 0.01
A = (a.t() if ta else a).double(); B = (b.t() if tb else b).double()
t = A @ B
s = A.abs() @ B.abs()
c = torch.zeros(m, n, device="cuda")
ref = None
for it in range(int(os.environ.get("REPS", "20"))):
    c.zero_()
    kcnn.gemm(a, b, c, bool(ta), bool(tb))
    torch.cuda.synchronize()
    r = (c.double() - t).abs() / s.clamp_min(1e-30)
    worst = float(r.max())
    same = ref is None or torch.equal(ref, c)
    if ref is None:
        ref = c.clone()
    bad = (r > 1e-5).nonzero()
    msg = f"run {it}: worst {worst:.3e} bitwise-same-as-run0 {same} bad {bad.shape[0]}"
    if bad.shape[0]:
        rows, cols = bad[:, 0], bad[:, 1]
        msg += (f" rows {int(rows.min())}..{int(rows.max())} (tiles {sorted(set((rows // 256).tolist()))[:8]})"
                f" cols {int(cols.min())}..{int(cols.max())} (tiles {sorted(set((cols // 128).tolist()))[:8]})"
                f" row%64 {sorted(set((rows % 64).tolist()))[:10]} col%64 {sorted(set((cols % 64).tolist()))[:10]}")
    print(msg, flush=True)
