"""Time the three FC GEMMs of the c2 stack (fp32) under torch's BLAS backends."""
import time, torch
M, K, N = 4096, 11616, 1024
P = torch.randn(M, K, device="cuda"); W = torch.randn(N, K, device="cuda") * 0.01
dY = torch.randn(M, N, device="cuda")
def run():
    Y = P @ W.t(); dP = dY @ W; gW = dY.t() @ P
    return Y, dP, gW
for lib in ("cublas", "hipblaslt"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print(lib, "unavailable", e); continue
    for _ in range(3): run()
    torch.cuda.synchronize()
    for name, f in (("fwd", lambda: P @ W.t()), ("dP", lambda: dY @ W), ("gW", lambda: dY.t() @ P)):
        for _ in range(3): f()
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(20): f()
        torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
        print(f"{lib:10s} {name:4s} {dt*1e3:7.3f} ms  {2*M*K*N/dt/1e12:6.1f} TF/s", flush=True)
