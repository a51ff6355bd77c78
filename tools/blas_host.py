"""Host cost per torch GEMM call (no sync) with hipBLASLt vs rocBLAS, KPFCNN
shapes: forward linear, and the two backward GEMMs."""
import time

import torch
import torch.nn.functional as F

dev = torch.device("cuda", 0)
x = torch.randn(40000, 32, device=dev, requires_grad=True)
w = torch.randn(128, 32, device=dev, requires_grad=True)
xs = torch.randn(2500, 256, device=dev, requires_grad=True)
ws = torch.randn(512, 256, device=dev, requires_grad=True)
print("default backend", torch.backends.cuda.preferred_blas_library())
for lib in ("cublaslt", "cublas", "cublaslt", "cublas"):
    torch.backends.cuda.preferred_blas_library(lib)
    for a, b in ((x, w), (xs, ws)):
        for _ in range(20):
            F.linear(a, b).sum().backward()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(200):
            y = F.linear(a, b)
        th = (time.perf_counter() - t) / 200
        torch.cuda.synchronize()
        tg = (time.perf_counter() - t) / 200
        g = torch.ones_like(y)
        t = time.perf_counter()
        for _ in range(100):
            torch.autograd.grad(y, (a, b), g, retain_graph=True)
        tb = (time.perf_counter() - t) / 100
        torch.cuda.synchronize()
        tbg = (time.perf_counter() - t) / 100
        print(f"{lib:9s} {tuple(a.shape)}x{tuple(b.shape)}: fwd host {th*1e6:6.1f} us (with GPU {tg*1e6:6.1f}), "
              f"bwd host {tb*1e6:6.1f} us (with GPU {tbg*1e6:6.1f})")
