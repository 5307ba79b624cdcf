"""Time the GPTQ Cholesky chain (gptq.py:169-174) with torch's linalg backends on the GPU."""
import time
import torch

dev = 'cuda'
for n in (4096, 14336):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(4 * n, n, device=dev, generator=g) / n ** 0.5
    H = x.T @ x + 0.01 * torch.eye(n, device=dev)
    for lib in ('default', 'cusolver', 'magma'):
        try:
            torch.backends.cuda.preferred_linalg_library(lib)
            for it in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                L = torch.linalg.cholesky(H)
                Hi = torch.cholesky_inverse(L)
                U = torch.linalg.cholesky(Hi, upper=True)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
            Lr = torch.linalg.cholesky(H.flip(0, 1))          # reversal trick: U = J inv(chol(JHJ)) J
            torch.cuda.synchronize(); t2 = time.perf_counter()
            for it in range(3):
                torch.cuda.synchronize(); t2 = time.perf_counter()
                Lr = torch.linalg.cholesky(H.flip(0, 1))
                Ui = torch.linalg.solve_triangular(Lr, torch.eye(n, device=dev), upper=False).flip(0, 1)
                torch.cuda.synchronize(); t3 = time.perf_counter()
            err = ((Ui - U).abs().max() / U.abs().max()).item()
            print(f'n={n} {lib}: chain {1e3*(t1-t0):.1f} ms; reversal {1e3*(t3-t2):.1f} ms (rel diff {err:.2e})', flush=True)
        except Exception as e:
            print(n, lib, 'failed', repr(e)[:200], flush=True)
