"""One 14336 inverse_cholesky_upper under the profiler: GPU kernel time vs wall time."""
import time
import torch
from lightcompress_amd import gptq_core

dev = 'cuda'
n = 14336
x = torch.randn(4 * n, n, device=dev) / n ** 0.5
H = x.T @ x + 0.01 * torch.eye(n, device=dev)
del x
for i in range(3):
    Hc = H.clone()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    U = gptq_core.inverse_cholesky_upper(Hc)
    torch.cuda.synchronize()
    print(f'wall {1e3 * (time.perf_counter() - t0):.1f} ms', flush=True)
