"""inverse_cholesky_upper time vs the triangular-split threshold (_TRI_MIN), rocBLAS."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from lightcompress_amd import gptq_core  # noqa: E402

dev = 'cuda'
for n in (4096, 14336):
    x = torch.randn(2 * n, n, device=dev) / n ** 0.5
    H = x.T @ x + 0.01 * torch.eye(n, device=dev)
    del x
    for tm in (256, 512, 1024, 2048, 4096):
        gptq_core._TRI_MIN = tm
        for _ in range(2):
            U = gptq_core.inverse_cholesky_upper(H.clone())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            U = gptq_core.inverse_cholesky_upper(H.clone())
        e1.record()
        torch.cuda.synchronize()
        print(f'n={n} tri_min={tm}: {e0.elapsed_time(e1) / 3:.2f} ms', flush=True)
