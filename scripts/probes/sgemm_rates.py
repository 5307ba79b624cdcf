"""fp32 GEMM rates on MI355X: torch.mm (rocBLAS/hipBLASLt) at the Cholesky-recursion shapes vs
the lcq fp32 MFMA trailing kernel (W -= err^T U)."""
import time
import torch
from lightcompress_amd import ops

dev = 'cuda'


def tm(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


for m in (7168, 3584, 2048, 1792, 896):
    a = torch.randn(m, m, device=dev); b = torch.randn(m, m, device=dev)
    t = tm(lambda: a @ b)
    t2 = tm(lambda: a @ b.t())
    c = torch.randn(m, m, device=dev)
    t3 = tm(lambda: c.addmm_(a, b.t(), alpha=-1.0))
    print(f'torch.mm {m}^3: NN {2*m**3/t/1e12:.1f} TF/s  NT {2*m**3/t2/1e12:.1f}  addmm NT {2*m**3/t3/1e12:.1f}', flush=True)
for rows, K, cols in ((7168, 1024, 7168), (7168, 7168, 7168), (4096, 4096, 4096), (3584, 3584, 3584)):
    W = torch.randn(rows, cols, device=dev)
    U = torch.randn(K, cols, device=dev)
    err = torch.randn(K, rows, device=dev)
    t = tm(lambda: ops.gptq_trailing(W, 0, K, K if K < cols else 0, err, U) if K < cols else None)
    if K < cols:
        print(f'trailing rows {rows} K {K} cols {cols - K}: {2*rows*K*(cols-K)/t/1e12:.1f} TF/s', flush=True)
