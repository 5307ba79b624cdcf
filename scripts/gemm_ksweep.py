"""Per-tile fixed cost of the lcq GEMM: time vs K at M = 65536, N = 4096 (lcq vs torch).
Fits t = a + b * K per kernel: `a` is the prologue + epilogue cost of one tile round."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from lightcompress_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


M, N = 65536, 4096
g = torch.Generator(device='cuda').manual_seed(0)
rows = []
for K in (256, 512, 1024, 2048, 4096, 8192):
    x = torch.randn(M, K, generator=g, device='cuda').to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device='cuda') * 0.02).to(torch.bfloat16)
    org = torch.randn(M, N, generator=g, device='cuda').to(torch.bfloat16)
    lb = ops.LossBuffer(1, 'cuda')
    a = min(timeit(lambda: ops.linear(x, w)) for _ in range(3))
    c = min(timeit(lambda: ops.linear_sq_diff(x, w, org, lb, 0)) for _ in range(3))
    b = min(timeit(lambda: F.linear(x, w)) for _ in range(3))
    rows.append((K, a, c, b))
    print(f'K {K:5d}: lcq store {a:7.3f} ms  lcq loss {c:7.3f} ms  torch {b:7.3f} ms  '
          f'({2 * M * N * K / a / 1e9:6.0f} / {2 * M * N * K / b / 1e9:6.0f} TF/s)', flush=True)
for idx, name in ((1, 'lcq store'), (2, 'lcq loss'), (3, 'torch')):
    import numpy as np
    Ks = np.array([r[0] for r in rows], dtype=float)
    ts = np.array([r[idx] for r in rows])
    bb, aa = np.polyfit(Ks, ts, 1)
    print(f'{name}: t = {aa * 1e3:.1f} us + {bb * 1e3 * 64:.3f} us per 64-K step (16 tile rounds)')
