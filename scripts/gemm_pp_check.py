"""Output digests of every lcq projection-GEMM entry point (plain / 3-segment / SiLU pair /
residual / squared-error loss) on seeded random operands, including ragged M and N edges:
run once per library build (LCQ_LIB_PATH) and diff the two outputs to check that two GEMM
kernels give bit-identical results.

usage: python scripts/gemm_pp_check.py
"""
import hashlib
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402


def h(t):
    return hashlib.sha256(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


g = torch.Generator(device='cuda').manual_seed(0)


def rnd(*s, sc=1.0, dt=torch.bfloat16):
    return (torch.randn(*s, generator=g, device='cuda') * sc).to(dt)


for (M, N, K) in [(65536, 4096, 4096), (1000, 784, 512), (257, 272, 128), (4096, 14336, 4096)]:
    for dt in (torch.bfloat16, torch.float16):
        x, w, b = rnd(M, K, dt=dt), rnd(N, K, sc=0.05, dt=dt), rnd(N, sc=0.1, dt=dt)
        print('linear', M, N, K, dt, h(ops.linear(x, w)), h(ops.linear(x, w, b)))
        ws = [rnd(n, K, sc=0.05, dt=dt) for n in (512, 256, 144)]
        print('multi', M, K, dt, *[h(o) for o in ops.linear_multi(x, ws)])
        wg, wu = rnd(N, K, sc=0.05, dt=dt), rnd(N, K, sc=0.05, dt=dt)
        print('silu', M, N, K, dt, h(ops.linear_silu_mul(x, wg, wu)))
        res = rnd(M, N, dt=dt)
        print('resid', M, N, K, dt, h(ops.linear_residual(x, w, res, bias=b)))
        lb = ops.LossBuffer(2, 'cuda')
        org = rnd(M, N, dt=dt)
        ops.linear_sq_diff(x, w, org, lb, 0)
        ops.linear_sq_diff(x, w, org, lb, 1, bias=b)
        print('sqdiff', M, N, K, dt, h(lb.out), lb.out.tolist())
torch.cuda.synchronize()
print('done')
