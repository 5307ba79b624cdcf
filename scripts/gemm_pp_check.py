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
# q/k/v with the rotary in the epilogue (lcq_gemm_rope), ragged rows
for B, S in ((2, 384), (3, 100)):
    x = rnd(B, S, 512)
    ws = [rnd(n, 512, sc=0.05) for n in (512, 256, 256)]
    cos, sin = rnd(B, S, 128), rnd(B, S, 128)
    print('rope', B, S, *[h(o) for o in ops.linear_multi_rope(x, ws, [None] * 3, cos, sin,
                                                             rope_segs=2)])
# split-plane fp32 products (lcq_gemm_f32x6): split K below 256 tiles, k-major A, row ranges
for (M, N, K, at) in [(3584, 3584, 7168, False), (1792, 1792, 1792, False),
                      (4096, 3072, 1024, True), (1000, 528, 1100, False)]:
    A = torch.randn((K, M) if at else (M, K), generator=g, device='cuda')
    Bm = torch.randn(K, N, generator=g, device='cuda')
    C = torch.randn(M, N, generator=g, device='cuda')
    ops.gemm_f32x6(A, Bm, C, -1.0, 1.0, False, a_trans=at)
    C2 = torch.randn(M, N, generator=g, device='cuda')
    ops.gemm_f32x6(A, Bm, C2, 1.0, 0.0, False, M // 4, M // 2, a_trans=at)
    print('x6', M, N, K, at, h(C), h(C2[M // 4:M // 2]))
torch.cuda.synchronize()
print('done')
