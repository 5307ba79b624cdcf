"""Probe (GPU): rate of the factorisation chain's large fp32 products (lcq_gemm_f32 /
gemm_f32_rows, 32x32x2 / 16x16x4 fp32 MFMA) against the same products as ONE bf16 GEMM over
6 split-plane segments (K' = 6K: [A0 A0 A1 A0 A1 A2] x [B0 B1 B0 B2 B1 B0], lcq k_gemm16h) --
the bf16x6 emulation whose accuracy scripts/chain_split_study.py measures (as accurate as the
fp32 GEMM on the chain). Also times the plane split (torch elementwise, an upper bound for a
fused split kernel). bf16 output here (rate only; the product would need an fp32 epilogue).
usage: chain_split_rate.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import ops  # noqa: E402

SHAPES = [(7168, 1792, 1792), (1792, 7168, 1792), (1792, 1792, 7168), (3584, 3584, 7168),
          (7168, 3584, 3584), (3584, 1792, 1792), (1792, 1792, 1792), (896, 896, 896),
          (4096, 4096, 4096)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def planes(a):
    a0 = a.to(torch.bfloat16)
    r = a - a0.float()
    a1 = r.to(torch.bfloat16)
    a2 = (r - a1.float()).to(torch.bfloat16)
    return a0, a1, a2


def main():
    dev = torch.device('cuda:0')
    for M, N, K in SHAPES:
        A = torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev)
        C = torch.empty(M, N, device=dev)
        f32 = timeit(lambda: ops.gemm_f32_rows(A, B, C, 1.0, 0.0, True, 0, M))
        f32sk = timeit(lambda: ops.gemm_f32(A, B, C, 1.0, 0.0, b_trans=True))
        a0, a1, a2 = planes(A)
        b0, b1, b2 = planes(B)
        Ap = torch.cat([a0, a0, a1, a0, a1, a2], dim=1).contiguous()
        Bp = torch.cat([b0, b1, b0, b2, b1, b0], dim=1).contiguous()
        x6 = timeit(lambda: ops.linear(Ap, Bp))
        Ap3 = torch.cat([a0, a0, a1], dim=1).contiguous()
        Bp3 = torch.cat([b0, b1, b0], dim=1).contiguous()
        x3 = timeit(lambda: ops.linear(Ap3, Bp3))
        sp = timeit(lambda: (planes(A), planes(B)), reps=5)
        # accuracy of the bf16x6 product vs fp64 (bf16 output dominates: fp32 ref instead)
        fl = 2.0 * M * N * K
        print(f'M {M:5d} N {N:5d} K {K:5d}: f32 tiled {f32:7.3f} ms ({fl / f32 / 1e9:6.1f} TF/s)'
              f' | f32 stream-K {f32sk:7.3f} | bf16x6 {x6:7.3f} ms ({fl / x6 / 1e9:6.1f} TF/s eq)'
              f' | bf16x3 {x3:7.3f} | split (torch) {sp:6.3f} ms', flush=True)


if __name__ == '__main__':
    main()
