"""Probe: internal accumulation error of the gfx950 f8f6f4 MFMAs behind lcq_fp8_gemm. One
128-wide K block (a single MFMA dot per output for 16x16x128, two chained 32x32x64 for the
<= 64-row kernel), unit scales, so C = sum_k a[m,k] b[n,k] computed by the hardware; compared
with the exact sum (fp64, e4m3 products are exact) relative to sum_k |a b|."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator().manual_seed(0)
for M, N in ((64, 4096), (2048, 2048)):
    for dist in ('randn', 'uniform+'):
        K = 128
        if dist == 'randn':
            a = torch.randn(M, K, generator=g) * 50
            b = torch.randn(N, K, generator=g) * 50
        else:
            a = torch.rand(M, K, generator=g) * 400
            b = torch.rand(N, K, generator=g) * 400
        a8, b8 = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
        ones_a = torch.ones(M, 1)
        ones_b = torch.ones((N + 127) // 128, 1)
        got = ops.fp8_gemm(a8.to(dev), ones_a.to(dev), b8.to(dev), ones_b.to(dev),
                           out_dtype=torch.float32).cpu().double()
        af, bf = a8.double(), b8.double()
        exact = af @ bf.T
        absd = af.abs() @ bf.abs().T
        rel = (got - exact).abs() / absd.clamp_min(1e-300)
        # fp32 sequential-sum bound for comparison: K * 2^-24
        print(f'M{M} N{N} {dist:9s}: max |err| / sum|ab| = {rel.max().item():.3e}  '
              f'mean = {rel.mean().item():.3e}  (fp32 RNE sequential bound {K * 2**-24:.3e}); '
              f'signed mean err/sum|ab| = {((got - exact) / absd).mean().item():+.3e}', flush=True)
