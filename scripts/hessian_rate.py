"""GPTQ Hessian (lcq_hessian_accum: k_syrk_x reading token-major X with transposed LDS reads)
rate at the GPTQ calibration size (128 x 2048 tokens), random bf16 activations, and its error
against an fp64 product on a token slice. Flops = n * ic * (ic + 1) (the upper triangle).

usage: python scripts/hessian_rate.py [--n 262144] [--ics 4096,14336,8192] [--iters 5]
"""
import argparse
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--n', type=int, default=262144)
ap.add_argument('--ics', default='4096,14336,8192')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--iters', type=int, default=3)
a = ap.parse_args()
g = torch.Generator(device='cuda').manual_seed(0)
for ic in map(int, a.ics.split(',')):
    x = torch.randn(a.n, ic, generator=g, device='cuda').to(torch.bfloat16)
    H = torch.zeros(ic, ic, device='cuda')
    ops.hessian_accum(x, H, 1.0, 0.0)
    xs = x[:4096].double()
    Hs = torch.zeros(ic, ic, device='cuda')
    ops.hessian_accum(x[:4096], Hs, 1.0, 0.0)
    ref = xs.t() @ xs
    bound = xs.abs().t() @ xs.abs()
    err = ((Hs.double() - ref).abs() / bound).max().item()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.hessian_accum(x, H, 1.0, 0.0)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / a.iters)
    fl = a.n * ic * (ic + 1)
    t = statistics.median(ts)
    print(f'ic {ic} n {a.n}: {t:8.3f} ms {fl / t / 1e9:8.1f} TFLOP/s '
          f'({fl / t / 1e9 / 2500:.3f} of 2.5 PF); 4096-token max rel err vs fp64 {err:.2e}; '
          f'symmetric {bool(torch.equal(H, H.t()))}', flush=True)
    del x, H, Hs
    torch.cuda.empty_cache()
