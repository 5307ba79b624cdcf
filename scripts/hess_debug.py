"""Hessian kernel debug: error vs fp64 over (n, ic, dtype, beta) cases, with the positions of
the worst elements."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from lightcompress_amd import ops

dev = 'cuda'
cases = [(48, 512, torch.bfloat16, 0.0), (48, 512, torch.bfloat16, 0.5), (192, 512, torch.bfloat16, 0.0),
         (144, 512, torch.bfloat16, 0.0), (128, 512, torch.bfloat16, 0.0), (64, 512, torch.bfloat16, 0.0),
         (300, 520, torch.float16, 0.5), (300, 520, torch.bfloat16, 0.0), (320, 512, torch.bfloat16, 0.0),
         (64, 256, torch.bfloat16, 0.0), (16, 256, torch.bfloat16, 0.0), (37, 136, torch.bfloat16, 0.0)]
for n, ic, dt, beta in cases:
    g = torch.Generator().manual_seed(n + ic)
    x = (torch.randn(n, ic, generator=g) * torch.exp(torch.randn(ic, generator=g))).to(dt)
    H = torch.full((ic, ic), 0.5, device=dev)
    ops.hessian_accum(x.to(dev), H, 0.25, beta)
    xd = x.double()
    ref = 0.25 * xd.t() @ xd + beta * 0.5
    bound = 0.25 * (xd.abs().t() @ xd.abs()) + beta * 0.5
    err = (H.cpu().double() - ref).abs() / (bound + 1e-30)
    bad = (err > 1e-5).nonzero()
    rows = sorted(set(bad[:, 0].tolist()))
    cols = sorted(set(bad[:, 1].tolist()))
    print(f'n {n} ic {ic} {dt} beta {beta}: max rel {err.max().item():.2e} bad {bad.shape[0]} '
          f'rows {rows[:12]}{"..." if len(rows) > 12 else ""} cols {cols[:12]}', flush=True)
