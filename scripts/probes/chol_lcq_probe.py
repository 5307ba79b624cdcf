"""Time U = chol(H^-1, upper): lcq recursive tiles + fp32 GEMMs vs MAGMA's reversal chain."""
import os
import time
import torch
from lightcompress_amd import gptq_core, ops
from lightcompress_amd import _native as N

dev = 'cuda'


def tm(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, out


A = torch.randn(128, 256, device=dev)
T = A @ A.t() / 128 + 0.1 * torch.eye(128, device=dev)
info = torch.zeros(1, dtype=torch.int32, device=dev)
Tc = T.clone()
t, X = tm(lambda: ops.chol_inv_tile(Tc.copy_(T), info), 10)
L = torch.linalg.cholesky(T)
print(f'chol_inv_tile 128: {t*1e3:.0f} us (incl copy); |L-Lref| {(Tc - L).abs().max().item():.2e} '
      f'|LX-I| {(L @ X - torch.eye(128, device=dev)).abs().max().item():.2e}')
with N.KernelTimer() as kt:
    for _ in range(5):
        ops.chol_inv_tile(Tc.copy_(T), info)
print(kt.summary())

for n in (4096, 14336):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(4 * n, n, device=dev, generator=g) / n ** 0.5
    H = x.T @ x + 0.01 * torch.eye(n, device=dev)
    del x
    torch.backends.cuda.preferred_linalg_library('magma')

    def magma():
        C = torch.linalg.cholesky(H.flip(0, 1))
        return torch.linalg.solve_triangular(C, torch.eye(n, device=dev), upper=False).flip(0, 1).contiguous()

    tmg, Um = tm(magma)
    tl, Ul = tm(lambda: gptq_core.inverse_cholesky_upper(H.clone()))
    rel = ((Ul - Um).abs().max() / Um.abs().max()).item()
    print(f'n={n}: magma {tmg:.1f} ms, lcq {tl:.1f} ms, rel diff {rel:.2e}', flush=True)
    with N.KernelTimer() as kt:
        gptq_core.inverse_cholesky_upper(H.clone())
    print(kt.summary() if hasattr(kt, 'summary') else '', flush=True)
