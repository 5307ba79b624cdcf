"""Probe: where the inverse-Cholesky chain's time goes (gptq_core._chol_inv_rec, eager, no
graph, no side stream): every lcq_gemm_f32 call timed with events on the compute stream and
grouped by (M, N, K, b_trans), the diagonal lcq_chol_inv_tile launches summed, at the
Llama-3-8B Hessian sizes."""
import sys
from collections import defaultdict
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import gptq_core, ops  # noqa: E402

dev = torch.device('cuda:0')
gptq_core._OVERLAP_MIN = 10 ** 9   # serial: event pairs bracket single launches
rec = []
orig_gemm, orig_tile = gptq_core._gemm, ops.chol_inv_tile


def gemm(A, B, out, alpha, beta, b_trans=False):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = orig_gemm(A, B, out, alpha, beta, b_trans)
    e1.record()
    rec.append(('gemm', (A.shape[0], out.shape[1], A.shape[1], int(b_trans)), e0, e1))
    return r


def tile(A, info, row0=0, L=None, out=None):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = orig_tile(A, info, row0, L=L, out=out)
    e1.record()
    rec.append(('tile', (A.shape[0],), e0, e1))
    return r


gptq_core._gemm = gemm
ops.chol_inv_tile = tile
gptq_core.CHAIN_GRAPHS = False
for n in (4096, 14336):
    g = torch.Generator(device=dev).manual_seed(n)
    X = torch.randn(n, 2 * n, device=dev, generator=g)
    H = X @ X.T / (2 * n)
    H.diagonal().add_(0.01)
    del X
    gptq_core.inverse_cholesky_upper(H.clone())   # warm
    rec.clear()
    torch.cuda.synchronize()
    w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0.record()
    gptq_core.inverse_cholesky_upper(H.clone())
    w1.record()
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for kind, key, e0, e1 in rec:
        ms = e0.elapsed_time(e1)
        a = agg[(kind, key)]
        a[0] += 1
        a[1] += ms
        if kind == 'gemm':
            a[2] += 2.0 * key[0] * key[1] * key[2]
    tot = sum(v[1] for v in agg.values())
    print(f'n {n}: chain wall {w0.elapsed_time(w1):.2f} ms, sum of timed launches '
          f'{tot:.2f} ms, {len(rec)} launches', flush=True)
    for (kind, key), (cnt, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        rate = f'{fl / (ms * 1e-3) / 1e12:6.1f} TF/s' if fl else ''
        print(f'  {kind:5s} {str(key):28s} x{cnt:4d} {ms:8.3f} ms {rate}', flush=True)
