"""Timing-only diagnostic builds of k_gemm16 (LCQ_GEMM_DIAG, outputs wrong) against the real
kernel and torch F.linear (hipBLASLt), interleaved rounds in one process, random data.
DIAG 1 = no memory traffic (zero-record descriptors), 2 = no K-loop barriers, 3 = both.

usage: python scripts/gemm_diag.py [--m 65536] [--n 4096] [--k 4096] [--rounds 5]
"""
import argparse
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--m', type=int, default=65536)
ap.add_argument('--n', type=int, default=4096)
ap.add_argument('--k', type=int, default=4096)
ap.add_argument('--rounds', type=int, default=5)
ap.add_argument('--iters', type=int, default=10)
ap.add_argument('--diags', default='0,1,2,3')
a = ap.parse_args()
g = torch.Generator(device='cuda').manual_seed(0)
x = (torch.rand(a.m, a.k, generator=g, device='cuda') * 2 - 1).to(torch.bfloat16)
w = (torch.rand(a.n, a.k, generator=g, device='cuda') * 2 - 1).to(torch.bfloat16)
fl = 2.0 * a.m * a.n * a.k


def run(d):
    if d == 'torch':
        return lambda: F.linear(x, w)
    def f():
        if d == '-':
            os.environ.pop('LCQ_GEMM_DIAG', None)
        else:
            os.environ['LCQ_GEMM_DIAG'] = d
        ops.linear(x, w)
    return f


def timeit(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters


variants = ['-'] + a.diags.split(',') + ['torch']
res = {v: [] for v in variants}
for v in variants:
    run(v)()
torch.cuda.synchronize()
for _ in range(a.rounds):
    for v in variants:
        res[v].append(timeit(run(v)))
print(f'M {a.m} N {a.n} K {a.k}: median of {a.rounds} rounds x {a.iters} (ms, TFLOP/s)')
for v in variants:
    t = statistics.median(res[v])
    print(f'  {"lcq" if v == "-" else ("diag " + v if v != "torch" else "torch"):8s} {t:8.3f} ms '
          f'{fl / t / 1e9:8.1f} TF/s')
