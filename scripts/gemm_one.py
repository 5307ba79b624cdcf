"""One projection shape, lcq GEMM and torch F.linear (hipBLASLt) back to back, for rocprofv3
PMC / kernel-trace comparisons of the two kernels on identical random data.

usage: python scripts/gemm_one.py [--m 65536] [--n 4096] [--k 4096] [--iters 20] [--only lcq|torch]
"""
import argparse
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
ap.add_argument('--iters', type=int, default=20)
ap.add_argument('--only', default='')
a = ap.parse_args()
g = torch.Generator(device='cuda').manual_seed(0)
x = torch.randn(a.m, a.k, generator=g, device='cuda').to(torch.bfloat16)
w = (torch.randn(a.n, a.k, generator=g, device='cuda') * 0.02).to(torch.bfloat16)
for _ in range(a.iters):
    if a.only != 'torch':
        ops.linear(x, w)
    if a.only != 'lcq':
        F.linear(x, w)
torch.cuda.synchronize()
print('done')
