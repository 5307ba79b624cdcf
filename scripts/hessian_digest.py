"""Output digests of the GPTQ Hessian entry points (lcq_hessian_accum, lcq_hessian_grouped) on
seeded token-major activations, ragged token counts and channel counts included: run once per
library build (LCQ_LIB_PATH) and diff the outputs to check two schedules are bit-identical.

usage: python scripts/hessian_digest.py
"""
import hashlib
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402


def h(t):
    return hashlib.sha256(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]


dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
for n, ic in [(262144, 4096), (32768 + 37, 1000), (5000, 4096), (65536, 14336)]:
    x = torch.randn(n, ic, generator=g, device=dev).to(torch.bfloat16)
    H = torch.randn(ic, ic, generator=g, device=dev)
    ops.hessian_accum(x, H, 0.5, 0.25)
    per = n // 8
    bounds = [i * per for i in range(8)] + [n]
    G = torch.empty(ic, ic, device=dev)
    ops.hessian_grouped(x, bounds, G, 2.0 / 128)
    print(n, ic, 'accum', h(H), 'grouped', h(G))
    del x, H, G
torch.cuda.synchronize()
print('done')
