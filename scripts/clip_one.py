"""One auto-clip search shape, a few launches, for rocprofv3 PMC passes (VALU issue / wait and
scalar-cache behaviour of k_auto_clip vs the token-lane kernels).

usage: python scripts/clip_one.py [tl|tw|pair] [oc] [ic] [iters]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'tl'
oc = int(sys.argv[2]) if len(sys.argv) > 2 else 14336
ic = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 2
ops.CLIP_TOKEN_LANE = kind in ('tl', 'tw')
from lightcompress_amd import _native as N  # noqa: E402
N.load().lcq_auto_clip_force_variant({'tl': 1, 'tw': 3}.get(kind, 0))
dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
w = (torch.randn(oc, ic, generator=g, device=dev) * 0.02).to(torch.bfloat16)
x = (torch.randn(512, ic, generator=g, device=dev) *
     torch.exp(torch.randn(ic, generator=g, device=dev))).to(torch.bfloat16)
for _ in range(iters):
    ops.auto_clip_search(w, x, 128, 10, 20, -8, 7, True, True)
torch.cuda.synchronize()
print('done', kind, oc, ic, iters)
