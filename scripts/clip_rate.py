"""Device rate of the per-group auto-clip search (lcq_auto_clip_search_act, k_auto_clip) at the
Llama-3-8B linear shapes of the AWQ headline (w4 g128, 512 sampled tokens, 10 shrink steps):
products = oc * ic * T * (1 + steps), each rounded to bf16 before its fp32 sum (VALU-bound).

usage: python scripts/clip_rate.py [--act]
"""
import argparse
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import _native as N  # noqa: E402
from lightcompress_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--act', action='store_true', help='w_only False: qx = x (the act path)')
a = ap.parse_args()
dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
tot_ms = 0.0
for oc, ic in [(1024, 4096), (4096, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]:
    w = (torch.randn(oc, ic, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    x = (torch.randn(512, ic, generator=g, device=dev) *
         torch.exp(torch.randn(ic, generator=g, device=dev))).to(torch.bfloat16)
    qx = x.clone() if a.act else None
    for sym in (True, False):
        qmin, qmax = (-8, 7) if sym else (0, 15)
        res = {}
        lib = N.load()
        for tl in ('token-lds ', 'token-lane', 'lane-pair '):
            ops.CLIP_TOKEN_LANE = tl != 'lane-pair '
            lib.lcq_auto_clip_force_variant({'token-lane': 1, 'token-lds ': 3}.get(tl, 2))
            res[tl] = ops.auto_clip_search(w, x, 128, 10, 20, qmin, qmax, sym, sym, qx=qx)
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.auto_clip_search(w, x, 128, 10, 20, qmin, qmax, sym, sym, qx=qx)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            if sym and tl == 'token-lds ':
                tot_ms += ms
            prods = oc * ic * 512 * 11
            print(f'{oc}x{ic} sym={sym} {tl}: {ms:7.2f} ms  {prods / ms / 1e9:6.1f} G products/s',
                  flush=True)
        same = all(torch.equal(a.view(torch.int16), b.view(torch.int16))
                   for k in res for a, b in zip(res[k], res['lane-pair ']))
        print(f'  bit-identical: {same}', flush=True)
ops.CLIP_TOKEN_LANE = True
N.load().lcq_auto_clip_force_variant(0)
print(f'one Llama-3-8B block (v, o, gate, up, down; sym, token-lds): {tot_ms:.1f} ms')
