"""A/B of the auto-clip search kernel's quotient (default: Markstein from RN(1/s);
LCQ_CLIP_DIV=ieee: the IEEE division sequence) at Llama-3-8B shapes (w4 g128 sym and asym),
interleaved rounds in one process; the two outputs must be identical."""
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
for oc, ic, sym in [(14336, 4096, True), (4096, 14336, True), (14336, 4096, False)]:
    w = (torch.randn(oc, ic, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    x = (torch.randn(512, ic, generator=g, device=dev) *
         torch.exp(torch.randn(ic, generator=g, device=dev))).to(torch.bfloat16)
    qmin, qmax = (-8, 7) if sym else (0, 15)
    outs, res = {}, {'ieee': [], 'mk': []}
    for v in res:
        os.environ['LCQ_CLIP_DIV'] = v
        outs[v] = ops.auto_clip_search(w, x, 128, 10, 20, qmin, qmax, sym, sym)
    same = all(torch.equal(a, b) for a, b in zip(outs['ieee'], outs['mk']))
    for _ in range(3):
        for v in res:
            os.environ['LCQ_CLIP_DIV'] = v
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(2):
                ops.auto_clip_search(w, x, 128, 10, 20, qmin, qmax, sym, sym)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 2)
    os.environ.pop('LCQ_CLIP_DIV', None)
    print(f'{oc}x{ic} sym={sym}: ieee {statistics.median(res["ieee"]):.2f} ms, markstein '
          f'{statistics.median(res["mk"]):.2f} ms, identical outputs: {same}', flush=True)
