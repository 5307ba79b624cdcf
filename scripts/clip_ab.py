"""A/B of the auto-clip search kernel's bf16 product widening (LCQ_CLIP_CVT=0: convert +
shift / mask; default: one convert per product) at Llama-3-8B shapes, interleaved rounds in
one process; the two outputs must be identical."""
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
for oc, ic in [(14336, 4096), (4096, 14336)]:
    w = (torch.randn(oc, ic, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    x = (torch.randn(512, ic, generator=g, device=dev) *
         torch.exp(torch.randn(ic, generator=g, device=dev))).to(torch.bfloat16)
    outs, res = {}, {'0': [], '1': []}
    for v in res:
        os.environ['LCQ_CLIP_CVT'] = v
        outs[v] = ops.auto_clip_search(w, x, 128, 10, 20, -8, 7, True, True)
    same = all(torch.equal(a, b) for a, b in zip(outs['0'], outs['1']))
    for _ in range(3):
        for v in res:
            os.environ['LCQ_CLIP_CVT'] = v
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(2):
                ops.auto_clip_search(w, x, 128, 10, 20, -8, 7, True, True)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 2)
    print(f'{oc}x{ic}: cvt+shift/mask {statistics.median(res["0"]):.2f} ms, one cvt per product '
          f'{statistics.median(res["1"]):.2f} ms, identical outputs: {same}')
