"""Quick device timing of the grouped quant kernels on Llama-3-8B linear shapes (dev aid)."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch

from lightcompress_amd import ops

dev = torch.device('cuda:0')
res = {}
for shape in [(4096, 4096), (14336, 4096), (4096, 14336)]:
    w = (torch.randn(*shape, device=dev) * 0.02).to(torch.bfloat16)
    for mode in ['fq', 'pack4']:
        kw = dict(fq=True, qparams=False) if mode == 'fq' else dict(fq=False, pack_bits=4)
        for _ in range(3):
            ops.int_quant_dynamic(w, 128, 0, 15, False, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            ops.int_quant_dynamic(w, 128, 0, 15, False, **kw)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        nbytes = w.numel() * (2 + (2 if mode == 'fq' else 0.5)) + w.numel() / 128 * 4
        res[f'{shape}-{mode}'] = dict(ms=ms, GBps=nbytes / ms / 1e6)
print(json.dumps(res, indent=1))
