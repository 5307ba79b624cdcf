"""Time lcq_hessian_accum at the GPTQ bench shapes for forced split-K counts (LCQ_SYRK_NS)."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import ops  # noqa: E402

n = 262144
for ic, nss in ((4096, (0, 4, 6, 8, 11, 15)), (14336, (0, 1, 2, 3, 4))):
    x = (torch.randn(n, ic, device='cuda') * 0.5).to(torch.bfloat16)
    H = torch.zeros(ic, ic, device='cuda')
    for ns in nss:
        if ns:
            os.environ['LCQ_SYRK_NS'] = str(ns)
        else:
            os.environ.pop('LCQ_SYRK_NS', None)
        for _ in range(2):
            ops.hessian_accum(x, H, 1.0, 0.0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ops.hessian_accum(x, H, 1.0, 0.0)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        fl = n * ic * (ic + 1)
        print(f'ic={ic} ns={ns or "auto"}: {ms:.3f} ms, {fl / ms / 1e9:.1f} TFLOP/s', flush=True)
    del x, H
    torch.cuda.empty_cache()
