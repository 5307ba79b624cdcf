"""k_syrk256 throughput vs N (tokens) and IC, kernel-only (workspace preallocated)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from lightcompress_amd import _native as N  # noqa: E402

lib = N.load()
for ic in (4096, 14336):
    for n in (8192, 32768, 131072, 262144):
        x = (torch.randn(n, ic, device='cuda') * 0.5).to(torch.bfloat16)
        H = torch.zeros(ic, ic, device='cuda')
        wsb = lib.lcq_hessian_workspace_bytes(n, ic)
        ws = torch.empty(wsb, dtype=torch.uint8, device='cuda')
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            lib.lcq_hessian_accum(x.data_ptr(), 2, n, ic, H.data_ptr(), 1.0, 0.0, ws.data_ptr(), wsb, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            lib.lcq_hessian_accum(x.data_ptr(), 2, n, ic, H.data_ptr(), 1.0, 0.0, ws.data_ptr(), wsb, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(f'ic={ic:6d} n={n:7d} {ms:8.3f} ms  {n * ic * (ic + 1) / ms / 1e9:7.1f} TFLOP/s', flush=True)
        del x, H, ws
        torch.cuda.empty_cache()
