"""Time lcq_hessian_accum at the GPTQ bench shapes (n = 128 x 2048 tokens)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from lightcompress_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
for ic in (4096, 14336):
    x = (torch.randn(n, ic, device='cuda') * 0.5).to(torch.bfloat16)
    H = torch.zeros(ic, ic, device='cuda')
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
    print(f'ic={ic} n={n}: {ms:.3f} ms/launch, {fl / ms / 1e9:.1f} TFLOP/s (symmetric flops)', flush=True)
    del x, H
    torch.cuda.empty_cache()
