"""lcq_scale_bcast (x / s per column) at the AWQ loss-search shape: the per-column fast kernel
(k_scale_cols) vs the generic grid-stride kernel (LCQ_SCALE_GENERIC=1), interleaved rounds.
Traffic = 2 B read + 2 B written per element."""
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

for rows, cols in ((65536, 4096), (65536, 14336)):
    x = torch.randn(rows, cols, device='cuda').to(torch.bfloat16)
    s = torch.exp(torch.randn(cols, device='cuda')).to(torch.bfloat16)
    out = torch.empty_like(x)
    res = {'fast': [], 'generic': []}
    outs = {}
    for r in range(5):
        for v in res:
            if v == 'generic':
                os.environ['LCQ_SCALE_GENERIC'] = '1'
            else:
                os.environ.pop('LCQ_SCALE_GENERIC', None)
            ops.scale_bcast(x, s, 'div', out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.scale_bcast(x, s, 'div', out=out)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 10)
            outs[v] = out.clone()
    os.environ.pop('LCQ_SCALE_GENERIC', None)
    same = torch.equal(outs['fast'].view(torch.int16), outs['generic'].view(torch.int16))
    for v in res:
        ms = statistics.median(res[v])
        print(f'{rows}x{cols} {v}: {ms:.4f} ms  {4 * rows * cols / ms / 1e9:.0f} GB/s  '
              f'bit-equal fast/generic {same}', flush=True)
