"""Print where the use_qtorch=False emulation kernel differs from the reference fixture."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tests' / 'golden'))
import fixtures as F  # noqa: E402
from lightcompress_amd import ops  # noqa: E402

for name in ['e4m3_pc_bf16', 'e4m3_pc_f16', 'e3m2_pc_bf16']:
    c = F.load(f'fp8emul_{name}')
    e, m, gs = (int(v) for v in c['meta'])
    w = c['w']
    out = ops.fp_emul_quant(w.cuda(), gs, e, m).cpu().float()
    ref = c['fq'].float()
    bad = ~((out == ref) | (out.isnan() & ref.isnan()))
    print(name, 'mismatch', int(bad.sum()), 'of', bad.numel(), 'rows', bad.any(1).nonzero().flatten().tolist()[:10])
    idx = bad.nonzero()[:8]
    for r, k in idx.tolist():
        mx = w[r].float().abs().max().item()
        print(f'  r{r} c{k} x={w[r, k].item():.6g} ref={ref[r, k].item():.6g} got={out[r, k].item():.6g} maxval={mx:.6g}')
