"""Diagnostics for tests/test_pipeline_golden_gpu.py: per-layer GPTQ Hessians and per-subset
AWQ scales of our pipeline vs the reference's (tests/golden/pipe_*_diag.npz)."""
import sys
import types
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / 'tests'), str(ROOT / 'tests' / 'golden')]
import fixtures as F  # noqa: E402
from test_pipeline_golden_gpu import run_ours  # noqa: E402

dev = torch.device('cuda:0')
which = sys.argv[1] if len(sys.argv) > 1 else 'gptq'
ref = F.load(f'pipe_{which}_diag')
ours = {}
if which == 'gptq':
    from lightcompress_amd.gptq import GPTQ
    orig = GPTQ.layer_transform

    def lt(self, layer, name):
        ours[f'H_b{self.block_idx}__{name.replace(".", "__")}'] = \
            self.layers_cache[name]['acc'].H.detach().cpu().clone()
        return orig(self, layer, name)
    GPTQ.layer_transform = lt
else:
    from lightcompress_amd.awq import Awq
    orig = Awq.search_scale_subset

    def ss(self, *a, **k):
        best = orig(self, *a, **k)
        n = len([d for d in ours if d.startswith(f'S_b{self.block_idx}')])
        ours[f'S_b{self.block_idx}__{n}'] = best.detach().cpu().clone()
        ours[f'L_b{self.block_idx}__{n}'] = torch.tensor(self.last_search['losses'],
                                                         dtype=torch.float64)
        return best
    Awq.search_scale_subset = ss
run_ours(which, dev)
for k in ref:
    r = ref[k].float()
    if k not in ours:
        print(f'{k:32s} MISSING in ours')
        continue
    o = ours[k].float()
    if k.startswith('L_'):
        print(k, 'ref argmin', int(r.argmin()), 'ours', int(o.argmin()))
        print('   ref ', ' '.join(f'{v:.6e}' for v in r.tolist()))
        print('   ours', ' '.join(f'{v:.6e}' for v in o.tolist()))
    rel = ((o - r).norm() / r.norm()).item()
    eq = (o == r).float().mean().item()
    print(f'{k:32s} rel {rel:.3e} equal {eq * 100:7.3f} %  diag rel '
          f'{((o.diagonal() - r.diagonal()).norm() / r.diagonal().norm()).item() if o.dim() == 2 else 0:.3e}')
