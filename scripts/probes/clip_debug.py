import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'tests' / 'golden'))
import torch
import fixtures as F
from lightcompress_amd import ops
from lightcompress_amd.auto_clip import AutoClipper
c = F.load('clip_sym_s')
dev = torch.device('cuda:0')
x = AutoClipper.sample_tokens(c['x'].to(dev), 64)
bmax, bmin = ops.auto_clip_search(c['w'].to(dev), x, 128, 10, 20, -8, 7, True, True)
got = bmax.cpu().float().squeeze(-1)
ref = c['best_max'].float().squeeze(-1)
orgmax = c['w'].float().reshape(128, 2, 128).abs().amax(-1)
print('shape', got.shape)
mis = (got != ref)
print('mismatch per row parity', mis[0::2].float().mean().item(), mis[1::2].float().mean().item())
print('mismatch per group', mis.float().mean(0))
print('ratio got/orgmax (first rows)', (got / orgmax)[:8])
print('ratio ref/orgmax (first rows)', (ref / orgmax)[:8])
