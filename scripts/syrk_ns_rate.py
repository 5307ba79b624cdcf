"""lcq_hessian_accum at the GPTQ shapes for forced split-K counts (LCQ_SYRK_NS) vs the
cost-model default (plan() in csrc/hessian256.hip); interleaved rounds in one process, random
bf16 activations, 128 x 2048 tokens. Flops = n * ic * (ic + 1) (upper triangle).

usage: python scripts/syrk_ns_rate.py [--rounds 3]
"""
import argparse
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--rounds', type=int, default=3)
a = ap.parse_args()
n = 262144
for ic, nss in ((4096, (0, 8, 16, 24)), (14336, (0, 1, 2)), (8192, (0, 1, 4))):
    x = (torch.randn(n, ic, device='cuda') * 0.5).to(torch.bfloat16)
    H = torch.zeros(ic, ic, device='cuda')
    res = {ns: [] for ns in nss}
    outs = {}
    for r in range(a.rounds):
        for ns in nss:
            if ns:
                os.environ['LCQ_SYRK_NS'] = str(ns)
            else:
                os.environ.pop('LCQ_SYRK_NS', None)
            ops.hessian_accum(x, H, 1.0, 0.0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                ops.hessian_accum(x, H, 1.0, 0.0)
            e1.record()
            torch.cuda.synchronize()
            res[ns].append(e0.elapsed_time(e1) / 3)
            if r == 0:
                outs[ns] = H.clone()
    os.environ.pop('LCQ_SYRK_NS', None)
    fl = n * ic * (ic + 1)
    ref = outs[nss[0]]
    for ns in nss:
        ms = statistics.median(res[ns])
        d = (outs[ns] - ref).abs().max().item() / ref.abs().max().item()
        print(f'ic {ic} ns {ns or "auto"}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s  '
              f'rel max diff vs auto {d:.2e}', flush=True)
    del x, H, outs
    torch.cuda.empty_cache()
