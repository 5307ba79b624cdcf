"""GPTQ Hessian (lcq_hessian_accum) rate: the 4-wave k_syrk16 (default) vs the 8-wave
k_syrk256 (LCQ_SYRK=256), interleaved rounds in one process, random bf16 activations at the
GPTQ calibration size (128 x 2048 tokens). Flops = n * ic * (ic + 1) (the upper triangle).

usage: python scripts/hessian_rate.py [--n 262144] [--ics 4096,14336] [--rounds 3]
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
ap.add_argument('--n', type=int, default=262144)
ap.add_argument('--ics', default='4096,14336')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--iters', type=int, default=3)
a = ap.parse_args()
g = torch.Generator(device='cuda').manual_seed(0)
for ic in map(int, a.ics.split(',')):
    x = torch.randn(a.n, ic, generator=g, device='cuda').to(torch.bfloat16)
    H = torch.zeros(ic, ic, device='cuda')
    res = {'16': [], '256': []}

    def run(v):
        if v == '16':
            os.environ.pop('LCQ_SYRK', None)
        else:
            os.environ['LCQ_SYRK'] = v
        ops.hessian_accum(x, H, 1.0, 0.0)

    for v in res:
        run(v)
    ref = H.clone()
    run('16')
    diff = (H - ref).abs().max().item()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for v in res:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run(v)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.iters)
    fl = a.n * ic * (ic + 1)
    for v, ts in res.items():
        t = statistics.median(ts)
        print(f'ic {ic} n {a.n} syrk{v}: {t:8.3f} ms {fl / t / 1e9:8.1f} TFLOP/s '
              f'(incl. the X^T pack); max |H16 - H256| {diff:.3e}')
    del x, H, ref
    torch.cuda.empty_cache()
