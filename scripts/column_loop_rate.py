"""Probe: GPTQ's blocked column loop (gptq_core.column_loop) alone on the Llama-3-8B subset
shapes -- wall time (host included) vs the summed device time of its kernels, per superblock
size, with the near updates left-looking inside the block kernels or as one trailing launch
per block (round 6). (Round 4 also A/B'd a side-stream pipeline of the near-column updates here: slower,
removed; profiles/r4_column_loop.txt.)
usage: column_loop_rate.py"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import _native, gptq_core  # noqa: E402

dev = torch.device('cuda:0')
SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]


def make_u(n, g):
    # a well-conditioned upper factor: unit-ish diagonal, small upper part
    U = torch.triu(torch.randn(n, n, device=dev, generator=g) * (0.3 / n ** 0.5), 1)
    U += torch.diag(1.0 + torch.rand(n, device=dev, generator=g))
    return U.contiguous()


def run(rows, cols, sb, reps=3):
    g = torch.Generator(device=dev).manual_seed(rows + cols)
    W0 = torch.randn(rows, cols, device=dev, generator=g) * 0.02
    U = make_u(cols, g)
    out = None
    walls, dev_ms = [], []
    for r in range(reps + 1):
        W = W0.clone()
        torch.cuda.synchronize()
        timer = _native.KernelTimer()
        t0 = time.perf_counter()
        with timer:
            gptq_core.column_loop(W, U, 4, False, 128, 0, 15, superblock=sb)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        if r == 0:
            out = W
            continue
        if not torch.equal(out, W):
            print('  NOT REPEATABLE')
        k = timer.summary()
        walls.append(wall)
        dev_ms.append(sum(v['total_ms'] for v in k.values()))
    return min(walls), min(dev_ms), out


for rows, cols in SHAPES:
    for sb in (1024, 2048):
        res = {}
        for left in (False, True):
            gptq_core.LEFT_LOOKING = left
            wall, dms, W = run(rows, cols, sb)
            res[left] = W
            print(f'rows {rows:6d} cols {cols:6d} sb {sb:5d} {"left-looking" if left else "trailing    "}'
                  f': wall {wall:7.2f} ms  device sum {dms:7.2f} ms', flush=True)
        print(f'  identical: {torch.equal(res[False], res[True])}', flush=True)
gptq_core.LEFT_LOOKING = True
