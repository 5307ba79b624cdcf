"""Probe: chain wall time vs ops.X6_MIN_TILES (the split-plane product threshold), eager and graph."""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import gptq_core, ops
dev = torch.device('cuda:0')
for n in (4096, 14336):
    g = torch.Generator(device=dev).manual_seed(n)
    X = torch.randn(n, 2 * n, device=dev, generator=g)
    H = X @ X.T / (2 * n)
    H.diagonal().add_(0.01)
    del X
    for rnd in range(2):
        for thr in (40, 16, 8):
            ops.X6_MIN_TILES = thr
            for graph in (False, True):
                gptq_core.CHAIN_GRAPHS = graph
                gptq_core.clear_chain_graphs()
                gptq_core.inverse_cholesky_upper(H.clone())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    gptq_core.inverse_cholesky_upper(H.clone())
                e1.record()
                torch.cuda.synchronize()
                print(f'n {n} thr {thr} graph {graph}: {e0.elapsed_time(e1) / 3:.2f} ms', flush=True)
