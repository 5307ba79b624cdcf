"""Probe: GPTQ's blocked column loop (gptq_core.column_loop) eager vs captured once into a HIP
graph and replayed (static W / U buffers), on the Llama-3-8B subset shapes -- how much of the
loop's time is host issue (the ~11 us gaps between block and trailing kernels of
profiles/r5_gptq_block_gaps.txt). Also checks that the replay's W equals the eager W bit for
bit. Not a product path.
usage: column_loop_graph_probe.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import gptq_core  # noqa: E402

dev = torch.device('cuda:0')
SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]


def make_u(n, g):
    U = torch.triu(torch.randn(n, n, device=dev, generator=g) * (0.3 / n ** 0.5), 1)
    U += torch.diag(1.0 + torch.rand(n, device=dev, generator=g))
    return U.contiguous()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for rows, cols in SHAPES:
    g = torch.Generator(device=dev).manual_seed(rows + cols)
    W0 = torch.randn(rows, cols, device=dev, generator=g) * 0.02
    U = make_u(cols, g)
    W = W0.clone()

    def eager():
        W.copy_(W0)
        gptq_core.column_loop(W, U, 4, False, 128, 0, 15)

    t_eager = timed(eager)
    W_eager = W.clone()
    Ws = W0.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):   # warm-up on a side stream before capture
        Ws.copy_(W0)
        gptq_core.column_loop(Ws, U, 4, False, 128, 0, 15)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        Ws.copy_(W0)
        gptq_core.column_loop(Ws, U, 4, False, 128, 0, 15)
    t_graph = timed(graph.replay)
    print(f'rows {rows:5d} cols {cols:5d}: eager {t_eager:7.2f} ms | graph replay {t_graph:7.2f} ms'
          f' | W identical {torch.equal(Ws, W_eager)}', flush=True)
    del graph
