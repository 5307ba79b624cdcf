"""Probe: wall time of one inverse_cholesky_upper chain (gptq_core: recursion on lcq_gemm_f32
+ lcq_chol_inv_tile) at the Llama-3-8B Hessian sizes, eager without / with the side-stream
overlap of T = L21 X11 (gptq_core._OVERLAP_MIN), and replayed as a captured HIP graph;
large products on the split-plane bf16 kernel (ops.X6, lcq_gemm_f32x6) or on fp32 MFMA."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import gptq_core, ops  # noqa: E402

dev = torch.device('cuda:0')
for n in (4096, 14336):
    g = torch.Generator(device=dev).manual_seed(n)
    X = torch.randn(n, 2 * n, device=dev, generator=g)
    H = X @ X.T / (2 * n)
    H.diagonal().add_(0.01)
    for ov, graph, sk, x6 in ((10 ** 9, False, True, True), (1024, False, True, True),
                              (1024, True, True, True), (1024, True, False, True),
                              (1024, False, True, False), (1024, True, True, False)):
        ops.X6 = x6
        gptq_core._OVERLAP_MIN = ov
        gptq_core.CHAIN_GRAPHS = graph
        ops.STREAM_K = sk
        gptq_core.clear_chain_graphs()
        U0 = gptq_core.inverse_cholesky_upper(H.clone())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record()
        for _ in range(reps):
            U = gptq_core.inverse_cholesky_upper(H.clone())
        e1.record()
        torch.cuda.synchronize()
        print(f'n {n} overlap_min {ov} graph {graph} stream_k {sk} x6 {x6}: '
              f'{e0.elapsed_time(e1) / reps:.2f} ms per chain '
              f'(incl. one H copy); identical to the first run: {torch.equal(U, U0)}', flush=True)
    print(flush=True)
