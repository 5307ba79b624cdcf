"""Probe: one lcq_gemm_f32 shape (the GPTQ Cholesky recursion's products) launched `iters`
times, for rocprofv3 kernel-trace / PMC passes; prints TFLOP/s from HIP events.
usage: f32_gemm_one.py M N K bt [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import ops  # noqa: E402

M, N, K, bt = (int(v) for v in sys.argv[1:5])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dev = torch.device('cuda:0')
A = torch.randn(M, K, device=dev)
B = torch.randn(N, K, device=dev) if bt else torch.randn(K, N, device=dev)
C = torch.empty(M, N, device=dev)
ops.gemm_f32(A, B, C, 1.0, 0.0, b_trans=bool(bt))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    ops.gemm_f32(A, B, C, 1.0, 0.0, b_trans=bool(bt))
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
print(f'M{M} N{N} K{K} bt{bt}: {ms * 1e3:.1f} us  {2 * M * N * K / ms / 1e9:.1f} TF/s')
