"""Probe: one lcq_fp8_gemm shape launched `iters` times (for rocprofv3 kernel-trace / PMC
passes). usage: fp8_gemm_one.py M N K [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import kernel, ops  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
dev = torch.device('cuda:0')
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
a, a_s = kernel.act_quant(x)
b, b_s = kernel.weight_cast_to_fp8(w)
for _ in range(iters):
    ops.fp8_gemm(a, a_s, b, b_s, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
print('done', M, N, K, iters)
