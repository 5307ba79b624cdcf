"""Probe: lcq_fp8_gemm TFLOP/s at calibration-forward shapes vs the bf16 round trip the
reference falls back to (weight_cast_to_bf16 + F.linear) and torch bf16 matmul."""
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import kernel, ops  # noqa: E402

dev = torch.device('cuda:0')
shapes = [(512, 7168, 2048), (512, 2048, 7168), (2048, 2048, 7168), (2048, 7168, 2048),
          (2048, 7168, 7168), (4096, 4096, 4096), (8192, 8192, 8192)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it


for M, N, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    a, a_s = kernel.act_quant(x)
    b, b_s = kernel.weight_cast_to_fp8(w)
    fl = 2.0 * M * N * K
    t_g = timeit(lambda: ops.fp8_gemm(a, a_s, b, b_s, out_dtype=torch.bfloat16))
    t_bf = timeit(lambda: F.linear(x, w))
    t_rt = timeit(lambda: F.linear(x, kernel.weight_cast_to_bf16(b, b_s).to(torch.bfloat16)))
    print(f'M{M} N{N} K{K}: fp8_gemm {t_g*1e6:8.1f} us {fl/t_g/1e12:7.1f} TF/s | '
          f'bf16 linear {t_bf*1e6:8.1f} us {fl/t_bf/1e12:7.1f} TF/s | '
          f'cast+linear {t_rt*1e6:8.1f} us', flush=True)
