"""Probe: lcq_fp8_gemm TFLOP/s at calibration-forward shapes for every tile plan (auto, the
<= 64-row kernel, 128^2 and 256^2 with their split-K; lcq_fp8_gemm_force_plan) against the
bf16 round trip the reference falls back to (weight_cast_to_bf16 + F.linear) and torch bf16
matmul (hipBLASLt). HIP-event timing over 20 launches after 3 warm-ups."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import _native as N  # noqa: E402
from lightcompress_amd import kernel, ops  # noqa: E402

dev = torch.device('cuda:0')
shapes = [(512, 7168, 2048), (512, 2048, 7168), (2048, 2048, 7168), (2048, 7168, 2048),
          (2048, 7168, 7168), (4096, 4096, 4096), (8192, 8192, 8192)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e-3


lib = N.load()
for M, Nn, K in shapes:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(Nn, K, device=dev, dtype=torch.bfloat16) * 0.05
    a, a_s = kernel.act_quant(x)
    b, b_s = kernel.weight_cast_to_fp8(w)
    fl = 2.0 * M * Nn * K
    parts = []
    for plan in (0, 1, 128, 256):
        lib.lcq_fp8_gemm_force_plan(plan)
        t = timeit(lambda: ops.fp8_gemm(a, a_s, b, b_s, out_dtype=torch.bfloat16))
        parts.append(f'{["auto", "64row", "128^2", "256^2"][(0, 1, 128, 256).index(plan)]} '
                     f'{t * 1e6:6.1f} us {fl / t / 1e12:6.1f} TF/s')
    lib.lcq_fp8_gemm_force_plan(0)
    t_bf = timeit(lambda: F.linear(x, w))
    t_rt = timeit(lambda: F.linear(x, kernel.weight_cast_to_bf16(b, b_s).to(torch.bfloat16)))
    print(f'M{M} N{Nn} K{K}: ' + ' | '.join(parts) +
          f' || bf16 linear {t_bf * 1e6:6.1f} us {fl / t_bf / 1e12:6.1f} TF/s | '
          f'cast+linear {t_rt * 1e6:6.1f} us', flush=True)
