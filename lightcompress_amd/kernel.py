"""Block-FP8 casts and activation quant (drop-in for ``llmc/compression/quantization/kernel.py``).

The reference implements these as Triton kernels and picks them on FP8-capable GPUs
(``base_blockwise_quantization.py:20-26``); here they are the lcq HIP kernels:

* ``act_quant`` (kernel.py:7-54): per 128 contiguous elements, s = max|x| / 448 (fp32, no
  clamp), y = cast_e4m3(x / s);
* ``weight_cast_to_fp8`` (kernel.py:57-81): per 128x128 block, same rule, fp32 scales
  ``[ceil(M/128), ceil(N/128)]``;
* ``weight_cast_to_bf16`` (kernel.py:84-138): y = float(w) * s[block], stored in
  ``torch.get_default_dtype()`` like the reference (callers then ``.to(torch.bfloat16)``);
* ``fp8_gemm`` (kernel.py:141-242): block-scaled e4m3 GEMM, per 128-wide K block
  ``acc += (dot(a, b) * a_s) * b_s`` in fp32 on the fp8 MFMA (csrc/fp8_gemm.hip).

Triton's fp32 ``/`` may be approximate on the reference's hardware; this build divides with
IEEE round-to-nearest (the torch-CPU result), and casts with c10's RNE rule.
"""
from __future__ import annotations

import torch

from . import ops


def act_quant(x: torch.Tensor, block_size: int = 128):
    assert x.is_contiguous(), 'Input tensor must be contiguous'
    assert x.size(-1) % block_size == 0, (
        f'Last dimension size must be divisible by block_size (block_size={block_size})')
    r = ops.fp8_quant(x.reshape(-1, block_size), block_size, torch.float8_e4m3fn,
                      ct_dtype=torch.float32, qmax=448.0, clamp_min=0.0, add_zero=False)
    y = r['codes'].reshape(x.shape)
    s = r['scales'].reshape(*x.shape[:-1], x.shape[-1] // block_size)
    return y, s


def weight_cast_to_fp8(x: torch.Tensor, block_size: int = 128):
    assert x.is_contiguous()
    assert x.dim() == 2
    r = ops.fp8_quant_blocks(x, torch.float8_e4m3fn, block_size, qmax=448.0, clamp_min=0.0,
                             add_zero=False)
    return r['codes'], r['scales']


def weight_cast_to_bf16(x: torch.Tensor, s: torch.Tensor, block_size: int = 128):
    assert x.is_contiguous() and s.is_contiguous(), 'Input tensors must be contiguous'
    assert x.dim() == 2 and s.dim() == 2, 'Input tensors must have 2 dimensions'
    return ops.fp8_dequant_blocks(x, s, block_size, out_dtype=torch.get_default_dtype())


def fp8_gemm(a: torch.Tensor, a_s: torch.Tensor, b: torch.Tensor, b_s: torch.Tensor):
    return ops.fp8_gemm(a, a_s, b, b_s)
