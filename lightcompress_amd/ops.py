"""Torch-tensor front end of the lcq C ABI.

Each function validates shapes/dtypes on the host, allocates outputs with torch (device
memory is torch's caching allocator), and launches the HIP kernel on torch's current stream
through ``_native``. There is no CPU path: CPU tensors raise ``LcqError``.
"""
from __future__ import annotations

import torch

from . import _native as N

__all__ = ['int_quant_dynamic', 'int_quant_static', 'pack_vllm', 'pack_autoawq_gemm',
           'hessian_accum', 'gptq_block']


def _code_dtype(bit: int, qmin: int) -> torch.dtype:
    # quant.py:890-896 / 929-935
    if bit == 8:
        return torch.int8 if qmin != 0 else torch.uint8
    return torch.int32


def int_quant_dynamic(x: torch.Tensor, group: int, qmin: int, qmax: int, sym: bool, *,
                      pre_scale: torch.Tensor | None = None,
                      clip_max: torch.Tensor | None = None,
                      clip_min: torch.Tensor | None = None,
                      fq: bool = True, fq_dtype: torch.dtype | None = None,
                      codes_dtype: torch.dtype | None = None,
                      pack_bits: int | None = None,
                      qparams: bool = True,
                      out: torch.Tensor | None = None) -> dict:
    """Grouped min/max quantization of a 2-D tensor ``x`` [rows, cols] (groups along cols).

    Returns a dict with any of ``fq`` (fake-quant, ``fq_dtype``), ``codes``, ``packed``
    (vLLM int32), ``scales``/``zeros`` ([rows*cols/group, 1] in x.dtype).
    """
    assert x.dim() == 2, 'x must be 2-D'
    rows, cols = x.shape
    group = cols if group in (0, None) else int(group)
    ng = rows * cols // group
    res = {}
    fq_t = None
    if fq:
        fq_dtype = fq_dtype or x.dtype
        fq_t = out if out is not None else torch.empty((rows, cols), dtype=fq_dtype, device=x.device)
        res['fq'] = fq_t
    codes_t = None
    if codes_dtype is not None:
        codes_t = torch.empty((rows, cols), dtype=codes_dtype, device=x.device)
        res['codes'] = codes_t
    packed_t = None
    if pack_bits:
        pf = 32 // pack_bits
        packed_t = torch.empty((rows, (cols + pf - 1) // pf), dtype=torch.int32, device=x.device)
        res['packed'] = packed_t
    s_t = z_t = None
    if qparams:
        s_t = torch.empty((ng, 1), dtype=x.dtype, device=x.device)
        res['scales'] = s_t
        if not sym:
            z_t = torch.empty((ng, 1), dtype=x.dtype, device=x.device)
            res['zeros'] = z_t
    for t in (pre_scale, clip_max, clip_min):
        if t is not None and t.dtype != x.dtype:
            raise ValueError('pre_scale / clip bounds must have the weight dtype')
    N.call('lcq_int_quant_dynamic', N.ptr(x), N.dt(x), rows, cols, group,
           N.ptr(pre_scale), N.ptr(clip_max), N.ptr(clip_min), int(qmin), int(qmax), int(sym),
           N.ptr(fq_t), N.dt(fq_dtype) if fq else 0,
           N.ptr(codes_t), N.dt(codes_dtype) if codes_t is not None else 0,
           N.ptr(packed_t), int(pack_bits or 0), N.ptr(s_t), N.ptr(z_t), N.stream_of(x))
    return res


def int_quant_static(x: torch.Tensor, group: int, scales: torch.Tensor,
                     zeros: torch.Tensor | None, qmin: int, qmax: int, *,
                     ct_dtype: torch.dtype, fq: bool = True,
                     fq_dtype: torch.dtype | None = None,
                     codes_dtype: torch.dtype | None = None,
                     pack_bits: int | None = None) -> dict:
    """Quantize ``x`` [rows, cols] with given per-group scales/zeros (flat group order)."""
    assert x.dim() == 2
    rows, cols = x.shape
    group = cols if group in (0, None) else int(group)
    ng = rows * cols // group
    scales = scales.contiguous()
    if scales.numel() != ng:
        raise ValueError(f'scales has {scales.numel()} elements, expected {ng}')
    if zeros is not None:
        zeros = zeros.contiguous()
        if zeros.numel() != ng:
            raise ValueError(f'zeros has {zeros.numel()} elements, expected {ng}')
    res = {}
    fq_t = codes_t = packed_t = None
    if fq:
        fq_dtype = fq_dtype or ct_dtype
        fq_t = torch.empty((rows, cols), dtype=fq_dtype, device=x.device)
        res['fq'] = fq_t
    if codes_dtype is not None:
        codes_t = torch.empty((rows, cols), dtype=codes_dtype, device=x.device)
        res['codes'] = codes_t
    if pack_bits:
        pf = 32 // pack_bits
        packed_t = torch.empty((rows, (cols + pf - 1) // pf), dtype=torch.int32, device=x.device)
        res['packed'] = packed_t
    N.call('lcq_int_quant_static', N.ptr(x), N.dt(x), rows, cols, group,
           N.ptr(scales), N.dt(scales), N.ptr(zeros), N.dt(zeros) if zeros is not None else 0,
           N.dt(ct_dtype), int(qmin), int(qmax),
           N.ptr(fq_t), N.dt(fq_dtype) if fq else 0,
           N.ptr(codes_t), N.dt(codes_dtype) if codes_t is not None else 0,
           N.ptr(packed_t), int(pack_bits or 0), N.stream_of(x))
    return res


def pack_vllm(codes: torch.Tensor, bits: int) -> torch.Tensor:
    """VllmRealQuantLinear.pack bit layout (module_utils.py:929-955) on device."""
    assert codes.dim() == 2
    rows, cols = codes.shape
    pf = 32 // bits
    out = torch.empty((rows, (cols + pf - 1) // pf), dtype=torch.int32, device=codes.device)
    N.call('lcq_pack_vllm', N.ptr(codes), N.dt(codes), rows, cols, int(bits), N.ptr(out),
           N.stream_of(codes))
    return out


def pack_autoawq_gemm(weight: torch.Tensor, scales: torch.Tensor, zeros: torch.Tensor,
                      group: int, bits: int = 4):
    """AutoawqRealQuantLinear.gemm_pack (module_utils.py:1097-1158) on device.

    weight [oc, ic], scales [oc, ic/group], zeros [oc, ic/group] int32.
    Returns (qweight int32 [ic, oc/8], scales fp16 [ic/group, oc], qzeros int32 [ic/group, oc/8]).
    """
    oc, ic = weight.shape
    ng = ic // group
    zeros = zeros.to(torch.int32).contiguous()
    scales = scales.contiguous()
    qweight = torch.empty((ic, oc * bits // 32), dtype=torch.int32, device=weight.device)
    scales_t = torch.empty((ng, oc), dtype=torch.float16, device=weight.device)
    qzeros = torch.empty((ng, oc * bits // 32), dtype=torch.int32, device=weight.device)
    N.call('lcq_pack_autoawq_gemm', N.ptr(weight), N.dt(weight), oc, ic, int(group),
           N.ptr(scales), N.dt(scales), N.ptr(zeros), int(bits), N.ptr(qweight),
           N.ptr(scales_t), N.ptr(qzeros), N.stream_of(weight))
    return qweight, scales_t, qzeros


def hessian_accum(x: torch.Tensor, H: torch.Tensor, alpha: float, beta: float) -> torch.Tensor:
    """H <- beta*H + alpha * x^T x (in place); x [n, ic] bf16/fp16, H [ic, ic] fp32."""
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    n, ic = x2.shape
    if H.dtype != torch.float32 or tuple(H.shape) != (ic, ic):
        raise ValueError('H must be fp32 [ic, ic]')
    N.call('lcq_hessian_accum', N.ptr(x2), N.dt(x2), n, ic, N.ptr(H), float(alpha),
           float(beta), N.stream_of(x2))
    return H


def gptq_block(W: torch.Tensor, col0: int, count: int, U: torch.Tensor, group: int,
               qmin: int, qmax: int, sym: bool, s_out, z_out, err: torch.Tensor,
               losses=None, s_in=None, z_in=None):
    """One 128-column GPTQ block in place on fp32 W (see include/lcq.h lcq_gptq_block)."""
    rows, ld = W.shape
    ng_total = s_out.shape[1] if s_out is not None else 0
    N.call('lcq_gptq_block', N.ptr(W), rows, ld, int(col0), int(count), N.ptr(U), U.shape[1],
           int(group), int(qmin), int(qmax), int(sym), N.ptr(s_in), N.ptr(z_in), N.ptr(s_out),
           N.ptr(z_out), int(ng_total), N.ptr(err), N.ptr(losses), N.stream_of(W))


code_dtype = _code_dtype
