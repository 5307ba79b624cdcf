"""ORACLE (test infrastructure only) — FP8 FloatQuantizer + block-fp8 casts, CPU restatement.

Follows llmc/compression/quantization/quant.py (FloatQuantizer :963-1229, weight_cast_* :18-43)
and llmc/compression/quantization/kernel.py (Triton act_quant / weight_cast_* :7-138) with
torch-CPU ops, keeping the reference's dtype promotion. Pinning (tests/golden, gen_fp8):
* use_qtorch=False (get_float_qparams emulation): the reference itself ran here -> pinned.
* use_qtorch=True: the scales / minmax / dequant / per_block layout are the reference's own
  methods -> pinned; the value rounding is qtorch.float_quantize, which is absent from this
  image -> the restatement uses torch's native cast (c10 RNE) there: parity UNPINNED for that
  one step.
* kernel.py: Triton cannot run without a GPU -> restated from source, unpinned.
* fp8_gemm (kernel.py:141-214): restated from source, parity unpinned (no Triton here); the
  restatement is itself checked against an exact float64 dequantized matmul
  (tests/test_oracle_fp8.py).
"""
from __future__ import annotations

import torch

FP8 = {'e4m3': torch.float8_e4m3fn, 'e5m2': torch.float8_e5m2}


def qmax_of(bit: str) -> torch.Tensor:
    """quant.py:982-996 (use_qtorch): finfo(fp8).max as a 0-dim fp32 tensor."""
    return torch.tensor(torch.finfo(FP8[bit]).max)


def group_view(t: torch.Tensor, granularity: str, group: int | None = None, block: int = 128):
    """quant.py:612-642."""
    if granularity == 'per_group':
        return t.reshape(-1, group)
    if granularity == 'per_block':
        m, n = t.shape
        pm, pn = -(-m // block) * block, -(-n // block) * block
        p = torch.zeros((pm, pn), dtype=t.dtype)
        p[:m, :n] = t
        return p.view(-1, block, pn // block, block)
    return t


def minmax(t: torch.Tensor, granularity: str):
    """quant.py:132-143."""
    if granularity == 'per_tensor':
        return torch.min(t), torch.max(t)
    if granularity == 'per_block':
        return (t.abs().float().amin(dim=(1, 3), keepdim=True),
                t.abs().float().amax(dim=(1, 3), keepdim=True))
    return t.amin(dim=-1, keepdim=True), t.amax(dim=-1, keepdim=True)


def sym_scales(mn, mx, qmax):
    """quant.py:545-553 (sym): clamp(max(|max|, |min|), 1e-5) / qmax."""
    return torch.max(mx.abs(), mn.abs()).clamp(min=1e-5) / qmax


def float_quantize(x: torch.Tensor, bit: str) -> torch.Tensor:
    """The stand-in for qtorch's float_quantize(x, e, m, 'nearest') (absent from this image):
    saturate at +-finfo.max (NaN kept), then the native OCP RNE cast, as fp32. Equal to the
    plain cast wherever |x| < the format's overflow band, which every dynamic scale guarantees;
    differs only for static scales. Pins: tests/golden clipfp8_ / gptqfp8_ /
    pipe_*fp8 were made by the reference with this very function as its float_quantize."""
    dt = FP8[bit]
    m = torch.finfo(dt).max
    x = x.float()
    return torch.where(x.isnan(), x, x.clamp(-m, m)).to(dt).float()


def qdq_given(x: torch.Tensor, s: torch.Tensor, bit: str) -> torch.Tensor:
    """FloatQuantizer(use_qtorch).quant_dequant with given scales and zeros = 0.0
    (quant.py:1061-1080): float_quantize(x / s + 0) then (q - 0) * s, torch dtype promotion."""
    s = s.clone()
    s[s == 0] = 1
    zeros = torch.tensor(0.0)
    return (float_quantize(x / s + zeros, bit) - zeros) * s


def fp8_qdq(x: torch.Tensor, bit: str, granularity: str, group: int | None = None,
            block: int = 128):
    """FloatQuantizer(use_qtorch=True) fake + real quant, native cast for float_quantize.

    Returns (fake-quant in x.dtype, fp8 codes [x.shape], scales as real_quant returns them)."""
    fp8 = FP8[bit]
    qmax = qmax_of(bit)
    t = group_view(x, granularity, group, block)
    mn, mx = minmax(t, granularity)
    s = sym_scales(mn, mx, qmax)
    zeros = torch.tensor(0.0)
    s = s.clone()
    s[s == 0] = 1
    scaled = t / s + zeros                                  # quant.py:1063
    q = scaled.float().to(fp8).float()                      # float_quantize -> native cast
    dq = (q - zeros) * s                                    # quant.py:1078-1080

    def restore(v):
        if granularity == 'per_block':
            m, n = x.shape
            pn = v.shape[2] * v.shape[3]
            return v.reshape(-1, pn)[:m, :n]
        return v.reshape(x.shape)

    fq = restore(dq).to(x.dtype)
    codes = restore(q).to(fp8)
    if granularity == 'per_tensor':
        rs = s.view(1)
    elif granularity == 'per_block':
        rs = s.view(s.shape[0], s.shape[2])
    else:
        rs = s.view(x.shape[0], -1)
    return fq, codes, rs


def emul_fake_quant(x: torch.Tensor, e_bits: int, m_bits: int, granularity: str,
                    group: int | None = None) -> torch.Tensor:
    """FloatQuantizer(use_qtorch=False).fake_quant_*_dynamic: get_float_qparams
    (quant.py:1005-1027) + quant/dequant (:1061-1080) + restore/.to(dtype)."""
    t = group_view(x, granularity, group)
    mn, mx = minmax(t, granularity)
    maxval = torch.max(mx, -mn)
    e = torch.tensor(e_bits, dtype=torch.float32)
    m = torch.tensor(m_bits, dtype=torch.float32)
    if e >= 5:
        maxval = maxval.to(dtype=torch.float32)
    bias = 2 ** e - torch.log2(maxval) + torch.log2(2 - 2 ** (-m)) - 1
    xc = torch.min(torch.max(t, -maxval), maxval)
    log_scales = torch.clamp(torch.floor(torch.log2(torch.abs(xc)) + bias), 1.0)
    scales = 2.0 ** (log_scales - m - bias)
    zeros = torch.tensor(0)
    scales[scales == 0] = 1
    q = torch.round(xc / scales + zeros)
    return ((q - zeros) * scales).reshape(x.shape).to(x.dtype)


# ---- kernel.py (Triton) restated -------------------------------------------------------------
def act_quant(x: torch.Tensor, block: int = 128):
    """kernel.py:7-54."""
    v = x.reshape(-1, block).float()
    s = v.abs().amax(dim=-1, keepdim=True) / 448.0
    y = (v / s).to(torch.float8_e4m3fn)
    return y.reshape(x.shape), s.reshape(*x.shape[:-1], x.shape[-1] // block)


def weight_cast_to_fp8(x: torch.Tensor, block: int = 128):
    """kernel.py:57-81 (masked tiles: padding does not enter the max)."""
    M, N = x.shape
    nb_m, nb_n = -(-M // block), -(-N // block)
    y = torch.empty((M, N), dtype=torch.float8_e4m3fn)
    s = torch.empty((nb_m, nb_n), dtype=torch.float32)
    xf = x.float()
    for i in range(nb_m):
        for j in range(nb_n):
            tile = xf[i * block:(i + 1) * block, j * block:(j + 1) * block]
            sc = tile.abs().max() / 448.0
            s[i, j] = sc
            y[i * block:(i + 1) * block, j * block:(j + 1) * block] = \
                (tile / sc).to(torch.float8_e4m3fn)
    return y, s


def weight_cast_to_bf16(y: torch.Tensor, s: torch.Tensor, block: int = 128,
                        out_dtype=torch.bfloat16):
    """kernel.py:84-138 / quant.py:18-31: float(y) * s[block] in fp32, then out dtype."""
    M, N = y.shape
    se = s.repeat_interleave(block, 0).repeat_interleave(block, 1)[:M, :N]
    return (y.float() * se).to(out_dtype)


def fp8_gemm(a: torch.Tensor, a_s: torch.Tensor, b: torch.Tensor, b_s: torch.Tensor):
    """kernel.py:141-214 (fp8_gemm_kernel): per 128-wide K block kb,
    acc += (dot(a[:, kb], b[:, kb]^T) * a_s[:, kb, None]) * b_s[n / 128, kb]; fp32 result.
    The block dot is formed in float64 and rounded once to fp32 (the exact sum the MFMA's fp32
    accumulation approximates), then scaled and accumulated in fp32 in the kernel's order."""
    K = a.shape[-1]
    M = a.numel() // K
    Nn = b.shape[0]
    af = a.reshape(M, K).double()
    bf = b.double()
    asf = a_s.reshape(M, K // 128).float()
    bse = b_s.float().repeat_interleave(128, 0)[:Nn]
    acc = torch.zeros(M, Nn, dtype=torch.float32)
    for kb in range(K // 128):
        d = (af[:, kb * 128:(kb + 1) * 128] @ bf[:, kb * 128:(kb + 1) * 128].T).float()
        acc = acc + (d * asf[:, kb:kb + 1]) * bse[:, kb][None, :]
    return acc.reshape(*a.shape[:-1], Nn)
