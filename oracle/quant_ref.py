"""ORACLE (test infrastructure only) — grouped integer quantizer + packers, CPU restatement.

Follows llmc/compression/quantization/quant.py (IntegerQuantizer, min/max calibration) and
llmc/compression/quantization/module_utils.py (vLLM / AutoAWQ packers). Torch-CPU ops keep
the reference's dtype semantics exactly (bf16 ops round per op); numpy does the bit packing.
"""
from __future__ import annotations

import numpy as np
import torch


def int_range(bit: int, sym: bool, int_range=None):
    """quant.py:665-677 — qmin/qmax as 0-dim tensors (their dtypes drive type promotion:
    asym qmin is float32, everything else int64)."""
    if int_range is not None:
        qmin, qmax = int_range
    elif sym:
        qmin, qmax = -(2 ** (bit - 1)), 2 ** (bit - 1) - 1
    else:
        qmin, qmax = 0.0, 2 ** bit - 1
    return torch.tensor(qmin), torch.tensor(qmax)


def group_view(t: torch.Tensor, granularity: str, group: int | None = None) -> torch.Tensor:
    """quant.py:612-642 (reshape_tensor) for per_group / per_channel / per_tensor / per_token."""
    if granularity == 'per_group':
        if t.shape[-1] >= group:
            if t.shape[-1] % group:
                raise ValueError(f'Dimension {t.shape[-1]} not divisible by group size {group}')
            return t.reshape(-1, group)
        return t
    return t


def minmax(t: torch.Tensor, granularity: str = 'per_group'):
    """quant.py:132-143."""
    if granularity == 'per_tensor':
        return torch.min(t), torch.max(t)
    return t.amin(dim=-1, keepdim=True), t.amax(dim=-1, keepdim=True)


def qparams(mn, mx, qmin, qmax, sym: bool):
    """quant.py:545-559 (round_zp=True)."""
    if sym:
        am = torch.max(mx.abs(), mn.abs()).clamp(min=1e-5)
        return am / qmax, torch.tensor(0.0)
    s = (mx - mn).clamp(min=1e-5) / (qmax - qmin)
    z = (qmin - torch.round(mn / s)).clamp(qmin, qmax)
    return s, z


def quant(t, s, z, qmin, qmax):
    """quant.py:699-708 (round_zp=True, torch.round half-to-even)."""
    return torch.clamp(torch.round(t / s) + z, qmin, qmax)


def dequant(q, s, z):
    """quant.py:710-712."""
    return (q - z) * s


def _prescale_clip(w, pre_scale=None, clip_max=None, clip_min=None, group=None):
    if pre_scale is not None:  # awq.py:39-46 (w.mul_(scales.view(1, -1)))
        w = w * pre_scale.view(1, -1)
    if clip_max is not None:  # auto_clip.py:193-212 (apply_clip v1)
        shp = w.shape
        g = w.reshape(shp[0], -1, group)
        mx = clip_max.reshape(shp[0], -1, 1)
        mn = -mx if clip_min is None else clip_min.reshape(shp[0], -1, 1)
        w = torch.clamp(g, mn, mx).reshape(shp)
    return w


def fake_quant_dynamic(w, bit, sym, granularity='per_group', group=128, pre_scale=None,
                       clip_max=None, clip_min=None, int_rng=None):
    """quant.py:833-869 (+ get_tensor_qparams :690-697). Returns (w_fq, scales, zeros)."""
    qmin, qmax = int_range(bit, sym, int_rng)
    w = _prescale_clip(w, pre_scale, clip_max, clip_min, group)
    shape, dtype = w.shape, w.dtype
    t = group_view(w, granularity, group)
    mn, mx = minmax(t, granularity)
    s, z = qparams(mn, mx, qmin, qmax, sym)
    out = dequant(quant(t, s, z, qmin, qmax), s, z)
    return out.reshape(shape).to(dtype), s, z


def learnable_range(t, low, up, sym: bool):
    """quant.py:205-219 get_learnable_range (torch.nn.Sigmoid factors of the group range)."""
    mn, mx = minmax(t)
    if sym:
        if up is not None:
            am = torch.max(mx.abs(), mn.abs()).clamp(min=1e-5)
            am = torch.sigmoid(up) * am
            mn, mx = -am, am
    elif up is not None and low is not None:
        mn = torch.sigmoid(low) * mn
        mx = torch.sigmoid(up) * mx
    return mn, mx


def fake_quant_learnable(w, bit, sym, granularity='per_group', group=128, low=None, up=None):
    """fake_quant_weight_dynamic with calib_algo learnable and clip factors (quant.py:127-128,
    205-219, 833-869): the group ranges of get_learnable_range."""
    qmin, qmax = int_range(bit, sym)
    shape, dtype = w.shape, w.dtype
    t = group_view(w, granularity, group)
    mn, mx = learnable_range(t, low, up, sym)
    s, z = qparams(mn, mx, qmin, qmax, sym)
    return dequant(quant(t, s, z, qmin, qmax), s, z).reshape(shape).to(dtype)


def code_dtype(bit, qmin):
    """quant.py:890-896."""
    if bit == 8:
        return torch.int8 if qmin != 0 else torch.uint8
    return torch.int32


def real_quant_dynamic(w, bit, sym, granularity='per_group', group=128, int_rng=None):
    """quant.py:916-953. Returns (codes, scales [rows,-1], zeros [rows,-1] | None)."""
    qmin, qmax = int_range(bit, sym, int_rng)
    shape = w.shape
    t = group_view(w, granularity, group)
    mn, mx = minmax(t, granularity)
    s, z = qparams(mn, mx, qmin, qmax, sym)
    q = quant(t, s, z, qmin, qmax).reshape(shape)
    cd = code_dtype(bit, qmin)
    q = q.to(cd)
    z = z.to(cd) if not sym else None
    qshape = 1 if granularity == 'per_tensor' else (shape[0], -1)
    if z is not None:
        z = z.view(qshape)
    return q, s.view(qshape), z


def fake_quant_static(w, s, z, bit, sym, granularity='per_group', group=128, int_rng=None):
    """quant.py:785-831."""
    qmin, qmax = int_range(bit, sym, int_rng)
    shape, dtype = w.shape, w.dtype
    t = group_view(w, granularity, group)
    if z is None:
        z = torch.tensor(0.0)
    return dequant(quant(t, s, z, qmin, qmax), s, z).reshape(shape).to(dtype)


def real_quant_static(w, s, z, bit, sym, granularity='per_group', group=128, int_rng=None):
    """quant.py:871-914."""
    qmin, qmax = int_range(bit, sym, int_rng)
    shape = w.shape
    t = group_view(w, granularity, group)
    zz = torch.tensor(0.0) if z is None else z
    q = quant(t, s, zz, qmin, qmax).reshape(shape)
    cd = code_dtype(bit, qmin)
    q = q.to(cd)
    z = zz.to(cd) if not sym else None
    if z is not None:
        z = z.view(shape[0], -1)
    return q, s.view(shape[0], -1), z


def pack_vllm(codes: torch.Tensor, bits: int) -> np.ndarray:
    """module_utils.py:929-955 — little-endian pack of uint8(code + 2^(b-1)) into int32."""
    off = 2 ** bits // 2
    u = (codes.to(torch.int64) + off).numpy().astype(np.int64) & 0xFF
    u = u.astype(np.uint32)
    pf = 32 // bits
    pc = -(-u.shape[1] // pf)
    u = np.pad(u, [(0, 0), (0, pc * pf - u.shape[1])])
    out = np.zeros((u.shape[0], pc), dtype=np.uint32)
    for i in range(pf):
        out |= u[:, i::pf] << np.uint32(bits * i)
    return out.view(np.int32)


_AWQ_ORDER = [0, 2, 4, 6, 1, 3, 5, 7]


def gemm_pack_autoawq(w: torch.Tensor, scales: torch.Tensor, zeros: torch.Tensor, group: int,
                      bits: int = 4):
    """module_utils.py:1097-1158 (vectorised over columns; identical elementwise ops).

    Returns (qweight int32 [ic, oc/8], scales fp16 [ng, oc], qzeros int32 [ng, oc/8])."""
    assert bits == 4, 'Only 4-bit are supported for now.'
    s16 = scales.t().contiguous().to(torch.float16)   # [ng, oc]
    zt = zeros.t().contiguous()                         # [ng, oc] int
    sz = zt * s16                                       # int * fp16 -> fp16
    oc, ic = w.shape
    gidx = torch.arange(ic) // group
    # weight[:, idx] (bf16) + fp16 -> fp32 ; / fp16 -> fp32 ; round ; .to(int)
    iw = torch.round((w + sz[gidx].t()) / s16[gidx].t()).to(torch.int)
    iw = iw.t().contiguous().numpy().astype(np.int64) & 0xFFFFFFFF  # [ic, oc] raw bits
    iw = iw.astype(np.uint32)
    pn = 32 // bits
    qw = np.zeros((ic, oc // pn), dtype=np.uint32)
    for i in range(pn):
        qw |= iw[:, _AWQ_ORDER[i]::pn] << np.uint32(i * bits)
    z = (zt.to(torch.int32).numpy().astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)
    qz = np.zeros((z.shape[0], oc // pn), dtype=np.uint32)
    for i in range(pn):
        qz |= z[:, _AWQ_ORDER[i]::pn] << np.uint32(i * bits)
    return qw.view(np.int32), s16, qz.view(np.int32)


def mse_range(t: torch.Tensor, bit: int, sym: bool, maxshrink=0.8, grid=100, norm=2.4):
    """get_mse_range (quant.py:145-203) on a reshaped [groups, group] tensor: candidates
    p * (min, max) with p = 1 - i / grid, kept when sum |qdq(x) - x|^norm improves strictly.
    The reference's best_min_val / best_max_val alias the running min / max (slice views
    updated in place), so an accepted candidate becomes the base the later p's shrink.
    Returns fp32 (min, max) [groups, 1]."""
    qmin, qmax = int_range(bit, sym)
    x = t.float()
    mn, mx = x.amin(dim=-1, keepdim=True), x.amax(dim=-1, keepdim=True)
    best = torch.full([x.shape[0]], float('inf'))
    for i in range(int(maxshrink * grid)):
        p = 1 - i / grid
        lo, hi = p * mn, p * mx
        s, z = qparams(lo, hi, qmin, qmax, sym)
        err = (dequant(quant(x, s, z, qmin, qmax), s, z) - x).abs().pow(norm).sum(1)
        better = err < best
        best[better] = err[better]
        mn[better] = lo[better]
        mx[better] = hi[better]
    return mn, mx


def qparams_nozp(mn, mx, qmin, qmax, sym: bool):
    """quant.py:545-559 with round_zp False: zeros = qmin - min / scales (no round, no clamp)."""
    if sym:
        return qparams(mn, mx, qmin, qmax, sym)
    s = (mx - mn).clamp(min=1e-5) / (qmax - qmin)
    return s, qmin - (mn / s)


def quant_nozp(t, s, z, qmin, qmax):
    """quant.py:703-707 (round_zp False)."""
    return torch.clamp(torch.round(t / s.clamp_min(1e-9) + z), qmin, qmax)


def hqq_proximal(t: torch.Tensor, s, z, qmin, qmax, lp_norm=0.7, beta=10, iters=20):
    """optimize_weights_proximal (quant.py:588-610) on fp32 groups t [ng, gs]. shrink_op
    (quant.py:92-101) uses the quantizer's own beta (the lambda reads self.beta), so the
    kappa schedule never reaches it. The zeros of the stopping iteration are kept."""
    if lp_norm == 1:
        def shrink(x):
            return torch.sign(x) * torch.nn.functional.relu(torch.abs(x) - 1.0 / beta)
    else:
        def shrink(x):
            return torch.sign(x) * torch.nn.functional.relu(
                torch.abs(x) - (1.0 / beta) * torch.pow(torch.abs(x), lp_norm - 1))
    best = 1e4
    s = 1 / s
    for _ in range(iters):
        wq = torch.round(t * s + z).clamp(qmin, qmax)
        wr = (wq - z) / s
        we = shrink(t - wr)
        z = torch.mean(wq - (t - we) * s, axis=-1, keepdim=True)
        err = float(torch.abs(t - wr).mean())
        if err < best:
            best = err
        else:
            break
    return 1 / s, z


def hqq_qparams(w, bit, sym, granularity='per_group', group=128, round_zp=True, lp_norm=0.7,
                beta=10, iters=20):
    """get_hqq_qparams (quant.py:680-689): (fp32 groups, scales, zeros, qmin, qmax)."""
    qmin, qmax = int_range(bit, sym)
    t = group_view(w.float(), granularity, group)
    mn, mx = minmax(t, granularity)
    s, z = (qparams if round_zp else qparams_nozp)(mn, mx, qmin, qmax, sym)
    s, z = hqq_proximal(t, s, z, qmin, qmax, lp_norm, beta, iters)
    return t, s, z, qmin, qmax


def fake_quant_hqq(w, bit, sym, granularity='per_group', group=128, round_zp=True, **kw):
    """fake_quant_weight_dynamic with calib_algo hqq: quant_dequant of tensor.float()."""
    t, s, z, qmin, qmax = hqq_qparams(w, bit, sym, granularity, group, round_zp, **kw)
    q = quant(t, s, z, qmin, qmax) if round_zp else quant_nozp(t, s, z, qmin, qmax)
    return dequant(q, s, z).reshape(w.shape).to(w.dtype), s, z


def fake_quant_nozp(w, bit, sym, granularity='per_group', group=128):
    """fake_quant_weight_dynamic with calib_algo minmax and round_zp False (dtype of w)."""
    qmin, qmax = int_range(bit, sym)
    t = group_view(w, granularity, group)
    mn, mx = minmax(t, granularity)
    s, z = qparams_nozp(mn, mx, qmin, qmax, sym)
    return dequant(quant_nozp(t, s, z, qmin, qmax), s, z).reshape(w.shape).to(w.dtype), s, z
