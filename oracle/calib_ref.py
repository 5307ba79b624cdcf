"""ORACLE (test infrastructure only) — static per-tensor activation calibration, CPU restatement.

Follows llmc/compression/quantization/quant.py in torch-CPU, op for op:
reshape_batch_tensors (:103-120), get_minmax_stats (:221-251) over per_tensor ranges
(:132-135), get_static_minmax_range (:253-262: mean of the per-entry fp32 min / max),
get_static_moving_minmax_range (:431-450: EMA in the activation dtype), get_qparams
(:545-559, torch's 0-dim type promotion decides every dtype), fake_quant_act_static (:719-743
-> quant_dequant :699-717). Pinned bit-exact by tests/test_oracle_calib.py against
tests/golden/actstatic_*.npz (generated from the reference by gen_golden.py act_static).
"""
from __future__ import annotations

import torch


def batch_entries(act_tensors):
    """quant.py:103-120 (non-mutating): per module input, the list of calibration segments."""
    assert len(act_tensors) > 0
    if len(act_tensors) == 1:
        return [[act_tensors[0][i] for i in range(act_tensors[0].size(0))]]
    return [list(act_tensors)]


def static_range(tensors, algo: str, alpha: float = 0.01):
    """(min, max) 0-dim tensors of one module input."""
    if algo == 'static_minmax':
        mins = torch.tensor([torch.min(t).item() for t in tensors], dtype=torch.float32)
        maxs = torch.tensor([torch.max(t).item() for t in tensors], dtype=torch.float32)
        # torch.tensor([min_val]) of a 0-dim tensor keeps its value exactly (bf16/f16 -> fp32)
        return mins.mean(), maxs.mean()
    if algo == 'static_moving_minmax':
        mn = mx = None
        for t in tensors:
            a, b = torch.min(t), torch.max(t)
            if mn is None:
                mn, mx = a, b
            else:
                mn = mn + alpha * (a - mn)
                mx = mx + alpha * (b - mx)
        return mn, mx
    raise ValueError(f'Unsupported calibration algorithm: {algo}')


def qparams(mn, mx, qmin, qmax, sym: bool):
    """quant.py:545-559 (round_zp True)."""
    if sym:
        abs_max = torch.max(mx.abs(), mn.abs()).clamp(min=1e-5)
        return abs_max / qmax, torch.tensor(0.0)
    scales = (mx - mn).clamp(min=1e-5) / (qmax - qmin)
    zeros = (qmin - torch.round(mn / scales)).clamp(qmin, qmax)
    return scales, zeros


def int_range(bit: int, sym: bool):
    """IntegerQuantizer qmin / qmax tensors (quant.py:661-678)."""
    if sym:
        return torch.tensor(-(2 ** (bit - 1))), torch.tensor(2 ** (bit - 1) - 1)
    return torch.tensor(0.0), torch.tensor(2 ** bit - 1)


def fake_quant_act_static_int(act, scales, zeros, qmin, qmax):
    """IntegerQuantizer.fake_quant_act_static, per_tensor (quant.py:699-717, 719-743)."""
    q = torch.clamp(torch.round(act / scales) + zeros, qmin, qmax)
    return ((q - zeros) * scales).to(act.dtype)


# ---- static_hist (quant.py:264-529) ----------------------------------------------------------
BINS, UPSAMPLE = 2048, 16


def _upscale(hist, lo, hi, new_lo, new_hi):
    """_upscale_histogram (quant.py:332-366): the old histogram's 16x-refined midpoints,
    re-binned into the new range with their (1/16) counts."""
    w = hist.repeat_interleave(UPSAMPLE) / UPSAMPLE
    step = (hi - lo) / (BINS * UPSAMPLE)
    mids = torch.linspace(lo, hi, BINS * UPSAMPLE + 1)[:-1] + 0.5 * step
    edges = torch.linspace(new_lo, new_hi, BINS + 1)
    idx = (torch.bucketize(mids, edges, right=True) - 1).clamp(0, BINS - 1)
    return torch.bincount(idx, weights=w, minlength=BINS)


def hist_range(tensors):
    """get_static_hist_range for one module input: (min, max) after the threshold search."""
    hist, lo, hi = None, None, None
    for t in tensors:
        t = t.float()
        t_lo, t_hi = torch.min(t), torch.max(t)
        if hist is None:
            hist = torch.histc(t, BINS, min=t_lo.item(), max=t_hi.item())
            lo, hi = t_lo, t_hi
            continue
        n_lo, n_hi = torch.min(lo, t_lo), torch.max(hi, t_hi)
        upd = torch.histc(t, BINS, min=n_lo.item(), max=n_hi.item())
        if n_lo == lo and n_hi == hi:
            hist = hist + upd
        elif lo == hi:  # _combine_histograms' single-value branch (quant.py:381-389)
            hist = torch.histc(lo, BINS, min=n_lo, max=n_hi) * torch.sum(upd) + upd
        else:
            hist = upd + _upscale(hist, lo, hi, n_lo, n_hi)
        lo, hi = n_lo, n_hi
    return hist_threshold(hist, lo, hi)


def _l2(b, e, dens):
    return dens * ((e * e * e - b * b * b) / 3)


def _quant_error(hist, lo, hi, s, e, dst_nbins):
    """get_quantization_error (quant.py:275-330)."""
    bw = (hi.item() - lo.item()) / BINS
    dbw = bw * (e - s + 1) / dst_nbins
    if dbw == 0.0:
        return 0.0
    src = torch.arange(BINS)
    sb = (src - s) * bw
    se = sb + bw
    db = torch.clamp(torch.div(sb, dbw, rounding_mode='floor'), 0, dst_nbins - 1)
    de = torch.clamp(torch.div(se, dbw, rounding_mode='floor'), 0, dst_nbins - 1)
    dens = hist / bw
    norm = torch.zeros(BINS)
    norm += _l2(sb - (db + 0.5) * dbw, torch.ones(BINS) * (dbw / 2), dens)
    norm += (de - db - 1) * _l2(torch.tensor(-dbw / 2), torch.tensor(dbw / 2), dens)
    norm += _l2(torch.tensor(-dbw / 2), se - (de * dbw + dbw / 2), dens)
    return norm.sum().item()


def hist_threshold(hist, lo, hi, dst_nbins=256):
    """get_hist_threshold (quant.py:403-451): walk the quantile bounds in 1e-8 steps, keep
    the last bin pair before the L2 error stops decreasing."""
    bw = (hi - lo) / BINS
    total = torch.sum(hist).item()
    csum = torch.cumsum(hist, dim=0)
    a, b, s, e, best = 0.0, 1.0, 0, BINS - 1, float('inf')
    while a < b:
        na, nb = a + 1e-8, b - 1e-8
        left, right = s, e
        while left < e and csum[left] < na * total:
            left += 1
        while right > s and csum[right] > nb * total:
            right -= 1
        ns, ne = s, e
        if left - s > e - right:
            ns, a = left, na
        else:
            ne, b = right, nb
        if ns == s and ne == e:
            continue
        err = _quant_error(hist, lo, hi, ns, ne, dst_nbins)
        if err > best:
            break
        best, s, e = err, ns, ne
    return lo + bw * s, lo + bw * (e + 1)
