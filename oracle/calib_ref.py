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
