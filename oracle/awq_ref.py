"""ORACLE (test infrastructure only) — AWQ scale search and auto-clip, CPU restatement.

Follows llmc/compression/quantization/awq.py (trans_version v1 / v2, w_only, awq_bs None) and
auto_clip.py (clip_version v1, w_only) op by op in torch-CPU with the reference's dtypes.
The inspect module forward (HF Llama attention / MLP / Linear) is the same third-party
torch module the reference calls.
"""
from __future__ import annotations

import torch

from . import quant_ref as Q


def act_scale(x: torch.Tensor) -> torch.Tensor:
    """awq.py:74-85 (batch == _bs)."""
    return x.abs().view(-1, x.shape[-1]).mean(0)


def scales_v2(x_mean: torch.Tensor, ratio: float) -> torch.Tensor:
    """awq.py:87-108 (trans_version v2, not GQA)."""
    s = x_mean.pow(ratio).clamp(min=1e-4).view(-1)
    return s / (s.max() * s.min()).sqrt()


def weight_scale(weights: list, group) -> torch.Tensor:
    """awq.py:48-72 (get_weight_scale, bf16/fp16 weights): per group |w| / max|w| in the weight
    dtype, mean over rows (torch-CPU: fp32 sum, / rows, back to the dtype), summed over the
    subset's layers in the dtype, / len(layers)."""
    total = None
    for w in weights:
        a = w.clone().reshape(-1, group).abs() if group else w.clone().abs()
        mx = a.amax(dim=1, keepdim=True)
        ls = a.div_(mx).view(w.shape)
        total = ls.mean(0) if total is None else total.add_(ls.mean(0))
    return total.div_(len(weights))


def scales_v1(x_mean: torch.Tensor, w_max: torch.Tensor, ratio: float) -> torch.Tensor:
    """awq.py:87-108 (trans_version v1, not GQA)."""
    s = (x_mean.pow(ratio) / w_max.pow(1 - ratio)).clamp(min=1e-4).view(-1)
    return s / (s.max() * s.min()).sqrt()


def fake_quant_scaled(w: torch.Tensor, s: torch.Tensor, bit, sym, group):
    """awq.py:39-46 + 147-164: W.mul_(s) then fake_quant_weight_dynamic, weight dtype."""
    ws = w.clone().mul_(s.view(1, -1))
    return Q.fake_quant_dynamic(ws, bit, sym, 'per_group', group)[0]


def loss(org_out: torch.Tensor, out: torch.Tensor) -> float:
    """awq.py:134-145."""
    return (org_out - out).float().pow(2).mean().item()


def search_scale(x: torch.Tensor, weights: list, forward, bit, sym, group, n_grid=20,
                 version='v2'):
    """awq.py:178-278 for one input tensor (len(input)==1, world_size 1).

    ``forward(x, qweights)`` runs the inspect module with the given (fake-quantised) weights.
    Returns (losses[n_grid], best_index, best_scales)."""
    w_max = weight_scale(weights, group) if version == 'v1' else None
    x_mean = act_scale(x)
    org_out = forward(x, None)
    best, best_i, best_s = float('inf'), -1, None
    losses = []
    for n in range(n_grid):
        ratio = n * 1 / n_grid
        s = scales_v1(x_mean, w_max, ratio) if version == 'v1' else scales_v2(x_mean, ratio)
        qw = [fake_quant_scaled(w, s, bit, sym, group) for w in weights]
        out = forward(x / s.view(1, -1), qw)
        lo = loss(org_out, out)
        lm = x.shape[0] * 1.0 / x.shape[0] * lo
        losses.append(lm)
        if lm < best:
            best, best_i, best_s = lm, n, x.shape[0] * 1.0 / x.shape[0] * s
    return losses, best_i, best_s


def _fq_mse(cur: torch.Tensor, bit, sym, group):
    """fake_quant_weight_dynamic with calib_algo mse (quant.py:145-203, 690-697, 833-869):
    fp32 range search, fp32 qparams, quant-dequant in fp32 (bf16 / fp16 tensor promoted by the
    fp32 scales), back to the weight dtype."""
    qmin, qmax = Q.int_range(bit, sym)
    t = cur.reshape(-1, group)
    mn, mx = Q.mse_range(t, bit, sym)
    s, z = Q.qparams(mn, mx, qmin, qmax, sym)
    out = Q.dequant(Q.quant(t.float(), s, z, qmin, qmax), s, z)
    return out.reshape(cur.shape).to(cur.dtype)


def _fq_fp8(cur: torch.Tensor, fmt: str, per_tensor: bool):
    """FloatQuantizer(use_qtorch).fake_quant_weight_dynamic of a clamped [rows, 1, 1, ic]
    batch (quant.py:1142-1159): per_channel scales in the weight dtype, per_tensor scale of
    the whole batch in fp32 (0-dim / 0-dim promotion); q fp32, (q - 0) * s, weight dtype."""
    from . import fp8_ref as P
    qmax = P.qmax_of(fmt)
    if per_tensor:
        mn, mx = torch.min(cur), torch.max(cur)
    else:
        mn, mx = cur.amin(dim=-1, keepdim=True), cur.amax(dim=-1, keepdim=True)
    s = P.sym_scales(mn, mx, qmax)
    return P.qdq_given(cur, s, fmt).to(cur.dtype)


def logit(x):
    """auto_clip.py:41."""
    return torch.log(x / (1 - x))


def _fq_v2(wb, min_val, max_val, org_min, org_max, bit, sym):
    """auto_clip.py:258-267 (clip_version v2): the unclamped weights' static fake quant with
    the qparams of get_learnable_range(w, logit(min/org_min), logit(max/org_max))."""
    low = logit(min_val / org_min)
    up = logit(max_val / org_max)
    mn, mx = Q.learnable_range(wb, low, up, sym)
    qmin, qmax = Q.int_range(bit, sym)
    s, z = Q.qparams(mn, mx, qmin, qmax, sym)
    return Q.dequant(Q.quant(wb, s, z, qmin, qmax), s, z).to(wb.dtype)


def clip_layer(w: torch.Tensor, x: torch.Tensor, bit, sym, group, clip_sym, n_grid=20,
               max_shrink=0.5, n_sample_token=512, mse=False, act=None, fp8=None, version=1):
    """auto_clip.py:83-191 (clip v1, single input). Returns (best_max, best_min) shaped
    [oc, ng, 1]. mse=True: the weight quantizer's calib_algo is mse. group = ic is the
    per_channel case (auto_clip.py:96-99). act = (bits, sym): w_only False, the shrink steps
    see fake_quantize_input(x) = per_token fake quant of the [1, T, ng, group] view
    (auto_clip.py:176-177, 269-274; quant.py:754-771 with reshape_tensor's per_token no-op).
    fp8 = (fmt, per_tensor, act_quant | None): FloatQuantizer weights (group = ic); act_quant is
    a function giving fake_quantize_input(x) for w_only False. version 2: clip_version v2
    candidates (_fq_v2, integer weights)."""
    w = w.reshape(w.shape[0], 1, -1, group)
    ocb = 256 if w.shape[0] % 256 == 0 else 64
    x = x.view(-1, x.shape[-1]).reshape(1, -1, x.shape[-1] // group, group)
    step = max(1, x.shape[1] // n_sample_token)
    x = x[:, 0::step]
    bmx_all, bmn_all = [], []
    for ib in range(w.shape[0] // ocb):
        wb = w[ib * ocb:(ib + 1) * ocb]
        org_max = wb.abs().amax(dim=-1, keepdim=True) if clip_sym else wb.amax(dim=-1, keepdim=True)
        org_min = wb.amin(dim=-1, keepdim=True)
        best_max, best_min = org_max.clone(), org_min.clone()
        min_errs = torch.ones_like(org_max) * 1e9
        org_out = (x * wb).sum(dim=-1)
        qx = x if act is None else Q.fake_quant_dynamic(x, act[0], act[1], 'per_token')[0]
        if fp8 is not None and fp8[2] is not None:
            qx = fp8[2](x)
        for i_s in range(int(max_shrink * n_grid)):
            max_val = org_max * (1 - i_s / n_grid)
            min_val = -max_val if clip_sym else org_min * (1 - i_s / n_grid)
            cur = torch.clamp(wb, min_val, max_val)
            if version == 2:
                q_w = _fq_v2(wb, min_val, max_val, org_min, org_max, bit, sym)
            elif fp8 is not None:
                q_w = _fq_fp8(cur, fp8[0], fp8[1])
            else:
                q_w = (_fq_mse(cur, bit, sym, group) if mse else
                       Q.fake_quant_dynamic(cur, bit, sym, 'per_group', group)[0])
            cur_out = (qx * q_w).sum(dim=-1)
            err = (cur_out - org_out).pow(2).mean(dim=1).view(min_errs.shape)
            err_mean = 0 + err
            err_mean /= 1
            idx = err_mean < min_errs
            min_errs[idx] = err_mean[idx]
            best_max[idx] = max_val[idx]
            best_min[idx] = min_val[idx]
        bmx_all.append(best_max)
        bmn_all.append(best_min)
    return torch.cat(bmx_all, 0).squeeze(1), torch.cat(bmn_all, 0).squeeze(1)


def clip_factors(w: torch.Tensor, max_val, min_val, clip_sym, group):
    """auto_clip.py:235-256 get_clip_factor: (up, low | None) [groups, 1]."""
    mn, mx = Q.minmax(Q.group_view(w, 'per_group', group))
    shape = mx.shape
    if clip_sym:
        am = torch.max(mx.abs(), mn.abs()).clamp(min=1e-5).reshape(*max_val.shape[:2], -1)
        return logit(max_val / am).reshape(shape), None
    up = logit(max_val / mx.reshape(*max_val.shape[:2], -1)).reshape(shape)
    low = logit(min_val / mn.reshape(*min_val.shape[:2], -1)).reshape(shape)
    return up, low


def apply_clip(w: torch.Tensor, max_val, min_val, clip_sym):
    """auto_clip.py:193-212 (v1)."""
    shape = w.shape
    wg = w.reshape(*max_val.shape[:2], -1)
    if clip_sym:
        min_val = -max_val
    return torch.clamp(wg, min_val, max_val).reshape(shape)
