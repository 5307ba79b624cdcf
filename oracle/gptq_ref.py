"""ORACLE (test infrastructure only) — GPTQ layer algorithm, CPU restatement.

Follows llmc/compression/quantization/gptq.py op by op in fp32 torch-CPU:
Hessian running average (add_batch :253-295, world_size 1), act-order permutation
(hessian_sorting :58-64), dead columns + damping + Cholesky chain (process_hessian_and_weights
:128-176), blocked OBS column loop with per-group min/max qparams from the block-start weights
(weight_transform :198-244, search_column_qparams :358-366), inverse permutation and merged
group qparams (update_layer_with_transformed_weights :178-196, merge_qparams :344-356).
"""
from __future__ import annotations

import math

import torch

from . import quant_ref as Q


def hessian(samples, ic: int):
    """gptq.py:253-295 — running average over per-sample batches; returns (H, nsamples)."""
    H = torch.zeros((ic, ic))
    n = 0
    for inp in samples:
        if inp.dim() == 2:
            inp = inp.unsqueeze(0)
        b = inp.shape[0]
        x = inp.reshape(-1, inp.shape[-1]).t()
        H *= n / (n + b)
        n += b
        x = math.sqrt(2 / n) * x.float()
        H += x.matmul(x.t())
    return H, n


def prepare(W: torch.Tensor, H: torch.Tensor, actorder: bool, percdamp: float):
    """gptq.py:58-64, 128-176. Returns (W fp32 permuted, U upper chol of H^-1, perm|None)."""
    H = H.clone()
    perm = torch.argsort(torch.diag(H), descending=True) if actorder else None
    W = W.clone().float()
    dead = torch.diag(H) == 0
    H[dead, dead] = 1
    W[:, dead] = 0
    if perm is not None:
        W = W[:, perm]
        H = H[perm][:, perm]
    cols = H.shape[0]
    damp = percdamp * torch.mean(torch.diag(H))
    d = torch.arange(cols)
    H[d, d] += damp
    H = torch.linalg.cholesky(H)
    H = torch.cholesky_inverse(H)
    U = torch.linalg.cholesky(H, upper=True)
    return W, U, perm


def prepare_owq(W: torch.Tensor, H: torch.Tensor, nout: int, percdamp: float):
    """OWQ hessian_sorting (gptq.py:58-83, actorder off) + process_hessian_and_weights."""
    H = H.clone()
    desc = torch.argsort(torch.diag(H), descending=True)
    keep = torch.ones(H.shape[0], dtype=torch.bool)
    keep[desc[:nout]] = False
    perm = torch.cat([torch.arange(H.shape[0])[keep], desc[:nout]])
    W = W.clone().float()
    dead = torch.diag(H) == 0
    H[dead, dead] = 1
    W[:, dead] = 0
    W = W[:, perm]
    H = H[perm][:, perm]
    d = torch.arange(H.shape[0])
    H[d, d] += percdamp * torch.mean(torch.diag(H))
    H = torch.linalg.cholesky(H)
    H = torch.cholesky_inverse(H)
    U = torch.linalg.cholesky(H, upper=True)
    return W, U, perm


def column_loop(W: torch.Tensor, U: torch.Tensor, bit, sym: bool, group: int | None,
                blocksize: int = 128, fixed=None, static=None, ncols_q: int | None = None,
                mse: bool = False, fp8: str | None = None):
    """gptq.py:198-244 on permuted fp32 W (modified in place to the compensated weights).

    group=None with fixed=(scale[rows,1], zero) -> per-channel fixed qparams.
    static=(scales [rows, ng], zeros | None, perm | None): static_groups (gptq.py:224-227,
    split_qparams :333-341) -- permuted column j uses original group perm[j] // group.
    mse=True: calib_algo mse, the group range from get_mse_range (search_column_qparams
    :359-366 -> get_tensor_qparams) of the group's columns of the global W.
    fp8='e4m3' / 'e5m2': FloatQuantizer(use_qtorch) weights (gptq_fp8.yml): group qparams
    max(|min|, |max|).clamp(1e-5) / finfo.max (quant.py:545-553 on the fp32 columns) and
    quant_dequant = float_quantize(w / s + 0) * s (quant.py:1061-1080, fp8_ref stand-in).
    Returns (tmp, Losses, scales [rows, ng], zeros [rows, ng] | None)."""
    if fp8 is not None:
        from . import fp8_ref
        qmax = fp8_ref.qmax_of(fp8)
        qmin = -qmax
    else:
        qmin, qmax = Q.int_range(bit, sym)
    rows, cols = W.shape
    ncq = cols if ncols_q is None else ncols_q  # OWQ: the outlier tail is not quantized
    Losses = torch.zeros_like(W)
    tmp = torch.zeros_like(W)
    groups = {}
    qp = fixed
    for i1 in range(0, ncq, blocksize):
        i2 = min(i1 + blocksize, ncq)
        W1, U1 = W[:, i1:i2].clone(), U[i1:i2, i1:i2]
        tmp1, Err1, L1 = torch.zeros_like(W1), torch.zeros_like(W1), torch.zeros_like(W1)
        for i in range(i2 - i1):
            w, d = W1[:, i], U1[i, i]
            if static is not None:
                ss, zs, sp = static
                g = (int(sp[i1 + i]) if sp is not None else i1 + i) // group
                qp = (ss[:, g:g + 1], torch.tensor(0.0) if zs is None else zs[:, g:g + 1])
            elif group is not None and (i1 + i) % group == 0:
                ct = W[:, i1 + i:min(i1 + i + group, ncq)]
                t = Q.group_view(ct, 'per_group', group)
                mn, mx = Q.mse_range(t, bit, sym) if mse else Q.minmax(t)
                if fp8 is not None:
                    from . import fp8_ref
                    qp = (fp8_ref.sym_scales(mn, mx, qmax), torch.tensor(0.0))
                else:
                    s, z = Q.qparams(mn, mx, qmin, qmax, sym)
                    qp = (s, z)
                groups[(i1 + i) // group] = qp
            s, z = qp
            if fp8 is not None:
                from . import fp8_ref
                q = fp8_ref.qdq_given(w.unsqueeze(1), s, fp8).squeeze(1)
            else:
                q = Q.dequant(Q.quant(w.unsqueeze(1), s, z, qmin, qmax), s, z).squeeze(1)
            tmp1[:, i] = w
            L1[:, i] = ((w - q) ** 2) / (2 * d ** 2)
            err1 = (w - q) / d
            W1[:, i:] -= err1.unsqueeze(1).matmul(U1[i, i:].unsqueeze(0))
            Err1[:, i] = err1
        tmp[:, i1:i2], Losses[:, i1:i2] = tmp1, L1
        W[:, i2:] -= Err1.matmul(U[i1:i2, i2:])
    if ncq < cols:
        tmp[:, ncq:] = W[:, ncq:]  # gptq.py:187-188
    if group is None or static is not None:
        return tmp, Losses, None, None
    ng = len(groups)
    scales = torch.stack([groups[g][0] for g in range(ng)], dim=1).reshape(rows, ng)
    zeros = None
    if not sym and fp8 is None:
        zeros = torch.stack([groups[g][1] for g in range(ng)], dim=1).reshape(rows, ng)
    return tmp, Losses, scales, zeros


def quantize_layer(W: torch.Tensor, H: torch.Tensor, bit=4, sym=False, group=128,
                   actorder=True, percdamp=0.01, blocksize=128, mse=False):
    """Whole GPTQ layer transform. Returns dict(weight (fp32, original column order),
    scales/zeros [rows*ng, 1] (merge_qparams order), perm, invperm, U, loss)."""
    Wp, U, perm = prepare(W, H, actorder, percdamp)
    tmp, Losses, s, z = column_loop(Wp, U, bit, sym, group, blocksize, mse=mse)
    invperm = torch.argsort(perm) if perm is not None else None
    weight = tmp[:, invperm] if invperm is not None else tmp
    return dict(weight=weight, scales=s.reshape(-1, 1), zeros=None if z is None else z.reshape(-1, 1),
                perm=perm, invperm=invperm, U=U, loss=Losses.sum().item())


def quantize_layer_static(W: torch.Tensor, H: torch.Tensor, scales, zeros, bit=4, sym=False,
                          group=128, actorder=True, percdamp=0.01, blocksize=128):
    """GPTQ with static_groups: the group qparams (buf_scales / buf_zeros [rows*ng, 1],
    collected from the original weights) are used as they are and stay the layer's qparams."""
    Wp, U, perm = prepare(W, H, actorder, percdamp)
    rows = Wp.shape[0]
    st = (scales.reshape(rows, -1), None if sym else zeros.reshape(rows, -1), perm)
    tmp, Losses, _, _ = column_loop(Wp, U, bit, sym, group, blocksize, static=st)
    invperm = torch.argsort(perm) if perm is not None else None
    weight = tmp[:, invperm] if invperm is not None else tmp
    return dict(weight=weight, scales=scales, zeros=zeros, perm=perm, invperm=invperm, U=U,
                loss=Losses.sum().item())


def deploy_fake(weight, scales, zeros, perm, invperm, bit, sym, group, model_dtype):
    """GPTQ.w_qdq (gptq.py:424-452): static fake quant in permuted space, then invperm."""
    w = weight[:, perm] if perm is not None else weight
    out = Q.fake_quant_static(w, scales, zeros, bit, sym, 'per_group', group).to(model_dtype)
    return out[:, invperm] if invperm is not None else out


def quantize_layer_owq(W: torch.Tensor, H: torch.Tensor, nout: int, bit=4, sym=False, group=128,
                       percdamp=0.01, blocksize=128):
    """GPTQ + OWQ layer transform; returns dict like quantize_layer (+ n_nonout).
    group=None: per_channel -- the qparams of the permuted non-outlier columns
    (gptq.py:157-166, get_tensor_qparams(W[:, :n_nonout]) on the fp32 weights)."""
    Wp, U, perm = prepare_owq(W, H, nout, percdamp)
    ncq = Wp.shape[1] - nout
    if group is None:
        qmin, qmax = Q.int_range(bit, sym)
        mn, mx = Q.minmax(Wp[:, :ncq], 'per_channel')
        fs, fz = Q.qparams(mn, mx, qmin, qmax, sym)
        tmp, Losses, _, _ = column_loop(Wp, U, bit, sym, None, blocksize, fixed=(fs, fz),
                                        ncols_q=ncq)
        invperm = torch.argsort(perm)
        return dict(weight=tmp[:, invperm], scales=fs, zeros=None if sym else fz, perm=perm,
                    invperm=invperm, U=U, n_nonout=ncq, loss=Losses.sum().item())
    tmp, Losses, s, z = column_loop(Wp, U, bit, sym, group, blocksize, ncols_q=ncq)
    invperm = torch.argsort(perm)
    return dict(weight=tmp[:, invperm], scales=s.reshape(-1, 1),
                zeros=None if z is None else z.reshape(-1, 1), perm=perm, invperm=invperm, U=U,
                n_nonout=ncq, loss=Losses.sum().item())


def deploy_fake_owq(weight, scales, zeros, perm, invperm, n_nonout, bit, sym, group,
                    model_dtype):
    """GPTQ.w_qdq with OWQ (gptq.py:424-452): the float outlier columns are put back."""
    w = weight[:, perm]
    gran = 'per_group' if group else 'per_channel'
    out = Q.fake_quant_static(w, scales, zeros, bit, sym, gran, group).to(model_dtype)
    out[:, n_nonout:] = w[:, n_nonout:].to(model_dtype)
    return out[:, invperm]
