"""AWQ weight clipping (drop-in for llmc ``quantization/auto_clip.py``, clip_version v1 / v2).

``auto_clip_layer`` is one HIP launch per linear (``lcq_auto_clip_search``): the reference
materialises a [256, T, ng, 128] bf16 broadcast product per shrink step and batch of rows
(1 GiB at ng=32); the kernel keeps weights in VGPRs and streams token tiles through LDS.
per_channel weights (group = ic, the w8a8 AWQ configs) take ``lcq_auto_clip_search_pc``;
w_only False feeds the shrink steps the activation fake-quant (``fake_quantize_input``).
clip_version v2 (calib_algo learnable; awq_comb_omni w6a6 / w8a8 step_1_awq.yml) searches the
same bounds with learnable-range candidates (unclamped weight) and stores them as logit factors
(``buf_upbound_factor`` / ``buf_lowbound_factor``) that the deploy fake quant applies.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops
from .module_utils import _LLMC_LINEAR_TYPES_, _TRANSFORMERS_LINEAR_TYPES_
from .utils import world

_LINEAR_TYPES = tuple(_LLMC_LINEAR_TYPES_ + _TRANSFORMERS_LINEAR_TYPES_)


class AutoClipper:
    """auto_clip.py:22-281."""

    def __init__(self, w_only, wquantizer, aquantizer, clip_version, clip_sym, save_clip,
                 padding_mask):
        self.wquantizer = wquantizer
        self.aquantizer = aquantizer
        self.clip_version = clip_version
        self.clip_sym = clip_sym
        self.save_clip = save_clip
        self.padding_mask = padding_mask
        self.weight_clips = {}
        self.w_only = w_only
        self.reduce_across_ranks = False  # set by the algorithm in replicate (DP) mode
        self.shard_rows = False           # shard_search: each rank searches its row range
        if clip_version not in ('v1', 'v2'):
            raise Exception('Not support other clip version')

    @torch.no_grad()
    def run(self, block, block_idx, input_feat, n_sample_token):
        """auto_clip.py:43-81: every block linear except q/k projections."""
        for n, m in block.named_modules():
            if not isinstance(m, _LINEAR_TYPES):
                continue
            if any(k in n for k in ('q_', 'k_', 'query', 'key', 'Wqkv')):
                continue
            feats = input_feat[n]
            inputs = [torch.cat(feats)] if len(feats) != 1 else feats
            _, ws, _ = world()
            if self.shard_rows and ws > 1 and dist.is_initialized():
                # rows are independent (auto_clip.py:72-76 batches them): search this rank's
                # share, gather the bounds (bit-identical to one GPU)
                from .parallel import dist_world, gather_rows, row_shard
                rank, wsz = dist_world()
                align = self._float_quant(m.weight)[1] or 1  # per-tensor fp8: whole batches
                r0, r1 = row_shard(m.weight.shape[0], rank, wsz, align)
                mx, mn = self.auto_clip_layer(block_idx, n, m.weight.data[r0:r1], inputs,
                                              n_sample_token=n_sample_token,
                                              tensor_batch=align if align > 1 else None)
                max_val = gather_rows(mx.contiguous(), m.weight.shape[0], align)
                min_val = gather_rows(mn.contiguous(), m.weight.shape[0], align)
                self.apply_clip(block_idx, m, min_val, max_val, n)
                continue
            max_val, min_val = self.auto_clip_layer(block_idx, n, m.weight, inputs,
                                                    n_sample_token=n_sample_token)
            _, ws, _ = world()
            if self.reduce_across_ranks and ws > 1 and dist.is_initialized():
                dist.all_reduce(max_val, op=dist.ReduceOp.SUM)
                max_val /= ws
                dist.all_reduce(min_val, op=dist.ReduceOp.SUM)
                min_val /= ws
            self.apply_clip(block_idx, m, min_val, max_val, n)

    @staticmethod
    def sample_tokens(x: torch.Tensor, n_sample_token):
        """auto_clip.py:134-147: flatten tokens and keep every step-th one."""
        x = x.reshape(-1, x.shape[-1])
        if n_sample_token is None:
            n_sample_token = min(x.shape[0], 512)
        step = max(1, x.shape[0] // n_sample_token)
        return x[0::step].contiguous()

    @torch.no_grad()
    def auto_clip_layer(self, block_idx, layer_name, w, inputs, n_grid=20, max_shrink=0.5,
                        n_sample_token=512, eps=0.0, tensor_batch=None):
        """Returns (best_max_val, best_min_val) shaped [oc, ng, 1] like the reference.
        tensor_batch: the per-tensor FP8 batch rows of the whole layer when ``w`` is a row
        shard of it (the shard's own row count would pick a different batch size)."""
        assert w.dim() == 2
        wq = self.wquantizer
        group = wq.group_size if wq.granularity == 'per_group' else w.shape[1]
        if len(inputs) != 1:
            raise NotImplementedError('auto-clip over several calibration tensors')
        if w.dtype not in (torch.bfloat16, torch.float16):
            raise NotImplementedError('device auto-clip kernel takes bf16 / fp16 weights')
        fp8, tb = self._float_quant(w)
        tensor_batch = tb if (tensor_batch is None or not tb) else tensor_batch
        per_channel = wq.granularity in ('per_channel', 'per_tensor')
        if not per_channel and group not in (32, 64, 128, 256):
            raise NotImplementedError(f'device auto-clip kernel: group size {group}')
        if per_channel and (w.shape[1] % 128 or wq.calib_algo == 'mse'):
            raise NotImplementedError('per_channel auto-clip: ic % 128 == 0, minmax qparams')
        if self.clip_version == 'v2' and (fp8 is not None or wq.granularity != 'per_channel'):
            # every reference v2 config (awq_comb_omni w6a6 / w8a8) is integer per_channel
            raise NotImplementedError('clip_version v2: integer per_channel weights')
        if wq.granularity == 'per_tensor' and fp8 is None:
            raise NotImplementedError('per_tensor integer auto-clip is not on the device path')
        if (getattr(wq, 'quant_type', 'int-quant') == 'int-quant'
                and (not getattr(wq, 'round_zp', True) or wq.calib_algo == 'hqq')):
            # the kernels form round_zp / minmax (or mse) qparams of every candidate
            raise NotImplementedError('auto-clip with round_zp False / calib_algo hqq is not '
                                      'on the device path')
        x = self.sample_tokens(inputs[0], n_sample_token)
        qx = None
        if not self.w_only:
            # fake_quantize_input (auto_clip.py:269-274) sees x as [1, T, ic/group, group]:
            # per_token act quant then runs per (token, group) (reshape_tensor is a no-op)
            qx = self.aquantizer.fake_quant_act_dynamic(
                x.reshape(1, x.shape[0], -1, group)).reshape(x.shape)
        qmin, qmax = int(wq.qmin.item()), int(wq.qmax.item())
        mse = None
        if wq.calib_algo == 'mse':  # every step's fake quant searches its range
            mse = (wq._mse_nsteps(), wq.mse_grid, 2.4)
        return ops.auto_clip_search(w.data, x, group, int(max_shrink * n_grid), n_grid, qmin,
                                    qmax, wq.sym, self.clip_sym, mse=mse, qx=qx, fp8=fp8,
                                    tensor_batch=tensor_batch,
                                    version=2 if self.clip_version == 'v2' else 1)

    def _float_quant(self, w):
        """(fp8 dtype, per-tensor batch rows) for FloatQuantizer weights, (None, 0) for
        integer ones. The reference fake-quantizes 256 (else 64) rows at a time
        (auto_clip.py:108-114), so a per_tensor scale is one per such batch of clamped rows."""
        wq = self.wquantizer
        if getattr(wq, 'quant_type', 'int-quant') == 'int-quant':
            return None, 0
        if (not getattr(wq, 'use_qtorch', False) or getattr(wq, 'fp8_dtype', None) is None
                or 'float_range' in getattr(wq, 'kwargs', {}) or wq.calib_algo != 'minmax'
                or wq.granularity not in ('per_channel', 'per_tensor')):
            raise NotImplementedError('float-quant auto-clip: use_qtorch e4m3 / e5m2, minmax, '
                                      'per_channel or per_tensor weights')
        if wq.granularity == 'per_tensor':
            return wq.fp8_dtype, (256 if w.shape[0] % 256 == 0 else 64)
        return wq.fp8_dtype, 0

    @torch.no_grad()
    def apply_clip(self, block_idx, layer, min_val, max_val, layer_name):
        """auto_clip.py:193-233. v1: clamp the weight per group in place. v2: keep the weight,
        register the logit factors of the bounds (get_clip_factor) as buffers."""
        w = layer.weight.data
        group = w.shape[1] // max_val.shape[1]
        if self.clip_version == 'v2':
            up, low = self.get_clip_factor(block_idx, layer, min_val, max_val, layer_name)
            layer.register_buffer('buf_upbound_factor', up)
            layer.register_buffer('buf_lowbound_factor', low)
            if self.save_clip:
                n = f'{layer_name}.weight_quantizer.'
                d = self.weight_clips.setdefault(block_idx, {})
                d[n + 'upbound_factor'] = up.cpu()
                d[n + 'lowbound_factor'] = low.cpu() if low is not None else None
            return
        cmax = max_val.reshape(-1).to(w.dtype)
        cmin = None if self.clip_sym else min_val.reshape(-1).to(w.dtype)
        ops.clip_apply(w, group, cmax, cmin, out=w)
        # v1 stores nothing under save_clip (only v2 saves clip factors, auto_clip.py:218-233)

    def get_clip_factor(self, block_idx, layer, min_val, max_val, layer_name):
        """auto_clip.py:235-256 (one HIP launch, lcq_clip_factors): (up, low | None) shaped
        like get_minmax_range of the reshaped weight, [groups, 1], in the weight dtype."""
        w = layer.weight.data
        group = w.shape[1] // max_val.shape[1]
        cmax = max_val.reshape(-1).to(w.dtype)
        cmin = None if self.clip_sym else min_val.reshape(-1).to(w.dtype)
        return ops.clip_factors(w, group, cmax, cmin, self.clip_sym)
