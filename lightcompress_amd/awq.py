"""AWQ (drop-in for llmc ``quantization/awq.py``; trans_version v1 / v2, clip v1).

Device design of ``search_scale_subset`` (awq.py:178-278):
* the calibration input, the original module output and the original weights stay in HBM;
  the reference copies inputs CPU->GPU per ratio and restores weights from a CPU state dict;
* per ratio: ``lcq_awq_scales`` (one workgroup), ``lcq_int_quant_dynamic`` with the fused
  ``W * s`` pre-scale writing into a reusable buffer that the module's weight points to,
  ``lcq_scale_bcast`` for ``x / s`` into a reusable buffer, the inspect module's own forward,
  and ``lcq_sq_diff_mean`` writing the loss into a device slot — one host sync per subset
  instead of one ``.item()`` + ``gc.collect()`` per ratio.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .base_blockwise_quantization import BaseBlockwiseQuantization, is_norm
from .llama import _mkey
from .module_utils import FakeQuantLinear
from .registry import ALGO_REGISTRY


@ALGO_REGISTRY
class Awq(BaseBlockwiseQuantization):
    # quant_out at world > 1 (every backend AWQ config): every rank holds the block's
    # calibration tokens and evaluates its share of the ratio grid and of the clip rows; the
    # losses and clip bounds are gathered (bit-identical to one GPU)
    sequential_parallel_mode = 'shard_search'

    def __init__(self, model, quant_config, input, padding_mask, config):
        super().__init__(model, quant_config, input, padding_mask, config)
        special = self.quant_config.get('special', {}) or {}
        self.trans = special.get('trans', True)
        self.trans_version = special.get('trans_version', 'v2')
        self.awq_bs = special.get('awq_bs', None)
        self.save_mem = special.get('save_mem', True)
        if self.trans_version not in ('v1', 'v2'):
            raise ValueError(f'trans_version {self.trans_version}')
        self.n_grid = 20
        self.last_search = {}
        self._org_cache = {}
        self._org_capture_active = False
        self.org_reuse_stats = {'reused': 0, 'recomputed': 0}
        self.reuse_org = True

    # -- original inspect outputs from the block's own forward ------------------------------
    # search_scale_subset starts from the inspect module's output on the captured input
    # (awq.py:204-206: one extra forward of self_attn / mlp / down_proj per subset). The
    # block's capture forward already ran every inspect module on exactly that input and
    # batch (quant_out False: the forward that feeds the next block; True: the capture
    # forward, then run to completion instead of stopping after the last input is seen), so
    # its outputs are kept: same modules, kernels and shapes -> bit-identical, one forward
    # per subset saved. An output is used only if the module's linear weights are unchanged
    # since the capture (identity + storage + in-place version) and the search runs the
    # whole batch at once (awq_bs unset); otherwise the forward is recomputed.
    class _EndCapture:
        def __init__(self, algo):
            self.algo = algo

        def remove(self):
            self.algo._org_capture_active = False

    def run(self, block, input_feat, handles):
        self._org_cache = {}
        extra = []
        if self.trans and not self.data_free:
            extra = self._hook_org_outputs(block) + [Awq._EndCapture(self)]
            self._org_capture_active = True
        try:
            super().run(block, input_feat, list(handles) + extra)
        finally:
            self._org_cache = {}
            self._org_capture_active = False

    def capture_names(self, names):
        if self._org_capture_active:
            return set()  # run the capture forward to completion: its outputs are kept
        return super().capture_names(names)

    def _hook_org_outputs(self, block):
        handles = []
        for subset in self.model.get_subsets_in_block(block):
            m = subset.get('inspect')
            if m is None or not subset.get('do_trans', True):
                continue
            lins = [x for x in m.modules() if isinstance(x, (nn.Linear, FakeQuantLinear))]

            def hook(mod, inp, out, _lins=lins):
                if not self._org_capture_active:
                    return
                if id(mod) in self._org_cache:  # called twice in one forward: do not reuse
                    self._org_cache[id(mod)] = None
                    return
                o = out[0] if isinstance(out, tuple) else out
                self._org_cache[id(mod)] = (o.detach(), _mkey(*_lins), _lins)
            handles.append(m.register_forward_hook(hook))
        return handles

    def _org_cached(self, x, inspect_module):
        """The capture forward's output of inspect_module on x, if still valid, else None."""
        hit = getattr(self, '_org_cache', {}).pop(id(inspect_module), None)
        if (getattr(self, 'reuse_org', False) and hit is not None and self._bs == x.shape[0]
                and hit[1] == _mkey(*hit[2]) and tuple(hit[0].shape[:-1]) == tuple(x.shape[:-1])):
            self.org_reuse_stats['reused'] += 1
            return hit[0]
        if hasattr(self, 'org_reuse_stats'):
            self.org_reuse_stats['recomputed'] += 1
        return None

    def _org_output(self, x, inspect_module, kwargs):
        hit = self._org_cached(x, inspect_module)
        return hit if hit is not None else self.inspect_module_forward(x, inspect_module, kwargs)

    # -- awq.py:74-108 ----------------------------------------------------------------------
    def get_act_scale(self, x):
        if x.shape[0] == self._bs:
            return ops.absmean_cols(x)
        means = [ops.absmean_cols(x[i * self._bs:(i + 1) * self._bs])
                 for i in range(x.shape[0] // self._bs)]
        return sum(means) / len(means)

    def get_weight_scale(self, layers_dict):
        """awq.py:48-72 (trans_version v1): one pass per linear, HBM-resident."""
        wq = self.wquantizer
        if wq.granularity != 'per_group':
            raise NotImplementedError('trans_version v1 supports per_group weights')
        return ops.awq_weight_scale([m.weight.data for m in layers_dict.values()],
                                    wq.group_size)

    def get_scales(self, prev_op, x_mean, ratio, out=None, w_max=None):
        return ops.awq_scales(x_mean, ratio, out=out,
                              w_max=w_max if getattr(self, 'trans_version', 'v2') == 'v1'
                              else None)

    def inspect_module_forward(self, x, inspect_module, kwargs):
        if self._bs == x.shape[0]:
            out = inspect_module(x, **kwargs)
            return out[0] if isinstance(out, tuple) else out
        outs = []
        for i in range(x.shape[0] // self._bs):
            o = inspect_module(x[i * self._bs:(i + 1) * self._bs], **kwargs)
            outs.append(o[0] if isinstance(o, tuple) else o)
        return torch.cat(outs, dim=0)

    def fake_quantize_weight(self, fc, scales, out):
        """awq.py:147-164: Q(W * s) in the weight dtype, fused in one kernel for integer
        minmax quantizers; W * s then the quantizer's own fake_quant_weight_dynamic otherwise
        (calib_algo mse / hqq, round_zp False, FloatQuantizer weights: awq_fp8*.yml)."""
        wq = self.wquantizer
        w = fc.weight.data
        if (wq.calib_algo in ('mse', 'hqq') or getattr(wq, 'quant_type', 'int-quant') != 'int-quant'
                or not getattr(wq, 'round_zp', True)):
            ops.scale_bcast(w, scales.to(w.dtype), 'mul', out=out)
            out.copy_(wq.fake_quant_weight_dynamic(out))
            return out
        x2, group = wq._kernel_view(w)
        ops.int_quant_dynamic(x2, group, int(wq.qmin.item()), int(wq.qmax.item()), wq.sym,
                              pre_scale=scales.to(w.dtype), qparams=False, out=out)
        return out

    # -- fused inspect forward + loss (awq.py:110-145 on the lcq GEMM epilogues) ------------
    @staticmethod
    def _qbufs(weights):
        """Buffers for the fake-quantized weights; linears of one input (q/k/v, gate/up) get
        row ranges of ONE buffer, so a fused GEMM reads them as one weight panel."""
        w0 = weights[0]
        if len(weights) > 1 and all(w.dim() == 2 and w.shape[1] == w0.shape[1] and w.dtype ==
                                    w0.dtype and w.device == w0.device for w in weights):
            cat = torch.empty((sum(w.shape[0] for w in weights), w0.shape[1]), dtype=w0.dtype,
                              device=w0.device)
            return list(torch.split(cat, [w.shape[0] for w in weights], dim=0))
        return [torch.empty_like(w) for w in weights]

    fused_search = True  # class switch for A/B runs (LCQ_GEMM=0 also disables it)

    def _fused_paths(self, inspect_module, layers, qbufs, orig_w, kwargs, x):
        """`inspect_module(x/s)` + calculate_loss as lcq GEMM launches whose epilogues do the
        elementwise tail (SiLU product, squared error against org_out), so the module's
        output is never written. Returns (org_fn(x) -> org_out with the original weights,
        loss_factory(org_out, losses) -> fn(xin, slot)), or None for any other module or
        setting (activation quant, awq_bs batching, padding masks: the module forward runs).
        Same math as the module forward on the lcq GEMM (fp32 accumulation, one rounding per
        output), so a reused capture-forward org_out and the ratios' outputs stay comparable."""
        if not (self.fused_search and getattr(self, 'w_only', True)
                and self._bs == x.shape[0] and not getattr(self, 'padding_mask', None)):
            return None
        mods = list(layers)
        if isinstance(inspect_module, nn.Linear) and mods == [inspect_module]:
            b = inspect_module.bias
            if not (ops.gemm_supported(x, *qbufs, *orig_w) and (b is None or b.dtype == x.dtype)):
                return None
            qw = qbufs[0]
            return (lambda xx: ops.linear(xx, orig_w[0], b),
                    lambda org, losses: (lambda xin, n: ops.linear_sq_diff(xin, qw, org, losses,
                                                                           n, bias=b)))
        name = type(inspect_module).__name__
        if name == 'LlamaMLP' and getattr(inspect_module.config, 'hidden_act', None) == 'silu':
            gp, up, dp = inspect_module.gate_proj, inspect_module.up_proj, inspect_module.down_proj
            if not (mods == [gp, up] and gp.bias is None and up.bias is None
                    and isinstance(dp, nn.Linear) and ops.gemm_supported(x, *qbufs, *orig_w)
                    and ops.gemm_supported(x.new_empty((1, dp.weight.shape[1])), dp.weight)
                    and (dp.bias is None or dp.bias.dtype == x.dtype)
                    and qbufs[0].stride(0) == qbufs[1].stride(0)
                    and orig_w[0].stride(0) == orig_w[1].stride(0)):
                return None
            wd, bd = dp.weight, dp.bias

            def org_fn(xx):
                return ops.linear(ops.linear_silu_mul(xx, orig_w[0], orig_w[1]), wd, bd)

            def factory(org, losses):
                return lambda xin, n: ops.linear_sq_diff(
                    ops.linear_silu_mul(xin, qbufs[0], qbufs[1]), wd, org, losses, n, bias=bd)
            return org_fn, factory
        if name == 'LlamaAttention':
            from .llama import _attn_core
            a = inspect_module
            o = a.o_proj
            kw = dict(kwargs)
            pe = kw.pop('position_embeddings', None)
            am = kw.pop('attention_mask', None)
            kw = {k: v for k, v in kw.items() if k in ('position_ids', 'cache_position')}
            if not (mods == [a.q_proj, a.k_proj, a.v_proj] and isinstance(o, nn.Linear)
                    and pe is not None and ops.gemm_supported(x, *qbufs, *orig_w)
                    and ops.gemm_supported(x.new_empty((1, o.weight.shape[1])), o.weight)
                    and (o.bias is None or o.bias.dtype == x.dtype)):
                return None

            def org_fn(xx):
                return ops.linear(_attn_core(a, xx, pe, am, qkv_weights=orig_w, **kw),
                                  o.weight, o.bias)

            def factory(org, losses):
                return lambda xin, n: ops.linear_sq_diff(
                    _attn_core(a, xin, pe, am, qkv_weights=qbufs, **kw), o.weight, org, losses,
                    n, bias=o.bias)
            return org_fn, factory
        return None

    # -- awq.py:178-278 --------------------------------------------------------------------
    @torch.no_grad()
    def search_scale_subset(self, prev_op, layers_dict, input, inspect_module, is_gqa,
                            subset_kwargs):
        if len(input) != 1:
            raise NotImplementedError('multiple calibration tensors per subset')
        x = input[0]
        self._bs = x.shape[0] if self.awq_bs is None else self.awq_bs
        kwargs = subset_kwargs[0] if isinstance(subset_kwargs, list) else subset_kwargs
        layers = list(layers_dict.values())
        # is_gqa (do_gqa_trans, awq.py:88-108 / 40-46): x is v_proj's input; the scales live
        # on v_proj's outputs (act scale of prev_op(x), v2 formula) and multiply o_proj's
        # columns / divide x repeated over the query heads of each kv head
        v1 = getattr(self, 'trans_version', 'v2') == 'v1' and not is_gqa
        w_max = self.get_weight_scale(layers_dict) if v1 else None
        orig_w = [fc.weight.data for fc in layers]
        qbufs = self._qbufs(orig_w)
        x_tmp = torch.empty_like(x)
        x_mean = self.get_act_scale(prev_op(x) if is_gqa else x)
        losses = ops.LossBuffer(self.n_grid, x.device)
        paths = self._fused_paths(inspect_module, layers, qbufs, orig_w, kwargs, x)
        # the capture forward ran o_proj on the attention output, not on this x
        org_out = None if is_gqa else self._org_cached(x, inspect_module)
        if org_out is None:  # recompute: through the fused kernels when the ratios use them
            org_out = (paths[0](x) if paths is not None
                       else self.inspect_module_forward(x, inspect_module, kwargs))
        fused = paths[1](org_out, losses) if paths is not None else None
        all_scales = torch.empty((self.n_grid, x_mean.shape[-1]), dtype=x.dtype,
                                 device=x.device)
        mine = range(self.n_grid)
        shard = self.parallel_mode() == 'shard_search'
        if shard:  # this rank's ratios; the others' loss slots stay 0 for the sum below
            from .parallel import dist_world
            rank, world = dist_world()
            mine = range(rank, self.n_grid, world)
        try:
            for n in mine:
                ratio = n * 1 / self.n_grid
                s = self.get_scales(prev_op, x_mean, ratio, out=all_scales[n], w_max=w_max)
                sw = self.repeat_gqa_scales(s) if is_gqa else s
                for fc, buf in zip(layers, qbufs):
                    fc.weight.data = self.fake_quantize_weight(fc, sw, buf)
                self.scaling_input(x, sw, False, out=x_tmp)
                xin = x_tmp
                if not self.w_only:
                    xin = self.aquantizer.fake_quant_act_dynamic(x_tmp)
                if fused is not None:
                    fused(xin, n)
                else:
                    out = self.inspect_module_forward(xin, inspect_module, kwargs)
                    losses.record(org_out, out, n)
                for fc, w in zip(layers, orig_w):
                    fc.weight.data = w
        finally:
            for fc, w in zip(layers, orig_w):
                fc.weight.data = w
        if shard:  # gather the grid: each slot has exactly one non-zero contributor (exact)
            import torch.distributed as dist
            dist.all_reduce(losses.out, op=dist.ReduceOp.SUM)
        loss_list = losses.out.tolist()  # the one host sync of the search
        best_i, best = -1, float('inf')
        for n, lo in enumerate(loss_list):
            if lo < best:  # strict: the first minimum wins, as the reference's is_best
                best, best_i = lo, n
        self.last_search = {'losses': loss_list, 'best_index': best_i}
        if shard and best_i % world != rank:  # the winner's scales, rebuilt locally (same op)
            self.get_scales(prev_op, x_mean, best_i * 1 / self.n_grid, out=all_scales[best_i],
                            w_max=w_max)
        best_scales = all_scales[best_i].clone()
        if self.parallel_mode() == 'replicate':
            from .parallel import awq_pick_best
            best_scales = awq_pick_best(best, best_scales)  # awq.py:255-273
        return best_scales

    @torch.no_grad()
    def block_transform(self, block, input_feat, block_kwargs):
        if self.trans:
            super().block_transform(block, input_feat, block_kwargs)
        if self.weight_clip:
            n_tok = self.config.get('calib', {}).get('seq_len', None)
            self.auto_clipper.reduce_across_ranks = self.parallel_mode() == 'replicate'
            self.auto_clipper.shard_rows = self.parallel_mode() == 'shard_search'
            self.auto_clipper.run(block, self.block_idx, input_feat, n_sample_token=n_tok)

    @torch.no_grad()
    def subset_transform(self, subset, input_feat, subset_kwargs):
        """awq.py:298-372."""
        layers_dict = subset['layers']
        prev_op = subset['prev_op']
        input_name = subset['input'][0]
        inspect_module = subset['inspect']
        if not subset.get('do_trans', True):
            return
        if len(prev_op) == 0 or prev_op[0] is None:
            return
        layers = list(layers_dict.values())
        if isinstance(prev_op[0], (nn.Linear, FakeQuantLinear)):
            of = prev_op[0].out_features
            is_gqa = False
            if of not in (layers[0].in_features, 2 * layers[0].in_features,
                          3 * layers[0].in_features):
                if not (self.has_gqa and self.do_gqa_trans):
                    return  # 'Cannot apply scale. Do not transform this subset.'
                # awq.py:338-351: search on the input of the linear captured before this one
                # (v_proj: the block's normalized hidden states)
                is_gqa = True
                keys = list(input_feat.keys())
                input_name = keys[keys.index(input_name) - 1]
        elif not is_norm(prev_op[0]):
            return
        else:
            is_gqa = False
        scale = self.search_scale_subset(prev_op[0], layers_dict, input_feat[input_name],
                                         inspect_module, is_gqa, subset_kwargs)
        self.apply_scale(scale, prev_op, layers)
        self.update_input_feat(scale, input_feat, layers_dict, is_gqa)
        if self.save_scale:  # awq.py:367-370
            for n in layers_dict:
                name = f'{self.model.block_name_prefix}.{self.block_idx}.{n}'
                self.act_scales[name] = scale.clone()
