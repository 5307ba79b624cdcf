"""GPTQ (drop-in for llmc ``quantization/gptq.py``).

Same plugin hooks as the reference (block_init / subset_init / layer_init, cache_input_hook ->
add_batch, subset_transform -> layer_transform, w_q / w_qdq with act-order permutation,
deploy). Device differences: the Hessian update is the MFMA SYRK (``lcq_hessian_accum``),
the column loop is the HIP in-block kernel + fp32 trailing GEMM, and layers that read the same
input (q/k/v, gate/up) share one Hessian accumulator instead of accumulating identical copies.
"""
from __future__ import annotations


import torch
import torch.distributed as dist

from . import gptq_core, ops
from .base_blockwise_quantization import BaseBlockwiseQuantization
from .module_utils import _LLMC_LINEAR_TYPES_, _TRANSFORMERS_LINEAR_TYPES_
from .registry import ALGO_REGISTRY
from .utils import world

_LINEAR_TYPES = tuple(_LLMC_LINEAR_TYPES_ + _TRANSFORMERS_LINEAR_TYPES_)


@ALGO_REGISTRY
class GPTQ(BaseBlockwiseQuantization):
    # quant_out at world > 1: each rank forwards its share of the samples, the partial
    # Hessians are summed once per distinct input, the column loop is row-sharded
    sequential_parallel_mode = 'shard_tokens'

    def __init__(self, model, quant_config, input, padding_mask, config, modality='language'):
        super().__init__(model, quant_config, input, padding_mask, config)
        self.model_dtype = next(self.model.model.parameters()).dtype
        self.add_quant_config()
        self.layers_cache = {}
        # the original weights' qparams (buf_scales / zeros / qmax / qmin, gptq.py:27-33 via
        # collect_model_qparams) are taken per block when the block is reached, before any
        # of its weights change: the same values, without a pass over the whole model here
        # (a streamed model's blocks are on the host until visited)

    def add_quant_config(self):
        sp = self.quant_config['special']
        self.true_sequential = sp['true_sequential']
        self.static_groups = sp['static_groups']
        self.actorder = sp['actorder']
        self.percdamp = sp['percdamp']
        self.blocksize = sp['blocksize']
        self.owq = sp.get('owq', False)
        self.chunk_num = sp.get('chunk_num', 1)
        if self.owq:  # gptq.py:44-50
            self.n_outs = sp['n_outs']
            self.static_groups = False
            self.actorder = False
        if self.blocksize != gptq_core.BLOCK:
            raise NotImplementedError('device GPTQ uses blocksize 128')
        self.need_perm = (self.wquantizer.granularity == 'per_group' and not self.static_groups
                          and self.actorder) or self.owq

    def run_block_loop(self):
        try:
            super().run_block_loop()
        finally:
            gptq_core.clear_chain_graphs()  # the chain graphs' pools end with the run

    def _release_device_state(self):
        # a caller that drove block_opt directly (no run_block_loop) leaves the chain graphs
        # captured: their pools (~4-5 n^2 fp32 per Hessian size) go with the algorithm
        gptq_core.release_device_state()

    @torch.no_grad()
    def collect_model_qparams(self):
        for block in self.blocks:
            self.collect_block_qparams(block)

    # ---- Hessian collection (gptq.py:246-322) -------------------------------------------------
    def sample_shard(self, total, rank, world):
        """Token shards on the grouped Hessian's group boundaries (world | 8): rank r takes
        groups [8r/N, 8(r+1)/N), samples [ceil(r n / N), ceil((r + 1) n / N))."""
        if gptq_core.HESSIAN_GROUPS % world == 0:
            return (-(-rank * total // world), -(-(rank + 1) * total // world))
        return super().sample_shard(total, rank, world)

    def _hessian_plan(self):
        """The grouped-Hessian plan of this process (gptq_core.GroupPlan), or None where the
        running average is kept: the reference's data-parallel replicas, or a world that does
        not divide the group count."""
        if self.data_free:
            return None
        mode = self.parallel_mode()
        if mode in ('single', 'shard_blocks', 'replicate'):
            # replicas: every rank's own full tree (the averaging all-reduce of identical
            # replicas is then exact, as on one GPU)
            return gptq_core.GroupPlan(self.n_samples)
        if mode == 'shard_tokens':
            from .parallel import dist_world
            rank, wsz = dist_world()
            if gptq_core.HESSIAN_GROUPS % wsz == 0:
                return gptq_core.GroupPlan(getattr(self, 'n_samples_global', self.n_samples),
                                           rank, wsz)
        return None

    # The reference keeps one Hessian per linear, each fed by that linear's own hook. Linears of
    # one subset read the same tensor (q/k/v, gate/up), so their Hessians are identical: here the
    # subset's input layer (subset['input'][0]) owns one accumulator that its members share.
    def _init_subset(self, subset):
        layers = subset['layers']
        owner = subset['input'][0]
        acc = None
        for name, m in layers.items():
            if acc is None:
                acc = gptq_core.HessianAccumulator(m.weight.shape[1], m.weight.device,
                                                   plan=self._hessian_plan())
            self.layers_cache[name] = {'acc': acc, 'owner': name == owner,
                                       'columns': m.weight.shape[1]}

    @torch.no_grad()
    def subset_init(self, subset):
        self.named_layers = subset['layers']
        self._init_subset(subset)

    @torch.no_grad()
    def block_init(self, block):
        self.named_layers = self.model.get_block_linears(block)
        # the reference collects every block's original-weight qparams at construction
        # (gptq.py __init__ -> collect_model_qparams); here on this instance's first visit of the
        # block (same weights: nothing else has touched them), never reusing buf_scales an
        # earlier pass (HQQ, a reused model) left behind
        done = self.__dict__.setdefault('_qparams_collected', set())
        if self.block_idx not in done:
            self.collect_block_qparams(block)
            done.add(self.block_idx)
        subsets = self.model.get_subsets_in_block(block)
        # with true_sequential the reference re-initialises every later subset's Hessian in
        # rehook_next_subset, so only the first subset's first-pass Hessian is ever used
        for subset in (subsets[:1] if self.true_sequential else subsets):
            self._init_subset(subset)

    def capture_names(self, names):
        """Only the Hessian owners' inputs are consumed (the forward output is discarded)."""
        return {n for n in names if self.layers_cache.get(n, {}).get('owner', False)}

    hook_needs_output = False  # add_batch never reads `out` (gptq.py:253-295)

    @torch.no_grad()
    def cache_input_hook(self, m, inp, out, name, feat_dict):
        if isinstance(m, _LINEAR_TYPES):
            self.add_batch(m, name, inp[0].data, None if out is None else out.data)
        if self.act_static:  # gptq.py:250-251: static act qparams need the inputs themselves
            super().cache_input_hook(m, inp, out, name, feat_dict)

    @torch.no_grad()
    def add_batch(self, layer, name, inp, out):
        """gptq.py:253-295 (one call per calibration batch, on the owner's hook)."""
        entry = self.layers_cache.get(name)
        if entry is None or not entry['owner']:
            return
        v = self.entry_view(layer, inp)
        if isinstance(v, list):  # a routed expert: one sample per entry that reached it
            entry['acc'].add_batch(torch.cat(v, dim=0), samples=len(v))
        else:
            entry['acc'].add_batch(v)

    # ---- transform (gptq.py:96-244) -------------------------------------------------------------
    # Linears fed the same input (q/k/v, gate/up) share H, perm, damping and U, and GPTQ's
    # rows are independent given U, so their column loops run as ONE loop over
    # the concatenated rows: the same per-row arithmetic (each element's update order is fixed
    # by its column, not by the row count), one latency-bound chain of block / trailing kernels
    # instead of one per linear. (Tests set concat_rows False to quantize them one by one.)
    concat_rows = True

    @torch.no_grad()
    def block_transform(self, block, input_feat=None, block_kwargs=None):
        if getattr(self, 'owq', False) and not hasattr(self, 'n_out_dict'):  # gptq.py:298-306
            names = list(self.model.get_block_linears(block).keys())
            self.n_out_dict = {n: self.n_outs[i] for i, n in enumerate(names)}
        super().block_transform(block, input_feat, block_kwargs)

    def _n_out(self, name):
        return self.n_out_dict[name] if getattr(self, 'owq', False) else 0

    def _owq_pad_groups(self, r, layers, rows_total, cols):
        """OWQ: groups past the last quantized column keep the construction qparams the
        reference seeded `groups` with (search_group_qparams, gptq.py:383-396; only the
        searched ones are overwritten) -- merged into buf_scales / buf_zeros in group order."""
        if r['scales'] is None or self.wquantizer.granularity != 'per_group':
            return r
        ng_all = -(-cols // self.wquantizer.group_size)
        ng_q = r['scales'].shape[0] // rows_total
        if ng_q >= ng_all:
            return r
        for key, buf in (('scales', 'buf_scales'), ('zeros', 'buf_zeros')):
            if r[key] is None:
                continue
            orig = torch.cat([getattr(m, buf).reshape(m.weight.shape[0], ng_all) for m in layers])
            got = r[key].reshape(rows_total, ng_q)
            r[key] = torch.cat([got, orig[:, ng_q:].to(got.dtype)], 1).reshape(-1, 1)
        return r

    @torch.no_grad()
    def subset_transform(self, subset, input_feat, subset_kwargs):
        groups = {}
        for name, layer in subset['layers'].items():
            if not isinstance(layer, _LINEAR_TYPES):
                continue
            acc = self.layers_cache[name]['acc']
            # OWQ's permutation depends on the layer's n_out: share only equal ones
            groups.setdefault((id(acc), self._n_out(name)), []).append((name, layer))
        for grp in groups.values():
            if len(grp) > 1 and self.concat_rows:
                self.group_transform(grp)
            else:
                for name, layer in grp:
                    self.layer_transform(layer, name)
            for name, _ in grp:
                self.free(name)

    def _prepared(self, acc, replicate, ws, nout=0):
        cache = getattr(acc, 'prepared_by', None)
        if cache is None:
            cache = acc.prepared_by = {}
        if nout not in cache:
            grouped = acc.ready_grouped()
            shard = replicate and self.parallel_mode() == 'shard_tokens'
            if shard:
                # every rank must take the same road: grouped only if all ranks are
                flag = torch.tensor([int(grouped)], dtype=torch.int32, device=acc.H.device)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                if grouped and not int(flag.item()):
                    acc.fallback()
                    grouped = False
            # grouped: the fixed group tree (finished across the token shards when sharded:
            # bit-identical to one GPU, nothing else to reduce)
            H = (acc.finalize() if grouped else acc.H).clone()
            if shard and grouped:
                pass
            elif shard:
                # token shards: H = sum_r n_r H_r / N (each H_r the running average over the
                # rank's n_r samples) -- the single-GPU Hessian up to fp32 summation order
                n = torch.tensor([float(acc.nsamples)], dtype=torch.float64, device=H.device)
                H *= float(acc.nsamples)
                dist.all_reduce(H, op=dist.ReduceOp.SUM)
                dist.all_reduce(n, op=dist.ReduceOp.SUM)
                if n.item() > 0:  # no sample on any rank (an expert no token reached): H
                    H /= float(n.item())  # stays 0 as on one GPU -> dead-column path
            elif replicate:
                # one all-reduce of the finished Hessian per distinct input (the reference
                # reduces after every sample); averaging matches its H /= world_size
                dist.all_reduce(H, op=dist.ReduceOp.SUM)
                H /= ws
            # every rank now holds the same H: the factorisation's large products are
            # row-split over the ranks (bit-identical to one GPU; gptq_core.chain_sharding)
            rank = dist.get_rank() if replicate else 0
            with gptq_core.chain_sharding(rank, ws if replicate else 1):
                cache[nout] = gptq_core.prepare_hessian(H, self.actorder, self.percdamp, nout)
        acc.prepared = cache[nout]
        return acc.prepared

    @torch.no_grad()
    def group_transform(self, grp):
        """layer_transform of several linears sharing one Hessian, as one column loop."""
        acc = self.layers_cache[grp[0][0]]['acc']
        _, ws, _ = world()
        replicate = ws > 1 and dist.is_initialized() and self.parallel_mode() in (
            'replicate', 'shard_tokens')
        nout = self._n_out(grp[0][0])
        prepared = self._prepared(acc, replicate, ws, nout)
        W = torch.cat([layer.weight.data for _, layer in grp], 0)
        fixed = None
        if self.wquantizer.granularity != 'per_group' or self.static_groups:
            s = torch.cat([layer.buf_scales.reshape(-1, 1) for _, layer in grp], 0)
            z = None if self.wquantizer.sym else torch.cat(
                [layer.buf_zeros.reshape(-1, 1) for _, layer in grp], 0)
            fixed = (s, z)
        r = gptq_core.quantize_layer(W, None, self.wquantizer, actorder=self.actorder,
                                     percdamp=self.percdamp, fixed=fixed, shard_rows=replicate,
                                     prepared=prepared, static_groups=self.static_groups,
                                     owq_nout=nout)
        if getattr(self, 'owq', False):
            r = self._owq_pad_groups(r, [layer for _, layer in grp], W.shape[0], W.shape[1])
        ng = 1 if r['scales'] is None else r['scales'].shape[0] // W.shape[0]
        o0 = 0
        for _, layer in grp:
            o1 = o0 + layer.weight.shape[0]
            layer.weight.data = r['weight'][o0:o1].clone()
            if r['perm'] is not None:
                layer.register_buffer('buf_perm', r['perm'])
                layer.register_buffer('buf_invperm', r['invperm'])
            if getattr(self, 'owq', False):
                layer.register_buffer('buf_n_nonout', torch.tensor(W.shape[1] - nout))
            if r['scales'] is not None:
                layer.buf_scales = r['scales'][o0 * ng:o1 * ng].clone()
                if not self.wquantizer.sym:
                    layer.buf_zeros = r['zeros'][o0 * ng:o1 * ng].clone()
            o0 = o1

    @torch.no_grad()
    def layer_transform(self, layer, name):
        acc = self.layers_cache[name]['acc']  # shared by the linears fed the same input
        _, ws, _ = world()
        replicate = ws > 1 and dist.is_initialized() and self.parallel_mode() in (
            'replicate', 'shard_tokens')
        nout = self._n_out(name)
        prepared = self._prepared(acc, replicate, ws, nout)
        fixed = None
        if self.wquantizer.granularity != 'per_group' or self.static_groups:
            fixed = (layer.buf_scales, getattr(layer, 'buf_zeros', None))
        r = gptq_core.quantize_layer(layer.weight.data, None, self.wquantizer,
                                     actorder=self.actorder, percdamp=self.percdamp,
                                     fixed=fixed, shard_rows=replicate, prepared=prepared,
                                     static_groups=self.static_groups, owq_nout=nout)
        if getattr(self, 'owq', False):
            r = self._owq_pad_groups(r, [layer], layer.weight.shape[0], layer.weight.shape[1])
        layer.weight.data = r['weight']
        if r['perm'] is not None:
            layer.register_buffer('buf_perm', r['perm'])
            layer.register_buffer('buf_invperm', r['invperm'])
        if getattr(self, 'owq', False):
            layer.register_buffer('buf_n_nonout', torch.tensor(layer.weight.shape[1] - nout))
        if r['scales'] is not None:
            layer.buf_scales = r['scales']
            if not self.wquantizer.sym:
                layer.buf_zeros = r['zeros']

    @torch.no_grad()
    def free(self, name):
        self.layers_cache.pop(name, None)

    # ---- deploy (gptq.py:411-459) --------------------------------------------------------------
    @torch.no_grad()
    def w_q(self, module, wquantizer):
        args = {'scales': module.buf_scales.to(self.model_dtype),
                'zeros': getattr(module, 'buf_zeros', None),
                'qmax': module.buf_qmax, 'qmin': module.buf_qmin}
        return wquantizer.real_quant_weight_static(module.weight.data, args)

    @torch.no_grad()
    def w_qdq(self, module, wquantizer):
        if getattr(self, 'owq', False):  # gptq.py:424-452: outlier columns stay in float
            w = module.weight[:, module.buf_perm].contiguous()
            nn_ = int(module.buf_n_nonout)
            args = {'scales': module.buf_scales, 'zeros': getattr(module, 'buf_zeros', None),
                    'qmax': module.buf_qmax, 'qmin': module.buf_qmin}
            fq = wquantizer.fake_quant_weight_static(w, args).to(self.model_dtype)
            fq[:, nn_:] = w[:, nn_:].to(self.model_dtype)
            return fq[:, module.buf_invperm].contiguous()
        fast = self._w_qdq_cols(module, wquantizer)
        if fast is not None:
            return fast
        weight = module.weight
        if self.need_perm:
            weight = module.weight[:, module.buf_perm].contiguous()
        args = {'scales': module.buf_scales, 'zeros': getattr(module, 'buf_zeros', None),
                'qmax': module.buf_qmax, 'qmin': module.buf_qmin}
        weight = wquantizer.fake_quant_weight_static(weight, args).to(self.model_dtype)
        if self.need_perm:
            weight = weight[:, module.buf_invperm].contiguous()
        return weight

    @torch.no_grad()
    def _w_qdq_cols(self, module, wquantizer):
        """w_qdq under act-order, per-group int quant: fake_quant_static(W[:, perm])[:, invperm]
        as ONE pass over W in its own column order (lcq_int_quant_static_cols: column c takes
        group invperm[c] // group) -- the same per-element arithmetic without the two column
        gathers. None when the layout is not that case."""
        from .quant import IntegerQuantizer
        if not (self.need_perm and isinstance(wquantizer, IntegerQuantizer)
                and wquantizer.granularity == 'per_group' and module.weight.dim() == 2
                and module.weight.is_cuda and module.weight.shape[1] % 8 == 0):
            return None
        W = module.weight.data
        s = module.buf_scales
        z = getattr(module, 'buf_zeros', None)
        zz = z if (torch.is_tensor(z) and z.dim() > 0) else None
        if zz is None and torch.is_tensor(z) and z.numel() == 1 and float(z) != 0:
            return None
        cg = getattr(module, '_lcq_cgroup', None)
        if cg is None or cg.numel() != W.shape[1]:
            cg = (module.buf_invperm // wquantizer.group_size).to(torch.int32).contiguous()
            module._lcq_cgroup = cg
        ct = torch.promote_types(W.dtype, s.dtype)   # quant.py _static's compute dtype
        if zz is not None and zz.is_floating_point():
            ct = torch.promote_types(ct, zz.dtype)
        qmin, qmax = wquantizer._iq
        return ops.int_quant_static_cols(W, cg, s.reshape(-1), None if zz is None else
                                         zz.reshape(-1), qmin, qmax, ct_dtype=ct,
                                         fq_dtype=self.model_dtype)

    @torch.no_grad()
    def deploy(self, quant_format, keep_device=True):
        if quant_format not in ('fake_quant', 'origin_float'):
            assert not self.need_perm
        super().deploy(quant_format)
        self.model.convert_dtype(self.model_dtype)

    @torch.no_grad()
    def save_model(self, path):
        self.model.convert_dtype(self.model_dtype)
        super().save_model(path)
