"""Block-wise driver + quantization plugin base (drop-in for llmc
``compression/blockwise_optimization.py`` and ``quantization/base_blockwise_quantization.py``).

Same hook points and call order as the reference (block_opt -> run -> block_transform ->
subset_transform, true_sequential re-hooking, quant_out forwarding, deploy / save_model) so the
reference's algorithm subclasses and YAML configs keep working. MI355X-first differences:

* the whole model stays resident in HBM (288 GB holds Llama-3-70B bf16), so there are no
  per-block ``.cuda()/.cpu()`` round trips;
* cached linear inputs stay on the device and are shared, not copied, between linears that
  read the same tensor (q/k/v, gate/up) — the reference keeps one CPU copy per linear;
* every weight/activation transform (AWQ scaling, clipping, fake/real quant, packing) is a HIP
  kernel from ``liblcq.so``; block forwards are the model's own torch modules.
"""
from __future__ import annotations

import functools
import gc
from collections import defaultdict
from functools import partial

import torch
import torch.distributed as dist
import torch.nn as nn

from . import ops
from . import parallel as P
from .base_model import retire_module
from .module_utils import (_LLMC_LINEAR_TYPES_, _REALQUANT_LINEAR_MAP_,
                           _TRANSFORMERS_LINEAR_TYPES_, EffcientFakeQuantLinear,
                           FakeQuantLinear, OriginFloatLinear)
from .quant import FloatQuantizer, IntegerQuantizer
from .utils import world

_LINEAR_TYPES = tuple(_LLMC_LINEAR_TYPES_ + _TRANSFORMERS_LINEAR_TYPES_)


def is_norm(m) -> bool:
    """RMSNorm / LayerNorm of any HF model (the reference registers them per adapter)."""
    n = type(m).__name__.lower()
    return isinstance(m, nn.LayerNorm) or n.endswith('rmsnorm') or n.endswith('layernorm')


class BlockwiseOpt:
    """llmc/compression/blockwise_optimization.py:8-114."""

    def __init__(self, model, compress_config, input, padding_mask, config):
        self.model = model
        self.blocks = model.get_blocks()
        self.quant_config = compress_config
        self.input = input
        self.padding_mask = padding_mask
        self.data_free = not input
        self.config = config
        self.block_idx = None
        self.num_blocks = len(self.blocks)
        if self.input:
            for kw in input['kwargs']:
                kw.pop('use_cache', None)
                if 'past_key_value' in kw:
                    kw['past_key_value'] = None
                if 'past_key_values' in kw:
                    kw['past_key_values'] = None
            self.n_samples = sum(d.shape[0] for d in input['data'])
        calib = (config or {}).get('calib', {}) or {}
        self.batch_calib = bool(calib.get('batch_forward', True))
        self._batch_ok = None
        if self.input and self.parallel_mode() == 'shard_tokens':
            self._shard_input_tokens()

    def release(self):
        """Give back what this algorithm object holds on the device beyond the model: the
        calibration inputs and per-block caches, the algorithm's device-side caches
        (_release_device_state: GPTQ's captured chain graphs and their pools), the reference
        cycles that deployed modules form through their quant callables (module.a_qdq ->
        algorithm -> model), and the caching allocator's free blocks. The reference collects
        after every block (base_blockwise_quantization.py:420: gc.collect() +
        torch.cuda.empty_cache()); a finished run -- or a caller that drove block_opt itself --
        calls this once. deploy / save_model still work afterwards (they read the model only)."""
        self.input = None
        for name in ('layers_cache', '_org_cache'):
            c = self.__dict__.get(name)
            if isinstance(c, dict):
                c.clear()
        self._release_device_state()
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    def _release_device_state(self):
        """Algorithm-specific device caches (overridden by GPTQ)."""

    # how ranks split a block whose input depends on the previous block's quantization
    # (quant_out True): 'shard_search' (AWQ: the ratio grid and the clip rows),
    # 'shard_tokens' (GPTQ: calibration samples, partial Hessians summed), or 'replicate'
    # (the reference's data-parallel replicas with averaged statistics)
    sequential_parallel_mode = 'replicate'

    def parallel_mode(self) -> str:
        """'single' | 'shard_blocks' | 'shard_units' | 'shard_search' | 'shard_tokens' |
        'replicate'.

        Blocks can be sharded when each block's input does not depend on the quantization of
        the previous one (quant_out False); otherwise the work inside a block
        is sharded (sequential_parallel_mode) or ranks run the reference's data-parallel
        replica scheme (special.parallel: replicate). The sharded modes reproduce the
        single-GPU result (bit for bit, or to GPTQ's Hessian summation order)."""
        _, world = P.dist_world()
        if world == 1:
            return 'single'
        mode = (self.quant_config.get('special', {}) or {}).get('parallel', None)
        if mode:
            return mode
        if self.data_free:
            return 'shard_units'   # independent linears / experts
        if not self.quant_config.get('quant_out', False):
            return 'shard_blocks'
        return self.sequential_parallel_mode

    def _shard_input_tokens(self):
        """shard_tokens: keep this rank's contiguous share of the calibration samples (the
        reference's per-rank slicing, base_dataset.py:169-184, of ONE global set), entries
        and their batch-dim kwargs sliced alike."""
        rank, world = P.dist_world()
        data, kws = self.input['data'], self.input['kwargs']
        total = sum(d.shape[0] for d in data)
        s, e = self.sample_shard(total, rank, world)
        new_d, new_k, off = [], [], 0
        for d, kw in zip(data, kws):
            b = d.shape[0]
            lo, hi = max(s, off), min(e, off + b)
            if hi > lo:
                new_d.append(d[lo - off:hi - off])
                new_k.append({k: (v[lo - off:hi - off] if torch.is_tensor(v) and v.dim() > 0
                                  and v.shape[0] == b and b > 1 else v) for k, v in kw.items()})
            off += b
        self.input['data'], self.input['kwargs'] = new_d, new_k
        self.global_entry_sizes = [d.shape[0] for d in data]
        self.n_samples_global = total
        self.n_samples = e - s

    def sample_shard(self, total: int, rank: int, world: int) -> tuple[int, int]:
        """[start, end) of this rank's calibration samples under shard_tokens."""
        return P.row_shard(total, rank, world)

    def run_block_loop(self):
        self._in_block_loop = True
        try:
            self._block_loop()
        finally:
            self._in_block_loop = False

    def _block_loop(self):
        mode = self.parallel_mode()
        rank, world = P.dist_world()
        own = getattr(self.model, 'ownership', None)
        if own is not None and own.mode != mode:
            raise RuntimeError(f'model materialised for {own.mode}, algorithm runs {mode}')
        if mode == 'shard_blocks' and not self.data_free and self._handoff_ok():
            self._run_block_loop_ring(rank, world)
            return
        if own is not None and mode == 'shard_blocks':
            raise NotImplementedError('materialize: owned with shard_blocks needs the ring '
                                      'pipeline (tensor block inputs, the base block_opt)')
        n = len(self.blocks)
        for i in range(n):
            self.block_idx = i
            if mode == 'shard_blocks' and i % world != rank:
                # not ours: only advance the float activation chain (quant_out False); the
                # staged forward's memo of this block (stage outputs: GBs at calibration
                # sizes) is dropped at once, as block_opt does for owned blocks
                if not self.data_free:
                    def fwd(i=i):
                        self.input['data'] = self.block_forward(self.blocks[i])
                        self._clear_block_cache(self.blocks[i])
                    self.visit_block(i, fwd, next_i=i + 1, dirty=False)
                continue
            if not self.block_has_work():
                continue   # nothing to do per block (weight-only RTN): deploy streams itself
            self.visit_block(i, lambda i=i: self.block_opt(self.blocks[i]), next_i=i + 1)
        self._drain_blocks()
        if mode == 'shard_blocks':
            # blocks stay on their owners until it is known what the other ranks need: a
            # real-quant deploy gathers the quantized shards only (packed codes + scales,
            # P.publish), anything else the transformed float blocks (materialize)
            self._pending_owner = {i: i % world for i in range(len(self.blocks))}
        self.save_transforms()

    def block_has_work(self) -> bool:
        """Whether block_opt does anything (RTN weight-only: no -- its blocks are not even
        uploaded by a streaming run's block loop)."""
        return True

    # ---- block residency (residency.py) --------------------------------------------------
    def visit_block(self, i, fn, next_i=None, dirty=True):
        """Run fn with block i in HBM. Streaming models upload block i (or take the prefetch
        already in flight), start block next_i's upload on the H2D stream, run fn, and write
        block i back on the D2H stream (``dirty`` False: forward only, nothing to write)."""
        st = getattr(self.model, 'streamer', None)
        if st is None:
            return fn()
        st.fetch(i)
        if next_i is not None:
            st.prefetch(next_i)
        try:
            return fn()
        finally:
            st.evict(i, dirty=dirty)

    def _drain_blocks(self):
        st = getattr(self.model, 'streamer', None)
        if st is not None:
            st.drain()

    def _handoff_ok(self):
        """The ring hand-off passes self.input['data'] as a list of tensors whose shapes every
        rank already knows (block outputs have their inputs' shapes)."""
        data = self.input.get('data') if isinstance(self.input, dict) else None
        return (bool(data) and all(torch.is_tensor(t) for t in data)
                and type(self).block_opt is BaseBlockwiseQuantization.block_opt)

    def _run_block_loop_ring(self, rank, world):
        """shard_blocks as a ring pipeline: the owner of block i forwards it first (the float
        output is the next block's input, quant_out False), hands that output to the owner of
        block i + 1 over the ring edge, and only then runs the long transform. A rank touches
        only its own blocks: no rank replays the float chain of the blocks before its own."""
        groups = P.ring_groups(world)
        n = len(self.blocks)
        for i in range(rank, n, world):
            if i > 0:  # this block's input: the float output of block i - 1
                src = (i - 1) % world
                self.input['data'] = [torch.empty_like(t) for t in self.input['data']]
                P.pass_tensors(self.input['data'], src, groups[src])
            self.block_idx = i
            self._handoff = (rank, groups[rank]) if i + 1 < n else None
            self.visit_block(i, lambda i=i: self.block_opt(self.blocks[i]), next_i=i + world)
            # every owner of a non-last block hands its output on exactly once (run() does it
            # right after the forward; a path that did not forward must not leave the next
            # owner waiting)
            self._send_handoff()
        self._drain_blocks()
        self._pending_owner = {i: i % world for i in range(n)}
        self.save_transforms()

    def _send_handoff(self):
        h = getattr(self, '_handoff', None)
        if h is not None:
            P.pass_tensors(self.input['data'], h[0], h[1])
            self._handoff = None

    def materialize_blocks(self):
        """shard_blocks: publish every transformed float block from its owner (the state one
        GPU would hold after run_block_loop); a no-op otherwise or once done."""
        pending = getattr(self, '_pending_owner', None)
        if not pending:
            return
        if getattr(self.model, 'ownership', None) is not None:
            raise RuntimeError('materialize: owned -- this rank holds only its own blocks '
                               '(save_model writes per-rank shards)')

        def pub(block, owner):
            P.broadcast_block(block, owner=owner)
            # the broadcast writes weights through .data (no version bump): no memoised
            # stage may survive it
            self._clear_block_cache(block)
        for i, block in enumerate(self.blocks):
            self.visit_block(i, lambda b=block, o=pending[i]: pub(b, o), next_i=i + 1)
        self._drain_blocks()
        self._pending_owner = None

    def save_transforms(self):
        """blockwise_optimization.py:40-52: the AWQ scales (save_scale) and v2 clip factors
        (save_clip) as scales.pth / clips.pth, the files OmniQuant's LET / LWC load. Under
        shard_blocks every rank holds its own blocks' entries: they are merged on rank 0,
        which alone writes."""
        import os
        want_s = getattr(self, 'save_scale', False) and hasattr(self, 'act_scales')
        want_c = getattr(self, 'save_clip', False) and hasattr(self, 'auto_clipper')
        if not (want_s or want_c):
            return
        rank, world = P.dist_world()
        scales = dict(getattr(self, 'act_scales', {}))
        clips = dict(self.auto_clipper.weight_clips) if want_c else {}
        if world > 1 and self.parallel_mode() == 'shard_blocks':
            got = [None] * world
            dist.all_gather_object(got, ({k: v.cpu() for k, v in scales.items()}, clips))
            scales, clips = {}, {}
            for sc, cl in got:
                scales.update(sc)
                clips.update(cl)
            clips = dict(sorted(clips.items()))
        if rank != 0:
            return
        if want_s:
            os.makedirs(self.scale_path, exist_ok=True)
            torch.save(scales, os.path.join(self.scale_path, 'scales.pth'))
            if getattr(self, 'act_shifts', None):
                torch.save(self.act_shifts, os.path.join(self.scale_path, 'shifts.pth'))
        if want_c:
            os.makedirs(self.clip_path, exist_ok=True)
            torch.save(clips, os.path.join(self.clip_path, 'clips.pth'))

    def _clear_block_cache(self, block):
        if hasattr(self.model, 'clear_block_cache'):
            self.model.clear_block_cache(block)

    # rows (tokens) of each calibration entry while block_forward runs several entries as one
    # stacked batch, else None; entries may differ in batch size (a token shard can cut an
    # entry part-way, _shard_input_tokens)
    _batch_ctx = None

    def entry_view(self, m, inp):
        """A linear input captured during a stacked forward, as the reference's per-entry
        forwards would have seen it. 3-D inputs carry the entries in their batch dim already.
        A 2-D input (OPT's MLP, routed MoE experts) counts as ONE sample per forward in the
        reference (cache_input_hook / add_batch unsqueeze it), so here it is split back:
        a dense one (every token of every entry) is viewed [entries, tokens, C]; a routed
        one (ExpertList tags each expert's linears with the global token index of every row)
        becomes the list of its non-empty per-entry row blocks, in entry order, each in the
        order the reference's single-entry forward produces them. Other inputs pass as is."""
        counts = self._batch_ctx
        if counts is None or inp.dim() != 2:
            return inp
        n = len(counts)
        rows = getattr(m, '_lcq_rows', None)
        if rows is None or rows.numel() != inp.shape[0]:
            if inp.shape[0] != sum(counts):
                return inp
            if all(c == counts[0] for c in counts):
                return inp.view(n, counts[0], inp.shape[-1])
            return list(torch.split(inp, counts, dim=0))
        bounds = torch.tensor(counts, device=rows.device).cumsum(0)[:-1]
        ent = torch.bucketize(rows, bounds, right=True)
        order = torch.argsort(ent, stable=True)
        counts = torch.bincount(ent, minlength=n).tolist()
        xs = inp.index_select(0, order)
        return [t for t in torch.split(xs, counts, dim=0) if t.shape[0] > 0]

    def cache_input_hook(self, m, x, y, name, feat_dict):
        # device-resident, shared (no copy): see module docstring
        inputs = [t.detach() for t in x]
        if len(inputs) == 1:
            inp = self.entry_view(m, inputs[0])
            if isinstance(inp, list):  # per-entry row blocks of a routed expert
                feat_dict[name].extend(t.unsqueeze(0) for t in inp)
                return
            if inp.dim() == 2:
                inp = inp.unsqueeze(0)
            feat_dict[name].append(inp)
        else:
            feat_dict[name].append(tuple(inputs))

    def block_opt(self, block):
        raise NotImplementedError

    def layer_init(self, layer, name=None):
        pass

    def subset_init(self, subset):
        pass

    def block_init(self, block):
        pass


class _StopForward(Exception):
    """Raised by a capture hook once every input a discarded forward exists for is captured."""


def _same(a, b):
    if a is b:
        return True
    if torch.is_tensor(a) or torch.is_tensor(b):
        return (torch.is_tensor(a) and torch.is_tensor(b) and a.shape == b.shape
                and a.dtype == b.dtype and a.device == b.device and torch.equal(a, b))
    if isinstance(a, (tuple, list)):
        return (isinstance(b, (tuple, list)) and len(a) == len(b)
                and all(_same(x, y) for x, y in zip(a, b)))
    if isinstance(a, dict):
        return (isinstance(b, dict) and a.keys() == b.keys()
                and all(_same(a[k], b[k]) for k in a))
    try:
        return bool(a == b)
    except Exception:
        return False


def _batchable(inputs, kwargs):
    """Several entries of equal sample shape whose kwargs (rotary tables, masks, positions)
    agree; a per-sample attention mask (padding) keeps the per-sample loop. Entries of
    different batch sizes (calibration sets of unequal batches, or a token shard that cut an
    entry) stack only when no kwarg tensor carries a batch dim."""
    if len(inputs) < 2 or len(kwargs) != len(inputs):
        return False
    s0 = inputs[0].shape
    if any(x.shape[1:] != s0[1:] for x in inputs):
        return False
    def tensors(v):
        if torch.is_tensor(v):
            yield v
        elif isinstance(v, (tuple, list)):
            for u in v:
                yield from tensors(u)

    if any(x.shape[0] != s0[0] for x in inputs) and any(
            t.dim() > 0 and t.shape[0] > 1
            for kw in kwargs for v in kw.values() for t in tensors(v)):
        return False
    if any(torch.is_tensor(v) and v.dim() > 0 and v.shape[0] == s0[0] and k == 'attention_mask'
           for k, v in kwargs[0].items()):
        return False
    return all(_same(kwargs[0], kw) for kw in kwargs[1:])


class BaseBlockwiseQuantization(BlockwiseOpt):
    """llmc/compression/quantization/base_blockwise_quantization.py:41-1029 (hot-path part)."""

    def __init__(self, model, quant_config, input, padding_mask, config):
        super().__init__(model, quant_config, input, padding_mask, config)
        self.dev = torch.device('cuda', torch.cuda.current_device()) \
            if torch.cuda.is_available() else torch.device('cpu')
        self.set_quant_config()

    # ---- weight / activation quant callbacks (:46-82) ---------------------------------------
    def w_qdq(self, module, wquantizer):
        """:46-66; block-fp8 weights (DeepSeek-V3 checkpoints) round-trip through bf16 with
        the kernel.py casts, which the reference selects on FP8-capable GPUs (:20-26)."""
        args = {'lowbound_factor': getattr(module, 'buf_lowbound_factor', None),
                'upbound_factor': getattr(module, 'buf_upbound_factor', None)}
        if module.weight.data.dtype == torch.float8_e4m3fn:
            from .kernel import weight_cast_to_bf16, weight_cast_to_fp8
            bs = getattr(self, 'fp8_block_size', 128)
            tmp = weight_cast_to_bf16(module.weight, module.weight_scale_inv,
                                      bs).to(torch.bfloat16)
            tmp = wquantizer.fake_quant_weight_dynamic(tmp, args)
            tmp, module.weight_scale_inv.data = weight_cast_to_fp8(tmp, bs)
            return tmp
        return wquantizer.fake_quant_weight_dynamic(module.weight, args)

    def w_q(self, module, wquantizer):
        return wquantizer.real_quant_weight_dynamic(module.weight.data)

    def a_qdq(self, act, module, aquantizer, input_index=0):
        if self.act_static:
            args = {k: getattr(module, f'buf_act_{k}_{input_index}', None)
                    for k in ('scales', 'zeros', 'qmax', 'qmin')}
            return aquantizer.fake_quant_act_static(act, args)
        return aquantizer.fake_quant_act_dynamic(act)

    def get_replacement_params(self, mode='fake_quant', w_only=False, name=None):
        params = {}
        if mode in ('fake_quant', 'fake_quant_wo_kv'):
            params['a_qdq'] = None if w_only else partial(self.a_qdq, aquantizer=self.aquantizer)
            params['w_qdq'] = partial(self.w_qdq, wquantizer=self.wquantizer)
        elif mode in _REALQUANT_LINEAR_MAP_:
            params['w_q'] = partial(self.w_q, wquantizer=self.wquantizer)
            params['quant_config'] = self.quant_config
        return params

    # ---- config (:133-268) ---------------------------------------------------------------
    def set_quant_config(self):
        qc = self.quant_config
        self.mixed_precision = 'ignored_layers' in self.config
        self.quant_out = qc.get('quant_out', False)
        self.tp = qc.get('tp', 1)
        qc['weight']['tp'] = self.tp
        qtype = qc['weight'].get('quant_type', 'int-quant')
        self.weight_quant_module = IntegerQuantizer if qtype == 'int-quant' else FloatQuantizer
        self.wquantizer = self.weight_quant_module(**qc['weight'])
        if 'act' in qc:
            self.w_only = False
            atype = qc['act'].get('quant_type', 'int-quant')
            self.act_quant_module = IntegerQuantizer if atype == 'int-quant' else FloatQuantizer
            qc['act']['tp'] = self.tp
            self.aquantizer = self.act_quant_module(**qc['act'])
            self.act_static = qc['act'].get('static', False)
            if self.act_static:
                assert qc['act']['granularity'] == 'per_tensor', \
                    'Only support per_tensor static quant'
            for k in ('quant_attn', 'quant_act_fn'):
                if qc['act'].get(k, False):
                    raise NotImplementedError(f'act.{k} (non-linear quant) is out of scope')
        else:
            self.w_only, self.aquantizer, self.act_static = True, None, False
        self.quant_kvcache = 'kvcache' in qc
        if self.quant_kvcache:
            raise NotImplementedError('kv-cache quantization is out of scope (SURVEY.md §2)')
        special = qc.get('special', {}) or {}
        self.true_sequential = special.get('true_sequential', False)
        self.weight_clip = special.get('weight_clip', False)
        if self.weight_clip or special.get('search_clip_init', False):
            from .auto_clip import AutoClipper
            self.save_clip = special.get('save_clip', False)
            if self.save_clip:
                self.clip_path = special['clip_path']
            self.clip_version = special.get('clip_version', 'v1')
            if self.clip_version == 'v2':
                assert self.wquantizer.calib_algo == 'learnable'
            clip_sym = special.get('clip_sym', self.wquantizer.sym)
            self.auto_clipper = AutoClipper(w_only=self.w_only, wquantizer=self.wquantizer,
                                            aquantizer=self.aquantizer,
                                            clip_version=self.clip_version, clip_sym=clip_sym,
                                            save_clip=self.save_clip,
                                            padding_mask=self.padding_mask)
        self.save_scale = special.get('save_scale', False)
        if self.save_scale:
            self.scale_path = special['scale_path']
            self.act_scales = {}
        self.online_rotate = special.get('online_rotate', False)
        if self.online_rotate:
            raise NotImplementedError('online rotation (QuaRot) is out of scope')
        self.modality = qc.get('modality', 'language')
        self.set_model_config()
        self.do_gqa_trans = special.get('do_gqa_trans', False)

    def set_model_config(self):
        mc = self.model.model_config
        self.hidden_size = mc.hidden_size
        self.num_heads = mc.num_attention_heads
        self.head_dim = getattr(mc, 'head_dim', None) or self.hidden_size // self.num_heads
        self.intermediate_size = getattr(mc, 'intermediate_size', None)
        kv = getattr(mc, 'num_key_value_heads', None)
        if kv is not None:
            self.num_key_value_heads = kv
            self.num_key_value_groups = self.num_heads // kv
            self.has_gqa = self.num_key_value_groups > 1
        else:
            self.has_gqa = False

    # ---- block driver (:337-526) -----------------------------------------------------------
    @torch.no_grad()
    def collect_block_qparams(self, block):
        for n, m in self.model.get_block_linears(block).items():
            _, s, z, qmax, qmin = self.wquantizer.get_tensor_qparams(m.weight.data)
            m.register_buffer('buf_scales', s.detach())
            m.register_buffer('buf_zeros', z.detach() if torch.is_tensor(z) else torch.tensor(z))
            m.register_buffer('buf_qmax', qmax.clone().to(m.weight.device))
            m.register_buffer('buf_qmin', qmin.clone().to(m.weight.device))

    @torch.no_grad()
    def capture_names(self, names):
        """Hooked modules whose inputs a forward exists to capture (all of them by default;
        GPTQ narrows this to the Hessian owners)."""
        return set(names)

    # cache_input_hook reads only the module's input (GPTQ's add_batch, gptq.py:245-295): the
    # forward that exists to capture inputs stops BEFORE the last needed module runs
    hook_needs_output = True

    def _capture_hook(self, m, x, y, name, feat_dict):
        self.cache_input_hook(m, x, y, name=name, feat_dict=feat_dict)
        pending = getattr(self, '_capture_pending', None)
        if pending is not None:
            pending.discard(name)
            if not pending:
                raise _StopForward

    def _capture_pre_hook(self, m, x, name, feat_dict):
        pending = getattr(self, '_capture_pending', None)
        if pending is not None and pending == {name}:
            self.cache_input_hook(m, x, None, name=name, feat_dict=feat_dict)
            pending.discard(name)
            raise _StopForward   # the module's own output is never used

    def _call_block(self, block, x, kw, stop_after):
        self._capture_pending = set(stop_after) if stop_after else None
        try:
            y = block(x, **kw)
        except _StopForward:
            return None
        finally:
            self._capture_pending = None
        return y[0] if isinstance(y, tuple) else y

    def block_forward(self, block, input_data=None, stop_after=None):
        """base_blockwise_quantization.py:367-381. Calibration inputs stored one sample per
        entry (bs 1, e.g. GPTQ's 128 x 2048) whose kwargs are equal run as ONE batch: the
        per-sample loop launches 128x more, 128x smaller GEMMs and elementwise kernels. The
        math per sample is unchanged (hooks see the stacked batch; GPTQ's running-average
        Hessian over one batch of b samples equals b single-sample updates).

        ``stop_after``: the caller discards the output (GPTQ's quant_out first pass, the
        true_sequential re-forwards) -> each forward ends right after the hooks of these modules
        have captured their inputs; the layers behind them would only feed the discarded output.
        """
        if input_data is None:
            input_data = self.input['data']
        kwargs = self.input['kwargs']
        key = (id(kwargs), len(kwargs), tuple(x.shape for x in input_data[:1]), len(input_data))
        if self.batch_calib and (self._batch_ok is None or self._batch_ok[0] != key):
            self._batch_ok = (key, _batchable(input_data, kwargs))
        if self.batch_calib and self._batch_ok[1]:
            xb = None
            for cached in (getattr(self, '_split_cache', None), getattr(self, '_cat_cache', None)):
                if cached is not None and len(cached[0]) == len(input_data) and all(
                        a is b for a, b in zip(cached[0], input_data)):
                    xb = cached[1]  # same entries as a batch we already hold: no re-cat
                    break
            if xb is None:
                xb = torch.cat(list(input_data), dim=0)
                self._cat_cache = (list(input_data), xb)
            self._batch_ctx = [x.numel() // x.shape[-1] for x in input_data]
            try:
                y = self._call_block(block, xb, kwargs[0], stop_after)
            finally:
                self._batch_ctx = None
            if y is None:
                return None
            outs = list(torch.split(y, [x.shape[0] for x in input_data], dim=0))
            self._split_cache = (outs, y)
            return outs
        out = []
        for i, x in enumerate(input_data):
            out.append(self._call_block(block, x, kwargs[i], stop_after))
        return None if stop_after else out

    def block_opt(self, block):
        named_linears = self.model.get_block_linears(block)
        extra = self.model.get_extra_modules(block)
        modules = {**named_linears, **extra}
        input_feat = defaultdict(list)
        handles = self.register_hooks(modules, input_feat)
        self.block_init(block)
        self.run(block, input_feat, handles)
        del input_feat
        self._clear_block_cache(block)

    def register_hooks(self, modules, input_feat):
        if self.data_free:
            return []
        self._hooked_names = list(modules)
        hooks = {n: functools.partial(self._capture_hook, name=n, feat_dict=input_feat)
                 for n in modules}
        pre = {}
        if not self.hook_needs_output:
            pre = {n: functools.partial(self._capture_pre_hook, name=n, feat_dict=input_feat)
                   for n in modules}
            # the capture reads only the module inputs: a fused forward may fire these hooks
            # itself with out=None and skip materialising the module outputs
            # (llama._gate_up_silu: the GPTQ calibration forward's gate / up projections)
            for h in (*hooks.values(), *pre.values()):
                h._lcq_input_only = True
        handles = [m.register_forward_hook(hooks[n]) for n, m in modules.items()]
        handles += [m.register_forward_pre_hook(pre[n]) for n, m in modules.items() if n in pre]
        return handles

    def run(self, block, input_feat, handles):
        if not self.data_free:
            if self.quant_out:
                self.block_forward(block, stop_after=self.capture_names(self._hooked_names))
            else:
                self.input['data'] = self.block_forward(block)
                self._send_handoff()  # ring shard_blocks: the next owner starts now
            for h in handles:
                h.remove()
            self.block_transform(block, input_feat, self.input['kwargs'])
        else:
            self.block_transform(block)
        if not self.data_free and self.quant_out:
            self.model.replace_module_block(FakeQuantLinear, block, self.block_idx,
                                            self.get_replacement_params('fake_quant',
                                                                        self.w_only))
            self.input['data'] = self.block_forward(block)

    def block_transform(self, block, input_feat=None, block_kwargs=None):
        subsets = self.model.get_subsets_in_block(block)
        for index, subset in enumerate(subsets):
            if subset.get('has_kwargs', False):
                if 'sub_keys' in subset:
                    subset_kwargs = [{k: kw[v] for k, v in subset['sub_keys'].items()}
                                     for kw in block_kwargs]
                else:
                    subset_kwargs = block_kwargs
            else:
                subset_kwargs = {}
            self.subset_transform(subset, input_feat, subset_kwargs)
            if self.act_static:
                self.register_act_qparams(subset['layers'], input_feat[subset['input'][0]])
            if self.true_sequential and index != len(subsets) - 1:
                nxt = subsets[index + 1]
                input_feat.update(self.rehook_next_subset(block, subset, nxt))

    def subset_transform(self, subset, input_feat, subset_kwargs):
        raise NotImplementedError

    # ---- static activation qparams (:567-588) --------------------------------------------------
    def _reference_entries(self, feats):
        """The calibration entries as the reference's hooks hold them: block_forward may run
        the stored entries as one stacked batch, so its captured input is split back into the
        entries' batch sizes (the reference calibrates per entry, or per sample when there is
        a single entry)."""
        sizes = [x.shape[0] for x in (self.input or {}).get('data', [])]
        if (len(feats) == 1 and len(sizes) > 1 and torch.is_tensor(feats[0])
                and feats[0].shape[0] == sum(sizes)):
            return list(torch.split(feats[0], sizes, dim=0))
        return list(feats)

    @torch.no_grad()
    def register_act_qparams(self, layers_dict, act_tensors):
        """base_blockwise_quantization.py:567-588: per-tensor static activation qparams from
        the calibration inputs (HBM-resident, not copied), averaged over ranks in the
        reference's replica mode, registered as buf_act_{scales,zeros,qmin,qmax}_{i}."""
        entries = self._reference_entries(act_tensors)
        if self.parallel_mode() == 'shard_tokens':
            scales_l, zeros_l, qmin_l, qmax_l = self._token_sharded_act_qparams(entries)
        else:
            scales_l, zeros_l, qmin_l, qmax_l = self.aquantizer.get_batch_tensors_qparams(
                entries)
        _, ws, _ = world()
        for i, (scales, zeros, qmin, qmax) in enumerate(zip(scales_l, zeros_l, qmin_l, qmax_l)):
            if ws > 1 and dist.is_initialized() and self.parallel_mode() == 'replicate':
                dist.all_reduce(scales, op=dist.ReduceOp.SUM)
                scales = scales / ws
            for name, layer in layers_dict.items():
                if not isinstance(layer, _LINEAR_TYPES):
                    continue
                layer.register_buffer(f'buf_act_scales_{i}', scales)
                layer.register_buffer(f'buf_act_zeros_{i}', zeros)
                layer.register_buffer(f'buf_act_qmin_{i}', qmin)
                layer.register_buffer(f'buf_act_qmax_{i}', qmax)

    @torch.no_grad()
    def _token_sharded_act_qparams(self, entries):
        """Static act qparams under shard_tokens, equal to the one-process result: the
        reference ranges are functions of one (min, max) per calibration segment (a sample
        when the calibration set is one batch, else an entry; quant.py:103-120, 221-263,
        524-543), and a segment's min / max is the min / max of its samples'. Each rank takes
        (min, max) of each of its samples (lcq_minmax_segments), the per-sample table is
        all-gathered in rank order (= global sample order, _shard_input_tokens), folded into the
        global segments, and the range + get_qparams kernel runs on the full table on every
        rank. static_hist merges whole-tensor histograms in segment order and stays
        single-process (the reference's replica mode averages per-rank scales instead)."""
        from . import ops
        aq = self.aquantizer
        if aq.calib_algo not in ('static_minmax', 'static_moving_minmax'):
            raise NotImplementedError(f'{aq.calib_algo} with token-sharded calibration data: '
                                      'set special.parallel: replicate')
        if aq.granularity != 'per_tensor' or not aq.round_zp:
            raise NotImplementedError('token-sharded static act qparams: per_tensor, round_zp')
        if not entries or any(not torch.is_tensor(e) for e in entries):
            raise NotImplementedError('token-sharded static act qparams take one input tensor')
        rank, world = P.dist_world()
        total = self.n_samples_global
        ranges = [self.sample_shard(total, r, world) for r in range(world)]
        samples = [e[i] for e in entries for i in range(e.shape[0])]
        if len(samples) != ranges[rank][1] - ranges[rank][0]:
            raise RuntimeError('captured inputs do not match this rank\'s calibration samples')
        dev = samples[0].device if samples else self.model.device
        local = (ops.minmax_segments(samples) if samples
                 else torch.empty((0, 2), dtype=torch.float32, device=dev))
        mm = P.gather_ranges(local, ranges)
        sizes = self.global_entry_sizes
        if len(sizes) > 1:   # segments = entries: fold their samples
            seg = torch.repeat_interleave(torch.arange(len(sizes), device=mm.device),
                                          torch.tensor(sizes, device=mm.device))
            lo = torch.full((len(sizes),), float('inf'), device=mm.device).scatter_reduce(
                0, seg, mm[:, 0], 'amin')
            hi = torch.full((len(sizes),), float('-inf'), device=mm.device).scatter_reduce(
                0, seg, mm[:, 1], 'amax')
            mm = torch.stack([lo, hi], dim=1)
        rdt = torch.float32 if aq.calib_algo == 'static_minmax' else entries[0].dtype
        sdt = aq._static_scale_dtype(rdt)
        r = ops.act_static_qparams(mm, aq.calib_algo, 0.01, rdt, sdt, aq.sym, float(aq.qmin),
                                   float(aq.qmax))
        return ([r[0].to(sdt)],
                [torch.tensor(0.0, device=dev) if aq.sym else r[1].to(sdt)],
                [aq.qmin.to(dev)], [aq.qmax.to(dev)])

    def rehook_next_subset(self, block, subset, next_subset):
        self.subset_init(next_subset)
        self.model.replace_module_subset(FakeQuantLinear, block, subset, self.block_idx,
                                         self.get_replacement_params('fake_quant', self.w_only))
        feat = defaultdict(list)
        handles = self.register_hooks(next_subset['layers'], feat)
        self.block_forward(block, stop_after=self.capture_names(next_subset['layers']))
        for h in handles:
            h.remove()
        return feat

    # ---- scale application (:596-778, 880-897) ------------------------------------------------
    @torch.no_grad()
    def apply_scale(self, scales, prev_op, layers):
        assert len(prev_op) == 1, 'Only support single prev_op.'
        if isinstance(prev_op[0], _LINEAR_TYPES):
            assert len(layers) == 1
            self.scale_fc_fc(prev_op[0], layers[0], scales)
        elif is_norm(prev_op[0]):
            self.scale_ln_fcs(prev_op[0], layers, scales)
        else:
            raise NotImplementedError(f'prev_op {type(prev_op[0])} not supported yet!')

    @torch.no_grad()
    def scale_fc_fc(self, fc1, fc2, scales):
        scales = scales.to(fc1.weight.device)
        if fc1.out_features == fc2.in_features:
            if getattr(fc1, 'bias', None) is not None:
                ops.scale_bcast(fc1.bias.data.view(1, -1), scales.to(fc1.bias.dtype), 'div',
                                out=fc1.bias.data.view(1, -1))
            ops.scale_bcast(fc1.weight.data, scales.to(fc1.weight.dtype), 'div', axis=1,
                            out=fc1.weight.data)
        elif fc1.out_features == fc2.in_features * 2:
            half = fc1.weight.data[fc1.weight.data.shape[0] // 2:]
            ops.scale_bcast(half, scales.to(half.dtype), 'div', axis=1, out=half)
            if getattr(fc1, 'bias', None) is not None:
                hb = fc1.bias.data[fc1.bias.data.shape[0] // 2:].view(1, -1)
                ops.scale_bcast(hb, scales.to(hb.dtype), 'div', out=hb)
        elif self.has_gqa and self.do_gqa_trans:
            # :678-685: v_proj rows / s, o_proj columns * s repeated over the query heads of
            # each kv head (an exact transfer through the attention's value path)
            if getattr(fc1, 'bias', None) is not None:
                ops.scale_bcast(fc1.bias.data.view(1, -1), scales.to(fc1.bias.dtype), 'div',
                                out=fc1.bias.data.view(1, -1))
            ops.scale_bcast(fc1.weight.data, scales.to(fc1.weight.dtype), 'div', axis=1,
                            out=fc1.weight.data)
            if fc1.out_features != fc2.in_features:
                scales = self.repeat_gqa_scales(scales)
        else:
            raise NotImplementedError('fc-fc scaling for this shape is not on the device path')
        ops.scale_bcast(fc2.weight.data, scales.to(fc2.weight.dtype), 'mul', axis=0,
                        out=fc2.weight.data)

    @torch.no_grad()
    def scale_ln_fcs(self, ln, fcs, scales):
        if not isinstance(fcs, list):
            fcs = [fcs]
        scales = scales.to(ln.weight.device).to(ln.weight.dtype)
        ops.scale_bcast(ln.weight.data.view(1, -1), scales, 'div', out=ln.weight.data.view(1, -1))
        if getattr(ln, 'bias', None) is not None:
            ops.scale_bcast(ln.bias.data.view(1, -1), scales, 'div', out=ln.bias.data.view(1, -1))
        for fc in fcs:
            ops.scale_bcast(fc.weight.data, scales.to(fc.weight.dtype), 'mul', axis=0,
                            out=fc.weight.data)

    def repeat_gqa_scales(self, scales):
        """:591-595: per-kv-channel scales [kv_heads * head_dim] repeated for the query heads
        of each kv head (repeat_interleave over heads), flattened to [heads * head_dim]."""
        s = scales.reshape(1, self.num_key_value_heads, self.head_dim)
        return torch.repeat_interleave(s, dim=1, repeats=self.num_key_value_groups).reshape(-1)

    @torch.no_grad()
    def scaling_input(self, x, scales, is_gqa=False, out=None):
        """:877-890: x / s (GQA: s repeated over the query heads)."""
        if is_gqa:
            scales = self.repeat_gqa_scales(scales)
        return ops.scale_bcast(x, scales.to(x.dtype), 'div', out=out)

    @torch.no_grad()
    def update_input_feat(self, scale, input_feat, layers_dict, is_gqa=False):
        done = {}
        for name in layers_dict:
            for i, inp in enumerate(input_feat[name]):
                key = id(inp)
                if key not in done:
                    done[key] = self.scaling_input(inp, scale.to(inp.device), is_gqa)
                input_feat[name][i] = done[key]

    # ---- deploy / save (:932-1029) ---------------------------------------------------------
    def unit_owner(self, block_idx: int, linear_name: str) -> int:
        """The rank that quantizes (and packs) this linear in a sharded deploy: its block's
        owner under shard_blocks, else the LPT unit plan (residency.Ownership, shared by the
        loader of a ``materialize: owned`` model)."""
        own = getattr(self.model, 'ownership', None)
        if own is not None:
            return own.owner_of(block_idx, linear_name)
        pending = getattr(self, '_pending_owner', None)
        if pending:
            return pending[block_idx]
        if getattr(self, '_unit_plan', None) is None:
            from .residency import Ownership
            rank, world = P.dist_world()
            self._unit_plan = Ownership.plan('shard_units', rank, world, self.model)
        return self._unit_plan.owner_of(block_idx, linear_name)

    def owned_linears(self, block) -> dict:
        """The block linears this rank works on: all of them, except under shard_units."""
        lins = self.model.get_block_linears(block)
        if self.parallel_mode() != 'shard_units':
            return lins
        rank, _ = P.dist_world()
        return {n: m for n, m in lins.items() if self.unit_owner(self.block_idx, n) == rank}

    @torch.no_grad()
    def deploy(self, quant_format, keep_device=True):
        """base_blockwise_quantization.py:932-977. Sharded runs (shard_units, shard_blocks
        with a real-quant format, or a ``materialize: owned`` model) quantize on each rank
        only what it owns; the results -- packed codes + scales for real-quant formats -- are
        then published to every rank (P.publish: one flat broadcast per block and owner), or
        stay on their owners for a sharded save when each rank holds only its own units.
        Streaming models pass every block through HBM once (visit_block)."""
        mapping = {'origin_float': OriginFloatLinear, 'fake_quant': EffcientFakeQuantLinear,
                   'fake_quant_wo_kv': EffcientFakeQuantLinear, **_REALQUANT_LINEAR_MAP_}
        if quant_format not in mapping:
            raise NotImplementedError(f"Quant format '{quant_format}' is not implemented.")
        module = mapping[quant_format]
        real = quant_format in _REALQUANT_LINEAR_MAP_
        params = self.get_replacement_params(quant_format, self.w_only)
        rank, world = P.dist_world()
        own = getattr(self.model, 'ownership', None)
        pending = getattr(self, '_pending_owner', None)
        sharded = world > 1 and (self.parallel_mode() == 'shard_units' or own is not None
                                 or (pending and real))
        # what a published module cannot carry (callables, dicts) is rebuilt from these on the
        # non-owners: the same a_qdq / w_qdq / quant_config objects the owner's new() received
        local_attrs = {**params, 'debug_print': {}}
        if not sharded:
            self.materialize_blocks()   # shard_blocks + a float format: publish first
        # The objects that exist before the deployed modules are built (the model, the
        # algorithm) are frozen out of the cyclic collector meanwhile: a MoE block allocates
        # thousands of module containers, and every collection they trigger walked every
        # tracked object of the model, so the per-layer host time grew with the layer count
        # (20 DSv3 layers: 11.1 ms per layer against 2.9 at 3 layers, 78 % of it in those
        # collections; scripts/fp8_layers_probe.py). New objects are still collected;
        # retire_module breaks each replaced module's cycle, so refcounting frees them.
        gc.freeze()
        try:
            self._deploy_blocks(module, real, params, rank, own, pending, sharded, local_attrs)
        finally:
            gc.unfreeze()

    def _deploy_blocks(self, module, real, params, rank, own, pending, sharded, local_attrs):
        for i, block in enumerate(self.blocks):
            if not sharded and self._deploy_from_memos(i, block, module, params):
                continue

            def one(i=i, block=block):
                self.block_idx = i
                lins = self.model.get_block_linears(block)
                if not sharded:
                    pre = self._prequant_fp8_block(block, lins) if real else None
                    self.model.replace_module_subset(module, block, {'layers': lins}, i, params,
                                                     prequant=pre)
                    return
                assign = {n: self.unit_owner(i, n) for n in lins}
                mine = {n: m for n, m in lins.items() if assign[n] == rank}
                pre = self._prequant_fp8_block(block, mine) if real else None
                self.model.replace_module_subset(module, block, {'layers': mine}, i, params,
                                                 prequant=pre)
                if own is None:
                    P.publish(block, assign, rest_owner=pending[i] if pending else None,
                              local_attrs=local_attrs)
                self._clear_block_cache(block)
            self.visit_block(i, one, next_i=i + 1)
        self._drain_blocks()
        self._pending_owner = None

    def _deploy_from_memos(self, i, block, module, params) -> bool:
        """A host-streamed block deployed as EffcientFakeQuantLinear without passing through
        HBM: the quant_out forward left every FakeQuantLinear of the block with its memo
        tmp_weight = w_qdq(self) (module_utils.FakeQuantLinear.forward, written back to pinned
        host memory with the block), which is what EffcientFakeQuantLinear.new computes from
        the same weight, qparams buffers and w_qdq (module_utils.py:815-819) -- the same bits,
        with no upload of the fp32 weights and no download of the result (VERDICT r5 next 7:
        the streamed GPTQ deploy moved 28 GB each way). Taken only when the block is on the
        host and every linear has such a memo made by the deploy's own callbacks; otherwise
        the block goes through visit_block as before."""
        st = getattr(self.model, 'streamer', None)
        if (st is None or module is not EffcientFakeQuantLinear or i in st.resident
                or i in st.pending):
            return False
        lins = self.model.get_block_linears(block)
        todo = {n: m for n, m in lins.items() if not getattr(m, 'no_quant', False)}
        same = self.model._same_fake_quant
        for m in todo.values():
            tw = m._buffers.get('tmp_weight') if isinstance(m, FakeQuantLinear) else None
            if (tw is None or tw.device.type != 'cpu' or tw.dtype == torch.float8_e4m3fn
                    or m.dynamic_quant_weight or m.dynamic_quant_tmp_weight
                    or not same(m, FakeQuantLinear, params)):
                return False
        self.block_idx = i
        for name, m in todo.items():
            new = EffcientFakeQuantLinear(m._buffers['tmp_weight'], m.bias, ori_module=m,
                                          a_qdq=params.get('a_qdq'))
            new.in_features, new.out_features = m.in_features, m.out_features
            new.w_qdq_name, new.a_qdq_name = m.w_qdq_name, m.a_qdq_name
            new.debug_print = {}
            parent_name, _, child = name.rpartition('.')
            parent = block.get_submodule(parent_name) if parent_name else block
            setattr(parent, child, new)
            retire_module(m)
            st.stats['host_deployed_modules'] += 1
        self._clear_block_cache(block)
        return True

    @torch.no_grad()
    def _prequant_fp8_block(self, block, mods: dict):
        """Block-fp8 checkpoint linears (DeepSeek-V3 experts) headed for a per-tensor FP8
        real-quant format: requantize every such linear of the block in ONE batched launch
        (lcq_fp8_block_to_tensor_many) instead of one dequant + quant chain per linear;
        the real-quant module's new_batch takes the results (bit-identical to the per-linear
        chain). Returns {id(module): (codes, scale)}, or None when the format does not apply."""
        wq = self.wquantizer
        if not (isinstance(wq, FloatQuantizer) and wq.granularity == 'per_tensor'
                and wq.use_qtorch and wq.fp8_dtype is not None):
            return None
        if self.quant_config['weight'].get('need_pack', False):
            return None
        sel = []   # (module, weight, weight_scale_inv): read from the slot dicts directly
        for m in mods.values():
            d = m.__dict__
            w = d['_parameters'].get('weight', d['_buffers'].get('weight'))
            if w is None or d.get('no_quant', False) or w.dtype != torch.float8_e4m3fn:
                continue
            si = d['_parameters'].get('weight_scale_inv', d['_buffers'].get('weight_scale_inv'))
            if si is not None:
                sel.append((m, w, si))
        if not sel:
            return None
        bs = getattr(sel[0][0], 'block_size', getattr(self, 'fp8_block_size', 128))
        codes, scales = ops.fp8_block_to_tensor_many(
            [w.data for _, w, _ in sel], [si.data for _, _, si in sel], bs, wq.fp8_dtype,
            qmax=wq._qmax_f())
        sv = scales.view(-1, 1)
        return {id(m): (codes[i], sv[i]) for i, (m, _, _) in enumerate(sel)}

    @torch.no_grad()
    def save_model(self, path):
        rank, world = P.dist_world()
        if getattr(self.model, 'ownership', None) is not None and world > 1:
            # every rank holds only its own blocks / units: per-rank safetensors shards and
            # one index, loadable as a whole HF checkpoint
            self._drain_blocks()
            self.model.save_sharded(path, self.unit_owner)
            return
        self.materialize_blocks()
        self._drain_blocks()
        if rank != 0:
            return
        self.model.save_pretrained(path)


def all_reduce_mean_(t: torch.Tensor):
    """all_reduce(SUM) / world_size in place (the reference's statistic averaging)."""
    _, ws, _ = world()
    if ws > 1 and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= ws
    return t
