"""Model-adapter contract (drop-in for llmc ``models/base_model.py:22-470``, the part the
quantization hot path consumes): blocks, block linears, subsets, extra modules, module
replacement, first-block input capture, save. Family adapters (``llama.Llama``, ``opt.Opt``,
``deepseekv3.DeepseekV3``) supply ``find_blocks`` / ``find_embed_layers`` /
``get_subsets_in_block`` and the family's layer norms, as the reference's do.

MI355X-first differences: the whole model stays in HBM (no per-block ``.cuda()/.cpu()``), the
Catcher runs on the device, and every exact ``nn.Linear`` of the model runs on the lcq
projection GEMM (``module_utils.lcq_linear``).
"""
from __future__ import annotations

import glob
import inspect
import json
import os
import types
from collections import defaultdict

import torch
import torch.nn as nn

from .module_utils import _LLMC_LINEAR_TYPES_, _TRANSFORMERS_LINEAR_TYPES_

_LINEAR_TYPES = tuple(_LLMC_LINEAR_TYPES_ + _TRANSFORMERS_LINEAR_TYPES_)


def _linear_forward(self, x):
    """nn.Linear.forward on the lcq projection GEMM (module_utils.lcq_linear)."""
    from .module_utils import lcq_linear
    return lcq_linear(x, self.weight, self.bias)


def install_linear_forward(model: nn.Module):
    """Every exact nn.Linear of `model` onto the lcq GEMM."""
    for m in model.modules():
        if type(m) is nn.Linear:
            m.forward = types.MethodType(_linear_forward, m)


def retire_module(m: nn.Module):
    """A module just replaced in the model: drop the instance-level forward that
    install_linear_forward bound to it (module -> bound method -> module is a reference cycle,
    which would keep the replaced linear -- and its device weight -- alive until the next cyclic
    garbage collection: a whole model's float weights through a deploy)."""
    f = m.__dict__.get('forward')
    if isinstance(f, types.MethodType) and f.__self__ is m:
        del m.__dict__['forward']


def _torch_dtype(name, default=torch.bfloat16):
    """The YAML's model.torch_dtype ('auto', 'bfloat16', 'torch.float16', ...)."""
    if name in (None, 'auto'):
        return default
    if isinstance(name, torch.dtype):
        return name
    return getattr(torch, str(name).replace('torch.', ''))


def _checkpoint_bytes(path) -> int:
    import glob
    return sum(os.path.getsize(f) for f in glob.glob(os.path.join(path, '*.safetensors')))


def _safetensor_files(path):
    idx = os.path.join(path, 'model.safetensors.index.json')
    if os.path.exists(idx):
        with open(idx) as f:
            return sorted({os.path.join(path, v) for v in json.load(f)['weight_map'].values()})
    return sorted(glob.glob(os.path.join(path, '*.safetensors')))


class BaseModel:
    """base_model.py:22-470 (hot-path contract).

    Placement (residency.py): ``model.residency`` = ``device`` (all blocks in HBM), ``stream``
    (blocks in pinned host memory, streamed through HBM by the block loop and deploy) or
    ``auto`` (default: ``stream`` when the checkpoint exceeds ``model.device_budget_gb``, by
    default 70 % of the GPU's HBM); ``model.materialize: owned`` (world > 1 under a sharded plan)
    loads on each rank only the blocks / units it owns, the rest stays on the meta device."""

    block_name_prefix = 'model.layers'
    default_dtype = torch.bfloat16
    block_fp8 = False   # DeepSeek-V3 block-fp8 checkpoints (base_model.py:205-239)

    def __init__(self, config=None, hf_model=None, device='cuda', dtype=None, residency=None,
                 materialize=None, hf_config=None, random_init=None):
        mcfg = ((config or {}).get('model', {}) or {}) if config is not None else {}
        self.config = config
        self.device = torch.device(device)
        self.residency = residency or mcfg.get('residency', 'auto')
        materialize = materialize or mcfg.get('materialize', 'all')
        self.ownership = None
        self.streamer = None
        plan = None
        if materialize == 'owned':
            from .parallel import dist_world, planned_mode
            rank, world = dist_world()
            if world > 1:
                plan = (planned_mode(config, world), rank, world)
        if hf_model is None and random_init is not None:
            # synthetic model of hf_config's architecture (bench): built like a checkpoint
            # load -- meta skeleton, owned tensors only -- with seeded random values
            if self.residency == 'auto':
                self.residency = 'device'
            dtype = dtype or self.default_dtype
            hf_model = self.random_checkpoint(hf_config, dtype, self.block_fp8, plan,
                                              **random_init)
        elif hf_model is None:
            path = mcfg['path']
            dtype = dtype or _torch_dtype(mcfg.get('torch_dtype', 'auto'), self.default_dtype)
            fp8 = self.block_fp8 or dtype == torch.float8_e4m3fn
            if fp8:
                assert mcfg.get('block_wise_quant', self.block_fp8), \
                    'fp8 checkpoints need block_wise_quant'
            if self.residency == 'auto':
                budget = float(mcfg.get('device_budget_gb', 0) or 0) * 2 ** 30
                if not budget and torch.cuda.is_available():
                    budget = 0.7 * torch.cuda.get_device_properties(self.device).total_memory
                big = budget and _checkpoint_bytes(path) > budget
                self.residency = 'stream' if big else 'device'
            if plan is not None or fp8 or self.residency == 'stream':
                hf_model = self.load_checkpoint(path, dtype, fp8, plan)
            else:
                from transformers import AutoModelForCausalLM
                hf_model = self.prepare_model(AutoModelForCausalLM.from_pretrained(
                    path, torch_dtype=dtype, local_files_only=True))
        else:
            if self.residency == 'auto':
                self.residency = 'device'
            hf_model = self.prepare_model(hf_model)
        self.model = hf_model.eval()
        self.model_config = hf_model.config
        if hasattr(self.model_config, 'use_cache'):
            self.model_config.use_cache = False  # base_model.py:201-203
        self.find_blocks()
        self.find_embed_layers()
        if plan is not None and self.ownership is None:
            # a model handed over whole: drop what this rank does not own
            from .residency import Ownership
            self.ownership = Ownership.plan(plan[0], plan[1], plan[2], self)
            self._drop_unowned()
        self.torch_dtype = next(t for t in self.model.parameters() if not t.is_meta).dtype
        self.mm_model = None
        self.modality = 'language'
        self.place()
        self.install_fused_forward()

    # -- placement (residency.py) ---------------------------------------------------------------
    def _block_tensor_names(self):
        """block index -> {tensor name relative to the block: (module, kind, name)}"""
        from .residency import _tensor_slots
        out = []
        for block in self.blocks:
            names = {id(m): n for n, m in block.named_modules()}
            out.append({(f'{names[id(m)]}.{tn}' if names[id(m)] else tn): (m, kind, tn)
                        for m, kind, tn, _ in _tensor_slots(block)})
        return out

    def _owned_slots(self):
        """(module, kind, name) of every block tensor this rank materialises, per block."""
        per = []
        for bi, slots in enumerate(self._block_tensor_names()):
            lin = set(self.get_block_linears(self.blocks[bi]))
            per.append({rel: slot for rel, slot in slots.items()
                        if self.ownership.owns_block_tensor(bi, rel, lin)})
        return per

    @torch.no_grad()
    def _drop_unowned(self):
        from .residency import _install
        owned = self._owned_slots()
        for bi, slots in enumerate(self._block_tensor_names()):
            for rel, (m, kind, tn) in slots.items():
                if rel not in owned[bi]:
                    t = getattr(m, kind)[tn]
                    _install(m, kind, tn, torch.empty(t.shape, dtype=t.dtype, device='meta'))

    def blocks_container_name(self) -> str:
        for n, mod in self.model.named_modules():
            if mod is self.blocks:
                return n
        raise RuntimeError('blocks not found in the model')

    @torch.no_grad()
    def place(self):
        """Every non-meta tensor outside the blocks to the device; the blocks too (``device``)
        or into pinned host memory behind a BlockStreamer (``stream``)."""
        from .residency import BlockStreamer, _install, _tensor_slots
        in_blocks = {id(m) for b in self.blocks for m in b.modules()}
        for m, kind, tn, t in list(_tensor_slots(self.model)):
            if t.is_meta or t.device == self.device:
                continue
            if id(m) in in_blocks and self.residency == 'stream':
                continue
            _install(m, kind, tn, t.to(self.device))
        if self.residency == 'stream':
            self.streamer = BlockStreamer(self.blocks, self.device)
            self.streamer.pin_all()

    @torch.no_grad()
    def _skeleton(self, cfg, dtype, fp8, plan, bs=128):
        """The model on the meta device (block-fp8 linears as LlmcFp8Linear, the modules
        from_pretrained keeps in fp32 in fp32), this rank's ownership, and every tensor it
        keeps allocated (uninitialised) on the device -- or in host memory when streaming.
        Returns (model, {checkpoint name: (module, kind, name)} of the allocated tensors)."""
        from transformers import AutoModelForCausalLM

        from .residency import Ownership, _install, _tensor_slots
        with torch.device('meta'):
            model = AutoModelForCausalLM.from_config(
                cfg, torch_dtype=torch.bfloat16 if fp8 else dtype)
        # from_pretrained keeps these in fp32 whatever torch_dtype says (DeepSeek-V3's router
        # e_score_correction_bias); the copy below upcasts the checkpoint's values alike
        fp32 = (set(getattr(model, '_keep_in_fp32_modules', None) or ())
                | set(getattr(model, '_keep_in_fp32_modules_strict', None) or ()))
        if fp32:
            names = {id(m): n for n, m in model.named_modules()}
            for m, kind, tn, t in list(_tensor_slots(model)):
                full = f'{names[id(m)]}.{tn}'.split('.')
                if t.is_floating_point() and any(k in full for k in fp32):
                    _install(m, kind, tn, torch.empty(t.shape, dtype=torch.float32,
                                                      device='meta'))
        model = self.prepare_model(model)
        self.model = model
        self.find_blocks()
        if fp8:
            from .module_utils import LlmcFp8Linear
            with torch.device('meta'):
                for block in self.blocks:
                    for name, m in list(block.named_modules()):
                        if type(m) is not nn.Linear:
                            continue
                        parent_name, _, child = name.rpartition('.')
                        parent = block.get_submodule(parent_name) if parent_name else block
                        new = LlmcFp8Linear.new(m, bs)
                        if new.bias is not None:
                            new.bias.data = new.bias.data.to(torch.bfloat16)
                        setattr(parent, child, new)
        if plan is not None:
            self.ownership = Ownership.plan(plan[0], plan[1], plan[2], self)
        target = torch.device('cpu') if self.residency == 'stream' else self.device
        owned = self._owned_slots() if self.ownership is not None else None
        prefix = self.blocks_container_name()
        keep = {}   # full checkpoint name -> (module, kind, name)
        for bi, slots in enumerate(self._block_tensor_names()):
            for rel, slot in slots.items():
                if owned is None or rel in owned[bi]:
                    keep[f'{prefix}.{bi}.{rel}'] = slot
        in_blocks = {id(m) for b in self.blocks for m in b.modules()}
        rebuild = []
        for mn, mod in model.named_modules():
            if id(mod) in in_blocks:
                continue
            if any(b in mod._non_persistent_buffers_set for b in mod._buffers):
                rebuild.append(mn)   # computed at construction (rotary inv_freq): rebuild
                continue
            for tn, t in list(mod._parameters.items()) + list(mod._buffers.items()):
                if t is not None:
                    keep[f'{mn}.{tn}' if mn else tn] = (mod, '_parameters' if tn in
                                                         mod._parameters else '_buffers', tn)
        for mn in rebuild:
            parent_name, _, child = mn.rpartition('.')
            parent = model.get_submodule(parent_name) if parent_name else model
            old = getattr(parent, child)
            with torch.device(target):
                setattr(parent, child, type(old)(config=cfg))
        for name, (m, kind, tn) in keep.items():
            t = getattr(m, kind)[tn]
            if t.is_meta:
                _install(m, kind, tn, torch.empty(t.shape, dtype=t.dtype, device=target))
        return model, keep

    @torch.no_grad()
    def load_checkpoint(self, path, dtype, fp8, plan):
        """Build the model on the meta device and materialise only what this process keeps --
        every tensor outside the blocks, and the block tensors this rank owns (all of them
        unless ``plan``) -- on the device, or in host memory when streaming; then read exactly
        those tensors from the safetensors shards (a non-owned tensor is never read). Block-fp8
        checkpoints (base_model.py:205-264) load into LlmcFp8Linear modules (e4m3 weight +
        128x128 weight_scale_inv), no bf16 copy made."""
        from safetensors import safe_open
        from transformers import AutoConfig
        cfg = AutoConfig.from_pretrained(path, local_files_only=True)
        bs = 128
        if fp8:
            qc = getattr(cfg, 'quantization_config', None) or {}
            qc = qc if isinstance(qc, dict) else qc.to_dict()
            bs = int(qc.get('weight_block_size', [128, 128])[0])
            if hasattr(cfg, 'quantization_config'):
                del cfg.quantization_config  # plain linears; the fp8 ones are built here
        model, keep = self._skeleton(cfg, dtype, fp8, plan, bs)
        seen = set()
        for f in _safetensor_files(path):
            with safe_open(f, framework='pt', device='cpu') as st:
                for k in st.keys():
                    slot = keep.get(k)
                    if slot is None:
                        continue
                    m, kind, tn = slot
                    dst = getattr(m, kind)[tn]
                    src = st.get_tensor(k)
                    if tuple(dst.shape) != tuple(src.shape):
                        raise ValueError(f'{k}: checkpoint {tuple(src.shape)} vs model '
                                         f'{tuple(dst.shape)}')
                    dst.copy_(src)
                    seen.add(k)
        tied = getattr(cfg, 'tie_word_embeddings', False)
        missing = [k for k, (m, kind, tn) in keep.items() if k not in seen
                   and not (kind == '_buffers' and tn in m._non_persistent_buffers_set)
                   and not (tied and k.endswith('lm_head.weight'))]
        if missing:
            raise ValueError(f'checkpoint lacks {len(missing)} tensors, e.g. {missing[:3]}')
        if tied and hasattr(model, 'tie_weights'):
            model.tie_weights()
        model.config = cfg
        return model

    @torch.no_grad()
    def random_checkpoint(self, cfg, dtype, fp8, plan, seed=0, std=0.02):
        """_skeleton filled with seeded random values instead of a checkpoint (synthetic
        benchmarks: no network, no checkpoints): matrices N(0, std^2), vectors U(0.8, 1.2),
        block-fp8 linears as the 128x128-block e4m3 quantization of N(0, std^2) weights (the
        checkpoints' layout), each tensor from its own generator seeded by its name, so a
        rank's owned tensors are the same whatever the world size."""
        import zlib

        from . import ops
        from .module_utils import LlmcFp8Linear
        model, keep = self._skeleton(cfg, dtype, fp8, plan)
        gdev = self.device if self.device.type == 'cuda' else torch.device('cpu')
        done = set()
        for name, (m, kind, tn) in keep.items():
            t = getattr(m, kind)[tn]
            g = torch.Generator(device=gdev).manual_seed(seed + zlib.crc32(name.encode()))
            if isinstance(m, LlmcFp8Linear) and tn in ('weight', 'weight_scale_inv'):
                if id(m) in done:
                    continue
                done.add(id(m))
                w = (torch.randn(m.weight.shape, generator=g, device=gdev) * std).to(
                    torch.bfloat16)
                r = ops.fp8_quant_blocks(w, torch.float8_e4m3fn, m.block_size, qmax=448.0,
                                         clamp_min=0.0, add_zero=False)
                m.weight.data.copy_(r['codes'])
                m.weight_scale_inv.data.copy_(r['scales'])
                continue
            if not t.is_floating_point():
                t.zero_()
            elif t.dim() >= 2:
                t.copy_(torch.randn(t.shape, generator=g, device=gdev) * std)
            else:
                t.copy_(torch.rand(t.shape, generator=g, device=gdev) * 0.4 + 0.8)
        model.config = cfg
        return model

    # -- family hooks ---------------------------------------------------------------------------
    def prepare_model(self, hf_model):
        """Structural conversion before the model goes to the device (e.g. DeepSeek-V3's
        fused expert tensors into per-expert linears)."""
        return hf_model

    def install_fused_forward(self):
        install_linear_forward(self.model)

    def find_blocks(self):
        raise NotImplementedError

    def find_embed_layers(self):
        self.embed_tokens = None

    def get_subsets_in_block(self, block):
        raise NotImplementedError

    def get_layernorms_in_block(self, block):
        return {}

    # -- contract -------------------------------------------------------------------------------
    def get_model(self):
        return self.model

    def get_model_config(self):
        return self.model_config

    def skip_layer_name(self):
        return ['lm_head']

    def has_bias(self):
        return False

    def get_blocks(self):
        return self.blocks

    def get_block_linears(self, block):
        """base_model.py:361-366."""
        return {n: m for n, m in block.named_modules() if isinstance(m, _LINEAR_TYPES)}

    def get_extra_modules(self, block):
        return {}

    def get_moe_gate(self, block):
        return None

    def clear_block_cache(self, block):
        """Drop any memoised stage outputs of a finished block (their tensors are large)."""
        for mod in block.modules():
            mod.__dict__.pop('_lcq_stage', None)

    def get_num_attention_heads(self):
        return self.model_config.num_attention_heads

    def set_modality(self, modality):
        self.modality = modality

    @staticmethod
    def _same_fake_quant(m, module, params_dict):
        """m is already `module` (exact class) built with the same quant callbacks: a new one
        would re-derive the identical fake-quant weight from the same weight and buffers, so
        the existing object is kept (memoised stage outputs stay valid)."""
        if type(m) is not module or not hasattr(m, 'w_qdq'):
            return False

        def same(a, b):
            if a is b:
                return True
            fa, fb = getattr(a, 'func', None), getattr(b, 'func', None)
            return (fa is not None and fa == fb and a.args == b.args
                    and a.keywords.keys() == b.keywords.keys()
                    and all(a.keywords[k] is b.keywords[k] for k in a.keywords))
        return (same(m.w_qdq, params_dict.get('w_qdq')) and
                same(m.a_qdq, params_dict.get('a_qdq')))

    def replace_module_subset(self, module, block, subset, block_idx, params_dict,
                              prequant=None):
        """base_model.py:405-436 (linears only; the MoE router and other non-linear layers of
        a subset keep their class). Classes with new_batch (the real-quant linears) build the
        whole subset at once, with `prequant` (module -> (codes, scales), a block's batched
        requant) for the modules it covers."""
        if hasattr(module, 'new_batch'):
            items = [(name, m) for name, m in subset['layers'].items()
                     if isinstance(m, _LINEAR_TYPES) and not getattr(m, 'no_quant', False)]
            pre = None if prequant is None else [prequant.get(id(m)) for _, m in items]
            news = module.new_batch([m for _, m in items], prequant=pre, **params_dict)
            parents = {}
            for (name, old), new in zip(items, news):
                parent_name, _, child = name.rpartition('.')
                parent = parents.get(parent_name)
                if parent is None:
                    parent = parents[parent_name] = (block.get_submodule(parent_name)
                                                     if parent_name else block)
                if parent._modules.get(child) is old:
                    parent._modules[child] = new   # what nn.Module.__setattr__ does here
                else:
                    setattr(parent, child, new)
                retire_module(old)
            return
        for name, m in subset['layers'].items():
            if not isinstance(m, _LINEAR_TYPES) or getattr(m, 'no_quant', False):
                continue
            if self._same_fake_quant(m, module, params_dict):
                continue
            new = module.new(m, **params_dict)
            parent_name, _, child = name.rpartition('.')
            parent = block.get_submodule(parent_name) if parent_name else block
            setattr(parent, child, new)
            retire_module(m)

    def replace_module_block(self, module, block, block_idx, params_dict, prequant=None):
        self.replace_module_subset(module, block, {'layers': self.get_block_linears(block)},
                                   block_idx, params_dict, prequant=prequant)

    def replace_module_all(self, module, params_dict, keep_device=True):
        for i, block in enumerate(self.blocks):
            self.replace_module_block(module, block, i, params_dict)

    def convert_dtype(self, dtype):
        for block in self.blocks:
            for m in block.modules():
                if isinstance(m, nn.Linear) and m.weight.dtype != dtype:
                    m.weight.data = m.weight.data.to(dtype)

    def save_pretrained(self, path):
        self.model.save_pretrained(path)

    @torch.no_grad()
    def save_sharded(self, path, owner_of):
        """materialize: owned -- each rank writes the tensors it holds as
        model-<r+1>-of-<world>.safetensors: its blocks' / units' tensors (``owner_of(block,
        linear)``), plus, on rank 0, everything outside the units (embeddings, norms, ...).
        Rank 0 writes model.safetensors.index.json (the union of the key lists) and
        config.json: one HF checkpoint, written without any rank holding the whole model."""
        import re

        import torch.distributed as dist
        from safetensors.torch import save_file
        rank, world = dist.get_rank(), dist.get_world_size()
        prefix = re.escape(self.blocks_container_name())
        lin_names = [set(self.get_block_linears(b)) for b in self.blocks]
        own = self.ownership
        mine = {}
        for k, t in self.model.state_dict(keep_vars=True).items():
            if t is None or t.is_meta:
                continue
            writer = 0
            m = re.match(rf'^{prefix}\.(\d+)\.(.*)$', k)
            if m:
                bi, mod = int(m.group(1)), m.group(2).rpartition('.')[0]
                if mod in lin_names[bi]:
                    writer = owner_of(bi, mod)
                elif own is not None and own.mode == 'shard_blocks':
                    writer = own.block_of(bi)
            if writer == rank:
                mine[k] = t.detach().to('cpu', copy=True).contiguous()
        os.makedirs(path, exist_ok=True)
        fname = f'model-{rank + 1:05d}-of-{world:05d}.safetensors'
        save_file(mine, os.path.join(path, fname), metadata={'format': 'pt'})
        listing = [None] * world
        dist.all_gather_object(listing, (fname, {k: t.numel() * t.element_size()
                                                 for k, t in mine.items()}))
        if rank == 0:
            wmap, total = {}, 0
            for fn, keys in listing:
                for k, nb in keys.items():
                    if k in wmap:
                        raise RuntimeError(f'{k} written by two ranks')
                    wmap[k] = fn
                    total += nb
            with open(os.path.join(path, 'model.safetensors.index.json'), 'w') as f:
                json.dump({'metadata': {'total_size': total},
                           'weight_map': dict(sorted(wmap.items()))}, f, indent=2)
            self.model_config.save_pretrained(path)
        dist.barrier()

    # -- calibration capture (base_model.py:174-192, 279-336) -----------------------------------
    @torch.no_grad()
    def collect_first_block_input(self, calib_data, padding_mask=None):
        first = defaultdict(list)
        block0 = self.blocks[0]
        sig = list(inspect.signature(block0.forward).parameters.keys())

        class Catcher(nn.Module):
            def __init__(self, module):
                super().__init__()
                self.module = module

            def forward(self, *args, **kwargs):
                for i, a in enumerate(args):
                    if i > 0:
                        kwargs[sig[i]] = a
                first['data'].append(args[0])
                first['kwargs'].append(kwargs)
                raise ValueError

        self.blocks[0] = Catcher(block0)
        dev = self.device
        try:
            for data in calib_data:
                data = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in data.items()}
                try:
                    self.model(**data)
                except ValueError:
                    pass
        finally:
            self.blocks[0] = block0
        assert len(first) > 0, 'Catch input data failed.'
        self.first_block_input = first
        self.padding_mask = padding_mask
        return first

    def get_first_block_input(self):
        return self.first_block_input

    def get_padding_mask(self):
        return getattr(self, 'padding_mask', None)
