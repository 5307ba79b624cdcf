"""Model-adapter contract (drop-in for llmc ``models/base_model.py:22-470``, the part the
quantization hot path consumes): blocks, block linears, subsets, extra modules, module
replacement, first-block input capture, save. Family adapters (``llama.Llama``, ``opt.Opt``,
``deepseekv3.DeepseekV3``) supply ``find_blocks`` / ``find_embed_layers`` /
``get_subsets_in_block`` and the family's layer norms, as the reference's do.

MI355X-first differences: the whole model stays in HBM (no per-block ``.cuda()/.cpu()``), the
Catcher runs on the device, and every exact ``nn.Linear`` of the model runs on the lcq
projection GEMM (``module_utils.lcq_linear``) unless ``LCQ_FUSED_FORWARD=0``.
"""
from __future__ import annotations

import inspect
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
    """Every exact nn.Linear of `model` onto the lcq GEMM (LCQ_FUSED_FORWARD=0 disables)."""
    if os.environ.get('LCQ_FUSED_FORWARD', '1') == '0':
        return
    for m in model.modules():
        if type(m) is nn.Linear:
            m.forward = types.MethodType(_linear_forward, m)


def _torch_dtype(name, default=torch.bfloat16):
    """The YAML's model.torch_dtype ('auto', 'bfloat16', 'torch.float16', ...)."""
    if name in (None, 'auto'):
        return default
    if isinstance(name, torch.dtype):
        return name
    return getattr(torch, str(name).replace('torch.', ''))


class BaseModel:
    """base_model.py:22-470 (hot-path contract)."""

    block_name_prefix = 'model.layers'
    default_dtype = torch.bfloat16

    def __init__(self, config=None, hf_model=None, device='cuda', dtype=None):
        if hf_model is None:
            from transformers import AutoModelForCausalLM
            path = config['model']['path']
            dtype = dtype or _torch_dtype(config['model'].get('torch_dtype', 'auto'),
                                          self.default_dtype)
            hf_model = AutoModelForCausalLM.from_pretrained(path, torch_dtype=dtype,
                                                            local_files_only=True)
        self.config = config
        hf_model = self.prepare_model(hf_model)
        self.model = hf_model.to(device).eval()
        self.model_config = hf_model.config
        if hasattr(self.model_config, 'use_cache'):
            self.model_config.use_cache = False  # base_model.py:201-203
        self.torch_dtype = next(self.model.parameters()).dtype
        self.mm_model = None
        self.modality = 'language'
        self.find_blocks()
        self.find_embed_layers()
        self.install_fused_forward()

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

    def replace_module_subset(self, module, block, subset, block_idx, params_dict):
        """base_model.py:405-436 (linears only; the MoE router and other non-linear layers of
        a subset keep their class)."""
        for name, m in subset['layers'].items():
            if not isinstance(m, _LINEAR_TYPES) or getattr(m, 'no_quant', False):
                continue
            if self._same_fake_quant(m, module, params_dict):
                continue
            new = module.new(m, **params_dict)
            parent_name, _, child = name.rpartition('.')
            parent = block.get_submodule(parent_name) if parent_name else block
            setattr(parent, child, new)

    def replace_module_block(self, module, block, block_idx, params_dict):
        self.replace_module_subset(module, block, {'layers': self.get_block_linears(block)},
                                   block_idx, params_dict)

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
        dev = next(self.model.parameters()).device
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
