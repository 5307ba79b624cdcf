"""Llama model adapter (drop-in for llmc ``models/llama.py`` + the BaseModel contract the hot
path consumes, base_model.py:174-436): blocks, block linears, AWQ/GPTQ subsets, module
replacement, first-block input capture. The model lives in HBM for the whole run.
"""
from __future__ import annotations

import inspect
import os
import types
from collections import defaultdict

import torch
import torch.nn as nn

from .module_utils import _LLMC_LINEAR_TYPES_, _TRANSFORMERS_LINEAR_TYPES_
from .registry import MODEL_REGISTRY

_LINEAR_TYPES = tuple(_LLMC_LINEAR_TYPES_ + _TRANSFORMERS_LINEAR_TYPES_)


_ORIG_ROTARY = None


def _fused_apply_rotary(q, k, cos, sin, unsqueeze_dim=1):
    """modeling_llama.apply_rotary_pos_emb on one lcq_rotary pass (bit-identical); other
    layouts / dtypes / devices go to the original function."""
    from . import ops
    if (unsqueeze_dim == 1 and q.is_cuda and q.dim() == 4 and k.dim() == 4
            and q.dtype in (torch.bfloat16, torch.float16) and k.dtype == q.dtype
            and cos.dtype == q.dtype and sin.dtype == q.dtype and cos.dim() == 3
            and q.shape[-1] % 16 == 0 and q.transpose(1, 2).is_contiguous()
            and k.transpose(1, 2).is_contiguous() and cos.shape[0] in (1, q.shape[0])
            and cos.shape[1:] == (q.shape[2], q.shape[3])):
        return ops.rotary(q, k, cos, sin)
    return _ORIG_ROTARY(q, k, cos, sin, unsqueeze_dim)


def _fused_mlp_forward(self, x):
    """LlamaMLP.forward with act_fn(gate) * up on one lcq_silu_mul pass; the projections are
    still called as modules (hooks fire in the original order: gate, up, down)."""
    from . import ops
    g = self.gate_proj(x)
    u = self.up_proj(x)
    if g.is_cuda and g.dtype in (torch.bfloat16, torch.float16) and g.shape == u.shape \
            and u.dtype == g.dtype and g.numel() % 8 == 0:
        h = ops.silu_mul(g, u)
    else:
        h = self.act_fn(g) * u
    return self.down_proj(h)


def _fused_rmsnorm_forward(self, hidden_states):
    """LlamaRMSNorm.forward on one lcq_rmsnorm pass (same formula; the variance is summed in
    a fixed order of its own)."""
    from . import ops
    if (hidden_states.is_cuda and hidden_states.dtype in (torch.bfloat16, torch.float16)
            and self.weight.dtype == hidden_states.dtype and hidden_states.shape[-1] % 8 == 0):
        return ops.rmsnorm(hidden_states, self.weight, self.variance_epsilon)
    input_dtype = hidden_states.dtype
    h = hidden_states.to(torch.float32)
    variance = h.pow(2).mean(-1, keepdim=True)
    h = h * torch.rsqrt(variance + self.variance_epsilon)
    return self.weight * h.to(input_dtype)


def install_fused_forward(model: nn.Module):
    """Route the Llama calibration forward's elementwise chains through the lcq fusions
    (env LCQ_FUSED_FORWARD=0 disables)."""
    global _ORIG_ROTARY
    if os.environ.get('LCQ_FUSED_FORWARD', '1') == '0':
        return
    from transformers.models.llama import modeling_llama as ml
    if _ORIG_ROTARY is None:
        _ORIG_ROTARY = ml.apply_rotary_pos_emb
        ml.apply_rotary_pos_emb = _fused_apply_rotary
    for m in model.modules():
        if isinstance(m, ml.LlamaMLP) and getattr(m.config, 'hidden_act', None) == 'silu':
            m.forward = types.MethodType(_fused_mlp_forward, m)
        elif isinstance(m, ml.LlamaRMSNorm):
            m.forward = types.MethodType(_fused_rmsnorm_forward, m)


class _Blocks(nn.Module):
    """Decoder layers + rotary embedding only (no vocab), for synthetic-input workloads."""

    def __init__(self, layers, rotary_emb):
        super().__init__()
        self.layers = nn.ModuleList(layers)
        self.rotary_emb = rotary_emb


@MODEL_REGISTRY
class Llama:
    block_name_prefix = 'model.layers'

    def __init__(self, config=None, hf_model=None, device='cuda', dtype=None):
        if hf_model is None:
            from transformers import AutoModelForCausalLM
            path = config['model']['path']
            td = config['model'].get('torch_dtype', 'auto')
            dtype = dtype or (torch.bfloat16 if td == 'auto' else getattr(torch, td))
            hf_model = AutoModelForCausalLM.from_pretrained(path, torch_dtype=dtype,
                                                            local_files_only=True)
        self.model = hf_model.to(device).eval()
        self.model_config = hf_model.config
        inner = getattr(hf_model, 'model', hf_model)
        self.blocks = inner.layers
        self.rotary_emb = inner.rotary_emb
        self.embed_tokens = getattr(inner, 'embed_tokens', None)
        self.torch_dtype = next(self.model.parameters()).dtype
        self.mm_model = None
        install_fused_forward(self.model)

    # -- random-init constructor (synthetic benchmark / tests) --------------------------------
    @classmethod
    def random(cls, model_config, num_layers=None, device='cuda', dtype=torch.bfloat16,
               seed=0, std=0.02):
        from transformers.models.llama import modeling_llama as ml
        cfg = model_config
        cfg._attn_implementation = getattr(cfg, '_attn_implementation', None) or 'sdpa'
        n = num_layers or cfg.num_hidden_layers
        g = torch.Generator(device=device).manual_seed(seed)
        layers = []
        with torch.device(device):
            for i in range(n):
                lay = ml.LlamaDecoderLayer(cfg, layer_idx=i).to(dtype)
                with torch.no_grad():
                    for name, p in lay.named_parameters():
                        if p.dim() == 2:
                            p.normal_(0.0, std, generator=g)
                        else:
                            p.uniform_(0.8, 1.2, generator=g)
                layers.append(lay)
            rot = ml.LlamaRotaryEmbedding(cfg)
        blocks = _Blocks(layers, rot)
        blocks.config = cfg
        return cls(hf_model=blocks, device=device)

    def rotary_kwargs(self, seq_len, device=None):
        """Block kwargs the Catcher would capture for an unpadded causal batch."""
        device = device or next(self.model.parameters()).device
        pos = torch.arange(seq_len, device=device).unsqueeze(0)
        dummy = torch.empty((1, seq_len, 1), dtype=self.torch_dtype, device=device)
        cos, sin = self.rotary_emb(dummy, pos)
        return {'position_embeddings': (cos, sin), 'attention_mask': None, 'position_ids': pos}

    # -- BaseModel contract ---------------------------------------------------------------------
    def get_blocks(self):
        return self.blocks

    def get_block_linears(self, block):
        return {n: m for n, m in block.named_modules() if isinstance(m, _LINEAR_TYPES)}

    def get_extra_modules(self, block):
        return {}

    def get_num_attention_heads(self):
        return self.model_config.num_attention_heads

    def get_subsets_in_block(self, block):
        """llama.py:52-91."""
        return [
            {'layers': {'self_attn.q_proj': block.self_attn.q_proj,
                        'self_attn.k_proj': block.self_attn.k_proj,
                        'self_attn.v_proj': block.self_attn.v_proj},
             'prev_op': [block.input_layernorm], 'input': ['self_attn.q_proj'],
             'inspect': block.self_attn, 'has_kwargs': True},
            {'layers': {'self_attn.o_proj': block.self_attn.o_proj},
             'prev_op': [block.self_attn.v_proj], 'input': ['self_attn.o_proj'],
             'inspect': block.self_attn.o_proj, 'has_kwargs': False},
            {'layers': {'mlp.gate_proj': block.mlp.gate_proj, 'mlp.up_proj': block.mlp.up_proj},
             'prev_op': [block.post_attention_layernorm], 'input': ['mlp.gate_proj'],
             'inspect': block.mlp, 'has_kwargs': False, 'is_mlp': True},
            {'layers': {'mlp.down_proj': block.mlp.down_proj},
             'prev_op': [block.mlp.up_proj], 'input': ['mlp.down_proj'],
             'inspect': block.mlp.down_proj, 'has_kwargs': False, 'is_mlp': True},
        ]

    def replace_module_subset(self, module, block, subset, block_idx, params_dict):
        for name, m in subset['layers'].items():
            if not isinstance(m, _LINEAR_TYPES) or getattr(m, 'no_quant', False):
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

    def set_modality(self, modality):
        self.modality = modality

    def save_pretrained(self, path):
        self.model.save_pretrained(path)

    # -- calibration capture (base_model.py:174-192, 279-336) -----------------------------------
    @torch.no_grad()
    def collect_first_block_input(self, calib_data):
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
        try:
            for data in calib_data:
                data = {k: (v.to(next(self.model.parameters()).device) if torch.is_tensor(v)
                            else v) for k, v in data.items()}
                try:
                    self.model(**data)
                except ValueError:
                    pass
        finally:
            self.blocks[0] = block0
        self.first_block_input = first
        return first
