"""DeepSeek-V3 model adapter (drop-in for llmc ``models/deepseekv3.py:1-167``): MLA attention
subsets, the MoE subset (every routed expert's gate/up + the shared expert's + the router),
one down_proj subset per expert, and the dense-MLP layers before ``first_k_dense_replace``.

The reference adapter expects the checkpoint's own modeling code, where ``mlp.experts`` is a
ModuleList of per-expert MLPs (``experts[i].gate_proj`` ...). transformers' built-in
DeepseekV3 stores the routed experts as two 3-D tensors (``DeepseekV3Experts``);
``unfuse_experts`` rewrites them into that per-expert layout (same weights, same routing and
combine math) so every expert linear is an nn.Linear the hot path can hook, search, quantize
and deploy. Block-fp8 checkpoints (``torch_dtype: torch.float8_e4m3fn``,
``block_wise_quant: True``, base_model.py:205-239) load into ``LlmcFp8Linear`` modules.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .base_model import BaseModel
from .registry import MODEL_REGISTRY


class ExpertList(nn.ModuleList):
    """Routed experts as separate MLP modules with the DeepseekV3Experts forward contract
    (hidden [T, H], top-k indices / weights [T, k]): each hit expert runs on its tokens and its
    output, times the routing weight, is index-added into the result (same order of
    experts and of the combine as the fused module). Each expert's linears are tagged with the
    token index of every row they get (``_lcq_rows``), so a stacked calibration forward's
    captured expert inputs can be split back into the reference's per-entry samples
    (BaseBlockwiseQuantization.entry_view)."""

    def forward(self, hidden_states, top_k_index, top_k_weights):
        out = torch.zeros_like(hidden_states)
        with torch.no_grad():
            mask = torch.nn.functional.one_hot(top_k_index, num_classes=len(self)).permute(2, 1, 0)
            hit = torch.greater(mask.sum(dim=(-1, -2)), 0).nonzero()
        for e in hit:
            e = int(e[0])
            pos, tok = torch.where(mask[e])
            for lin in self[e].children():  # row -> token map for input capture hooks
                lin._lcq_rows = tok
            h = self[e](hidden_states[tok]) * top_k_weights[tok, pos, None]
            out.index_add_(0, tok, h.to(out.dtype))
        return out


@torch.no_grad()
def unfuse_experts(model: nn.Module) -> nn.Module:
    """Replace every transformers DeepseekV3Experts (3-D gate_up / down tensors) by an
    ExpertList of DeepseekV3MLP modules holding the same weights."""
    try:
        from transformers.models.deepseek_v3 import modeling_deepseek_v3 as md
    except ImportError:  # pragma: no cover - transformers without DeepSeek-V3
        return model
    for mod in list(model.modules()):
        if not (isinstance(mod, md.DeepseekV3MoE)
                and isinstance(mod.experts, md.DeepseekV3Experts)):
            continue
        fused, cfg = mod.experts, mod.config
        inter = fused.intermediate_dim
        experts = ExpertList()
        dev = fused.gate_up_proj.device
        for e in range(fused.num_experts):
            with torch.device(dev):   # meta stays meta (BaseModel.load_checkpoint)
                mlp = md.DeepseekV3MLP(cfg, intermediate_size=inter).to(
                    dtype=fused.gate_up_proj.dtype)
            if dev.type != 'meta':
                mlp.gate_proj.weight.copy_(fused.gate_up_proj[e, :inter])
                mlp.up_proj.weight.copy_(fused.gate_up_proj[e, inter:])
                mlp.down_proj.weight.copy_(fused.down_proj[e])
            experts.append(mlp)
        mod.experts = experts
    return model


@MODEL_REGISTRY
class DeepseekV3(BaseModel):
    block_name_prefix = 'model.layers'

    def __init__(self, config=None, hf_model=None, device='cuda', dtype=None, **kw):
        mcfg = (config or {}).get('model', {}) if config is not None else {}
        td = mcfg.get('torch_dtype', 'auto')
        # block-fp8 checkpoints (torch_dtype float8_e4m3fn + block_wise_quant) load into
        # LlmcFp8Linear modules (BaseModel.load_checkpoint)
        self.block_fp8 = td in ('torch.float8_e4m3fn', 'float8_e4m3fn') or \
            dtype == torch.float8_e4m3fn
        super().__init__(config, hf_model=hf_model, device=device, dtype=dtype, **kw)

    def prepare_model(self, hf_model):
        return unfuse_experts(hf_model)

    def find_blocks(self):
        self.blocks = self.model.model.layers

    def find_embed_layers(self):
        self.embed_tokens = self.model.model.embed_tokens

    def get_embed_layers(self):
        return [self.embed_tokens]

    def get_layers_except_blocks(self):
        return [self.embed_tokens, self.model.model.norm, self.model.lm_head]

    def get_head_layers(self):
        return [self.model.lm_head]

    def get_pre_head_layernorm_layers(self):
        return [self.model.model.norm]

    def get_extra_modules(self, block):
        """deepseekv3.py:30-33: the MoE module's input feeds the expert subset."""
        return {'mlp': block.mlp}

    def has_bias(self):
        return False

    def get_layernorms_in_block(self, block):
        return {'input_layernorm': block.input_layernorm,
                'post_attention_layernorm': block.post_attention_layernorm}

    def get_attn_in_block(self, block):
        return {'self_attn': block.self_attn}

    def get_moe_gate(self, block):
        return {'mlp.gate': block.mlp.gate} if hasattr(block.mlp, 'gate') else None

    def get_subsets_in_block(self, block):
        """deepseekv3.py:69-167."""
        a, mlp = block.self_attn, block.mlp
        subs = []
        if hasattr(a, 'q_proj'):
            subs.append({'layers': {'self_attn.q_proj': a.q_proj,
                                    'self_attn.kv_a_proj_with_mqa': a.kv_a_proj_with_mqa},
                         'prev_op': [block.input_layernorm], 'input': ['self_attn.q_proj'],
                         'inspect': a, 'has_kwargs': True})
        else:
            subs.append({'layers': {'self_attn.q_a_proj': a.q_a_proj,
                                    'self_attn.kv_a_proj_with_mqa': a.kv_a_proj_with_mqa},
                         'prev_op': [block.input_layernorm], 'input': ['self_attn.q_a_proj'],
                         'inspect': a, 'has_kwargs': True})
            subs.append({'layers': {'self_attn.q_b_proj': a.q_b_proj},
                         'prev_op': [a.q_a_layernorm], 'input': ['self_attn.q_b_proj'],
                         'inspect': a.q_b_proj, 'has_kwargs': False, 'skip_rotate': True})
        subs.append({'layers': {'self_attn.o_proj': a.o_proj}, 'prev_op': [None],
                     'input': ['self_attn.o_proj'], 'inspect': a.o_proj, 'has_kwargs': False})
        subs.append({'layers': {'self_attn.kv_b_proj': a.kv_b_proj},
                     'prev_op': [a.kv_a_layernorm], 'input': ['self_attn.kv_b_proj'],
                     'inspect': a.kv_b_proj, 'has_kwargs': False, 'skip_rotate': True})
        if hasattr(mlp, 'gate'):
            n = len(mlp.experts)
            layers = {f'mlp.experts.{i}.gate_proj': mlp.experts[i].gate_proj for i in range(n)}
            layers.update({f'mlp.experts.{i}.up_proj': mlp.experts[i].up_proj
                           for i in range(n)})
            layers.update({'mlp.shared_experts.gate_proj': mlp.shared_experts.gate_proj,
                           'mlp.shared_experts.up_proj': mlp.shared_experts.up_proj,
                           'mlp.gate': mlp.gate})
            subs.append({'layers': layers, 'prev_op': [block.post_attention_layernorm],
                         'input': ['mlp'], 'inspect': mlp, 'has_kwargs': False,
                         'is_mlp': True})
            for i in range(n):
                subs.append({'layers': {f'mlp.experts.{i}.down_proj': mlp.experts[i].down_proj},
                             'prev_op': [mlp.experts[i].up_proj],
                             'input': [f'mlp.experts.{i}.down_proj'],
                             'inspect': mlp.experts[i].down_proj, 'has_kwargs': False,
                             'is_mlp': True})
            subs.append({'layers': {'mlp.shared_experts.down_proj':
                                    mlp.shared_experts.down_proj},
                         'prev_op': [mlp.shared_experts.up_proj],
                         'input': ['mlp.shared_experts.down_proj'],
                         'inspect': mlp.shared_experts.down_proj, 'has_kwargs': False})
        else:
            subs.append({'layers': {'mlp.gate_proj': mlp.gate_proj, 'mlp.up_proj': mlp.up_proj},
                         'prev_op': [block.post_attention_layernorm],
                         'input': ['mlp.gate_proj'], 'inspect': mlp, 'has_kwargs': False})
            subs.append({'layers': {'mlp.down_proj': mlp.down_proj},
                         'prev_op': [mlp.up_proj], 'input': ['mlp.down_proj'],
                         'inspect': mlp.down_proj, 'has_kwargs': False})
        return subs
