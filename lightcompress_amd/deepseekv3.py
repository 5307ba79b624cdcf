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
        if (top_k_weights.dtype in (torch.float32, torch.bfloat16, torch.float16)
                and self._grouped_fp8_ok(hidden_states)):
            return self._forward_grouped_fp8(hidden_states, top_k_index, top_k_weights)
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

    # ---- one launch per projection for block-fp8 experts ----------------------------------
    # The loop above is the reference's expert loop: per hit expert, act_quant + fp8 GEMM for
    # gate, up and down on that expert's tokens (3 x E launches of a few hundred workgroups,
    # 0.18 of the fp8 MFMA peak at 2048 tokens per expert). When every expert is a plain
    # block-fp8 MLP and nothing observes the per-expert calls (no hooks: calibration capture
    # registers them and then takes the loop), the experts run as grouped GEMMs instead: the
    # token slots are sorted by expert on the device (no host sync), act_quant runs once per
    # token (it is per row), one lcq_fp8_gemm_grouped launch computes gate and up of every
    # expert (the kernel gathers each slot's token row) and, for SiLU, act_fn(gate) * up in its
    # epilogue as the MLP computes it on the bf16 projections; one launch for down, then lcq_moe_combine in the loop's order (per token, experts in
    # ascending index, each product rounded to bf16 before its add, as index_add_ does).
    # Every row's GEMM value equals lcq_fp8_gemm's on an unsplit 256^2 plan.
    def _grouped_fp8_ok(self, x) -> bool:
        from .module_utils import USE_FP8GEMM_TRITON_KERNEL, LlmcFp8Linear
        if (not USE_FP8GEMM_TRITON_KERNEL or not len(self) or x.dim() != 2 or not x.is_cuda
                or x.dtype != torch.bfloat16 or len(self) > 1 << 20
                or torch.nn.modules.module._global_forward_hooks
                or torch.nn.modules.module._global_forward_pre_hooks):
            return False
        mlp_forward = _mlp_forward()
        for mlp in self:
            if mlp_forward is None or type(mlp).forward is not mlp_forward:
                return False
            for m in (mlp, mlp.gate_proj, mlp.up_proj, mlp.down_proj):
                if m._forward_hooks or m._forward_pre_hooks:
                    return False
            for lin in (mlp.gate_proj, mlp.up_proj, mlp.down_proj):
                if (type(lin) is not LlmcFp8Linear or lin.bias is not None
                        or lin.block_size != 128 or lin.weight.dtype != torch.float8_e4m3fn
                        or lin.weight.device != x.device):
                    return False
        return True

    def _fp8_tables(self, device):
        """([2, E, 2] gate + up, [E, 2] down) device tables of the experts' (weight, scale)
        addresses, rebuilt when any weight tensor changed (the modules keep the tensors)."""
        key = tuple((lin.weight.data_ptr(), lin.weight_scale_inv.data_ptr())
                    for mlp in self for lin in (mlp.gate_proj, mlp.up_proj, mlp.down_proj))
        cached = getattr(self, '_lcq_fp8_tables', None)
        if cached is None or cached[0] != key:
            from . import ops
            gate, up, down = (ops.fp8_weight_table(
                [(getattr(mlp, p).weight.data, getattr(mlp, p).weight_scale_inv.data)
                 for mlp in self], device) for p in ('gate_proj', 'up_proj', 'down_proj'))
            cached = (key, (torch.stack([gate, up]).contiguous(), down))
            self._lcq_fp8_tables = cached
        return cached[1]

    def _forward_grouped_fp8(self, hidden_states, top_k_index, top_k_weights):
        from . import ops
        from .kernel import act_quant
        T, k = top_k_index.shape
        E, H = len(self), hidden_states.shape[1]
        if T == 0:
            return torch.zeros_like(hidden_states)
        inter = self[0].gate_proj.out_features
        gate_up, down = self._fp8_tables(hidden_states.device)
        # C in the default dtype, then bf16, as block_wise_fp8_forward_func (fp32 default:
        # the kernel's round-to-nearest-even bf16 store is the same single rounding)
        cdt = torch.get_default_dtype()
        cdt = torch.bfloat16 if cdt == torch.float32 else cdt
        with torch.no_grad():
            flat = top_k_index.reshape(-1)
            order = torch.argsort(flat, stable=True)          # sorted row -> (token, slot)
            row_off = torch.zeros(E + 1, dtype=torch.int64, device=flat.device)
            torch.cumsum(torch.bincount(flat, minlength=E), 0, out=row_off[1:])
            slot_row = torch.empty_like(order)                # (token, slot) -> sorted row
            slot_row[order] = torch.arange(order.numel(), device=order.device)
        # act_quant is per token row: quantize each token once, the GEMM gathers its k copies
        xq, xs = act_quant(hidden_states.contiguous(), 128)
        if cdt == torch.bfloat16 and getattr(self[0].config, 'hidden_act', None) == 'silu':
            # act_fn(gate) * up in the GEMM epilogue (the bf16 projections never stored)
            h = ops.fp8_gemm_grouped(xq, xs.reshape(-1), row_off, gate_up, inter, cdt,
                                     a_rows=order // k, silu_mul=True)
        else:
            gu = ops.fp8_gemm_grouped(xq, xs.reshape(-1), row_off, gate_up, inter, cdt,
                                      a_rows=order // k).to(torch.bfloat16)
            h = (self[0].act_fn(gu[0]) * gu[1]).contiguous()
            del gu
        del xq, xs
        hq, hs = act_quant(h, 128)
        del h
        y = ops.fp8_gemm_grouped(hq, hs.reshape(-1), row_off, down, H, cdt).to(torch.bfloat16)
        del hq, hs
        w = top_k_weights if top_k_weights.dtype != torch.float16 else top_k_weights.float()
        return ops.moe_combine(y, slot_row, top_k_index.to(torch.int64), w, T)

def _mlp_forward():
    try:
        from transformers.models.deepseek_v3 import modeling_deepseek_v3 as md
    except ImportError:  # pragma: no cover - transformers without DeepSeek-V3
        return None
    return md.DeepseekV3MLP.forward


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
