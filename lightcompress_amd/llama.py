"""Llama model adapter (drop-in for llmc ``models/llama.py`` + the BaseModel contract the hot
path consumes, base_model.py:174-436): blocks, block linears, AWQ/GPTQ subsets, module
replacement, first-block input capture. The model lives in HBM for the whole run.
"""
from __future__ import annotations

import types

import torch
import torch.nn as nn

from .base_model import BaseModel, _linear_forward
from .registry import MODEL_REGISTRY


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


_ORIG_SDPA = None
# measured on MI355X (scripts/attn_rate.py, B 128, H 32, KV 8): the lcq flash kernel vs torch's
# SDPA (aotriton) 0.87 vs 1.66 ms at S 512 (AWQ calibration), 9.26 vs 10.79 ms at S 2048 (GPTQ);
# longer sequences (not measured) go to torch.
_LCQ_ATTN_MAX_S = 4096


def _lcq_sdpa(module, query, key, value, attention_mask, dropout=0.0, scaling=None,
              is_causal=None, **kwargs):
    """transformers' sdpa attention function with the calibration case routed to
    lcq_attn_fwd_causal: causal, no mask / dropout / position bias, bf16, head dim 128,
    q_len == kv_len. Anything else goes to the original sdpa_attention_forward."""
    from . import ops
    causal = is_causal if is_causal is not None else getattr(module, 'is_causal', True)
    S = query.shape[2]
    if (causal and attention_mask is None and dropout == 0.0 and query.is_cuda
            and query.dtype == torch.bfloat16 and key.dtype == torch.bfloat16
            and value.dtype == torch.bfloat16 and query.shape[-1] == 128
            and key.shape[2] == S and 1 < S <= _LCQ_ATTN_MAX_S
            and kwargs.get('position_bias') is None and not kwargs.get('output_attentions')
            and query.shape[1] % key.shape[1] == 0
            and all(t.stride(-1) == 1 and all(st % 8 == 0 for st in t.stride()[:3])
                    for t in (query, key, value))):
        scale = scaling if scaling is not None else query.shape[-1] ** -0.5
        return ops.attn_fwd_causal(query, key, value, scale), None
    return _ORIG_SDPA(module, query, key, value, attention_mask, dropout=dropout,
                      scaling=scaling, is_causal=is_causal, **kwargs)


def _linear_wb(m):
    """(weight, bias) of a module whose forward is exactly x W^T + b through lcq_linear: an
    nn.Linear, or a weight-only fake-quant linear (its fake-quantised weight, materialised the
    way its own first forward would); None for anything else."""
    from .module_utils import EffcientFakeQuantLinear, FakeQuantLinear
    t = type(m)
    if t is nn.Linear:
        return m.weight, m.bias
    if t is EffcientFakeQuantLinear and m.a_qdq is None:
        return m.weight, m.bias
    if (t is FakeQuantLinear and m.a_qdq is None and not m.dynamic_quant_weight
            and not m.dynamic_quant_tmp_weight):
        if not hasattr(m, 'tmp_weight'):  # FakeQuantLinear.forward's first call
            m.register_buffer('tmp_weight', m.w_qdq(m), persistent=False)
            m.tmp_bias = m.bias
        return m.tmp_weight, m.tmp_bias
    return None


def _input_only_hooked(*mods):
    """Linear-like modules (_linear_wb) whose hooks (if any) all read only the module inputs
    (the capture hooks of algorithms whose add_batch ignores the output, marked
    `_lcq_input_only` by BaseBlockwiseQuantization.register_hooks)."""
    return all(_linear_wb(m) is not None and all(
        getattr(h, '_lcq_input_only', False)
        for h in (*m._forward_pre_hooks.values(), *m._forward_hooks.values()))
        for m in mods)


def _fire_input_hooks(m, x):
    """The hooks a module call would fire, in the same order (pre, then forward), with the
    output None: only for input-only hooks (_input_only_hooked)."""
    for h in m._forward_pre_hooks.values():
        h(m, (x,))
    for h in m._forward_hooks.values():
        h(m, (x,), None)


def _gate_up_silu(mlp, x):
    """act_fn(gate_proj(x)) * up_proj(x): one lcq GEMM with the SiLU product in its epilogue
    when both projections are bias-free linears the GEMM takes and carry no hooks, or only
    input-capture hooks (GPTQ's calibration forward: the hooks fire first, in module order,
    and the two [M, I] projections are never written); otherwise the projections run as
    modules (hooks fire in order) and lcq_silu_mul makes the product."""
    from . import ops
    gp, up = mlp.gate_proj, mlp.up_proj
    if (getattr(mlp.config, 'hidden_act', None) == 'silu'
            and _input_only_hooked(gp, up)):
        (gw, gb), (uw, ub) = _linear_wb(gp), _linear_wb(up)
        if (gb is None and ub is None and ops.gemm_supported(x, gw, uw)
                and gw.stride(0) == uw.stride(0)):
            _fire_input_hooks(gp, x)
            _fire_input_hooks(up, x)
            return ops.linear_silu_mul(x, gw, uw)
    g = gp(x)
    u = up(x)
    if g.is_cuda and g.dtype in (torch.bfloat16, torch.float16) and g.shape == u.shape \
            and u.dtype == g.dtype and g.numel() % 8 == 0 \
            and getattr(mlp.config, 'hidden_act', None) == 'silu':
        return ops.silu_mul(g, u)
    return mlp.act_fn(g) * u


def _fused_mlp_forward(self, x):
    """LlamaMLP.forward with act_fn(gate) * up fused (see _gate_up_silu)."""
    return self.down_proj(_gate_up_silu(self, x))




def _fused_rmsnorm_forward(self, hidden_states):
    """LlamaRMSNorm.forward on one lcq_rmsnorm pass (same formula; the variance is summed in
    a fixed order of its own)."""
    from . import ops
    if (hidden_states.is_cuda and hidden_states.dtype in (torch.bfloat16, torch.float16)
            and self.weight.dtype == hidden_states.dtype and hidden_states.shape[-1] % 8 == 0
            and hidden_states.shape[-1] <= 16384):
        return ops.rmsnorm(hidden_states, self.weight, self.variance_epsilon)
    input_dtype = hidden_states.dtype
    h = hidden_states.to(torch.float32)
    variance = h.pow(2).mean(-1, keepdim=True)
    h = h * torch.rsqrt(variance + self.variance_epsilon)
    return self.weight * h.to(input_dtype)


def _proj_residual(mod, x, res):
    """res + mod(x) (the decoder block's residual adds after o_proj and down_proj) with the
    add in the GEMM epilogue when mod is a linear the GEMM takes and carries no hooks, or only
    input-capture hooks (fired first, as the module call would); otherwise the module runs."""
    from . import ops
    if _input_only_hooked(mod):
        w, b = _linear_wb(mod)
        if (ops.gemm_supported(x, w) and res.dtype == x.dtype
                and res.shape[:-1] == x.shape[:-1] and res.shape[-1] == w.shape[0]
                and (b is None or b.dtype == x.dtype)):
            _fire_input_hooks(mod, x)
            return ops.linear_residual(x, w, res, b)
    return res + mod(x)


def _mkey(*mods):
    """Identity + weight storage/version of the modules a cached stage depends on (an in-place
    weight update bumps _version, a replaced module or re-pointed .data changes the rest)."""
    out = []
    for m in mods:
        w = getattr(m, 'weight', None)
        out.append((id(m), type(m).__name__, None if w is None else
                    (w.data_ptr(), w._version, tuple(w.shape), w.dtype)))
    return tuple(out)


def _hooked(*mods):
    return any(m._forward_hooks or m._forward_pre_hooks for m in mods)


STAGE_STATS = {}  # (stage, 'hit' | 'miss' | 'hooked') -> count, for diagnostics


def _stage(cache, name, key, mods, fn):
    hit = cache.get(name)
    hooked = _hooked(*mods)
    if hit is not None and hit[0] == key and not hooked:
        STAGE_STATS[(name, 'hit')] = STAGE_STATS.get((name, 'hit'), 0) + 1
        return hit[1]
    why = 'hooked' if hooked else ('miss' if hit is None else 'stale')
    STAGE_STATS[(name, why)] = STAGE_STATS.get((name, why), 0) + 1
    val = fn()
    cache[name] = (key, val)
    return val


def _rope_fusable(attn, xn, rope):
    """The rotary embedding can go into the q/k/v GEMM's epilogue (lcq_gemm_rope): the
    patched apply_rotary_pos_emb would have run lcq_rotary on these shapes, heads of 128."""
    if rope is None or xn.dim() != 3 or getattr(attn, 'head_dim', None) != 128:
        return False
    from transformers.models.llama import modeling_llama as ml
    cos, sin = rope
    B, S = xn.shape[0], xn.shape[1]
    return (ml.apply_rotary_pos_emb is _fused_apply_rotary and cos.dim() == 3
            and cos.dtype == xn.dtype and sin.dtype == xn.dtype and sin.shape == cos.shape
            and cos.shape[0] in (1, B) and tuple(cos.shape[1:]) == (S, 128))


def qkv_proj(attn, xn, weights=None, rope=None):
    """q / k / v projections of LlamaAttention: one lcq GEMM launch for the three when they
    are linears the GEMM takes with no hooks or only input-capture hooks (x read once), else
    the three modules. `weights` overrides the three weights (the AWQ search's
    fake-quantized copies; their modules' hooks are not fired). `rope` = (cos, sin): when
    the launch can take it, q and k come back already rotated (lcq_gemm_rope) and the
    returned flag is True; callers then skip apply_rotary_pos_emb."""
    from . import ops
    mods = (attn.q_proj, attn.k_proj, attn.v_proj)
    fused = weights is not None or _input_only_hooked(*mods)
    if weights is not None:
        ws, bs = list(weights), [m.bias for m in mods]
    elif fused:
        wb = [_linear_wb(m) for m in mods]
        ws, bs = [w for w, _ in wb], [b for _, b in wb]
    if (fused and ops.gemm_supported(xn, *ws)
            and len({w.stride(0) for w in ws}) == 1
            and all(w.shape[0] % 256 == 0 for w in ws[:2])
            and all(b is None or b.dtype == xn.dtype for b in bs)):
        if weights is None:  # input-capture hooks fire first, in module order
            for m in mods:
                _fire_input_hooks(m, xn)
        if _rope_fusable(attn, xn, rope):
            return (*ops.linear_multi_rope(xn, ws, bs, rope[0], rope[1], rope_segs=2), True)
        return (*ops.linear_multi(xn, ws, bs), False)
    if weights is not None:
        from .module_utils import lcq_linear
        return (*[lcq_linear(xn, w, m.bias) for w, m in zip(ws, mods)], False)
    return (*[m(xn) for m in mods], False)


def _attn_core(attn, xn, position_embeddings, attention_mask, qkv_weights=None, **kwargs):
    """LlamaAttention.forward up to (not including) o_proj, exactly as transformers runs it."""
    from transformers.models.llama import modeling_llama as ml
    input_shape = xn.shape[:-1]
    hidden_shape = (*input_shape, -1, attn.head_dim)
    cos, sin = position_embeddings
    q, k, v, rotated = qkv_proj(attn, xn, qkv_weights, rope=(cos, sin))
    q = q.view(hidden_shape).transpose(1, 2)
    k = k.view(hidden_shape).transpose(1, 2)
    v = v.view(hidden_shape).transpose(1, 2)
    if not rotated:
        q, k = ml.apply_rotary_pos_emb(q, k, cos, sin)
    iface = ml.ALL_ATTENTION_FUNCTIONS.get_interface(attn.config._attn_implementation,
                                                      ml.eager_attention_forward)
    out, _ = iface(attn, q, k, v, attention_mask,
                   dropout=0.0 if not attn.training else attn.attention_dropout,
                   scaling=attn.scaling, **kwargs)
    return out.reshape(*input_shape, -1).contiguous()


_STOCK_DECODER_FORWARD = None


def _staged_decoder_forward(self, hidden_states, attention_mask=None, position_ids=None,
                            past_key_values=None, use_cache=False, position_embeddings=None,
                            **kwargs):
    """LlamaDecoderLayer.forward as four memoised stages: [norm1, q/k/v, attention],
    [o_proj + residual], [norm2, gate/up, SiLU product], [down + residual].

    GPTQ's true_sequential re-forwards and its quant_out forward re-run a block on the same
    input with one subset replaced each time (o_proj, then gate/up, then down): the stages
    before the replaced modules are identical and come from the memo. A stage is recomputed
    when its input, a module object or a weight (storage or in-place version) changed, and
    always when one of its modules carries hooks (so input captures keep firing)."""
    attn, mlp = self.self_attn, self.mlp
    if (past_key_values is not None or not hidden_states.is_cuda
            or _hooked(self, attn, mlp)):
        return _STOCK_DECODER_FORWARD(self, hidden_states, attention_mask=attention_mask,
                                      position_ids=position_ids,
                                      past_key_values=past_key_values, use_cache=use_cache,
                                      position_embeddings=position_embeddings, **kwargs)
    cache = self.__dict__.setdefault('_lcq_stage', {})
    key = (id(hidden_states), hidden_states.data_ptr(), hidden_states._version,
           tuple(hidden_states.shape), id(attention_mask), id(position_embeddings),
           id(position_ids), tuple(sorted(kwargs)))
    key = key + _mkey(self.input_layernorm, attn.q_proj, attn.k_proj, attn.v_proj)
    core = _stage(cache, 'core', key,
                  (self.input_layernorm, attn.q_proj, attn.k_proj, attn.v_proj),
                  lambda: _attn_core(attn, self.input_layernorm(hidden_states),
                                     position_embeddings, attention_mask,
                                     position_ids=position_ids, use_cache=use_cache, **kwargs))
    key = key + _mkey(attn.o_proj)
    h = _stage(cache, 'h', key, (attn.o_proj,),
               lambda: _proj_residual(attn.o_proj, core, hidden_states))
    key = key + _mkey(self.post_attention_layernorm, mlp.gate_proj, mlp.up_proj)

    def _mlp_in():
        return _gate_up_silu(mlp, self.post_attention_layernorm(h))

    m = _stage(cache, 'm', key, (self.post_attention_layernorm, mlp.gate_proj, mlp.up_proj),
               _mlp_in)
    return _proj_residual(mlp.down_proj, m, h)


def clear_stage_cache(block: nn.Module):
    for mod in block.modules():
        mod.__dict__.pop('_lcq_stage', None)


def install_fused_forward(model: nn.Module):
    """Route the Llama calibration forward's elementwise chains through the lcq fusions."""
    global _ORIG_ROTARY
    from transformers.models.llama import modeling_llama as ml
    if _ORIG_ROTARY is None:
        _ORIG_ROTARY = ml.apply_rotary_pos_emb
        ml.apply_rotary_pos_emb = _fused_apply_rotary
    global _ORIG_SDPA
    if _ORIG_SDPA is None:
        from transformers.modeling_utils import AttentionInterface
        _ORIG_SDPA = AttentionInterface._global_mapping['sdpa']
        AttentionInterface.register('sdpa', _lcq_sdpa)
    global _STOCK_DECODER_FORWARD
    if _STOCK_DECODER_FORWARD is None:
        _STOCK_DECODER_FORWARD = ml.LlamaDecoderLayer.forward
    for m in model.modules():
        if type(m) is nn.Linear:
            m.forward = types.MethodType(_linear_forward, m)
        elif isinstance(m, ml.LlamaMLP) and getattr(m.config, 'hidden_act', None) == 'silu':
            m.forward = types.MethodType(_fused_mlp_forward, m)
        elif isinstance(m, ml.LlamaRMSNorm):
            m.forward = types.MethodType(_fused_rmsnorm_forward, m)
        elif isinstance(m, ml.LlamaDecoderLayer):
            m.forward = types.MethodType(_staged_decoder_forward, m)


class _Blocks(nn.Module):
    """Decoder layers + rotary embedding only (no vocab), for synthetic-input workloads."""

    def __init__(self, layers, rotary_emb):
        super().__init__()
        self.layers = nn.ModuleList(layers)
        self.rotary_emb = rotary_emb


@MODEL_REGISTRY
class Llama(BaseModel):
    """llama.py:1-91 on the BaseModel contract, with the Llama calibration-forward fusions."""
    block_name_prefix = 'model.layers'

    def find_blocks(self):
        inner = getattr(self.model, 'model', self.model)
        self.blocks = inner.layers
        self.rotary_emb = inner.rotary_emb

    def find_embed_layers(self):
        self.embed_tokens = getattr(getattr(self.model, 'model', self.model), 'embed_tokens',
                                    None)

    def install_fused_forward(self):
        install_fused_forward(self.model)

    def get_layernorms_in_block(self, block):
        return {'input_layernorm': block.input_layernorm,
                'post_attention_layernorm': block.post_attention_layernorm}

    # -- random-init constructor (synthetic benchmark / tests) --------------------------------
    @classmethod
    def random(cls, model_config, num_layers=None, device='cuda', dtype=torch.bfloat16,
               seed=0, std=0.02, residency=None):
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
        return cls(hf_model=blocks, device=device, residency=residency)

    def rotary_kwargs(self, seq_len, device=None):
        """Block kwargs the Catcher would capture for an unpadded causal batch."""
        device = device or self.device
        pos = torch.arange(seq_len, device=device).unsqueeze(0)
        cos, sin = self._rotary_table(pos)
        return {'position_embeddings': (cos, sin), 'attention_mask': None, 'position_ids': pos}

    def _rotary_table(self, pos):
        """LlamaRotaryEmbedding.forward's cos / sin (the model's own inv_freq and attention
        scaling, rope_scaling included) with its `inv_freq @ position_ids` -- a K = 1 product,
        one rounding per element -- as an elementwise outer product: the same values bit for
        bit, without a vendor GEMM launch. Rope types whose table depends on the sequence
        length (dynamic, longrope: `@dynamic_rope_update` rescales inv_freq) run the module."""
        re = self.rotary_emb
        if getattr(re, 'rope_type', 'default') not in ('default', 'llama3'):
            dummy = torch.empty(1, dtype=self.torch_dtype, device=pos.device)
            return re(dummy, pos)
        inv = re.inv_freq.float().to(pos.device)
        freqs = pos[0].float()[:, None] * inv[None, :]
        emb = torch.cat((freqs, freqs), dim=-1)
        scale = getattr(re, 'attention_scaling', 1.0)
        dt = self.torch_dtype
        return (emb.cos() * scale).to(dt)[None], (emb.sin() * scale).to(dt)[None]

    # -- BaseModel contract ---------------------------------------------------------------------
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

    def save_pretrained(self, path):
        if hasattr(self.model, 'save_pretrained'):
            self.model.save_pretrained(path)
            return
        # decoder-only stand-in (Llama.random): safetensors of the blocks + the HF config
        import os
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        sd = {f'model.{k}': v.detach().contiguous() for k, v in self.model.state_dict().items()
              if torch.is_tensor(v)}
        save_file(sd, os.path.join(path, 'model.safetensors'))
        self.model_config.to_json_file(os.path.join(path, 'config.json'))
