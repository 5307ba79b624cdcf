"""Helpers shared by the AWQ tests: rebuild the tiny HF Llama layer of the golden fixtures
and run its inspect modules with substituted weights."""
import torch

import fixtures as F


def build_layer(device='cpu'):
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml
    c = F.load('awq_layer')
    h, i, nh, kv = c['cfg'].tolist()
    cfg = LlamaConfig(hidden_size=h, intermediate_size=i, num_attention_heads=nh,
                      num_key_value_heads=kv, num_hidden_layers=1, vocab_size=128,
                      max_position_embeddings=2048, rms_norm_eps=1e-5)
    cfg._attn_implementation = 'sdpa'
    layer = ml.LlamaDecoderLayer(cfg, layer_idx=0).to(torch.bfloat16)
    sd = {k.replace('__', '.'): v for k, v in c.items()
          if k not in ('hidden', 'cos', 'sin', 'cfg')}
    layer.load_state_dict(sd)
    layer = layer.to(device).eval()
    kwargs = {'position_embeddings': (c['cos'].to(device), c['sin'].to(device)),
              'attention_mask': None,
              'position_ids': torch.arange(c['cos'].shape[1], device=device).unsqueeze(0)}
    return cfg, layer, kwargs


SUBSETS = {
    'qkv': (('self_attn.q_proj', 'self_attn.k_proj', 'self_attn.v_proj'), 'self_attn', True),
    'mlp': (('mlp.gate_proj', 'mlp.up_proj'), 'mlp', False),
    'down': (('mlp.down_proj',), 'mlp.down_proj', False),
}


def forward_fn(layer, subset, kwargs):
    names, inspect_name, has_kw = SUBSETS[subset]
    mods = [layer.get_submodule(n) for n in names]
    inspect = layer.get_submodule(inspect_name)

    @torch.no_grad()
    def fwd(x, qweights):
        saved = [m.weight.data for m in mods]
        if qweights is not None:
            for m, w in zip(mods, qweights):
                m.weight.data = w
        out = inspect(x, **kwargs) if has_kw else inspect(x)
        if isinstance(out, tuple):
            out = out[0]
        for m, w in zip(mods, saved):
            m.weight.data = w
        return out
    return fwd, [m.weight.data for m in mods]
