"""Tiny random models of the three adapter families for the end-to-end pipeline goldens
(tests/golden/gen_pipeline.py writes them next to this file; tests load the same files).

* Llama: 2 layers, GQA (hidden 256, MLP 512, 4 heads / 2 kv heads), bf16.
* OPT: 2 layers (hidden 256, ffn 1024, 4 heads of 64), biased linears + LayerNorms, fp16 —
  OPT-125M's layout at a quarter of its width.
* DeepSeek-V3: 2 layers, MLA (q_lora 128, kv_lora 128, rope 64, nope 32, v 32; kv_a_proj
  has 192 rows: auto-clip needs OC % 64, auto_clip.py:109), layer 0 dense
  (first_k_dense_replace 1), layer 1 MoE with 4 routed experts (top-2, sigmoid router with
  group-limited top-k) + 1 shared expert, bf16.

Every matrix parameter ~ N(0, 0.02²) (router: N(0, 0.1²), for decisive routing); norm weights ~ U(0.8, 1.2); biases ~ N(0, 0.02²); the
token embedding has log-normal per-channel magnitudes so that AWQ's scale search has outlier
channels to find.
"""
from __future__ import annotations

import shutil
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
MODEL_DIRS = {'Llama': HERE / 'pipeline_llama', 'Opt': HERE / 'pipeline_opt',
              'DeepseekV3': HERE / 'pipeline_dsv3'}
# block linears: Llama 2 x 7; OPT 2 x 6; DSv3 dense block 5 MLA + 3 MLP, MoE block
# 5 MLA + 4 experts x 3 + shared 3 (the router is not a linear)
N_LINEARS = {'Llama': 14, 'Opt': 12, 'DeepseekV3': 8 + 5 + 4 * 3 + 3}


def _init(m, emb):
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2:  # linears and DSv3's fused 3-D expert tensors
                p.normal_(0, 0.02, generator=g)
            elif n.endswith('bias'):
                p.normal_(0, 0.02, generator=g)
            else:
                p.uniform_(0.8, 1.2, generator=g)
        emb.copy_(torch.randn(emb.shape, generator=g) *
                  torch.exp(torch.randn(emb.shape[1], generator=g) * 0.8))


def llama_config():
    from transformers import LlamaConfig
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=2, vocab_size=128,
                      max_position_embeddings=512, rms_norm_eps=1e-5, tie_word_embeddings=False)
    cfg._attn_implementation = 'sdpa'
    return cfg


def opt_config():
    from transformers import OPTConfig
    cfg = OPTConfig(hidden_size=256, ffn_dim=1024, num_attention_heads=4, num_hidden_layers=2,
                    vocab_size=128, max_position_embeddings=512, word_embed_proj_dim=256,
                    do_layer_norm_before=True, enable_bias=True, dropout=0.0,
                    attention_dropout=0.0, tie_word_embeddings=False)
    cfg._attn_implementation = 'sdpa'
    return cfg


def dsv3_config():
    from transformers import DeepseekV3Config
    cfg = DeepseekV3Config(hidden_size=256, intermediate_size=512, moe_intermediate_size=128,
                           num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=4,
                           n_shared_experts=1, n_routed_experts=4, num_experts_per_tok=2,
                           n_group=1, topk_group=1, first_k_dense_replace=1, q_lora_rank=128,
                           kv_lora_rank=128, qk_nope_head_dim=32, qk_rope_head_dim=64,
                           v_head_dim=32, vocab_size=128, max_position_embeddings=512,
                           rms_norm_eps=1e-6, tie_word_embeddings=False, norm_topk_prob=True,
                           routed_scaling_factor=2.5)
    cfg._attn_implementation = 'sdpa'
    return cfg


def build(family):
    """The random model of `family` (CPU, its storage dtype), built from the seeds above."""
    torch.manual_seed(0)
    if family == 'Llama':
        from transformers import LlamaForCausalLM
        m = LlamaForCausalLM(llama_config())
        _init(m, m.model.embed_tokens.weight)
        return m.to(torch.bfloat16)
    if family == 'Opt':
        from transformers import OPTForCausalLM
        m = OPTForCausalLM(opt_config())
        _init(m, m.model.decoder.embed_tokens.weight)
        return m.to(torch.float16)
    if family == 'DeepseekV3':
        from transformers import DeepseekV3ForCausalLM
        m = DeepseekV3ForCausalLM(dsv3_config())
        _init(m, m.model.embed_tokens.weight)
        g = torch.Generator().manual_seed(2)
        with torch.no_grad():  # decisive routing: router logits of O(1), not O(0.02 sqrt(H))
            for lay in m.model.layers:
                if hasattr(lay.mlp, 'gate'):
                    lay.mlp.gate.weight.normal_(0, 0.1, generator=g)
        return m.to(torch.bfloat16)
    raise KeyError(family)


def save(family):
    d = MODEL_DIRS[family]
    if d.exists():
        shutil.rmtree(d)
    build(family).save_pretrained(d)
    return d
