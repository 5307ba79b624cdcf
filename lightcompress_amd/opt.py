"""OPT model adapter (drop-in for llmc ``models/opt.py:1-89``): decoder layers, biased
linears and LayerNorms, and the four AWQ/GPTQ subsets. fc2's subset has ``do_trans: False``
(opt.py:88): AWQ leaves it unscaled (awq.py:309-312), GPTQ and RTN still quantize it.
OPT stores fp16 weights; every exact nn.Linear runs on the lcq GEMM (fp16 operands, bias in
the epilogue)."""
from __future__ import annotations

import torch

from .base_model import BaseModel
from .registry import MODEL_REGISTRY


@MODEL_REGISTRY
class Opt(BaseModel):
    block_name_prefix = 'model.decoder.layers'
    default_dtype = torch.float16
    pairs = {'q_proj': 'qkv', 'out_proj': 'out', 'fc1': 'fc1'}

    def find_blocks(self):
        self.blocks = self.model.model.decoder.layers

    def find_embed_layers(self):
        dec = self.model.model.decoder
        self.embed_tokens = dec.embed_tokens
        self.embed_positions = dec.embed_positions

    def get_embed_layers(self):
        return [self.embed_tokens, self.embed_positions]

    def get_head_layers(self):
        return [self.model.lm_head]

    def get_pre_head_layernorm_layers(self):
        return [self.model.model.decoder.final_layer_norm]

    def has_bias(self):
        return True

    def get_layernorms_in_block(self, block):
        return {'self_attn_layer_norm': block.self_attn_layer_norm,
                'final_layer_norm': block.final_layer_norm}

    def get_subsets_in_block(self, block):
        """opt.py:53-89."""
        a = block.self_attn
        return [
            {'layers': {'self_attn.q_proj': a.q_proj, 'self_attn.k_proj': a.k_proj,
                        'self_attn.v_proj': a.v_proj},
             'prev_op': [block.self_attn_layer_norm], 'input': ['self_attn.q_proj'],
             'inspect': a, 'has_kwargs': True},
            {'layers': {'self_attn.out_proj': a.out_proj},
             'prev_op': [a.v_proj], 'input': ['self_attn.out_proj'],
             'inspect': a.out_proj, 'has_kwargs': False},
            {'layers': {'fc1': block.fc1},
             'prev_op': [block.final_layer_norm], 'input': ['fc1'],
             'inspect': block.fc1, 'has_kwargs': False, 'is_mlp': True},
            {'layers': {'fc2': block.fc2},
             'prev_op': [block.fc1], 'input': ['fc2'],
             'inspect': block.fc2, 'has_kwargs': False, 'is_mlp': True, 'do_trans': False},
        ]
