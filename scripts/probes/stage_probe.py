"""Count staged-forward memo hits/misses through a small GPTQ run (2 blocks)."""
import os
import sys
from pathlib import Path

import torch

os.environ['LCQ_STAGE_DEBUG'] = '1'
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from transformers import LlamaConfig  # noqa: E402
import bench  # noqa: E402
from lightcompress_amd import llama as L  # noqa: E402
from lightcompress_amd.pipeline import build_algo  # noqa: E402

cfg = LlamaConfig(hidden_size=512, intermediate_size=1024, num_attention_heads=8,
                  num_key_value_heads=2, num_hidden_layers=3, vocab_size=128)
model = L.Llama.random(cfg, device='cuda', seed=1)
seq, n = 128, 8
hidden = bench.synthetic_hidden(n, seq, 512, 'cuda', 3)
kw = model.rotary_kwargs(seq)
calib = {'data': [hidden[i:i + 1] for i in range(n)], 'kwargs': [kw] * n}
algo = build_algo(model, bench.gptq_config(seq, n), calib)
for i, b in enumerate(model.get_blocks()):
    L.STAGE_STATS.clear()
    algo.block_idx = i
    algo.block_opt(b)
    print('block', i, dict(sorted(L.STAGE_STATS.items())), flush=True)
