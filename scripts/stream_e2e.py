"""Host-resident (residency: stream) Llama-3-8B-shaped AWQ run over a few blocks, for the
rocprofv3 kernel + memory-copy trace that shows the block uploads overlapping the compute
(scripts/copy_overlap.py summarises it)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from lightcompress_amd.llama import Llama  # noqa: E402
from lightcompress_amd.pipeline import build_algo  # noqa: E402
from transformers import LlamaConfig  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = torch.device('cuda:0')
cfg = LlamaConfig(**bench.LLAMA3_8B)
model = Llama.random(cfg, num_layers=nb, device=dev, seed=3000, residency='stream')
torch.cuda.empty_cache()
hidden = bench.synthetic_hidden(128, 512, cfg.hidden_size, dev, 41)
algo = build_algo(model, bench.awq_config(512, 128),
                  {'data': [hidden], 'kwargs': [model.rotary_kwargs(512)]})
algo.run_block_loop()
algo.deploy('vllm_quant')
torch.cuda.synchronize()
print('stream stats', model.streamer.stats, flush=True)
