"""Device memory of a streamed vs an HBM-resident AWQ run (the shapes of
tests/test_residency_gpu.py::test_stream_bounds_device_memory): allocated bytes at every
block visit, the peak per phase, and how many blocks the streamer holds."""
import gc
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from transformers import LlamaConfig  # noqa: E402

from lightcompress_amd import base_blockwise_quantization as B  # noqa: E402
from lightcompress_amd.llama import Llama  # noqa: E402
from lightcompress_amd.pipeline import build_algo  # noqa: E402
from lightcompress_amd.utils import load_config  # noqa: E402

dev = torch.device('cuda:0')
cfg = LlamaConfig(hidden_size=512, intermediate_size=2048, num_attention_heads=8,
                  num_key_value_heads=4, num_hidden_layers=12, vocab_size=128,
                  max_position_embeddings=512, rms_norm_eps=1e-5)
conf = load_config({'calib': {'seq_len': 64},
                    'quant': {'method': 'Awq', 'weight': {'bit': 4, 'symmetric': True,
                                                          'granularity': 'per_group',
                                                          'group_size': 128, 'need_pack': True},
                              'special': {'trans': True, 'trans_version': 'v2',
                                          'weight_clip': True, 'clip_sym': True},
                              'quant_out': False}})
orig = B.BlockwiseOpt.visit_block
log = []


def visit(self, i, fn, next_i=None, dirty=True):
    r = orig(self, i, fn, next_i, dirty)
    st = getattr(self.model, 'streamer', None)
    log.append((i, torch.cuda.memory_allocated(dev) / 2**20,
                torch.cuda.max_memory_allocated(dev) / 2**20,
                None if st is None else (len(st.resident), len(st.pending))))
    return r


B.BlockwiseOpt.visit_block = visit
for res in ('device', 'stream'):
    log.clear()
    model = Llama.random(cfg, device=dev, seed=3, residency=res)
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    start = torch.cuda.memory_allocated(dev) / 2**20
    torch.cuda.reset_peak_memory_stats(dev)
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(4, 64, 512, generator=g, device=dev).to(torch.bfloat16)
    algo = build_algo(model, conf, {'data': [x], 'kwargs': [model.rotary_kwargs(64)]})
    algo.run_block_loop()
    torch.cuda.synchronize()
    p1 = torch.cuda.max_memory_allocated(dev) / 2**20
    algo.deploy('vllm_quant')
    torch.cuda.synchronize()
    p2 = torch.cuda.max_memory_allocated(dev) / 2**20
    print(f'{res}: start {start:.1f} MiB, peak block loop {p1:.1f}, peak incl. deploy {p2:.1f}')
    for row in log:
        print('   block %d: allocated %.1f MiB, peak so far %.1f, (resident, pending) %s' % row)
    algo.release()
    del algo, x, model
    gc.collect()
    torch.cuda.empty_cache()
