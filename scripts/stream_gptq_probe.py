"""Where the host-streamed GPTQ run's extra time goes (streamed 9.85 s vs
resident 7.05 s over 32 Llama-3-8B blocks). Times fresh pinned host allocations of the sizes the
fp32 write-back asks for, then runs N blocks resident and streamed (run_block_loop + deploy
fake_quant, the bench's e2e recipe) with the streamed run under cProfile.

usage: python scripts/stream_gptq_probe.py [N]
"""
import cProfile
import pstats
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from lightcompress_amd.llama import Llama  # noqa: E402
from lightcompress_amd.pipeline import build_algo  # noqa: E402
from transformers import LlamaConfig  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
profile = len(sys.argv) <= 2 or sys.argv[2] != "noprof"
dev = torch.device('cuda:0')
from lightcompress_amd import _native  # noqa: E402
_native.load()

for shape in [(14336, 4096), (4096, 14336), (4096, 4096)]:
    t0 = time.perf_counter()
    h = torch.empty(shape, dtype=torch.float32, pin_memory=True)
    t1 = time.perf_counter()
    print(f'pinned alloc fp32 {shape}: {(t1 - t0) * 1e3:.1f} ms '
          f'({h.numel() * 4 / 2**20:.0f} MiB)', flush=True)
    del h

cfg = LlamaConfig(**bench.LLAMA3_8B)
seq, ns = 2048, 128


def run(residency, prof=None):
    model = Llama.random(cfg, num_layers=nb, device=dev, seed=4000, residency=residency)
    torch.cuda.empty_cache()
    hidden = bench.synthetic_hidden(ns, seq, cfg.hidden_size, dev, 43)
    kw = model.rotary_kwargs(seq)
    calib = {'data': [hidden[i:i + 1] for i in range(ns)], 'kwargs': [kw] * ns}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if prof is not None:
        prof.enable()
    algo = build_algo(model, bench.gptq_config(seq, ns), calib)
    algo.run_block_loop()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    algo.deploy('fake_quant')
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if prof is not None:
        prof.disable()
    st = model.streamer.stats if model.streamer is not None else None
    print(f'{residency}: block loop {t1 - t0:.2f} s, deploy {t2 - t1:.2f} s, stats {st}',
          flush=True)
    algo.release()
    del algo, model, hidden, calib
    bench.free_device()


run('device')
prof = cProfile.Profile() if profile else None
run('stream', prof)
if prof is not None:
    st = pstats.Stats(prof)
    st.sort_stats('tottime').print_stats(25)
