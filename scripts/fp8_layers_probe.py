"""Where the FP8 deploy leg's host time goes as the model grows: build the
bench's DSv3 model at L layers, run run_block_loop + deploy('vllm_quant') under cProfile and
print the per-layer wall time of both phases plus the top functions.

usage: python scripts/fp8_layers_probe.py L [L ...]   (writes gpurun_out/fp8_probe_L.prof)
"""
import cProfile
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402


def run(L, dev, prof):
    from lightcompress_amd.deepseekv3 import DeepseekV3
    from lightcompress_amd.pipeline import build_algo
    config = bench.fp8_rtn_config(1)
    model = DeepseekV3(config, device=dev, dtype=torch.float8_e4m3fn,
                       hf_config=bench.dsv3_config(L, 32), random_init={'seed': 77, 'std': 0.02})
    algo = build_algo(model, config, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if prof is not None:
        prof.enable()
    algo.run_block_loop()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    algo.deploy('vllm_quant')
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if prof is not None:
        prof.disable()
    print(f'L {L}: block loop {(t1 - t0) / L * 1e3:.2f} ms/layer, deploy '
          f'{(t2 - t1) / L * 1e3:.2f} ms/layer, alloc {torch.cuda.memory_allocated() / 2**30:.1f}'
          f' GB reserved {torch.cuda.memory_reserved() / 2**30:.1f} GB', flush=True)
    algo.release()
    del algo, model
    bench.free_device()


def main():
    from lightcompress_amd import _native
    _native.load()
    dev = torch.device('cuda:0')
    run(1, dev, None)   # warm-up
    for L in map(int, sys.argv[1:]):
        prof = cProfile.Profile()
        run(L, dev, prof)
        out = ROOT / 'gpurun_out' / f'fp8_probe_{L}.prof'
        out.parent.mkdir(exist_ok=True)
        prof.dump_stats(str(out))
        st = pstats.Stats(prof)
        st.sort_stats('tottime').print_stats(25)
        st.sort_stats('cumulative').print_stats(30)


if __name__ == '__main__':
    main()
