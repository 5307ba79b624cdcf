"""A/B of the GPTQ bench leg (bench.bench_gptq: Llama-3-8B blocks, 128 x 2048 tokens) under
host-side switches of gptq_core, alternating variants in one process.

usage: python scripts/gptq_ab.py [rounds]
  variants: graph = the chain captured and replayed as a HIP graph (product default),
            eager = the recursion launched eagerly (side-stream overlap kept)
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from lightcompress_amd import gptq_core  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
sys.argv = [sys.argv[0]]
args = bench.parse()
dev = torch.device('cuda:0')
for r in range(rounds):
    for name, graphs in (('graph', True), ('eager', False)):
        gptq_core.CHAIN_GRAPHS = graphs
        out = bench.bench_gptq(args, 0, 1, dev)
        k = out['lcq_kernels']
        chain = k.get('lcq_chol_chain_graph', {}).get('avg_ms')
        print(f'round {r} {name}: {out["ms_per_block"]} ms/block, chain graph avg {chain}, '
              f'hessian {k["lcq_hessian_grouped"]["avg_ms"]:.2f} ms', flush=True)
