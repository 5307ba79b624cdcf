"""Sweep lcq_fp8_block_to_tensor_many's group size / pass-1 unroll (env knobs) on DSv3
expert linears; prints ms per 96-linear batch and GB/s at 2 B/element."""
import os
import sys
import torch
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
cs, ss = [], []
for e in range(int(os.environ.get('E', '32'))):
    for (m, n) in [(2048, 7168), (2048, 7168), (7168, 2048)]:
        w = (torch.randn(m, n, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        r = ops.fp8_quant_blocks(w, torch.float8_e4m3fn, 128, qmax=448.0, clamp_min=0.0, add_zero=False)
        cs.append(r['codes']); ss.append(r['scales'])
elems = sum(c.numel() for c in cs)
ref = None
for gm in os.environ.get('SWEEP_GROUPS', '16,32,48,64,96,128,192').split(','):
    for bu in ['2', '4']:
        os.environ['LCQ_FP8_GROUP_MIB'] = gm
        os.environ['LCQ_FP8_BMAX_UNROLL'] = bu
        for _ in range(2):
            o, s = ops.fp8_block_to_tensor_many(cs, ss, 128)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            o, s = ops.fp8_block_to_tensor_many(cs, ss, 128)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 10
        if ref is None:
            ref = (o, s)
        ok = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8)) for x, y in zip(o, ref[0]))
        print(f'group {gm:>4} MiB unroll {bu}: {ms:.3f} ms  {2 * elems / ms / 1e6:.0f} GB/s  same={ok}', flush=True)
