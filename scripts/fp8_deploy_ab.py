"""A/B of the block-fp8 -> per-tensor fp8 deploy over 96 DSv3 expert linears (32 experts x
gate/up 2048x7168 + down 7168x2048): the one-launch streaming kernel (LCQ_FP8_DEPLOY=stream)
vs the two-pass pair (default), interleaved rounds, kernel time from HIP events around the launch.
Algorithmic traffic 2 B per element."""
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
cs, ss = [], []
for e in range(32):
    for (m, n) in ((2048, 7168), (2048, 7168), (7168, 2048)):
        w = (torch.randn(m, n, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        r = ops.fp8_quant_blocks(w, torch.float8_e4m3fn, 128, qmax=448.0, clamp_min=0.0,
                                 add_zero=False)
        cs.append(r['codes'])
        ss.append(r['scales'])
elems = sum(c.numel() for c in cs)
from lightcompress_amd import _native  # noqa: E402
ktime = {'stream': [], 'pair': []}
res = {'stream': [], 'pair': []}
outs = {}
for r in range(5):
    for v in res:
        os.environ['LCQ_FP8_DEPLOY'] = v
        ops.fp8_block_to_tensor_many(cs, ss, 128)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        timer = _native.KernelTimer()
        e0.record()
        with timer:
            for _ in range(5):
                o = ops.fp8_block_to_tensor_many(cs, ss, 128)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 5)
        ktime[v].append(sum(t['avg_ms'] for t in timer.summary().values()))
        outs[v] = o
same = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8))
           for a, b in zip(outs['stream'][0], outs['pair'][0])) and \
    torch.equal(outs['stream'][1], outs['pair'][1])
for v in res:
    ms = statistics.median(res[v])
    km = statistics.median(ktime[v])
    print(f'{v}: {ms:.3f} ms per call (incl. host plan + descriptor copy); launch (HIP events '
          f'around the C call) {km:.3f} ms = {2 * elems / km / 1e6:.0f} GB/s; identical: {same}',
          flush=True)
