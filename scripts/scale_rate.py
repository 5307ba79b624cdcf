"""Device rate of lcq_scale_bcast (x / s per column, AWQ's scaling_input) at the AWQ search
shapes: 128 x 512 tokens x 4096 / 14336 channels, bf16 (2 B read + 2 B write per element)."""
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(0)
for c in (4096, 14336):
    x = torch.randn(65536, c, generator=g, device=dev).to(torch.bfloat16)
    s = torch.exp(torch.randn(c, generator=g, device=dev)).to(torch.bfloat16)
    out = torch.empty_like(x)
    ops.scale_bcast(x, s, 'div', out=out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.scale_bcast(x, s, 'div', out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    h = int(out.view(torch.int16).to(torch.int64).mul(torch.arange(out.numel(), device=dev).view(out.shape) % 1009 + 1).sum())
    print(f'65536 x {c}: {ms:.3f} ms  {x.numel() * 4 / ms / 1e9:.2f} TB/s  checksum {h}', flush=True)
