"""Device timing of the auto-clip search kernel on Llama-3-8B shapes (dev aid)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from lightcompress_amd import ops
dev = torch.device('cuda:0')
for oc, ic in [(4096, 4096), (14336, 4096), (4096, 14336), (1024, 4096)]:
    w = (torch.randn(oc, ic, device=dev) * 0.02).to(torch.bfloat16)
    x = (torch.randn(512, ic, device=dev) * torch.exp(torch.randn(ic, device=dev))).to(torch.bfloat16)
    ops.auto_clip_search(w, x, 128, 10, 20, -8, 7, True, True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        ops.auto_clip_search(w, x, 128, 10, 20, -8, 7, True, True)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    prods = oc * ic * 512 * 11
    print(f'{oc}x{ic}: {ms:.2f} ms  {prods/ms/1e9:.1f} Gprod/s')
