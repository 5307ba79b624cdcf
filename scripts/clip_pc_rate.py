"""Per-channel auto-clip (lcq_auto_clip_search_pc, w8a8 AWQ) at Llama-3-8B linear shapes:
time per launch and products/s (11 candidates x T x oc x ic DT-rounded products)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

T = 512
for oc, ic in ((4096, 4096), (14336, 4096), (4096, 14336), (1024, 4096)):
    w = (torch.randn(oc, ic, device='cuda') * 0.02).to(torch.bfloat16)
    x = (torch.randn(T, ic, device='cuda') * torch.exp(torch.randn(ic, device='cuda'))).to(
        torch.bfloat16)
    qx = x.clone()
    for _ in range(2):
        ops.auto_clip_search(w, x, ic, 10, 20, -128, 127, True, True, qx=qx)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        ops.auto_clip_search(w, x, ic, 10, 20, -128, 127, True, True, qx=qx)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f'{oc}x{ic}: {ms:.2f} ms  {11 * T * oc * ic / ms / 1e9:.1f} T products/s', flush=True)
