"""lcq_attn_fwd_causal vs torch SDPA (aotriton) at the AWQ / GPTQ calibration shapes."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from lightcompress_amd import ops  # noqa: E402


def timed(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


shapes = [(128, 32, 8, 512), (128, 32, 8, 2048)]
if len(sys.argv) > 1:  # e.g. `512`: only that sequence length (counter passes)
    shapes = [c for c in shapes if c[3] == int(sys.argv[1])]
for (B, H, KVH, S) in shapes:
    D = 128
    qs = torch.randn(B, S, H, D, device='cuda').to(torch.bfloat16)
    ks = torch.randn(B, S, KVH, D, device='cuda').to(torch.bfloat16)
    vs = torch.randn(B, S, KVH, D, device='cuda').to(torch.bfloat16)
    q, k, v = qs.transpose(1, 2), ks.transpose(1, 2), vs.transpose(1, 2)
    fl = 2.0 * B * H * S * (S + 1) * D
    ms = timed(lambda: ops.attn_fwd_causal(q, k, v, D ** -0.5))
    mt = timed(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True))
    print(f'B{B} H{H} KV{KVH} S{S}: lcq {ms:.3f} ms {fl / ms / 1e9:.0f} TF/s | '
          f'torch {mt:.3f} ms {fl / mt / 1e9:.0f} TF/s', flush=True)
    del qs, ks, vs
