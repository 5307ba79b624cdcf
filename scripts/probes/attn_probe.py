"""Time SDPA for the AWQ calibration attention shape under the ROCm FA libraries."""
import torch
import torch.nn.functional as F

dev = 'cuda'
B, H, KV, S, D = 128, 32, 8, 512, 128
q = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16)
k = torch.randn(B, KV, S, D, device=dev, dtype=torch.bfloat16)
v = torch.randn(B, KV, S, D, device=dev, dtype=torch.bfloat16)
kr = k.repeat_interleave(H // KV, 1)
vr = v.repeat_interleave(H // KV, 1)
fl = 4 * B * H * S * S * D / 2


def t(fn, n=10):
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


print('fa libs:', getattr(torch.backends.cuda, 'preferred_rocm_fa_library', None))
ref = F.scaled_dot_product_attention(q, kr, vr, is_causal=True)
for lib in ('aotriton', 'ck'):
    try:
        torch.backends.cuda.preferred_rocm_fa_library(lib)
    except Exception as e:
        print(lib, 'unavailable:', e)
        continue
    for name, fn in (('repeat_kv', lambda: F.scaled_dot_product_attention(q, kr, vr, is_causal=True)),
                     ('enable_gqa', lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True))):
        try:
            ms = t(fn)
            out = fn()
            d = (out.float() - ref.float()).abs().max().item()
            print(f'{lib:9s} {name:10s} {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s  max|d| vs aotriton {d:.2e}', flush=True)
        except Exception as e:
            print(lib, name, 'failed:', str(e)[:200])
