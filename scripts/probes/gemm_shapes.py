"""hipBLASLt bf16 GEMM time for the AWQ search shapes: separate gate/up vs one concatenated."""
import torch
import torch.nn.functional as F

x = torch.randn(65536, 4096, device='cuda').to(torch.bfloat16)
wg = torch.randn(14336, 4096, device='cuda').to(torch.bfloat16) * 0.02
wu = torch.randn(14336, 4096, device='cuda').to(torch.bfloat16) * 0.02
wc = torch.cat([wg, wu], 0)
wq = torch.randn(6144, 4096, device='cuda').to(torch.bfloat16) * 0.02


def t(fn, n=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


sep = t(lambda: (F.linear(x, wg), F.linear(x, wu)))
cat = t(lambda: F.linear(x, wc))
qkv = t(lambda: F.linear(x, wq))
fl = 2 * 65536 * 4096 * 28672
print(f'gate+up separate {sep:.3f} ms ({fl / sep / 1e9:.0f} TF)  concatenated {cat:.3f} ms '
      f'({fl / cat / 1e9:.0f} TF)  qkv-concat {qkv:.3f} ms')
