"""Per-call shapes / strides / rate of the GEMMs in the Cholesky-inverse recursion (n=14336)."""
import collections
import torch
from lightcompress_amd import gptq_core

dev = 'cuda'
n = 14336
x = torch.randn(4 * n, n, device=dev) / n ** 0.5
H = x.T @ x + 0.01 * torch.eye(n, device=dev)
del x
log = []
orig = torch.Tensor.addmm_


def rec(self, a, b, *args, **kw):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); r = orig(self, a, b, *args, **kw); e1.record()
    log.append((tuple(a.shape), tuple(b.shape), a.stride(), b.stride(), self.stride(), e0, e1))
    return r


gptq_core.inverse_cholesky_upper(H.clone())
torch.Tensor.addmm_ = rec
gptq_core.inverse_cholesky_upper(H.clone())
torch.Tensor.addmm_ = orig
torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for a, b, sa, sb, so, e0, e1 in log:
    ms = e0.elapsed_time(e1)
    key = (a, b, sa, sb, so)
    agg[key][0] += 1; agg[key][1] += ms; agg[key][2] += 2 * a[0] * a[1] * b[1]
tot = sum(v[1] for v in agg.values())
print(f'{len(log)} addmm calls, {tot:.1f} ms')
for k, (c, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f'{ms:7.2f} ms x{c:3d} {fl / ms / 1e9:6.1f} TF/s  A{k[0]} s{k[2]}  B{k[1]} s{k[3]}  out s{k[4]}')
