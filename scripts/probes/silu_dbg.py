import os, sys, torch
sys.path.insert(0, '/root/repo')
from lightcompress_amd import ops
dev='cuda'
g = torch.Generator(device=dev).manual_seed(1)
def ex(shape): return (torch.randint(-3, 4, shape, generator=g, device=dev).float() / 8).to(torch.bfloat16)
M, I, K = 512, 1024, 256
x, wg, wu = ex((M, K)), ex((I, K)), ex((I, K))
h = ops.linear_silu_mul(x, wg, wu)
gate = (x.float() @ wg.float().T).to(torch.bfloat16); up = (x.float() @ wu.float().T).to(torch.bfloat16)
ref = ops.silu_mul(gate, up)
bad = (h.view(torch.int16) != ref.view(torch.int16))
print(os.environ.get('LCQ_GEMM_KERNEL'), 'bad', bad.sum().item(), 'of', bad.numel())
if bad.any():
    r = bad.any(1).nonzero().flatten(); c = bad.any(0).nonzero().flatten()
    print('rows', r.min().item(), r.max().item(), len(r), 'cols', c.min().item(), c.max().item(), len(c))
    print('bad per 128-col block', [int(bad[:, i*128:(i+1)*128].sum()) for i in range(I//128)])
    print('bad per 64-row block', [int(bad[i*64:(i+1)*64].sum()) for i in range(M//64)])
    # is h equal to silu(gate)*gate or up*up etc?
    for nm, a_, b_ in (('gate,gate', gate, gate), ('up,up', up, up), ('up,gate', up, gate)):
        alt = ops.silu_mul(a_, b_)
        print(nm, (alt.view(torch.int16) == h.view(torch.int16)).float().mean().item())
