import ctypes, subprocess, sys
from pathlib import Path
import torch
here = Path(__file__).resolve().parent
so = here / 'probe_tr.so'
lib = ctypes.CDLL(str(so))
dev = torch.device('cuda:0')
out = torch.zeros(64 * 4, dtype=torch.int32, device=dev)
torch.cuda.synchronize()
print('tr rc', lib.probe_tr(ctypes.c_void_p(out.data_ptr())))
o = out.cpu().view(64, 4)
for lane in [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 63]:
    print('lane', lane, o[lane].tolist())
A = (torch.arange(16)[:, None] + 100 * torch.arange(32)[None, :]).float() % 7 - 3
B = (torch.arange(32)[:, None] * 3 + torch.arange(16)[None, :] * 5).float() % 11 - 5
C = torch.zeros(16, 16)
Ad, Bd, Cd = A.to(dev).contiguous(), B.to(dev).contiguous(), C.to(dev)
print('mfma rc', lib.probe_mfma(ctypes.c_void_p(Ad.data_ptr()), ctypes.c_void_p(Bd.data_ptr()), ctypes.c_void_p(Cd.data_ptr())))
ref = A @ B
print('mfma max err', (Cd.cpu() - ref).abs().max().item())
