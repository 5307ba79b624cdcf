"""Stage timing of the round-5 k_chol_inv_tile: loads scripts/_lib/libchol_prof2.so (chol.hip built
with -DLCQ_CHOL_PROF: lane 0 of wave 0 / 1 writes s_memtime stamps into the info buffer) and
prints per-panel cycles: S2 (+ its barrier), wave 0's diagonal update + S1 of the next panel,
wave 1's trailing jobs, and the clock (s_memtime over s_memrealtime at 100 MHz)."""
import ctypes
import os
import time

import torch

here = os.path.dirname(os.path.abspath(__file__))
import sys
lib = ctypes.CDLL(os.path.join(here, '_lib', sys.argv[1] if len(sys.argv) > 1 else 'libchol_prof2.so'))
f = lib.lcq_chol_inv_tile
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
              ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
n = 128
A0 = torch.randn(n, 2 * n, device='cuda')
H = A0 @ A0.t() / n + 0.1 * torch.eye(n, device='cuda')
X = torch.empty(n, n, device='cuda')
info = torch.zeros(64, dtype=torch.int64, device='cuda')
for rep in range(5):
    info.zero_()
    f(H.data_ptr(), n, n, None, 0, X.data_ptr(), n, info.data_ptr(), 0, None)
    torch.cuda.synchronize()
t = info.cpu().tolist()[1:]
t0 = t[0]
clk = (t[41] - t0) / ((t[43] - t[42]) / 100.0)   # cycles per us
print(f'clock {clk:.0f} MHz; total {t[41] - t0} cycles = {(t[43] - t[42]) / 100:.1f} us in-kernel')
print('load', t[1] - t0, ' S1(0)', t[2] - t[1])
for p in range(8):
    b = 3 + 4 * p
    st = t[30 + p]
    nxt = t[30 + p + 1] if p < 7 else t[40]
    row = f'panel {p}: total {nxt - st:5d}'
    if p < 7:
        row += (f'  w0: L+diag {t[b] - st:5d}  S1 {t[b + 2] - t[b]:5d}'
                f'  w1: S2 {t[52 + p] - st:5d}'
                f'  +meet {t[b + 1] - st:5d}  S3 {t[b + 3] - t[b + 1]:5d}')
    print(row)
print('X + L store', t[40 + 1] - t[40])
torch.cuda.synchronize()
t1 = time.perf_counter()
for _ in range(200):
    f(H.data_ptr(), n, n, None, 0, X.data_ptr(), n, info.data_ptr(), 0, None)
torch.cuda.synchronize()
print(f'{(time.perf_counter() - t1) / 200 * 1e6:.1f} us per tile (200 back-to-back, host wall)')
