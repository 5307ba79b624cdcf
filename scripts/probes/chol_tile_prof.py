"""Stage timing of k_chol_inv_tile: builds a -DLCQ_CHOL_PROF copy of the library (probe only)
whose thread 0 writes s_memtime stamps into the info buffer, and prints per-stage cycles."""
import ctypes
import os
import subprocess
import torch

here = os.path.dirname(os.path.abspath(__file__))
root = os.path.dirname(os.path.dirname(here))
pw = int(os.environ.get('PW', '16'))
nt = int(os.environ.get('NT', '256'))
so = os.path.join(here, f'libchol_prof{pw}_{nt}.so')
if not os.path.exists(so):
    csrc = os.path.join(root, 'lightcompress_amd', 'csrc')
    subprocess.check_call(['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-shared', '-fPIC',
                           '-DLCQ_CHOL_PROF', f'-DLCQ_CHOL_PW={pw}', f'-DLCQ_CHOL_NT={nt}', '-I', csrc, '-I', os.path.join(root, 'include'),
                           os.path.join(csrc, 'chol.hip'), os.path.join(csrc, 'lcq_common.hip'),
                           '-o', so])
lib = ctypes.CDLL(so)
f = lib.lcq_chol_inv_tile
f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
              ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
dev = 'cuda'
n = 128
A0 = torch.randn(n, 2 * n, device=dev)
H = A0 @ A0.t() / n + 0.1 * torch.eye(n, device=dev)
X = torch.empty(n, n, device=dev)
for rep in range(3):
    A = H.clone()
    info = torch.zeros(80, dtype=torch.int64, device=dev)
    f(A.data_ptr(), n, n, None, 0, X.data_ptr(), n, info.data_ptr(), 0, None)
    torch.cuda.synchronize()
ts = info.cpu().tolist()[1:73]
t0 = ts[0]
print('PW', pw, 'load', ts[1] - t0)
for p in range(128 // pw):
    b = 2 + 4 * p
    print(f'panel {p}: S1 {ts[b] - (ts[b - 1] if p else ts[1])}  bar+S2 {ts[b + 1] - ts[b]}  '
          f'bar {ts[b + 2] - ts[b + 1]}  S3 {ts[b + 3] - ts[b + 2]}')
print('store', ts[71] - ts[70], 'total', ts[71] - t0, 'cycles (s_memtime)')
import time
for rep in range(3):
    torch.cuda.synchronize(); t1 = time.perf_counter()
    for _ in range(100):
        f(A.data_ptr(), n, n, None, 0, X.data_ptr(), n, info.data_ptr(), 0, None)
    torch.cuda.synchronize()
print(f'PW {pw} NT {nt}: {(time.perf_counter() - t1) * 1e4:.1f} us per tile (100 back-to-back)')
