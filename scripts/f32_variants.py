"""Probe: the recursion's fp32 GEMM (csrc/chol.hip, LDS-DMA k_gemm_f32d_*) built with other
ring depths / occupancies, timed side by side on the chain's shapes (no stream-K: plain tiled
grids). `build` (CPU, this container) compiles one library per variant under
scripts/_lib/; `run` (GPU) times every variant.
usage: f32_variants.py build | run"""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / 'scripts' / '_lib'
VARIANTS = {'ns3_occ1': (3, 1), 'ns2_occ2': (2, 2), 'ns2_occ1': (2, 1)}
SHAPES = [(7168, 1792, 1792, 1), (7168, 1792, 1792, 0), (1792, 7168, 1792, 0),
          (1792, 1792, 7168, 1), (7168, 3584, 3584, 1), (3584, 3584, 7168, 1),
          (3584, 1792, 1792, 0), (1792, 1792, 1792, 1), (4096, 4096, 4096, 0)]


def build():
    LIB.mkdir(parents=True, exist_ok=True)
    csrc = ROOT / 'lightcompress_amd' / 'csrc'
    for name, (ns, occ) in VARIANTS.items():
        out = LIB / f'libf32_{name}.so'
        cmd = ['/opt/rocm/bin/hipcc', '-O3', '-fPIC', '-std=c++17', '--offload-arch=gfx950',
               '-ffp-contract=off', f'-I{ROOT / "include"}', f'-I{csrc}', '-shared',
               f'-DLCQ_F32D_NS={ns}', f'-DLCQ_F32D_OCC={occ}',
               str(csrc / 'chol.hip'), str(csrc / 'lcq_common.hip'), '-o', str(out)]
        subprocess.run(cmd, check=True)
        print('built', out)


def run():
    import torch
    dev = torch.device('cuda:0')
    libs = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(str(LIB / f'libf32_{name}.so'))
        f = lib.lcq_gemm_f32
        f.argtypes = [ctypes.c_int64] * 3 + [ctypes.c_float, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_float, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p]
        f.restype = ctypes.c_int
        libs[name] = f
    stream = torch.cuda.current_stream(dev).cuda_stream
    for M, N, K, bt in SHAPES:
        A = torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev) if bt else torch.randn(K, N, device=dev)
        ref = None
        line = f'M{M} N{N} K{K} bt{bt}:'
        for name, f in libs.items():
            C = torch.empty(M, N, device=dev)

            def go():
                rc = f(M, N, K, 1.0, A.data_ptr(), K, B.data_ptr(), B.shape[1], bt, 0.0,
                       C.data_ptr(), N, stream)
                assert rc == 0, rc
            go()
            torch.cuda.synchronize()
            if ref is None:
                ref = C.clone()
            same = torch.equal(ref, C)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                go()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            line += f' | {name} {ms * 1e3:7.1f} us {2 * M * N * K / ms / 1e9:6.1f} TF/s' + \
                ('' if same else ' DIFF')
        print(line, flush=True)


if __name__ == '__main__':
    {'build': build, 'run': run}[sys.argv[1]]()
