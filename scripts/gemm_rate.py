"""Rate of the lcq projection GEMMs (csrc/gemm256.hip) at the AWQ loss-search shapes of
Llama-3-8B (128 x 512 calibration tokens) against torch's F.linear (hipBLASLt) and the
unfused chains they replace. Random data (cdna_hip_programming.md §5.4 rule 25), interleaved
rounds in one process (rule 24), median of rounds.

usage: python scripts/gemm_rate.py [--m 65536] [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from lightcompress_amd import ops  # noqa: E402


def timeit(fn, iters):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


_SET = set()


def setenv(v):
    for k in list(_SET):
        os.environ.pop(k, None)
    _SET.clear()
    if v != '-':
        for kv in v.split('+'):
            k, val = kv.split('=')
            os.environ[k] = val
            _SET.add(k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--m', type=int, default=65536)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--hidden', type=int, default=4096)
    ap.add_argument('--inter', type=int, default=14336)
    ap.add_argument('--kv', type=int, default=1024)
    ap.add_argument('--variants', default='-',
                    help="comma list of env settings to A/B, e.g. '-,LCQ_GEMM_KERNEL=b' "
                         "('-' = defaults)")
    args = ap.parse_args()
    orders = args.variants.split(',')
    dev = 'cuda'
    M, H, I, KV = args.m, args.hidden, args.inter, args.kv
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16

    def rnd(*s, sc=1.0):
        return (torch.randn(*s, generator=g, device=dev) * sc).to(bf)

    x = rnd(M, H)
    xi = rnd(M, I, sc=0.1)
    wq, wk, wv, wo = rnd(H, H, sc=0.02), rnd(KV, H, sc=0.02), rnd(KV, H, sc=0.02), rnd(H, H, sc=0.02)
    wg, wu, wd = rnd(I, H, sc=0.02), rnd(I, H, sc=0.02), rnd(H, I, sc=0.02)
    org = rnd(M, H)
    lb = ops.LossBuffer(1, dev)

    cases = {
        'qkv  (K %d, N %d+%d+%d)' % (H, H, KV, KV): (
            2.0 * M * H * (H + 2 * KV),
            lambda: ops.linear_multi(x, [wq, wk, wv]),
            lambda: (F.linear(x, wq), F.linear(x, wk), F.linear(x, wv))),
        'o    (K %d, N %d)' % (H, H): (
            2.0 * M * H * H, lambda: ops.linear(x, wo), lambda: F.linear(x, wo)),
        'gate/up+silu (K %d, N 2x%d)' % (H, I): (
            4.0 * M * H * I, lambda: ops.linear_silu_mul(x, wg, wu),
            lambda: ops.silu_mul(F.linear(x, wg), F.linear(x, wu))),
        'down (K %d, N %d)' % (I, H): (
            2.0 * M * I * H, lambda: ops.linear(xi, wd), lambda: F.linear(xi, wd)),
        'down+loss (K %d, N %d)' % (I, H): (
            2.0 * M * I * H, lambda: ops.linear_sq_diff(xi, wd, org, lb, 0),
            lambda: lb.record(org, F.linear(xi, wd), 0)),
    }
    res = {k: ({o: [] for o in orders}, []) for k in cases}
    for name, (fl, f_lcq, f_ref) in cases.items():  # warm up (kernels, allocator)
        for o in orders:
            setenv(o)
            f_lcq()
        f_ref()
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for name, (fl, f_lcq, f_ref) in cases.items():
            for o in orders:
                setenv(o)
                res[name][0][o].append(timeit(f_lcq, args.iters))
            res[name][1].append(timeit(f_ref, args.iters))
    print(f'M = {M} tokens, median of {args.rounds} rounds x {args.iters} calls (ms, TFLOP/s)')
    for name, (fl, _, _) in cases.items():
        b = statistics.median(res[name][1])
        for o in orders:
            a = statistics.median(res[name][0][o])
            print(f'{name:30s} lcq[{o}] {a:8.3f} ms {fl / a / 1e9:7.1f} TF/s | torch '
                  f'{b:8.3f} ms {fl / b / 1e9:7.1f} TF/s | lcq/torch time {a / b:5.3f}')


if __name__ == '__main__':
    main()
