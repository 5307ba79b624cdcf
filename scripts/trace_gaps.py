"""Idle gaps of the GPU in a rocprofv3 kernel trace (run_kernel_trace.csv): kernels sorted by
start, gap = start - (latest end so far); the largest gaps and the gap total per (previous
kernel -> next kernel) pair, over a time window [t0, t1] in ms from the first kernel.

usage: python scripts/trace_gaps.py <run_kernel_trace.csv> [t0_ms] [t1_ms]
"""
import csv
import sys
from collections import defaultdict


def short(n):
    n = n.split('(')[0]
    for p in ('void ', 'lcq::', 'at::native::'):
        n = n.replace(p, '')
    return n[:48]


rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name']))
            for r in rows)
base = ev[0][0]
t0 = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 0
t1 = float(sys.argv[3]) * 1e6 if len(sys.argv) > 3 else float('inf')
ev = [e for e in ev if t0 <= e[0] - base <= t1]
busy_end, prev = ev[0][1], ev[0][2]
tot = defaultdict(lambda: [0, 0.0])
busy = 0.0
gaps = []
for s, e, n in ev[1:]:
    if s > busy_end:
        g = (s - busy_end) / 1e3
        tot[(prev, n)][0] += 1
        tot[(prev, n)][1] += g
        gaps.append((g, prev, n, (s - base) / 1e6))
    if e > busy_end:
        busy += (e - max(s, busy_end)) / 1e3
        busy_end, prev = e, n
span = (busy_end - ev[0][0]) / 1e3
print(f'window {span / 1e3:.2f} ms: busy {busy / 1e3:.2f} ms, idle {(span - busy) / 1e3:.2f} ms, '
      f'{len(ev)} kernels')
print('largest gaps (us, prev -> next, at ms):')
for g, p, n, at in sorted(gaps, reverse=True)[:15]:
    print(f'  {g:9.1f}  {p} -> {n}  @{at:.1f}')
print('gap totals by pair (us):')
for (p, n), (c, g) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f'  {g:9.1f} x{c:<5d} {p} -> {n}')
