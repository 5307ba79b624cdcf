"""Summarise a rocprofv3 --kernel-trace --memory-copy-trace run: total H2D / D2H copy time and
the part of it during which a kernel was executing (copy/compute overlap of the streamed block
residency)."""
import csv
import sys
from pathlib import Path


def rows(p):
    with open(p) as f:
        return list(csv.DictReader(f))


root = Path(sys.argv[1])
kt = next(root.rglob('*kernel_trace.csv'))
mc = next(root.rglob('*memory_copy_trace.csv'))
kern = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows(kt))
merged = []
for s, e in kern:   # union of kernel busy intervals
    if merged and s <= merged[-1][1]:
        merged[-1][1] = max(merged[-1][1], e)
    else:
        merged.append([s, e])


def covered(s, e):
    tot = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


out = {}
for r in rows(mc):
    d = r.get('Direction', r.get('Operation', '?'))
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    nb = int(r.get('Bytes', r.get('Size', 0)) or 0)
    o = out.setdefault(d, [0, 0, 0, 0])
    o[0] += 1
    o[1] += e - s
    o[2] += covered(s, e)
    o[3] += nb
span = merged[-1][1] - merged[0][0] if merged else 0
busy = sum(b - a for a, b in merged)
print(f'kernel span {span / 1e6:.1f} ms, kernels busy {busy / 1e6:.1f} ms')
for d, (n, t, c, nb) in out.items():
    print(f'{d}: {n} copies, {nb / 2**30:.2f} GiB, {t / 1e6:.2f} ms copying, '
          f'{c / 1e6:.2f} ms of it ({100 * c / max(t, 1):.1f} %) under running kernels')
