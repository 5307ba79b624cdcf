"""Host cost of fresh pinned allocations (the streamed GPTQ write-back allocates a pinned fp32
host copy of every transformed weight): N fresh 224 MiB / 64 MiB tensors
kept alive, one large chunk, and the same sizes after a free (the caching host allocator).

usage: python scripts/pinned_alloc_probe.py
"""
import time

import torch

torch.cuda.init()
torch.empty(1, device='cuda')
keep = []
for shape, n in [((14336, 4096), 12), ((4096, 4096), 12)]:
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        keep.append(torch.empty(shape, dtype=torch.float32, pin_memory=True))
        ts.append((time.perf_counter() - t0) * 1e3)
    mb = shape[0] * shape[1] * 4 / 2 ** 20
    print(f'fresh pinned {shape} ({mb:.0f} MiB) x{n}: ' + ' '.join(f'{t:.1f}' for t in ts) +
          f' ms -> {mb * n / sum(ts) * 1e3 / 1024:.1f} GiB/s', flush=True)
t0 = time.perf_counter()
big = torch.empty(2 ** 30, dtype=torch.float32, pin_memory=True)
dt = time.perf_counter() - t0
print(f'one 4 GiB pinned chunk: {dt * 1e3:.1f} ms -> {4 / dt:.1f} GiB/s', flush=True)
t0 = time.perf_counter()
pg = torch.empty(2 ** 30, dtype=torch.float32)
pg.fill_(0)
dt = time.perf_counter() - t0
print(f'one 4 GiB pageable chunk + first touch: {dt * 1e3:.1f} ms', flush=True)
del keep
ts = []
for _ in range(12):
    t0 = time.perf_counter()
    x = torch.empty((14336, 4096), dtype=torch.float32, pin_memory=True)
    ts.append((time.perf_counter() - t0) * 1e3)
    del x
print('after free (cached) 224 MiB: ' + ' '.join(f'{t:.2f}' for t in ts) + ' ms', flush=True)
# D2H rate into pinned vs pageable
d = torch.empty((14336, 4096), dtype=torch.float32, device='cuda')
for name, h in [('pinned', torch.empty(d.shape, dtype=d.dtype, pin_memory=True)),
                ('pageable', torch.empty(d.shape, dtype=d.dtype))]:
    h.copy_(d)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 4
    print(f'D2H 224 MiB into {name}: {dt * 1e3:.1f} ms ({224 / 1024 / dt:.1f} GiB/s)', flush=True)
