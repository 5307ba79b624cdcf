"""Probe: the grouped GPTQ Hessian (one lcq_hessian_grouped launch over 8 sample groups) against
the round-3 form (one lcq_hessian_accum per group + lcq_tree_sum), at the Llama-3-8B GPTQ
calibration size (128 x 2048 tokens), IC 4096 and 14336. A probe library
(scripts/probe_build.py LCQ_PROBE_SYRK_GNS=<n>, loaded via LCQ_LIB_PATH) forces the per-group
split count of the grouped plan."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
n = 128 * 2048
for ic in (4096, 14336):
    g = torch.Generator(device=dev).manual_seed(ic)
    x = torch.randn(n, ic, generator=g, device=dev).to(torch.bfloat16)
    per = n // 8
    bounds = [i * per for i in range(9)]
    H = torch.empty(ic, ic, device=dev)
    fl = n * ic * (ic + 1)

    def grouped():
        ops.hessian_grouped(x, bounds, H, 2.0 / 128)

    parts = [torch.empty(ic, ic, device=dev) for _ in range(8)]

    def old():
        for k in range(8):
            ops.hessian_accum(x[k * per:(k + 1) * per], parts[k], 1.0, 0.0)
        ops.tree_sum(parts, 2.0 / 128, out=H)

    for name, fn in (('grouped', grouped), ('per-group+tree', old)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f'ic {ic:6d} {name:15s}: {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TF/s', flush=True)
    del x, parts, H
    torch.cuda.empty_cache()
