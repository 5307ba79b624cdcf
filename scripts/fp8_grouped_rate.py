"""Probe: lcq_fp8_gemm_grouped per projection at the bench's MoE calibration shape (16 DSv3
experts, 4096 tokens routed top-8: ~2048 rows per expert, gate / up 2048 x 7168, down
7168 x 2048): gate + up as two weight sets, gate + up in the SiLU pair mode, down; and the
single-problem lcq_fp8_gemm on one expert's rows for reference. TF/s from HIP events.
usage: fp8_grouped_rate.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from lightcompress_amd import ops  # noqa: E402
from lightcompress_amd.kernel import act_quant, weight_cast_to_fp8  # noqa: E402

dev = torch.device('cuda:0')
E, k, T, H, I = 16, 8, 4096, 7168, 2048
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
idx = torch.argsort(torch.rand(T, E, device=dev, generator=g), dim=1)[:, :k]
flat = idx.reshape(-1)
order = torch.argsort(flat, stable=True)
row_off = torch.zeros(E + 1, dtype=torch.int64, device=dev)
torch.cumsum(torch.bincount(flat, minlength=E), 0, out=row_off[1:])
rows = order // k
R = rows.numel()


def wts(n, kk):
    return [weight_cast_to_fp8((torch.randn(n, kk, device=dev, generator=g) * 0.02)
                               .to(torch.bfloat16).contiguous()) for _ in range(E)]


gate, up, down = wts(I, H), wts(I, H), wts(H, I)
gu_tab = torch.stack([ops.fp8_weight_table(gate, dev), ops.fp8_weight_table(up, dev)])
d_tab = ops.fp8_weight_table(down, dev)
xq, xs = act_quant(x.contiguous(), 128)
h = (torch.randn(R, I, device=dev, generator=g) * 0.1).to(torch.bfloat16)
hq, hs = act_quant(h, 128)


def timeit(fn, flops, name, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f'{name:40s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TF/s', flush=True)


timeit(lambda: ops.fp8_gemm_grouped(xq, xs.reshape(-1), row_off, gu_tab, I, torch.bfloat16,
                                    a_rows=rows), 2 * 2.0 * R * I * H, 'gate+up two sets')
timeit(lambda: ops.fp8_gemm_grouped(xq, xs.reshape(-1), row_off, gu_tab, I, torch.bfloat16,
                                    a_rows=rows, silu_mul=True), 2 * 2.0 * R * I * H,
       'gate+up pair mode (silu * up)')
timeit(lambda: ops.fp8_gemm_grouped(hq, hs.reshape(-1), row_off, d_tab, H, torch.bfloat16),
       2.0 * R * I * H, 'down')
m0 = int(row_off[1])
xa, sa = xq[rows[:m0]].contiguous(), xs[rows[:m0]].contiguous()
timeit(lambda: ops.fp8_gemm(xa, sa, gate[0][0], gate[0][1], out_dtype=torch.bfloat16),
       2.0 * m0 * I * H, f'single gate expert ({m0} rows)')
ha, hsa = hq[:m0].contiguous(), hs[:m0].contiguous()
timeit(lambda: ops.fp8_gemm(ha, hsa, down[0][0], down[0][1], out_dtype=torch.bfloat16),
       2.0 * m0 * I * H, f'single down expert ({m0} rows)')
