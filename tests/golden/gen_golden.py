"""Generate golden fixtures by running the REAL reference (``/root/reference``) on CPU.

Run in the build container only:  ``python tests/golden/gen_golden.py [quant|gptq|awq|clip|fp8|all]``
Inputs are seeded and stored with the outputs, so the fixtures do not depend on the RNG.
The reference ships no golden vectors of its own; these pin the oracle and
the HIP kernels.
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import _ref_import as R  # noqa: E402
import fixtures as F  # noqa: E402


def weights(rows, cols, dtype, seed, edge=True):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(rows, cols, generator=g) * 0.02
    if edge and rows >= 8:
        gs = min(cols, 128)
        w[0, :gs] = 0.0                                   # all-zero group -> clamp(1e-5)
        w[1, :gs] = 0.0123                                # constant group
        w[2, :gs] = torch.randn(gs, generator=g) * 1e-7   # below the 1e-5 floor
        base = 2.0 ** -6                                  # exact ties at .5 (asym, 4 bit)
        ties = torch.arange(gs, dtype=torch.float32) % 15 + 0.5
        w[3, :gs] = ties * base
        w[3, 0], w[3, 1] = 0.0, 15 * base
        w[4, :gs] = (torch.arange(gs) % 7 - 3 + 0.5) * base   # sym ties
        w[4, 0] = 7 * base
        w[5, 7] = 1.0                                     # outliers
        w[5, 9] = -0.75
        w[6, :gs] = -w[6, :gs].abs() - 0.01              # negative-only group
    return w.to(dtype)


def gen_quant():
    q = R.quant_module()
    mu = R.module_utils()
    cases = [
        # name, bit, sym, granularity, group, dtype, rows, cols
        ('int4_asym_g128_bf16', 4, False, 'per_group', 128, torch.bfloat16, 32, 512),
        ('int4_sym_g128_bf16', 4, True, 'per_group', 128, torch.bfloat16, 32, 512),
        ('int8_sym_pc_bf16', 8, True, 'per_channel', None, torch.bfloat16, 24, 768),
        ('int8_asym_pc_f16', 8, False, 'per_channel', None, torch.float16, 16, 768),
        ('int4_asym_g64_f32', 4, False, 'per_group', 64, torch.float32, 16, 256),
        ('int4_sym_g32_bf16', 4, True, 'per_group', 32, torch.bfloat16, 16, 256),
        ('int3_asym_g128_bf16', 3, False, 'per_group', 128, torch.bfloat16, 16, 256),
        ('int8_asym_g128_bf16', 8, False, 'per_group', 128, torch.bfloat16, 16, 256),
    ]
    for i, (name, bit, sym, gran, gs, dt, rows, cols) in enumerate(cases):
        kw = {'group_size': gs} if gs else {}
        wq = q.IntegerQuantizer(bit, sym, gran, **kw)
        w = weights(rows, cols, dt, 100 + i)
        fq = wq.fake_quant_weight_dynamic(w.clone())
        codes, s, z = wq.real_quant_weight_dynamic(w.clone())
        out = dict(w=w, fq=fq, codes=codes, scales=s, zeros=z,
                   meta=torch.tensor([bit, int(sym), gs or cols, int(wq.qmin), int(wq.qmax)]))
        if bit in (4, 8):
            packed, s16 = mu.VllmRealQuantLinear.pack(codes.clone(), s.clone(),
                                                      {'weight': {'bit': bit}})
            out.update(packed=packed, scales_fp16=s16)
        F.save(f'quant_{name}', **out)

    # AWQ: w.mul_(s) then fake_quant_weight_dynamic, in the weight dtype (awq.py:147-164)
    wq = q.IntegerQuantizer(4, True, 'per_group', group_size=128)
    w = weights(48, 512, torch.bfloat16, 7)
    g = torch.Generator().manual_seed(8)
    s = torch.exp(torch.randn(512, generator=g) * 0.7).to(torch.bfloat16)
    ws = w.clone().mul_(s.view(1, -1))
    F.save('quant_awq_prescale_int4_sym_g128_bf16', w=w, pre=s,
           fq=wq.fake_quant_weight_dynamic(ws))

    # auto-clip v1 apply (auto_clip.py:193-212) followed by the deploy fake quant
    for sym in (True, False):
        wq = q.IntegerQuantizer(4, sym, 'per_group', group_size=128)
        w = weights(32, 512, torch.bfloat16, 9 + sym)
        wg = w.reshape(32, 4, 128)
        mx = (wg.amax(-1, keepdim=True) * 0.7).to(torch.bfloat16)
        mn = (wg.amin(-1, keepdim=True) * 0.8).to(torch.bfloat16)
        if sym:
            mx = (wg.abs().amax(-1, keepdim=True) * 0.75).to(torch.bfloat16)
            mn = -mx
        clipped = torch.clamp(wg, mn, mx).reshape(32, 512)
        F.save(f'quant_clip_int4_{"sym" if sym else "asym"}_g128_bf16', w=w, cmax=mx,
               cmin=mn, fq=wq.fake_quant_weight_dynamic(clipped))

    # static (GPTQ deploy): fp32 weights + fp32 qparams (gptq.py:424-452), and real quant
    # with scales cast to the model dtype first (gptq.py:411-422)
    wq = q.IntegerQuantizer(4, False, 'per_group', group_size=128)
    w32 = weights(32, 512, torch.float32, 11)
    _, s32, z32, qmax, qmin = wq.get_tensor_qparams(w32 * 0.9)
    fq = wq.fake_quant_weight_static(w32, {'scales': s32, 'zeros': z32, 'qmax': qmax,
                                           'qmin': qmin}).to(torch.bfloat16)
    codes, s_rq, z_rq = wq.real_quant_weight_static(
        w32, {'scales': s32.to(torch.bfloat16), 'zeros': z32, 'qmax': qmax, 'qmin': qmin})
    F.save('quant_static_int4_asym_g128_f32', w=w32, scales=s32, zeros=z32, fq_bf16=fq,
           codes=codes, scales_rq=s_rq, zeros_rq=z_rq)

    # AutoAWQ gemm_pack incl. its unclamped fp32 re-quantisation
    for bit_sym, (oc, ic, seed) in {'asym': (256, 512, 12), 'asym_big': (512, 1024, 13)}.items():
        wq = q.IntegerQuantizer(4, False, 'per_group', group_size=128)
        w = weights(oc, ic, torch.bfloat16, seed)
        _, s, z = wq.real_quant_weight_dynamic(w.clone())
        module = types.SimpleNamespace(in_features=ic)
        qcfg = {'weight': {'bit': 4, 'group_size': 128}}
        qw, s16, qz = mu.AutoawqRealQuantLinear.gemm_pack(module, w.clone(), s.clone(),
                                                         z.clone(), qcfg)
        F.save(f'awqpack_int4_{bit_sym}_g128_bf16', w=w, scales=s, zeros=z, qweight=qw,
               scales_t=s16, qzeros=qz)
    print('quant fixtures written')


GENERATORS = {'quant': gen_quant}


if __name__ == '__main__':
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    R.install()
    for k, fn in GENERATORS.items():
        if which in ('all', k):
            fn()
