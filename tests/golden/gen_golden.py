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


def _acts(n_samples, seq, ic, seed, dtype=torch.bfloat16):
    """Calibration activations with log-normal per-channel magnitudes (outlier channels)."""
    g = torch.Generator().manual_seed(seed)
    mag = torch.exp(torch.randn(ic, generator=g))
    return [(torch.randn(1, seq, ic, generator=g) * mag).to(dtype) for _ in range(n_samples)]


def gen_gptq():
    """Drive the reference GPTQ layer methods (gptq.py) on one linear: Hessian via add_batch,
    qparams via collect_block_qparams' quantizer call, layer_transform, w_qdq / w_q deploy."""
    import torch.nn as nn
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.gptq as gm
    cases = [
        # name, oc, ic, bit, sym, group, actorder, dead_cols
        ('int4_asym_g128_act', 192, 512, 4, False, 128, True, False),
        ('int4_sym_g128_noact', 128, 384, 4, True, 128, False, False),
        ('int4_asym_g64_act_dead', 128, 256, 4, False, 64, True, True),
        ('int8_sym_g128_act', 64, 256, 8, True, 128, True, False),
    ]
    for i, (name, oc, ic, bit, sym, gs, act, dead) in enumerate(cases):
        torch.manual_seed(1000 + i)
        layer = nn.Linear(ic, oc, bias=False)
        layer.weight.data = weights(oc, ic, torch.bfloat16, 200 + i, edge=False)
        xs = _acts(3, 48, ic, 300 + i)
        if dead:
            for x in xs:
                x[..., 5] = 0
                x[..., 77] = 0
        obj = gm.GPTQ.__new__(gm.GPTQ)
        obj.wquantizer = q.IntegerQuantizer(bit, sym, 'per_group', group_size=gs)
        obj.dev = torch.device('cpu')
        obj.model_dtype = torch.bfloat16
        obj.owq, obj.actorder, obj.static_groups = False, act, False
        obj.percdamp, obj.blocksize, obj.chunk_num = 0.01, 128, 1
        obj.true_sequential = True
        obj.need_perm = act
        obj.layers_cache = {'l': {}}
        obj.qparams = {}
        gm.GPTQ.layer_init(obj, layer, 'l')
        for x in xs:
            gm.GPTQ.add_batch(obj, layer, 'l', x, None)
        H = obj.layers_cache['l']['H'].clone()
        # collect_block_qparams (base_blockwise_quantization.py:337-365)
        _, s0, z0, qmax, qmin = obj.wquantizer.get_tensor_qparams(layer.weight.data)
        layer.register_buffer('buf_scales', s0)
        layer.register_buffer('buf_zeros', z0)
        layer.register_buffer('buf_qmax', torch.tensor(qmax))
        layer.register_buffer('buf_qmin', torch.tensor(qmin))
        w_in = layer.weight.data.clone()
        # capture U through process_hessian_and_weights on a copy of the state
        obj.layers_cache['l']['H'] = H.clone()
        obj.initialize_qparams_and_prepare_weights(layer, 'l')
        Wp, U = obj.process_hessian_and_weights(layer, 'l')
        # fresh transform for the outputs
        obj.layers_cache['l']['H'] = H.clone()
        obj.qparams = {}
        layer.weight.data = w_in.clone()
        obj.layer_transform(layer, 'l')
        out = dict(x=torch.cat(xs, 0), w=w_in, H=H, U=U,
                   perm=getattr(layer, 'buf_perm', None), weight=layer.weight.data.clone(),
                   scales=layer.buf_scales, zeros=None if sym else layer.buf_zeros,
                   meta=torch.tensor([bit, int(sym), gs, int(act), oc, ic]))
        out['fq'] = obj.w_qdq(layer, obj.wquantizer)
        if not act:
            codes, s_rq, z_rq = obj.w_q(layer, obj.wquantizer)
            out.update(codes=codes, scales_rq=s_rq, zeros_rq=z_rq)
        F.save(f'gptq_{name}', **out)
    print('gptq fixtures written')


GENERATORS = {'quant': gen_quant, 'gptq': gen_gptq}


if __name__ == '__main__':
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    R.install()
    for k, fn in GENERATORS.items():
        if which in ('all', k):
            fn()
