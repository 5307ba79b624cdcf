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
from inputs import fp8_inputs  # noqa: E402


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
        # name, oc, ic, bit, sym, group, actorder, dead_cols[, calib_algo]
        ('int4_asym_g128_act', 192, 512, 4, False, 128, True, False),
        ('int4_sym_g128_noact', 128, 384, 4, True, 128, False, False),
        ('int4_asym_g64_act_dead', 128, 256, 4, False, 64, True, True),
        ('int8_sym_g128_act', 64, 256, 8, True, 128, True, False),
        # calib_algo mse: group ranges searched in the loop (gptq_w_only.yml's commented
        # option); prefix gptqmse_
        ('mse:int4_asym_g128_act', 192, 512, 4, False, 128, True, False),
        ('mse:int4_sym_g64_act', 128, 256, 4, True, 64, True, False),
        ('mse:int3_asym_g128_noact', 64, 384, 3, False, 128, False, False),
    ]
    for i, (name, oc, ic, bit, sym, gs, act, dead) in enumerate(cases):
        calib = 'minmax'
        if name.startswith('mse:'):
            calib, name = 'mse', name[4:]
        torch.manual_seed(1000 + i)
        layer = nn.Linear(ic, oc, bias=False)
        layer.weight.data = weights(oc, ic, torch.bfloat16, 200 + i, edge=False)
        xs = _acts(3, 48, ic, 300 + i)
        if dead:
            for x in xs:
                x[..., 5] = 0
                x[..., 77] = 0
        obj = gm.GPTQ.__new__(gm.GPTQ)
        obj.wquantizer = q.IntegerQuantizer(bit, sym, 'per_group', group_size=gs,
                                            calib_algo=calib)
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
        F.save(f'gptq{"mse" if calib == "mse" else ""}_{name}', **out)
    print('gptq fixtures written')


def tiny_llama(seed=0, hidden=256, inter=512, heads=4, kv=2):
    """A random-init HF Llama decoder layer (bf16) + its rotary embedding, CPU."""
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml
    cfg = LlamaConfig(hidden_size=hidden, intermediate_size=inter, num_attention_heads=heads,
                      num_key_value_heads=kv, num_hidden_layers=1, vocab_size=128,
                      max_position_embeddings=2048, rms_norm_eps=1e-5)
    cfg._attn_implementation = 'sdpa'
    torch.manual_seed(seed)
    layer = ml.LlamaDecoderLayer(cfg, layer_idx=0)
    with torch.no_grad():
        for n, p in layer.named_parameters():
            if p.dim() == 2:
                p.normal_(0, 0.02)
            else:
                p.uniform_(0.5, 1.5)
    layer = layer.to(torch.bfloat16).eval()
    rot = ml.LlamaRotaryEmbedding(cfg)
    return cfg, layer, rot


def _awq_obj(wq, nsamples, version='v2'):
    import llmc.compression.quantization.awq as am
    obj = am.Awq.__new__(am.Awq)
    obj.wquantizer = wq
    obj.trans_version, obj.awq_bs, obj.save_mem = version, None, True
    obj.padding_mask, obj.w_only, obj.n_samples = None, True, nsamples
    obj.losses_seen = []
    orig = am.Awq.calculate_loss

    def rec(org_out, out, _o=obj):
        v = orig(_o, org_out, out)
        _o.losses_seen.append(v)
        return v
    obj.calculate_loss = rec
    return obj


def gen_awq(only_v1=False):
    """Reference Awq.search_scale_subset (+ apply_scale) on the three Llama subsets that AWQ
    transforms (qkv / gate-up / down; o_proj is skipped under GQA) of a tiny bf16 layer."""
    R.init_dist()
    q = R.quant_module()
    cfg, layer, rot = tiny_llama()
    # base_model.py registers the model's norm class as an LN type (what the adapter does)
    mu = R.module_utils()
    if type(layer.input_layernorm) not in mu._TRANSFORMERS_LN_TYPES_:
        mu._TRANSFORMERS_LN_TYPES_.append(type(layer.input_layernorm))
    n, seq = 4, 32
    g = torch.Generator().manual_seed(5)
    hidden = (torch.randn(n, seq, cfg.hidden_size, generator=g) *
              torch.exp(torch.randn(cfg.hidden_size, generator=g) * 0.5)).to(torch.bfloat16)
    pos = torch.arange(seq).unsqueeze(0)
    cos, sin = rot(hidden, pos)
    kwargs = {'position_embeddings': (cos, sin), 'attention_mask': None, 'position_ids': pos}
    for sym, version in ((True, 'v2'), (False, 'v2'), (True, 'v1'), (False, 'v1')):
        if only_v1 and version != 'v1':
            continue
        wq = q.IntegerQuantizer(4, sym, 'per_group', group_size=128)
        tag = ('sym' if sym else 'asym') + ('' if version == 'v2' else '_v1')
        import copy
        lay = copy.deepcopy(layer)
        with torch.no_grad():
            x_qkv = lay.input_layernorm(hidden)
            attn_out = lay.self_attn(x_qkv, **kwargs)[0]
            h2 = hidden + attn_out
            x_mlp = lay.post_attention_layernorm(h2)
            x_down = lay.mlp.act_fn(lay.mlp.gate_proj(x_mlp)) * lay.mlp.up_proj(x_mlp)
        subsets = [
            ('qkv', lay.input_layernorm, {'q': lay.self_attn.q_proj, 'k': lay.self_attn.k_proj,
                                          'v': lay.self_attn.v_proj}, x_qkv, lay.self_attn, [kwargs]),
            ('mlp', lay.post_attention_layernorm, {'gate': lay.mlp.gate_proj,
                                                   'up': lay.mlp.up_proj}, x_mlp, lay.mlp, {}),
            ('down', lay.mlp.up_proj, {'down': lay.mlp.down_proj}, x_down, lay.mlp.down_proj, {}),
        ]
        for name, prev, layers, x, inspect, kw in subsets:
            obj = _awq_obj(wq, n, version)
            w_before = {k: m.weight.data.clone() for k, m in layers.items()}
            w_max = obj.get_weight_scale(layers) if version == 'v1' else None
            if version == 'v1':
                # awq.py:199 backs the weights up with `.cpu()`: a copy on the GPU, the SAME
                # tensors on a CPU-only run, where the in-place W.mul_(s) of the first ratio
                # (awq.py:40-46) then leaks into every later ratio. v2's first scales are all
                # 1 (x^0), v1's are not: back up real copies, as the reference's GPU run does.
                inspect.state_dict = (lambda *a, _m=inspect, **k: {
                    kk: vv.clone() for kk, vv in type(_m).state_dict(_m, *a, **k).items()})
            prev_before = prev.weight.data.clone()
            best = obj.search_scale_subset(prev, layers, [x.clone()], inspect, False, kw)
            losses = torch.tensor(obj.losses_seen, dtype=torch.float64)
            obj.num_key_value_heads, obj.has_gqa = cfg.num_key_value_heads, True
            obj.apply_scale(best, [prev], list(layers.values()))
            out = dict(x=x, scales=best, losses=losses, prev_w=prev_before,
                       prev_w_after=prev.weight.data.clone(), w_max=w_max)
            for k in layers:
                out[f'w_{k}'] = w_before[k]
                out[f'w_{k}_after'] = layers[k].weight.data.clone()
            F.save(f'awq_{name}_{tag}', **out)
    # layer weights/config for re-building the module on the test side
    F.save('awq_layer', **{k.replace('.', '__'): v for k, v in layer.state_dict().items()},
           hidden=hidden, cos=cos, sin=sin,
           cfg=torch.tensor([cfg.hidden_size, cfg.intermediate_size,
                             cfg.num_attention_heads, cfg.num_key_value_heads]))
    print('awq fixtures written')


def gen_clip():
    """Reference AutoClipper.auto_clip_layer (clip v1) + apply_clip on bf16 / fp16 layers,
    group sizes 32 .. 256."""
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.auto_clip as ac
    bf, hf = torch.bfloat16, torch.float16
    # (name, sym, clip_sym, oc, ic, tokens, n_sample_token, group, model dtype)
    cases = [('sym_s', True, True, 128, 256, 512, 64, 128, bf),
             ('asym_s', False, False, 128, 256, 512, 64, 128, bf),
             ('sym_w_asym_clip', True, False, 256, 512, 1024, 128, 128, bf),
             ('asym_g64', False, False, 192, 256, 512, 64, 64, bf),      # DSv3 configs
             ('sym_g256', True, True, 128, 512, 512, 64, 256, bf),
             ('asym_g128_f16', False, False, 128, 512, 512, 64, 128, hf),  # OPT (fp16)
             ('sym_g32_f16', True, True, 64, 256, 512, 64, 32, hf),
             # calib_algo mse: every shrink step's fake quant searches its range
             ('mse_asym_g128', False, False, 128, 256, 512, 64, 128, bf),
             ('mse_sym_g64', True, True, 64, 256, 512, 64, 64, bf)]
    for i, (name, sym, clip_sym, oc, ic, ntok, nst, grp, dt) in enumerate(cases):
        calib = 'mse' if name.startswith('mse_') else 'minmax'
        wq = q.IntegerQuantizer(4, sym, 'per_group', group_size=grp, calib_algo=calib)
        clipper = ac.AutoClipper(w_only=True, wquantizer=wq, aquantizer=None,
                                 clip_version='v1', clip_sym=clip_sym, save_clip=False,
                                 padding_mask=None)
        w = weights(oc, ic, dt, 400 + i, edge=False)
        x = _acts(1, ntok, ic, 500 + i, dtype=dt)[0]
        bmax, bmin = clipper.auto_clip_layer(0, 'l', w.clone(), [x.clone()],
                                             n_sample_token=nst)
        m = torch.nn.Linear(ic, oc, bias=False).to(dt)
        m.weight.data = w.clone()
        clipper.apply_clip(0, m, bmin.clone(), bmax.clone(), 'l')
        F.save(f'clip_{name}', w=w, x=x, best_max=bmax, best_min=bmin,
               w_clipped=m.weight.data.clone(),
               meta=torch.tensor([int(sym), int(clip_sym), nst, grp, int(calib == 'mse')]))
    print('clip fixtures written')


def gen_clip_act():
    """Reference AutoClipper.auto_clip_layer for per_channel weights (group = ic) and with
    activation fake-quant (w_only False: awq_w8a8.yml's int8 per_token act), bf16 / fp16."""
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.auto_clip as ac
    bf, hf = torch.bfloat16, torch.float16
    # (name, wbit, sym, clip_sym, granularity, group, act (bit, sym) or None, oc, ic, dtype)
    cases = [('pc_w8a8', 8, True, True, 'per_channel', -1, (8, True), 256, 512, bf),
             ('pc_w8_wonly', 8, True, True, 'per_channel', -1, None, 256, 512, bf),
             ('pc_w4_asym', 4, False, False, 'per_channel', -1, None, 128, 1024, bf),
             ('pc_w8a8_asym_f16', 8, False, False, 'per_channel', -1, (8, False), 128, 512, hf),
             ('pg_w4a8', 4, False, False, 'per_group', 128, (8, True), 128, 512, bf)]
    for i, (name, wb, sym, clip_sym, gran, grp, act, oc, ic, dt) in enumerate(cases):
        kw = {'group_size': grp} if gran == 'per_group' else {}
        wq = q.IntegerQuantizer(wb, sym, gran, **kw)
        aq = q.IntegerQuantizer(act[0], act[1], 'per_token') if act else None
        clipper = ac.AutoClipper(w_only=act is None, wquantizer=wq, aquantizer=aq,
                                 clip_version='v1', clip_sym=clip_sym, save_clip=False,
                                 padding_mask=None)
        w = weights(oc, ic, dt, 700 + i, edge=False)
        x = _acts(1, 512, ic, 800 + i, dtype=dt)[0]
        bmax, bmin = clipper.auto_clip_layer(0, 'l', w.clone(), [x.clone()],
                                             n_sample_token=64)
        F.save(f'clipact_{name}', w=w, x=x, best_max=bmax, best_min=bmin,
               meta=torch.tensor([wb, int(sym), int(clip_sym), 64, grp,
                                  act[0] if act else 0, int(act[1]) if act else 0]))
    print('clip act / per-channel fixtures written')


GENERATORS = {'quant': gen_quant, 'gptq': gen_gptq, 'awq': gen_awq, 'clip': gen_clip,
              'clip_act': gen_clip_act}


def gen_fp8():
    """FloatQuantizer pieces the reference runs without qtorch: the use_qtorch=False
    (get_float_qparams) fake quant end to end, the use_qtorch scales (get_minmax_range +
    get_qparams with qmax = finfo.max, as quant.py:982-996 sets it), and the per_block
    weight_cast_to_bf16 sequence (reshape_tensor -> dequant -> restore_tensor)."""
    q = R.quant_module()
    emul = [
        # name, bit, gran, group, dtype
        ('e4m3_pc_bf16', 'e4m3', 'per_channel', None, torch.bfloat16),
        ('e4m3_g128_bf16', 'e4m3', 'per_group', 128, torch.bfloat16),
        ('e5m2_pc_bf16', 'e5m2', 'per_channel', None, torch.bfloat16),
        ('e4m3_pc_f16', 'e4m3', 'per_channel', None, torch.float16),
        ('e3m2_pc_bf16', 'e3m2', 'per_channel', None, torch.bfloat16),
    ]
    for i, (name, bit, gran, gs, dt) in enumerate(emul):
        kw = {'group_size': gs} if gs else {}
        fq = q.FloatQuantizer(bit, True, gran, **kw)
        w = fp8_inputs(16, 512, dt, 200 + i)
        aq = q.FloatQuantizer(bit, True, 'per_token')
        a = fp8_inputs(24, 256, dt, 300 + i)
        F.save(f'fp8emul_{name}', w=w, fq=fq.fake_quant_weight_dynamic(w.clone()), act=a,
               act_fq=aq.fake_quant_act_dynamic(a.clone()),
               meta=torch.tensor([int(bit[1]), int(bit[-1]), gs or 512]))

    scl = [
        ('e4m3_pc_bf16', 'e4m3', 'per_channel', {}, torch.bfloat16, (16, 512)),
        ('e4m3_g128_bf16', 'e4m3', 'per_group', {'group_size': 128}, torch.bfloat16, (16, 512)),
        ('e4m3_pt_bf16', 'e4m3', 'per_tensor', {}, torch.bfloat16, (16, 512)),
        ('e5m2_pc_f16', 'e5m2', 'per_channel', {}, torch.float16, (16, 512)),
        ('e4m3_blk_bf16', 'e4m3', 'per_block', {'block_size': 128}, torch.bfloat16, (256, 384)),
        ('e4m3_blk_ragged_bf16', 'e4m3', 'per_block', {'block_size': 128}, torch.bfloat16,
         (200, 256)),
    ]
    fp8 = {'e4m3': torch.float8_e4m3fn, 'e5m2': torch.float8_e5m2}
    for i, (name, bit, gran, kw, dt, shape) in enumerate(scl):
        qz = q.FloatQuantizer(bit, True, gran, **kw)
        fi = torch.finfo(fp8[bit])
        qz.qmin, qz.qmax = torch.tensor(fi.min), torch.tensor(fi.max)
        w = fp8_inputs(*shape, dt, 400 + i)
        t = qz.reshape_tensor(w)
        s, z, _, _ = qz.get_qparams(qz.get_minmax_range(t), 'cpu')
        F.save(f'fp8scale_{name}', w=w, scales=s)

    # weight_cast_to_bf16 (quant.py:18-31) through the reference's own per_block methods
    for name, (M, N) in {'even': (256, 384), 'ragged_m': (200, 256)}.items():
        g = torch.Generator().manual_seed(500 + M)
        codes = torch.randint(0, 256, (M, N), generator=g, dtype=torch.uint8)
        codes[(codes & 0x7f) == 0x7f] = 0x3c  # no NaN encodings
        codes = codes.view(torch.float8_e4m3fn)
        sc = (torch.rand(-(-M // 128), -(-N // 128), generator=g) * 1e-3 + 1e-4).float()
        qz = q.FloatQuantizer('e4m3', True, 'per_block', block_size=128)
        t = qz.reshape_tensor(codes)
        deq = qz.dequant(t.float(), sc.view(sc.shape[0], 1, sc.shape[1], 1), 0)
        out = qz.restore_tensor(deq, codes.shape).to(torch.bfloat16)
        F.save(f'fp8cast_bf16_{name}', codes=codes, scales=sc, out=out)


GENERATORS['fp8'] = gen_fp8


def gen_gptq_static():
    """GPTQ with static_groups (gptq.py:224-227): the group qparams collected from the
    original weights before the transform are used unchanged; with actorder the permuted
    column j takes group perm[j] // group_size."""
    import torch.nn as nn
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.gptq as gm
    cases = [
        # name, oc, ic, bit, sym, group, actorder, dead_cols
        ('int4_asym_g128_act', 192, 512, 4, False, 128, True, False),
        ('int4_sym_g64_act_dead', 128, 384, 4, True, 64, True, True),
        ('int4_asym_g128_noact', 128, 256, 4, False, 128, False, False),
        ('int8_asym_g32_act', 64, 256, 8, False, 32, True, False),
    ]
    for i, (name, oc, ic, bit, sym, gs, act, dead) in enumerate(cases):
        torch.manual_seed(2000 + i)
        layer = nn.Linear(ic, oc, bias=False)
        layer.weight.data = weights(oc, ic, torch.bfloat16, 400 + i, edge=False)
        xs = _acts(3, 48, ic, 500 + i)
        if dead:
            for x in xs:
                x[..., 3] = 0
                x[..., 101] = 0
        obj = gm.GPTQ.__new__(gm.GPTQ)
        obj.wquantizer = q.IntegerQuantizer(bit, sym, 'per_group', group_size=gs,
                                            calib_algo=calib)
        obj.dev = torch.device('cpu')
        obj.model_dtype = torch.bfloat16
        obj.owq, obj.actorder, obj.static_groups = False, act, True
        obj.percdamp, obj.blocksize, obj.chunk_num = 0.01, 128, 1
        obj.true_sequential = True
        obj.need_perm = False  # gptq.py:52-56
        obj.layers_cache = {'l': {}}
        obj.qparams = {}
        gm.GPTQ.layer_init(obj, layer, 'l')
        for x in xs:
            gm.GPTQ.add_batch(obj, layer, 'l', x, None)
        H = obj.layers_cache['l']['H'].clone()
        _, s0, z0, qmax, qmin = obj.wquantizer.get_tensor_qparams(layer.weight.data)
        layer.register_buffer('buf_scales', s0)
        layer.register_buffer('buf_zeros', z0)
        layer.register_buffer('buf_qmax', torch.tensor(qmax))
        layer.register_buffer('buf_qmin', torch.tensor(qmin))
        w_in = layer.weight.data.clone()
        obj.layers_cache['l']['H'] = H.clone()
        obj.initialize_qparams_and_prepare_weights(layer, 'l')
        Wp, U = obj.process_hessian_and_weights(layer, 'l')
        obj.layers_cache['l']['H'] = H.clone()
        obj.qparams = {}
        layer.weight.data = w_in.clone()
        obj.layer_transform(layer, 'l')
        out = dict(x=torch.cat(xs, 0), w=w_in, H=H, U=U,
                   perm=getattr(layer, 'buf_perm', None), weight=layer.weight.data.clone(),
                   scales=layer.buf_scales, zeros=None if sym else layer.buf_zeros,
                   meta=torch.tensor([bit, int(sym), gs, int(act), oc, ic]))
        out['fq'] = obj.w_qdq(layer, obj.wquantizer)
        codes, s_rq, z_rq = obj.w_q(layer, obj.wquantizer)
        out.update(codes=codes, scales_rq=s_rq, zeros_rq=z_rq)
        F.save(f'gptqsg_{name}', **out)
    print('gptq static_groups fixtures written')


GENERATORS['gptq_static'] = gen_gptq_static


def gen_act_static():
    """Static per-tensor activation qparams (get_batch_tensors_qparams, quant.py:561-586) for
    the act_tensors lists register_act_qparams passes: a single [n, T, H] entry (calib bs -1,
    split per sample), n [1, T, H] entries (bs 1) or [b, T, H] entries (bs b). FP8: the
    use_qtorch qparams (qmax = finfo.max, quant.py:982-996) on a use_qtorch=False object, as
    in gen_fp8 (qtorch is absent here); int cases also pin fake_quant_act_static."""
    q = R.quant_module()
    cases = [
        # name, quant, bit, sym, algo, n_entries, entry_bs, T, H, dtype
        ('int8_sym_minmax_bs1', 'int', 8, True, 'static_minmax', 6, 1, 48, 256, torch.bfloat16),
        ('int8_asym_minmax_single', 'int', 8, False, 'static_minmax', 1, 5, 32, 384,
         torch.bfloat16),
        ('int8_sym_moving_bs1', 'int', 8, True, 'static_moving_minmax', 7, 1, 40, 256,
         torch.bfloat16),
        ('int8_asym_moving_single', 'int', 8, False, 'static_moving_minmax', 1, 6, 32, 512,
         torch.bfloat16),
        ('int4_asym_moving_bs2_f16', 'int', 4, False, 'static_moving_minmax', 4, 2, 24, 256,
         torch.float16),
        ('int8_sym_minmax_bs3_f32', 'int', 8, True, 'static_minmax', 3, 3, 16, 128,
         torch.float32),
        ('int8_asym_moving_bs1_f32', 'int', 8, False, 'static_moving_minmax', 5, 1, 16, 256,
         torch.float32),
        ('fp8e4m3_minmax_bs1', 'e4m3', 8, True, 'static_minmax', 5, 1, 32, 256, torch.bfloat16),
        ('fp8e4m3_moving_single', 'e4m3', 8, True, 'static_moving_minmax', 1, 6, 32, 256,
         torch.bfloat16),
        ('fp8e5m2_moving_bs1', 'e5m2', 8, True, 'static_moving_minmax', 4, 1, 32, 256,
         torch.bfloat16),
    ]
    for i, (name, qt, bit, sym, algo, ne, eb, T, H, dt) in enumerate(cases):
        g = torch.Generator().manual_seed(900 + i)
        mag = torch.exp(torch.randn(H, generator=g))
        shift = 0.3 * torch.randn(H, generator=g)   # asymmetric ranges
        x = ((torch.randn(ne * eb, T, H, generator=g) + shift) * mag).to(dt)
        entries = [x] if ne == 1 else [x[j * eb:(j + 1) * eb] for j in range(ne)]
        if qt == 'int':
            quant = q.IntegerQuantizer(bit, sym, 'per_tensor', calib_algo=algo)
        else:
            quant = q.FloatQuantizer(qt, True, 'per_tensor', calib_algo=algo, use_qtorch=False)
            fi = torch.finfo(torch.float8_e4m3fn if qt == 'e4m3' else torch.float8_e5m2)
            quant.qmin, quant.qmax = torch.tensor(fi.min), torch.tensor(fi.max)
        sc, zc, qmn, qmx = quant.get_batch_tensors_qparams([e.clone() for e in entries])
        out = dict(x=x, scales=sc[0], zeros=zc[0],
                   meta=torch.tensor([ne, eb, bit if qt == 'int' else 0, int(sym),
                                      ['static_minmax', 'static_moving_minmax'].index(algo)]))
        if qt == 'int':
            args = dict(scales=sc[0], zeros=zc[0], qmax=qmx[0], qmin=qmn[0])
            out['fq'] = quant.fake_quant_act_static(entries[0].clone(), args)
        F.save(f'actstatic_{qt}_{name}' if qt != 'int' else f'actstatic_{name}', **out)
    print('act static fixtures written')


GENERATORS['act_static'] = gen_act_static


def gen_act_hist():
    """static_hist (quant.py:264-529): IntegerQuantizer(8, sym, per_tensor) qparams and the
    thresholded range, for growing ranges (histogram upscaling), shrinking ones (plain adds)
    and one entry split per sample."""
    q = R.quant_module()
    cases = [
        # name, n_entries, entry_bs, T, H, dtype, growth per entry
        ('bs1_grow', 6, 1, 48, 256, torch.bfloat16, 1.3),
        ('bs1_shrink', 5, 1, 40, 256, torch.bfloat16, 0.8),
        ('single', 1, 5, 32, 384, torch.bfloat16, 1.1),
        ('bs2_f32', 4, 2, 24, 256, torch.float32, 1.2),
    ]
    for i, (name, ne, eb, T, H, dt, grow) in enumerate(cases):
        g = torch.Generator().manual_seed(1200 + i)
        mag = torch.exp(torch.randn(H, generator=g))
        xs = [((torch.randn(eb, T, H, generator=g) + 0.2) * mag * grow ** j).to(dt)
              for j in range(ne)]
        x = torch.cat(xs, 0)
        entries = [x] if ne == 1 else xs
        quant = q.IntegerQuantizer(8, True, 'per_tensor', calib_algo='static_hist')
        mn, mx = quant.get_static_hist_range([e.clone() for e in entries])
        sc, zc, _, _ = quant.get_batch_tensors_qparams([e.clone() for e in entries])
        F.save(f'acthist_{name}', x=x, scales=sc[0], zeros=zc[0], rmin=mn[0], rmax=mx[0],
               meta=torch.tensor([ne, eb, 8, 1, 2]))
    print('act hist fixtures written')


GENERATORS['act_hist'] = gen_act_hist


def gen_mse():
    """calib_algo 'mse' weight qparams (quant.py:145-203): the searched ranges, get_tensor_qparams
    scales / zeros, fake_quant_weight_dynamic and real_quant_weight_dynamic outputs."""
    q = R.quant_module()
    cases = [
        # name, bit, sym, granularity, group, rows, cols, mse_b_num
        ('int4_asym_g128', 4, False, 'per_group', 128, 256, 512, 1),
        ('int4_sym_g128', 4, True, 'per_group', 128, 128, 512, 2),
        ('int8_sym_pc', 8, True, 'per_channel', None, 128, 1024, 1),
        ('int4_asym_pc', 4, False, 'per_channel', None, 96, 768, 1),
    ]
    for i, (name, bit, sym, gran, gs, rows, cols, bnum) in enumerate(cases):
        w = weights(rows, cols, torch.bfloat16, 1500 + i, edge=False)
        kw = dict(calib_algo='mse', mse_b_num=bnum)
        if gs:
            kw['group_size'] = gs
        quant = q.IntegerQuantizer(bit, sym, gran, **kw)
        t = quant.reshape_tensor(w.clone())
        mn, mx = quant.get_mse_range(t)
        _, s, z, _, _ = quant.get_tensor_qparams(w.clone())
        fq = quant.fake_quant_weight_dynamic(w.clone())
        codes, s_rq, z_rq = quant.real_quant_weight_dynamic(w.clone())
        F.save(f'mse_{name}', w=w, rmin=mn, rmax=mx, scales=s, zeros=None if sym else z, fq=fq,
               codes=codes, meta=torch.tensor([bit, int(sym), gs or 0, bnum]))
    print('mse fixtures written')


GENERATORS['mse'] = gen_mse
GENERATORS['awq_v1'] = lambda: gen_awq(only_v1=True)


def gen_gptq_owq():
    """GPTQ with OWQ (gptq.py:44-83, 178-196, 424-452): the n_out largest-diag input columns
    move to the end of the permutation, stay in float (error-compensated) and are excluded
    from the quantized groups."""
    import torch.nn as nn
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.gptq as gm
    cases = [
        # name, oc, ic, bit, sym, group, n_out, dead_cols
        ('int4_asym_g128_out6', 192, 512, 4, False, 128, 6, False),
        ('int4_sym_g64_out2_dead', 128, 384, 4, True, 64, 2, True),
        ('int8_asym_g32_out32', 96, 256, 8, False, 32, 32, False),
    ]
    for i, (name, oc, ic, bit, sym, gs, nout, dead) in enumerate(cases):
        torch.manual_seed(3000 + i)
        layer = nn.Linear(ic, oc, bias=False)
        layer.weight.data = weights(oc, ic, torch.bfloat16, 600 + i, edge=False)
        xs = _acts(3, 48, ic, 700 + i)
        if dead:
            for x in xs:
                x[..., 9] = 0
        obj = gm.GPTQ.__new__(gm.GPTQ)
        obj.wquantizer = q.IntegerQuantizer(bit, sym, 'per_group', group_size=gs,
                                            calib_algo=calib)
        obj.dev = torch.device('cpu')
        obj.model_dtype = torch.bfloat16
        obj.owq, obj.actorder, obj.static_groups = True, False, False
        obj.percdamp, obj.blocksize, obj.chunk_num = 0.01, 128, 1
        obj.true_sequential = True
        obj.need_perm = True
        obj.n_out_dict = {'l': nout}
        obj.layers_cache = {'l': {}}
        obj.qparams = {}
        gm.GPTQ.layer_init(obj, layer, 'l')
        for x in xs:
            gm.GPTQ.add_batch(obj, layer, 'l', x, None)
        H = obj.layers_cache['l']['H'].clone()
        _, s0, z0, qmax, qmin = obj.wquantizer.get_tensor_qparams(layer.weight.data)
        layer.register_buffer('buf_scales', s0)
        layer.register_buffer('buf_zeros', z0)
        layer.register_buffer('buf_qmax', torch.tensor(qmax))
        layer.register_buffer('buf_qmin', torch.tensor(qmin))
        w_in = layer.weight.data.clone()
        obj.layers_cache['l']['H'] = H.clone()
        obj.qparams = {}
        obj.layer_transform(layer, 'l')
        out = dict(x=torch.cat(xs, 0), w=w_in, H=H, perm=layer.buf_perm,
                   weight=layer.weight.data.clone(), scales=layer.buf_scales,
                   zeros=None if sym else layer.buf_zeros,
                   meta=torch.tensor([bit, int(sym), gs, nout, oc, ic]))
        out['fq'] = obj.w_qdq(layer, obj.wquantizer)
        F.save(f'gptqowq_{name}', **out)
    print('gptq owq fixtures written')


GENERATORS['gptq_owq'] = gen_gptq_owq


def gen_gptq_owq_pc():
    """GPTQ OWQ with per_channel weights (gptq.py:157-166): the per-channel qparams are taken
    from the permuted, dead-zeroed fp32 non-outlier columns and replace buf_scales / buf_zeros."""
    import torch.nn as nn
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.gptq as gm
    cases = [
        # name, oc, ic, bit, sym, n_out, dead_cols
        ('int4_asym_pc_out6', 160, 384, 4, False, 6, False),
        ('int8_sym_pc_out16_dead', 96, 256, 8, True, 16, True),
    ]
    for i, (name, oc, ic, bit, sym, nout, dead) in enumerate(cases):
        torch.manual_seed(3100 + i)
        layer = nn.Linear(ic, oc, bias=False)
        layer.weight.data = weights(oc, ic, torch.bfloat16, 650 + i, edge=False)
        xs = _acts(3, 48, ic, 750 + i)
        if dead:
            for x in xs:
                x[..., 5] = 0
        obj = gm.GPTQ.__new__(gm.GPTQ)
        obj.wquantizer = q.IntegerQuantizer(bit, sym, 'per_channel')
        obj.dev = torch.device('cpu')
        obj.model_dtype = torch.bfloat16
        obj.owq, obj.actorder, obj.static_groups = True, False, False
        obj.percdamp, obj.blocksize, obj.chunk_num = 0.01, 128, 1
        obj.true_sequential = True
        obj.need_perm = True
        obj.n_out_dict = {'l': nout}
        obj.layers_cache = {'l': {}}
        obj.qparams = {}
        gm.GPTQ.layer_init(obj, layer, 'l')
        for x in xs:
            gm.GPTQ.add_batch(obj, layer, 'l', x, None)
        H = obj.layers_cache['l']['H'].clone()
        _, s0, z0, qmax, qmin = obj.wquantizer.get_tensor_qparams(layer.weight.data)
        layer.register_buffer('buf_scales', s0)
        layer.register_buffer('buf_zeros', z0)
        layer.register_buffer('buf_qmax', torch.tensor(qmax))
        layer.register_buffer('buf_qmin', torch.tensor(qmin))
        w_in = layer.weight.data.clone()
        obj.layers_cache['l']['H'] = H.clone()
        obj.layer_transform(layer, 'l')
        out = dict(x=torch.cat(xs, 0), w=w_in, H=H, perm=layer.buf_perm,
                   weight=layer.weight.data.clone(), scales=layer.buf_scales,
                   zeros=None if sym else layer.buf_zeros,
                   meta=torch.tensor([bit, int(sym), 0, nout, oc, ic]))
        out['fq'] = obj.w_qdq(layer, obj.wquantizer)
        F.save(f'gptqowqpc_{name}', **out)
    print('gptq owq per_channel fixtures written')


GENERATORS['gptq_owq_pc'] = gen_gptq_owq_pc


def gen_hqq():
    """calib_algo hqq (quant.py:588-610, 680-697) and round_zp False (quant.py:545-559,
    699-707): get_tensor_qparams, fake_quant_weight_dynamic, real_quant_weight_dynamic."""
    q = R.quant_module()
    cases = [
        # name, bit, sym, granularity, group, rows, cols, calib, round_zp, extra kwargs
        ('hqq_int4_asym_g128_nozp', 4, False, 'per_group', 128, 256, 512, 'hqq', False, {}),
        ('hqq_int4_asym_g64_rzp', 4, False, 'per_group', 64, 128, 512, 'hqq', True, {}),
        ('hqq_int3_sym_g128', 3, True, 'per_group', 128, 128, 384, 'hqq', True, {}),
        ('hqq_int4_asym_pc_l1', 4, False, 'per_channel', None, 96, 768, 'hqq', False,
         dict(lp_norm=1, beta=20, iters=8)),
        ('nozp_int4_asym_g128_bf16', 4, False, 'per_group', 128, 256, 512, 'minmax', False, {}),
        ('nozp_int8_asym_pc_bf16', 8, False, 'per_channel', None, 64, 1024, 'minmax', False, {}),
        ('nozp_int4_asym_g128_f32', 4, False, 'per_group', 128, 64, 256, 'minmax', False, {}),
    ]
    for i, (name, bit, sym, gran, gs, rows, cols, calib, rzp, kw) in enumerate(cases):
        dt = torch.float32 if name.endswith('f32') else torch.bfloat16
        w = weights(rows, cols, dt, 1700 + i, edge=False)
        kwa = dict(calib_algo=calib, round_zp=rzp, **kw)
        if gs:
            kwa['group_size'] = gs
        quant = q.IntegerQuantizer(bit, sym, gran, **kwa)
        _, s, z, _, _ = quant.get_tensor_qparams(w.clone())
        fq = quant.fake_quant_weight_dynamic(w.clone())
        codes, s_rq, z_rq = quant.real_quant_weight_dynamic(w.clone())
        lp, beta, iters = kw.get('lp_norm', 0.7), kw.get('beta', 10), kw.get('iters', 20)
        F.save(name, w=w, scales=s, zeros=z if torch.is_tensor(z) and z.dim() else None,
               fq=fq, codes=codes, zeros_rq=z_rq,
               meta=torch.tensor([bit, int(sym), gs or 0, int(rzp), int(calib == 'hqq'),
                                  iters]),
               hqq=torch.tensor([float(lp), float(beta)]))
    print('hqq / round_zp fixtures written')


GENERATORS['hqq'] = gen_hqq


def gen_fp8_algos():
    """Float-quant (FP8) weights inside auto-clip and the GPTQ column loop (the
    backend/{vllm,sglang}/fp8 awq_fp8*.yml / gptq_fp8.yml recipes): the reference's own
    AutoClipper.auto_clip_layer and GPTQ layer methods with FloatQuantizer(use_qtorch=True),
    qtorch's float_quantize replaced by the saturating native cast (R.native_float_quantize,
    DESIGN.md §5). Prefixes clipfp8_ / gptqfp8_."""
    import torch.nn as nn
    R.init_dist()
    q = R.quant_module()
    R.native_float_quantize()
    import llmc.compression.quantization.auto_clip as ac
    import llmc.compression.quantization.gptq as gm
    bf, hf = torch.bfloat16, torch.float16
    # (name, fmt, granularity, act granularity or None, oc, ic, dtype)
    cases = [('pc_e4m3', 'e4m3', 'per_channel', None, 256, 512, bf),
             ('pc_e4m3_a8', 'e4m3', 'per_channel', 'per_token', 256, 512, bf),
             ('pt_e4m3_b64', 'e4m3', 'per_tensor', 'per_tensor', 384, 512, bf),   # 64-row batches
             ('pt_e4m3_b256', 'e4m3', 'per_tensor', None, 512, 256, bf),
             ('pc_e4m3_f16', 'e4m3', 'per_channel', None, 128, 512, hf),
             ('pc_e5m2', 'e5m2', 'per_channel', None, 128, 384, bf)]
    for i, (name, fmt, gran, agran, oc, ic, dt) in enumerate(cases):
        wq = q.FloatQuantizer(fmt, True, gran, use_qtorch=True)
        aq = q.FloatQuantizer(fmt, True, agran, use_qtorch=True) if agran else None
        clipper = ac.AutoClipper(w_only=aq is None, wquantizer=wq, aquantizer=aq,
                                 clip_version='v1', clip_sym=True, save_clip=False,
                                 padding_mask=None)
        w = weights(oc, ic, dt, 1700 + i, edge=False)
        w[3, 5] = 0.4  # a row outlier: the clip has something to cut
        x = _acts(1, 512, ic, 1800 + i, dtype=dt)[0]
        bmax, bmin = clipper.auto_clip_layer(0, 'l', w.clone(), [x.clone()],
                                             n_sample_token=64)
        F.save(f'clipfp8_{name}', w=w, x=x, best_max=bmax, best_min=bmin,
               meta=torch.tensor([4 if fmt == 'e4m3' else 5, int(gran == 'per_tensor'),
                                  {None: 0, 'per_token': 1, 'per_tensor': 2}[agran], 64]))
    gcases = [  # name, fmt, granularity, group, actorder, oc, ic
        ('pc_e4m3_act', 'e4m3', 'per_channel', None, True, 192, 512),
        ('pc_e4m3_noact', 'e4m3', 'per_channel', None, False, 128, 384),
        ('pg_e4m3_g128_act', 'e4m3', 'per_group', 128, True, 128, 512),
        ('pc_e5m2_act', 'e5m2', 'per_channel', None, True, 128, 256)]
    for i, (name, fmt, gran, gs, act, oc, ic) in enumerate(gcases):
        torch.manual_seed(2000 + i)
        layer = nn.Linear(ic, oc, bias=False)
        layer.weight.data = weights(oc, ic, torch.bfloat16, 2100 + i, edge=False)
        xs = _acts(3, 48, ic, 2200 + i)
        obj = gm.GPTQ.__new__(gm.GPTQ)
        kw = {'group_size': gs} if gs else {}
        obj.wquantizer = q.FloatQuantizer(fmt, True, gran, use_qtorch=True, **kw)
        obj.dev = torch.device('cpu')
        obj.model_dtype = torch.bfloat16
        obj.owq, obj.actorder, obj.static_groups = False, act, False
        obj.percdamp, obj.blocksize, obj.chunk_num = 0.01, 128, 1
        obj.true_sequential = True
        obj.need_perm = act and gran == 'per_group'
        obj.layers_cache = {'l': {}}
        obj.qparams = {}
        gm.GPTQ.layer_init(obj, layer, 'l')
        for x in xs:
            gm.GPTQ.add_batch(obj, layer, 'l', x, None)
        H = obj.layers_cache['l']['H'].clone()
        _, s0, z0, qmax, qmin = obj.wquantizer.get_tensor_qparams(layer.weight.data)
        layer.register_buffer('buf_scales', s0)
        layer.register_buffer('buf_zeros', z0)
        layer.register_buffer('buf_qmax', torch.tensor(qmax))
        layer.register_buffer('buf_qmin', torch.tensor(qmin))
        w_in = layer.weight.data.clone()
        obj.layers_cache['l']['H'] = H.clone()
        obj.initialize_qparams_and_prepare_weights(layer, 'l')
        Wp, U = obj.process_hessian_and_weights(layer, 'l')
        obj.layers_cache['l']['H'] = H.clone()
        obj.qparams = {}
        layer.weight.data = w_in.clone()
        obj.layer_transform(layer, 'l')
        out = dict(x=torch.cat(xs, 0), w=w_in, H=H, U=U,
                   perm=getattr(layer, 'buf_perm', None), weight=layer.weight.data.clone(),
                   scales=layer.buf_scales,
                   meta=torch.tensor([4 if fmt == 'e4m3' else 5, gs or 0, int(act), oc, ic]))
        out['fq'] = obj.w_qdq(layer, obj.wquantizer)
        if not obj.need_perm:
            codes, s_rq, _ = obj.w_q(layer, obj.wquantizer)
            out.update(codes=codes, scales_rq=s_rq)
        F.save(f'gptqfp8_{name}', **out)
    print('fp8 clip / gptq fixtures written')


GENERATORS['fp8_algos'] = gen_fp8_algos


def gen_clip_v2():
    """clip_version v2 (awq_comb_omni w6a6 / w8a8 step_1_awq.yml): the reference's
    AutoClipper.auto_clip_layer with learnable-range candidates, apply_clip's logit factors
    (get_clip_factor) and the deploy fake quant with those factors
    (fake_quant_weight_dynamic with calib_algo learnable). Prefix clipv2_."""
    R.init_dist()
    q = R.quant_module()
    import llmc.compression.quantization.auto_clip as ac
    bf, hf = torch.bfloat16, torch.float16
    # (name, wbit, wsym, clip_sym, act (bit, sym) or None, oc, ic, dtype)
    cases = [('w8a8_asym', 8, False, False, (8, False), 256, 512, bf),
             ('w6a6_asym', 6, False, False, (6, False), 256, 384, bf),
             ('w4_asym_wonly', 4, False, False, None, 128, 256, bf),
             ('w4_sym', 4, True, True, None, 128, 512, bf),
             ('w6a6_asym_clipsym', 6, False, True, (6, False), 128, 256, bf),
             ('w6a8_sym_asymclip', 6, True, False, (8, True), 128, 256, bf),
             ('w8a8_asym_f16', 8, False, False, (8, False), 128, 512, hf)]
    for i, (name, wb, sym, clip_sym, act, oc, ic, dt) in enumerate(cases):
        wq = q.IntegerQuantizer(wb, sym, 'per_channel', calib_algo='learnable')
        aq = q.IntegerQuantizer(act[0], act[1], 'per_token') if act else None
        clipper = ac.AutoClipper(w_only=act is None, wquantizer=wq, aquantizer=aq,
                                 clip_version='v2', clip_sym=clip_sym, save_clip=True,
                                 padding_mask=None)
        w = weights(oc, ic, dt, 2500 + i, edge=False)
        w[3, 5] = 0.4   # row outliers: the clip has something to cut
        w[7, 9] = -0.3
        x = _acts(1, 512, ic, 2600 + i, dtype=dt)[0]
        bmax, bmin = clipper.auto_clip_layer(0, 'l', w.clone(), [x.clone()],
                                             n_sample_token=64)
        m = torch.nn.Linear(ic, oc, bias=False).to(dt)
        m.weight.data = w.clone()
        clipper.apply_clip(0, m, bmin.clone(), bmax.clone(), 'l')
        out = dict(w=w, x=x, best_max=bmax, best_min=bmin, up=m.buf_upbound_factor.clone(),
                   meta=torch.tensor([wb, int(sym), int(clip_sym), 64,
                                      act[0] if act else 0, int(act[1]) if act else 0]))
        args = {'lowbound_factor': m.buf_lowbound_factor, 'upbound_factor': m.buf_upbound_factor}
        if m.buf_lowbound_factor is not None:
            out['low'] = m.buf_lowbound_factor.clone()
        out['fq'] = wq.fake_quant_weight_dynamic(w.clone(), args)
        F.save(f'clipv2_{name}', **out)
    print('clip v2 fixtures written')


GENERATORS['clip_v2'] = gen_clip_v2


if __name__ == '__main__':
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    R.install()
    for k, fn in GENERATORS.items():
        if which in ('all', k):
            fn()
