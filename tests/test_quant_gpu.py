"""GPU parity: HIP grouped quant / pack kernels vs golden vectors and vs the oracle.

Bar: bit-exact (codes, packed words, bf16/fp16/fp32 scales, zeros, fake-quant values).
"""
import numpy as np
import pytest
import torch

import fixtures as F
from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu


def _bits(t):
    t = t.detach().cpu()
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.view(torch.int16)
    if t.dtype == torch.float32:
        return t.view(torch.int32)
    return t


def assert_bit_equal(got, exp, what=''):
    assert got.dtype == exp.dtype, (what, got.dtype, exp.dtype)
    assert tuple(got.shape) == tuple(exp.shape), (what, got.shape, exp.shape)
    g, e = _bits(got), _bits(exp)
    diff = g != e
    if got.is_floating_point():  # NaN sign / payload is not part of the value semantics
        diff &= ~(got.detach().cpu().isnan() & exp.isnan())
    n = diff.sum().item()
    assert n == 0, f'{what}: {n} / {g.numel()} elements differ'


@pytest.mark.parametrize('name', F.names('quant_int'))
def test_golden_dynamic(dev, name):
    from lightcompress_amd.quant import IntegerQuantizer
    from lightcompress_amd.module_utils import VllmRealQuantLinear
    c = F.load(name)
    bit, sym, gs, qmin, qmax = c['meta'].tolist()
    gran = 'per_channel' if 'pc' in name else 'per_group'
    kw = {'group_size': gs} if gran == 'per_group' else {}
    wq = IntegerQuantizer(bit, bool(sym), gran, **kw)
    w = c['w'].to(dev)
    assert_bit_equal(wq.fake_quant_weight_dynamic(w), c['fq'], 'fq')
    codes, s, z = wq.real_quant_weight_dynamic(w)
    assert_bit_equal(codes, c['codes'], 'codes')
    assert_bit_equal(s, c['scales'], 'scales')
    if sym:
        assert z is None
    else:
        assert_bit_equal(z, c['zeros'], 'zeros')
    if 'packed' in c:
        packed, s16 = VllmRealQuantLinear.pack(codes, s, {'weight': {'bit': bit}})
        assert_bit_equal(packed, c['packed'], 'packed')
        assert_bit_equal(s16, c['scales_fp16'], 'scales fp16')
    _, s2, z2, _, _ = wq.get_tensor_qparams(w)
    assert_bit_equal(s2.view(s.shape), c['scales'], 'get_tensor_qparams scales')


def test_golden_prescale(dev):
    from lightcompress_amd import ops
    c = F.load('quant_awq_prescale_int4_sym_g128_bf16')
    r = ops.int_quant_dynamic(c['w'].to(dev), 128, -8, 7, True, pre_scale=c['pre'].to(dev))
    assert_bit_equal(r['fq'], c['fq'], 'awq prescale fq')


@pytest.mark.parametrize('sym', [True, False])
def test_golden_clip(dev, sym):
    from lightcompress_amd import ops
    c = F.load(f'quant_clip_int4_{"sym" if sym else "asym"}_g128_bf16')
    qmin, qmax = (-8, 7) if sym else (0, 15)
    r = ops.int_quant_dynamic(c['w'].to(dev), 128, qmin, qmax, sym,
                              clip_max=c['cmax'].reshape(-1).to(dev),
                              clip_min=c['cmin'].reshape(-1).to(dev))
    assert_bit_equal(r['fq'], c['fq'], 'clip fq')


def test_golden_static(dev):
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load('quant_static_int4_asym_g128_f32')
    wq = IntegerQuantizer(4, False, 'per_group', group_size=128)
    args = {'scales': c['scales'].to(dev), 'zeros': c['zeros'].to(dev),
            'qmax': wq.qmax, 'qmin': wq.qmin}
    fq = wq.fake_quant_weight_static(c['w'].to(dev), args).to(torch.bfloat16)
    assert_bit_equal(fq, c['fq_bf16'], 'static fq')
    args['scales'] = args['scales'].to(torch.bfloat16)
    codes, s, z = wq.real_quant_weight_static(c['w'].to(dev), args)
    assert_bit_equal(codes, c['codes'], 'static codes')
    assert_bit_equal(s, c['scales_rq'], 'static scales')
    assert_bit_equal(z, c['zeros_rq'], 'static zeros')


@pytest.mark.parametrize('name', F.names('awqpack_'))
def test_golden_gemm_pack(dev, name):
    from lightcompress_amd import ops
    c = F.load(name)
    qw, s16, qz = ops.pack_autoawq_gemm(c['w'].to(dev), c['scales'].to(dev),
                                        c['zeros'].to(dev), 128)
    assert_bit_equal(qw, c['qweight'], 'qweight')
    assert_bit_equal(s16, c['scales_t'], 'scales_t')
    assert_bit_equal(qz, c['qzeros'], 'qzeros')


# ---- larger random shapes vs the oracle (Llama-3-8B linear shapes included) -------------
SHAPES = [(1024, 4096), (4096, 14336), (14336, 4096)]


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('bit,sym,gran,g', [(4, True, 'per_group', 128),
                                             (4, False, 'per_group', 128),
                                             (8, True, 'per_channel', None)])
def test_random_vs_oracle(dev, shape, bit, sym, gran, g):
    from lightcompress_amd.quant import IntegerQuantizer
    gen = torch.Generator().manual_seed(hash((shape, bit, sym)) & 0xffff)
    w = (torch.randn(*shape, generator=gen) * 0.02).to(torch.bfloat16)
    kw = {'group_size': g} if g else {}
    wq = IntegerQuantizer(bit, sym, gran, **kw)
    fq_ref, _, _ = Q.fake_quant_dynamic(w, bit, sym, gran, g)
    codes_ref, s_ref, z_ref = Q.real_quant_dynamic(w, bit, sym, gran, g)
    wd = w.to(dev)
    assert_bit_equal(wq.fake_quant_weight_dynamic(wd), fq_ref, 'fq')
    codes, s, z = wq.real_quant_weight_dynamic(wd)
    assert_bit_equal(codes, codes_ref, 'codes')
    assert_bit_equal(s, s_ref, 'scales')
    if not sym:
        assert_bit_equal(z, z_ref, 'zeros')
    if bit in (4, 8):
        from lightcompress_amd import ops
        r = ops.int_quant_dynamic(wd.reshape(-1, shape[1]), g or shape[1],
                                  int(wq.qmin), int(wq.qmax), sym, fq=False, pack_bits=bit)
        assert np.array_equal(r['packed'].cpu().numpy(), Q.pack_vllm(codes_ref, bit))


@pytest.mark.parametrize('bit,sym,gran,g', [(4, True, 'per_group', 128),
                                             (4, False, 'per_group', 128),
                                             (3, False, 'per_group', 64),
                                             (8, True, 'per_channel', None)])
def test_every_bf16_value_vs_oracle(dev, bit, sym, gran, g):
    """Every finite bf16 bit pattern (subnormals, signed zeros, extremes), shuffled into
    groups so each group's scale differs: the kernels' Markstein quotient (div_mk) and
    hardware bf16 rounding must equal torch-CPU's IEEE x / s and RNE bit for bit."""
    from lightcompress_amd.quant import IntegerQuantizer
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    fin = allb[torch.isfinite(allb.float())]
    gen = torch.Generator().manual_seed(bit * 10 + int(sym))
    # magnitudes grouped by exponent band so groups keep a mix of scales and tiny values
    w = fin[torch.randperm(fin.numel(), generator=gen)]
    w = w[: (w.numel() // 1024) * 1024].reshape(-1, 1024)
    kw = {'group_size': g} if g else {}
    wq = IntegerQuantizer(bit, sym, gran, **kw)
    fq_ref, _, _ = Q.fake_quant_dynamic(w, bit, sym, gran, g)
    codes_ref, s_ref, z_ref = Q.real_quant_dynamic(w, bit, sym, gran, g)
    wd = w.to(dev)
    assert_bit_equal(wq.fake_quant_weight_dynamic(wd), fq_ref, 'fq')
    codes, s, z = wq.real_quant_weight_dynamic(wd)
    assert_bit_equal(codes, codes_ref, 'codes')
    assert_bit_equal(s, s_ref, 'scales')
    # small-magnitude rows: every value of a group within a few binades of the others
    small = fin[(fin.float().abs() < 1e-30)]
    small = small[: (small.numel() // 1024) * 1024].reshape(-1, 1024)
    fq_ref, _, _ = Q.fake_quant_dynamic(small, bit, sym, gran, g)
    assert_bit_equal(wq.fake_quant_weight_dynamic(small.to(dev)), fq_ref, 'fq small')


@pytest.mark.parametrize('name', F.names('mse_'))
def test_mse_qparams_vs_reference(dev, name):
    """calib_algo 'mse' (quant.py:145-203) on the device: the searched ranges and fp32 qparams
    equal the reference's for >= 99 % of the groups (the rest are near ties of the error sums,
    whose order and powf rounding differ: T2), and the fake / real quant outputs follow."""
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, gs, bnum = c['meta'].tolist()
    gran = 'per_group' if gs else 'per_channel'
    kw = dict(calib_algo='mse', mse_b_num=bnum)
    if gs:
        kw['group_size'] = gs
    q = IntegerQuantizer(bit, bool(sym), gran, **kw)
    w = c['w'].to(dev)
    mn, mx = q.get_mse_range(q.reshape_tensor(w))
    same = ((mn.cpu() == c['rmin']) & (mx.cpu() == c['rmax'])).float().mean().item()
    assert same >= 0.99, same
    _, s, z, _, _ = q.get_tensor_qparams(w)
    assert s.dtype == torch.float32 and s.shape == c['scales'].shape
    assert (s.cpu() == c['scales']).float().mean().item() >= 0.99
    fq = q.fake_quant_weight_dynamic(w).cpu()
    assert fq.dtype == c['fq'].dtype
    assert (fq == c['fq']).float().mean().item() >= 0.99
    codes, _, _ = q.real_quant_weight_dynamic(w)
    assert (codes.cpu().to(torch.int32) == c['codes'].to(torch.int32)).float().mean().item() >= 0.99


def _hqq_quantizer(c):
    from lightcompress_amd.quant import IntegerQuantizer
    bit, sym, gs, rzp, hqq, iters = c['meta'].tolist()
    lp, beta = c['hqq'].tolist()
    kw = dict(calib_algo='hqq' if hqq else 'minmax', round_zp=bool(rzp))
    if hqq:
        kw.update(lp_norm=lp, beta=beta, iters=iters)
    if gs:
        kw['group_size'] = gs
    return IntegerQuantizer(bit, bool(sym), 'per_group' if gs else 'per_channel', **kw), bool(hqq)


@pytest.mark.parametrize('name', F.names('nozp_'))
def test_round_zp_false_vs_reference(dev, name):
    """round_zp False (quant.py:545-559, 701-707, 937-941): float zeros qmin - min / s,
    quant round(x / s.clamp_min(1e-9) + z): qparams, fake quant and codes bit-exact, zeros of
    the real quant kept float."""
    c = F.load(name)
    q, _ = _hqq_quantizer(c)
    w = c['w'].to(dev)
    _, s, z, _, _ = q.get_tensor_qparams(w)
    assert_bit_equal(s.cpu(), c['scales'], 'scales')
    assert_bit_equal(z.cpu(), c['zeros'], 'zeros')
    assert_bit_equal(q.fake_quant_weight_dynamic(w).cpu(), c['fq'], 'fq')
    codes, _, zr = q.real_quant_weight_dynamic(w)
    assert torch.equal(codes.cpu().to(torch.int32), c['codes'].to(torch.int32))
    assert_bit_equal(zr.cpu(), c['zeros_rq'], 'real-quant zeros')


@pytest.mark.parametrize('name', F.names('hqq_'))
def test_hqq_vs_reference(dev, name):
    """calib_algo hqq (optimize_weights_proximal, quant.py:588-610) on the device: scales
    (1 / (1 / s) of the minmax qparams) bit-exact, zeros (per-group means of the last step)
    within fp32 summation-order noise for >= 97 % of the groups (a code flipped at a tie moves
    a mean by 1 / group), fake quant and codes >= 99 % equal (T2: the group means and the global error
    mean sum in a different order than torch-CPU)."""
    c = F.load(name)
    q, _ = _hqq_quantizer(c)
    w = c['w'].to(dev)
    _, s, z, _, _ = q.get_tensor_qparams(w)
    assert_bit_equal(s.cpu(), c['scales'], 'scales')
    # a zero is a mean over the group: one code flipped at a rounding tie (the running zero
    # differs in its last bits) moves it by 1 / group -- allowed for a few groups
    zc, zr = z.cpu().reshape(-1), c['zeros'].reshape(-1)
    gsz = w.numel() // zr.numel()
    close = ((zc - zr).abs() <= 1e-5 + 1e-5 * zr.abs()).float().mean().item()
    assert close >= 0.97, close
    assert (zc - zr).abs().max().item() <= 2.0 / gsz + 1e-5
    # elements of a group whose zero moved may round the other way: >= 99 % equal overall
    # (per_channel cases have ~100 groups, so one moved zero is ~1 % of the tensor)
    fq = q.fake_quant_weight_dynamic(w).cpu()
    assert fq.dtype == c['fq'].dtype
    assert (fq == c['fq']).float().mean().item() >= 0.99
    codes, _, _ = q.real_quant_weight_dynamic(w)
    assert (codes.cpu().to(torch.int32) == c['codes'].to(torch.int32)).float().mean().item() \
        >= 0.99


def test_hqq_state_and_early_stop(dev):
    """The device loop stops where the oracle's does: iteration count and best error."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(5)
    w = (torch.randn(512, 256, generator=g) * 0.02)
    t = w.reshape(-1, 128)
    qmin, qmax = Q.int_range(4, False)
    mn, mx = Q.minmax(t)
    s0, z0 = Q.qparams(mn, mx, qmin, qmax, False)
    for iters in (0, 1, 3, 20):
        s_ref, z_ref = Q.hqq_proximal(t.clone(), s0, z0, qmin, qmax, iters=iters)
        s, z, st = ops.hqq_proximal(t.to(dev), 128, s0.to(dev), z0.to(dev), 0, 15, 0.7, 10.0,
                                    iters)
        assert torch.equal(s.cpu(), s_ref.reshape(-1))
        d = (z.cpu() - z_ref.reshape(-1)).abs()
        assert (d <= 1e-6 + 1e-5 * z_ref.abs().reshape(-1)).float().mean().item() >= 0.99
        assert d.max().item() <= 2.0 / 128 + 1e-6  # a code flipped at a tie: 1 / group
        assert int(st[2]) <= iters
