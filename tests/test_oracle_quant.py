"""Pin the oracle (CPU restatement) against golden vectors produced by the real reference."""
import numpy as np
import pytest
import torch

import fixtures as F
from oracle import quant_ref as Q

QUANT_CASES = [n for n in F.names('quant_int')]


def _eq(a, b):
    assert a.dtype == b.dtype, (a.dtype, b.dtype)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                       b.view(torch.int16) if b.dtype == torch.bfloat16 else b)


@pytest.mark.parametrize('name', QUANT_CASES)
def test_dynamic_quant_matches_reference(name):
    c = F.load(name)
    bit, sym, gs, qmin, qmax = c['meta'].tolist()
    gran = 'per_channel' if 'pc' in name else 'per_group'
    fq, s, z = Q.fake_quant_dynamic(c['w'], bit, bool(sym), gran, gs)
    _eq(fq, c['fq'])
    codes, s2, z2 = Q.real_quant_dynamic(c['w'], bit, bool(sym), gran, gs)
    _eq(codes, c['codes'])
    _eq(s2, c['scales'])
    if sym:
        assert 'zeros' not in c and z2 is None
    else:
        _eq(z2, c['zeros'])
    if 'packed' in c:
        assert np.array_equal(Q.pack_vllm(codes, bit), c['packed'].numpy())


def test_prescale_matches_reference():
    c = F.load('quant_awq_prescale_int4_sym_g128_bf16')
    fq, _, _ = Q.fake_quant_dynamic(c['w'], 4, True, 'per_group', 128, pre_scale=c['pre'])
    _eq(fq, c['fq'])


@pytest.mark.parametrize('sym', [True, False])
def test_clip_matches_reference(sym):
    c = F.load(f'quant_clip_int4_{"sym" if sym else "asym"}_g128_bf16')
    fq, _, _ = Q.fake_quant_dynamic(c['w'], 4, sym, 'per_group', 128, clip_max=c['cmax'],
                                    clip_min=c['cmin'])
    _eq(fq, c['fq'])


def test_static_matches_reference():
    c = F.load('quant_static_int4_asym_g128_f32')
    fq = Q.fake_quant_static(c['w'], c['scales'], c['zeros'], 4, False).to(torch.bfloat16)
    _eq(fq, c['fq_bf16'])
    codes, s, z = Q.real_quant_static(c['w'], c['scales'].to(torch.bfloat16), c['zeros'], 4,
                                      False)
    _eq(codes, c['codes'])
    _eq(s, c['scales_rq'])
    _eq(z, c['zeros_rq'])


@pytest.mark.parametrize('name', F.names('awqpack_'))
def test_gemm_pack_matches_reference(name):
    c = F.load(name)
    qw, s16, qz = Q.gemm_pack_autoawq(c['w'], c['scales'], c['zeros'], 128)
    assert np.array_equal(qw, c['qweight'].numpy())
    _eq(s16, c['scales_t'])
    assert np.array_equal(qz, c['qzeros'].numpy())


def test_gemm_pack_fixture_exercises_out_of_range_codes():
    """The reference's un-clamped re-quantisation produces codes outside [0, 15]; the
    fixture must contain some so the bit-spill behaviour is actually pinned."""
    c = F.load('awqpack_int4_asym_big_g128_bf16')
    w, s, z = c['w'], c['scales'], c['zeros']
    s16 = s.t().to(torch.float16)
    sz = z.t() * s16
    g = torch.arange(w.shape[1]) // 128
    iw = torch.round((w + sz[g].t()) / s16[g].t())
    assert ((iw < 0) | (iw > 15)).sum() > 0


@pytest.mark.parametrize('name', F.names('mse_'))
def test_mse_oracle_matches_reference(name):
    """calib_algo 'mse' range search (quant.py:145-203): the oracle reproduces the reference's
    searched ranges bit for bit (same torch-CPU ops)."""
    c = F.load(name)
    bit, sym, gs, bnum = c['meta'].tolist()
    t = c['w'].reshape(-1, gs) if gs else c['w']
    mn, mx = Q.mse_range(t, bit, bool(sym))
    assert torch.equal(mn, c['rmin']) and torch.equal(mx, c['rmax'])


HQQ_CASES = F.names('hqq_') + F.names('nozp_')


def _hqq_meta(c):
    bit, sym, gs, rzp, hqq, iters = c['meta'].tolist()
    lp, beta = c['hqq'].tolist()
    return bit, bool(sym), gs or None, bool(rzp), bool(hqq), iters, lp, beta


@pytest.mark.parametrize('name', HQQ_CASES)
def test_hqq_and_nozp_oracle_matches_reference(name):
    """calib_algo hqq (quant.py:588-610, 680-689) and round_zp False (quant.py:545-559,
    701-707): qparams and fake quant of the oracle equal the reference's."""
    c = F.load(name)
    bit, sym, gs, rzp, hqq, iters, lp, beta = _hqq_meta(c)
    gran = 'per_group' if gs else 'per_channel'
    if hqq:
        fq, s, z = Q.fake_quant_hqq(c['w'], bit, sym, gran, gs, round_zp=rzp, lp_norm=lp,
                                    beta=beta, iters=iters)
    else:
        fq, s, z = Q.fake_quant_nozp(c['w'], bit, sym, gran, gs)
    assert torch.equal(s, c['scales'])
    if 'zeros' in c:
        assert torch.equal(z, c['zeros'])
    assert torch.equal(fq, c['fq'])
