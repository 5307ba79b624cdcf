"""Pin the clip_version v2 restatement (oracle/awq_ref.py clip_layer(version=2), clip_factors;
oracle/quant_ref.py fake_quant_learnable) against the reference's own outputs
(tests/golden/gen_golden.py gen_clip_v2: AutoClipper(clip_version='v2') with
IntegerQuantizer(calib_algo='learnable'), the awq_comb_omni w6a6 / w8a8 step_1_awq.yml
settings and variants). CPU, bit-exact. Also the host-side rules of the learnable quantizer."""
import pytest
import torch

import fixtures as F
from oracle import awq_ref as A
from oracle import quant_ref as Q


def _case(c):
    wb, sym, cs, nst, ab, asy = c['meta'].tolist()
    return wb, bool(sym), bool(cs), nst, ((ab, bool(asy)) if ab else None)


@pytest.mark.parametrize('name', F.names('clipv2_'))
def test_clip_v2_oracle_matches_reference(name):
    c = F.load(name)
    wb, sym, cs, nst, act = _case(c)
    ic = c['w'].shape[1]
    bmax, bmin = A.clip_layer(c['w'], c['x'], wb, sym, ic, cs, n_sample_token=nst, act=act,
                              version=2)
    assert torch.equal(bmax, c['best_max']) and torch.equal(bmin, c['best_min'])
    up, low = A.clip_factors(c['w'], c['best_max'], c['best_min'], cs, ic)
    assert torch.equal(up, c['up'])
    assert (low is None) == ('low' not in c)
    if low is not None:
        assert torch.equal(low, c['low'])
    fq = Q.fake_quant_learnable(c['w'], wb, sym, 'per_channel', low=c.get('low'), up=c['up'])
    assert torch.equal(fq, c['fq'])


def test_learnable_quantizer_factor_rules():
    """calib_algo learnable reads the factors (sym: up; asym: both, else plain min/max); every
    other calib_algo ignores them (quant.py:122-130); v2 factors on float quantizers or with
    round_zp False are refused."""
    from lightcompress_amd.quant import FloatQuantizer, IntegerQuantizer
    up, low = torch.zeros(4, 1), torch.ones(4, 1)
    args = {'upbound_factor': up, 'lowbound_factor': low}
    a = IntegerQuantizer(8, False, 'per_channel', calib_algo='learnable')
    assert a._factors(args)[0] is up and a._factors(args)[1] is low
    assert a._factors({'upbound_factor': up, 'lowbound_factor': None}) is None
    s = IntegerQuantizer(4, True, 'per_channel', calib_algo='learnable')
    assert s._factors({'upbound_factor': up, 'lowbound_factor': None}) == (up, None)
    assert IntegerQuantizer(4, False, 'per_channel')._factors(args) is None
    with pytest.raises(NotImplementedError):
        IntegerQuantizer(4, False, 'per_channel', calib_algo='learnable',
                         round_zp=False)._check_supported(args)
    with pytest.raises(NotImplementedError):
        FloatQuantizer('e4m3', True, 'per_channel', calib_algo='learnable',
                       use_qtorch=True)._check_supported({'upbound_factor': up})


def test_clip_version_rules():
    from lightcompress_amd.auto_clip import AutoClipper
    from lightcompress_amd.quant import IntegerQuantizer
    wq = IntegerQuantizer(8, False, 'per_group', group_size=128, calib_algo='learnable')
    with pytest.raises(Exception):
        AutoClipper(True, wq, None, 'v3', False, False, None)
    c = AutoClipper(True, wq, None, 'v2', False, False, None)
    with pytest.raises(NotImplementedError):  # every reference v2 config is per_channel
        c.auto_clip_layer(0, 'l', torch.zeros(128, 256, dtype=torch.bfloat16),
                          [torch.zeros(64, 256, dtype=torch.bfloat16)])
