"""Pin the float-quant (FP8) restatements of auto-clip and the GPTQ column loop against the
reference's own outputs (tests/golden/gen_golden.py gen_fp8_algos: the reference's
AutoClipper / GPTQ methods with FloatQuantizer(use_qtorch=True) and the saturating native-cast
stand-in for qtorch's float_quantize). CPU, bit-exact. Also the guards that keep unsupported
quantizer settings off the device path (pure host logic)."""
import pytest
import torch

import fixtures as F
from oracle import awq_ref as A
from oracle import fp8_ref as P
from oracle import gptq_ref as G

FMT = {4: 'e4m3', 5: 'e5m2'}


def _act_fn(kind, fmt):
    if kind == 0:
        return None
    gran = 'per_token' if kind == 1 else 'per_tensor'
    return lambda x: P.fp8_qdq(x, fmt, gran)[0]


@pytest.mark.parametrize('name', F.names('clipfp8_'))
def test_clip_fp8_oracle_matches_reference(name):
    c = F.load(name)
    e, pt, act, nst = c['meta'].tolist()
    fmt = FMT[e]
    ic = c['w'].shape[1]
    bmax, bmin = A.clip_layer(c['w'], c['x'], None, True, ic, True, n_sample_token=nst,
                              fp8=(fmt, bool(pt), _act_fn(act, fmt)))
    assert torch.equal(bmax, c['best_max']) and torch.equal(bmin, c['best_min'])


@pytest.mark.parametrize('name', F.names('gptqfp8_'))
def test_gptq_fp8_column_loop_matches_reference(name):
    c = F.load(name)
    e, gs, act, oc, ic = c['meta'].tolist()
    fmt = FMT[e]
    W = c['w'].float().clone()
    dead = torch.diag(c['H']) == 0
    W[:, dead] = 0
    if act:
        W = W[:, c['perm']]
    fixed = None if gs else (c['scales'], torch.tensor(0.0))
    tmp, _, s, _ = G.column_loop(W, c['U'], None, True, gs or None, fixed=fixed, fp8=fmt)
    if act:
        tmp = tmp[:, torch.argsort(c['perm'])]
    assert torch.equal(tmp, c['weight'])
    if gs:
        assert torch.equal(s.reshape(-1, 1), c['scales'])


def test_float_quantize_stand_in():
    """Saturating at +-finfo.max, NaN kept, otherwise torch's RNE cast."""
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16).float()
    for fmt, dt in P.FP8.items():
        got = P.float_quantize(allb, fmt)
        m = torch.finfo(dt).max
        fin = allb.abs() <= m
        assert torch.equal(got[fin], allb[fin].to(dt).float())
        big = (~fin) & ~allb.isnan()
        assert torch.equal(got[big], torch.sign(allb[big]) * m)
        assert bool(got[allb.isnan()].isnan().all())


# ---- guards: settings the device kernels do not implement must raise, not run silently -----
def test_gptq_quantizer_guards():
    from lightcompress_amd.gptq_core import check_quantizer
    from lightcompress_amd.quant import FloatQuantizer, IntegerQuantizer
    assert check_quantizer(IntegerQuantizer(4, False, 'per_group', group_size=128)) is None
    fq = FloatQuantizer('e4m3', True, 'per_channel', use_qtorch=True)
    assert check_quantizer(fq) == torch.float8_e4m3fn
    with pytest.raises(NotImplementedError):
        check_quantizer(IntegerQuantizer(4, False, 'per_group', group_size=128, round_zp=False))
    with pytest.raises(NotImplementedError):
        check_quantizer(IntegerQuantizer(4, False, 'per_group', group_size=128,
                                         calib_algo='hqq'))
    with pytest.raises(NotImplementedError):
        check_quantizer(FloatQuantizer('e4m3', True, 'per_channel', use_qtorch=False))
    with pytest.raises(NotImplementedError):
        check_quantizer(fq, static_groups=True)
    with pytest.raises(NotImplementedError):
        check_quantizer(FloatQuantizer('e4m3', True, 'per_tensor', use_qtorch=True))


def test_auto_clip_quantizer_guards():
    from lightcompress_amd.auto_clip import AutoClipper
    from lightcompress_amd.quant import FloatQuantizer
    w = torch.zeros(384, 256)

    def clipper(wq):
        return AutoClipper(True, wq, None, 'v1', True, False, None)
    assert clipper(FloatQuantizer('e4m3', True, 'per_tensor', use_qtorch=True))._float_quant(w) \
        == (torch.float8_e4m3fn, 64)
    assert clipper(FloatQuantizer('e5m2', True, 'per_channel', use_qtorch=True))._float_quant(w) \
        == (torch.float8_e5m2, 0)
    for bad in (FloatQuantizer('e4m3', True, 'per_channel', use_qtorch=False),
                FloatQuantizer('e4m3', True, 'per_group', group_size=128, use_qtorch=True)):
        with pytest.raises(NotImplementedError):
            clipper(bad)._float_quant(w)


def test_row_shard_alignment():
    from lightcompress_amd.parallel import row_shard
    for rows, world, align in ((384, 2, 64), (512, 3, 256), (1000, 4, 1), (64, 4, 64)):
        spans = [row_shard(rows, r, world, align) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == rows
        for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
            assert a1 == b0
        assert all(s0 % align == 0 for s0, _ in spans)


def test_hessian_group_plan():
    """gptq_core.GroupPlan: 8 groups covering every sample once; a world dividing 8 takes
    contiguous power-of-two blocks of them, balanced (the shard GPTQ.sample_shard cuts)."""
    from lightcompress_amd.gptq_core import GroupPlan, group_bounds
    for n in (4, 5, 16, 128, 131):
        b = group_bounds(n)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
        for world in (1, 2, 4, 8):
            plans = [GroupPlan(n, r, world) for r in range(world)]
            assert sum(p.n_local for p in plans) == n
            for r, p in enumerate(plans):
                assert p.first == -(-r * n // world)
                assert len(p.local) == 8 // world
                assert p.local[0][1] == 0 and p.local[-1][2] == p.n_local
