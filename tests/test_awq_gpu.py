"""GPU parity for the AWQ / auto-clip kernels and the device scale search (tier T3 of
SURVEY.md §8c: bit-exact building blocks; chosen ratio + scales equal to the reference on the
golden subsets; clip argmins equal)."""
import pytest
import torch

import fixtures as F
from awq_helpers import SUBSETS, build_layer, forward_fn
from oracle import awq_ref as A
from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu


def bits(t):
    return t.detach().cpu().view(torch.int16)


def test_awq_scales_exhaustive_pow(dev):
    """Every positive normal bf16 in [2^-12, 2^8) x 20 ratios: device == torch-CPU."""
    from lightcompress_amd import ops
    u = torch.arange(0x3980, 0x4380, dtype=torch.int32).to(torch.int16)
    xm = u.view(torch.bfloat16).clone()
    xd = xm.to(dev)
    for n in range(20):
        r = n / 20
        exp = A.scales_v2(xm, r)
        got = ops.awq_scales(xd, r)
        assert torch.equal(bits(got), bits(exp)), f'ratio {r}'


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_awq_scales_random(dev, seed):
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(seed)
    xm = torch.exp(torch.randn(4096, generator=g) * 2).to(torch.bfloat16)
    xm[:3] = 0  # pow(0, r) and the clamp(1e-4) floor
    for n in range(20):
        assert torch.equal(bits(ops.awq_scales(xm.to(dev), n / 20)), bits(A.scales_v2(xm, n / 20)))


@pytest.mark.parametrize('n,c', [(128, 256), (4096, 4096), (1000, 1024), (65536, 512),
                                 (70001, 128), (3, 64)])
def test_absmean(dev, n, c):
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(n)
    x = (torch.randn(n, c, generator=g) * torch.exp(torch.randn(c, generator=g))).to(torch.bfloat16)
    got = ops.absmean_cols(x.to(dev)).cpu()
    exp = A.act_scale(x)
    # torch-CPU's fp32 cascade summation order reproduced: bit-equal
    assert torch.equal(bits(got), bits(exp))


def test_scale_bcast(dev):
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 512, generator=g).to(torch.bfloat16)
    sc = torch.exp(torch.randn(512, generator=g)).to(torch.bfloat16)
    sr = torch.exp(torch.randn(64, generator=g)).to(torch.bfloat16)
    xd = x.to(dev)
    assert torch.equal(bits(ops.scale_bcast(xd, sc.to(dev), 'div')), bits(x / sc.view(1, -1)))
    assert torch.equal(bits(ops.scale_bcast(xd, sc.to(dev), 'mul')), bits(x * sc.view(1, -1)))
    assert torch.equal(bits(ops.scale_bcast(xd, sr.to(dev), 'div', axis=1)),
                       bits(x / sr.view(-1, 1)))
    y = xd.clone()
    ops.scale_bcast(y, sc.to(dev), 'mul', out=y)
    assert torch.equal(bits(y), bits(x * sc.view(1, -1)))


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16, torch.float32])
def test_scale_bcast_rows_every_value(dev, dt):
    """The division's fast path (Markstein quotient from RN(1/s), IEEE fallback off the normal
    range) equals torch's x / s on every bf16 value (incl. subnormals, +-inf, NaN, +-0)
    against scales from 1e-30 to 1e30, per row (axis 1) and per column, 100 rows (not a
    multiple of the 32-row block)."""
    from lightcompress_amd import ops
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    x = allb.to(dt).reshape(-1, 512)[:100]
    g = torch.Generator().manual_seed(5)
    sc = torch.exp(torch.randn(512, generator=g) * 6)
    sc[:4] = torch.tensor([1e-30, 1e30, 3e-39, 1.0])
    sc = sc.to(dt)
    sc = torch.where(sc == 0, torch.ones_like(sc), sc)
    got = ops.scale_bcast(x.to(dev), sc.to(dev), 'div').cpu()
    ref = x / sc.view(1, -1)
    assert torch.equal(got.isnan(), ref.isnan())
    ok = ~ref.isnan()
    assert torch.equal(got[ok], ref[ok])
    sr = sc[:100]
    got = ops.scale_bcast(x.to(dev), sr.to(dev), 'div', axis=1).cpu()
    ref = x / sr.view(-1, 1)
    ok = ~ref.isnan()
    assert torch.equal(got[ok], ref[ok]) and torch.equal(got.isnan(), ref.isnan())


def test_sq_diff_mean(dev):
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(4)
    a = torch.randn(32, 64, 256, generator=g).to(torch.bfloat16)
    b = (a.float() + torch.randn(a.shape, generator=g) * 0.01).to(torch.bfloat16)
    got = ops.sq_diff_mean(a.to(dev), b.to(dev))
    exp = A.loss(a, b)
    assert abs(got - exp) <= 1e-6 * abs(exp)


@pytest.mark.parametrize('name', F.names('clip_'))
def test_auto_clip_vs_reference(dev, name):
    from lightcompress_amd import ops
    from lightcompress_amd.auto_clip import AutoClipper
    c = F.load(name)
    sym, clip_sym, nst, group, mse = c['meta'].tolist()
    qmin, qmax = (-8, 7) if sym else (0, 15)
    x = AutoClipper.sample_tokens(c['x'].to(dev), nst)
    bmax, bmin = ops.auto_clip_search(c['w'].to(dev), x, group, 10, 20, qmin, qmax, bool(sym),
                                      bool(clip_sym), mse=(80, 100, 2.4) if mse else None)
    assert bmax.dtype == c['w'].dtype
    eq_max = (bits(bmax) == bits(c['best_max'])).float().mean().item()
    eq_min = (bits(bmin) == bits(c['best_min'])).float().mean().item()
    if mse:
        # the range search's |d|^2.4 sums: device powf and a fixed pair order vs the
        # reference's vectorised powf and row-sum order -> near-tie range choices (T2)
        assert eq_max >= 0.98 and eq_min >= 0.98, (eq_max, eq_min)
        return
    assert eq_max == 1.0 and eq_min == 1.0, (eq_max, eq_min)
    w = c['w'].to(dev).clone()
    ops.clip_apply(w, group, bmax.reshape(-1), None if clip_sym else bmin.reshape(-1), out=w)
    assert torch.equal(bits(w), bits(c['w_clipped']))


@pytest.mark.parametrize('variant', [3, 2, 1])
@pytest.mark.parametrize('oc,ic,T,dt,sym,clip_sym,small_ws', [
    (1024, 4096, 512, torch.bfloat16, True, True, False),     # v_proj, the AWQ headline
    (100, 384, 300, torch.bfloat16, False, False, True),      # ragged rows / tokens
    (77, 256, 40, torch.float16, True, False, False),         # fp16, fewer tokens than a wave
    (400, 512, 512, torch.bfloat16, False, True, True)])      # 3 row chunks
def test_auto_clip_scalar_operand_matches_pair_kernel(dev, monkeypatch, variant, oc, ic, T, dt,
                                                      sym, clip_sym, small_ws):
    """lcq_auto_clip_search_ws (the candidate table + the row-lane kernel with the tokens as
    scalar operands, the token-lane kernel with the candidates as scalar operands, or the
    token-lane kernel with the candidates staged in LDS, k_auto_clip_tw) is
    bit-identical to k_auto_clip (lcq_auto_clip_search_act) -- the same products, 8-way
    partial sums, halving tree and token-order error sums -- including ragged tokens and rows,
    fp16, and row chunks of a small workspace."""
    from lightcompress_amd import _native as N
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(oc + ic + T)
    w = (torch.randn(oc, ic, generator=g, device=dev) * 0.02).to(dt)
    x = (torch.randn(T, ic, generator=g, device=dev) *
         torch.exp(torch.randn(ic, generator=g, device=dev))).to(dt)
    if dt == torch.float16:
        x = (x.float() * 1e-3).to(dt)
    qmin, qmax = (-8, 7) if sym else (0, 15)
    monkeypatch.setattr(ops, 'CLIP_TOKEN_LANE', False)
    ref = ops.auto_clip_search(w, x, 128, 10, 20, qmin, qmax, sym, clip_sym)
    monkeypatch.setattr(ops, 'CLIP_TOKEN_LANE', True)
    lib = N.load()
    assert lib.lcq_auto_clip_force_variant(variant) == 0
    try:
        if not small_ws:
            got = ops.auto_clip_search(w, x, 128, 10, 20, qmin, qmax, sym, clip_sym)
        else:   # a 192-row table: several chunks
            per = int(lib.lcq_auto_clip_workspace_bytes(1, ic, T, 128, 10))
            assert per > 0
            ws = torch.empty(per, dtype=torch.uint8, device=dev)
            factors = torch.tensor([1 - i / 20 for i in range(10)], dtype=torch.float32,
                                   device=dev)
            ng = ic // 128
            got = (torch.empty((oc, ng, 1), dtype=dt, device=dev),
                   torch.empty((oc, ng, 1), dtype=dt, device=dev))
            N.call('lcq_auto_clip_search_ws', w.data_ptr(), x.data_ptr(), None, N.dt(w), oc, ic,
                   T, 128, 10, factors.data_ptr(), qmin, qmax, int(sym), int(clip_sym), 0, None,
                   0.0, got[0].data_ptr(), got[1].data_ptr(), ws.data_ptr(), per,
                   N.stream_of(w))
    finally:
        lib.lcq_auto_clip_force_variant(0)
    for a, b in zip(got, ref):
        assert torch.equal(bits(a), bits(b))


@pytest.mark.parametrize('subset', ['qkv', 'mlp', 'down'])
@pytest.mark.parametrize('sym', [True, False])
@pytest.mark.parametrize('version', ['v2', 'v1'])
def test_search_scale_vs_reference(dev, subset, sym, version):
    """Device search on the HF module (GPU GEMMs / SDPA): same chosen ratio and bit-equal
    scales as the reference CPU run; losses agree to the bf16-output level. v1 adds the
    weight-scale term (get_weight_scale, bit-equal to the reference's)."""
    from lightcompress_amd.awq import Awq
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(f'awq_{subset}_{"sym" if sym else "asym"}' + ('_v1' if version == 'v1' else ''))
    cfg, layer, kwargs = build_layer(dev)
    names, inspect_name, has_kw = SUBSETS[subset]
    obj = Awq.__new__(Awq)
    obj.wquantizer = IntegerQuantizer(4, sym, 'per_group', group_size=128)
    obj.awq_bs, obj.w_only, obj.n_grid = None, True, 20
    obj.trans_version = version
    layers = {n: layer.get_submodule(n) for n in names}
    if version == 'v1':
        assert torch.equal(bits(obj.get_weight_scale(layers).cpu()), bits(c['w_max']))
    inspect = layer.get_submodule(inspect_name)
    best = obj.search_scale_subset(None, layers, [c['x'].to(dev)], inspect, False,
                                   [kwargs] if has_kw else {})
    ref_losses = c['losses'].tolist()
    ref_best = min(range(20), key=lambda i: (ref_losses[i], i))
    assert obj.last_search['best_index'] == ref_best
    assert torch.equal(bits(best), bits(c['scales']))
    got = torch.tensor(obj.last_search['losses'], dtype=torch.float64)
    assert torch.allclose(got, c['losses'], rtol=5e-2, atol=1e-9)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16, torch.float32])
def test_scale_bcast_every_value(dev, dt):
    """x / s and x * s per column for every finite bf16 value against up to 64 scales from
    1e-30 to 1e30: bit-equal to torch-CPU, including subnormal, zero and overflowing results."""
    from lightcompress_amd import ops
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    fin = allb[torch.isfinite(allb.float())]
    x = fin[: (fin.numel() // 64) * 64].reshape(-1, 64).to(dt)
    g = torch.Generator().manual_seed(9)
    s = torch.cat([torch.logspace(-30, 30, 32), torch.rand(32, generator=g) * 4 + 0.01]).to(dt)
    s = s[torch.isfinite(s.float()) & (s.float() != 0)]
    s = s[: s.numel() // 8 * 8]
    x = x[:, : s.numel()].contiguous()
    for op, ref in (('div', x / s.view(1, -1)), ('mul', x * s.view(1, -1))):
        got = ops.scale_bcast(x.to(dev), s.to(dev), op).cpu()
        same = (got.view(torch.int16 if dt != torch.float32 else torch.int32) ==
                ref.view(torch.int16 if dt != torch.float32 else torch.int32))
        same |= got.isnan() & ref.isnan()
        assert bool(same.all()), (op, int((~same).sum()))


@pytest.mark.parametrize('rows,cols,group,nl', [(4096, 4096, 128, 3), (14336, 4096, 128, 2),
                                                (4096, 14336, 128, 1), (300, 512, 64, 2),
                                                (1000, 256, 32, 1)])
def test_awq_weight_scale_vs_oracle(dev, rows, cols, group, nl):
    """get_weight_scale (trans_version v1) at Llama-3-8B shapes: bit-equal to torch-CPU."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(rows + cols)
    ws = [(torch.randn(rows, cols, generator=g) * 0.02).to(torch.bfloat16) for _ in range(nl)]
    got = ops.awq_weight_scale([w.to(dev) for w in ws], group).cpu()
    assert torch.equal(bits(got), bits(A.weight_scale(ws, group)))


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
def test_scale_bcast_cols_every_x_every_scale(dev, dt):
    """x / s and x * s per column at an AWQ-like width: every finite bf16 x in every column
    against 1024 scales covering every bf16 mantissa across exponents -16..15 (plus tiny and
    huge scales), bit-equal to torch-CPU's x / s and x * s."""
    from lightcompress_amd import ops
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    fin = allb[torch.isfinite(allb.float())]
    mant = torch.arange(128, dtype=torch.int32)
    exps = torch.arange(127 - 16, 127 + 16, dtype=torch.int32)
    sb = ((exps.view(-1, 1) << 7) | mant.view(1, -1)).reshape(-1)[::4]  # 1024 positive bf16
    s = sb.to(torch.int16).view(torch.bfloat16)
    s[:4] = torch.tensor([1e-35, 3e-30, 1e30, 3e35]).to(torch.bfloat16)
    s = s.to(dt)
    s = torch.where(torch.isfinite(s.float()) & (s.float() != 0), s, torch.ones_like(s))
    nc = s.numel()
    idx = (torch.arange(fin.numel()).view(-1, 1) + torch.arange(nc).view(1, -1) * 37) % fin.numel()
    x = fin[idx].to(dt)
    ib = torch.int16
    for op, ref in (('div', x / s.view(1, -1)), ('mul', x * s.view(1, -1))):
        got = ops.scale_bcast(x.to(dev), s.to(dev), op).cpu()
        same = got.view(ib) == ref.view(ib)
        same |= got.isnan() & ref.isnan()
        assert bool(same.all()), (op, int((~same).sum()))
    # a 4096-wide layout (512 threads' worth of columns per row: two workgroups per row span)
    x4 = x[:4096].reshape(-1, 4096)[:, :4096].contiguous()
    s4 = s.repeat(4)
    ref = x4 / s4.view(1, -1)
    got = ops.scale_bcast(x4.to(dev), s4.to(dev), 'div').cpu()
    assert torch.equal(got.view(ib), ref.view(ib))


@pytest.mark.parametrize('name', F.names('clipact_'))
def test_auto_clip_pc_act_vs_reference(dev, name):
    """AutoClipper.auto_clip_layer through the plugin class for per_channel weights
    (lcq_auto_clip_search_pc) and with activation fake-quant (w_only False), against the
    reference's own bounds. Per-group with act: exact emulation, bit-equal. Per-channel: the
    ic-long fp32 sums run in k order instead of torch-CPU's cascade, so a cur/org output can
    round to the neighbouring bf16 value and move a near-tie step choice (T2)."""
    from lightcompress_amd.auto_clip import AutoClipper
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    wb, sym, clip_sym, nst, grp, abit, asym = c['meta'].tolist()
    gran = 'per_channel' if grp == -1 else 'per_group'
    kw = {'group_size': grp} if grp != -1 else {}
    wq = IntegerQuantizer(wb, bool(sym), gran, **kw)
    aq = IntegerQuantizer(abit, bool(asym), 'per_token') if abit else None
    clipper = AutoClipper(w_only=not abit, wquantizer=wq, aquantizer=aq, clip_version='v1',
                          clip_sym=bool(clip_sym), save_clip=False, padding_mask=None)
    bmax, bmin = clipper.auto_clip_layer(0, 'l', c['w'].to(dev), [c['x'].to(dev)],
                                         n_sample_token=nst)
    assert bmax.shape == c['best_max'].shape
    eq_max = (bits(bmax.cpu()) == bits(c['best_max'])).float().mean().item()
    eq_min = (bits(bmin.cpu()) == bits(c['best_min'])).float().mean().item()
    if grp != -1:
        assert eq_max == 1.0 and eq_min == 1.0, (eq_max, eq_min)
    else:
        assert eq_max >= 0.97 and eq_min >= 0.97, (eq_max, eq_min)


def test_auto_clip_pc_llama_shape(dev):
    """per_channel w8a8 clip at a Llama-3-8B o_proj shape (4096 x 4096, 512 sampled tokens)
    against the oracle on 64 rows: bounds equal on >= 97 % of the rows, and every chosen
    bound is one of the shrink grid's values of its row."""
    from lightcompress_amd import ops
    from oracle import awq_ref as A
    from oracle import quant_ref as Q
    g = torch.Generator().manual_seed(11)
    oc, ic, T = 4096, 4096, 512
    w = (torch.randn(oc, ic, generator=g) * 0.02).to(torch.bfloat16)
    mag = torch.exp(torch.randn(ic, generator=g))
    x = (torch.randn(T, ic, generator=g) * mag).to(torch.bfloat16)
    qx = Q.fake_quant_dynamic(x, 8, True, 'per_token')[0]
    bmax, bmin = ops.auto_clip_search(w.to(dev), x.to(dev), ic, 10, 20, -128, 127, True, True,
                                      qx=qx.to(dev))
    rows = torch.arange(0, oc, oc // 64)
    emax, emin = A.clip_layer(w[rows], x, 8, True, ic, True, n_sample_token=T, act=(8, True))
    eq = (bits(bmax.cpu()[rows]) == bits(emax)).float().mean().item()
    assert eq >= 0.97, eq
    am = w.float().abs().amax(dim=1)
    grid = torch.stack([(am * (1 - i / 20)).to(torch.bfloat16).float() for i in range(10)], 1)
    assert bool((grid == bmax.cpu().float().view(-1, 1)).any(dim=1).all())
    assert torch.equal(bits(bmin), bits(-bmax))
