"""GPU parity for clip_version v2 (learnable clip factors; combination/awq_comb_omni
w6a6 / w8a8 step_1_awq.yml): the per-channel clip kernel's learnable-range candidates
(lcq_auto_clip_search_pc version 2), get_clip_factor (lcq_clip_factors) and the deployed fake
quant with the factors (lcq_int_quant_learnable), against the reference's own outputs
(tests/golden clipv2_*) and the oracle."""
import pytest
import torch

import fixtures as F
from oracle import awq_ref as A
from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu


def bits(t):
    return t.cpu().view(torch.int16)


def _case(c):
    wb, sym, cs, nst, ab, asy = c['meta'].tolist()
    return wb, bool(sym), bool(cs), nst, ((ab, bool(asy)) if ab else None)


def _quantizers(wb, sym, act):
    from lightcompress_amd.quant import IntegerQuantizer
    wq = IntegerQuantizer(wb, sym, 'per_channel', calib_algo='learnable')
    aq = IntegerQuantizer(act[0], act[1], 'per_token') if act else None
    return wq, aq


@pytest.mark.parametrize('name', F.names('clipv2_'))
def test_auto_clip_v2_vs_reference(dev, name):
    """AutoClipper(clip_version='v2').auto_clip_layer through the plugin class. The ic-long
    fp32 sums run in k order (T2, as the v1 per-channel clip): bounds equal on >= 97 % of the
    rows, the rest on the row's shrink grid."""
    from lightcompress_amd.auto_clip import AutoClipper
    c = F.load(name)
    wb, sym, cs, nst, act = _case(c)
    wq, aq = _quantizers(wb, sym, act)
    clipper = AutoClipper(w_only=aq is None, wquantizer=wq, aquantizer=aq, clip_version='v2',
                          clip_sym=cs, save_clip=True, padding_mask=None)
    bmax, bmin = clipper.auto_clip_layer(0, 'l', c['w'].to(dev), [c['x'].to(dev)],
                                         n_sample_token=nst)
    assert bmax.shape == c['best_max'].shape and bmax.dtype == c['best_max'].dtype
    eq = ((bits(bmax) == bits(c['best_max'])) & (bits(bmin) == bits(c['best_min'])))
    eq = eq.float().mean().item()
    print(f'{name}: rows with equal bounds {eq * 100:.2f} %')
    assert eq >= 0.97, eq
    w = c['w'].float()
    om = w.abs().amax(1) if cs else w.amax(1)
    grid = torch.stack([(om * (1 - i / 20)).to(c['w'].dtype).float() for i in range(10)], 1)
    assert bool((grid == bmax.cpu().float().view(-1, 1)).any(dim=1).all())


@pytest.mark.parametrize('name', F.names('clipv2_'))
def test_clip_factors_and_deploy_bit_exact(dev, name):
    """With the reference's bounds: apply_clip v2 registers the reference's factors
    (buf_upbound_factor / buf_lowbound_factor, None for clip_sym), leaves the weight alone,
    stores them for clips.pth; the deployed fake quant (w_qdq -> fake_quant_weight_dynamic
    with the factors) equals the reference's, bit for bit."""
    from lightcompress_amd.auto_clip import AutoClipper
    from lightcompress_amd.base_blockwise_quantization import BaseBlockwiseQuantization
    c = F.load(name)
    wb, sym, cs, nst, act = _case(c)
    wq, aq = _quantizers(wb, sym, act)
    clipper = AutoClipper(w_only=aq is None, wquantizer=wq, aquantizer=aq, clip_version='v2',
                          clip_sym=cs, save_clip=True, padding_mask=None)
    oc, ic = c['w'].shape
    m = torch.nn.Linear(ic, oc, bias=False).to(c['w'].dtype).to(dev)
    m.weight.data = c['w'].to(dev).clone()
    clipper.apply_clip(0, m, c['best_min'].to(dev), c['best_max'].to(dev), 'l')
    assert torch.equal(bits(m.weight.data), bits(c['w']))
    assert torch.equal(bits(m.buf_upbound_factor), bits(c['up']))
    if 'low' in c:
        assert torch.equal(bits(m.buf_lowbound_factor), bits(c['low']))
    else:
        assert m.buf_lowbound_factor is None
    saved = clipper.weight_clips[0]
    assert torch.equal(bits(saved['l.weight_quantizer.upbound_factor']), bits(c['up']))
    fq = BaseBlockwiseQuantization.w_qdq(None, m, wq)
    assert torch.equal(bits(fq), bits(c['fq']))


@pytest.mark.parametrize('sym', [False, True])
def test_learnable_fake_quant_llama_shape(dev, sym):
    """lcq_int_quant_learnable at a Llama-3-8B down_proj shape (4096 x 14336, per_channel
    rows through the wide-group kernel) and per_group 128 (the lane kernel), random finite
    factors, vs the oracle: bit-exact except where the fp32 sigmoid (expf vs torch-CPU's
    vectorised exp) lands on a bf16 rounding tie -- such a row's scale moves by one bf16 ulp
    (allowed on <= 0.1 % of the rows)."""
    from lightcompress_amd.quant import IntegerQuantizer
    g = torch.Generator().manual_seed(5)
    for gran, oc, ic in (('per_channel', 4096, 14336), ('per_group', 512, 4096)):
        w = (torch.randn(oc, ic, generator=g) * 0.02).to(torch.bfloat16)
        kw = {'group_size': 128} if gran == 'per_group' else {}
        ng = oc * (ic // 128 if gran == 'per_group' else 1)
        up = (torch.randn(ng, 1, generator=g) * 2 + 2).to(torch.bfloat16)
        low = None if sym else (torch.randn(ng, 1, generator=g) * 2 + 2).to(torch.bfloat16)
        wq = IntegerQuantizer(4, sym, gran, calib_algo='learnable', **kw)
        args = {'upbound_factor': up.to(dev),
                'lowbound_factor': None if low is None else low.to(dev)}
        got = wq.fake_quant_weight_dynamic(w.to(dev), args).cpu()
        ref = Q.fake_quant_learnable(w, 4, sym, gran, 128, low=low, up=up)
        gsz = ic if gran == 'per_channel' else 128
        bad = (bits(got) != bits(ref)).reshape(-1, gsz).any(dim=1).float().mean().item()
        print(f'{gran} sym={sym}: groups with any differing element {bad * 100:.4f} %')
        assert bad <= 1e-3, bad
