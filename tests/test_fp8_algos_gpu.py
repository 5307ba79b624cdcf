"""GPU parity for float-quant (FP8) weights inside the algorithms (backend/{vllm,sglang}/fp8
awq_fp8*.yml / gptq_fp8.yml): the AWQ search's fake quant of W * s, auto-clip of per_channel /
per_tensor FloatQuantizer weights, and the GPTQ column loop with float_quantize. Checked
against the reference's own outputs (tests/golden clipfp8_ / gptqfp8_, made with the
saturating native-cast stand-in for qtorch's float_quantize) and the oracle."""
import types

import pytest
import torch

import fixtures as F
from oracle import awq_ref as A
from oracle import fp8_ref as P
from oracle import gptq_ref as G

pytestmark = pytest.mark.gpu

FMT = {4: 'e4m3', 5: 'e5m2'}


def bits(t):
    t = t.cpu()
    return t.view(torch.int16) if t.element_size() == 2 else t.view(torch.uint8)


@pytest.mark.parametrize('fmt', ['e4m3', 'e5m2'])
def test_static_fp8_saturating_every_bf16_value(dev, fmt):
    """lcq_fp8_quant_static(saturate=1): codes and fake quant equal the float_quantize
    stand-in on every bf16 value (in range, in c10's overflow band, beyond it, +-inf)."""
    from lightcompress_amd import ops
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    allb = allb[~allb.float().isnan()]
    allb = torch.cat([allb, allb.new_zeros((-allb.numel()) % 8)]).reshape(-1, 8)
    s = torch.tensor([0.75], dtype=torch.float32)
    r = ops.fp8_quant_static(allb.to(dev), s.to(dev), P.FP8[fmt], ct_dtype=torch.float32,
                             add_zero=True, fq=True, fq_dtype=torch.float32, saturate=True)
    q = P.float_quantize(allb.float() / s + torch.tensor(0.0), fmt)
    assert torch.equal(r['codes'].cpu().float(), q)
    assert torch.equal(r['fq'].cpu(), q * s)


@pytest.mark.parametrize('group', [None, 128, 64])
@pytest.mark.parametrize('fmt', ['e4m3', 'e5m2'])
def test_gptq_fp8_single_block_bit_exact(dev, group, fmt):
    """One 128-column block (no trailing GEMM): the float-quant column kernel equals the
    oracle bit for bit (weights, losses, group scales). Static per-row scales from a smaller
    absmax make compensated columns overflow the format: the saturating cast is exercised."""
    from lightcompress_amd import gptq_core
    g = torch.Generator().manual_seed(7 + (group or 0))
    rows, cols = 300, 128
    W = torch.randn(rows, cols, generator=g) * 0.02
    Am = torch.randn(cols, 2 * cols, generator=g)
    Hm = Am @ Am.t() / cols + 0.1 * torch.eye(cols)
    U = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(Hm)), upper=True)
    fixed = None
    if group is None:
        s = (W.abs().amax(1, keepdim=True) * 0.9).to(torch.bfloat16)
        s = (s / P.qmax_of(fmt)).to(torch.bfloat16)
        fixed = (s, torch.tensor(0.0))
    tmp, L, so, _ = G.column_loop(W.clone(), U, None, True, group, fixed=fixed, fp8=fmt)
    Wd = W.clone().to(dev)
    qmax = int(P.qmax_of(fmt))
    s_d, _, L_d = gptq_core.column_loop(Wd, U.to(dev), None, True, group, -qmax, qmax,
                                        fixed=None if fixed is None else
                                        (fixed[0].to(dev), None),
                                        losses=True, fp8=P.FP8[fmt])
    assert torch.equal(Wd.cpu(), tmp)
    assert torch.equal(L_d.cpu(), L)
    if group:
        assert torch.equal(s_d.cpu(), so)


def _layer_case(c):
    e, gs, act, oc, ic = c['meta'].tolist()
    return FMT[e], gs or None, bool(act)


@pytest.mark.parametrize('name', F.names('gptqfp8_'))
def test_gptq_fp8_layer_vs_reference(dev, name):
    """gptq_core.quantize_layer with the reference's U / perm (T2: only the trailing fp32
    GEMM's summation order differs): compensated weights within 1e-4, and the deployed fake
    quant (FloatQuantizer.fake_quant_weight_static, gptq.py:424-452) / real-quant codes
    (gptq.py:411-422) >= 99.9 % bit-equal."""
    from lightcompress_amd import gptq_core
    from lightcompress_amd.quant import FloatQuantizer
    c = F.load(name)
    fmt, gs, act = _layer_case(c)
    gran = 'per_group' if gs else 'per_channel'
    wq = FloatQuantizer(fmt, True, gran, use_qtorch=True, **({'group_size': gs} if gs else {}))
    dead = torch.diag(c['H']) == 0
    perm = c['perm'].to(dev) if act else None
    prepared = (c['U'].to(dev), perm, dead.to(dev))
    fixed = None if gs else (c['scales'].to(dev), None)
    r = gptq_core.quantize_layer(c['w'].to(dev), None, wq, actorder=act, fixed=fixed,
                                 prepared=prepared)
    torch.testing.assert_close(r['weight'].cpu(), c['weight'], rtol=1e-4, atol=1e-6)
    if gs:
        torch.testing.assert_close(r['scales'].cpu(), c['scales'], rtol=1e-5, atol=1e-9)
    scales = r['scales'] if gs else c['scales'].to(dev)
    w = r['weight'][:, perm] if (act and gs) else r['weight']
    fq = wq.fake_quant_weight_static(w.contiguous(), {'scales': scales.clone(),
                                                      'zeros': torch.tensor(0.0)})
    fq = fq.to(torch.bfloat16)
    if act and gs:
        fq = fq[:, torch.argsort(perm)]
    eq = (bits(fq) == bits(c['fq'])).float().mean().item()
    assert eq >= 0.999, eq
    if 'codes' in c:
        codes, s_rq, _ = wq.real_quant_weight_static(
            r['weight'].contiguous(), {'scales': c['scales'].to(dev).to(torch.bfloat16),
                                       'zeros': torch.tensor(0.0)})
        assert codes.dtype == c['codes'].dtype
        assert (bits(codes) == bits(c['codes'])).float().mean().item() >= 0.999
        assert torch.equal(s_rq.cpu(), c['scales_rq'])


@pytest.mark.parametrize('name', F.names('clipfp8_'))
def test_auto_clip_fp8_vs_reference(dev, name):
    """AutoClipper.auto_clip_layer through the plugin class for FloatQuantizer weights
    (per_channel; per_tensor with one scale per 256- or 64-row batch) with and without the
    activation fake quant. The ic-long fp32 sums run in k order (T2, as the integer
    per-channel clip): bounds equal on >= 97 % of the rows, the rest on the row's shrink grid."""
    from lightcompress_amd.auto_clip import AutoClipper
    from lightcompress_amd.quant import FloatQuantizer
    c = F.load(name)
    e, pt, act, nst = c['meta'].tolist()
    fmt = FMT[e]
    wq = FloatQuantizer(fmt, True, 'per_tensor' if pt else 'per_channel', use_qtorch=True)
    aq = None
    if act:
        aq = FloatQuantizer(fmt, True, 'per_token' if act == 1 else 'per_tensor',
                            use_qtorch=True)
    clipper = AutoClipper(w_only=aq is None, wquantizer=wq, aquantizer=aq, clip_version='v1',
                          clip_sym=True, save_clip=False, padding_mask=None)
    bmax, bmin = clipper.auto_clip_layer(0, 'l', c['w'].to(dev), [c['x'].to(dev)],
                                         n_sample_token=nst)
    assert bmax.shape == c['best_max'].shape and bmax.dtype == c['best_max'].dtype
    eq = (bits(bmax) == bits(c['best_max'])).float().mean().item()
    assert eq >= 0.97, eq
    assert torch.equal(bits(bmin), bits(-bmax))
    am = c['w'].float().abs().amax(dim=1)
    grid = torch.stack([(am * (1 - i / 20)).to(c['w'].dtype).float() for i in range(10)], 1)
    assert bool((grid == bmax.cpu().float().view(-1, 1)).any(dim=1).all())


@pytest.mark.parametrize('gran', ['per_channel', 'per_tensor'])
def test_awq_fake_quantize_weight_fp8(dev, gran):
    """Awq.fake_quantize_weight with FloatQuantizer weights (awq.py:147-164): W * s in the
    weight dtype, then the dynamic FP8 fake quant -- bit-equal to the oracle; before this
    round the integer kernel ran on the 897-level [-448, 448] grid instead."""
    from lightcompress_amd.awq import Awq
    from lightcompress_amd.quant import FloatQuantizer
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(512, 1024, generator=g) * 0.02).to(torch.bfloat16)
    s = torch.exp(torch.randn(1024, generator=g) * 0.5).to(torch.bfloat16)
    wq = FloatQuantizer('e4m3', True, gran, use_qtorch=True)
    fc = torch.nn.Linear(1024, 512, bias=False).to(torch.bfloat16).to(dev)
    fc.weight.data = w.to(dev)
    out = torch.empty_like(fc.weight.data)
    Awq.fake_quantize_weight(types.SimpleNamespace(wquantizer=wq), fc, s.to(dev), out)
    ref = P.fp8_qdq(w.clone().mul_(s.view(1, -1)), 'e4m3', gran)[0]
    assert torch.equal(bits(out), bits(ref))


def test_clip_fp8_per_tensor_llama_shape(dev):
    """Per-tensor e4m3 clip at a Llama-3-8B down_proj shape (4096 x 14336, 512 tokens) vs
    the oracle on one 256-row batch (the per-tensor scale couples a batch's rows)."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(12)
    oc, ic, T = 4096, 14336, 512
    w = (torch.randn(oc, ic, generator=g) * 0.02).to(torch.bfloat16)
    x = (torch.randn(T, ic, generator=g) * torch.exp(torch.randn(ic, generator=g))).to(
        torch.bfloat16)
    bmax, _ = ops.auto_clip_search(w.to(dev), x.to(dev), ic, 10, 20, -448, 448, True, True,
                                   fp8=torch.float8_e4m3fn, tensor_batch=256)
    emax, _ = A.clip_layer(w[:256], x, None, True, ic, True, n_sample_token=T,
                           fp8=('e4m3', True, None))
    eq = (bits(bmax.cpu()[:256]) == bits(emax)).float().mean().item()
    assert eq >= 0.97, eq
