"""FP8 kernels (lcq_fp8_* / lcq_fp_emul_quant) vs the oracle and the reference fixtures."""
import pytest
import torch

import fixtures as F
from oracle import fp8_ref as O

pytestmark = pytest.mark.gpu


def same(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return torch.equal(a.isnan(), b.isnan()) and torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))


def bits(t):
    return t.cpu().view(torch.uint8)


@pytest.mark.parametrize('fp8', [torch.float8_e4m3fn, torch.float8_e5m2])
def test_cast_exhaustive_bf16_and_random_f32(dev, fp8):
    from lightcompress_amd import ops
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    one = torch.ones(1, dtype=torch.float32, device=dev)
    r = ops.fp8_quant_static(allb.to(dev).reshape(256, 256), one, fp8, ct_dtype=torch.float32,
                             add_zero=False)
    want = allb.float().to(fp8).view(torch.uint8).reshape(256, 256)
    nan = allb.float().isnan().reshape(256, 256)
    assert torch.equal(bits(r['codes'])[~nan], want[~nan])
    g = torch.Generator().manual_seed(3)
    x = torch.randn(512, 1024, generator=g) * torch.exp(torch.randn(512, 1, generator=g) * 4)
    r = ops.fp8_quant_static(x.to(dev), one, fp8, add_zero=False)
    assert torch.equal(bits(r['codes']), x.to(fp8).view(torch.uint8))


EMUL = ['e4m3_pc_bf16', 'e4m3_g128_bf16', 'e5m2_pc_bf16', 'e4m3_pc_f16', 'e3m2_pc_bf16']


@pytest.mark.parametrize('name', EMUL)
def test_emulation_vs_reference(dev, name):
    from lightcompress_amd.quant import FloatQuantizer
    c = F.load(f'fp8emul_{name}')
    e, m, gs = (int(v) for v in c['meta'])
    bit = f'e{e}m{m}'
    kw = {'group_size': gs} if gs != c['w'].shape[1] else {}
    gran = 'per_group' if kw else 'per_channel'
    q = FloatQuantizer(bit, True, gran, **kw)
    out = q.fake_quant_weight_dynamic(c['w'].to(dev))
    assert out.dtype == c['fq'].dtype and same(out, c['fq'])
    aq = FloatQuantizer(bit, True, 'per_token')
    assert same(aq.fake_quant_act_dynamic(c['act'].to(dev)), c['act_fq'])


CASES = [('e4m3', 'per_channel', {}, torch.bfloat16, (64, 512)),
         ('e4m3', 'per_group', {'group_size': 128}, torch.bfloat16, (64, 512)),
         ('e4m3', 'per_token', {}, torch.bfloat16, (48, 7168)),
         ('e4m3', 'per_tensor', {}, torch.bfloat16, (256, 1024)),
         ('e4m3', 'per_block', {'block_size': 128}, torch.bfloat16, (384, 256)),
         ('e4m3', 'per_block', {'block_size': 128}, torch.bfloat16, (200, 264)),
         ('e5m2', 'per_channel', {}, torch.float16, (64, 512)),
         ('e4m3', 'per_channel', {}, torch.float32, (32, 256))]


@pytest.mark.parametrize('bit,gran,kw,dt,shape', CASES)
def test_qtorch_path_vs_oracle(dev, bit, gran, kw, dt, shape):
    from lightcompress_amd.quant import FloatQuantizer
    from inputs import fp8_inputs
    w = fp8_inputs(*shape, dt, 77)
    q = FloatQuantizer(bit, True, gran, use_qtorch=True, **kw)
    fq_ref, codes_ref, s_ref = O.fp8_qdq(w, bit, gran, kw.get('group_size'))
    fq = q.fake_quant_weight_dynamic(w.to(dev))
    assert fq.dtype == dt and same(fq, fq_ref)
    codes, s, z = q.real_quant_weight_dynamic(w.to(dev))
    assert z is None and codes.dtype == O.FP8[bit]
    assert torch.equal(bits(codes), codes_ref.view(torch.uint8))
    assert s.shape == s_ref.shape and s.dtype == s_ref.dtype and torch.equal(s.cpu(), s_ref)
    if gran != 'per_block':  # static path with the dynamic scales reproduces the dynamic one
        _, s4, zz, qmax, qmin = q.get_tensor_qparams(w.to(dev))
        st = q.fake_quant_weight_static(w.to(dev), {'scales': s4, 'zeros': zz, 'qmax': qmax,
                                                     'qmin': qmin})
        assert same(st, fq_ref)


@pytest.mark.parametrize('name', ['even', 'ragged_m'])
def test_block_dequant_vs_reference(dev, name):
    from lightcompress_amd.quant import weight_cast_to_bf16
    c = F.load(f'fp8cast_bf16_{name}')
    out = weight_cast_to_bf16(c['codes'].to(dev), c['scales'].to(dev), 128)
    assert torch.equal(out.cpu().view(torch.int16), c['out'].view(torch.int16))


@pytest.mark.parametrize('shape', [(256, 384), (200, 264), (2048, 7168)])
def test_kernel_py_casts_vs_oracle(dev, shape):
    from lightcompress_amd import kernel as K
    g = torch.Generator().manual_seed(shape[0])
    x = (torch.randn(*shape, generator=g) * 0.02).to(torch.bfloat16)
    x[:128, :128] = 0  # all-zero block: s = 0 -> NaN, as the Triton kernel
    y, s = K.weight_cast_to_fp8(x.to(dev))
    y_ref, s_ref = O.weight_cast_to_fp8(x)
    assert torch.equal(s.cpu(), s_ref) if not s_ref.isnan().any() else same(s, s_ref)
    assert torch.equal(bits(y), y_ref.view(torch.uint8))
    back = K.weight_cast_to_bf16(y, s).to(torch.bfloat16)
    assert same(back, O.weight_cast_to_bf16(y_ref, s_ref))
    a = (torch.randn(4, shape[1] // 128 * 128, generator=g)).to(torch.bfloat16)
    ya, sa = K.act_quant(a.to(dev))
    ya_ref, sa_ref = O.act_quant(a)
    assert torch.equal(sa.cpu(), sa_ref) and torch.equal(bits(ya), ya_ref.view(torch.uint8))


def test_per_tensor_expert_shape(dev):
    """A DeepSeek-V3 expert linear (2048 x 7168) per-tensor real quant: bit-exact codes."""
    from lightcompress_amd.quant import FloatQuantizer
    g = torch.Generator().manual_seed(11)
    w = (torch.randn(2048, 7168, generator=g) * 0.02).to(torch.bfloat16)
    q = FloatQuantizer('e4m3', True, 'per_tensor', use_qtorch=True)
    codes, s, _ = q.real_quant_weight_dynamic(w.to(dev))
    _, codes_ref, s_ref = O.fp8_qdq(w, 'e4m3', 'per_tensor')
    assert torch.equal(s.cpu(), s_ref)
    assert torch.equal(bits(codes), codes_ref.view(torch.uint8))


@pytest.mark.parametrize('M,N', [(2048, 7168), (7168, 2048), (200, 264)])
def test_block_fp8_to_tensor_fused_equals_composed(dev, M, N):
    """The fused deploy of a block-fp8 weight equals weight_cast_to_bf16 + per-tensor real
    quant bit for bit (and the oracle)."""
    from lightcompress_amd import ops
    from lightcompress_amd.quant import FloatQuantizer, weight_cast_to_bf16
    g = torch.Generator().manual_seed(M + N)
    w = (torch.randn(M, N, generator=g) * 0.02).to(torch.bfloat16)
    r = ops.fp8_quant_blocks(w.to(dev), torch.float8_e4m3fn, 128, qmax=448.0, clamp_min=0.0,
                             add_zero=False)
    c, s = r['codes'], r['scales']
    q = FloatQuantizer('e4m3', True, 'per_tensor', use_qtorch=True)
    fc, fs, _ = q.real_quant_weight_from_block_fp8(c, s, 128)
    wb = weight_cast_to_bf16(c, s, 128)
    cc, cs, _ = q.real_quant_weight_dynamic(wb)
    assert torch.equal(bits(fc), bits(cc)) and torch.equal(fs.cpu(), cs.cpu())
    _, oc, os_ = O.fp8_qdq(O.weight_cast_to_bf16(c.cpu(), s.cpu()), 'e4m3', 'per_tensor')
    assert torch.equal(bits(fc), oc.view(torch.uint8)) and torch.equal(fs.cpu(), os_)


def test_block_fp8_to_tensor_batched_equals_single(dev):
    """One launch pair over a list of expert weights == the per-weight fused path."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(5)
    cs, ss = [], []
    for (m, n) in [(256, 512), (512, 256), (200, 264), (128, 128)]:
        w = (torch.randn(m, n, generator=g) * 0.03).to(torch.bfloat16).to(dev)
        r = ops.fp8_quant_blocks(w, torch.float8_e4m3fn, 128, qmax=448.0, clamp_min=0.0,
                                 add_zero=False)
        cs.append(r['codes'])
        ss.append(r['scales'])
    outs, scales = ops.fp8_block_to_tensor_many(cs, ss, 128)
    for i, (c, s) in enumerate(zip(cs, ss)):
        oc, os_ = ops.fp8_block_to_tensor(c, s, 128)
        assert torch.equal(bits(outs[i]), bits(oc)) and scales[i].item() == os_.item()


def _random_block_fp8(shape, fin, seed, dev, nan_free=True):
    """Random code bytes (every finite code of ``fin`` reachable) + random-sign block scales."""
    g = torch.Generator().manual_seed(seed)
    M, N = shape
    b = torch.randint(0, 256, (M, N), generator=g, dtype=torch.int32).to(torch.uint8)
    if nan_free:
        v = b.view(fin).float()
        b[~torch.isfinite(v)] = 0x11
    s = torch.randn((M + 127) // 128, (N + 127) // 128, generator=g) * 1e-3
    return b.view(fin).to(dev), s.to(dev)


@pytest.mark.parametrize('fin', [torch.float8_e4m3fn, torch.float8_e5m2])
@pytest.mark.parametrize('fout', [torch.float8_e4m3fn, torch.float8_e5m2])
def test_block_fp8_to_tensor_many_random_codes(dev, fin, fout):
    """The 16-codes-per-lane path of lcq_fp8_block_to_tensor_many (byte-max amax, hardware
    OCP conversions) equals the oracle for every finite input code, both formats, on
    expert-sized and ragged tensors (ragged ones take the row-walk fallback)."""
    from lightcompress_amd import ops
    shapes = [(2048, 7168), (7168, 2048), (200, 264), (384, 136)]
    cs, ss = zip(*[_random_block_fp8(sh, fin, 11 + i, dev) for i, sh in enumerate(shapes)])
    outs, scales = ops.fp8_block_to_tensor_many(list(cs), list(ss), 128, fout)
    bit = 'e4m3' if fout == torch.float8_e4m3fn else 'e5m2'
    for i, (c, s) in enumerate(zip(cs, ss)):
        _, oc, os_ = O.fp8_qdq(O.weight_cast_to_bf16(c.cpu(), s.cpu()), bit, 'per_tensor')
        assert torch.equal(bits(outs[i]), oc.view(torch.uint8)), shapes[i]
        assert scales[i].item() == os_.item()
        sc, ssc = ops.fp8_block_to_tensor(c, s, 128, fout)
        assert torch.equal(bits(outs[i]), bits(sc)) and scales[i].item() == ssc.item()


@pytest.mark.parametrize('fout,qmax', [(torch.float8_e4m3fn, 1000.0), (torch.float8_e5m2, 90000.0)])
def test_block_fp8_to_tensor_many_overflow_band(dev, fout, qmax):
    """A qmax above the format's range pushes quotients into c10's overflow band (e4m3fn
    (464, 480) -> NaN code, e5m2 -> inf): the fast path's software-encoder fallback must give
    the same codes as the generic path."""
    from lightcompress_amd import ops
    cs, ss = zip(*[_random_block_fp8((512, 1024), torch.float8_e4m3fn, 40 + i, dev)
                   for i in range(3)])
    outs, scales = ops.fp8_block_to_tensor_many(list(cs), list(ss), 128, fout, qmax=qmax)
    for i, (c, s) in enumerate(zip(cs, ss)):
        sc, ssc = ops.fp8_block_to_tensor(c, s, 128, fout, qmax=qmax)
        assert torch.equal(bits(outs[i]), bits(sc)) and scales[i].item() == ssc.item()


@pytest.mark.parametrize('block', [64, 128])
@pytest.mark.parametrize('shape', [(300, 520), (1024, 2048)])
def test_block_fp8_to_tensor_single_vs_oracle(dev, block, shape):
    """lcq_fp8_block_to_tensor (one weight, descriptor by value) on both the 16-code path
    (block 128) and the row-walk path (other block sizes), vs the oracle."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(block + shape[0])
    M, N = shape
    b = torch.randint(0, 256, (M, N), generator=g, dtype=torch.int32).to(torch.uint8)
    b[~torch.isfinite(b.view(torch.float8_e4m3fn).float())] = 0x22
    s = torch.rand((M + block - 1) // block, (N + block - 1) // block, generator=g) * 1e-2
    c = b.view(torch.float8_e4m3fn)
    oc, os_ = ops.fp8_block_to_tensor(c.to(dev), s.to(dev), block)
    _, rc, rs = O.fp8_qdq(O.weight_cast_to_bf16(c, s, block), 'e4m3', 'per_tensor')
    assert torch.equal(bits(oc), rc.view(torch.uint8)) and os_.item() == rs.item()
    am = ops.absmax(O.weight_cast_to_bf16(c, s, block).to(dev))
    assert am.item() == O.weight_cast_to_bf16(c, s, block).float().abs().max().item()


def _gemm_inputs(M, Nn, K, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, K, generator=g) * torch.exp(torch.randn(M, 1, generator=g))
    w = torch.randn(Nn, K, generator=g) * 0.05
    a, a_s = O.act_quant(x)
    b, b_s = O.weight_cast_to_fp8(w)
    return a, a_s, b, b_s


# The gfx950 f8f6f4 MFMAs (16x16x128 and 32x32x64) do not sum a 128-wide block like a
# sequential fp32 loop: one block's dot product is off the exact sum by up to 2.7e-5 of
# sum|a b| (scripts/fp8_mfma_precision.py, profiles/r3c_fp8_mfma_precision.txt: max 2.05e-5 /
# 2.73e-5, mean 1.5e-6, unbiased on symmetric data). The reference's Triton tl.dot on this
# chip issues the same instructions; the tolerance is that hardware bound with margin.
GEMM_RTOL = 5e-5


def _abs_gemm(a, a_s, b, b_s):
    return O.fp8_gemm(a.view(torch.uint8).bitwise_and(0x7F).view(torch.float8_e4m3fn), a_s.abs(),
                      b.view(torch.uint8).bitwise_and(0x7F).view(torch.float8_e4m3fn), b_s.abs())


# ragged M / N tiles, one K block, the DeepSeek-V3 hidden size (K 7168); the automatic tile
# plans of fp8_gemm.hip: the 32x32x64 kernel (<= 64 rows or < 64 tiles of 256^2, incl. its
# split-K), 256^2 unsplit (2048 x 7168); the forced plans: test_fp8_gemm_forced_plans
@pytest.mark.parametrize('M,Nn,K', [(1, 128, 128), (37, 200, 384), (256, 512, 1024),
                                    (130, 2048, 7168), (1000, 1500, 384), (2048, 1536, 256),
                                    (2048, 7168, 256)])
def test_fp8_gemm_vs_oracle(dev, M, Nn, K):
    """lcq_fp8_gemm vs the fp8_gemm restatement (kernel.py:141-214): same per-block scaling
    order; only the accumulation inside a 128-wide block differs (the MFMA's own, GEMM_RTOL of
    the |a||b| product)."""
    from lightcompress_amd import ops
    a, a_s, b, b_s = _gemm_inputs(M, Nn, K, seed=M * 7 + Nn)
    got = ops.fp8_gemm(a.to(dev), a_s.to(dev), b.to(dev), b_s.to(dev),
                       out_dtype=torch.float32).cpu()
    want = O.fp8_gemm(a, a_s, b, b_s)
    tol = GEMM_RTOL * _abs_gemm(a, a_s, b, b_s) + 1e-30
    err = (got - want).abs()
    assert (err <= tol).all(), float((err / tol).max())


@pytest.mark.parametrize('plan', [1, 128, 256])
@pytest.mark.parametrize('M,Nn,K', [(200, 264, 1024), (1000, 1500, 896), (2048, 1536, 2048)])
def test_fp8_gemm_forced_plans(dev, plan, M, Nn, K):
    """Every kernel / tile plan of lcq_fp8_gemm (forced through lcq_fp8_gemm_force_plan: the
    32x32x64 kernel, 128^2 and 256^2 with their split-K) against the oracle, ragged tiles."""
    from lightcompress_amd import _native as N
    from lightcompress_amd import ops
    a, a_s, b, b_s = _gemm_inputs(M, Nn, K, seed=M + Nn + plan)
    lib = N.load()
    lib.lcq_fp8_gemm_force_plan(plan)
    try:
        got = ops.fp8_gemm(a.to(dev), a_s.to(dev), b.to(dev), b_s.to(dev),
                           out_dtype=torch.float32).cpu()
    finally:
        lib.lcq_fp8_gemm_force_plan(0)
    want = O.fp8_gemm(a, a_s, b, b_s)
    tol = GEMM_RTOL * _abs_gemm(a, a_s, b, b_s) + 1e-30
    assert ((got - want).abs() <= tol).all()


def test_fp8_gemm_bf16_out_and_leading_dims(dev):
    from lightcompress_amd import kernel
    a, a_s, b, b_s = _gemm_inputs(24, 384, 512, seed=11)
    a3, s3 = a.reshape(2, 12, 512), a_s.reshape(2, 12, 4)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        got = kernel.fp8_gemm(a3.to(dev), s3.to(dev), b.to(dev), b_s.to(dev)).cpu()
    finally:
        torch.set_default_dtype(prev)
    assert got.dtype == torch.bfloat16 and got.shape == (2, 12, 384)
    want = O.fp8_gemm(a, a_s, b, b_s).reshape(2, 12, 384)
    tol = GEMM_RTOL * _abs_gemm(a, a_s, b, b_s).reshape(2, 12, 384) + want.abs() * 2.0 ** -8
    assert ((got.float() - want).abs() <= tol).all()


def test_llmc_fp8_linear_forward(dev):
    """LlmcFp8Linear.forward = block_wise_fp8_forward_func (module_utils.py:41-46, 244-262):
    act_quant bit-exact, then the fp8 GEMM, bf16, + bias."""
    import torch.nn as nn
    from lightcompress_amd.module_utils import LlmcFp8Linear
    g = torch.Generator().manual_seed(2)
    lin = nn.Linear(512, 320, bias=True)
    m = LlmcFp8Linear.new(lin, 128)
    w = torch.randn(320, 512, generator=g) * 0.05
    b, b_s = O.weight_cast_to_fp8(w)
    bias = (torch.randn(320, generator=g) * 0.1).to(torch.bfloat16)
    m.weight.data = b
    m.weight_scale_inv.data = b_s
    m.bias = nn.Parameter(bias, requires_grad=False)
    m = m.to(dev)
    x = (torch.randn(3, 5, 512, generator=g)).to(torch.bfloat16)
    got = m(x.to(dev)).cpu()
    a, a_s = O.act_quant(x)
    want = O.fp8_gemm(a, a_s, b, b_s).to(torch.bfloat16) + bias
    assert got.dtype == torch.bfloat16 and got.shape == (3, 5, 320)
    assert (got.float() - want.float()).abs().max() <= 2.0 ** -6 * want.float().abs().max()
    from lightcompress_amd import kernel
    ya, sa = kernel.act_quant(x.to(dev).contiguous())
    assert torch.equal(ya.cpu().view(torch.uint8), a.view(torch.uint8))
    assert torch.equal(sa.cpu(), a_s)


def test_fp8_gemm_rejects_bad_shapes(dev):
    from lightcompress_amd import ops
    a, a_s, b, b_s = _gemm_inputs(8, 128, 256, seed=1)
    with pytest.raises(ValueError):
        ops.fp8_gemm(a.to(dev), a_s.to(dev), b[:, :128].contiguous().to(dev), b_s.to(dev))
    with pytest.raises(ValueError):
        ops.fp8_gemm(a.to(dev), a_s[:, :1].contiguous().to(dev), b.to(dev), b_s.to(dev))
    with pytest.raises(TypeError):
        ops.fp8_gemm(a.float().to(dev), a_s.to(dev), b.to(dev), b_s.to(dev))


def test_fp8_gemm_split_k_matches_unsplit_and_is_deterministic(dev):
    """Short batch (M 96, K 7168): the K-split path (fp32 partials summed in split order) vs
    the same GEMM without a workspace (one split): both within the oracle tolerance, and the
    split result is bitwise repeatable."""
    from lightcompress_amd import _native as N
    from lightcompress_amd import ops
    M, Nn, K = 96, 1024, 7168
    assert N.load().lcq_fp8_gemm_workspace_bytes(M, Nn, K) > 0
    a, a_s, b, b_s = _gemm_inputs(M, Nn, K, seed=21)
    ad, asd, bd, bsd = a.to(dev), a_s.to(dev), b.to(dev), b_s.to(dev)
    split1 = ops.fp8_gemm(ad, asd, bd, bsd, out_dtype=torch.float32)
    split2 = ops.fp8_gemm(ad, asd, bd, bsd, out_dtype=torch.float32)
    one = torch.empty(M, Nn, dtype=torch.float32, device=dev)
    N.call('lcq_fp8_gemm', N.ptr(ad), N.ptr(asd), N.ptr(bd), N.ptr(bsd), M, Nn, K, N.ptr(one),
           N.dt(torch.float32), None, 0, N.stream_of(ad))
    assert torch.equal(split1, split2)
    want = O.fp8_gemm(a, a_s, b, b_s)
    tol = GEMM_RTOL * _abs_gemm(a, a_s, b, b_s) + 1e-30
    assert ((split1.cpu() - want).abs() <= tol).all()
    assert ((one.cpu() - want).abs() <= tol).all()


def test_fp8_gemm_f16_default_dtype(dev):
    """out_dtype follows torch.get_default_dtype() as in the reference's Triton kernel: with an
    fp16 default the GEMM stores fp16 (split and unsplit paths)."""
    from lightcompress_amd import kernel
    for M in (24, 96):
        a, a_s, b, b_s = _gemm_inputs(M, 384, 1024 if M == 24 else 7168, seed=12 + M)
        prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.float16)
        try:
            got = kernel.fp8_gemm(a.to(dev), a_s.to(dev), b.to(dev), b_s.to(dev)).cpu()
        finally:
            torch.set_default_dtype(prev)
        assert got.dtype == torch.float16 and got.shape == (M, 384)
        want = O.fp8_gemm(a, a_s, b, b_s)
        tol = GEMM_RTOL * _abs_gemm(a, a_s, b, b_s) + want.abs() * 2.0 ** -11
        assert ((got.float() - want).abs() <= tol).all()
