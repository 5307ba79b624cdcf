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


def test_block_fp8_to_tensor_many_one_class_unsorted(dev):
    """Sizes within 2x of each other (ONE size class) given out of size order: the per-tensor
    scales must still come back in input order (the kernel writes them in class order)."""
    from lightcompress_amd import ops
    cs, ss = zip(*[_random_block_fp8(sh, torch.float8_e4m3fn, 60 + i, dev)
                   for i, sh in enumerate([(1024, 1280), (1536, 1280), (1280, 1280)])])
    outs, scales = ops.fp8_block_to_tensor_many(list(cs), list(ss), 128)
    for i, (c, s) in enumerate(zip(cs, ss)):
        oc, os_ = ops.fp8_block_to_tensor(c, s, 128)
        assert torch.equal(bits(outs[i]), bits(oc)) and scales[i].item() == os_.item(), i


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


def _grouped(dev, counts, Nn, K, seed):
    """Rows sorted by group (counts[g] rows each) + per-group fp8 weights, on the device."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(seed)
    rows = sum(counts)
    x = torch.randn(rows, K, generator=g) * torch.exp(torch.randn(rows, 1, generator=g))
    a, a_s = O.act_quant(x)
    ws = [O.weight_cast_to_fp8(torch.randn(Nn, K, generator=g) * 0.05) for _ in counts]
    wd = [(b.to(dev), s.to(dev)) for b, s in ws]
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int64)
    return a, a_s, ws, wd, off, ops.fp8_weight_table(wd, dev)


@pytest.mark.parametrize('counts,Nn,K', [([0, 37, 300, 600, 1, 513, 0], 384, 512),
                                         ([1000, 64, 257], 1500 - 1500 % 4, 896)])
def test_fp8_gemm_grouped_vs_oracle(dev, counts, Nn, K):
    """lcq_fp8_gemm_grouped (one launch over ragged groups, empty ones included) vs the
    fp8_gemm restatement per group (kernel.py:141-214, GEMM_RTOL of |a||b|)."""
    from lightcompress_amd import ops
    a, a_s, ws, _, off, tab = _grouped(dev, counts, Nn, K, seed=sum(counts))
    got = ops.fp8_gemm_grouped(a.to(dev), a_s.to(dev).reshape(-1), off.to(dev), tab, Nn,
                               torch.float32).cpu()
    for i, (b, b_s) in enumerate(ws):
        r0, r1 = int(off[i]), int(off[i + 1])
        if r1 == r0:
            continue
        want = O.fp8_gemm(a[r0:r1], a_s[r0:r1], b, b_s)
        tol = GEMM_RTOL * _abs_gemm(a[r0:r1], a_s[r0:r1], b, b_s) + 1e-30
        assert ((got[r0:r1] - want).abs() <= tol).all(), i


def test_fp8_gemm_grouped_rows_equal_single_unsplit(dev):
    """Each group's rows are bit-identical to lcq_fp8_gemm where that runs the unsplit 256^2
    plan (2048 x 7168: 224 tiles), in bf16 and fp32 output; and repeatable."""
    from lightcompress_amd import ops
    counts, Nn, K = [2048, 2048], 7168, 256
    a, a_s, _, wd, off, tab = _grouped(dev, counts, Nn, K, seed=3)
    ad, asd, offd = a.to(dev), a_s.to(dev), off.to(dev)
    for dt in (torch.float32, torch.bfloat16):
        got = ops.fp8_gemm_grouped(ad, asd.reshape(-1), offd, tab, Nn, dt)
        again = ops.fp8_gemm_grouped(ad, asd.reshape(-1), offd, tab, Nn, dt)
        assert torch.equal(got, again)
        for i, (b, b_s) in enumerate(wd):
            r0, r1 = int(off[i]), int(off[i + 1])
            one = ops.fp8_gemm(ad[r0:r1], asd[r0:r1].contiguous(), b, b_s, out_dtype=dt)
            assert torch.equal(got[r0:r1], one), (dt, i)


def test_fp8_gemm_grouped_gather_and_two_sets(dev):
    """a_rows (the kernel gathers each sorted row from the token matrix) and two weight sets
    in one launch (gate and up) give exactly the rows of the plain one-set launches on the
    pre-gathered matrix."""
    from lightcompress_amd import ops
    counts, Nn, K = [300, 0, 77, 513], 512, 384
    g = torch.Generator().manual_seed(8)
    T = 400
    x = torch.randn(T, K, generator=g) * torch.exp(torch.randn(T, 1, generator=g))
    a, a_s = O.act_quant(x)
    rows = torch.randint(0, T, (sum(counts),), generator=g)
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int64).to(dev)
    sets = [[O.weight_cast_to_fp8(torch.randn(Nn, K, generator=g) * 0.05) for _ in counts]
            for _ in range(2)]
    keep = [[(b.to(dev), s.to(dev)) for b, s in ws] for ws in sets]  # the tables point here
    tabs = [ops.fp8_weight_table(ws, dev) for ws in keep]
    ad, asd, rd = a.to(dev), a_s.to(dev), rows.to(dev)
    both = ops.fp8_gemm_grouped(ad, asd.reshape(-1), off, torch.stack(tabs), Nn,
                                torch.float32, a_rows=rd)
    assert both.shape == (2, sum(counts), Nn)
    ag, sg = ad[rd].contiguous(), asd[rd].contiguous()
    for i in range(2):
        one = ops.fp8_gemm_grouped(ag, sg.reshape(-1), off, tabs[i], Nn, torch.float32)
        assert torch.equal(both[i], one), i


def test_fp8_gemm_grouped_silu_mul_equals_two_sets(dev):
    """The pair mode (gate and up tiles in one workgroup, act_fn(gate) * up in the epilogue)
    equals torch's silu(gate) * up on the two-set launch's bf16 projections, bit for bit,
    ragged groups and a partial 128-column block included."""
    from lightcompress_amd import ops
    counts, Nn, K = [300, 0, 77, 513], 384 + 64, 512
    g = torch.Generator().manual_seed(9)
    T = 500
    x = torch.randn(T, K, generator=g) * torch.exp(torch.randn(T, 1, generator=g))
    a, a_s = O.act_quant(x)
    rows = torch.randint(0, T, (sum(counts),), generator=g).to(dev)
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int64).to(dev)
    keep = [[tuple(t.to(dev) for t in O.weight_cast_to_fp8(
        torch.randn(Nn, K, generator=g) * 0.2)) for _ in counts] for _ in range(2)]
    tab = torch.stack([ops.fp8_weight_table(ws, dev) for ws in keep])
    ad, asd = a.to(dev), a_s.to(dev).reshape(-1)
    gu = ops.fp8_gemm_grouped(ad, asd, off, tab, Nn, torch.bfloat16, a_rows=rows)
    h = ops.fp8_gemm_grouped(ad, asd, off, tab, Nn, torch.bfloat16, a_rows=rows,
                             silu_mul=True)
    want = torch.nn.functional.silu(gu[0]) * gu[1]
    assert h.shape == want.shape
    assert torch.equal(h.view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize('wdt', [torch.float32, torch.bfloat16])
def test_moe_combine_equals_index_add_loop(dev, wdt):
    """lcq_moe_combine == the expert loop's combine: out.index_add_(0, tok, (y_e * w).to(bf16))
    for the hit experts in ascending index (torch on the device)."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(int(wdt == torch.bfloat16))
    T, E, k, H = 333, 12, 5, 264
    idx = torch.stack([torch.randperm(E, generator=g)[:k] for _ in range(T)]).to(dev)
    w = torch.rand(T, k, generator=g).to(wdt).to(dev)
    flat = idx.reshape(-1)
    order = torch.argsort(flat, stable=True)
    slot_row = torch.empty_like(order)
    slot_row[order] = torch.arange(order.numel(), device=dev)
    y = (torch.randn(T * k, H, generator=g) * 3).to(torch.bfloat16).to(dev)
    got = ops.moe_combine(y, slot_row, idx, w, T)
    want = torch.zeros(T, H, dtype=torch.bfloat16, device=dev)
    for e in range(E):
        tok, pos = torch.where(idx == e)
        if tok.numel():
            want.index_add_(0, tok, (y[slot_row.view(T, k)[tok, pos]] * w[tok, pos, None]).to(
                torch.bfloat16))
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


def test_fp8_gemm_grouped_rejects_bad_tables(dev):
    from lightcompress_amd import ops
    _, _, _, wd, _, _ = _grouped(dev, [4, 4], 256, 256, seed=1)
    with pytest.raises(ValueError):   # shapes differ
        ops.fp8_weight_table([wd[0], (wd[1][0][:128].contiguous(), wd[1][1][:1].contiguous())],
                             dev)
    with pytest.raises(TypeError):
        ops.fp8_weight_table([(wd[0][0].float(), wd[0][1])], dev)


def _fp8_experts(dev, E, H, inter, seed):
    from transformers.models.deepseek_v3 import modeling_deepseek_v3 as md

    from lightcompress_amd.deepseekv3 import ExpertList
    from lightcompress_amd.module_utils import LlmcFp8Linear
    cfg = md.DeepseekV3Config(hidden_size=H, intermediate_size=inter, hidden_act='silu')
    g = torch.Generator().manual_seed(seed)
    experts = ExpertList()
    for _ in range(E):
        mlp = md.DeepseekV3MLP(cfg, intermediate_size=inter)
        for p in ('gate_proj', 'up_proj', 'down_proj'):
            lin = getattr(mlp, p)
            m = LlmcFp8Linear.new(lin, 128)
            b, s = O.weight_cast_to_fp8(torch.randn(lin.out_features, lin.in_features,
                                                    generator=g) * 0.05)
            m.weight.data, m.weight_scale_inv.data = b, s
            setattr(mlp, p, m)
        experts.append(mlp)
    return experts.to(dev)


def _routing(dev, T, E, k, seed):
    g = torch.Generator().manual_seed(seed)
    idx = torch.stack([torch.randperm(E, generator=g)[:k] for _ in range(T)])
    w = torch.rand(T, k, generator=g)
    return idx.to(dev), (w / w.sum(1, keepdim=True)).to(dev)


def test_expert_list_grouped_equals_loop(dev, monkeypatch):
    """ExpertList's grouped block-fp8 forward (one lcq_fp8_gemm_grouped per projection) equals
    the per-expert loop (models/deepseekv3.py's expert loop: act_quant + fp8 GEMM per expert,
    index_add_ in expert order) bit for bit when each loop GEMM runs the same per-row
    arithmetic (a one-group launch); with the loop's own per-expert plans (32x32x64 kernel,
    split-K for short experts) within the fp8 GEMM tolerance. A forward hook (calibration
    capture) sends the call back to the loop."""
    from lightcompress_amd import module_utils, ops
    from lightcompress_amd.kernel import act_quant
    E, H, inter, T, k = 8, 512, 384, 300, 3
    experts = _fp8_experts(dev, E, H, inter, seed=4)
    idx, w = _routing(dev, T, E, k, seed=5)
    x = (torch.randn(T, H, generator=torch.Generator().manual_seed(6)) * 2).to(
        torch.bfloat16).to(dev)
    assert experts._grouped_fp8_ok(x)
    grouped = experts(x, idx, w)

    def one_group(x, wt, ws, block, bias):
        xq, xs = act_quant(x.contiguous(), block)
        off = torch.tensor([0, xq.shape[0]], dtype=torch.int64, device=x.device)
        return ops.fp8_gemm_grouped(xq, xs.reshape(-1), off,
                                    ops.fp8_weight_table([(wt.data, ws.data)], x.device),
                                    wt.shape[0], torch.bfloat16)

    monkeypatch.setattr(type(experts), '_grouped_fp8_ok', lambda s, x: False)
    loop_default = experts(x, idx, w)
    monkeypatch.setattr(module_utils, 'block_wise_fp8_forward_func', one_group)
    loop_same = experts(x, idx, w)
    assert torch.equal(grouped, loop_same)
    tol = 2.0 ** -6 * loop_default.float().abs().max()
    assert (grouped.float() - loop_default.float()).abs().max() <= tol
    monkeypatch.undo()
    h = experts[0].down_proj.register_forward_hook(lambda *a: None)
    try:
        assert not experts._grouped_fp8_ok(x)
    finally:
        h.remove()
