"""lcq projection GEMMs (csrc/gemm256.hip) against torch: the nn.Linear calls of the AWQ
loss-search / calibration forwards (awq.py:110-126) and calculate_loss (awq.py:134-145).

Two kinds of check:
* exact data (small integers / 8 in bf16): every product and fp32 partial sum is exact, so the
  accumulation order cannot matter and outputs must equal torch's bit for bit, including the
  fused SiLU product and the loss's per-element terms;
* random data against an fp32 reference: |out - fp32| <= one bf16 ulp of the fp32 value
  (fp32 accumulation in another order can move the single rounding by at most one ulp), which
  catches any layout / tile / segment / edge-masking error.
"""
import pytest
import torch

from lightcompress_amd import ops

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _exact(shape, gen, lo=-3, hi=4):
    return (torch.randint(lo, hi, shape, generator=gen, device=DEV).float() / 8).to(torch.bfloat16)


def _ulp_ok(out, ref32, dtype=torch.bfloat16, absum=None):
    """|out - ref| <= one ulp of the dtype at the reference value + the fp32 accumulation
    bound of either side (2^-21 * sum |x||w|, `absum`)."""
    r = ref32.abs().clamp_min(1e-30)
    mant = 7 if dtype == torch.bfloat16 else 10
    ulp = torch.pow(2.0, torch.floor(torch.log2(r)) - mant)
    slack = 1e-6 if absum is None else absum * 2.0 ** -21
    bad = (out.float() - ref32).abs() > ulp + slack
    if bad.any():
        i = bad.nonzero()[:5].tolist()
        print('mismatch at', i, out.float()[bad][:5].tolist(), ref32[bad][:5].tolist())
    return not bad.any().item()


@pytest.mark.parametrize('M,N,K', [(256, 256, 64), (100, 768, 128), (513, 1024, 4096),
                                   (4096, 512, 256), (1, 16, 64), (300, 272, 192)])
def test_linear_exact(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    x = _exact((M, K), g)
    w = _exact((N, K), g)
    out = ops.linear(x, w)
    ref = (x.float() @ w.float().T).to(torch.bfloat16)
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('M,N,K', [(2048, 1024, 4096), (777, 512, 1024), (64, 4096, 512)])
def test_linear_random_within_one_ulp(M, N, K, dtype):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g, device=DEV).to(dtype)
    w = (torch.randn(N, K, generator=g, device=DEV) * 0.02).to(dtype)
    out = ops.linear(x, w)
    ref = x.float() @ w.float().T
    absum = x.float().abs() @ w.float().abs().T
    assert out.dtype == dtype and out.shape == (M, N)
    assert _ulp_ok(out, ref, dtype, absum)


def test_linear_bias_and_batch_dims():
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(3, 100, 256, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(512, 256, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(512, generator=g, device=DEV).to(torch.bfloat16)
    out = ops.linear(x, w, b)
    ref = x.float() @ w.float().T + b.float()
    assert out.shape == (3, 100, 512)
    assert _ulp_ok(out, ref, absum=x.float().abs() @ w.float().abs().T + b.float().abs())


def test_linear_strided_input_rows():
    """A row-strided input (a column slice of a wider activation) is read in place."""
    g = torch.Generator(device=DEV).manual_seed(4)
    big = torch.randn(300, 640, generator=g, device=DEV).to(torch.bfloat16)
    x = big[:, :512]
    w = (torch.randn(256, 512, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    assert _ulp_ok(ops.linear(x, w), x.float() @ w.float().T,
                   absum=x.float().abs() @ w.float().abs().T)


def test_linear_multi_segments_qkv_shape():
    """q / k / v (4096 / 1024 / 1024 rows at Llama scale; here 512 / 256 / 256 + bias on k)
    from one launch equal three separate launches bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(2, 300, 512, generator=g, device=DEV).to(torch.bfloat16)
    ws = [(torch.randn(n, 512, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
          for n in (512, 256, 256)]
    bk = torch.randn(256, generator=g, device=DEV).to(torch.bfloat16)
    outs = ops.linear_multi(x, ws, [None, bk, None])
    for o, w, b in zip(outs, ws, [None, bk, None]):
        one = ops.linear(x, w, b)
        assert o.shape == one.shape
        assert torch.equal(o.view(torch.int16), one.view(torch.int16))
    assert _ulp_ok(outs[1], x.float() @ ws[1].float().T + bk.float(),
                   absum=x.float().abs() @ ws[1].float().abs().T + bk.float().abs())


def test_linear_multi_segments_from_one_buffer():
    """Segments that are row ranges of one buffer (the AWQ search's concatenated q/k/v
    fake-quant weights)."""
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.randn(513, 256, generator=g, device=DEV).to(torch.bfloat16)
    wall = (torch.randn(1024, 256, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    q, k, v = wall[:512], wall[512:768], wall[768:]
    outs = ops.linear_multi(x, [q, k, v])
    full = ops.linear(x, wall)
    assert torch.equal(torch.cat(outs, dim=1).view(torch.int16), full.view(torch.int16))


def _rope_tables(B, S, g):
    """HF-style cos / sin [B or 1, S, 128] (emb = cat(freqs, freqs), positions per sample)."""
    inv = 1.0 / (500000.0 ** (torch.arange(0, 128, 2, device=DEV).float() / 128))
    pos = torch.arange(S, device=DEV).float()[None, :] + (
        torch.randint(0, 50, (B, 1), generator=g, device=DEV).float())
    fr = pos[..., None] * inv[None, None, :]
    emb = torch.cat([fr, fr], -1)
    return emb.cos().to(torch.bfloat16), emb.sin().to(torch.bfloat16)


@pytest.mark.parametrize('B,S,shared,dt', [(2, 300, True, torch.bfloat16),
                                           (3, 128, False, torch.bfloat16),
                                           (1, 2048, True, torch.bfloat16),
                                           (4, 77, False, torch.bfloat16),
                                           (2, 200, False, torch.float16)])
def test_linear_multi_rope_equals_gemm_then_rotary(B, S, shared, dt):
    """lcq_gemm_rope (q / k rotated in the GEMM epilogue) equals lcq_gemm followed by
    lcq_rotary bit for bit: shared ([1, S, 128]) and per-sample ([B, S, 128]) cos / sin,
    ragged row counts (B * S not a multiple of 256), a bias on k, bf16 and fp16."""
    g = torch.Generator(device=DEV).manual_seed(11 + S)
    x = torch.randn(B, S, 512, generator=g, device=DEV).to(dt)
    ws = [(torch.randn(n, 512, generator=g, device=DEV) * 0.05).to(dt) for n in (512, 256, 256)]
    bs = [None, torch.randn(256, generator=g, device=DEV).to(dt), None]
    cos, sin = _rope_tables(B, S, g)
    cos, sin = cos.to(dt), sin.to(dt)
    if shared:
        cos, sin = cos[:1].contiguous(), sin[:1].contiguous()
    q, k, v = ops.linear_multi_rope(x, ws, bs, cos, sin, rope_segs=2)
    q0, k0, v0 = ops.linear_multi(x, ws, bs)
    qh = q0.view(B, S, 4, 128).transpose(1, 2)
    kh = k0.view(B, S, 2, 128).transpose(1, 2)
    qr, kr = ops.rotary(qh, kh, cos, sin)
    for a, b in ((q, qr.transpose(1, 2).reshape(B, S, 512)),
                 (k, kr.transpose(1, 2).reshape(B, S, 256)), (v, v0)):
        assert torch.equal(a.view(torch.int16), b.reshape(a.shape).view(torch.int16))


def test_attention_core_rope_fused_equals_unfused(monkeypatch):
    """LlamaAttention up to o_proj (llama._attn_core) with the rotary in the q/k/v GEMM
    epilogue equals the path through apply_rotary_pos_emb (lcq_rotary) bit for bit."""
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaAttention, LlamaRotaryEmbedding

    from lightcompress_amd import llama
    cfg = LlamaConfig(hidden_size=512, num_attention_heads=4, num_key_value_heads=2,
                      head_dim=128, intermediate_size=1024)
    cfg._attn_implementation = 'sdpa'
    torch.manual_seed(0)
    attn = LlamaAttention(cfg, 0).to(DEV, torch.bfloat16).eval()
    llama.install_fused_forward(attn)   # the lcq rotary / attention patches
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(2, 256, 512, generator=g, device=DEV).to(torch.bfloat16)
    rot = LlamaRotaryEmbedding(cfg).to(DEV)
    pe = rot(x, torch.arange(256, device=DEV)[None].expand(2, -1))
    fused = llama._attn_core(attn, x, pe, None)
    calls = []
    monkeypatch.setattr(llama, '_rope_fusable', lambda *a: calls.append(1) or False)
    plain = llama._attn_core(attn, x, pe, None)
    assert calls, 'the unfused path was not taken'
    assert torch.equal(fused.view(torch.int16), plain.view(torch.int16))


@pytest.mark.parametrize('M,I,K', [(512, 1024, 256), (300, 272, 512), (4096, 512, 4096)])
def test_linear_silu_mul_exact(M, I, K):
    g = torch.Generator(device=DEV).manual_seed(M + I)
    x = _exact((M, K), g)
    wg = _exact((I, K), g)
    wu = _exact((I, K), g)
    h = ops.linear_silu_mul(x, wg, wu)
    gate = (x.float() @ wg.float().T).to(torch.bfloat16)
    up = (x.float() @ wu.float().T).to(torch.bfloat16)
    ref = ops.silu_mul(gate, up)  # bit-exact vs torch's act_fn(g) * u (test_forward_fused_gpu)
    assert torch.equal(h.view(torch.int16), ref.view(torch.int16))


def test_linear_silu_mul_random():
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(1000, 512, generator=g, device=DEV).to(torch.bfloat16)
    wg = (torch.randn(768, 512, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    wu = (torch.randn(768, 512, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    h = ops.linear_silu_mul(x, wg, wu)
    gate = (x.float() @ wg.float().T).to(torch.bfloat16)
    up = (x.float() @ wu.float().T).to(torch.bfloat16)
    ref = ops.silu_mul(gate, up)
    # identical wherever gate and up rounded the same way (accumulation order moves a rounding
    # by at most one ulp): nearly everywhere, and within a few bf16 ulps elsewhere
    same = (h.view(torch.int16) == ref.view(torch.int16)).float().mean().item()
    assert same > 0.97, same
    err = (h.float() - ref.float()).abs()
    assert (err <= 0.03 * ref.float().abs() + 2e-3).all()


@pytest.mark.parametrize('M,N,K', [(512, 256, 512), (777, 1024, 256), (4096, 768, 1024)])
def test_linear_sq_diff_exact(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M + 3 * N)
    x = _exact((M, K), g)
    w = _exact((N, K), g)
    ref_out = _exact((M, N), g, -40, 40)
    lb = ops.LossBuffer(3, DEV)
    ops.linear_sq_diff(x, w, ref_out, lb, 1)
    out = (x.float() @ w.float().T).to(torch.bfloat16)
    want = ops.sq_diff_mean(ref_out, out)
    got = lb.out[1].item()
    assert lb.out[0].item() == 0.0 and lb.out[2].item() == 0.0
    assert abs(got - want) <= 2e-7 * abs(want)


def test_linear_sq_diff_random_and_deterministic():
    g = torch.Generator(device=DEV).manual_seed(21)
    x = torch.randn(2, 300, 512, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(512, 512, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(512, generator=g, device=DEV).to(torch.bfloat16)
    org = ops.linear(x, w, b) + (torch.randn(2, 300, 512, generator=g, device=DEV) * 0.01).to(torch.bfloat16)
    lb = ops.LossBuffer(2, DEV)
    ops.linear_sq_diff(x, w, org, lb, 0, bias=b)
    ops.linear_sq_diff(x, w, org, lb, 1, bias=b)
    want = ops.sq_diff_mean(org, ops.linear(x, w, b))
    assert lb.out[0].item() == lb.out[1].item()
    assert abs(lb.out[0].item() - want) <= 1e-6 * abs(want)


def test_gemm_rejects_bad_shapes():
    x = torch.zeros(16, 100, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(16, 100, dtype=torch.bfloat16, device=DEV)
    assert not ops.gemm_supported(x, w)
    with pytest.raises(ValueError):
        ops.linear(x, w)


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('M,N,K', [(2048, 4096, 4096), (777, 512, 1024), (300, 272, 192)])
def test_linear_residual_equals_add(M, N, K, dtype):
    """lcq_gemm_residual (the block's residual + o_proj / down_proj in the epilogue) equals the
    separate residual + linear bit for bit: the same two roundings, with and without bias."""
    g = torch.Generator(device=DEV).manual_seed(M + 5 * N + K)
    x = torch.randn(M, K, generator=g, device=DEV).to(dtype)
    w = (torch.randn(N, K, generator=g, device=DEV) * 0.02).to(dtype)
    r = torch.randn(M, N, generator=g, device=DEV).to(dtype)
    b = (torch.randn(N, generator=g, device=DEV) * 0.1).to(dtype)
    for bias in (None, b):
        got = ops.linear_residual(x, w, r, bias)
        ref = r + ops.linear(x, w, bias)
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
