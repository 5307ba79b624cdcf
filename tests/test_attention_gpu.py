"""Causal flash-attention kernel (lcq_attn_fwd_causal) vs an fp32 reference; its error must
stay within the error of torch's own bf16 SDPA (aotriton on this image) on the same inputs."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(q, k, v, scale, dtype=torch.float32):
    rep = q.shape[1] // k.shape[1]
    kr = k.repeat_interleave(rep, 1)
    vr = v.repeat_interleave(rep, 1)
    return F.scaled_dot_product_attention(q.to(dtype), kr.to(dtype), vr.to(dtype),
                                          is_causal=True, scale=scale).transpose(1, 2)


@pytest.mark.parametrize('B,H,KVH,S', [(2, 4, 2, 64), (1, 8, 8, 200), (3, 8, 2, 33),
                                        (2, 32, 8, 512), (1, 4, 1, 1000), (1, 2, 2, 1),
                                        (1, 6, 2, 300), (3, 3, 1, 129),
                                        (128, 32, 8, 512), (1, 32, 8, 2048)])
def test_attention_vs_fp32(dev, B, H, KVH, S):
    """(1, 6, 2, 300) and (3, 3, 1, 129): workgroup counts 18 and 18 (not multiples of the 8
    XCDs) for the XCD-contiguous work order. (128, 32, 8, 512) and (1, 32, 8, 2048): the
    shapes bench.py runs (the AWQ calibration forward, 128 x 512 tokens, and the GPTQ one,
    2048-token samples) at Llama-3-8B's 32 query / 8 K/V heads."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(B * 1000 + S)
    D = 128
    # projection-output layout [B, S, heads, D], viewed head-transposed like LlamaAttention
    qs = (torch.randn(B, S, H, D, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    ks = (torch.randn(B, S, KVH, D, generator=g, device=dev) * 1.5).to(torch.bfloat16)
    vs = torch.randn(B, S, KVH, D, generator=g, device=dev).to(torch.bfloat16)
    q, k, v = qs.transpose(1, 2), ks.transpose(1, 2), vs.transpose(1, 2)
    scale = D ** -0.5
    out = ops.attn_fwd_causal(q, k, v, scale)
    assert out.shape == (B, S, H, D) and out.is_contiguous()
    ref = _ref(q, k, v, scale)
    err = (out.float() - ref).abs().max().item()
    torch_bf16 = _ref(q, k, v, scale, torch.bfloat16).float()
    err_torch = (torch_bf16 - ref).abs().max().item()
    print(f'max |ours - fp32| {err:.3e}, max |torch bf16 - fp32| {err_torch:.3e}')
    assert torch.isfinite(out).all()
    assert err <= max(2.0 * err_torch, 1e-2)


def test_attention_contiguous_heads_layout(dev):
    """[B, H, S, D]-contiguous inputs (strides differ from the projection views)."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(7)
    q = torch.randn(2, 8, 256, 128, generator=g, device=dev).to(torch.bfloat16)
    k = torch.randn(2, 2, 256, 128, generator=g, device=dev).to(torch.bfloat16)
    v = torch.randn(2, 2, 256, 128, generator=g, device=dev).to(torch.bfloat16)
    out = ops.attn_fwd_causal(q, k, v, 0.1)
    ref = _ref(q, k, v, 0.1)
    assert (out.float() - ref).abs().max().item() < 2e-2


def test_attention_kv_span_limit(dev):
    """One (batch, K/V head)'s rows spanning just under the 2 GB the kernel's 32-bit buffer
    offsets reach (include/lcq.h: S * seq stride < 2^30 elements): K and V as views into
    2 GB buffers whose rows are 2^30 / S - 8 elements apart. Checked against the fp32
    reference like every other shape; one stride more is refused."""
    from lightcompress_amd import _native, ops
    B, H, KVH, S, D = 1, 4, 2, 128, 128
    kss = (1 << 30) // S - 8
    g = torch.Generator(device=dev).manual_seed(11)
    q = torch.randn(B, S, H, D, generator=g, device=dev).to(torch.bfloat16).transpose(1, 2)
    kv = []
    for _ in range(2):
        base = torch.empty(S * kss, dtype=torch.bfloat16, device=dev)
        rows = base.view(S, kss)
        rows[:, : KVH * D] = torch.randn(S, KVH * D, generator=g, device=dev).to(torch.bfloat16)
        kv.append(rows[:, : KVH * D].view(1, S, KVH, D).transpose(1, 2))  # seq stride kss
    k, v = kv
    assert k.stride(2) == kss and S * k.stride(2) < (1 << 30)
    scale = D ** -0.5
    out = ops.attn_fwd_causal(q, k, v, scale)
    ref = _ref(q, k.contiguous(), v.contiguous(), scale)
    err = (out.float() - ref).abs().max().item()
    err_torch = (_ref(q, k.contiguous(), v.contiguous(), scale, torch.bfloat16).float()
                 - ref).abs().max().item()
    assert torch.isfinite(out).all() and err <= max(2.0 * err_torch, 1e-2), (err, err_torch)
    del kv, k, v
    big = torch.empty(S * (kss + 16), dtype=torch.bfloat16, device=dev)
    kb = big.view(S, kss + 16)[:, : KVH * D].view(1, S, KVH, D).transpose(1, 2)
    with pytest.raises((ValueError, _native.LcqError)):   # LCQ_EINVAL surfaces as ValueError
        ops.attn_fwd_causal(q, kb, kb, scale)
