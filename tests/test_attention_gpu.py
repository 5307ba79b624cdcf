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
                                        (1, 6, 2, 300), (3, 3, 1, 129)])
def test_attention_vs_fp32(dev, B, H, KVH, S):
    """(1, 6, 2, 300) and (3, 3, 1, 129): workgroup counts 18 and 18 (not multiples of the 8
    XCDs) for the XCD-contiguous work order."""
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
