"""Fused calibration-forward kernels are bit-identical to the torch ops they replace."""
import pytest
import torch
import torch.nn.functional as Fn

pytestmark = pytest.mark.gpu


def _rot_ref(q, k, cos, sin):
    def rh(x):
        return torch.cat((-x[..., x.shape[-1] // 2:], x[..., : x.shape[-1] // 2]), dim=-1)
    c, s = cos.unsqueeze(1), sin.unsqueeze(1)
    return q * c + rh(q) * s, k * c + rh(k) * s


@pytest.mark.parametrize('B,S,Hq,Hk,D,dt,cb', [(2, 64, 4, 2, 128, torch.bfloat16, 1),
                                               (3, 17, 8, 8, 64, torch.float16, 3),
                                               (1, 512, 32, 8, 128, torch.bfloat16, 1)])
def test_rotary_bit_exact(dev, B, S, Hq, Hk, D, dt, cb):
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(B * S)
    qp = torch.randn(B, S, Hq * D, generator=g, device=dev).to(dt)
    kp = torch.randn(B, S, Hk * D, generator=g, device=dev).to(dt)
    q = qp.view(B, S, Hq, D).transpose(1, 2)
    k = kp.view(B, S, Hk, D).transpose(1, 2)
    ang = torch.rand(cb, S, D // 2, generator=g, device=dev) * 6.28
    cos = torch.cat([ang.cos(), ang.cos()], -1).to(dt)
    sin = torch.cat([ang.sin(), ang.sin()], -1).to(dt)
    oq, ok = ops.rotary(q, k, cos, sin)
    rq, rk = _rot_ref(q, k, cos, sin)
    assert oq.shape == rq.shape and ok.shape == rk.shape
    assert torch.equal(oq, rq) and torch.equal(ok, rk)


@pytest.mark.parametrize('n,dt', [(4096 * 33, torch.bfloat16), (8 * 1000, torch.float16)])
def test_silu_mul_bit_exact(dev, n, dt):
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(n)
    a = (torch.randn(n, generator=g, device=dev) * 4).to(dt)
    b = torch.randn(n, generator=g, device=dev).to(dt)
    assert torch.equal(ops.silu_mul(a, b), Fn.silu(a) * b)


def test_block_forward_unchanged(dev):
    """A Llama block forward with the fusions installed equals the stock forward bit for bit."""
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml
    from lightcompress_amd import llama as L
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=1, vocab_size=128)
    model = L.Llama.random(cfg, device=dev, seed=5)
    blk = model.get_blocks()[0]
    x = torch.randn(2, 64, 256, device=dev).to(torch.bfloat16)
    kw = model.rotary_kwargs(64)
    fused = blk(x, **kw)
    fused = fused[0] if isinstance(fused, tuple) else fused
    from transformers.modeling_utils import AttentionInterface
    saved = ml.apply_rotary_pos_emb
    ml.apply_rotary_pos_emb = L._ORIG_ROTARY
    saved_sdpa = AttentionInterface._global_mapping['sdpa']
    if L._ORIG_SDPA is not None:
        AttentionInterface.register('sdpa', L._ORIG_SDPA)
    patched = [m for m in blk.modules() if 'forward' in m.__dict__]
    fwds = [m.__dict__['forward'] for m in patched]
    for m in patched:
        del m.forward  # back to the class methods
    try:
        ref = blk(x, **kw)
        ref = ref[0] if isinstance(ref, tuple) else ref
    finally:
        ml.apply_rotary_pos_emb = saved
        AttentionInterface.register('sdpa', saved_sdpa)
        for m, f in zip(patched, fwds):
            m.forward = f
    # rotary and silu*up are bit-identical; RMSNorm's variance order may move a rounding; the
    # flash kernel vs torch's SDPA differ within bf16 rounding of the attention output
    torch.testing.assert_close(fused.float(), ref.float(), rtol=2e-2, atol=2e-2)
    assert (fused != ref).float().mean().item() < 0.02


@pytest.mark.parametrize('rows,H,dt', [(300, 4096, torch.bfloat16), (17, 256, torch.float16)])
def test_rmsnorm_close_to_torch(dev, rows, H, dt):
    """One-pass RMSNorm vs the HF chain: identical except where the variance's summation
    order moves a bf16 rounding (<= 1 ulp, on a tiny fraction of elements)."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(rows)
    x = (torch.randn(rows, H, generator=g, device=dev) * 3).to(dt)
    w = (torch.rand(H, generator=g, device=dev) + 0.5).to(dt)
    h = x.float()
    ref = w * (h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-5)).to(dt)
    out = ops.rmsnorm(x, w, 1e-5)
    diff = (out.float() - ref.float()).abs()
    ulp = ref.float().abs() * (2 ** -7 if dt == torch.bfloat16 else 2 ** -10)
    assert (diff <= ulp + 1e-30).all()
    assert (diff > 0).float().mean().item() < 0.01


def test_staged_forward_memo_invalidation(dev):
    """The memoised decoder forward equals the stock one after in-place weight updates,
    module replacement and with hooks registered (hooked stages recompute and fire)."""
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml
    from lightcompress_amd import llama as L
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=1, vocab_size=128)
    model = L.Llama.random(cfg, device=dev, seed=6)
    blk = model.get_blocks()[0]
    x = torch.randn(2, 32, 256, device=dev).to(torch.bfloat16)
    kw = model.rotary_kwargs(32)

    def stock():
        return L._STOCK_DECODER_FORWARD(blk, x, **kw)

    out1 = blk(x, **kw)
    assert torch.equal(out1, stock())
    assert torch.equal(blk(x, **kw), out1)                      # memo hit
    with torch.no_grad():
        blk.mlp.up_proj.weight.mul_(1.5)                        # in-place: _version bump
    assert torch.equal(blk(x, **kw), stock())
    new_o = torch.nn.Linear(256, 256, bias=False).to(dev, torch.bfloat16)
    blk.self_attn.o_proj = new_o                                # module replaced
    assert torch.equal(blk(x, **kw), stock())
    seen = []
    h = blk.mlp.gate_proj.register_forward_hook(lambda m, i, o: seen.append(i[0].shape))
    blk(x, **kw)                                                # hooked stage recomputes
    h.remove()
    assert len(seen) == 1
    L.clear_stage_cache(blk)
    assert '_lcq_stage' not in blk.__dict__
