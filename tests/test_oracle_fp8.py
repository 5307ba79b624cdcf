"""FP8 oracle vs the reference's golden fixtures (CPU), and the kernel's fp8 encoder
algorithm (restated in numpy) vs torch's native cast."""
import numpy as np
import pytest
import torch

import fixtures as F
from oracle import fp8_ref as O

EMUL = ['e4m3_pc_bf16', 'e4m3_g128_bf16', 'e5m2_pc_bf16', 'e4m3_pc_f16', 'e3m2_pc_bf16']
SCALES = {'e4m3_pc_bf16': ('e4m3', 'per_channel', None), 'e4m3_g128_bf16': ('e4m3', 'per_group', 128),
          'e4m3_pt_bf16': ('e4m3', 'per_tensor', None), 'e5m2_pc_f16': ('e5m2', 'per_channel', None),
          'e4m3_blk_bf16': ('e4m3', 'per_block', None),
          'e4m3_blk_ragged_bf16': ('e4m3', 'per_block', None)}


def same(a, b):
    """Bit-equal values, NaN where the reference has NaN (all-zero rows give NaN there)."""
    a, b = a.float(), b.float()
    return torch.equal(a.isnan(), b.isnan()) and torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))


@pytest.mark.parametrize('name', EMUL)
def test_emulation_matches_reference(name):
    c = F.load(f'fp8emul_{name}')
    e, m, gs = (int(v) for v in c['meta'])
    gran = 'per_group' if gs != c['w'].shape[1] else 'per_channel'
    out = O.emul_fake_quant(c['w'], e, m, gran, gs)
    assert out.dtype == c['fq'].dtype and same(out, c['fq'])
    act = O.emul_fake_quant(c['act'], e, m, 'per_token')
    assert same(act, c['act_fq'])


@pytest.mark.parametrize('name', list(SCALES))
def test_scales_match_reference(name):
    c = F.load(f'fp8scale_{name}')
    bit, gran, gs = SCALES[name]
    t = O.group_view(c['w'], gran, gs)
    mn, mx = O.minmax(t, gran)
    s = O.sym_scales(mn, mx, O.qmax_of(bit))
    assert s.dtype == c['scales'].dtype and torch.equal(s, c['scales'])
    _, codes, rs = O.fp8_qdq(c['w'], bit, gran, gs)
    assert codes.shape == c['w'].shape
    want = c['scales'].reshape(-1).float().clone()
    want[want == 0] = 1  # quant.py:1062 mutates the scales real_quant then returns
    assert torch.equal(rs.reshape(-1).float(), want)


@pytest.mark.parametrize('name', ['even', 'ragged_m'])
def test_block_dequant_matches_reference(name):
    c = F.load(f'fp8cast_bf16_{name}')
    out = O.weight_cast_to_bf16(c['codes'], c['scales'])
    assert torch.equal(out.view(torch.int16), c['out'].view(torch.int16))


# ---- the device encoder's bit algorithm (csrc/fp8.hip enc_e4m3 / enc_e5m2) in numpy ------------
def enc_model(f: np.ndarray, e4m3: bool) -> np.ndarray:
    b = f.astype(np.float32).view(np.uint32).astype(np.uint64)
    sign = b & 0x80000000
    b = b ^ sign
    out = np.zeros_like(b)
    if e4m3:
        big, small, mask, shift, bias = 1087 << 20, 121 << 23, 141 << 23, 20, 7
        rnd = 0x7FFFF
    else:
        big, small, mask, shift, bias = 143 << 23, 113 << 23, 134 << 23, 21, 15
        rnd = 0xFFFFF
    hi = b >= big
    lo = (~hi) & (b < small)
    mid = ~(hi | lo)
    if e4m3:
        out[hi] = 0x7F
    else:
        out[hi] = np.where(b[hi] > 0x7F800000, 0x7F, 0x7C)
    t = (b[lo].astype(np.uint32).view(np.float32) + np.uint32(mask).view(np.float32))
    out[lo] = (t.view(np.uint32).astype(np.uint64) - mask) & 0xFF
    odd = (b[mid] >> shift) & 1
    v = (b[mid] + (((bias - 127) << 23) & 0xFFFFFFFF) + rnd + odd) & 0xFFFFFFFF
    out[mid] = (v >> shift) & 0xFF
    return (out | (sign >> 24)).astype(np.uint8)


@pytest.mark.parametrize('fmt', ['e4m3', 'e5m2'])
def test_encoder_model_matches_torch_cast(fmt):
    allb = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16).float()
    g = torch.Generator().manual_seed(1)
    rnd = torch.randn(200000, generator=g) * torch.exp(torch.randn(200000, generator=g) * 4)
    x = torch.cat([allb, rnd, torch.tensor([464.0, 480.0, 447.9, 57344.0, 61440.0, 65536.0])])
    dt = O.FP8[fmt]
    ref = x.to(dt).view(torch.uint8).numpy()
    got = enc_model(x.numpy(), fmt == 'e4m3')
    nan = np.isnan(x.numpy())
    assert np.array_equal(got[~nan], ref[~nan])


def _gemm_case(M, Nn, K, seed, batch=None):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, K, generator=g) * torch.exp(torch.randn(M, 1, generator=g))
    w = torch.randn(Nn, K, generator=g) * 0.05
    a, a_s = O.act_quant(x)
    b, b_s = O.weight_cast_to_fp8(w)
    if batch is not None:
        a = a.reshape(*batch, K)
        a_s = a_s.reshape(*batch, K // 128)
    return a, a_s, b, b_s


def _dequant_gemm(a, a_s, b, b_s, absolute=False):
    K = a.shape[-1]
    ad = a.reshape(-1, K).double() * a_s.reshape(-1, K // 128).double().repeat_interleave(128, 1)
    bd = b.double() * b_s.double().repeat_interleave(128, 0)[:b.shape[0]].repeat_interleave(128, 1)
    if absolute:
        ad, bd = ad.abs(), bd.abs()
    return (ad @ bd.T).reshape(*a.shape[:-1], b.shape[0])


@pytest.mark.parametrize('M,Nn,K', [(1, 128, 128), (37, 200, 384), (64, 256, 1024)])
def test_fp8_gemm_oracle_vs_exact_dequant_matmul(M, Nn, K):
    """fp8_gemm restatement (kernel.py:141-214) vs the exact float64 dequantized product:
    fp32 accumulation error only (tolerance 1e-5 of the |a||b| product)."""
    a, a_s, b, b_s = _gemm_case(M, Nn, K, seed=M + Nn)
    got = O.fp8_gemm(a, a_s, b, b_s)
    assert got.dtype == torch.float32 and got.shape == (M, Nn)
    exact = _dequant_gemm(a, a_s, b, b_s)
    tol = 1e-5 * _dequant_gemm(a, a_s, b, b_s, absolute=True) + 1e-30
    assert ((got.double() - exact).abs() <= tol).all()


def test_fp8_gemm_oracle_batched_leading_dims():
    a, a_s, b, b_s = _gemm_case(6, 130, 256, seed=5, batch=(2, 3))
    got = O.fp8_gemm(a, a_s, b, b_s)
    assert got.shape == (2, 3, 130)
    flat = O.fp8_gemm(a.reshape(6, 256), a_s.reshape(6, 2), b, b_s)
    assert torch.equal(got.reshape(6, 130), flat)
