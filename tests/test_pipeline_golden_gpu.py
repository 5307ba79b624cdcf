"""End-to-end parity with the REAL reference's block driver (tests/golden/gen_pipeline.py):
the same tiny random Llama (tests/golden/pipeline_llama, 2 blocks, GQA), the same calibration
token ids through our Catcher, run_block_loop + deploy('fake_quant'); every deployed linear of
both blocks, every GPTQ Hessian and every AWQ loss curve compared with the reference's.

What "match" means here (SURVEY.md §8c tiers):
* RTN (data-free): bit-exact deployed weights (T1).
* AWQ (T3): the reference's forwards ran on torch-CPU, ours on hipBLASLt / the fused kernels,
  so loss curves agree to ~1e-4 relative in block 0 (bit-identical inputs). There the chosen
  ratio and the scales are equal and the first subset (q/k/v) deploys bit-equal. Every later
  subset sees inputs that already differ in the last bits (CPU vs GPU attention, clip choices
  upstream), so its curve may drift further (<= 1e-2) and the argmin may move only inside a
  near tie (our pick's loss within 0.2 % of the reference's minimum on the REFERENCE curve;
  measured: block 1's gate/up subset under quant_out, losses 8.4433e-6 vs 8.4482e-6).
* GPTQ (T2): per-layer Hessians equal to ~1e-7 relative for the first subset (identical
  inputs); later subsets' Hessians are built from fake-quantized predecessors whose few flipped
  codes perturb them (measured 1e-4 .. 2e-2). That is the reference's own noise floor: its
  Hessians move by 2.5e-3 (b0 o_proj), 1.0e-2 (b0 down), 1.4e-2 / 2.1e-2 (b1 o / down) when
  the last mantissa bit of 0.1 % of its first-block inputs flips (measured on torch-CPU); a
  wrong driver semantic, e.g. float instead of fake-quant predecessors, moves them by
  several %. Deployed first-subset weights >= 99.5 % bit-equal; GPTQ's error feedback spreads
  every flip along its row, so later layers are compared through their Hessians.
"""
import pytest
import torch

import fixtures as F
import pipeline_helpers as P

pytestmark = pytest.mark.gpu


def compare(ref, got, n=14):
    return P.compare(ref, got, n)


def run_ours(name, dev, monkeypatch=None):
    return P.run_ours(name, dev, monkeypatch)


def test_rtn_pipeline_bit_exact(dev):
    ref, got, _ = run_ours('rtn', dev)
    assert all(eq == 1.0 for eq in compare(ref, got).values())


def test_hqq_pipeline_vs_reference(dev):
    """HQQ (hqq.py, hqq_w_only.yml: axis 0, round_zp False, 20 proximal steps): most
    deployed linears bit-equal, every one >= 99 % (T2: the per-group zero means and the global
    error mean sum in another order than torch-CPU, so a code at a rounding tie can flip and
    move its group's zero by 1 / 128 -- up to a whole group of 128 values; scales are exact)."""
    ref, got, _ = run_ours('hqq', dev)
    eqs = compare(ref, got)
    assert len(eqs) == 14
    assert all(eq >= 0.99 for eq in eqs.values()), eqs
    assert sum(eq == 1.0 for eq in eqs.values()) >= 7, eqs


@pytest.mark.parametrize('name', ['awq', 'awq_qout_asym', 'awq_gqa'])
def test_awq_pipeline_vs_reference(dev, name, monkeypatch):
    """awq_gqa (do_gqa_trans): the o_proj subset is searched too (on v_proj's input, scales
    repeated over the query heads) and its scales divide v_proj's rows, so v_proj is no longer
    a first-subset-only linear."""
    gqa = name == 'awq_gqa'
    ref, got, diag = run_ours(name, dev, monkeypatch)
    res = compare(ref, got)
    first = ('b0__self_attn__q_proj', 'b0__self_attn__k_proj') + (
        () if gqa else ('b0__self_attn__v_proj',))
    for k in first:
        assert res[k] == 1.0, k
    rdiag = F.load(f'pipe_{name}_diag')
    lkeys = sorted(k for k in rdiag if k.startswith('L_'))
    assert lkeys == sorted(k for k in diag if k.startswith('L_'))
    moved = set()
    for k in lkeys:
        r, o = rdiag[k], diag[k]
        rel = ((o - r).abs() / r.abs()).max().item()
        ri, oi = int(r.argmin()), int(o.argmin())
        print(f'{k}: max rel loss diff {rel:.2e}, argmin ref {ri} ours {oi}')
        if k.startswith('L_b0'):
            assert rel < 1e-3 and ri == oi, k
            assert torch.equal(diag['S' + k[1:]], rdiag['S' + k[1:]]), k
        else:
            assert rel < 1e-2, k
            assert ri == oi or r[oi].item() <= r[ri].item() * 1.002, k  # near tie only
        if ri != oi:
            moved.add(k)
    # deployed weights: >= 95 % bit-equal wherever the same ratio was chosen (the rest are
    # clip choices downstream of last-bit input differences)
    subset_of = ({'self_attn__q_proj': 0, 'self_attn__k_proj': 0, 'self_attn__v_proj': 1,
                  'self_attn__o_proj': 1, 'mlp__gate_proj': 2, 'mlp__up_proj': 2,
                  'mlp__down_proj': 3} if gqa else
                 {'self_attn__q_proj': 0, 'self_attn__k_proj': 0, 'self_attn__v_proj': 0,
                  'mlp__gate_proj': 1, 'mlp__up_proj': 1, 'mlp__down_proj': 2})
    for k, eq in res.items():
        b, lin = k.split('__', 1)
        sub = subset_of.get(lin)
        if sub is not None and f'L_{b}__{sub}' in moved:
            continue
        assert eq >= 0.95, k


def test_awq_w8a8_pipeline_vs_reference(dev, monkeypatch):
    """configs/quantization/backend/vllm/awq_w8a8.yml (int8 per_channel weights, int8 dynamic
    per_token activations in the search and the clip, per-channel auto-clip, quant_out):
    block 0's q/k projections deploy bit-equal (no clip there, identical inputs), every block-0
    loss curve within 3e-3 with the same argmin, later curves near-tie (T3 as above). Clipped
    linears: the per-channel clip sums ic-long rows in k order (T2), so a row whose
    bound choice sits on a near tie may take the neighbouring bound -> >= 90 % bit-equal."""
    ref, got, diag = run_ours('awq_w8a8', dev, monkeypatch)
    res = compare(ref, got)
    print(res)
    for k in ('b0__self_attn__q_proj', 'b0__self_attn__k_proj'):
        assert res[k] == 1.0, k
    rdiag = F.load('pipe_awq_w8a8_diag')
    lkeys = sorted(k for k in rdiag if k.startswith('L_'))
    assert lkeys == sorted(k for k in diag if k.startswith('L_'))
    for k in lkeys:
        r, o = rdiag[k], diag[k]
        rel = ((o - r).abs() / r.abs()).max().item()
        ri, oi = int(r.argmin()), int(o.argmin())
        print(f'{k}: max rel loss diff {rel:.2e}, argmin ref {ri} ours {oi}')
        if k.startswith('L_b0'):
            # the per_token int8 fake quant of each GEMM's input turns a last-bit difference
            # of the CPU vs GPU forward into a whole int8 step now and then: 1.4e-3 measured
            assert rel < 3e-3 and ri == oi, k
        else:
            assert rel < 1e-2, k
            assert ri == oi or r[oi].item() <= r[ri].item() * 1.002, k
    for k, eq in res.items():
        assert eq >= 0.9, (k, eq)


def test_gptq_pipeline_vs_reference(dev, monkeypatch):
    ref, got, diag = run_ours('gptq', dev, monkeypatch)
    res = compare(ref, got)
    for k in ('b0__self_attn__q_proj', 'b0__self_attn__k_proj', 'b0__self_attn__v_proj'):
        assert res[k] >= 0.995, k
    rdiag = F.load('pipe_gptq_diag')
    assert sorted(rdiag) == sorted(diag)
    for k in sorted(rdiag):
        r, o = rdiag[k].float(), diag[k].float()
        rel = ((o - r).norm() / r.norm()).item()
        print(f'{k:32s} Hessian rel diff {rel:.2e}')
        if k.startswith('H_b0__self_attn') and not k.endswith('o_proj'):
            assert rel < 1e-6, k
        elif k.startswith('H_b0'):
            assert rel < 2e-2, k
        else:
            assert rel < 5e-2, k


def test_gptq_static_groups_pipeline_vs_reference(dev):
    """static_groups + act-order (group 64) through the whole block loop: the group qparams
    are the construction-time ones, so the first subset (identical inputs) deploys >= 99.5 %
    bit-equal (measured 100 %) and every later linear stays close to the reference (T2)."""
    ref, got, _ = run_ours('gptq_static', dev)
    res = compare(ref, got)
    for k in ('b0__self_attn__q_proj', 'b0__self_attn__k_proj', 'b0__self_attn__v_proj'):
        assert res[k] >= 0.995, k
    # later layers: inputs already differ in the last bits (module docstring) and GPTQ's error
    # feedback spreads each flipped code along its row (measured 78 .. 99 % bit-equal, every
    # max |dw| 2.7e-2)
    for k, eq in res.items():
        assert eq >= 0.7, k
        d = (ref[k].float() - got[k].float()).abs().max().item()
        assert d < 0.05, k


@pytest.mark.parametrize('name', ['rtn_a8_static', 'rtn_a8_hist'])
def test_rtn_static_act_pipeline_vs_reference(dev, name):
    """RTN w8a8 with static per-tensor activation qparams (rtn_w_a_pertensor_static.yml:
    static_hist as shipped, and static_minmax): the reference's block loop registers buf_act_scales_0 on every linear from
    its calibration inputs. Deployed weights bit-equal (T1); the first subset's inputs are
    identical, so its act scale equals the reference's (the fp32 mean may differ in its last
    bit: sum order, T2); later inputs come from GPU vs CPU float forwards (module docstring)."""
    ref, got, diag = run_ours(name, dev)
    assert all(eq == 1.0 for eq in compare(ref, got).values())
    akeys = sorted(k for k in ref if k.startswith('a_'))
    assert sorted(diag) == akeys and len(akeys) == 14
    for k in akeys:
        r, o = ref[k], diag[k]
        assert r.dtype == o.dtype and r.shape == o.shape, k
        rel = abs(o.item() - r.item()) / abs(r.item())
        print(f'{k:32s} act scale {o.item():.8e} ref {r.item():.8e} rel {rel:.1e}')
        if k.startswith('a_b0__self_attn') and not k.endswith('o_proj'):
            assert rel <= 2 ** -23, k
        else:
            assert rel < 1e-2, k


@pytest.mark.parametrize('name', ['awq_fp8', 'awq_fp8_static'])
def test_awq_fp8_pipeline_vs_reference(dev, name, monkeypatch):
    """backend/vllm/fp8/awq_fp8.yml (e4m3 per_channel weights, per_token dynamic e4m3 acts)
    and awq_fp8_static.yml (e4m3 per_tensor weights, static per_tensor e4m3 acts, calib_algo
    static_minmax) through the whole block loop with quant_out: float-quant fake quant of
    W * s in every ratio, FP8 activation fake quant in the search and the clip, float-quant
    auto-clip, static act calibration. Block 0's q / k projections deploy bit-equal (identical
    inputs, no clip); block-0 loss curves within 3e-3 with the same argmin (the e4m3 act quant
    of each GEMM input turns a last-bit forward difference into a whole e4m3 step now and
    then) and every block-0 linear >= 95 % bit-equal. Block 1 sees inputs that already differ
    (CPU vs GPU forwards through the FP8 act quant): its curves agree to 3e-2 with the argmin
    equal or near-tie (T3), and a clip bound moved by a near tie re-scales a whole row
    (per_channel) or the whole tensor (per_tensor), so block-1 weights are compared by their
    relative Frobenius distance (< 8e-2, one e4m3 step is 6.25 % of a value; measured ~1e-2)."""
    ref, got, diag = run_ours(name, dev, monkeypatch)
    res = compare(ref, got)
    for k in ('b0__self_attn__q_proj', 'b0__self_attn__k_proj'):
        assert res[k] == 1.0, k
    rdiag = F.load(f'pipe_{name}_diag')
    lkeys = sorted(k for k in rdiag if k.startswith('L_'))
    assert lkeys == sorted(k for k in diag if k.startswith('L_'))
    for k in lkeys:
        r, o = rdiag[k], diag[k]
        rel = ((o - r).abs() / r.abs()).max().item()
        ri, oi = int(r.argmin()), int(o.argmin())
        print(f'{k}: max rel loss diff {rel:.2e}, argmin ref {ri} ours {oi}')
        if k.startswith('L_b0'):
            assert rel < 3e-3 and (ri == oi or r[oi].item() <= r[ri].item() * 1.002), k
        else:
            assert rel < 3e-2, k
            assert ri == oi or r[oi].item() <= r[ri].item() * 1.005, k
    for k, eq in res.items():
        if k.startswith('b0__'):
            assert eq >= 0.95, (k, eq)
        else:
            d = ((got[k].float() - ref[k].float()).norm() / ref[k].float().norm()).item()
            print(f'{k:40s} rel Frobenius {d:.2e}')
            assert d < 8e-2, (k, d)
    if name == 'awq_fp8_static':
        akeys = sorted(k for k in ref if k.startswith('a_'))
        assert sorted(k for k in diag if k.startswith('a_')) == akeys and len(akeys) == 14
        for k in akeys:
            rel = abs(diag[k].float().item() - ref[k].float().item()) / abs(ref[k].float().item())
            print(f'{k:32s} act scale rel {rel:.1e}')
            assert diag[k].dtype == ref[k].dtype, k
            assert rel < 2e-2, k


def test_gptq_fp8_pipeline_vs_reference(dev, monkeypatch):
    """backend/vllm/fp8/gptq_fp8.yml (e4m3 per_channel weights, per_token e4m3 acts,
    act-order, true_sequential, quant_out): the float-quant column loop through the block
    driver. First-subset Hessians equal to 1e-6 (identical inputs), the rest within the
    reference's own noise floor (module docstring); first-subset linears >= 99.5 % bit-equal."""
    ref, got, diag = run_ours('gptq_fp8', dev, monkeypatch)
    res = compare(ref, got)
    for k in ('b0__self_attn__q_proj', 'b0__self_attn__k_proj', 'b0__self_attn__v_proj'):
        assert res[k] >= 0.995, k
    rdiag = F.load('pipe_gptq_fp8_diag')
    assert sorted(rdiag) == sorted(diag)
    for k in sorted(rdiag):
        r, o = rdiag[k].float(), diag[k].float()
        rel = ((o - r).norm() / r.norm()).item()
        print(f'{k:32s} Hessian rel diff {rel:.2e}')
        if k.startswith('H_b0__self_attn') and not k.endswith('o_proj'):
            assert rel < 1e-6, k
        else:
            assert rel < 5e-2, k
    for k, eq in res.items():
        assert eq >= 0.7, (k, eq)


@pytest.mark.parametrize('name', ['awq_omni_w8a8', 'awq_omni_w6a6'])
def test_awq_clip_v2_pipeline_vs_reference(dev, name, monkeypatch):
    """combination/awq_comb_omni/{w8a8,w6a6}/step_1_awq.yml (asym per_channel weights with
    calib_algo learnable, asym per_token acts, clip_version v2, save_scale / save_clip): the
    clip keeps the weights and registers logit factors that the deployed fake quant applies
    (get_learnable_range). Block 0's q / k projections deploy bit-equal (identical inputs, no
    clip); block-0 loss curves within 3e-3 with the same argmin (the per_token act quant turns
    a last-bit forward difference into a whole step now and then), later curves near-tie only.
    Clip factors: the per-channel clip sums ic-long rows in k order (T2), so a row on a near
    tie may take the neighbouring bound, and every clipped linear's input already went through
    a GPU forward (attention, SiLU * up) -> factors equal on >= 93 % of the rows of every
    linear (measured >= 95.7 %), deployed weights >= 90 % bit-equal. scales.pth holds the
    chosen scales of every searched linear under the reference's names (block 0's equal to
    the bit), clips.pth exactly the registered factors."""
    ref, got, diag = run_ours(name, dev, monkeypatch)
    res = compare(ref, got)
    for k in ('b0__self_attn__q_proj', 'b0__self_attn__k_proj'):
        assert res[k] == 1.0, k
    rdiag = F.load(f'pipe_{name}_diag')
    for k in sorted(k for k in rdiag if k.startswith('L_')):
        r, o = rdiag[k], diag[k]
        rel = ((o - r).abs() / r.abs()).max().item()
        ri, oi = int(r.argmin()), int(o.argmin())
        print(f'{k}: max rel loss diff {rel:.2e}, argmin ref {ri} ours {oi}')
        if k.startswith('L_b0'):
            assert rel < 3e-3 and ri == oi, k
        else:
            assert rel < 1e-2, k
            assert ri == oi or r[oi].item() <= r[ri].item() * 1.002, k
    for k, eq in res.items():
        assert eq >= 0.9, (k, eq)
    fkeys = sorted(k for k in ref if k[:3] in ('up_', 'lo_'))
    assert fkeys and fkeys == sorted(k for k in diag if k[:3] in ('up_', 'lo_'))
    for k in fkeys:
        r, o = ref[k], diag[k]
        assert r.dtype == o.dtype and r.shape == o.shape, k
        eq = (r.view(torch.int16) == o.view(torch.int16)).float().mean().item()
        print(f'{k:32s} factors equal {eq * 100:.2f} %')
        assert eq >= 0.93, (k, eq)
    skeys = sorted(k for k in ref if k.startswith('sc__'))
    assert skeys and skeys == sorted(k for k in diag if k.startswith('sc__'))
    for k in skeys:
        if '__0__' in k:
            assert torch.equal(ref[k].view(torch.int16), diag[k].view(torch.int16)), k
    ckeys = sorted(k for k in ref if k.startswith('cl'))
    assert ckeys == sorted(k for k in diag if k.startswith('cl'))
    for k in ckeys:  # clips.pth: the registered buffers themselves
        b, rest = k[2:].split('__', 1)
        lin, kind = rest.split('__weight_quantizer__')
        fk = f'{kind[:2]}_b{b}__{lin}'
        assert torch.equal(diag[k].view(torch.int16), diag[fk].view(torch.int16)), k
