"""Pin the GPTQ oracle against golden vectors from the real reference (CPU, same torch ops:
bit-exact on the machine that generated them; tiered on others)."""
import pytest
import torch

import fixtures as F
from oracle import gptq_ref as G
from oracle import quant_ref as Q

CASES = F.names('gptq_')


def _meta(c):
    bit, sym, gs, act, oc, ic = c['meta'].tolist()
    return bit, bool(sym), gs, bool(act), oc, ic


@pytest.mark.parametrize('name', CASES)
def test_hessian_matches_reference(name):
    c = F.load(name)
    H, n = G.hessian([x.unsqueeze(0) for x in c['x']], c['x'].shape[-1])
    assert n == c['x'].shape[0]
    torch.testing.assert_close(H, c['H'], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('name', CASES)
def test_layer_matches_reference(name):
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    r = G.quantize_layer(c['w'], c['H'], bit, sym, gs, act)
    torch.testing.assert_close(r['U'], c['U'], rtol=1e-5, atol=1e-6)
    if act:
        assert torch.equal(r['perm'], c['perm'])
    # codes of the error-compensated weight under the stored group qparams
    same_w = (r['weight'] == c['weight']).float().mean().item()
    assert same_w > 0.999, same_w
    torch.testing.assert_close(r['scales'], c['scales'], rtol=1e-5, atol=1e-7)
    fq = G.deploy_fake(r['weight'], r['scales'], r['zeros'], r['perm'], r['invperm'], bit, sym,
                       gs, torch.bfloat16)
    agree = (fq == c['fq']).float().mean().item()
    assert agree > 0.9999, agree


@pytest.mark.parametrize('name', CASES)
def test_column_loop_exact_given_reference_U(name):
    """With the reference's own U and permutation, the oracle column loop reproduces the
    reference weights and qparams bit for bit."""
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    W = c['w'].float().clone()
    dead = torch.diag(c['H']) == 0
    W[:, dead] = 0
    if act:
        W = W[:, c['perm']]
    tmp, _, s, z = G.column_loop(W, c['U'], bit, sym, gs)
    if act:
        tmp = tmp[:, torch.argsort(c['perm'])]
    assert torch.equal(tmp, c['weight'])
    assert torch.equal(s.reshape(-1, 1), c['scales'])
    if not sym:
        assert torch.equal(z.reshape(-1, 1), c['zeros'])


SG_CASES = F.names('gptqsg_')


@pytest.mark.parametrize('name', SG_CASES)
def test_static_groups_exact_given_reference_U(name):
    """static_groups (gptq.py:224-227): with the reference's U, the oracle column loop under
    the construction-time group qparams reproduces the reference weights bit for bit, and the
    layer's qparams are left as collected."""
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    W = c['w'].float().clone()
    dead = torch.diag(c['H']) == 0
    W[:, dead] = 0
    perm = c['perm'] if act else None
    if act:
        W = W[:, perm]
    rows = W.shape[0]
    st = (c['scales'].reshape(rows, -1), None if sym else c['zeros'].reshape(rows, -1), perm)
    tmp, _, _, _ = G.column_loop(W, c['U'], bit, sym, gs, static=st)
    if act:
        tmp = tmp[:, torch.argsort(perm)]
    assert torch.equal(tmp, c['weight'])
    # the qparams the reference kept are those of the ORIGINAL weights
    s0 = Q.qparams(*Q.minmax(Q.group_view(c['w'], 'per_group', gs)), *Q.int_range(bit, sym),
                   sym)[0]
    torch.testing.assert_close(s0.float().reshape(-1, 1), c['scales'].float(), rtol=0, atol=0)


@pytest.mark.parametrize('name', SG_CASES)
def test_static_groups_layer_and_deploy(name):
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    r = G.quantize_layer_static(c['w'], c['H'], c['scales'], c.get('zeros'), bit, sym, gs, act)
    if act:
        assert torch.equal(r['perm'], c['perm'])
    same_w = (r['weight'] == c['weight']).float().mean().item()
    assert same_w > 0.999, same_w
    # need_perm is False with static_groups: w_qdq quantizes the original column order
    fq = G.deploy_fake(r['weight'], c['scales'], c.get('zeros'), None, None, bit, sym, gs,
                       torch.bfloat16)
    agree = (fq == c['fq']).float().mean().item()
    assert agree > 0.9999, agree


OWQ_CASES = F.names('gptqowq_')


def _meta_owq(c):
    bit, sym, gs, nout, oc, ic = c['meta'].tolist()
    return bit, bool(sym), gs, nout, oc, ic


@pytest.mark.parametrize('name', OWQ_CASES)
def test_owq_layer_matches_reference(name):
    """OWQ: permutation (outliers last), compensated weights incl. the float outlier columns,
    group qparams over the non-outlier columns, and w_qdq with the outliers restored."""
    c = F.load(name)
    bit, sym, gs, nout, oc, ic = _meta_owq(c)
    r = G.quantize_layer_owq(c['w'], c['H'], nout, bit, sym, gs)
    assert torch.equal(r['perm'], c['perm'])
    same_w = (r['weight'] == c['weight']).float().mean().item()
    assert same_w > 0.999, same_w
    # groups past the quantized columns keep the construction qparams (gptq.py:383-396)
    ngq = r['scales'].shape[0] // oc
    torch.testing.assert_close(r['scales'].reshape(oc, ngq),
                               c['scales'].reshape(oc, -1)[:, :ngq], rtol=1e-5, atol=1e-7)
    fq = G.deploy_fake_owq(c['weight'], c['scales'], c.get('zeros'), c['perm'],
                           torch.argsort(c['perm']), ic - nout, bit, sym, gs, torch.bfloat16)
    assert torch.equal(fq, c['fq'])


MSE_CASES = F.names('gptqmse_')


@pytest.mark.parametrize('name', MSE_CASES)
def test_mse_column_loop_exact_given_reference_U(name):
    """calib_algo mse: the group ranges searched from the global W at each group's first
    column (search_column_qparams) -- oracle column loop bit-exact given the reference's U."""
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    W = c['w'].float().clone()
    if act:
        W = W[:, c['perm']]
    tmp, _, s, z = G.column_loop(W, c['U'], bit, sym, gs, mse=True)
    if act:
        tmp = tmp[:, torch.argsort(c['perm'])]
    assert torch.equal(tmp, c['weight'])
    assert torch.equal(s.reshape(-1, 1), c['scales'])
    if not sym:
        assert torch.equal(z.reshape(-1, 1), c['zeros'])


@pytest.mark.parametrize('name', MSE_CASES)
def test_mse_layer_matches_reference(name):
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    r = G.quantize_layer(c['w'], c['H'], bit, sym, gs, act, mse=True)
    fq = G.deploy_fake(r['weight'], r['scales'], r['zeros'], r['perm'], r['invperm'], bit, sym,
                       gs, torch.bfloat16)
    agree = (fq == c['fq']).float().mean().item()
    assert agree > 0.999, agree


@pytest.mark.parametrize('name', F.names('gptqowqpc_'))
def test_owq_per_channel_matches_reference(name):
    """OWQ per_channel (gptq.py:157-166): per-channel qparams of the permuted non-outlier
    columns, column loop with them, w_qdq with the outliers restored."""
    c = F.load(name)
    bit, sym, _, nout, oc, ic = _meta_owq(c)
    r = G.quantize_layer_owq(c['w'], c['H'], nout, bit, sym, None)
    assert torch.equal(r['perm'], c['perm'])
    torch.testing.assert_close(r['scales'], c['scales'], rtol=1e-6, atol=0)
    same_w = (r['weight'] == c['weight']).float().mean().item()
    assert same_w > 0.999, same_w
    fq = G.deploy_fake_owq(c['weight'], c['scales'], c.get('zeros'), c['perm'],
                           torch.argsort(c['perm']), ic - nout, bit, sym, None, torch.bfloat16)
    assert torch.equal(fq, c['fq'])
