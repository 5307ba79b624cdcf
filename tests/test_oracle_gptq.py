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
