"""Pin the AWQ / auto-clip oracle against golden vectors from the real reference."""
import pytest
import torch

import fixtures as F
from awq_helpers import build_layer, forward_fn
from oracle import awq_ref as A


@pytest.mark.parametrize('subset', ['qkv', 'mlp', 'down'])
@pytest.mark.parametrize('sym', [True, False])
def test_search_scale_matches_reference(subset, sym):
    c = F.load(f'awq_{subset}_{"sym" if sym else "asym"}')
    cfg, layer, kwargs = build_layer()
    fwd, ws = forward_fn(layer, subset, kwargs)
    losses, best_i, best_s = A.search_scale(c['x'], ws, fwd, 4, sym, 128)
    assert torch.equal(torch.tensor(losses, dtype=torch.float64), c['losses'])
    assert torch.equal(best_s.view(torch.int16), c['scales'].view(torch.int16))


@pytest.mark.parametrize('subset', ['qkv', 'mlp', 'down'])
@pytest.mark.parametrize('sym', [True, False])
def test_search_scale_v1_matches_reference(subset, sym):
    """trans_version v1 (weight-scale term): get_weight_scale and the whole search."""
    c = F.load(f'awq_{subset}_{"sym" if sym else "asym"}_v1')
    cfg, layer, kwargs = build_layer()
    fwd, ws = forward_fn(layer, subset, kwargs)
    assert torch.equal(A.weight_scale(ws, 128).view(torch.int16), c['w_max'].view(torch.int16))
    losses, best_i, best_s = A.search_scale(c['x'], ws, fwd, 4, sym, 128, version='v1')
    assert torch.equal(torch.tensor(losses, dtype=torch.float64), c['losses'])
    assert torch.equal(best_s.view(torch.int16), c['scales'].view(torch.int16))


@pytest.mark.parametrize('name', F.names('clip_'))
def test_auto_clip_matches_reference(name):
    c = F.load(name)
    sym, clip_sym, nst, group, mse = c['meta'].tolist()
    bmax, bmin = A.clip_layer(c['w'], c['x'], 4, bool(sym), group, bool(clip_sym),
                              n_sample_token=nst, mse=bool(mse))
    assert torch.equal(bmax.view(torch.int16), c['best_max'].view(torch.int16))
    assert torch.equal(bmin.view(torch.int16), c['best_min'].view(torch.int16))
    wc = A.apply_clip(c['w'], bmax, bmin, bool(clip_sym))
    assert torch.equal(wc.view(torch.int16), c['w_clipped'].view(torch.int16))


@pytest.mark.parametrize('name', F.names('clipact_'))
def test_auto_clip_pc_act_matches_reference(name):
    """per_channel weights (group = ic) and activation fake-quant (w_only False): the oracle
    restatement against the reference's own auto_clip_layer, bit-equal."""
    c = F.load(name)
    wb, sym, clip_sym, nst, grp, abit, asym = c['meta'].tolist()
    group = c['w'].shape[1] if grp == -1 else grp
    bmax, bmin = A.clip_layer(c['w'], c['x'], wb, bool(sym), group, bool(clip_sym),
                              n_sample_token=nst, act=(abit, bool(asym)) if abit else None)
    assert torch.equal(bmax.view(torch.int16), c['best_max'].view(torch.int16))
    assert torch.equal(bmin.view(torch.int16), c['best_min'].view(torch.int16))
