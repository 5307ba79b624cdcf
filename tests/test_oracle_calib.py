"""Pin the static activation-calibration oracle against the reference's own outputs
(tests/golden/actstatic_*.npz): every scale / zero bit-equal, and the int fake quant."""
import pytest
import torch

import fixtures as F
from oracle import calib_ref as C

CASES = F.names('actstatic_')
ALGOS = ['static_minmax', 'static_moving_minmax']


def case_entries(c):
    ne, eb = int(c['meta'][0]), int(c['meta'][1])
    x = c['x']
    return [x] if ne == 1 else [x[j * eb:(j + 1) * eb] for j in range(ne)]


def case_q(name, c):
    bit, sym = int(c['meta'][2]), bool(c['meta'][3])
    if bit == 0:  # FP8: qmax = finfo.max (quant.py:982-996)
        fi = torch.finfo(torch.float8_e4m3fn if '_e4m3_' in name else torch.float8_e5m2)
        return torch.tensor(fi.min), torch.tensor(fi.max), True
    qmin, qmax = C.int_range(bit, sym)
    return qmin, qmax, sym


@pytest.mark.parametrize('name', CASES)
def test_oracle_matches_reference(name):
    c = F.load(name)
    algo = ALGOS[int(c['meta'][4])]
    qmin, qmax, sym = case_q(name, c)
    (tensors,) = C.batch_entries(case_entries(c))
    mn, mx = C.static_range(tensors, algo)
    s, z = C.qparams(mn, mx, qmin, qmax, sym)
    assert s.dtype == c['scales'].dtype, (s.dtype, c['scales'].dtype)
    assert torch.equal(s.reshape(()), c['scales'].reshape(())), (s, c['scales'])
    assert torch.equal(z.float().reshape(()), c['zeros'].float().reshape(()))
    if 'fq' in c:
        fq = C.fake_quant_act_static_int(case_entries(c)[0], s, z, qmin, qmax)
        assert torch.equal(fq, c['fq'])


HIST = F.names('acthist_')


@pytest.mark.parametrize('name', HIST)
def test_hist_oracle_matches_reference(name):
    c = F.load(name)
    (tensors,) = C.batch_entries(case_entries(c))
    lo, hi = C.hist_range(tensors)
    assert torch.equal(lo.reshape(()), c['rmin'].reshape(())) and \
        torch.equal(hi.reshape(()), c['rmax'].reshape(()))
    s, _ = C.qparams(lo, hi, *C.int_range(8, True), True)
    assert torch.equal(s.reshape(()), c['scales'].reshape(()))
