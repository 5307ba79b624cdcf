"""GPU parity for static per-tensor activation calibration (lcq_minmax_segments,
lcq_act_static_qparams) against the reference's own outputs (tests/golden/actstatic_*.npz)
and torch's min / max."""
import pytest
import torch

import fixtures as F
from oracle import calib_ref as C

pytestmark = pytest.mark.gpu

CASES = F.names('actstatic_')
ALGOS = ['static_minmax', 'static_moving_minmax']


def _quantizer(name, c):
    from lightcompress_amd.quant import FloatQuantizer, IntegerQuantizer
    bit, sym, algo = int(c['meta'][2]), bool(c['meta'][3]), ALGOS[int(c['meta'][4])]
    if bit == 0:
        fmt = 'e4m3' if '_e4m3_' in name else 'e5m2'
        return FloatQuantizer(fmt, True, 'per_tensor', calib_algo=algo, use_qtorch=True)
    return IntegerQuantizer(bit, sym, 'per_tensor', calib_algo=algo)


def _entries(c, dev):
    ne, eb = int(c['meta'][0]), int(c['meta'][1])
    x = c['x'].to(dev)
    return [x] if ne == 1 else [x[j * eb:(j + 1) * eb] for j in range(ne)]


@pytest.mark.parametrize('name', CASES)
def test_static_qparams_vs_reference(dev, name):
    """scale / zero dtype equal to the reference's; static_moving_minmax bit-exact (every op
    rounded in the act dtype), static_minmax within one fp32 ulp (the reference's fp32 mean
    is a SIMD-width dependent cascade sum; ours rounds an fp64 sum once)."""
    c = F.load(name)
    q = _quantizer(name, c)
    sc, zc, qmn, qmx = q.get_batch_tensors_qparams(_entries(c, dev))
    s, z = sc[0].cpu(), zc[0].cpu()
    rs, rz = c['scales'].reshape(()), c['zeros'].reshape(())
    assert s.dtype == rs.dtype, (s.dtype, rs.dtype)
    assert z.float().item() == rz.float().item()
    if ALGOS[int(c['meta'][4])] == 'static_moving_minmax':
        assert torch.equal(s.reshape(()), rs)
    else:
        ulp = torch.finfo(torch.float32).eps * abs(rs.item())
        assert abs(s.item() - rs.item()) <= ulp, (s.item(), rs.item())
    if 'fq' in c:  # a_qdq with the device qparams: fake_quant_act_static
        args = dict(scales=sc[0], zeros=zc[0], qmax=qmx[0], qmin=qmn[0])
        fq = q.fake_quant_act_static(_entries(c, dev)[0], args).cpu()
        if torch.equal(s.reshape(()), rs):
            assert torch.equal(fq, c['fq'])


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16, torch.float32])
def test_minmax_segments_vs_torch(dev, dtype):
    """Ragged lengths (not multiples of 8), > 64 segments (several launches), one segment of
    16M elements (32 workgroups), infinities; exact."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(3)
    lens = [1, 7, 8, 9, 1023, 4096 + 5] + [777 + 16 * i for i in range(70)] + [1 << 24]
    segs = []
    for i, n in enumerate(lens):
        t = (torch.randn(n + 8, generator=g, device=dev) * (1 + i)).to(dtype)[:n]
        t = t.clone()  # 16-byte aligned allocation
        if i == 3:
            t[4] = float('inf')
        if i == 4:
            t[100] = float('-inf')
        segs.append(t)
    mm = ops.minmax_segments(segs).cpu()
    want = torch.tensor([[float(torch.min(t)), float(torch.max(t))] for t in segs])
    assert torch.equal(mm, want)


def test_minmax_segments_nan_propagates(dev):
    from lightcompress_amd import ops
    a = torch.randn(5000, device=dev, dtype=torch.bfloat16)
    b = a.clone()
    b[1234] = float('nan')
    mm = ops.minmax_segments([a, b]).cpu()
    assert not torch.isnan(mm[0]).any() and torch.isnan(mm[1]).all()
    s = ops.act_static_qparams(ops.minmax_segments([a, b]), 'static_minmax', 0.01,
                               torch.float32, torch.float32, True, -128.0, 127.0).cpu()
    assert torch.isnan(s[0])  # torch: the mean of a NaN range is NaN, so is the scale


def test_minmax_segments_rejects_bad_input(dev):
    from lightcompress_amd import ops
    x = torch.randn(64, device=dev, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        ops.minmax_segments([x[1:]])        # not 16-byte aligned
    with pytest.raises(ValueError):
        ops.minmax_segments([x[:0]])        # empty (torch.max raises)


def test_large_segment_qparams_oracle(dev):
    """Full-size shape (16 x 2048 x 4096 bf16 per entry, 4 entries) against the oracle."""
    from lightcompress_amd.quant import IntegerQuantizer
    g = torch.Generator(device=dev).manual_seed(5)
    entries = [(torch.randn(16, 2048, 4096, generator=g, device=dev) * (1 + i)).to(torch.bfloat16)
               for i in range(4)]
    for algo, sym in (('static_moving_minmax', False), ('static_minmax', True)):
        q = IntegerQuantizer(8, sym, 'per_tensor', calib_algo=algo)
        s, z, _, _ = q.get_batch_tensors_qparams(entries)
        (tensors,) = C.batch_entries([e.cpu() for e in entries])
        mn, mx = C.static_range(tensors, algo)
        rs, rz = C.qparams(mn, mx, *C.int_range(8, sym), sym)
        assert s[0].dtype == rs.dtype
        assert abs(s[0].cpu().item() - rs.item()) <= torch.finfo(torch.float32).eps * rs.item()
        assert z[0].cpu().float().item() == rz.float().item()


@pytest.mark.parametrize('name', F.names('acthist_'))
def test_static_hist_vs_reference(dev, name):
    """static_hist (quant.py:264-529) on the device: exact per-segment histograms, the
    reference's combination and threshold walk -> the same thresholded range and scale.
    (The reference's fp32 sums of the histogram / error vectors and its vectorised linspace
    are SIMD-width dependent; ours fix one order: T2, measured equal on every case.)"""
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    q = IntegerQuantizer(8, True, 'per_tensor', calib_algo='static_hist')
    sc, zc, _, _ = q.get_batch_tensors_qparams(_entries(c, dev))
    assert sc[0].dtype == torch.float32 and float(zc[0]) == 0.0
    rs = c['scales'].reshape(())
    assert torch.equal(sc[0].cpu().reshape(()), rs), (sc[0].item(), rs.item())


def test_static_hist_large_vs_oracle(dev):
    """16 calibration entries of 2048 x 1024 bf16 with growing ranges (every combination
    upscales) against the oracle."""
    from lightcompress_amd.quant import IntegerQuantizer
    g = torch.Generator().manual_seed(11)
    xs = [((torch.randn(1, 2048, 1024, generator=g) + 0.1) * (1 + 0.05 * i)).to(torch.bfloat16)
          for i in range(16)]
    q = IntegerQuantizer(8, True, 'per_tensor', calib_algo='static_hist')
    sc, _, _, _ = q.get_batch_tensors_qparams([x.to(dev) for x in xs])
    (tensors,) = C.batch_entries(xs)
    lo, hi = C.hist_range(tensors)
    rs, _ = C.qparams(lo, hi, *C.int_range(8, True), True)
    assert abs(sc[0].item() - rs.item()) <= 1e-3 * rs.item(), (sc[0].item(), rs.item())
