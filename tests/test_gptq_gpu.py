"""GPU parity for GPTQ: MFMA Hessian, in-block column loop (bit-exact given U), and the full
layer transform vs reference golden vectors (parity tier T2)."""
import math

import pytest
import torch

import fixtures as F
from oracle import gptq_ref as G
from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu


def _meta(c):
    bit, sym, gs, act, oc, ic = c['meta'].tolist()
    return bit, bool(sym), gs, bool(act), oc, ic


@pytest.mark.parametrize('name', F.names('gptq_'))
def test_hessian_vs_reference(dev, name):
    from lightcompress_amd.gptq_core import HessianAccumulator
    c = F.load(name)
    ic = c['x'].shape[-1]
    acc = HessianAccumulator(ic, dev)
    for x in c['x']:
        acc.add_batch(x.unsqueeze(0).to(dev))
    H = acc.H.cpu()
    # fp64 reference of the same running average; tolerance relative to sum |x_i x_j|
    torch.testing.assert_close(H, c['H'], rtol=2e-5, atol=2e-5 * c['H'].abs().max().item())
    assert torch.equal(H, H.t()), 'Hessian must be exactly symmetric'


@pytest.mark.parametrize('n,ic,dt', [(2048, 4096, torch.bfloat16), (1000, 1032, torch.bfloat16),
                                     (37, 136, torch.bfloat16), (640, 8192, torch.bfloat16),
                                     (300, 520, torch.float16)])
def test_hessian_large_vs_fp64(dev, n, ic, dt):
    """Covers split-K (few tiles), the single-pass path (ic 8192: 528 tiles), ragged ic / n."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(n + ic)
    x = (torch.randn(n, ic, generator=g) * torch.exp(torch.randn(ic, generator=g))).to(dt)
    H = torch.full((ic, ic), 0.5, device=dev)
    ops.hessian_accum(x.to(dev), H, 0.25, 0.5)
    xd = x.double()
    ref = 0.25 * xd.t() @ xd + 0.25
    bound = 0.25 * (xd.abs().t() @ xd.abs()) + 0.25
    err = (H.cpu().double() - ref).abs()
    assert (err <= 1e-6 * bound + 1e-30).all(), (err / bound).max().item()
    assert torch.equal(H, H.t())


@pytest.mark.parametrize('group,sym', [(128, False), (64, True), (32, False)])
def test_single_block_bit_exact(dev, group, sym):
    """One 128-column block has no trailing GEMM: the kernel must equal the oracle exactly."""
    from lightcompress_amd import gptq_core
    g = torch.Generator().manual_seed(group)
    rows, cols = 300, 128
    W = torch.randn(rows, cols, generator=g) * 0.02
    A = torch.randn(cols, 2 * cols, generator=g)
    Hm = A @ A.t() / cols + 0.1 * torch.eye(cols)
    U = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(Hm)), upper=True)
    bit = 4
    qmin, qmax = (-8, 7) if sym else (0, 15)
    tmp, L, s, z = G.column_loop(W.clone(), U, bit, sym, group)
    Wd = W.clone().to(dev)
    s_d, z_d, L_d = gptq_core.column_loop(Wd, U.to(dev), bit, sym, group, qmin, qmax,
                                          losses=True)
    assert torch.equal(Wd.cpu(), tmp)
    assert torch.equal(s_d.cpu(), s)
    assert torch.equal(L_d.cpu(), L)
    if not sym:
        assert torch.equal(z_d.cpu(), z)


@pytest.mark.parametrize('rows,cols', [(77, 128), (300, 100)])
def test_single_block_fixed_qparams_bit_exact(dev, rows, cols):
    """per_channel GPTQ (fixed per-row qparams, group None), incl. a ragged last block."""
    from lightcompress_amd import gptq_core
    g = torch.Generator().manual_seed(rows)
    W = torch.randn(rows, cols, generator=g) * 0.02
    A = torch.randn(cols, 2 * cols, generator=g)
    Hm = A @ A.t() / cols + 0.1 * torch.eye(cols)
    U = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(Hm)), upper=True)
    mn, mx = W.amin(1, keepdim=True), W.amax(1, keepdim=True)
    s, z = Q.qparams(mn, mx, 0.0, 15, False)
    tmp, L, _, _ = G.column_loop(W.clone(), U, 4, False, None, fixed=(s, z))
    Wd = W.clone().to(dev)
    _, _, L_d = gptq_core.column_loop(Wd, U.to(dev), 4, False, None, 0, 15,
                                      fixed=(s.to(dev), z.to(dev)), losses=True)
    assert torch.equal(Wd.cpu(), tmp)
    assert torch.equal(L_d.cpu(), L)


@pytest.mark.parametrize('name', F.names('gptq_'))
def test_column_loop_given_reference_U(dev, name):
    from lightcompress_amd import gptq_core
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    qmin, qmax = Q.int_range(bit, sym)
    W = c['w'].float().clone()
    dead = torch.diag(c['H']) == 0
    W[:, dead] = 0
    if act:
        W = W[:, c['perm']]
    Wd = W.contiguous().to(dev)
    s, z, _ = gptq_core.column_loop(Wd, c['U'].to(dev), bit, sym, gs, int(qmin), int(qmax))
    w = Wd.cpu()
    if act:
        w = w[:, torch.argsort(c['perm'])]
    # only the trailing fp32 GEMM's summation order differs from the reference
    torch.testing.assert_close(w, c['weight'], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(s.cpu().reshape(-1, 1), c['scales'], rtol=1e-5, atol=1e-8)
    # T2: codes under the reference's qparams agree >= 99.9 %
    perm = c['perm'] if act else None
    def codes(wt):
        wp = wt[:, perm] if perm is not None else wt
        zz = c['zeros'] if not sym else torch.tensor(0.0)
        return Q.quant(Q.group_view(wp, 'per_group', gs), c['scales'], zz, qmin, qmax)
    agree = (codes(w) == codes(c['weight'])).float().mean().item()
    assert agree >= 0.999, agree


@pytest.mark.parametrize('name', F.names('gptqmse_'))
def test_mse_column_loop_given_reference_U(dev, name):
    """calib_algo mse in the loop (gptq.py:213-222): every group's range searched on the
    block-start columns (lcq_mse_qparams) and quantized by the block kernel with those
    qparams; given the reference's U only the trailing GEMM's fp32 order differs (T2)."""
    from lightcompress_amd import gptq_core
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    qmin, qmax = Q.int_range(bit, sym)
    wq = IntegerQuantizer(bit, sym, 'per_group', group_size=gs, calib_algo='mse')
    W = c['w'].float().clone()
    if act:
        W = W[:, c['perm']]
    Wd = W.contiguous().to(dev)

    def col_qparams(v):
        _, _, sg, zg = wq._mse(v.contiguous())
        return sg, zg
    s, z, _ = gptq_core.column_loop(Wd, c['U'].to(dev), bit, sym, gs, int(qmin), int(qmax),
                                    col_qparams=col_qparams)
    w = Wd.cpu()
    if act:
        w = w[:, torch.argsort(c['perm'])]
    torch.testing.assert_close(w, c['weight'], rtol=1e-4, atol=1e-6)
    same_s = (s.cpu().reshape(-1, 1) == c['scales']).float().mean().item()
    assert same_s >= 0.99, same_s   # a range search may flip where the columns moved in ulps
    perm = c['perm'] if act else None

    def codes(wt):
        wp = wt[:, perm] if perm is not None else wt
        zz = c['zeros'] if not sym else torch.tensor(0.0)
        return Q.quant(Q.group_view(wp, 'per_group', gs), c['scales'], zz, qmin, qmax)
    agree = (codes(w) == codes(c['weight'])).float().mean().item()
    assert agree >= 0.999, agree


@pytest.mark.parametrize('name', F.names('gptqmse_'))
def test_mse_plugin_layer_vs_reference(dev, name):
    """quantize_layer with an mse quantizer (the GPTQ plugin's path): deployed fake-quant
    weights >= 99.9 % bit-equal to the reference's."""
    from lightcompress_amd import gptq_core
    from lightcompress_amd.gptq_core import HessianAccumulator
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    wq = IntegerQuantizer(bit, sym, 'per_group', group_size=gs, calib_algo='mse')
    acc = HessianAccumulator(ic, dev)
    for x in c['x']:
        acc.add_batch(x.unsqueeze(0).to(dev))
    r = gptq_core.quantize_layer(c['w'].to(dev), acc.H, wq, actorder=act, percdamp=0.01)
    perm = r['perm']
    wp = r['weight'][:, perm] if perm is not None else r['weight']
    args = {'scales': r['scales'], 'zeros': r['zeros'], 'qmax': wq.qmax, 'qmin': wq.qmin}
    fq = wq.fake_quant_weight_static(wp.contiguous(), args).to(torch.bfloat16)
    if perm is not None:
        fq = fq[:, r['invperm']]
    same = (fq.cpu() == c['fq']).float().mean().item()
    assert same >= 0.999, same


@pytest.mark.parametrize('name', F.names('gptq_'))
def test_layer_end_to_end_vs_reference(dev, name):
    """Full device transform (MFMA Hessian + rocSOLVER Cholesky + HIP loop) vs reference:
    T2 tier — deployed codes equal >= 99.9 %, every difference a +/-1 step."""
    from lightcompress_amd import gptq_core
    from lightcompress_amd.gptq_core import HessianAccumulator
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    wq = IntegerQuantizer(bit, sym, 'per_group', group_size=gs)
    acc = HessianAccumulator(ic, dev)
    for x in c['x']:
        acc.add_batch(x.unsqueeze(0).to(dev))
    r = gptq_core.quantize_layer(c['w'].to(dev), acc.H, wq, actorder=act, percdamp=0.01)
    w_dev = r['weight']
    perm = r['perm']
    wp = w_dev[:, perm] if perm is not None else w_dev
    args = {'scales': r['scales'], 'zeros': r['zeros'], 'qmax': wq.qmax, 'qmin': wq.qmin}
    fq = wq.fake_quant_weight_static(wp.contiguous(), args).to(torch.bfloat16)
    if perm is not None:
        fq = fq[:, r['invperm']]
    fq = fq.cpu()
    ref = c['fq']
    # compare in code space: (fq / scale) steps
    same = (fq == ref).float().mean().item()
    assert same >= 0.999, same
    assert torch.allclose(fq.float(), ref.float(), atol=2 * c['scales'].abs().max().item())


@pytest.mark.parametrize('rows,ic,c0,K,c2', [(300, 512, 128, 128, None), (256, 4096, 0, 128, None),
                                            (129, 392, 128, 128, None), (200, 2048, 0, 1024, None),
                                            (200, 2048, 128, 128, 1024)])
@pytest.mark.parametrize('padded', [True, False])
def test_trailing_update(dev, rows, ic, c0, K, c2, padded):
    """lcq_gptq_trailing vs fp64 (incl. K = 1024 superblock updates and a column window), and
    bit-identical on any row sub-range (row sharding) and between its two kernels. padded: the
    k-major error rows padded to a multiple of 4 floats as the column loop allocates them (the
    LDS-DMA GEMM path whenever cnt % 32 == 0); unpadded ragged rows take the register-staged
    kernel."""
    from lightcompress_amd import ops

    def kmajor(e):   # [K, r] -> [K, ceil4(r)] (the column loop's layout) when padded
        if not padded:
            return e.contiguous()
        buf = torch.zeros(e.shape[0], -(-e.shape[1] // 4) * 4, device=dev)
        buf[:, :e.shape[1]] = e
        return buf

    g = torch.Generator(device=dev).manual_seed(rows + ic)
    W = torch.randn(rows, ic, generator=g, device=dev)
    U = torch.randn(ic, ic, generator=g, device=dev).triu().contiguous()
    err = torch.randn(K, rows, generator=g, device=dev)  # k-major, as lcq_gptq_block writes
    cnt = min(K, ic - c0)
    c1 = c0 + cnt
    end = ic if c2 is None else c2
    ref = W.double().clone()
    ref[:, c1:end] -= err.t()[:, :cnt].double() @ U[c0:c1, c1:end].double()
    out = W.clone()
    ops.gptq_trailing(out, c0, cnt, c1, kmajor(err), U, c2=end)
    assert torch.equal(out[:, :c1], W[:, :c1]) and torch.equal(out[:, end:], W[:, end:])
    tol = 1e-5 * math.sqrt(cnt) * (1 + ref[:, c1:end].abs())
    assert ((out[:, c1:end].double() - ref[:, c1:end]).abs() <= tol).all()
    h = rows // 3   # both kernels are the k-ordered fmaf chain: any row range, any path
    part = W[h:].clone()
    ops.gptq_trailing(part, c0, cnt, c1, kmajor(err[:, h:]), U, c2=end)
    assert torch.equal(part, out[h:])


@pytest.mark.parametrize('M,N,K', [(200, 136, 64), (1000, 700, 512), (2100, 2300, 1024),
                                   (128, 4096, 4096), (1792, 1792, 1792), (3000, 1900, 1792)])
@pytest.mark.parametrize('bt', [False, True])
@pytest.mark.parametrize('stream_k', [True, False])
def test_gemm_f32_dma(dev, M, N, K, bt, stream_k, monkeypatch):
    """lcq_gemm_f32's LDS-DMA kernel (16-byte aligned rows, K % 32 == 0: the recursion's
    products on 128-multiple Hessians) on sub-views of larger matrices: ragged M / N at both
    tile sizes, past-the-end rows / columns read as zero; against fp64 (same bound as above)
    and deterministic -- the tiled grids and, where the last round of 256 workgroups would
    run ragged (2100 x 2300, 1792^2, 3000 x 1900), the stream-K split with its k-ordered
    fixup of the cut tiles."""
    from lightcompress_amd import ops
    monkeypatch.setattr(ops, 'STREAM_K', stream_k)
    g = torch.Generator().manual_seed(M + 3 * N + K)
    big_a = torch.randn(M + 8, K + 8, generator=g)
    big_b = torch.randn((N + 4, K + 12) if bt else (K + 4, N + 12), generator=g)
    A = big_a[4:M + 4, 4:K + 4]
    B = big_b[:N, 8:K + 8] if bt else big_b[4:K + 4, :N]
    C0 = torch.randn(M, N + 4, generator=g)[:, :N]
    ref_p = A.double() @ (B.double().t() if bt else B.double())
    bound0 = A.double().abs() @ (B.double().abs().t() if bt else B.double().abs())
    Ad = big_a.to(dev)[4:M + 4, 4:K + 4]
    Bd = big_b.to(dev)[:N, 8:K + 8] if bt else big_b.to(dev)[4:K + 4, :N]
    for alpha, beta in ((1.0, 0.0), (-1.0, 1.0)):
        Cd = C0.to(dev).clone()
        if beta == 0.0:
            Cd.fill_(float('nan'))
        ops.gemm_f32(Ad, Bd, Cd, alpha, beta, b_trans=bt)
        ref = alpha * ref_p + (beta * C0.double() if beta else 0)
        bound = abs(alpha) * bound0 + abs(beta) * C0.double().abs()
        err = ((Cd.cpu().double() - ref).abs() / (bound + 1e-30)).max().item()
        assert err < 2e-6, (alpha, beta, err)
    C1 = torch.empty(M, N, device=dev)
    C2 = torch.empty(M, N, device=dev)
    ops.gemm_f32(Ad, Bd, C1, 1.0, 0.0, b_trans=bt)
    ops.gemm_f32(Ad, Bd, C2, 1.0, 0.0, b_trans=bt)
    assert torch.equal(C1, C2)


@pytest.mark.parametrize('M,N,K', [(1, 1, 1), (130, 77, 33), (256, 384, 128), (1000, 700, 517),
                                   (2048, 1536, 2048)])
@pytest.mark.parametrize('bt', [False, True])
def test_gemm_f32(dev, M, N, K, bt):
    """lcq_gemm_f32 (the recursion's addmm_): C = beta C + alpha A op(B) on strided fp32 views
    (sub-views of larger matrices, unaligned row starts), against fp64; beta 0 ignores a
    NaN-filled C."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(M * 7 + N + K)
    big_a = torch.randn(M + 3, K + 5, generator=g)
    big_b = torch.randn((N + 2, K + 3) if bt else (K + 2, N + 3), generator=g)
    A = big_a[1:M + 1, 1:K + 1]
    B = big_b[:N, 2:K + 2] if bt else big_b[2:K + 2, :N]
    C0 = torch.randn(M, N, generator=g)
    ref_p = A.double() @ (B.double().t() if bt else B.double())
    for alpha, beta in ((1.0, 0.0), (-1.0, 1.0), (0.5, 2.0)):
        Cd = C0.to(dev).clone()
        if beta == 0.0:
            Cd.fill_(float('nan'))
        Ad = big_a.to(dev)[1:M + 1, 1:K + 1]
        Bd = big_b.to(dev)[:N, 2:K + 2] if bt else big_b.to(dev)[2:K + 2, :N]
        ops.gemm_f32(Ad, Bd, Cd, alpha, beta, b_trans=bt)
        ref = alpha * ref_p + (beta * C0.double() if beta else 0)
        bound = (abs(alpha) * (A.double().abs() @ (B.double().abs().t() if bt else
                                                      B.double().abs()))
                 + abs(beta) * C0.double().abs())
        err = ((Cd.cpu().double() - ref).abs() / (bound + 1e-30)).max().item()
        assert err < 2e-6, (alpha, beta, err)


@pytest.mark.parametrize('n', [100, 128, 300, 1000, 4096, 4500])
def test_inverse_cholesky_upper(dev, n):
    """Recursive lcq factorisation: U^T U = H^-1 with U upper (fp64 check), equal to the
    reference chain cholesky -> cholesky_inverse -> cholesky(upper) to fp32 accuracy."""
    from lightcompress_amd import gptq_core
    g = torch.Generator().manual_seed(n)
    A = torch.randn(n, 2 * n, generator=g, dtype=torch.float64)
    H = A @ A.t() / n + 0.05 * torch.eye(n, dtype=torch.float64)
    U = gptq_core.inverse_cholesky_upper(H.float().to(dev)).double().cpu()
    assert torch.equal(U, U.triu())
    ref = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(H)), upper=True)
    rel = ((U - ref).abs().max() / ref.abs().max()).item()
    assert rel < 5e-4, rel


def test_inverse_cholesky_graph_replay(dev, monkeypatch):
    """The per-size captured chain (gptq_core._chain_graphed): the first call of a size runs
    eagerly and captures, later calls replay; every result equals the eager recursion's bit
    for bit, on new inputs of the same size (the static input is refilled each time)."""
    from lightcompress_amd import gptq_core
    n = 1536
    g = torch.Generator().manual_seed(5)
    Hs = []
    for _ in range(3):
        X = torch.randn(n, 2 * n, generator=g)
        H = X @ X.T / (2 * n)
        H.diagonal().add_(0.05)
        Hs.append(H.to(dev))
    gptq_core._chain_graphs.pop((torch.device(dev).index or 0, n), None)
    monkeypatch.setattr(gptq_core, 'CHAIN_GRAPHS', False)
    eager = [gptq_core.inverse_cholesky_upper(H.clone()) for H in Hs]
    monkeypatch.setattr(gptq_core, 'CHAIN_GRAPHS', True)
    graphed = [gptq_core.inverse_cholesky_upper(H.clone()) for H in Hs + Hs[:1]]
    assert (torch.device(dev).index or 0, n) in gptq_core._chain_graphs
    for a, b in zip(eager + eager[:1], graphed):
        assert torch.equal(a, b)


@pytest.mark.parametrize('M,N,K,bt', [(3584, 1792, 1792, 1), (4096, 128, 128, 0),
                                       (1000, 384, 256, 1)])
def test_gemm_f32_rows_match_full_plan(dev, M, N, K, bt):
    """lcq_gemm_f32_rows: row ranges cut on lcq_gemm_f32_row_unit, assembled, equal the
    whole-range call bit for bit (the same kernel plan per element), and the whole range equals
    the tiled lcq_gemm_f32 product to fp32 accuracy."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(M + N)
    A = torch.randn(M, K, generator=g, device=dev)
    B = torch.randn((N, K) if bt else (K, N), generator=g, device=dev)
    C0 = torch.randn(M, N, generator=g, device=dev)
    full = ops.gemm_f32_rows(A, B, C0.clone(), 0.5, 1.0, bool(bt), 0, M)
    unit = ops.gemm_f32_row_unit(M, N)
    parts = C0.clone()
    cuts = list(range(0, M, 3 * unit)) + [M]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        ops.gemm_f32_rows(A, B, parts, 0.5, 1.0, bool(bt), r0, r1)
    assert torch.equal(parts, full)
    ref = C0.double() + 0.5 * (A.double() @ (B.double().T if bt else B.double()))
    assert ((full.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    with pytest.raises(Exception):
        ops.gemm_f32_rows(A, B, parts, 0.5, 1.0, bool(bt), unit // 2, M)


@pytest.mark.parametrize('M,N,K', [(1000, 384, 517), (2048, 1536, 2048), (300, 96, 64),
                                   (3584, 1792, 1792)])
@pytest.mark.parametrize('bt', [False, True])
def test_gemm_f32x6(dev, M, N, K, bt):
    """lcq_gemm_f32x6 (fp32 product on bf16 MFMA over split planes): C = beta C + alpha A op(B)
    on strided fp32 views (ragged K padded to 64, transposed and K-major B), against fp64 with
    the same elementwise bound as test_gemm_f32; beta 0 ignores a NaN-filled C; its error is
    within 2x the fp32 kernel's on the same product."""
    from lightcompress_amd import ops
    g = torch.Generator().manual_seed(M * 5 + N + K)
    big_a = torch.randn(M + 3, K + 5, generator=g)
    big_b = torch.randn((N + 2, K + 3) if bt else (K + 2, N + 4), generator=g)
    A = big_a[1:M + 1, 1:K + 1]
    B = big_b[:N, 2:K + 2] if bt else big_b[2:K + 2, :N]
    C0 = torch.randn(M, N, generator=g)
    ref_p = A.double() @ (B.double().t() if bt else B.double())
    Ad = big_a.to(dev)[1:M + 1, 1:K + 1]
    Bd = big_b.to(dev)[:N, 2:K + 2] if bt else big_b.to(dev)[2:K + 2, :N]
    bound_p = A.double().abs() @ (B.double().abs().t() if bt else B.double().abs())
    for alpha, beta in ((1.0, 0.0), (-1.0, 1.0), (0.5, 2.0)):
        ref = alpha * ref_p + (beta * C0.double() if beta else 0)
        bound = abs(alpha) * bound_p + abs(beta) * C0.double().abs() + 1e-30
        Cd = C0.to(dev).clone()
        if beta == 0.0:
            Cd.fill_(float('nan'))
        ops.gemm_f32x6(Ad, Bd, Cd, alpha, beta, bt)
        err6 = ((Cd.cpu().double() - ref).abs() / bound).max().item()
        Cf = C0.to(dev).clone()
        ops.gemm_f32(Ad, Bd, Cf, alpha, beta, b_trans=bt)
        err32 = ((Cf.cpu().double() - ref).abs() / bound).max().item()
        assert err6 < 2e-6 and err6 <= 2 * err32 + 1e-7, (alpha, beta, err6, err32)


@pytest.mark.parametrize('M,N,K', [(3584, 1792, 1792), (1792, 1792, 7168)])
@pytest.mark.parametrize('bt', [False, True])
def test_gemm_f32x6_rows_match_full(dev, M, N, K, bt):
    """Row ranges of lcq_gemm_f32x6 (as a token-sharded chain cuts them) assembled equal the
    whole product bit for bit, also where K is split (fewer than 256 tiles: the split count
    comes from the full shape)."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(17)
    A = torch.randn(M, K, generator=g, device=dev)
    B = torch.randn((N, K) if bt else (K, N), generator=g, device=dev)
    C0 = torch.randn(M, N, generator=g, device=dev)
    full = ops.gemm_f32x6(A, B, C0.clone(), -1.0, 1.0, bt)
    parts = C0.clone()
    cuts = [0, 128, M // 2, M // 2 + 128, M]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        ops.gemm_f32x6(A, B, parts, -1.0, 1.0, bt, r0, r1)
    assert torch.equal(parts, full)


def test_gemm_f32x6_a_trans(dev):
    """A given k-major ([K, M] view, GPTQ's stacked Err1) equals the row-major call on the
    transposed copy bit for bit (same planes, same k order), also on row ranges with K unsplit
    (max_splits 1, the trailing update's setting)."""
    from lightcompress_amd import ops
    M, N, K = 1000, 768, 1024
    g = torch.Generator(device=dev).manual_seed(23)
    At = torch.randn(K, M + 8, generator=g, device=dev)[:, :M]
    B = torch.randn(K, N, generator=g, device=dev)
    C0 = torch.randn(M, N, generator=g, device=dev)
    a = ops.gemm_f32x6(At, B, C0.clone(), -1.0, 1.0, False, a_trans=True, max_splits=1)
    b = ops.gemm_f32x6(At.t().contiguous(), B, C0.clone(), -1.0, 1.0, False, max_splits=1)
    assert torch.equal(a, b)
    parts = C0.clone()
    for r0, r1 in ((0, 64), (64, 640), (640, M)):
        ops.gemm_f32x6(At, B, parts, -1.0, 1.0, False, r0, r1, a_trans=True, max_splits=1)
    assert torch.equal(parts, a)
    ref = C0.double() - At.double().t() @ B.double()
    assert ((a.double() - ref).abs().max() / ref.abs().max()).item() < 1e-6


def test_gptq_trailing_far_update_x6(dev, monkeypatch):
    """The superblock's far update (cnt >= TRAIL_X6_MIN_K) on lcq_gemm_f32x6 agrees with the
    fp32 kernel's to fp32 accuracy and is independent of the row count (row shards)."""
    from lightcompress_amd import ops
    rows, cols, cnt = 512, 3072, 1024
    g = torch.Generator(device=dev).manual_seed(29)
    W0 = torch.randn(rows, cols, generator=g, device=dev)
    err = torch.randn(cnt, rows, generator=g, device=dev) * 0.01
    U = torch.randn(cols, cols, generator=g, device=dev).triu() * 0.05
    out = {}
    for x6 in (True, False):
        monkeypatch.setattr(ops, 'X6', x6)
        W = W0.clone()
        ops.gptq_trailing(W, 0, cnt, cnt, err, U)
        out[x6] = W
    assert torch.equal(out[True][:, :cnt], W0[:, :cnt])
    d = (out[True] - out[False]).abs().max().item()
    assert d <= 1e-5 * out[False].abs().max().item(), d
    monkeypatch.setattr(ops, 'X6', True)
    Ws = W0[128:384].clone()
    ops.gptq_trailing(Ws, 0, cnt, cnt, err[:, 128:384].contiguous(), U)
    assert torch.equal(Ws, out[True][128:384])


def test_inverse_cholesky_x6_vs_fp32_products(dev, monkeypatch):
    """The chain with its large products on lcq_gemm_f32x6 (n 8192: the 4096 x 2048 updates
    go there) is as accurate as with every product on the fp32 kernels, against fp64."""
    from lightcompress_amd import gptq_core, ops
    n = 8192
    g = torch.Generator(device=dev).manual_seed(3)
    mag = torch.exp(torch.randn(n, generator=g, device=dev))
    X = torch.randn(2 * n, n, generator=g, device=dev) * mag
    H = X.T @ X / (2 * n)
    H.diagonal().add_(0.01 * H.diagonal().mean())
    Hd = H.double()
    ref = torch.linalg.cholesky(torch.cholesky_inverse(torch.linalg.cholesky(Hd)),
                                upper=True).cpu()
    monkeypatch.setattr(gptq_core, 'CHAIN_GRAPHS', False)
    errs = {}
    for x6 in (True, False):
        monkeypatch.setattr(ops, 'X6', x6)
        calls = [0]
        orig = ops.gemm_f32x6

        def spy(*a, **k):
            calls[0] += 1
            return orig(*a, **k)
        monkeypatch.setattr(ops, 'gemm_f32x6', spy)
        U = gptq_core.inverse_cholesky_upper(H.clone()).double().cpu()
        monkeypatch.setattr(ops, 'gemm_f32x6', orig)
        assert (calls[0] > 0) == x6
        errs[x6] = ((U - ref).norm() / ref.norm()).item()
    assert errs[True] <= 1.5 * errs[False] + 1e-7, errs


def test_inverse_cholesky_not_pd(dev):
    from lightcompress_amd import gptq_core
    H = torch.eye(256, device=dev)
    H[200, 200] = -1.0
    with pytest.raises(torch.linalg.LinAlgError):
        gptq_core.inverse_cholesky_upper(H)


@pytest.mark.parametrize('n', [1, 5, 16, 17, 100, 127, 128, -128])
def test_chol_inv_tile(dev, n):
    """lcq_chol_inv_tile on a strided view: L == torch cholesky, L X == I (fp32 accuracy).
    n = -128: a 16-byte aligned 128-tile with 4-aligned leading dim (the float4 load path)."""
    from lightcompress_amd import ops
    vec = n < 0
    n = abs(n)
    g = torch.Generator().manual_seed(n)
    A = torch.randn(n, 2 * n + 3, generator=g, dtype=torch.float64)
    H = A @ A.t() / n + 0.1 * torch.eye(n, dtype=torch.float64)
    if vec:
        big = torch.full((n + 8, n + 8), float('nan'), device=dev)
        view = big[4:4 + n, 4:4 + n]
    else:
        big = torch.full((n + 7, n + 9), float('nan'), device=dev)
        view = big[3:3 + n, 5:5 + n]
    view.copy_(H.float().to(dev))
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    X = ops.chol_inv_tile(view, info, L=view)
    assert int(info.item()) == 0
    Lref = torch.linalg.cholesky(H)
    L = view.double().cpu()
    assert ((L - Lref).abs().max() / Lref.abs().max()).item() < 1e-5
    assert torch.equal(X.cpu(), X.cpu().tril())
    eye = torch.eye(n, dtype=torch.float64)
    assert (Lref @ X.double().cpu() - eye).abs().max().item() < 1e-4
    assert torch.isnan(big[:3]).all() and torch.isnan(big[:, :3]).all()  # nothing outside the view
    assert torch.isnan(big[3 + n + vec:]).all() and torch.isnan(big[:, 4 + n + 1:]).all()


def test_chol_inv_tile_info(dev):
    from lightcompress_amd import ops
    H = torch.eye(100, device=dev)
    H[40, 40] = -2.0
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.chol_inv_tile(H, info, row0=256)
    assert int(info.item()) == 256 + 41


@pytest.mark.parametrize('sym,group', [(False, 128), (True, 128), (False, 64)])
def test_static_cols_equals_permuted_static(dev, sym, group):
    """lcq_int_quant_static_cols with col_group = invperm // group == GPTQ.w_qdq's
    fake_quant_static(W[:, perm]).to(bf16)[:, invperm], bit for bit."""
    from lightcompress_amd import ops
    from lightcompress_amd.quant import IntegerQuantizer
    g = torch.Generator().manual_seed(group + int(sym))
    rows, cols = 192, 1024
    W = (torch.randn(rows, cols, generator=g) * 0.02).to(dev)
    perm = torch.randperm(cols, generator=g).to(dev)
    invperm = torch.argsort(perm)
    wq = IntegerQuantizer(4, sym, 'per_group', group_size=group)
    Wp = W[:, perm].contiguous()
    _, s, z, _, _ = wq.get_tensor_qparams(Wp)
    args = {'scales': s, 'zeros': z if not sym else torch.tensor(0.0), 'qmax': wq.qmax,
            'qmin': wq.qmin}
    ref = wq.fake_quant_weight_static(Wp, args).to(torch.bfloat16)[:, invperm]
    cg = (invperm // group).to(torch.int32)
    qmin, qmax = wq._iq
    got = ops.int_quant_static_cols(W, cg, s.reshape(-1), None if sym else z.reshape(-1),
                                    qmin, qmax, ct_dtype=torch.float32,
                                    fq_dtype=torch.bfloat16)
    assert torch.equal(got.view(torch.int16), ref.contiguous().view(torch.int16))


# ---- static_groups (gptq.py:224-227) ---------------------------------------------------------
def _static_inputs(c, sym, act):
    W = c['w'].float().clone()
    dead = torch.diag(c['H']) == 0
    W[:, dead] = 0
    perm = c['perm'] if act else None
    if act:
        W = W[:, perm]
    rows = W.shape[0]
    s = c['scales'].reshape(rows, -1).float()
    z = None if sym else c['zeros'].reshape(rows, -1).float()
    return W, s, z, perm


@pytest.mark.parametrize('name', F.names('gptqsg_'))
def test_static_block_bit_exact_vs_oracle(dev, name):
    """lcq_gptq_block_cols on the first 128 permuted columns (no trailing GEMM): bit-exact
    against the oracle's static_groups column loop, losses included."""
    from lightcompress_amd import gptq_core
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    qmin, qmax = Q.int_range(bit, sym)
    W, s, z, perm = _static_inputs(c, sym, act)
    W = W[:, :128].contiguous()
    U = c['U'][:128, :128].contiguous()
    tmp, L, _, _ = G.column_loop(W.clone(), U, bit, sym, gs,
                                 static=(s, z, None if perm is None else perm[:128]))
    src = perm[:128] if perm is not None else torch.arange(128)
    cg = (src // gs).to(torch.int32).to(dev)
    Wd = W.to(dev)
    _, _, L_d = gptq_core.column_loop(Wd, U.to(dev), bit, sym, gs, int(qmin), int(qmax),
                                      fixed=(s.to(dev), None if z is None else z.to(dev)),
                                      losses=True, col_group=cg)
    assert torch.equal(Wd.cpu(), tmp)
    assert torch.equal(L_d.cpu(), L)


@pytest.mark.parametrize('name', F.names('gptqsg_'))
def test_static_column_loop_given_reference_U(dev, name):
    from lightcompress_amd import gptq_core
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    qmin, qmax = Q.int_range(bit, sym)
    W, s, z, perm = _static_inputs(c, sym, act)
    src = perm if perm is not None else torch.arange(ic)
    cg = (src // gs).to(torch.int32).to(dev)
    Wd = W.contiguous().to(dev)
    so, zo, _ = gptq_core.column_loop(Wd, c['U'].to(dev), bit, sym, gs, int(qmin), int(qmax),
                                      fixed=(s.to(dev), None if z is None else z.to(dev)),
                                      col_group=cg)
    assert so is None and zo is None  # static qparams are not re-estimated
    w = Wd.cpu()
    if act:
        w = w[:, torch.argsort(perm)]
    torch.testing.assert_close(w, c['weight'], rtol=1e-4, atol=1e-6)
    zz = c['zeros'] if not sym else torch.tensor(0.0)
    def codes(wt):  # need_perm is False: original column order
        return Q.quant(Q.group_view(wt, 'per_group', gs), c['scales'], zz, qmin, qmax)
    agree = (codes(w) == codes(c['weight'])).float().mean().item()
    assert agree >= 0.999, agree


@pytest.mark.parametrize('name', F.names('gptqsg_'))
def test_static_plugin_layer_vs_reference(dev, name):
    """The GPTQ plugin's layer_transform with static_groups (MFMA Hessian, device Cholesky,
    HIP loop) vs the reference: qparams untouched, deployed fake-quant >= 99.9 % equal, and
    real-quant codes from w_q equal where the weights agree."""
    from lightcompress_amd import gptq_core
    from lightcompress_amd.gptq import GPTQ
    from lightcompress_amd.gptq_core import HessianAccumulator
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, gs, act, oc, ic = _meta(c)
    wq = IntegerQuantizer(bit, sym, 'per_group', group_size=gs)
    layer = torch.nn.Linear(ic, oc, bias=False, device=dev, dtype=torch.bfloat16)
    layer.weight.data = c['w'].to(dev)
    s0 = c['scales'].to(dev)
    layer.register_buffer('buf_scales', s0.clone())
    if not sym:
        layer.register_buffer('buf_zeros', c['zeros'].to(dev).clone())
    layer.register_buffer('buf_qmax', wq.qmax.clone().to(dev))
    layer.register_buffer('buf_qmin', wq.qmin.clone().to(dev))
    obj = GPTQ.__new__(GPTQ)
    obj.wquantizer = wq
    obj.actorder, obj.static_groups, obj.percdamp = act, True, 0.01
    obj.need_perm = False
    obj.model_dtype = torch.bfloat16
    obj.config = {}
    acc = HessianAccumulator(ic, dev)
    for x in c['x']:
        acc.add_batch(x.unsqueeze(0).to(dev))
    acc.prepared = None
    obj.layers_cache = {'l': {'acc': acc, 'owner': True, 'columns': ic}}
    obj.parallel_mode = lambda: 'single'
    obj.layer_transform(layer, 'l')
    assert torch.equal(layer.buf_scales, s0)  # gptq.py:195: static groups keep their qparams
    fq = obj.w_qdq(layer, wq).cpu()
    same = (fq == c['fq']).float().mean().item()
    assert same >= 0.999, same
    assert torch.allclose(fq.float(), c['fq'].float(), atol=2 * c['scales'].abs().max().item())
    codes, _, _ = obj.w_q(layer, wq)
    eq = (codes.cpu() == c['codes']).float().mean().item()
    assert eq >= 0.999, eq


# ---- OWQ (gptq.py:44-83) -----------------------------------------------------------------
@pytest.mark.parametrize('name', F.names('gptqowq_'))
def test_owq_plugin_layer_vs_reference(dev, name):
    """GPTQ plugin layer_transform with OWQ: same permutation (outlier columns last), float
    outlier columns restored by w_qdq, deployed weights >= 99.9 % bit-equal (T2), qparams of
    the quantized groups close, the remaining groups the construction ones."""
    from lightcompress_amd.gptq import GPTQ
    from lightcompress_amd.gptq_core import HessianAccumulator
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, gs, nout, oc, ic = c['meta'].tolist()
    sym = bool(sym)
    wq = IntegerQuantizer(bit, sym, 'per_group', group_size=gs)
    layer = torch.nn.Linear(ic, oc, bias=False, device=dev, dtype=torch.bfloat16)
    layer.weight.data = c['w'].to(dev)
    _, s0, z0, _, _ = wq.get_tensor_qparams(layer.weight.data)
    layer.register_buffer('buf_scales', s0)
    if not sym:
        layer.register_buffer('buf_zeros', z0)
    layer.register_buffer('buf_qmax', wq.qmax.clone().to(dev))
    layer.register_buffer('buf_qmin', wq.qmin.clone().to(dev))
    obj = GPTQ.__new__(GPTQ)
    obj.wquantizer = wq
    obj.actorder, obj.static_groups, obj.percdamp, obj.owq = False, False, 0.01, True
    obj.need_perm = True
    obj.n_out_dict = {'l': nout}
    obj.model_dtype = torch.bfloat16
    acc = HessianAccumulator(ic, dev)
    for x in c['x']:
        acc.add_batch(x.unsqueeze(0).to(dev))
    obj.layers_cache = {'l': {'acc': acc, 'owner': True, 'columns': ic}}
    obj.parallel_mode = lambda: 'single'
    obj.layer_transform(layer, 'l')
    assert torch.equal(layer.buf_perm.cpu(), c['perm'])
    assert int(layer.buf_n_nonout) == ic - nout
    s, rs = layer.buf_scales.cpu().reshape(oc, -1), c['scales'].reshape(oc, -1)
    assert s.shape == rs.shape
    ngq = -(-(ic - nout) // gs)
    torch.testing.assert_close(s[:, :ngq], rs[:, :ngq], rtol=1e-3, atol=1e-6)
    assert torch.equal(s[:, ngq:], rs[:, ngq:])
    fq = obj.w_qdq(layer, wq).cpu()
    same = (fq == c['fq']).float().mean().item()
    assert same >= 0.999, same
    # the float outlier columns: compensated weights (trailing updates), not quantized
    outl = c['perm'][ic - nout:]
    torch.testing.assert_close(fq[:, outl].float(), c['fq'][:, outl].float(), rtol=2e-2,
                               atol=1e-3)


@pytest.mark.parametrize('name', F.names('gptqowqpc_'))
def test_owq_per_channel_plugin_layer_vs_reference(dev, name):
    """GPTQ plugin layer_transform with OWQ and per_channel weights (gptq.py:157-166): the
    per-channel qparams come from the permuted non-outlier fp32 columns (bit-exact), deployed
    weights >= 99.9 % bit-equal (T2)."""
    from lightcompress_amd.gptq import GPTQ
    from lightcompress_amd.gptq_core import HessianAccumulator
    from lightcompress_amd.quant import IntegerQuantizer
    c = F.load(name)
    bit, sym, _, nout, oc, ic = c['meta'].tolist()
    sym = bool(sym)
    wq = IntegerQuantizer(bit, sym, 'per_channel')
    layer = torch.nn.Linear(ic, oc, bias=False, device=dev, dtype=torch.bfloat16)
    layer.weight.data = c['w'].to(dev)
    _, s0, z0, _, _ = wq.get_tensor_qparams(layer.weight.data)
    layer.register_buffer('buf_scales', s0)
    if not sym:
        layer.register_buffer('buf_zeros', z0)
    layer.register_buffer('buf_qmax', wq.qmax.clone().to(dev))
    layer.register_buffer('buf_qmin', wq.qmin.clone().to(dev))
    obj = GPTQ.__new__(GPTQ)
    obj.wquantizer = wq
    obj.actorder, obj.static_groups, obj.percdamp, obj.owq = False, False, 0.01, True
    obj.need_perm = True
    obj.n_out_dict = {'l': nout}
    obj.model_dtype = torch.bfloat16
    acc = HessianAccumulator(ic, dev)
    for x in c['x']:
        acc.add_batch(x.unsqueeze(0).to(dev))
    obj.layers_cache = {'l': {'acc': acc, 'owner': True, 'columns': ic}}
    obj.parallel_mode = lambda: 'single'
    obj.layer_transform(layer, 'l')
    assert torch.equal(layer.buf_perm.cpu(), c['perm'])
    assert layer.buf_scales.dtype == torch.float32
    torch.testing.assert_close(layer.buf_scales.cpu(), c['scales'], rtol=1e-6, atol=0)
    if not sym:
        torch.testing.assert_close(layer.buf_zeros.cpu(), c['zeros'], rtol=0, atol=0)
    fq = obj.w_qdq(layer, wq).cpu()
    same = (fq == c['fq']).float().mean().item()
    assert same >= 0.999, same


@pytest.mark.parametrize('n,tpe,ic', [(128, 64, 512), (5, 100, 264), (16, 2048, 4096)])
def test_grouped_hessian_world_independent(dev, n, tpe, ic):
    """The grouped Hessian of one process equals the subtrees of 2 / 4 / 8 token shards
    finished by the same tree, bit for bit; and it is the running-average Hessian up to fp32
    summation order (<= 1e-6 of sum |x_i x_j| against fp64)."""
    from lightcompress_amd import gptq_core, ops
    g = torch.Generator().manual_seed(n + ic)
    x = (torch.randn(n, tpe, ic, generator=g) *
         torch.exp(torch.randn(ic, generator=g))).to(torch.bfloat16).to(dev)
    one = gptq_core.HessianAccumulator(ic, dev, plan=gptq_core.GroupPlan(n))
    one.add_batch(x)
    assert one.grouped
    H1 = one.finalize().clone()
    for world in (2, 4, 8):
        subs = []
        for r in range(world):
            plan = gptq_core.GroupPlan(n, r, world)
            acc = gptq_core.HessianAccumulator(ic, dev, plan=plan)
            xs = x[plan.first:plan.first + plan.n_local]
            if plan.n_local:
                acc.add_batch(xs)
            assert acc.ready_grouped()
            subs.append(acc.subtree)
        H = ops.tree_sum(subs, gptq_core._alpha(n))
        assert torch.equal(H, H1), world
    xd = x.reshape(-1, ic).double()
    ref = (2 / n) * xd.t() @ xd
    bound = (2 / n) * xd.abs().t() @ xd.abs()
    err = (H1.double() - ref).abs()
    assert (err <= 2e-6 * bound + 1e-30).all().item(), (err / bound).max().item()
    assert torch.equal(H1, H1.t())


@pytest.mark.parametrize('n', [1000, 4096])
def test_gather_rc_equals_torch_prepare(dev, n):
    """lcq_gather_rc (one pass) against the torch form of gptq.py:58-64, 128-176 it replaces:
    H[dead, dead] = 1; H[perm][:, perm]; + damp on the diagonal; flipped for the chain
    (J H J) -- and on the weight: fp32 widening, dead columns zeroed, column gather, and the
    inverse permutation afterwards. Bit-equal."""
    from lightcompress_amd import ops
    g = torch.Generator(device=dev).manual_seed(n)
    X = torch.randn(n, n + 7, generator=g, device=dev)
    H = X @ X.T
    dead = torch.zeros(n, dtype=torch.bool, device=dev)
    dead[torch.randperm(n, generator=g, device=dev)[:5]] = True
    H[dead, :] = 0
    H[:, dead] = 0
    perm = torch.randperm(n, generator=g, device=dev)
    damp = 0.01 * torch.mean(torch.where(dead, torch.ones_like(torch.diag(H)),
                                         torch.diag(H))[perm])
    ref = H.clone()
    idx = torch.nonzero(dead).flatten()
    ref[idx, idx] = 1
    ref = ref[perm][:, perm]
    d = torch.arange(n, device=dev)
    ref[d, d] += damp
    ref = ref.flip(0, 1).contiguous()
    rev = perm.flip(0)
    got = ops.gather_rc(H, rsrc=rev, csrc=rev, dead_diag=dead, damp=damp)
    assert torch.equal(got, ref)
    W = (torch.randn(300, n, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    wref = W.float().clone()
    wref[:, dead] = 0
    wref = wref[:, perm].contiguous()
    wgot = ops.gather_rc(W, csrc=perm, dead_col=dead)
    assert torch.equal(wgot, wref)
    inv = torch.argsort(perm)
    assert torch.equal(ops.gather_rc(wgot, csrc=inv), wref[:, inv])


def test_gather_rc_wider_than_lds(dev):
    """Rows of 53248 fp32 columns (Llama-3.1-405B down_proj IC) exceed one LDS image: the
    unstaged path must give the same gathers (weight side, and a row slice of the Hessian side
    with the dead-diagonal fix and damp on the rows that hold the diagonal)."""
    from lightcompress_amd import ops
    n = 53248
    g = torch.Generator(device=dev).manual_seed(7)
    perm = torch.randperm(n, generator=g, device=dev)
    dead = torch.zeros(n, dtype=torch.bool, device=dev)
    dead[perm[:9]] = True
    W = (torch.randn(64, n, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    wref = W.float().clone()
    wref[:, dead] = 0
    wref = wref[:, perm].contiguous()
    assert torch.equal(ops.gather_rc(W, csrc=perm, dead_col=dead), wref)
    Hrows = torch.randn(48, n, generator=g, device=dev)   # the source rows 0..47 of H
    rsrc = torch.arange(48, device=dev)
    damp = torch.tensor(0.5, device=dev)
    csrc = torch.cat([torch.arange(48, device=dev), perm[perm >= 48][: n - 48]])
    got = ops.gather_rc(Hrows, rsrc=rsrc, csrc=csrc, dead_diag=dead, damp=damp)
    ref = Hrows[:, csrc].clone()
    d = torch.arange(48, device=dev)
    diag = torch.where(dead[csrc[:48]], torch.ones(48, device=dev), ref[d, d])
    ref[d, d] = diag + damp
    assert torch.equal(got, ref)
