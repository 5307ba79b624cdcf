"""GPTQ column loop with the near updates applied left-looking inside the block kernels
(lcq_gptq_block nprev > 0) against one lcq_gptq_trailing launch after each block: the same
per-element products (k-ordered fp32 fmaf chains, rounded, then subtracted in block order), so
the transformed weights, qparams and losses are bit-identical -- per-group, fixed per-channel,
static-groups, FP8 and OWQ column loops, ragged rows, partial last blocks and superblocks.
Reference: gptq.py:198-244 (W[:, i2:] -= Err1 @ Hinv[i1:i2, i2:])."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _upper(n, g, dev):
    """An upper-triangular fp32 U with a dominant positive diagonal (what the chain returns)."""
    A = torch.randn(n, n, generator=g) / n ** 0.5
    U = torch.triu(A, 1) + torch.diag(torch.rand(n, generator=g) + 0.5)
    return U.to(dev).contiguous()


def _run(monkeypatch, left, W, U, *args, **kw):
    from lightcompress_amd import gptq_core
    monkeypatch.setattr(gptq_core, 'LEFT_LOOKING', left)
    Wd = W.clone()
    out = gptq_core.column_loop(Wd, U, *args, losses=True, **kw)
    torch.cuda.synchronize()
    return Wd, out


def _same(a, b):
    if a is None or b is None:
        return a is None and b is None
    return torch.equal(a, b)


@pytest.mark.parametrize('rows,cols,mode', [
    (4096, 2304, 'group128'),      # superblocks of 8, 8 and 2 blocks
    (1000, 1100, 'group64'),       # ragged rows, a 76-column last block
    (640, 1536, 'fixed'),          # per-channel fixed qparams
    (512, 1280, 'static'),         # static groups (lcq_gptq_block_cols)
    (768, 1152, 'fp8'),            # FloatQuantizer weights
    (520, 1408, 'owq')])           # OWQ: the last 200 columns stay float
def test_left_looking_equals_trailing(dev, monkeypatch, rows, cols, mode):
    g = torch.Generator().manual_seed(rows + cols)
    W = (torch.randn(rows, cols, generator=g) * 0.02).to(dev)
    U = _upper(cols, g, dev)
    kw, args = {}, None
    if mode.startswith('group'):
        args = (4, False, int(mode[5:]), 0, 15)
    elif mode == 'fixed':
        s = (torch.rand(rows, generator=g) * 0.01 + 0.002).to(dev)
        z = torch.randint(0, 16, (rows,), generator=g).float().to(dev)
        args, kw = (4, False, None, 0, 15), {'fixed': (s, z)}
    elif mode == 'static':
        ngc = cols // 128
        s = (torch.rand(rows, ngc, generator=g) * 0.01 + 0.002).to(dev)
        z = torch.randint(0, 16, (rows, ngc), generator=g).float().to(dev)
        cg = (torch.randperm(cols, generator=g) // 128).to(torch.int32).to(dev)
        args, kw = (4, False, 128, 0, 15), {'fixed': (s, z), 'col_group': cg}
    elif mode == 'fp8':
        args, kw = (8, True, 128, -448, 448), {'fp8': torch.float8_e4m3fn}
    else:
        args, kw = (4, False, 128, 0, 15), {'ncols_q': cols - 200}
    W1, o1 = _run(monkeypatch, True, W, U, *args, **kw)
    W0, o0 = _run(monkeypatch, False, W, U, *args, **kw)
    assert torch.equal(W1, W0)
    assert all(_same(a, b) for a, b in zip(o1, o0))
    assert not torch.equal(W1, W)   # the loop did run


def test_left_looking_rows_shard_bit_identical(dev, monkeypatch):
    """A row range of the matrix (a token-sharded rank's rows) transforms exactly as those
    rows of the whole matrix: the left-looking products are per row."""
    g = torch.Generator().manual_seed(7)
    rows, cols = 1536, 2048
    W = (torch.randn(rows, cols, generator=g) * 0.02).to(dev)
    U = _upper(cols, g, dev)
    Wa, oa = _run(monkeypatch, True, W, U, 4, True, 128, -8, 7)
    Wb, ob = _run(monkeypatch, True, W[512:1024].contiguous(), U, 4, True, 128, -8, 7)
    assert torch.equal(Wa[512:1024], Wb)
    assert torch.equal(oa[0][512:1024], ob[0])
