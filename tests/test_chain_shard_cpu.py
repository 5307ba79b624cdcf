"""gptq_core.chain_sharding on CPU (gloo, world 2): the factorisation's large products are
computed by each rank for its row range and all-gathered in rank order -- U must equal the
unsharded chain bit for bit. The device kernels are replaced by CPU stand-ins whose every
output row is independent of the row range asked for (a full-shape fp64 product, rows taken
from it), the property lcq_gemm_f32_rows gives on the GPU (tests/test_multirank_gpu.py checks
the kernels themselves)."""
import functools
import sys
from pathlib import Path

import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from test_parallel_gloo import run2  # noqa: E402


def _cpu_kernels():
    from lightcompress_amd import ops

    def rows(A, B, out, alpha, beta, b_trans, r0, r1):
        full = A.double() @ (B.double().T if b_trans else B.double())
        new = alpha * full[r0:r1]
        if beta != 0.0:
            new = new + beta * out[r0:r1].double()
        out[r0:r1] = new.float()
        return out

    def tile(A, info, row0=0, L=None, out=None):
        out.copy_(torch.linalg.inv(torch.linalg.cholesky(A.double().tril()
                                                          + A.double().tril(-1).T)).float().tril())
        return out
    ops.gemm_f32 = lambda A, B, out, alpha=1.0, beta=0.0, b_trans=False: rows(
        A, B, out, alpha, beta, b_trans, 0, A.shape[0])
    ops.gemm_f32_rows = rows
    ops.gemm_f32x6 = lambda A, B, out, alpha, beta, b_trans, r0=0, r1=None: rows(
        A, B, out, alpha, beta, b_trans, r0, A.shape[0] if r1 is None else r1)
    ops.gemm_f32_row_unit = lambda m, n: 64
    ops.chol_inv_tile = tile


def _H(n):
    g = torch.Generator().manual_seed(n)
    X = torch.randn(n, 2 * n, generator=g)
    H = X @ X.T / (2 * n)
    H.diagonal().add_(0.05)
    return H


def _chain(rank, world, n=640, x6_tiles=10 ** 9):
    from lightcompress_amd import gptq_core, ops
    _cpu_kernels()
    gptq_core.SHARD_MIN_ROWS = 128
    ops.X6_MIN_TILES = x6_tiles   # 1: every product routed to the split-plane entry
    with gptq_core.chain_sharding(rank, world):
        U = gptq_core.inverse_cholesky_upper(_H(n))
    return U.numpy().tobytes(), gptq_core.shard_stats['split_products']


@pytest.mark.parametrize('x6_tiles', [10 ** 9, 1])
def test_chain_row_split_cpu_bit_identical(x6_tiles):
    single, split1 = run2(functools.partial(_chain, x6_tiles=x6_tiles), world=1)[0]   # in a child
    assert split1 == 0
    res = run2(functools.partial(_chain, x6_tiles=x6_tiles))
    for r in (0, 1):
        u, split = res[r]
        assert split > 0
        assert u == single, r
