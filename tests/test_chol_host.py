"""Host-side block algebra of the recursive Cholesky-inverse (gptq_core): the triangle-aware
products and the lower SYRK update, checked in fp64 on CPU with tiny split sizes so every
split path runs."""
import pytest
import torch

from lightcompress_amd import gptq_core as g


def _torch_gemm(A, B, out, alpha, beta, b_trans=False):
    """CPU stand-in for lcq_gemm_f32 (the split logic is what is under test here)."""
    return out.addmm_(A, B.t() if b_trans else B, beta=beta, alpha=alpha)


@pytest.fixture
def small_splits(monkeypatch):
    monkeypatch.setattr(g, '_TRI_MIN', 8)
    monkeypatch.setattr(g, '_TILE', 4)
    monkeypatch.setattr(g, '_gemm', _torch_gemm)


@pytest.mark.parametrize('k', [7, 16, 40, 64])
def test_triangular_products(small_splits, k):
    torch.manual_seed(k)
    d = torch.float64
    A = torch.randn(30, k, dtype=d)
    X = torch.randn(k, k, dtype=d).tril()
    B = torch.randn(k, 20, dtype=d)
    out = torch.randn(30, k, dtype=d)
    ref = 0.5 * out + 2 * A @ X.t()
    g._mm_lowT(A, X, out, 2.0, 0.5)
    torch.testing.assert_close(out, ref)
    out = torch.randn(30, k, dtype=d)
    ref = 0.5 * out + 2 * A @ X
    g._mm_low_right(A, X, out, 2.0, 0.5)
    torch.testing.assert_close(out, ref)
    out = torch.randn(k, 20, dtype=d)
    ref = 0.5 * out + 2 * X @ B
    g._mm_low_left(X, B, out, 2.0, 0.5)
    torch.testing.assert_close(out, ref)
    L = torch.randn(k, 7, dtype=d)
    C = torch.randn(k, k, dtype=d)
    ref = (C - L @ L.t()).tril()
    g._syrk_lower(L, C, -1.0)
    torch.testing.assert_close(C.tril(), ref)
