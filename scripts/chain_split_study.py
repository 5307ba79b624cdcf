"""Study (CPU): accuracy of the factorisation chain X = chol(H)^-1 (gptq_core._chol_inv_rec)
when its fp32 products are emulated with bf16 MFMA operands split into 3 bf16 planes
(a = a0 + a1 + a2) and 6 (or 3) plane products summed in fp32 -- the candidate route to
~2.7x (5.3x) the fp32 MFMA rate on gfx950, where fp32 MFMA runs at 1/16 of bf16.

Products: fp32 GEMM (torch CPU) vs split emulation (plane products exact in fp64, each
segment's sum rounded to fp32 and accumulated in fp32, as an MFMA chain with fp32 acc).
Hessians: X^T X of heavy-tailed activations + 1 % mean-diagonal damping (gptq.py:161-170).
usage: chain_split_study.py [n] [tile]"""
import sys

import torch


def split3(a):
    a0 = a.to(torch.bfloat16)
    r = a - a0.float()
    a1 = r.to(torch.bfloat16)
    a2 = (r - a1.float()).to(torch.bfloat16)
    return [p.double() for p in (a0, a1, a2)]


PAIRS = {6: [(0, 0), (0, 1), (1, 0), (0, 2), (1, 1), (2, 0)], 3: [(0, 0), (0, 1), (1, 0)]}


def make_gemm(mode):
    def gemm(A, B):  # returns fp32 A @ B
        if mode == 'f32':
            return A @ B
        pa, pb = split3(A), split3(B)
        acc = torch.zeros(A.shape[0], B.shape[1], dtype=torch.float32)
        for i, j in PAIRS[mode]:
            acc = (acc.double() + (pa[i] @ pb[j]).float().double()).float()
        return acc
    return gemm


def chol_inv(A, gemm, tile):
    """X = chol(A)^-1 (lower), recursive as gptq_core._chol_inv_rec."""
    n = A.shape[0]
    if n <= tile:
        L = torch.linalg.cholesky(A.double()).float()
        return torch.linalg.inv(L.double()).float()
    n1 = max(tile, (n // 2 + tile - 1) // tile * tile)
    X11 = chol_inv(A[:n1, :n1], gemm, tile)
    L21 = gemm(A[n1:, :n1], X11.T.contiguous())
    A22 = A[n1:, n1:] - gemm(L21, L21.T.contiguous())
    X22 = chol_inv(A22, gemm, tile)
    T = gemm(L21, X11)
    X21 = -gemm(X22, T)
    X = torch.zeros_like(A)
    X[:n1, :n1], X[n1:, n1:], X[n1:, :n1] = X11, X22, X21
    return X


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    tile = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    torch.manual_seed(0)
    for trial, (tok, tail) in enumerate([(4 * n, 1.0), (4 * n, 3.0), (2 * n, 2.0)]):
        mag = torch.exp(torch.randn(n) * tail)
        x = torch.randn(tok, n, dtype=torch.float64) * mag
        H = x.T @ x / tok
        H += torch.eye(n, dtype=torch.float64) * 0.01 * H.diag().mean()
        ref = torch.linalg.inv(torch.linalg.cholesky(H))
        Hf = H.float()
        cond = torch.linalg.cond(H).item()
        line = [f'trial {trial}: n {n} cond {cond:.2e}']
        for mode in ('f32', 6, 3):
            X = chol_inv(Hf.clone(), make_gemm(mode), tile).double()
            err = ((X - ref).norm() / ref.norm()).item()
            rowerr = ((X - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
            line.append(f'{mode}: rel {err:.2e} max-row {rowerr:.2e}')
        print(' | '.join(line), flush=True)


if __name__ == '__main__':
    main()
