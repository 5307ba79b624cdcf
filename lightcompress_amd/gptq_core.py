"""Device GPTQ layer transform (the math of GPTQ.layer_transform, gptq.py:113-244).

Kept separate from the plugin class (``gptq.py``) so the algorithm can be driven per layer
(tests, bench, multi-GPU row sharding) without a model.
"""
from __future__ import annotations

import contextlib
import math

import torch

from . import ops

BLOCK = 128
SUPERBLOCK = 1024  # column_loop's two-level trailing update (see there)


HESSIAN_GROUPS = 8  # fixed calibration-sample groups of the grouped Hessian (see below)


def _alpha(n: int) -> float:
    """fp32(sqrt(2 / n))^2: the reference's per-sample scale x <- sqrt(2/n) x, squared."""
    c = torch.tensor(math.sqrt(2 / n), dtype=torch.float32).item()
    return float(torch.tensor(c * c, dtype=torch.float32).item())


def group_bounds(n: int, groups: int = HESSIAN_GROUPS) -> list[tuple[int, int]]:
    """Sample range of every Hessian group: group g = samples s with floor(s * G / n) == g,
    i.e. [ceil(g n / G), ceil((g + 1) n / G)). Ranks of a world that divides G take
    contiguous blocks of G / world groups, which is also a balanced sample split."""
    return [(-(-g * n // groups), -(-(g + 1) * n // groups)) for g in range(groups)]


class GroupPlan:
    """Where this process's calibration samples sit in the grouped Hessian: the global sample
    count, and the local groups as (group, first local sample, end local sample)."""

    def __init__(self, n_global: int, rank: int = 0, world: int = 1,
                 groups: int = HESSIAN_GROUPS):
        if groups % world:
            raise ValueError('world size must divide the Hessian group count')
        self.n_global, self.rank, self.world, self.groups = n_global, rank, world, groups
        per = groups // world
        b = group_bounds(n_global, groups)
        self.first = b[rank * per][0]
        self.local = [(g, b[g][0] - self.first, b[g][1] - self.first)
                      for g in range(rank * per, (rank + 1) * per)]
        self.n_local = b[(rank + 1) * per - 1][1] - self.first


class HessianAccumulator:
    """Running-average Hessian of one linear input (GPTQ.add_batch, gptq.py:253-295).

    ``H_n = H_{n-1} * n_{prev}/n + (2/n) x^T x`` per calibration batch, with the product on
    MFMA (``lcq_hessian_accum``).

    Grouped form (``plan`` set and the whole calibration set of this process arrives in ONE
    batch, as the stacked calibration forward delivers it): the samples are cut into
    HESSIAN_GROUPS fixed groups, each group's x^T x is one MFMA pass into its own fp32
    partial, and H = alpha(n) * ((P0 + P1) + (P2 + P3)) + ((P4 + P5) + (P6 + P7)) -- one
    fixed binary tree (``lcq_tree_sum``). A rank of a token-sharded world keeps only its
    contiguous subtree; ``finalize`` exchanges the subtrees and finishes the same tree, so
    every rank ends with the single-GPU H bit for bit. Any other arrival
    pattern (several batches) falls back to the running average, and sharded ranks then
    combine by a weighted all-reduce (T2: the fp32 summation order differs).
    """

    def __init__(self, ic: int, device, plan: GroupPlan | None = None):
        self.H = torch.zeros((ic, ic), dtype=torch.float32, device=device)
        self.nsamples = 0
        self.ic = ic
        self.prepared = None  # (U, perm, dead) once the layer transform has factored H
        self.plan = plan
        self.subtree = None   # grouped: this process's unscaled tree over its local groups

    @property
    def grouped(self) -> bool:
        return self.subtree is not None

    @torch.no_grad()
    def add_batch(self, inp: torch.Tensor, samples: int | None = None):
        """`samples`: how many of the reference's add_batch calls this batch stands for
        (default: the batch dim of a 3-D input, 1 for a 2-D one)."""
        if inp.dim() == 2:
            inp = inp.unsqueeze(0)
        b = inp.shape[0] if samples is None else samples
        x = inp.reshape(-1, inp.shape[-1])
        if x.dtype not in (torch.bfloat16, torch.float16):
            x = x.to(torch.bfloat16)  # fp32 activations: bf16 MFMA path (documented tolerance)
        if (self.plan is not None and self.nsamples == 0 and not self.grouped
                and b == self.plan.n_local and inp.dim() == 3 and inp.shape[0] == b
                and b > 0):
            self._add_grouped(x, inp.shape[1])
            self.nsamples = b
            return
        if self.grouped:  # a second batch: continue as the running average of the local set
            self._materialize_local()
        beta = self.nsamples / (self.nsamples + b)
        self.nsamples += b
        ops.hessian_accum(x, self.H, _alpha(self.nsamples), beta)

    def _add_grouped(self, x: torch.Tensor, tpe: int):
        """Every local group's x^T x and their fixed tree in ONE launch (lcq_hessian_grouped):
        the whole H at world 1 (alpha(n)), else this rank's unscaled subtree."""
        bounds = [0] + [s1 * tpe for _, _, s1 in self.plan.local]
        if self.plan.world == 1:
            ops.hessian_grouped(x, bounds, self.H, _alpha(self.plan.n_global))
            self.subtree = self.H
            self.finalized = True
        else:
            self.subtree = ops.hessian_grouped(x, bounds, torch.empty_like(self.H), 1.0)
            self.finalized = False

    def ready_grouped(self) -> bool:
        """Grouped and waiting for (or done with) the cross-rank tree. A rank whose share of
        the samples is empty never sees a batch: its subtree is zero."""
        if (not self.grouped and self.plan is not None and self.plan.n_local == 0
                and self.nsamples == 0):
            self.subtree = torch.zeros_like(self.H)
            self.finalized = self.plan.world == 1
        return self.grouped

    def fallback(self):
        """Leave the grouped form (the ranks disagree): H = the local running average."""
        if self.grouped:
            self._materialize_local()

    def _materialize_local(self):
        """grouped -> running average over the local samples (the fallback)."""
        if not getattr(self, 'finalized', False):
            if self.plan.n_local:
                ops.tree_sum([self.subtree], _alpha(self.plan.n_local), out=self.H)
            else:
                self.H.zero_()
        self.subtree = None
        self.plan = None

    @torch.no_grad()
    def finalize(self):
        """Grouped and token-sharded: finish the tree across ranks (every rank gets H).
        RCCL: all_to_all of the subtrees' row slices, the upper tree levels on this rank's
        slice, all_gather of the slices; gloo (CPU-side tests): all_gather of whole subtrees."""
        if not self.grouped or self.finalized:
            return self.H
        import torch.distributed as dist
        world = self.plan.world
        flat = self.subtree.reshape(-1)
        n = flat.numel()
        alpha = _alpha(self.plan.n_global)
        if dist.get_backend() == 'nccl':
            chunk = -(-n // (4 * world)) * 4
            src = torch.zeros(chunk * world, dtype=torch.float32, device=flat.device)
            src[:n] = flat
            got = torch.empty_like(src)
            dist.all_to_all_single(got, src)
            mine = torch.empty(chunk, dtype=torch.float32, device=flat.device)
            ops.tree_sum([got[r * chunk:(r + 1) * chunk] for r in range(world)], alpha,
                         out=mine)
            full = torch.empty_like(src)
            dist.all_gather_into_tensor(full, mine)
            self.H.reshape(-1).copy_(full[:n])
        else:
            subs = [torch.empty_like(self.subtree) for _ in range(world)]
            dist.all_gather(subs, self.subtree.contiguous())
            ops.tree_sum(subs, alpha, out=self.H)
        self.subtree = self.H
        self.finalized = True
        return self.H


@torch.no_grad()
def prepare_hessian(H: torch.Tensor, actorder: bool, percdamp: float, owq_nout: int = 0):
    """Hessian side of gptq.py:58-64, 128-176 (H is consumed): act-order permutation, dead
    columns (diag 0 -> 1), damping, and U = upper Cholesky factor of H^-1.

    The reference computes U as cholesky(H) -> cholesky_inverse -> cholesky(upper). By
    uniqueness of the Cholesky factor, with J the reversal permutation,
    U = J chol(J H J)^-1 J: one factorisation and one triangular inverse instead of three
    dense factor/inverse steps (2.5x faster on MI355X at IC 14336, same U to ~1e-6). Returns
    (U, perm | None, dead mask)."""
    perm = torch.argsort(torch.diag(H), descending=True, stable=True) if actorder else None
    if owq_nout:
        # OWQ (gptq.py:58-83, actorder off): the n_out largest-diag columns (outliers) move to
        # the end and stay in float; the rest keep their order
        desc = torch.argsort(torch.diag(H), descending=True, stable=True)
        keep = torch.ones(H.shape[0], dtype=torch.bool, device=H.device)
        keep[desc[:owq_nout]] = False
        perm = torch.cat([torch.arange(H.shape[0], device=H.device)[keep], desc[:owq_nout]])
    # gptq.py:58-64, 128-176 in one gather pass (lcq_gather_rc): dead diagonal -> 1, the
    # act-order permutation, damp = percdamp * mean(diag) on the diagonal, written reversed
    # (J H J) straight into the chain's input -- the torch form (two index gathers, a flip copy,
    # a diagonal add) reads and writes the n^2 fp32 matrix four times
    d = torch.diag(H)
    dead = d == 0
    dfix = torch.where(dead, torch.ones_like(d), d)
    damp = percdamp * torch.mean(dfix if perm is None else dfix[perm])
    n = H.shape[0]
    rev = (perm if perm is not None else torch.arange(n, device=H.device)).flip(0)
    U = _inverse_cholesky_upper_filled(
        lambda buf: ops.gather_rc(H, rsrc=rev, csrc=rev, dead_diag=dead, damp=damp, out=buf),
        n, H.device)
    return U, perm, dead


# Products with at least SHARD_MIN_ROWS output rows (at n 14336: the ~20 of ~600 launches that
# carry ~60 % of the chain's flops) run on the tiled kernel planned for their full shape
# (lcq_gemm_f32_rows; never stream-K -- measured equal at n 14336, 39.09 vs 39.51 ms) in every
# world, so that a token-sharded run (chain_sharding) can row-split them over its ranks and
# all-gather the row blocks in rank order with every element computed exactly as on one GPU.
SHARD_MIN_ROWS = 3584
_chain_shard = None          # (rank, world) while a sharded chain runs
shard_stats = {'split_products': 0, 'gathered_rows': 0}   # per process, for tests / probes


@contextlib.contextmanager
def chain_sharding(rank: int, world: int):
    """Row-split the large products of every factorisation run inside this context over the
    `world` ranks of the default process group (each rank must hold the same Hessian: token
    shards after the Hessian's fixed-tree finish, or replicas). The sharded chain runs eagerly
    (an all-gather sits inside it) and without the side-stream overlap (one collective order
    on every rank); results are bit-identical to the unsharded chain."""
    global _chain_shard
    prev = _chain_shard
    _chain_shard = (rank, world) if world > 1 else None
    try:
        yield
    finally:
        _chain_shard = prev


def _gemm(A, B, out, alpha, beta, b_trans=False):
    """out = beta out + alpha A op(B): the recursion's products. Products with enough output
    tiles run on bf16 MFMA over split planes (lcq_gemm_f32x6: fp32 accuracy, ~2x the fp32
    MFMA rate), the rest on the fp32 MFMA kernels (lcq_gemm_f32 / _rows)."""
    M = out.shape[0]
    x6 = ops.gemm_f32x6_fits(M, out.shape[1], A.shape[1], out)
    if M < SHARD_MIN_ROWS:
        if x6:
            return ops.gemm_f32x6(A, B, out, alpha, beta, b_trans)
        return ops.gemm_f32(A, B, out, alpha, beta, b_trans=b_trans)
    sh = _chain_shard
    if sh is None:
        if x6:
            return ops.gemm_f32x6(A, B, out, alpha, beta, b_trans)
        return ops.gemm_f32_rows(A, B, out, alpha, beta, b_trans, 0, M)
    from . import parallel as P
    rank, world = sh
    unit = ops.gemm_f32_row_unit(M, out.shape[1])
    ranges = [tuple(min(u * unit, M) for u in P.row_shard(-(-M // unit), r, world))
              for r in range(world)]
    r0, r1 = ranges[rank]
    if x6:
        ops.gemm_f32x6(A, B, out, alpha, beta, b_trans, r0, r1)
    else:
        ops.gemm_f32_rows(A, B, out, alpha, beta, b_trans, r0, r1)
    full = P.gather_ranges(out[r0:r1], ranges)   # rank order: rows 0 .. M
    out.copy_(full)
    shard_stats['split_products'] += 1
    shard_stats['gathered_rows'] += M - (r1 - r0)
    return out


_TILE = 128
_TRI_MIN = 1024  # triangular / symmetric products split while both halves stay >= this


def _split(n):
    return max(_TILE, (n // 2 + _TILE - 1) // _TILE * _TILE)


def _mm_lowT(A, Xl, out, alpha, beta):
    """out = beta out + alpha A Xl^T, Xl lower-triangular: A Xl^T = [A1 X11^T, A1 X21^T + A2 X22^T]
    -- the zero block skipped, 3/4 of the flops per split level."""
    k = Xl.shape[0]
    if k < 2 * _TRI_MIN:
        _gemm(A, Xl, out, alpha, beta, b_trans=True)
        return
    h = _split(k)
    _mm_lowT(A[:, :h], Xl[:h, :h], out[:, :h], alpha, beta)
    _mm_lowT(A[:, h:], Xl[h:, h:], out[:, h:], alpha, beta)
    _gemm(A[:, :h], Xl[h:, :h], out[:, h:], alpha, 1.0, b_trans=True)


def _mm_low_right(A, Xl, out, alpha, beta):
    """out = beta out + alpha A Xl, Xl lower: A Xl = [A1 X11 + A2 X21, A2 X22]."""
    k = Xl.shape[0]
    if k < 2 * _TRI_MIN:
        _gemm(A, Xl, out, alpha, beta)
        return
    h = _split(k)
    _mm_low_right(A[:, :h], Xl[:h, :h], out[:, :h], alpha, beta)
    _gemm(A[:, h:], Xl[h:, :h], out[:, :h], alpha, 1.0)
    _mm_low_right(A[:, h:], Xl[h:, h:], out[:, h:], alpha, beta)


def _mm_low_left(Xl, B, out, alpha, beta):
    """out = beta out + alpha Xl B, Xl lower: Xl B = [X11 B1; X21 B1 + X22 B2]."""
    k = Xl.shape[0]
    if k < 2 * _TRI_MIN:
        _gemm(Xl, B, out, alpha, beta)
        return
    h = _split(k)
    _mm_low_left(Xl[:h, :h], B[:h], out[:h], alpha, beta)
    _mm_low_left(Xl[h:, h:], B[h:], out[h:], alpha, beta)
    _gemm(Xl[h:, :h], B[:h], out[h:], alpha, 1.0)


def _syrk_lower(L, C, alpha):
    """Lower part of C += alpha L L^T (the upper part of C is never read by the recursion;
    diagonal blocks are updated whole)."""
    m = C.shape[0]
    if m < 2 * _TRI_MIN:
        _gemm(L, L, C, alpha, 1.0, b_trans=True)
        return
    h = _split(m)
    _syrk_lower(L[:h], C[:h, :h], alpha)
    _gemm(L[h:], L[:h], C[h:, :h], alpha, 1.0, b_trans=True)
    _syrk_lower(L[h:], C[h:, h:], alpha)


_OVERLAP_MIN = 1024  # recursion levels from this size up run T = L21 X11 on a side stream
_side_streams: dict = {}


def _side_stream(dev, depth):
    key = (dev.index, depth)
    st = _side_streams.get(key)
    if st is None:
        st = _side_streams[key] = torch.cuda.Stream(device=dev)
    return st


def _chol_inv_rec(A: torch.Tensor, X: torch.Tensor, info: torch.Tensor, row0: int = 0,
                  depth: int = 0):
    """X (zeroed square fp32 view) <- L^-1 for the lower Cholesky factor L of A (square fp32
    row-major view, lower part read; consumed as workspace).

    [[A11, .], [A21, A22]]: X11 = chol(A11)^-1 (recursion); L21 = A21 X11^T; A22 -= L21 L21^T;
    X22 = chol(A22)^-1 (recursion); X21 = -X22 (L21 X11). Tiles of <= 128 are factored and
    inverted in one workgroup (lcq_chol_inv_tile); everything else is fp32 MFMA GEMM
    (lcq_gemm_f32), written in place through strided views, with the triangular / symmetric
    structure skipped block-wise (_mm_* / _syrk_lower). T = L21 X11 needs neither the A22
    update nor X22, so from _OVERLAP_MIN up it runs on a side stream (one per recursion depth:
    an inner level's T never queues behind an outer one) while the main stream walks the
    A22 -> X22 chain, whose mid-size products leave most of the chip idle; the streams join
    before X21. Every product is the same kernel on the same operands either way (results are
    identical). Under true_sequential the block's Hessians (q/k/v, o, gate/up, down) are built
    one after another from the previous subsets' quantized outputs, so their chains cannot
    overlap."""
    n = A.shape[0]
    if n <= _TILE:
        ops.chol_inv_tile(A, info, row0, out=X)
        return
    n1 = _split(n)
    A21, A22 = A[n1:, :n1], A[n1:, n1:]
    X11, X22 = X[:n1, :n1], X[n1:, n1:]
    _chol_inv_rec(A[:n1, :n1], X11, info, row0, depth + 1)
    L21 = torch.empty_like(A21)
    _mm_lowT(A21, X11, L21, 1.0, 0.0)
    T = torch.empty_like(A21)
    if n >= _OVERLAP_MIN and A.is_cuda and _chain_shard is None:
        main = torch.cuda.current_stream(A.device)
        side = _side_stream(A.device, depth)
        side.wait_stream(main)  # L21, X11 ready
        with torch.cuda.stream(side):
            _mm_low_right(L21, X11, T, 1.0, 0.0)
        _syrk_lower(L21, A22, -1.0)
        _chol_inv_rec(A22, X22, info, row0 + n1, depth + 1)
        main.wait_stream(side)  # T ready; L21 / T are released only after this join
    else:
        _syrk_lower(L21, A22, -1.0)
        _chol_inv_rec(A22, X22, info, row0 + n1, depth + 1)
        _mm_low_right(L21, X11, T, 1.0, 0.0)
    del L21
    _mm_low_left(X22, T, X[n1:, :n1], -1.0, 0.0)


def _chol_core(Hr: torch.Tensor):
    """(X, info): X = chol(Hr)^-1 (lower), Hr consumed as workspace."""
    info = torch.zeros(1, dtype=torch.int32, device=Hr.device)
    X = torch.zeros_like(Hr)
    _chol_inv_rec(Hr, X, info)
    return X, info


# One captured HIP graph per (device, Hessian size): the recursion issues ~600 launches per
# chain at n = 14336 (the Llama-3-8B down_proj Hessian), many shorter than the host time to
# issue them from Python; a replay issues them back to back. Every size's first chain runs
# eagerly (it also loads every kernel), the graph is captured right after and replayed for the
# following blocks. Same kernels, same operands: identical results. The graph's input buffer
# is filled in place by the caller's preparation kernel, and its output flipped into a fresh
# tensor (no staging copies around the replay).
_GRAPH_MIN = 1024
CHAIN_GRAPHS = True   # tests switch this off to compare the eager chain with the replay
_chain_graphs: dict = {}


def clear_chain_graphs():
    """Drop every captured chain graph with its private memory pool (static input, output and
    recursion temporaries: ~4-5 n^2 fp32 per Hessian size, ~4 GB at n 14336). GPTQ calls this
    when its block loop ends, so the pools do not outlive the run."""
    _chain_graphs.clear()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def release_device_state():
    """clear_chain_graphs + the recursion's side streams (BlockwiseOpt.release)."""
    clear_chain_graphs()
    _side_streams.clear()


def _inverse_cholesky_upper_filled(fill, n: int, device) -> torch.Tensor:
    """U = J chol(Hr)^-1 J where fill(buf) writes Hr = J H J (n x n fp32) into buf."""
    graphed = (torch.device(device).type == 'cuda' and n >= _GRAPH_MIN and CHAIN_GRAPHS
               and _chain_shard is None)
    key = (torch.device(device).index, n)
    ent = _chain_graphs.get(key) if graphed else None
    if ent is None:
        Hr = torch.empty((n, n), dtype=torch.float32, device=device)
        fill(Hr)
        X, info = _chol_core(Hr)
        del Hr
        if graphed:
            static_in = torch.empty((n, n), dtype=torch.float32, device=device)
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(device)
            timer, ops.N._timer = ops.N._timer, None  # captured launches do not run: no events
            try:
                with torch.cuda.graph(g):
                    Xs, infos = _chol_core(static_in)
            finally:
                ops.N._timer = timer
            _chain_graphs[key] = (g, static_in, Xs, infos)
    else:
        g, static_in, X, info = ent
        fill(static_in)
        timer = ops.N._timer
        if timer is not None:  # bench's per-kernel table: the replay as one entry
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            timer.events.setdefault('lcq_chol_chain_graph', []).append((e0, e1))
        else:
            g.replay()
    bad = int(info.item())   # (a static info is read before the next replay)
    if bad:
        raise torch.linalg.LinAlgError(
            f'linalg.cholesky: The factorization could not be completed because the input '
            f'is not positive-definite (the leading minor of order {bad} is not '
            f'positive-definite).')
    return X.flip(0, 1).contiguous()


def inverse_cholesky_upper(H: torch.Tensor) -> torch.Tensor:
    """U = chol(H^-1, upper) = J chol(J H J)^-1 J for SPD fp32 H."""
    return _inverse_cholesky_upper_filled(lambda buf: buf.copy_(H.flip(0, 1)), H.shape[0],
                                          H.device)


def prepare_weight(W: torch.Tensor, perm, dead):
    """Weight side of gptq.py:128-176: fp32 copy, dead columns zeroed, act-order permuted --
    one lcq_gather_rc pass from the (bf16) weight."""
    if W.is_cuda and W.dim() == 2 and W.dtype in (torch.bfloat16, torch.float32) \
            and W.stride(1) == 1:
        return ops.gather_rc(W, csrc=perm, dead_col=dead if bool(dead.any()) else None)
    W = W.float().clone()
    if bool(dead.any()):
        W[:, dead] = 0
    if perm is not None:
        W = W[:, perm].contiguous()
    return W


def prepare(W: torch.Tensor, H: torch.Tensor, actorder: bool, percdamp: float):
    """(W fp32 permuted, U, perm | None); H is consumed."""
    U, perm, dead = prepare_hessian(H, actorder, percdamp)
    return prepare_weight(W, perm, dead), U, perm


LEFT_LOOKING = True   # module switch for A/B runs and tests (False: a trailing launch per block)


@torch.no_grad()
def column_loop(W: torch.Tensor, U: torch.Tensor, bit: int, sym: bool, group: int | None,
                qmin: int, qmax: int, fixed=None, losses: bool = False,
                superblock: int | None = None, col_group: torch.Tensor | None = None,
                ncols_q: int | None = None, col_qparams=None, fp8=None):
    """Blocked OBS loop (gptq.py:198-244) on permuted fp32 W, in place.

    Per 128-column block: the HIP kernel runs the in-block sequential loop (bit-exact rank-1
    updates). The reference then applies ``W[:, i2:] -= Err @ U[i1:i2, i2:]`` to every later
    column; here that update is two-level: inside a superblock of ``superblock`` columns each
    block's columns receive the earlier blocks' updates (left-looking, inside the block kernel:
    the same products and order as one ``lcq_gptq_trailing`` per block), and the far columns
    receive the superblock's stacked errors in ONE K = superblock update (same terms, grouped
    differently -> T2; every element still has a fixed k order, so row sharding stays
    bit-identical). ``ncols_q`` (OWQ): only the first ncols_q
    columns are quantized; every block's error still updates all later columns.

    ``col_qparams`` (per_group with a searched range, calib_algo mse): a function of a
    [rows, width] fp32 column slice returning its per-row (scales, zeros | None). The reference
    computes a group's qparams when the loop reaches its first column, from the global W,
    whose columns of the current block are not updated inside the block (gptq.py:213-222,
    search_column_qparams :359-366): so every group starting in a block gets its qparams from
    the block-start W, here before the block kernel, which then quantizes with them.

    ``fp8`` (a torch float8 dtype): FloatQuantizer weights (gptq_fp8.yml) -- the in-block
    quant_dequant is float_quantize(w / s) * s (quant.py:1061-1080), symmetric."""
    rows, cols = W.shape
    dev = W.device
    U = U.contiguous()
    ncq = cols if ncols_q is None else int(ncols_q)
    searched = col_qparams is not None
    if searched:
        if group is None or col_group is not None or not (BLOCK % group == 0
                                                          or group % BLOCK == 0):
            raise NotImplementedError('searched column qparams need per_group with a group '
                                      'size dividing or divisible by 128')
        ngs = -(-ncq // group)
        s_srch = torch.empty((rows, ngs), dtype=torch.float32, device=dev)
        z_srch = None if sym else torch.empty((rows, ngs), dtype=torch.float32, device=dev)
        col_group = (torch.arange(cols, device=dev) // group).clamp(max=ngs - 1).to(
            torch.int32).contiguous()
    static = col_group is not None  # static_groups: fixed qparams of the original groups
    ng = 0 if (group is None or static) else -(-ncq // group)
    s_out = torch.empty((rows, ng), dtype=torch.float32, device=dev) if ng else None
    z_out = torch.empty((rows, ng), dtype=torch.float32, device=dev) if ng and not sym else None
    if superblock is None:
        superblock = SUPERBLOCK
    SB = max(BLOCK, superblock // BLOCK * BLOCK)
    # k-major stacked Err1, rows padded to 4 so that every k row is 16-byte aligned (the
    # trailing update's LDS-DMA kernel; a row shard gets the same kernel as the whole matrix)
    errT = torch.empty((SB, -(-rows // 4) * 4), dtype=torch.float32, device=dev)
    L = torch.zeros_like(W) if losses else None
    s_in = z_in = None
    if searched:
        s_in, z_in = s_srch, z_srch
    elif group is None or static:
        s_in = fixed[0].reshape(-1).float().contiguous()
        z_in = None if sym else fixed[1].reshape(-1).float().contiguous()
    # Near updates (the rest of the superblock after each block): left-looking inside the next
    # block kernels (lcq_gptq_block nprev > 0: the same products in the same order, bit for
    # bit, without a trailing launch and its dependent-kernel gap per block), except where the
    # host needs the block-start columns before the kernel (searched qparams).
    left = LEFT_LOOKING and not searched
    for sb0 in range(0, ncq, SB):
        sb1 = min(sb0 + SB, ncq)
        for i1 in range(sb0, sb1, BLOCK):
            i2 = min(i1 + BLOCK, sb1)
            cnt = i2 - i1
            e = errT[i1 - sb0:]
            npv = (i1 - sb0) // BLOCK if left else 0
            if searched:  # groups starting in this block, from the block-start columns
                for g0 in range(-(-i1 // group) * group, i2, group):
                    sg, zg = col_qparams(W[:, g0:min(g0 + group, ncq)])
                    s_srch[:, g0 // group] = sg.reshape(-1)
                    if z_srch is not None:
                        z_srch[:, g0 // group] = zg.reshape(-1)
            if static:
                ops.gptq_block_cols(W, i1, cnt, U, qmin, qmax, s_in, z_in, col_group, e, L,
                                    err_prev=errT, nprev=npv)
            else:
                ops.gptq_block(W, i1, cnt, U, group or 0, qmin, qmax, sym, s_out, z_out, e, L,
                               s_in, z_in, fp8=fp8, err_prev=errT, nprev=npv)
            if not left and i2 < sb1:  # near columns: the rest of this superblock
                ops.gptq_trailing(W, i1, cnt, i2, e, U, c2=sb1)
        if sb1 < cols:    # far columns: the whole superblock's errors at once
            ops.gptq_trailing(W, sb0, sb1 - sb0, sb1, errT, U, c2=cols)
    if searched:
        return s_srch, z_srch, L
    return s_out, z_out, L


def check_quantizer(wquantizer, static_groups=False, owq_nout=0):
    """The quantizer settings the device column loop implements; anything else raises
    instead of running a different quantizer. Returns the fp8 dtype for FloatQuantizer
    weights, else None."""
    qt = getattr(wquantizer, 'quant_type', 'int-quant')
    algo = getattr(wquantizer, 'calib_algo', 'minmax')
    if qt == 'int-quant':
        if algo not in ('minmax', 'mse'):
            raise NotImplementedError(f'GPTQ with calib_algo {algo} is not on the device path')
        if not getattr(wquantizer, 'round_zp', True):
            # the reference computes round(w / s + z) with a float zero (quant.py:699-705);
            # the column kernel's integer-zero form would differ silently
            raise NotImplementedError('GPTQ with round_zp False is not on the device path')
        return None
    if qt != 'float-quant':
        raise NotImplementedError(f'GPTQ with quant_type {qt}')
    if not getattr(wquantizer, 'use_qtorch', False):
        # use_qtorch False keeps per-element scales from get_float_qparams, which the
        # reference's column loop cannot broadcast against one column (gptq.py:229-238)
        raise NotImplementedError('GPTQ float-quant needs use_qtorch (the reference\'s '
                                  'get_float_qparams scales are per element)')
    if getattr(wquantizer, 'fp8_dtype', None) is None:
        raise NotImplementedError(f'GPTQ float-quant {wquantizer.bit}: only e4m3 / e5m2')
    if 'float_range' in getattr(wquantizer, 'kwargs', {}):
        raise NotImplementedError('GPTQ float-quant with a custom float_range')
    if algo != 'minmax' or static_groups or owq_nout:
        raise NotImplementedError('GPTQ float-quant: minmax qparams, no static_groups / OWQ')
    if wquantizer.granularity not in ('per_channel', 'per_group'):
        raise NotImplementedError(f'GPTQ float-quant with {wquantizer.granularity}')
    return wquantizer.fp8_dtype


@torch.no_grad()
def quantize_layer(W: torch.Tensor, H: torch.Tensor | None, wquantizer, actorder=True,
                   percdamp=0.01, fixed=None, losses=False, shard_rows=False, prepared=None,
                   static_groups=False, owq_nout=0):
    """Full GPTQ transform of one linear. Returns dict(weight fp32 (original column order),
    scales / zeros [rows*ng, 1] fp32 (merge_qparams order, permuted groups), perm, invperm,
    loss). ``prepared`` = prepare_hessian(...) output shared by linears with the same input
    (q/k/v, gate/up): their H -- hence perm, damping and U -- are identical. calib_algo mse
    per_group: the column qparams are searched in the loop (column_loop's col_qparams).
    FloatQuantizer weights (use_qtorch, e4m3 / e5m2): the float-quant column loop."""
    bit, sym = wquantizer.bit, wquantizer.sym
    fp8 = check_quantizer(wquantizer, static_groups, owq_nout)
    qmin, qmax = int(wquantizer.qmin.item()), int(wquantizer.qmax.item())
    group = wquantizer.group_size if wquantizer.granularity == 'per_group' else None
    if group is not None and not static_groups and group not in (32, 64, 128):
        raise NotImplementedError('device GPTQ supports group_size 32/64/128')
    col_qparams = None
    if (group is not None and not static_groups
            and getattr(wquantizer, 'calib_algo', 'minmax') == 'mse'):
        if owq_nout:
            raise NotImplementedError('OWQ with calib_algo mse')

        def col_qparams(cols_view):
            _, _, sg, zg = wquantizer._mse(cols_view.contiguous())
            return sg, zg
    if prepared is None:
        prepared = prepare_hessian(H, actorder, percdamp, owq_nout)
    U, perm, dead = prepared
    Wp = prepare_weight(W, perm, dead)
    ncq = Wp.shape[1] - int(owq_nout)
    owq_fixed = None
    if owq_nout and group is None:
        # gptq.py:157-166: OWQ per_channel takes its qparams from the permuted, dead-zeroed
        # fp32 non-outlier columns (they replace buf_scales / buf_zeros)
        Wn = Wp[:, :ncq]
        pad = (-ncq) % 8  # the grouped kernel reads 8-column chunks: repeat a column (same
        if pad:           # row min / max) up to the next multiple of 8
            Wn = torch.cat([Wn, Wn[:, :1].expand(-1, pad)], 1)
        _, fs, fz, _, _ = wquantizer.get_tensor_qparams(Wn.contiguous())
        owq_fixed = fixed = (fs, None if sym else fz)
    col_group = None
    if static_groups and group is not None:
        # gptq.py:224-227: permuted column j quantizes with groups[perm[j] // group_size], the
        # qparams collected from the ORIGINAL weights (fixed = buf_scales / buf_zeros)
        cols = Wp.shape[1]
        src = perm if perm is not None else torch.arange(cols, device=Wp.device)
        col_group = (src // group).to(torch.int32).contiguous()
    if shard_rows:
        # rows are independent given U: every rank runs the column loop on its
        # row range, then the quantized rows + qparams are all-gathered (bit-identical to 1 GPU)
        from . import parallel as P
        rank, world = P.dist_world()
        r0, r1 = P.row_shard(Wp.shape[0], rank, world)
        Wl = Wp[r0:r1].contiguous()
        fx = None if fixed is None else tuple(
            None if f is None else f.reshape(Wp.shape[0], -1)[r0:r1] for f in fixed)
        s, z, L = column_loop(Wl, U, bit, sym, group, qmin, qmax, fixed=fx, losses=losses,
                              col_group=col_group, ncols_q=ncq, col_qparams=col_qparams,
                              fp8=fp8)
        Wp = P.gather_rows(Wl, Wp.shape[0])
        s = None if s is None else P.gather_rows(s, Wp.shape[0])
        z = None if z is None else P.gather_rows(z, Wp.shape[0])
        L = None if L is None else P.gather_rows(L, Wp.shape[0])
    else:
        s, z, L = column_loop(Wp, U, bit, sym, group, qmin, qmax, fixed=fixed, losses=losses,
                              col_group=col_group, ncols_q=ncq, col_qparams=col_qparams,
                              fp8=fp8)
    invperm = torch.argsort(perm) if perm is not None else None
    weight = ops.gather_rc(Wp, csrc=invperm) if invperm is not None else Wp
    if owq_fixed is not None:
        s, z = owq_fixed
    return dict(weight=weight, scales=None if s is None else s.reshape(-1, 1),
                zeros=None if z is None else z.reshape(-1, 1), perm=perm, invperm=invperm,
                loss=None if L is None else L.sum())
