"""Torch-tensor front end of the lcq C ABI.

Each function validates shapes/dtypes on the host, allocates outputs with torch (device
memory is torch's caching allocator), and launches the HIP kernel on torch's current stream
through ``_native``. There is no CPU path: CPU tensors raise ``LcqError``.
"""
from __future__ import annotations


import torch

from . import _native as N

__all__ = ['int_quant_dynamic', 'int_quant_static', 'pack_vllm', 'pack_autoawq_gemm',
           'hessian_accum', 'gptq_block', 'absmean_cols', 'awq_weight_scale', 'awq_scales', 'scale_bcast',
           'sq_diff_mean', 'auto_clip_search', 'clip_apply', 'linear', 'linear_multi', 'linear_multi_rope',
           'linear_silu_mul', 'linear_sq_diff', 'gemm_supported']


def _code_dtype(bit: int, qmin: int) -> torch.dtype:
    # quant.py:890-896 / 929-935
    if bit == 8:
        return torch.int8 if qmin != 0 else torch.uint8
    return torch.int32


def int_quant_dynamic(x: torch.Tensor, group: int, qmin: int, qmax: int, sym: bool, *,
                      pre_scale: torch.Tensor | None = None,
                      clip_max: torch.Tensor | None = None,
                      clip_min: torch.Tensor | None = None,
                      fq: bool = True, fq_dtype: torch.dtype | None = None,
                      codes_dtype: torch.dtype | None = None,
                      pack_bits: int | None = None,
                      qparams: bool = True,
                      out: torch.Tensor | None = None) -> dict:
    """Grouped min/max quantization of a 2-D tensor ``x`` [rows, cols] (groups along cols).

    Returns a dict with any of ``fq`` (fake-quant, ``fq_dtype``), ``codes``, ``packed``
    (vLLM int32), ``scales``/``zeros`` ([rows*cols/group, 1] in x.dtype).
    """
    assert x.dim() == 2, 'x must be 2-D'
    rows, cols = x.shape
    group = cols if group in (0, None) else int(group)
    ng = rows * cols // group
    res = {}
    fq_t = None
    if fq:
        fq_dtype = fq_dtype or x.dtype
        fq_t = out if out is not None else torch.empty((rows, cols), dtype=fq_dtype, device=x.device)
        res['fq'] = fq_t
    codes_t = None
    if codes_dtype is not None:
        codes_t = torch.empty((rows, cols), dtype=codes_dtype, device=x.device)
        res['codes'] = codes_t
    packed_t = None
    if pack_bits:
        pf = 32 // pack_bits
        packed_t = torch.empty((rows, (cols + pf - 1) // pf), dtype=torch.int32, device=x.device)
        res['packed'] = packed_t
    s_t = z_t = None
    if qparams:
        s_t = torch.empty((ng, 1), dtype=x.dtype, device=x.device)
        res['scales'] = s_t
        if not sym:
            z_t = torch.empty((ng, 1), dtype=x.dtype, device=x.device)
            res['zeros'] = z_t
    for t in (pre_scale, clip_max, clip_min):
        if t is not None and t.dtype != x.dtype:
            raise ValueError('pre_scale / clip bounds must have the weight dtype')
    N.call('lcq_int_quant_dynamic', N.ptr(x), N.dt(x), rows, cols, group,
           N.ptr(pre_scale), N.ptr(clip_max), N.ptr(clip_min), int(qmin), int(qmax), int(sym),
           N.ptr(fq_t), N.dt(fq_dtype) if fq else 0,
           N.ptr(codes_t), N.dt(codes_dtype) if codes_t is not None else 0,
           N.ptr(packed_t), int(pack_bits or 0), N.ptr(s_t), N.ptr(z_t), N.stream_of(x))
    return res


def int_quant_static(x: torch.Tensor, group: int, scales: torch.Tensor,
                     zeros: torch.Tensor | None, qmin: int, qmax: int, *,
                     ct_dtype: torch.dtype, fq: bool = True,
                     fq_dtype: torch.dtype | None = None,
                     codes_dtype: torch.dtype | None = None,
                     pack_bits: int | None = None, round_zp: bool = True) -> dict:
    """Quantize ``x`` [rows, cols] with given per-group scales/zeros (flat group order).
    ``round_zp=False``: quant.py:701-707 (``round(x / s.clamp_min(1e-9) + z)``)."""
    assert x.dim() == 2
    rows, cols = x.shape
    group = cols if group in (0, None) else int(group)
    ng = rows * cols // group
    scales = scales.contiguous()
    if scales.numel() != ng:
        raise ValueError(f'scales has {scales.numel()} elements, expected {ng}')
    if zeros is not None:
        zeros = zeros.contiguous()
        if zeros.numel() != ng:
            raise ValueError(f'zeros has {zeros.numel()} elements, expected {ng}')
    res = {}
    fq_t = codes_t = packed_t = None
    if fq:
        fq_dtype = fq_dtype or ct_dtype
        fq_t = torch.empty((rows, cols), dtype=fq_dtype, device=x.device)
        res['fq'] = fq_t
    if codes_dtype is not None:
        codes_t = torch.empty((rows, cols), dtype=codes_dtype, device=x.device)
        res['codes'] = codes_t
    if pack_bits:
        pf = 32 // pack_bits
        packed_t = torch.empty((rows, (cols + pf - 1) // pf), dtype=torch.int32, device=x.device)
        res['packed'] = packed_t
    if not round_zp:
        if pack_bits:
            raise ValueError('round_zp=False codes are not packed')
        N.call('lcq_int_quant_static_nozp', N.ptr(x), N.dt(x), rows, cols, group,
               N.ptr(scales), N.dt(scales), N.ptr(zeros),
               N.dt(zeros) if zeros is not None else 0, N.dt(ct_dtype), int(qmin), int(qmax),
               N.ptr(fq_t), N.dt(fq_dtype) if fq else 0,
               N.ptr(codes_t), N.dt(codes_dtype) if codes_t is not None else 0, N.stream_of(x))
        return res
    N.call('lcq_int_quant_static', N.ptr(x), N.dt(x), rows, cols, group,
           N.ptr(scales), N.dt(scales), N.ptr(zeros), N.dt(zeros) if zeros is not None else 0,
           N.dt(ct_dtype), int(qmin), int(qmax),
           N.ptr(fq_t), N.dt(fq_dtype) if fq else 0,
           N.ptr(codes_t), N.dt(codes_dtype) if codes_t is not None else 0,
           N.ptr(packed_t), int(pack_bits or 0), N.stream_of(x))
    return res


def int_quant_static_scalar(x: torch.Tensor, scale: torch.Tensor, zero: torch.Tensor | None,
                            qmin: int, qmax: int, *, ct_dtype: torch.dtype, fq: bool = True,
                            codes_dtype: torch.dtype | None = None) -> dict:
    """Quantize ``x`` [rows, cols] with one fp32 scale / zero kept at full precision (0-dim
    CPU operands: torch's scalar semantics), every op rounded to ct_dtype."""
    assert x.dim() == 2
    x = x.contiguous()
    rows, cols = x.shape
    s = scale.reshape(1).to(torch.float32).contiguous()
    z = None if zero is None else zero.reshape(1).to(torch.float32).contiguous()
    res = {}
    fq_t = codes_t = None
    if fq:
        fq_t = torch.empty((rows, cols), dtype=ct_dtype, device=x.device)
        res['fq'] = fq_t
    if codes_dtype is not None:
        codes_t = torch.empty((rows, cols), dtype=codes_dtype, device=x.device)
        res['codes'] = codes_t
    N.call('lcq_int_quant_static_scalar', N.ptr(x), N.dt(x), rows, cols, N.ptr(s), N.ptr(z),
           N.dt(ct_dtype), int(qmin), int(qmax), N.ptr(fq_t), N.dt(ct_dtype) if fq else 0,
           N.ptr(codes_t), N.dt(codes_dtype) if codes_t is not None else 0, N.stream_of(x))
    return res


def int_quant_static_cols(x: torch.Tensor, col_group: torch.Tensor, scales: torch.Tensor,
                          zeros: torch.Tensor | None, qmin: int, qmax: int, *,
                          ct_dtype: torch.dtype, fq_dtype: torch.dtype) -> torch.Tensor:
    """Static fake quant of x [rows, cols] where element (r, c) uses group
    r * ngc + col_group[c] of scales / zeros ([rows * ngc] flat). Returns fq [rows, cols]."""
    assert x.dim() == 2 and col_group.dtype == torch.int32 and col_group.numel() == x.shape[1]
    x = x.contiguous()
    rows, cols = x.shape
    scales = scales.contiguous()
    ngc = scales.numel() // rows
    if ngc * rows != scales.numel():
        raise ValueError('scales do not tile the rows')
    if zeros is not None:
        zeros = zeros.contiguous()
        if zeros.numel() != scales.numel():
            raise ValueError('zeros / scales size mismatch')
    cg = col_group.contiguous()
    out = torch.empty((rows, cols), dtype=fq_dtype, device=x.device)
    N.call('lcq_int_quant_static_cols', N.ptr(x), N.dt(x), rows, cols, N.ptr(cg), ngc,
           N.ptr(scales), N.dt(scales), N.ptr(zeros), N.dt(zeros) if zeros is not None else 0,
           N.dt(ct_dtype), int(qmin), int(qmax), N.ptr(out), N.dt(fq_dtype), None, 0,
           N.stream_of(x))
    return out


def pack_vllm(codes: torch.Tensor, bits: int) -> torch.Tensor:
    """VllmRealQuantLinear.pack bit layout (module_utils.py:929-955) on device."""
    assert codes.dim() == 2
    rows, cols = codes.shape
    pf = 32 // bits
    out = torch.empty((rows, (cols + pf - 1) // pf), dtype=torch.int32, device=codes.device)
    N.call('lcq_pack_vllm', N.ptr(codes), N.dt(codes), rows, cols, int(bits), N.ptr(out),
           N.stream_of(codes))
    return out


def pack_autoawq_gemm(weight: torch.Tensor, scales: torch.Tensor, zeros: torch.Tensor,
                      group: int, bits: int = 4):
    """AutoawqRealQuantLinear.gemm_pack (module_utils.py:1097-1158) on device.

    weight [oc, ic], scales [oc, ic/group], zeros [oc, ic/group] int32.
    Returns (qweight int32 [ic, oc/8], scales fp16 [ic/group, oc], qzeros int32 [ic/group, oc/8]).
    """
    oc, ic = weight.shape
    ng = ic // group
    zeros = zeros.to(torch.int32).contiguous()
    scales = scales.contiguous()
    qweight = torch.empty((ic, oc * bits // 32), dtype=torch.int32, device=weight.device)
    scales_t = torch.empty((ng, oc), dtype=torch.float16, device=weight.device)
    qzeros = torch.empty((ng, oc * bits // 32), dtype=torch.int32, device=weight.device)
    N.call('lcq_pack_autoawq_gemm', N.ptr(weight), N.dt(weight), oc, ic, int(group),
           N.ptr(scales), N.dt(scales), N.ptr(zeros), int(bits), N.ptr(qweight),
           N.ptr(scales_t), N.ptr(qzeros), N.stream_of(weight))
    return qweight, scales_t, qzeros


def hessian_accum(x: torch.Tensor, H: torch.Tensor, alpha: float, beta: float) -> torch.Tensor:
    """H <- beta*H + alpha * x^T x (in place); x [n, ic] bf16/fp16, H [ic, ic] fp32."""
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    n, ic = x2.shape
    if H.dtype != torch.float32 or tuple(H.shape) != (ic, ic):
        raise ValueError('H must be fp32 [ic, ic]')
    ws_bytes = N.load().lcq_hessian_workspace_bytes(n, ic)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x2.device)
    N.call('lcq_hessian_accum', N.ptr(x2), N.dt(x2), n, ic, N.ptr(H), float(alpha),
           float(beta), N.ptr(ws), ws_bytes, N.stream_of(x2))
    N.note_work('lcq_hessian_accum', n * ic * (ic + 1))  # symmetric rank-n update (§8d)
    return H


def hessian_grouped(x: torch.Tensor, bounds, H: torch.Tensor, alpha: float) -> torch.Tensor:
    """H <- alpha * tree over token groups of the groups' x^T x (lcq_hessian_grouped: one
    launch; ``bounds`` = token offsets [0, ..., n] of the ng = 1 / 2 / 4 / 8 groups)."""
    import ctypes
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    n, ic = x2.shape
    if H.dtype != torch.float32 or tuple(H.shape) != (ic, ic) or not H.is_contiguous():
        raise ValueError('H must be contiguous fp32 [ic, ic]')
    if bounds[0] != 0 or bounds[-1] != n:
        raise ValueError('bounds must run from 0 to the token count')
    b = (ctypes.c_int64 * len(bounds))(*[int(v) for v in bounds])
    ng = len(bounds) - 1
    ws_bytes = N.load().lcq_hessian_grouped_workspace_bytes(b, ng, ic)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=x2.device)
    N.call('lcq_hessian_grouped', N.ptr(x2), N.dt(x2), ic, b, ng, N.ptr(H), float(alpha),
           N.ptr(ws), ws_bytes, N.stream_of(x2))
    N.note_work('lcq_hessian_grouped', n * ic * (ic + 1))  # symmetric rank-n update (§8d)
    return H


def tree_sum(parts, alpha: float = 1.0, out: torch.Tensor | None = None) -> torch.Tensor:
    """out = alpha * the fixed pairwise tree sum of 1 / 2 / 4 / 8 equal fp32 tensors
    (lcq_tree_sum; deterministic, the grouped Hessian's reduction order)."""
    import ctypes
    p0 = parts[0]
    for p in parts:
        if p.dtype != torch.float32 or p.shape != p0.shape or not p.is_contiguous():
            raise ValueError('tree_sum: contiguous fp32 tensors of one shape')
    if out is None:
        out = torch.empty_like(p0)
    if out.numel() % 4:
        raise ValueError('tree_sum: numel must be a multiple of 4')
    N.call('lcq_tree_sum', (ctypes.c_void_p * len(parts))(*[N.ptr(p) for p in parts]),
           len(parts), out.numel(), float(alpha), N.ptr(out), N.stream_of(out))
    return out


def _err_prev(err_prev, nprev: int, err: torch.Tensor, rows: int):
    """(pointer, nprev) of the left-looking near updates: err_prev the k-major errors of the
    nprev blocks before this one, with the same row stride as err."""
    if not nprev:
        return None, 0
    if (err_prev is None or err_prev.shape[0] < 128 * nprev
            or _ld_err(err_prev, rows) != _ld_err(err, rows)):
        raise ValueError('err_prev must be k-major [>= 128 nprev, ld_err] like err')
    return N.ptr(err_prev), int(nprev)


def gptq_block(W: torch.Tensor, col0: int, count: int, U: torch.Tensor, group: int,
               qmin: int, qmax: int, sym: bool, s_out, z_out, err: torch.Tensor,
               losses=None, s_in=None, z_in=None, fp8=None, err_prev=None, nprev: int = 0):
    """One 128-column GPTQ block in place on fp32 W (see include/lcq.h lcq_gptq_block);
    err is k-major [128, rows]. fp8 (torch.float8_e4m3fn / float8_e5m2): FloatQuantizer's
    quant_dequant instead of the integer one (qmin / qmax / sym / zeros ignored). nprev > 0:
    the near updates of the nprev blocks before col0 (their errors in err_prev) are applied
    first, inside the kernel (left-looking)."""
    rows, ld = W.shape
    ng_total = s_out.shape[1] if s_out is not None else 0
    fmt = 0 if fp8 is None else N.dt(fp8)
    ep, npv = _err_prev(err_prev, nprev, err, rows)
    N.call('lcq_gptq_block', N.ptr(W), rows, ld, int(col0), int(count), N.ptr(U), U.shape[1],
           int(group), int(qmin), int(qmax), int(sym), fmt, N.ptr(s_in), N.ptr(z_in), N.ptr(s_out),
           N.ptr(z_out), int(ng_total), N.ptr(err), _ld_err(err, rows), N.ptr(losses), ep, npv,
           N.stream_of(W))


def gptq_block_cols(W: torch.Tensor, col0: int, count: int, U: torch.Tensor, qmin: int,
                    qmax: int, s_in: torch.Tensor, z_in, col_group: torch.Tensor,
                    err: torch.Tensor, losses=None, err_prev=None, nprev: int = 0):
    """gptq_block with static per-(row, original group) qparams s_in / z_in [rows, ngc] and
    the permuted column -> group map col_group (int32 [ld])."""
    rows, ld = W.shape
    ngc = s_in.numel() // rows
    ep, npv = _err_prev(err_prev, nprev, err, rows)
    N.call('lcq_gptq_block_cols', N.ptr(W), rows, ld, int(col0), int(count), N.ptr(U), U.shape[1],
           int(qmin), int(qmax), N.ptr(s_in), N.ptr(z_in), N.ptr(col_group), int(ngc), N.ptr(err),
           _ld_err(err, rows), N.ptr(losses), ep, npv, N.stream_of(W))


def _ld_err(err: torch.Tensor, rows: int) -> int:
    """Row stride of a k-major error matrix [k, >= rows] (unit column stride)."""
    if err.dim() != 2 or err.stride(1) != 1 or err.stride(0) < rows or err.shape[1] < rows:
        raise ValueError('err must be a k-major [k, >= rows] fp32 view with unit column stride')
    return err.stride(0)


def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError('expected a row-major 2-D view')
    return t.stride(0)


def gemm_f32(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, alpha: float = 1.0,
             beta: float = 0.0, b_trans: bool = False) -> torch.Tensor:
    """out = beta * out + alpha * A @ (B.T if b_trans else B) on row-major fp32 views (the
    Cholesky recursion's `addmm_`, lcq_gemm_f32); beta 0 never reads out."""
    M, K = A.shape
    n_ = out.shape[1]
    ok = B.shape == ((n_, K) if b_trans else (K, n_))
    if not ok or out.shape[0] != M:
        raise ValueError('gemm_f32: shape mismatch')
    if any(t.dtype != torch.float32 for t in (A, B, out)):
        raise ValueError('gemm_f32: fp32 operands')
    ws_bytes = int(N.load().lcq_gemm_f32_workspace_bytes(M, n_, K)) if STREAM_K else 0
    if ws_bytes:   # stream-K: 32 MB of partial tiles (from the graph's pool under capture)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=A.device)
        N.call('lcq_gemm_f32_ws', M, n_, K, float(alpha), A.data_ptr(), _ld(A), B.data_ptr(),
               _ld(B), int(b_trans), float(beta), out.data_ptr(), _ld(out), ws.data_ptr(),
               ws_bytes, N.stream_of(A))
        return out
    N.call('lcq_gemm_f32', M, n_, K, float(alpha), A.data_ptr(), _ld(A), B.data_ptr(), _ld(B),
           int(b_trans), float(beta), out.data_ptr(), _ld(out), N.stream_of(A))
    return out


STREAM_K = True   # gemm_f32's stream-K grids (tests compare them with the tiled kernel)


def gemm_f32_row_unit(m: int, n: int) -> int:
    """Row granularity of a gemm_f32_rows range of an m x n product (its plan's tile rows)."""
    return int(N.load().lcq_gemm_f32_row_unit(m, n))


def gemm_f32_rows(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, alpha: float,
                  beta: float, b_trans: bool, row0: int, row1: int) -> torch.Tensor:
    """Rows [row0, row1) of gemm_f32(A, B, out, alpha, beta, b_trans) -- A and out the full
    operands -- computed with the kernel the full product is planned for (never stream-K):
    every element gets the same k order on any rank (lcq_gemm_f32_rows)."""
    M, K = A.shape
    n_ = out.shape[1]
    ok = B.shape == ((n_, K) if b_trans else (K, n_))
    if not ok or out.shape[0] != M:
        raise ValueError('gemm_f32_rows: shape mismatch')
    if any(t.dtype != torch.float32 for t in (A, B, out)):
        raise ValueError('gemm_f32_rows: fp32 operands')
    N.call('lcq_gemm_f32_rows', M, n_, K, float(alpha), A.data_ptr(), _ld(A), B.data_ptr(),
           _ld(B), int(b_trans), float(beta), out.data_ptr(), _ld(out), int(row0), int(row1),
           N.stream_of(A))
    return out


X6_MIN_TILES = 40   # 256 x 256 output tiles from which the split-plane product beats fp32 MFMA


def gemm_f32x6_fits(M: int, n: int, K: int, out: torch.Tensor) -> bool:
    """Whether the M x n x K product goes to gemm_f32x6: enough 256 x 256 tiles (with its K
    split below 256 tiles; scripts/chain_split_rate.py, profiles/r5_chain_x6.md), K >= 1024,
    n % 16 == 0 and 16-byte fp32 output rows. A function of the FULL product's shape and
    layout, so every rank of a row-split product makes the same choice."""
    return (X6 and -(-M // 256) * -(-n // 256) >= X6_MIN_TILES and K >= 1024 and n % 16 == 0
            and out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0)


X6 = True   # module switch for A/B runs and tests (False: every product on the fp32 kernels)


def gemm_f32x6(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, alpha: float, beta: float,
               b_trans: bool, row0: int = 0, row1: int | None = None, a_trans: bool = False,
               max_splits: int = 8) -> torch.Tensor:
    """Rows [row0, row1) of out = beta out + alpha op(A) op(B) (fp32 views as gemm_f32; a_trans:
    A given k-major as [K, M]) on bf16 MFMA over three bf16 planes per operand (lcq_gemm_f32x6:
    fp32-GEMM accuracy, ~2x the fp32 MFMA rate). Row ranges compute every element exactly as
    the whole product does; max_splits 1 keeps K unsplit whatever the shape."""
    K, M = A.shape if a_trans else A.shape[::-1]
    n_ = out.shape[1]
    row1 = M if row1 is None else row1
    ok = B.shape == ((n_, K) if b_trans else (K, n_))
    if not ok or out.shape[0] != M:
        raise ValueError('gemm_f32x6: shape mismatch')
    if any(t.dtype != torch.float32 for t in (A, B, out)):
        raise ValueError('gemm_f32x6: fp32 operands')
    ws_bytes = int(N.load().lcq_gemm_f32x6_workspace_bytes(M, row1 - row0, n_, K,
                                                            int(max_splits)))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=A.device)
    N.call('lcq_gemm_f32x6', M, n_, K, float(alpha), A.data_ptr(), _ld(A), int(a_trans),
           B.data_ptr(), _ld(B), int(b_trans), float(beta), out.data_ptr(), _ld(out), int(row0),
           int(row1), int(max_splits), ws.data_ptr(), ws_bytes, N.stream_of(A))
    return out


def chol_inv_tile(A: torch.Tensor, info: torch.Tensor, row0: int = 0,
                  L: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Returns L^-1 for the lower Cholesky factor L of A (<= 128 x 128 fp32 view, unit column
    stride); L itself is written to `L` when given (may be A). info (int32, 1 element) receives
    row0 + the first non-positive pivot (1-based) on failure. `out` (a view like A) receives
    L^-1 in place of a new tensor."""
    if A.dtype != torch.float32 or A.shape[0] != A.shape[1]:
        raise ValueError('chol_inv_tile expects a square fp32 tile')
    for t in (L, out):
        if t is not None and (t.shape != A.shape or t.dtype != torch.float32):
            raise ValueError('L / out must match A')
    X = torch.empty((A.shape[0], A.shape[0]), dtype=torch.float32, device=A.device) \
        if out is None else out
    N.call('lcq_chol_inv_tile', A.data_ptr(), _ld(A), A.shape[0],
           0 if L is None else L.data_ptr(), 0 if L is None else _ld(L),
           X.data_ptr(), _ld(X), N.ptr(info), row0, N.stream_of(A))
    return X


def gather_rc(A: torch.Tensor, rsrc=None, csrc=None, dead_col=None, dead_diag=None,
              damp=None, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i][j] = f(A[rsrc[i]][csrc[j]]) in fp32 (lcq_gather_rc): GPTQ's act-order
    permutation, dead-column handling and damping in one pass (see include/lcq.h)."""
    if A.dim() != 2 or A.stride(1) != 1:
        raise ValueError('gather_rc: 2-D row-major A')
    rows = A.shape[0] if rsrc is None else rsrc.numel()
    cols = A.shape[1] if csrc is None else csrc.numel()
    if out is None:
        out = torch.empty((rows, cols), dtype=torch.float32, device=A.device)
    idx = [None if t is None else t.to(torch.int64).contiguous() for t in (rsrc, csrc)]
    msk = [None if t is None else t.to(torch.uint8).contiguous() for t in (dead_col, dead_diag)]
    dmp = None if damp is None else damp.to(torch.float32).reshape(1).contiguous()
    N.call('lcq_gather_rc', N.ptr_strided(A), N.dt(A.dtype), rows, cols, A.stride(0),
           N.ptr(idx[0]), N.ptr(idx[1]), N.ptr(msk[0]), N.ptr(msk[1]), N.ptr(dmp),
           N.ptr(out), out.stride(0), N.stream_of(A))
    return out


TRAIL_X6_MIN_K = 1024   # trailing updates from this K (the superblock's far update) use x6


def gptq_trailing(W: torch.Tensor, c0: int, cnt: int, c1: int, err: torch.Tensor,
                  U: torch.Tensor, c2: int | None = None):
    """W[:, c1:c2] -= err.T[:, :cnt] @ U[c0:c0+cnt, c1:c2] in place (err k-major
    [cnt, >= rows] view; deterministic k order). c2 defaults to the last column. The far
    updates (cnt >= TRAIL_X6_MIN_K) run on split-plane bf16 MFMA (lcq_gemm_f32x6, K never split,
    the product rounded to fp32 then subtracted as on the fp32 kernel); the rest on fp32 MFMA.
    The choice depends on cnt and the column layout only, never on the row count, so a row
    shard computes its rows exactly as one GPU does."""
    rows, ld = W.shape
    c2 = ld if c2 is None else int(c2)
    if (X6 and cnt >= TRAIL_X6_MIN_K and (c2 - c1) % 16 == 0 and c1 % 4 == 0 and ld % 4 == 0
            and W.stride(1) == 1 and W.data_ptr() % 16 == 0 and err.stride(1) == 1
            and U.stride(1) == 1):
        gemm_f32x6(err[:cnt, :rows], U[c0:c0 + cnt, c1:c2], W[:, c1:c2], -1.0, 1.0, False,
                   a_trans=True, max_splits=1)
        return
    N.call('lcq_gptq_trailing', N.ptr(W), rows, ld, int(c0), int(cnt), int(c1), c2, N.ptr(err),
           _ld_err(err, rows), N.ptr(U), U.shape[1], N.stream_of(W))


def _colmean_ws(rows: int, cols: int, device) -> torch.Tensor:
    nbytes = int(N.load().lcq_colmean_workspace_bytes(rows, cols))
    return torch.empty((max(nbytes, 4) + 3) // 4, dtype=torch.float32, device=device)


def absmean_cols(x: torch.Tensor) -> torch.Tensor:
    """mean over all leading dims of |x| per channel (Awq.get_act_scale, awq.py:74-85), in
    torch-CPU's summation order."""
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    n, c = x2.shape
    ws = _colmean_ws(n, c, x.device)
    out = torch.empty((c,), dtype=x.dtype, device=x.device)
    N.call('lcq_absmean_cols', N.ptr(x2), N.dt(x2), n, c, N.ptr(out), N.ptr(ws), N.stream_of(x2))
    return out


def awq_weight_scale(weights, group: int) -> torch.Tensor:
    """Awq.get_weight_scale (awq.py:48-72) over the subset's linears (same dtype and cols)."""
    w0 = weights[0]
    cols = w0.shape[-1]
    total = torch.empty((cols,), dtype=w0.dtype, device=w0.device)
    ws = _colmean_ws(max(w.shape[0] for w in weights), cols, w0.device)
    for i, w in enumerate(weights):
        w2 = w.reshape(-1, cols).contiguous()
        if w2.dtype != w0.dtype:
            raise ValueError('subset weights must share the dtype')
        N.call('lcq_awq_weight_scale', N.ptr(w2), N.dt(w2), w2.shape[0], cols, int(group), i,
               len(weights), N.ptr(total), N.ptr(ws), N.stream_of(w2))
    return total


def ratio_in_dtype(ratio: float, dtype: torch.dtype) -> float:
    """The exponent as torch applies it to a `dtype` tensor (rounded to dtype)."""
    return float(torch.tensor(ratio, dtype=torch.float32).to(dtype).item())


def awq_scales(xmean: torch.Tensor, ratio: float, out: torch.Tensor | None = None,
               w_max: torch.Tensor | None = None) -> torch.Tensor:
    """AWQ scales for one grid ratio (awq.py:87-108): v2, or v1 when ``w_max`` is given."""
    out = torch.empty_like(xmean) if out is None else out
    if w_max is None:
        N.call('lcq_awq_scales', N.ptr(xmean), N.dt(xmean), xmean.numel(),
               ratio_in_dtype(ratio, xmean.dtype), N.ptr(out), N.stream_of(xmean))
    else:
        if w_max.dtype != xmean.dtype or w_max.numel() != xmean.numel():
            raise ValueError('w_max must match x_mean')
        N.call('lcq_awq_scales_v1', N.ptr(xmean), N.ptr(w_max.contiguous()), N.dt(xmean),
               xmean.numel(), ratio_in_dtype(ratio, xmean.dtype),
               ratio_in_dtype(1 - ratio, xmean.dtype), N.ptr(out), N.stream_of(xmean))
    return out


def scale_bcast(x: torch.Tensor, s: torch.Tensor, op: str, axis: int = 0,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """out = x * s or x / s broadcast over columns (axis 0) or rows (axis 1); in place if
    out is x. Per-op rounding in x.dtype."""
    x2 = x.reshape(-1, x.shape[-1])
    rows, cols = x2.shape
    if s.dtype != x.dtype:
        raise ValueError('scale must have the tensor dtype')
    s = s.contiguous()
    if s.numel() != (cols if axis == 0 else rows):
        raise ValueError('scale length does not match the broadcast axis')
    o = torch.empty_like(x) if out is None else out
    N.call('lcq_scale_bcast', N.ptr(x2), N.dt(x2), rows, cols, N.ptr(s),
           0 if op == 'mul' else 1, int(axis), N.ptr(o), N.stream_of(x2))
    return o


class LossBuffer:
    """Device-resident loss slots + fp64 workspace for lcq_sq_diff_mean (no per-ratio sync)."""

    def __init__(self, slots: int, device, nparts: int = 1024):
        self.out = torch.zeros((slots,), dtype=torch.float32, device=device)
        self.ws = torch.empty((nparts,), dtype=torch.float64, device=device)
        self.nparts = nparts
        self._gws = None

    def gemm_ws(self, m: int, n: int) -> torch.Tensor:
        """fp64 tile partials of lcq_gemm_sq_diff (grown on demand, reused across ratios)."""
        need = (N.load().lcq_gemm_sq_diff_workspace_bytes(m, n) + 7) // 8
        if self._gws is None or self._gws.numel() < need:
            self._gws = torch.empty((need,), dtype=torch.float64, device=self.out.device)
        return self._gws

    def record(self, a: torch.Tensor, b: torch.Tensor, slot: int):
        a = a.contiguous()
        b = b.contiguous()
        N.call('lcq_sq_diff_mean', N.ptr(a), N.ptr(b), N.dt(a), a.numel(), N.ptr(self.ws),
               self.nparts, N.ptr(self.out), int(slot), N.stream_of(a))


# ---- projection GEMMs (csrc/gemm256.hip; awq.py:110-145 inspect forwards + calculate_loss) ----
def _rows2d(x: torch.Tensor) -> torch.Tensor:
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    if x2.stride(-1) != 1 or x2.stride(0) % 8 != 0 or x2.data_ptr() % 16 != 0:
        x2 = x2.contiguous()
    return x2


def gemm_supported(x: torch.Tensor, *weights: torch.Tensor) -> bool:
    """Shapes / dtypes the lcq GEMMs take (others go to the caller's own path)."""
    K = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and K % 64 == 0
            and x.numel() > 0 and all(
                w.is_cuda and w.dtype == x.dtype and w.dim() == 2 and w.shape[1] == K
                and w.stride(1) == 1 and w.stride(0) % 8 == 0 and w.data_ptr() % 16 == 0
                and w.shape[0] % 16 == 0 for w in weights))


def _wstride(ws):
    ld = ws[0].stride(0)
    if any(w.stride(0) != ld for w in ws):
        raise ValueError('weights must share a row stride')
    return ld


def linear_multi(x: torch.Tensor, weights, biases=None):
    """[F.linear(x, w_s, b_s) for each weight] from one GEMM launch (x read once)."""
    import ctypes
    x2 = _rows2d(x)
    M, K = x2.shape
    n = len(weights)
    if not 1 <= n <= 3:
        raise ValueError('1..3 weights')
    for w in weights[:-1]:
        if w.shape[0] % 256 != 0:
            raise ValueError('all but the last weight need a multiple of 256 rows')
    outs = [torch.empty((M, w.shape[0]), dtype=x.dtype, device=x.device) for w in weights]
    bs = list(biases) if biases is not None else [None] * n
    for b, w in zip(bs, weights):
        if b is not None and (b.dtype != x.dtype or b.numel() != w.shape[0] or not b.is_contiguous()):
            raise ValueError('bias must be contiguous [N] in the input dtype')
    arr_b = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in weights])
    arr_r = (ctypes.c_int64 * 3)(*[w.shape[0] for w in weights])
    arr_bias = (ctypes.c_void_p * 3)(*[None if b is None else b.data_ptr() for b in bs])
    arr_c = (ctypes.c_void_p * 3)(*[o.data_ptr() for o in outs])
    arr_ld = (ctypes.c_int64 * 3)(*[o.shape[1] for o in outs])
    N.call('lcq_gemm', N.ptr_strided(x2), N.dt(x2), x2.stride(0), M, K, n, arr_b, arr_r,
           _wstride(weights), arr_bias, arr_c, arr_ld, N.stream_of(x2))
    Ntot = sum(w.shape[0] for w in weights)
    N.note_work('lcq_gemm', 2.0 * M * K * Ntot)
    N.note_bytes('lcq_gemm', 2.0 * (M * K + Ntot * K + M * Ntot))
    return [o.view(*x.shape[:-1], o.shape[1]) for o in outs]


def linear_multi_rope(x: torch.Tensor, weights, biases, cos: torch.Tensor, sin: torch.Tensor,
                      rope_segs: int = 2):
    """linear_multi with transformers' apply_rotary_pos_emb applied to the first `rope_segs`
    outputs in the GEMM epilogue (lcq_gemm_rope; the q / k of LlamaAttention): x [B, S, C],
    cos / sin [1 or B, S, 128] in x's dtype, heads of 128. Bit-identical to linear_multi
    followed by rotary on the head-transposed views, without the rotary kernel's extra
    read + write of q and k."""
    import ctypes
    if x.dim() != 3:
        raise ValueError('x must be [B, S, C]')
    B, S, _ = x.shape
    x2 = _rows2d(x)
    M, K = x2.shape
    n = len(weights)
    if not 1 <= n <= 3 or not 0 <= rope_segs <= n:
        raise ValueError('1..3 weights, rope_segs <= n')
    for w in weights[:-1]:
        if w.shape[0] % 256 != 0:
            raise ValueError('all but the last weight need a multiple of 256 rows')
    cos, sin = cos.contiguous(), sin.contiguous()
    if (cos.dim() != 3 or tuple(cos.shape[1:]) != (S, 128) or cos.shape[0] not in (1, B)
            or sin.shape != cos.shape or cos.dtype != x.dtype or sin.dtype != x.dtype):
        raise ValueError('cos / sin must be [1 or B, S, 128] in the input dtype')
    outs = [torch.empty((M, w.shape[0]), dtype=x.dtype, device=x.device) for w in weights]
    bs = list(biases) if biases is not None else [None] * n
    for b, w in zip(bs, weights):
        if b is not None and (b.dtype != x.dtype or b.numel() != w.shape[0] or not b.is_contiguous()):
            raise ValueError('bias must be contiguous [N] in the input dtype')
    arr_b = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in weights])
    arr_r = (ctypes.c_int64 * 3)(*[w.shape[0] for w in weights])
    arr_bias = (ctypes.c_void_p * 3)(*[None if b is None else b.data_ptr() for b in bs])
    arr_c = (ctypes.c_void_p * 3)(*[o.data_ptr() for o in outs])
    arr_ld = (ctypes.c_int64 * 3)(*[o.shape[1] for o in outs])
    N.call('lcq_gemm_rope', N.ptr_strided(x2), N.dt(x2), x2.stride(0), M, K, n, arr_b, arr_r,
           _wstride(weights), arr_bias, arr_c, arr_ld, int(rope_segs), N.ptr(cos), N.ptr(sin),
           S, 0 if cos.shape[0] == 1 else S * 128, 128, N.stream_of(x2))
    Ntot = sum(w.shape[0] for w in weights)
    N.note_work('lcq_gemm_rope', 2.0 * M * K * Ntot)
    N.note_bytes('lcq_gemm_rope', 2.0 * (M * K + Ntot * K + M * Ntot + 2 * cos.numel()))
    return [o.view(B, S, o.shape[1]) for o in outs]


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    """F.linear(x, weight, bias) on the lcq GEMM (fp32 accumulation, one rounding)."""
    return linear_multi(x, [weight], None if bias is None else [bias])[0]


def linear_residual(x: torch.Tensor, weight: torch.Tensor, residual: torch.Tensor,
                    bias=None) -> torch.Tensor:
    """residual + F.linear(x, weight, bias) with the add in the GEMM epilogue (lcq_gemm_residual:
    the same two roundings as the torch expression)."""
    x2 = _rows2d(x)
    M, K = x2.shape
    Nn = weight.shape[0]
    r2 = residual.reshape(-1, Nn)
    if r2.shape[0] != M or r2.dtype != x.dtype:
        raise ValueError('residual must be [.., N] matching x rows and dtype')
    if r2.stride(-1) != 1 or r2.stride(0) % 4 != 0 or r2.data_ptr() % 8 != 0:
        r2 = r2.contiguous()
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != Nn
                             or not bias.is_contiguous()):
        raise ValueError('bias must be contiguous [N] in the input dtype')
    out = torch.empty((M, Nn), dtype=x.dtype, device=x.device)
    N.call('lcq_gemm_residual', N.ptr_strided(x2), N.dt(x2), x2.stride(0), M, K,
           weight.data_ptr(), weight.stride(0), Nn, None if bias is None else N.ptr(bias),
           N.ptr_strided(r2), r2.stride(0), N.ptr(out), Nn, N.stream_of(x2))
    N.note_work('lcq_gemm_residual', 2.0 * M * K * Nn)
    N.note_bytes('lcq_gemm_residual', 2.0 * (M * K + Nn * K + 2 * M * Nn))
    return out.view(*x.shape[:-1], Nn)


def linear_silu_mul(x: torch.Tensor, gate_w: torch.Tensor, up_w: torch.Tensor) -> torch.Tensor:
    """act_fn(gate_proj(x)) * up_proj(x) (SiLU, no bias) in one GEMM; the [.., I] projections
    are never materialised."""
    x2 = _rows2d(x)
    M, K = x2.shape
    I = gate_w.shape[0]
    if tuple(up_w.shape) != tuple(gate_w.shape):
        raise ValueError('gate / up weights must match')
    h = torch.empty((M, I), dtype=x.dtype, device=x.device)
    N.call('lcq_gemm_silu_mul', N.ptr_strided(x2), N.dt(x2), x2.stride(0), M, K,
           gate_w.data_ptr(), up_w.data_ptr(), _wstride([gate_w, up_w]), I, N.ptr(h), I,
           N.stream_of(x2))
    N.note_work('lcq_gemm_silu_mul', 4.0 * M * K * I)
    N.note_bytes('lcq_gemm_silu_mul', 2.0 * (M * K + 2 * I * K + M * I))
    return h.view(*x.shape[:-1], I)


def linear_sq_diff(x: torch.Tensor, weight: torch.Tensor, ref: torch.Tensor,
                   losses: 'LossBuffer', slot: int, bias=None):
    """losses.out[slot] = mean((ref - F.linear(x, weight, bias))^2) (calculate_loss,
    awq.py:134-145) without writing the linear's output."""
    x2 = _rows2d(x)
    M, K = x2.shape
    Nn = weight.shape[0]
    r2 = ref.reshape(-1, Nn)
    if r2.shape[0] != M or r2.dtype != x.dtype:
        raise ValueError('ref must be [.., N] matching x rows and dtype')
    if r2.stride(-1) != 1 or r2.stride(0) % 4 != 0:
        r2 = r2.contiguous()
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != Nn):
        raise ValueError('bias must be [N] in the input dtype')
    ws = losses.gemm_ws(M, Nn)
    N.call('lcq_gemm_sq_diff', N.ptr_strided(x2), N.dt(x2), x2.stride(0), M, K,
           weight.data_ptr(), weight.stride(0), Nn, None if bias is None else N.ptr(bias),
           N.ptr_strided(r2), r2.stride(0), N.ptr(ws), ws.numel() * 8, N.ptr(losses.out),
           int(slot), N.stream_of(x2))
    N.note_work('lcq_gemm_sq_diff', 2.0 * M * K * Nn)
    N.note_bytes('lcq_gemm_sq_diff', 2.0 * (M * K + Nn * K + M * Nn))


def sq_diff_mean(a: torch.Tensor, b: torch.Tensor) -> float:
    lb = LossBuffer(1, a.device)
    lb.record(a, b, 0)
    return float(lb.out[0].item())


def auto_clip_search(w: torch.Tensor, x: torch.Tensor, group: int, nsteps: int, n_grid: int,
                     qmin: int, qmax: int, sym: bool, clip_sym: bool, mse=None,
                     qx: torch.Tensor | None = None, fp8=None, tensor_batch: int = 0,
                     version: int = 1):
    """AutoClipper.auto_clip_layer on device: returns (best_max, best_min) [oc, ng, 1].
    mse = (steps, grid, norm): the weight quantizer's calib_algo is mse. qx: the activation
    fake-quant of x (w_only False) that the shrink steps multiply with. group == ic takes the
    per_channel kernel (lcq_auto_clip_search_pc). fp8 (a float8 dtype): FloatQuantizer weights,
    per_channel (tensor_batch 0) or per_tensor over batches of tensor_batch rows (group == ic).
    version 2: clip_version v2 candidates (learnable range of the unclamped weight), integer
    per_channel weights only."""
    oc, ic = w.shape
    if version == 2 and (group != ic or fp8 is not None or mse is not None):
        raise NotImplementedError('clip_version v2 on the device: integer per_channel, minmax')
    if qx is not None and (qx.shape != x.shape or qx.dtype != x.dtype):
        raise ValueError('auto-clip: qx must match x in shape and dtype')
    if fp8 is not None and (group != ic or mse is not None):
        raise NotImplementedError('float-quant auto-clip: per_channel / per_tensor, minmax')
    if group == ic and (group not in (32, 64, 128, 256) or fp8 is not None):
        if mse is not None:
            raise NotImplementedError('per_channel auto-clip with calib_algo mse')
        return _auto_clip_search_pc(w, x, qx, nsteps, n_grid, qmin, qmax, sym, clip_sym,
                                    fp8=fp8, tensor_batch=tensor_batch, version=version)
    if version == 2:
        return _auto_clip_search_pc(w, x, qx, nsteps, n_grid, qmin, qmax, sym, clip_sym,
                                    version=2)
    T = x.shape[0]
    factors = _const_f32([float(1 - i / n_grid) for i in range(nsteps)], w.device)
    ng = ic // group
    bmax = torch.empty((oc, ng, 1), dtype=w.dtype, device=w.device)
    bmin = torch.empty((oc, ng, 1), dtype=w.dtype, device=w.device)
    if x.dtype != w.dtype:
        raise ValueError('auto-clip: x and w must share the model dtype')
    msteps, mp, norm = 0, None, 0.0
    if mse is not None:
        msteps, grid, norm = int(mse[0]), float(mse[1]), float(mse[2])
        mp = _const_f32([float(1 - i / grid) for i in range(msteps)], w.device)
    args = (N.ptr(w.contiguous()), N.ptr(x.contiguous()),
            N.ptr(qx.contiguous() if qx is not None else None), N.dt(w), oc, ic, T, int(group),
            int(nsteps), N.ptr(factors), int(qmin), int(qmax), int(sym), int(clip_sym), msteps,
            N.ptr(mp), norm, N.ptr(bmax), N.ptr(bmin))
    ws_bytes = (int(N.load().lcq_auto_clip_workspace_bytes(oc, ic, T, int(group), int(nsteps)))
                if CLIP_TOKEN_LANE and qx is None and mse is None else 0)
    if ws_bytes:   # the scalar-operand kernels (weight-only, group 128, minmax): same bits
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=w.device)
        N.call('lcq_auto_clip_search_ws', *args, ws.data_ptr(), ws_bytes, N.stream_of(w))
        name = 'lcq_auto_clip_search_ws'
    else:
        N.call('lcq_auto_clip_search_act', *args, N.stream_of(w))
        name = 'lcq_auto_clip_search_act'
    # algorithmic work: DT-rounded products, the original outputs and every shrink step
    N.note_work(name, float(oc) * ic * T * (1 + nsteps))
    return bmax, bmin


CLIP_TOKEN_LANE = True   # module switch for A/B runs and tests (False: k_auto_clip only)
# (the name predates the row-lane kernel: True = lcq_auto_clip_search_ws's kernels)


_CONST_CACHE: dict = {}


def _const_f32(values, device) -> torch.Tensor:
    """A small constant fp32 vector on the device, uploaded once per (device, values): a
    fresh torch.tensor(list, device=...) is a pageable copy that blocks the host until the
    stream drains (the host would stop running ahead of the kernels)."""
    key = (torch.device(device).index, tuple(values))
    t = _CONST_CACHE.get(key)
    if t is None:
        t = _CONST_CACHE[key] = torch.tensor(list(values), dtype=torch.float32, device=device)
    return t


def _auto_clip_search_pc(w, x, qx, nsteps, n_grid, qmin, qmax, sym, clip_sym, fp8=None,
                         tensor_batch=0, version=1):
    """per_channel weights: best bounds [oc, 1, 1] (auto_clip.py:96-99, group = ic)."""
    oc, ic = w.shape
    T = x.shape[0]
    if x.dtype != w.dtype:
        raise ValueError('auto-clip: x and w must share the model dtype')
    factors = _const_f32([float(1 - i / n_grid) for i in range(nsteps)], w.device)
    bmax = torch.empty((oc, 1, 1), dtype=w.dtype, device=w.device)
    bmin = torch.empty((oc, 1, 1), dtype=w.dtype, device=w.device)
    wsb = N.load().lcq_auto_clip_pc_workspace_bytes(oc, T, int(nsteps))
    ws = torch.empty(wsb, dtype=torch.uint8, device=w.device)
    N.call('lcq_auto_clip_search_pc', N.ptr(w.contiguous()), N.ptr(x.contiguous()),
           N.ptr(qx.contiguous() if qx is not None else None), N.dt(w), oc, ic, T, int(nsteps),
           N.ptr(factors), int(qmin), int(qmax), int(sym), int(clip_sym),
           0 if fp8 is None else N.dt(fp8), int(tensor_batch), int(version), N.ptr(ws), wsb,
           N.ptr(bmax), N.ptr(bmin), N.stream_of(w))
    return bmax, bmin


def clip_apply(w: torch.Tensor, group: int, cmax: torch.Tensor, cmin: torch.Tensor | None,
               out: torch.Tensor | None = None) -> torch.Tensor:
    rows, cols = w.shape
    o = torch.empty_like(w) if out is None else out
    N.call('lcq_clip_apply', N.ptr(w), N.dt(w), rows, cols, int(group), N.ptr(cmax.contiguous()),
           N.ptr(cmin.contiguous() if cmin is not None else None), N.ptr(o), N.stream_of(w))
    return o


def clip_factors(w: torch.Tensor, group: int, cmax: torch.Tensor, cmin: torch.Tensor | None,
                 clip_sym: bool):
    """AutoClipper.get_clip_factor (auto_clip.py:235-256): (up, low | None), [groups, 1] in
    the weight dtype, from the searched bounds and each group's own min / max."""
    rows, cols = w.shape
    ng = rows * cols // group
    up = torch.empty((ng, 1), dtype=w.dtype, device=w.device)
    low = None if clip_sym else torch.empty((ng, 1), dtype=w.dtype, device=w.device)
    for t in (cmax, cmin):
        if t is not None and (t.dtype != w.dtype or t.numel() != ng):
            raise ValueError('clip bounds: one per group, in the weight dtype')
    N.call('lcq_clip_factors', N.ptr(w.contiguous()), N.dt(w), rows, cols, int(group),
           N.ptr(cmax.contiguous()), N.ptr(cmin.contiguous() if cmin is not None else None),
           int(clip_sym), N.ptr(up), N.ptr(low), N.stream_of(w))
    return up, low


def int_quant_learnable(x: torch.Tensor, group: int, up: torch.Tensor, low: torch.Tensor | None,
                        qmin: int, qmax: int, sym: bool, *, fq_dtype=None, qparams=False):
    """Dynamic fake quant with calib_algo learnable and clip factors (quant.py:205-219):
    returns {'fq', ['scales', 'zeros']} like int_quant_dynamic."""
    rows, cols = x.shape
    ng = rows * cols // group
    for t in (up, low):
        if t is not None and (t.dtype != x.dtype or t.numel() != ng):
            raise ValueError('clip factors: one per group, in the tensor dtype')
    fq_dtype = fq_dtype or x.dtype
    res = {'fq': torch.empty((rows, cols), dtype=fq_dtype, device=x.device)}
    s_t = z_t = None
    if qparams:
        s_t = res['scales'] = torch.empty((ng, 1), dtype=x.dtype, device=x.device)
        if not sym:
            z_t = res['zeros'] = torch.empty((ng, 1), dtype=x.dtype, device=x.device)
    N.call('lcq_int_quant_learnable', N.ptr(x), N.dt(x), rows, cols, int(group),
           N.ptr(up.contiguous()), N.ptr(low.contiguous() if low is not None else None),
           int(qmin), int(qmax), int(sym), N.ptr(res['fq']), N.dt(fq_dtype), None, 0,
           N.ptr(s_t), N.ptr(z_t), N.stream_of(x))
    return res


code_dtype = _code_dtype


# ---------------------------------------------------------------------------------------
# FP8 (FloatQuantizer / kernel.py)
# ---------------------------------------------------------------------------------------
_FP8 = {'e4m3': torch.float8_e4m3fn, 'e5m2': torch.float8_e5m2}


def fp8_dtype(bit: str) -> torch.dtype:
    if bit not in _FP8:
        raise NotImplementedError(f'FP8 real quant supports e4m3 / e5m2, not {bit}')
    return _FP8[bit]


FP8_PARTIALS = 256  # LCQ_FP8_PARTIALS (include/lcq.h): scratch fp32 per per-tensor max


def absmax(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """max |x| as a device fp32 scalar (shape [1])."""
    x = x.contiguous()
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=x.device)
    ws = torch.empty(FP8_PARTIALS, dtype=torch.float32, device=x.device)
    N.call('lcq_absmax', N.ptr(x), N.dt(x.dtype), x.numel(), N.ptr(out), N.ptr(ws),
           N.stream_of(x))
    return out


def fp8_max(fp8: torch.dtype) -> float:
    return float(torch.finfo(fp8).max)


def fp8_quant(x: torch.Tensor, group: int, fp8: torch.dtype, *, ct_dtype=None,
              qmax: float | None = None, clamp_min: float = 1e-5, add_zero: bool = True, per_tensor: bool = False,
              codes: bool = True, fq: bool = False, fq_dtype=None,
              scales: bool = True) -> dict:
    """Dynamic FP8 quantization of a 2-D ``x`` over groups of ``group`` columns, or per tensor.

    Defaults follow FloatQuantizer (quant.py:545-559, 1061-1076): compute dtype = x dtype,
    scale clamp 1e-5, ``+ zeros``. kernel.py ``act_quant`` = ct fp32, clamp 0, no add_zero.
    """
    assert x.dim() == 2, 'x must be 2-D'
    x = x.contiguous()
    rows, cols = x.shape
    ct = x.dtype if ct_dtype is None else ct_dtype
    res = {}
    amax = absmax(x) if per_tensor else None
    if per_tensor:
        group = cols
    c = torch.empty((rows, cols), dtype=fp8, device=x.device) if codes else None
    f = torch.empty((rows, cols), dtype=fq_dtype or x.dtype, device=x.device) if fq else None
    ns = 1 if per_tensor else rows * cols // group
    sdt = torch.float32 if per_tensor else ct  # 0-dim / 0-dim promotes to fp32
    s = torch.empty((ns, 1), dtype=sdt, device=x.device) if scales else None
    qmax = fp8_max(fp8) if qmax is None else float(qmax)
    N.call('lcq_fp8_quant', N.ptr(x), N.dt(x.dtype), rows, cols, group, N.dt(fp8), N.dt(ct),
           qmax, float(clamp_min), int(add_zero), N.ptr(amax), N.ptr(c), N.ptr(f),
           N.dt(f.dtype) if f is not None else 0, N.ptr(s), N.stream_of(x))
    if codes:
        res['codes'] = c
    if fq:
        res['fq'] = f
    if scales:
        res['scales'] = s
    return res


def fp8_quant_static(x: torch.Tensor, scales: torch.Tensor, fp8: torch.dtype, *,
                     ct_dtype=None, add_zero: bool = True, codes: bool = True,
                     fq: bool = False, fq_dtype=None, saturate: bool = False) -> dict:
    """FP8 quant of ``x`` with given scales; one scale per ``x.numel() / scales.numel()``
    consecutive elements (per tensor / per row / per group layouts). saturate clamps the
    quotient to +-finfo.max first (FloatQuantizer's float_quantize stand-in); without it the
    cast is torch's ``.to()`` (out-of-range quotients -> NaN / inf)."""
    x = x.contiguous()
    s = scales.contiguous()
    if x.numel() % s.numel():
        raise ValueError('scales do not tile the tensor')
    group = x.numel() // s.numel()
    ct = ct_dtype or torch.promote_types(x.dtype, s.dtype)
    c = torch.empty(x.shape, dtype=fp8, device=x.device) if codes else None
    f = torch.empty(x.shape, dtype=fq_dtype or x.dtype, device=x.device) if fq else None
    rows = x.shape[0] if x.dim() > 1 else 1
    N.call('lcq_fp8_quant_static', N.ptr(x), N.dt(x.dtype), rows, x.numel() // rows, group,
           N.dt(fp8), N.dt(ct), N.ptr(s), N.dt(s.dtype), int(add_zero), int(saturate),
           N.ptr(c), N.ptr(f),
           N.dt(f.dtype) if f is not None else 0, N.stream_of(x))
    res = {}
    if codes:
        res['codes'] = c
    if fq:
        res['fq'] = f
    return res


def fp8_quant_blocks(x: torch.Tensor, fp8: torch.dtype = torch.float8_e4m3fn, block: int = 128,
                     *, qmax: float | None = None, clamp_min: float = 1e-5, add_zero: bool = True, codes: bool = True,
                     fq: bool = False, fq_dtype=None) -> dict:
    """128x128-block FP8 quant (per_block FloatQuantizer / weight_cast_to_fp8)."""
    assert x.dim() == 2, 'x must be 2-D'
    x = x.contiguous()
    M, Nn = x.shape
    c = torch.empty((M, Nn), dtype=fp8, device=x.device) if codes else None
    f = torch.empty((M, Nn), dtype=fq_dtype or x.dtype, device=x.device) if fq else None
    s = torch.empty(((M + block - 1) // block, (Nn + block - 1) // block), dtype=torch.float32,
                    device=x.device)
    qmax = fp8_max(fp8) if qmax is None else float(qmax)
    N.call('lcq_fp8_quant_blocks', N.ptr(x), N.dt(x.dtype), M, Nn, block, N.dt(fp8), qmax,
           float(clamp_min), int(add_zero), N.ptr(c), N.ptr(f),
           N.dt(f.dtype) if f is not None else 0, N.ptr(s), N.stream_of(x))
    res = {'scales': s}
    if codes:
        res['codes'] = c
    if fq:
        res['fq'] = f
    return res


def fp8_dequant_blocks(codes: torch.Tensor, scales: torch.Tensor, block: int = 128,
                       out_dtype: torch.dtype = torch.bfloat16,
                       out: torch.Tensor | None = None) -> torch.Tensor:
    """weight_cast_to_bf16: rnd_out(float(code) * scale[block])."""
    assert codes.dim() == 2 and scales.dim() == 2
    codes = codes.contiguous()
    scales = scales.contiguous().float()
    M, Nn = codes.shape
    if scales.shape != ((M + block - 1) // block, (Nn + block - 1) // block):
        raise ValueError(f'scale shape {tuple(scales.shape)} does not tile {M}x{Nn} by {block}')
    if out is None:
        out = torch.empty((M, Nn), dtype=out_dtype, device=codes.device)
    N.call('lcq_fp8_dequant_blocks', N.ptr(codes), N.dt(codes.dtype), M, Nn, block,
           N.ptr(scales), N.ptr(out), N.dt(out.dtype), N.stream_of(codes))
    return out


def fp8_gemm(a: torch.Tensor, a_s: torch.Tensor, b: torch.Tensor, b_s: torch.Tensor,
             out_dtype: torch.dtype | None = None) -> torch.Tensor:
    """fp8_gemm (kernel.py:216-242): a [..., K] e4m3 with a_s [..., K/128]; b [N, K] e4m3 with
    b_s [ceil(N/128), K/128]; returns c [..., N] in ``out_dtype`` (default
    torch.get_default_dtype(), as the reference allocates it)."""
    assert a.is_contiguous() and b.is_contiguous(), 'Input tensors must be contiguous'
    assert a_s.is_contiguous() and b_s.is_contiguous(), (
        'Scaling factor tensors must be contiguous')
    if a.dtype != torch.float8_e4m3fn or b.dtype != torch.float8_e4m3fn:
        raise TypeError(f'fp8_gemm takes float8_e4m3fn operands, got {a.dtype} / {b.dtype}')
    K = a.size(-1)
    M = a.numel() // K
    Nn = b.size(0)
    if b.dim() != 2 or b.size(1) != K:
        raise ValueError(f'b shape {tuple(b.shape)} does not match K={K}')
    if K % 128 != 0:
        raise ValueError(f'K={K} is not a multiple of the 128-column scale block')
    nkb = K // 128
    if a_s.numel() != M * nkb or a_s.dtype != torch.float32:
        raise ValueError(f'a_s must be fp32 with {M}x{nkb} elements')
    if tuple(b_s.shape) != ((Nn + 127) // 128, nkb) or b_s.dtype != torch.float32:
        raise ValueError(f'b_s must be fp32 [{(Nn + 127) // 128}, {nkb}]')
    out_dtype = torch.get_default_dtype() if out_dtype is None else out_dtype
    c = torch.empty(*a.shape[:-1], Nn, dtype=out_dtype, device=a.device)
    if M == 0:
        return c
    wsb = int(N.load().lcq_fp8_gemm_workspace_bytes(M, Nn, K))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=a.device)
    N.call('lcq_fp8_gemm', N.ptr(a), N.ptr(a_s), N.ptr(b), N.ptr(b_s), M, Nn, K, N.ptr(c),
           N.dt(out_dtype), N.ptr(ws), wsb, N.stream_of(a))
    return c


def fp8_weight_table(weights, device) -> torch.Tensor:
    """Device table [G, 2] int64 of (weight, block-scale) addresses for fp8_gemm_grouped, after
    checking every pair: weight [N, K] e4m3 contiguous 16-byte aligned, scales fp32 contiguous
    [ceil(N/128), K/128], one (N, K) for all. The tensors must outlive every launch that reads
    the table (the caller keeps them with it)."""
    rows = []
    shape = None
    for w, s in weights:
        if w.dtype != torch.float8_e4m3fn or not w.is_contiguous() or w.dim() != 2:
            raise TypeError('grouped fp8 weights must be contiguous 2-D float8_e4m3fn')
        if shape is None:
            shape = tuple(w.shape)
        if tuple(w.shape) != shape:
            raise ValueError(f'grouped fp8 weights differ in shape: {tuple(w.shape)} vs {shape}')
        n, k = shape
        if (s.dtype != torch.float32 or not s.is_contiguous()
                or tuple(s.shape) != ((n + 127) // 128, k // 128)):
            raise ValueError(f'block scales must be contiguous fp32 [{(n + 127) // 128}, '
                             f'{k // 128}]')
        if w.data_ptr() % 16:
            raise ValueError('grouped fp8 weights must be 16-byte aligned')
        rows.append((w.data_ptr(), s.data_ptr()))
    return torch.tensor(rows, dtype=torch.int64).to(device)


def fp8_gemm_grouped(a: torch.Tensor, a_s: torch.Tensor, row_off: torch.Tensor,
                     wtab: torch.Tensor, n: int, out_dtype: torch.dtype = torch.bfloat16,
                     a_rows: torch.Tensor | None = None, silu_mul: bool = False
                     ) -> torch.Tensor:
    """One launch of G block-scaled fp8 GEMMs (the routed experts of an MoE projection), for
    one or two weight sets. Rows: the token slots sorted by group, row_off int64 [G + 1] on
    the device (group g = rows [row_off[g], row_off[g + 1])). a [R, K] e4m3 with a_s [R, K/128]
    (act_quant): with ``a_rows`` (int64 [rows] on the device) sorted row i is a[a_rows[i]] --
    the gather happens in the kernel -- else a itself is sorted (rows = R). wtab from
    fp8_weight_table, [G, 2] or [2, G, 2] (two sets: gate and up of the same rows), all [n, K].
    Returns c [rows, n], or [2, rows, n] for two sets; each row equals fp8_gemm's on an
    unsplit 256^2 plan. ``silu_mul`` (two sets = gate, up; bf16): returns h [rows, n] =
    rnd(rnd(silu(rnd(gate))) * rnd(up)), the expert MLP's act_fn(gate) * up, with neither
    projection stored."""
    if a.dtype != torch.float8_e4m3fn or not a.is_contiguous() or a.dim() != 2:
        raise TypeError('a must be a contiguous 2-D float8_e4m3fn tensor')
    R, K = a.shape
    if K % 128:
        raise ValueError(f'K={K} is not a multiple of the 128-column scale block')
    if a_s.dtype != torch.float32 or not a_s.is_contiguous() or a_s.numel() != R * (K // 128):
        raise ValueError(f'a_s must be contiguous fp32 with {R}x{K // 128} elements')
    nsets = 1 if wtab.dim() == 2 else wtab.shape[0]
    G = wtab.shape[-2]
    if (wtab.dtype != torch.int64 or wtab.shape[-1] != 2 or nsets not in (1, 2)
            or wtab.dim() not in (2, 3) or not wtab.is_contiguous()
            or wtab.device != a.device):
        raise ValueError('wtab must be int64 [G, 2] or [2, G, 2] on a\'s device')
    if row_off.dtype != torch.int64 or row_off.numel() != G + 1 or row_off.device != a.device:
        raise ValueError('row_off must be int64 [G + 1] on a\'s device')
    if a_rows is not None:
        if (a_rows.dtype != torch.int64 or a_rows.dim() != 1 or not a_rows.is_contiguous()
                or a_rows.device != a.device):
            raise ValueError('a_rows must be a contiguous int64 vector on a\'s device')
        rows = a_rows.numel()
    else:
        rows = R
    if silu_mul and (nsets != 2 or out_dtype != torch.bfloat16):
        raise ValueError('silu_mul takes the gate and up tables ([2, G, 2]) and a bf16 output')
    shape = (rows, n) if nsets == 1 or silu_mul else (nsets, rows, n)
    c = torch.empty(shape, dtype=out_dtype, device=a.device)
    if rows == 0:
        return c
    wsb = int(N.load().lcq_fp8_gemm_grouped_workspace_bytes(rows, G, 2 * n if silu_mul else n,
                                                            K))
    ws = torch.empty(wsb, dtype=torch.uint8, device=a.device)
    N.call('lcq_fp8_gemm_grouped', N.ptr(a), N.ptr(a_s), R,
           None if a_rows is None else N.ptr(a_rows), rows, N.ptr(row_off), N.ptr(wtab), G,
           nsets, int(bool(silu_mul)), n, K, N.ptr(c), N.dt(out_dtype), N.ptr(ws), wsb,
           N.stream_of(a))
    return c


def moe_combine(y: torch.Tensor, slot_row: torch.Tensor, expert: torch.Tensor,
                weights: torch.Tensor, T: int) -> torch.Tensor:
    """out [T, H] bf16: per token, its k slots' expert rows y[slot_row] (bf16, the grouped
    GEMM's sorted order) times their routing weights, rounded to bf16 and summed in ascending
    expert id with a bf16 rounding per add -- the expert loop's index_add_ combine
    (lcq_moe_combine)."""
    if y.dtype != torch.bfloat16 or not y.is_contiguous() or y.dim() != 2:
        raise TypeError('y must be a contiguous 2-D bf16 tensor')
    k = expert.shape[-1]
    if (slot_row.dtype != torch.int64 or expert.dtype != torch.int64
            or slot_row.numel() != T * k or expert.numel() != T * k
            or weights.numel() != T * k or weights.dtype not in (torch.float32, torch.bfloat16)):
        raise ValueError('slot_row / expert int64 and weights fp32 / bf16, all [T, k]')
    H = y.shape[1]
    out = torch.empty((T, H), dtype=torch.bfloat16, device=y.device)
    N.call('lcq_moe_combine', N.ptr(y), N.ptr(slot_row.contiguous()),
           N.ptr(expert.contiguous()), N.ptr(weights.contiguous()), N.dt(weights.dtype), T, k,
           H, N.ptr(out), N.stream_of(y))
    return out

def fp8_block_to_tensor(codes: torch.Tensor, scales_inv: torch.Tensor, block: int = 128,
                        fp8: torch.dtype = torch.float8_e4m3fn, qmax: float | None = None):
    """Block-fp8 weight -> bf16 (weight_cast_to_bf16) -> per-tensor fp8 real quant, fused.
    Returns (codes [M, N] fp8, scale [1] fp32)."""
    codes = codes.contiguous()
    scales_inv = scales_inv.contiguous().float()
    M, Nn = codes.shape
    ws = torch.empty(FP8_PARTIALS, dtype=torch.float32, device=codes.device)
    out = torch.empty((M, Nn), dtype=fp8, device=codes.device)
    s = torch.empty(1, dtype=torch.float32, device=codes.device)
    qmax = fp8_max(fp8) if qmax is None else float(qmax)
    N.call('lcq_fp8_block_to_tensor', N.ptr(codes), N.dt(codes.dtype), M, Nn, block,
           N.ptr(scales_inv), N.dt(fp8), qmax, 1e-5, 1, N.ptr(ws), N.ptr(out), N.ptr(s),
           N.stream_of(codes))
    return out, s


def fp8_block_to_tensor_many(codes: list, scales_inv: list, block: int = 128,
                             fp8: torch.dtype = torch.float8_e4m3fn, qmax: float | None = None):
    """Batched fp8_block_to_tensor: block-fp8 weights (all on one device) requantized per
    tensor. Returns (list of fp8 codes, fp32 scales [n]). The launch pair sizes its grid by the
    largest tensor, so weights of very different sizes (a DeepSeek-V3 layer: o_proj 117 M
    elements, kv_a 4 M, experts 15 M) go in size classes -- one launch pair per class of
    tensors within 2x of each other -- instead of every small tensor carrying the largest one's
    idle workgroups. (Cutting a class into pairs of <= 96 MB, so that the requant pass would
    re-read the codes from the MALL, measured slower: 1.05 -> 1.29 ms per DSv3 layer.)"""
    n = len(codes)
    if n == 0:
        return [], torch.empty(0)
    dev = codes[0].device
    codes = [c.contiguous() for c in codes]
    sinv = [s.contiguous().float() for s in scales_inv]
    outs = [torch.empty(c.shape, dtype=fp8, device=dev) for c in codes]
    for c in codes:
        if c.shape[1] % 8:
            raise ValueError('N must be a multiple of 8')
    sc = torch.empty(n, dtype=torch.float32, device=dev)
    qmax = fp8_max(fp8) if qmax is None else float(qmax)
    order = sorted(range(n), key=lambda i: -codes[i].numel())
    classes, cur = [], []
    for i in order:
        if cur and codes[i].numel() * 2 < codes[cur[0]].numel():
            classes.append(cur)
            cur = []
        cur.append(i)
    classes.append(cur)
    ws = torch.empty(max(len(c) for c in classes) * FP8_PARTIALS, dtype=torch.float32,
                     device=dev)
    flat = [i for cls in classes for i in cls]    # class order
    rec = []
    for i in flat:
        M, Nn = codes[i].shape
        rec += [N.ptr(codes[i]), N.ptr(sinv[i]), N.ptr(outs[i]), M, Nn]
    # every class's descriptors (and the class order, to put the scales back) in ONE upload
    # pinned + non_blocking: a pageable upload would hold the host until the stream drains
    # (the deploy's host work would stop running ahead of its kernels)
    upload = torch.tensor(rec + flat, dtype=torch.int64, pin_memory=True).to(dev,
                                                                              non_blocking=True)
    descs = upload[:5 * n]
    # the kernel writes scale p for weight flat[p]: unless the class order is the input order,
    # the scales land in a temporary and are scattered back to input order
    in_order = flat == list(range(n))
    sc_cls = sc if in_order else torch.empty(n, dtype=torch.float32, device=dev)
    off = 0
    for cls in classes:
        N.call('lcq_fp8_block_to_tensor_many', len(cls), descs.data_ptr() + off * 40,
               codes[cls[0]].numel(), N.dt(codes[0].dtype), block, N.dt(fp8), qmax, 1e-5, 1,
               N.ptr(ws), sc_cls.data_ptr() + off * 4, N.stream_of(codes[0]))
        off += len(cls)
    if not in_order:
        sc[upload[5 * n:]] = sc_cls
    return outs, sc


def fp_emul_quant(x: torch.Tensor, group: int, e_bits: int, m_bits: int,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """FloatQuantizer use_qtorch=False fake quant over groups of ``group`` columns."""
    assert x.dim() == 2, 'x must be 2-D'
    x = x.contiguous()
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    N.call('lcq_fp_emul_quant', N.ptr(x), N.dt(x.dtype), rows, cols, group, e_bits, m_bits,
           N.ptr(out), N.dt(out.dtype), N.stream_of(x))
    return out


# ---------------------------------------------------------------------------------------
# calibration-forward fusions
# ---------------------------------------------------------------------------------------
def rotary(q: torch.Tensor, k: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor):
    """apply_rotary_pos_emb for head-transposed views q [B, Hq, S, D], k [B, Hk, S, D] whose
    storage is [B, S, H, D] (the projection output); cos / sin [Bc, S, D]. Returns (q', k') in
    the same layout, bit-identical to the torch ops."""
    B, Hq, S, D = q.shape
    Hk = k.shape[1]
    qs, ks = q.transpose(1, 2), k.transpose(1, 2)
    if not (qs.is_contiguous() and ks.is_contiguous()):
        raise ValueError('rotary expects head-transposed views of contiguous projections')
    cos = cos.contiguous()
    sin = sin.contiguous()
    if cos.dim() != 3 or cos.shape[-2:] != (S, D) or cos.shape[0] not in (1, B) or sin.shape != cos.shape:
        raise ValueError('cos / sin must be [1 or B, S, D]')
    oq = torch.empty_like(qs)
    ok = torch.empty_like(ks)
    N.call('lcq_rotary', N.ptr(qs), N.ptr(ks), N.ptr(cos), N.ptr(sin), N.dt(q.dtype), B, S, Hq,
           Hk, D, 0 if cos.shape[0] == 1 else S * D, N.ptr(oq), N.ptr(ok), N.stream_of(q))
    return oq.transpose(1, 2), ok.transpose(1, 2)


def silu_mul(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """act_fn(gate) * up with SiLU, one pass."""
    gate = gate.contiguous()
    up = up.contiguous()
    if gate.shape != up.shape or gate.dtype != up.dtype:
        raise ValueError('gate / up must match')
    out = torch.empty_like(gate)
    N.call('lcq_silu_mul', N.ptr(gate), N.ptr(up), N.dt(gate.dtype), gate.numel(), N.ptr(out),
           N.stream_of(gate))
    return out


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    """LlamaRMSNorm.forward in one pass per row (x [..., H], weight [H], same dtype)."""
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    w = weight.contiguous()
    if w.dtype != x.dtype or w.numel() != x2.shape[1]:
        raise ValueError('weight must match x dtype and hidden size')
    out = torch.empty_like(x2)
    N.call('lcq_rmsnorm', N.ptr(x2), N.ptr(w), N.dt(x.dtype), x2.shape[0], x2.shape[1],
           float(eps), N.ptr(out), N.stream_of(x2))
    return out.view(x.shape)


def attn_fwd_causal(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                    scale: float) -> torch.Tensor:
    """Causal softmax(q k^T * scale) v for q [B, H, S, 128], k / v [B, KVH, S, 128] bf16 (any
    strides with a contiguous head dim, e.g. the head-transposed projection views). Returns
    [B, S, H, 128] contiguous (the layout LlamaAttention reshapes to [B, S, H * 128])."""
    import ctypes
    B, H, S, D = q.shape
    KVH = k.shape[1]
    if tuple(k.shape) != (B, KVH, S, D) or tuple(v.shape) != tuple(k.shape):
        raise ValueError('k / v must be [B, KVH, S, D] matching q')
    strides = []
    for t in (q, k, v):
        if t.stride(-1) != 1:
            raise ValueError('head dim must be contiguous')
        strides.append((ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(2)))
    out = torch.empty((B, S, H, D), dtype=q.dtype, device=q.device)
    N.call('lcq_attn_fwd_causal', N.ptr_strided(q), N.ptr_strided(k), N.ptr_strided(v),
           N.dt(q.dtype), B, S, H, KVH, D, ctypes.addressof(strides[0]),
           ctypes.addressof(strides[1]), ctypes.addressof(strides[2]), float(scale), N.ptr(out),
           N.stream_of(q))
    N.note_work('lcq_attn_fwd_causal', 2.0 * B * H * S * (S + 1) * D)  # causal QK^T + PV flops
    return out


# ---- static activation calibration (quant.py:561-586) ---------------------------------------
MINMAX_WORKSPACE = 32 * 64  # LCQ_MINMAX_WORKSPACE (float2)
CALIB_ALGOS = {'static_minmax': 0, 'static_moving_minmax': 1}


def minmax_segments(segs) -> torch.Tensor:
    """(torch.min, torch.max) of every tensor in ``segs`` (same dtype, device) as fp32 [n, 2]
    (get_minmax_stats, quant.py:221-251, per_tensor ranges)."""
    import ctypes
    segs = [t if t.is_contiguous() else t.contiguous() for t in segs]
    if not segs:
        raise ValueError('no calibration tensors')
    dev, dt = segs[0].device, segs[0].dtype
    if any(t.dtype != dt or t.device != dev for t in segs):
        raise ValueError('calibration tensors must share dtype and device')
    n = len(segs)
    ptrs = (ctypes.c_void_p * n)(*[N.ptr(t) for t in segs])
    lens = (ctypes.c_int64 * n)(*[t.numel() for t in segs])
    out = torch.empty((n, 2), dtype=torch.float32, device=dev)
    ws = torch.empty((MINMAX_WORKSPACE, 2), dtype=torch.float32, device=dev)
    N.call('lcq_minmax_segments', ctypes.cast(ptrs, ctypes.c_void_p),
           ctypes.cast(lens, ctypes.c_void_p), n, N.dt(dt), N.ptr(out), N.ptr(ws),
           N.stream_of(out))
    N.note_work('lcq_minmax_segments', sum(t.numel() * t.element_size() for t in segs))
    return out


def act_static_qparams(minmax: torch.Tensor, algo: str, alpha: float, range_dtype: torch.dtype,
                       scale_dtype: torch.dtype, sym: bool, qmin: float, qmax: float):
    """Range (static_minmax / static_moving_minmax) + get_qparams on the device. Returns fp32
    [4] = scale, zero, min, max."""
    if algo not in CALIB_ALGOS:
        raise ValueError(f'Unsupported calibration algorithm: {algo}')
    out = torch.empty(4, dtype=torch.float32, device=minmax.device)
    N.call('lcq_act_static_qparams', N.ptr(minmax.contiguous()), minmax.shape[0],
           CALIB_ALGOS[algo], float(alpha), N.dt(range_dtype), N.dt(scale_dtype), int(bool(sym)),
           float(qmin), float(qmax), N.ptr(out), N.stream_of(minmax))
    return out


def act_static_hist_qparams(segs, minmax: torch.Tensor, bit: int, qmax: float) -> torch.Tensor:
    """static_hist range (histograms, combination, threshold search) + sym get_qparams on the
    device. Returns fp32 [4] = scale, 0, min, max."""
    import ctypes
    segs = [t if t.is_contiguous() else t.contiguous() for t in segs]
    n = len(segs)
    dev = segs[0].device
    ptrs = (ctypes.c_void_p * n)(*[N.ptr(t) for t in segs])
    lens = (ctypes.c_int64 * n)(*[t.numel() for t in segs])
    nbytes = int(N.load().lcq_act_hist_workspace_bytes(n))
    ws = torch.empty((nbytes + 3) // 4, dtype=torch.int32, device=dev)
    out = torch.empty(4, dtype=torch.float32, device=dev)
    N.call('lcq_act_static_hist_qparams', ctypes.cast(ptrs, ctypes.c_void_p),
           ctypes.cast(lens, ctypes.c_void_p), n, N.dt(segs[0]), N.ptr(minmax.contiguous()),
           2 ** int(bit), float(qmax), N.ptr(out), N.ptr(ws), N.stream_of(out))
    return out


def mse_qparams(x2: torch.Tensor, group: int, sym: bool, qmin: int, qmax: int, nsteps: int,
                grid: float, norm: float = 2.4):
    """get_mse_range + get_qparams (quant.py:145-203, 545-559) per group of `group`
    contiguous elements of x2. Returns fp32 (min, max, scales, zeros | None), one per group."""
    x2 = x2.contiguous()
    ng = x2.numel() // group
    dev = x2.device
    mn = torch.empty(ng, dtype=torch.float32, device=dev)
    mx = torch.empty_like(mn)
    s = torch.empty_like(mn)
    z = None if sym else torch.empty_like(mn)
    N.call('lcq_mse_qparams', N.ptr(x2), N.dt(x2), ng, int(group), int(bool(sym)), int(qmin),
           int(qmax), int(nsteps), float(grid), float(norm), N.ptr(mn), N.ptr(mx), N.ptr(s),
           N.ptr(z), N.stream_of(x2))
    return mn, mx, s, z


def minmax_qparams(x2: torch.Tensor, group: int, qmin: int, qmax: int, sym: bool,
                   round_zp: bool = True):
    """get_minmax_range + get_qparams (quant.py:132-143, 545-559) per group of `group`
    contiguous elements, every op in x2's dtype (incl. round_zp False). Returns (scales,
    zeros | None) [ng] in x2's dtype."""
    x2 = x2.contiguous()
    ng = x2.numel() // group
    s = torch.empty(ng, dtype=x2.dtype, device=x2.device)
    z = None if sym else torch.empty_like(s)
    N.call('lcq_minmax_qparams', N.ptr(x2), N.dt(x2), ng, int(group), int(qmin), int(qmax),
           int(bool(sym)), int(bool(round_zp)), N.ptr(s), N.ptr(z), N.stream_of(x2))
    return s, z


def hqq_proximal(w2: torch.Tensor, group: int, scales: torch.Tensor, zeros: torch.Tensor,
                 qmin: int, qmax: int, lp_norm: float, beta: float, iters: int):
    """optimize_weights_proximal (quant.py:588-610, hqq.py:36-61) on fp32 groups of w2.
    scales / zeros: fp32 [ng] starting qparams. Returns (best scales, zeros, state) where
    state = device int32 [4] view of {best error (float bits), stopped, iters run, pad}."""
    if w2.dtype != torch.float32:
        raise ValueError('hqq works on tensor.float()')
    w2 = w2.contiguous()
    ng = w2.numel() // group
    s = scales.to(torch.float32).reshape(ng).clone()
    z = zeros.to(torch.float32).reshape(ng).clone() if zeros.numel() == ng else \
        torch.full((ng,), float(zeros), dtype=torch.float32, device=w2.device)
    ws = torch.empty(int(N.load().lcq_hqq_workspace_bytes(ng)), dtype=torch.uint8, device=w2.device)
    state = torch.zeros(4, dtype=torch.int32, device=w2.device)
    N.call('lcq_hqq_proximal', N.ptr(w2), ng, int(group), N.ptr(s), N.ptr(z), int(qmin),
           int(qmax), float(lp_norm), float(beta), int(iters), N.ptr(ws), ws.numel(),
           N.ptr(state), N.stream_of(w2))
    return s, z, state
