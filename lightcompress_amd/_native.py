"""ctypes binding of the lcq C ABI (``include/lcq.h``).

The product path has no CPU fallback: if ``liblcq.so`` is missing or a tensor is not on a
ROCm device, the call raises. This is the binding a maintainer adds to the reference
(INTEGRATION.md shows the same stub against ``llmc``).
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

import torch

_LIB_PATH = Path(os.environ.get('LCQ_LIB_PATH') or
                 Path(__file__).resolve().parent / '_lib' / 'liblcq.so')  # env: A/B probes
_HEADER = Path(__file__).resolve().parent.parent / 'include' / 'lcq.h'

F32, F16, BF16, I8, U8, I32, FP8E4M3, F64, FP8E5M2 = range(9)
_DT = {
    torch.float32: F32, torch.float16: F16, torch.bfloat16: BF16, torch.int8: I8,
    torch.uint8: U8, torch.int32: I32, torch.float8_e4m3fn: FP8E4M3, torch.float64: F64,
    torch.float8_e5m2: FP8E5M2,
}

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_f32 = ctypes.c_float
_f64 = ctypes.c_double

# argument signatures of every exported entry point (kept in sync with include/lcq.h;
# tests/test_native_abi.py checks the two agree)
SIGNATURES = {
    'lcq_version': ([], _int),
    'lcq_last_error': ([], ctypes.c_char_p),
    'lcq_int_quant_dynamic': ([_vp, _int, _i64, _i64, _i64, _vp, _vp, _vp, _int, _int, _int,
                               _vp, _int, _vp, _int, _vp, _int, _vp, _vp, _vp], _int),
    'lcq_int_quant_learnable': ([_vp, _int, _i64, _i64, _i64, _vp, _vp, _int, _int, _int, _vp,
                                 _int, _vp, _int, _vp, _vp, _vp], _int),
    'lcq_int_quant_static': ([_vp, _int, _i64, _i64, _i64, _vp, _int, _vp, _int, _int, _int,
                              _int, _vp, _int, _vp, _int, _vp, _int, _vp], _int),
    'lcq_int_quant_static_nozp': ([_vp, _int, _i64, _i64, _i64, _vp, _int, _vp, _int, _int,
                                   _int, _int, _vp, _int, _vp, _int, _vp], _int),
    'lcq_minmax_qparams': ([_vp, _int, _i64, _i64, _int, _int, _int, _int, _vp, _vp, _vp], _int),
    'lcq_hqq_workspace_bytes': ([_i64], _i64),
    'lcq_hqq_proximal': ([_vp, _i64, _i64, _vp, _vp, _int, _int, _f32, _f32, _int, _vp, _i64,
                          _vp, _vp], _int),
    'lcq_int_quant_static_scalar': ([_vp, _int, _i64, _i64, _vp, _vp, _int, _int, _int, _vp,
                                     _int, _vp, _int, _vp], _int),
    'lcq_int_quant_static_cols': ([_vp, _int, _i64, _i64, _vp, _i64, _vp, _int, _vp, _int,
                                   _int, _int, _int, _vp, _int, _vp, _int, _vp], _int),
    'lcq_attn_fwd_causal': ([_vp, _vp, _vp, _int, _i64, _i64, _int, _int, _int, _vp, _vp, _vp,
                             _f32, _vp, _vp], _int),
    'lcq_pack_vllm': ([_vp, _int, _i64, _i64, _int, _vp, _vp], _int),
    'lcq_pack_autoawq_gemm': ([_vp, _int, _i64, _i64, _i64, _vp, _int, _vp, _int, _vp, _vp,
                               _vp, _vp], _int),
    'lcq_hessian_workspace_bytes': ([_i64, _i64], _i64),
    'lcq_hessian_accum': ([_vp, _int, _i64, _i64, _vp, _f32, _f32, _vp, _i64, _vp], _int),
    'lcq_tree_sum': ([_vp, _int, _i64, _f32, _vp, _vp], _int),
    'lcq_hessian_grouped_workspace_bytes': ([_vp, _int, _i64], _i64),
    'lcq_hessian_grouped': ([_vp, _int, _i64, _vp, _int, _vp, _f32, _vp, _i64, _vp], _int),
    'lcq_gptq_block': ([_vp, _i64, _i64, _i64, _int, _vp, _i64, _i64, _int, _int, _int, _int,
                        _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _int, _vp], _int),
    'lcq_gptq_block_cols': ([_vp, _i64, _i64, _i64, _int, _vp, _i64, _int, _int, _vp, _vp, _vp,
                             _i64, _vp, _i64, _vp, _vp, _int, _vp], _int),
    'lcq_chol_inv_tile': ([_vp, _i64, _int, _vp, _i64, _vp, _i64, _vp, _i64, _vp], _int),
    'lcq_gptq_trailing': ([_vp, _i64, _i64, _i64, _int, _i64, _i64, _vp, _i64, _vp, _i64, _vp],
                          _int),
    'lcq_gather_rc': ([_vp, _int, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp],
                      _int),
    'lcq_colmean_workspace_bytes': ([_i64, _i64], _i64),
    'lcq_absmean_cols': ([_vp, _int, _i64, _i64, _vp, _vp, _vp], _int),
    'lcq_awq_weight_scale': ([_vp, _int, _i64, _i64, _i64, _int, _int, _vp, _vp, _vp], _int),
    'lcq_awq_scales_v1': ([_vp, _vp, _int, _i64, _f32, _f32, _vp, _vp], _int),
    'lcq_awq_scales': ([_vp, _int, _i64, _f32, _vp, _vp], _int),
    'lcq_scale_bcast': ([_vp, _int, _i64, _i64, _vp, _int, _int, _vp, _vp], _int),
    'lcq_sq_diff_mean': ([_vp, _vp, _int, _i64, _vp, _int, _vp, _int, _vp], _int),
    'lcq_auto_clip_search': ([_vp, _vp, _int, _i64, _i64, _i64, _int, _int, _vp, _int, _int,
                              _int, _int, _int, _vp, _f32, _vp, _vp, _vp], _int),
    'lcq_auto_clip_search_act': ([_vp, _vp, _vp, _int, _i64, _i64, _i64, _int, _int, _vp, _int,
                                  _int, _int, _int, _int, _vp, _f32, _vp, _vp, _vp], _int),
    'lcq_auto_clip_workspace_bytes': ([_i64, _i64, _i64, _int, _int], _i64),
    'lcq_auto_clip_force_variant': ([_int], _int),
    'lcq_auto_clip_search_ws': ([_vp, _vp, _vp, _int, _i64, _i64, _i64, _int, _int, _vp, _int,
                                 _int, _int, _int, _int, _vp, _f32, _vp, _vp, _vp, _i64, _vp],
                                _int),
    'lcq_auto_clip_pc_workspace_bytes': ([_i64, _i64, _int], _i64),
    'lcq_auto_clip_search_pc': ([_vp, _vp, _vp, _int, _i64, _i64, _i64, _int, _vp, _int, _int,
                                 _int, _int, _int, _int, _int, _vp, _i64, _vp, _vp, _vp], _int),
    'lcq_gemm_f32': ([_i64, _i64, _i64, _f32, _vp, _i64, _vp, _i64, _int, _f32, _vp, _i64, _vp],
                     _int),
    'lcq_gemm_f32_workspace_bytes': ([_i64, _i64, _i64], _i64),
    'lcq_gemm_f32x6_workspace_bytes': ([_i64, _i64, _i64, _i64, _int], _i64),
    'lcq_gemm_f32x6': ([_i64, _i64, _i64, _f32, _vp, _i64, _int, _vp, _i64, _int, _f32, _vp,
                        _i64, _i64, _i64, _int, _vp, _i64, _vp], _int),
    'lcq_gemm_f32_row_unit': ([_i64, _i64], _i64),
    'lcq_gemm_f32_rows': ([_i64, _i64, _i64, _f32, _vp, _i64, _vp, _i64, _int, _f32, _vp, _i64,
                           _i64, _i64, _vp], _int),
    'lcq_gemm_f32_ws': ([_i64, _i64, _i64, _f32, _vp, _i64, _vp, _i64, _int, _f32, _vp, _i64,
                         _vp, _i64, _vp], _int),
    'lcq_clip_apply': ([_vp, _int, _i64, _i64, _i64, _vp, _vp, _vp, _vp], _int),
    'lcq_clip_factors': ([_vp, _int, _i64, _i64, _i64, _vp, _vp, _int, _vp, _vp, _vp], _int),
    'lcq_absmax': ([_vp, _int, _i64, _vp, _vp, _vp], _int),
    'lcq_fp8_quant': ([_vp, _int, _i64, _i64, _i64, _int, _int, _f32, _f32, _int, _vp, _vp, _vp,
                       _int, _vp, _vp], _int),
    'lcq_fp8_quant_static': ([_vp, _int, _i64, _i64, _i64, _int, _int, _vp, _int, _int, _int,
                              _vp, _vp, _int, _vp], _int),
    'lcq_fp8_quant_blocks': ([_vp, _int, _i64, _i64, _int, _int, _f32, _f32, _int, _vp, _vp,
                              _int, _vp, _vp], _int),
    'lcq_fp8_dequant_blocks': ([_vp, _int, _i64, _i64, _int, _vp, _vp, _int, _vp], _int),
    'lcq_fp8_gemm': ([_vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp, _i64, _vp],
                     _int),
    'lcq_fp8_gemm_workspace_bytes': ([_i64, _i64, _i64], _i64),
    'lcq_fp8_gemm_grouped': ([_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _int, _int, _i64,
                              _i64, _vp, _int, _vp, _i64, _vp], _int),
    'lcq_moe_combine': ([_vp, _vp, _vp, _vp, _int, _i64, _int, _i64, _vp, _vp], _int),
    'lcq_fp8_gemm_grouped_workspace_bytes': ([_i64, _i64, _i64, _i64], _i64),
    'lcq_rotary': ([_vp, _vp, _vp, _vp, _int, _i64, _i64, _int, _int, _int, _i64, _vp, _vp, _vp],
                   _int),
    'lcq_silu_mul': ([_vp, _vp, _int, _i64, _vp, _vp], _int),
    'lcq_rmsnorm': ([_vp, _vp, _int, _i64, _i64, _f32, _vp, _vp], _int),
    'lcq_fp8_block_to_tensor': ([_vp, _int, _i64, _i64, _int, _vp, _int, _f32, _f32, _int, _vp,
                                 _vp, _vp, _vp], _int),
    'lcq_fp8_gemm_force_plan': ([_int], _int),
    'lcq_fp8_block_to_tensor_many': ([_int, _vp, _i64, _int, _int, _int, _f32, _f32, _int, _vp,
                                      _vp, _vp], _int),
    'lcq_minmax_segments': ([_vp, _vp, _i64, _int, _vp, _vp, _vp], _int),
    'lcq_act_static_qparams': ([_vp, _i64, _int, _f32, _int, _int, _int, _f32, _f32, _vp, _vp],
                               _int),
    'lcq_act_hist_workspace_bytes': ([_i64], _i64),
    'lcq_act_static_hist_qparams': ([_vp, _vp, _i64, _int, _vp, _int, _f32, _vp, _vp, _vp], _int),
    'lcq_mse_qparams': ([_vp, _int, _i64, _i64, _int, _int, _int, _int, _f32, _f32, _vp, _vp,
                         _vp, _vp, _vp], _int),
    'lcq_gemm': ([_vp, _int, _i64, _i64, _i64, _int, _vp, _vp, _i64, _vp, _vp, _vp, _vp], _int),
    'lcq_gemm_rope': ([_vp, _int, _i64, _i64, _i64, _int, _vp, _vp, _i64, _vp, _vp, _vp, _int,
                       _vp, _vp, _i64, _i64, _i64, _vp], _int),
    'lcq_gemm_residual': ([_vp, _int, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _vp,
                           _i64, _vp], _int),
    'lcq_gemm_silu_mul': ([_vp, _int, _i64, _i64, _i64, _vp, _vp, _i64, _i64, _vp, _i64, _vp],
                          _int),
    'lcq_gemm_sq_diff_workspace_bytes': ([_i64, _i64], _i64),
    'lcq_gemm_sq_diff': ([_vp, _int, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _vp,
                          _i64, _vp, _int, _vp], _int),
    'lcq_fp_emul_quant': ([_vp, _int, _i64, _i64, _i64, _int, _int, _vp, _int, _vp], _int),
}

_lib = None


class LcqError(RuntimeError):
    pass


def lib_path() -> Path:
    return _LIB_PATH


def header_symbols() -> list[str]:
    """Names of all functions declared in include/lcq.h."""
    text = _HEADER.read_text()
    return sorted(set(re.findall(r'\b(lcq_[a-z0-9_]+)\s*\(', text)))


def load():
    """Load liblcq.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise LcqError(f'{_LIB_PATH} not built: run `python -m lightcompress_amd._build` '
                       '(or __graft_entry__.build()) first; there is no CPU fallback')
    lib = ctypes.CDLL(str(_LIB_PATH), mode=getattr(os, 'RTLD_NOW', 2))
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def dt(t: torch.Tensor | torch.dtype) -> int:
    d = t if isinstance(t, torch.dtype) else t.dtype
    if d not in _DT:
        raise LcqError(f'unsupported dtype {d}')
    return _DT[d]


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise LcqError('lightcompress_amd ops run on the GPU only (no CPU fallback); '
                       f'got a tensor on {t.device}')
    if not t.is_contiguous():
        raise LcqError('tensor must be contiguous')
    return t.data_ptr()


def ptr_strided(t):
    """Device pointer of a possibly strided tensor (the kernel takes its strides)."""
    if not t.is_cuda:
        raise LcqError('lightcompress_amd ops run on the GPU only (no CPU fallback); '
                       f'got a tensor on {t.device}')
    return t.data_ptr()


def stream_of(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


class KernelTimer:
    """Records a device event pair around every lcq call while active (bench.py uses this to
    time each kernel family live, on the stream the kernel is launched on)."""

    def __init__(self):
        self.events = {}
        self.work = {}
        self.bytes = {}

    def __enter__(self):
        global _timer
        _timer = self
        return self

    def __exit__(self, *exc):
        global _timer
        _timer = None

    def summary(self):
        import torch as _t
        _t.cuda.synchronize()
        out = {}
        for name, pairs in self.events.items():
            ms = [a.elapsed_time(b) for a, b in pairs]
            out[name] = {'launches': len(ms), 'total_ms': sum(ms), 'avg_ms': sum(ms) / len(ms)}
            if name in self.work:
                out[name]['flops'] = self.work[name]
            if name in self.bytes:
                out[name]['bytes'] = self.bytes[name]
        return out


_timer = None


def note_work(name: str, units: float):
    """Attribute algorithmic work (flops or bytes) to the last `name` launch while timing."""
    if _timer is not None:
        _timer.work[name] = _timer.work.get(name, 0.0) + float(units)


def note_bytes(name: str, nbytes: float):
    """Attribute algorithmic HBM bytes (operands read once, outputs written once) to the
    last `name` launch while timing."""
    if _timer is not None:
        _timer.bytes[name] = _timer.bytes.get(name, 0.0) + float(nbytes)


def call(name: str, *args):
    lib = load()
    if _timer is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib, name)(*args)
        e1.record()
        _timer.events.setdefault(name, []).append((e0, e1))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.lcq_last_error().decode(errors='replace')
        if rc == -1:
            raise ValueError(msg)
        raise LcqError(f'{name} failed ({rc}): {msg}')
    return rc
