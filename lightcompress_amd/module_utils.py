"""Linear wrappers and real-quant packers (drop-in for llmc ``module_utils``).

Same class names, ``new(...)`` constructors, buffer names and pack layouts as the reference
(module_utils.py:679-1231); packing runs on the device through ``liblcq.so`` instead of the
reference's CPU numpy loop (vLLM) and per-column Python loop (AutoAWQ).
"""
from __future__ import annotations

from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


# Calls of lcq_linear that took torch's F.linear (vendor BLAS) instead of the lcq GEMM, by
# (dtype, K, N): bench.py reports them per leg, and STRICT_LINEAR turns them into errors.
LINEAR_FALLBACKS: dict = {}
STRICT_LINEAR = False


def lcq_linear(x, weight, bias=None):
    """F.linear(x, weight, bias) on the lcq GEMM when the operands fit it (bf16 / fp16 on the
    device, K % 64 == 0, out_features % 16 == 0, bias in the input dtype); other operands
    (fp32 GPTQ weights, odd shapes) take torch's F.linear, counted in LINEAR_FALLBACKS (an
    error under STRICT_LINEAR)."""
    if (ops.gemm_supported(x, weight)
            and (bias is None or (bias.dtype == x.dtype and bias.is_contiguous()))):
        return ops.linear(x, weight, bias)
    key = (str(x.dtype).replace('torch.', ''), str(weight.dtype).replace('torch.', ''),
           int(weight.shape[-1]), int(weight.shape[0]))
    if STRICT_LINEAR:
        raise ops.N.LcqError(f'lcq_linear: operands {key} do not fit the lcq GEMM '
                             '(STRICT_LINEAR forbids the F.linear fallback)')
    LINEAR_FALLBACKS[key] = LINEAR_FALLBACKS.get(key, 0) + 1
    return F.linear(x, weight, bias)


def _fname(fn):
    if fn is None:
        return 'None'
    return fn.func.__name__ if isinstance(fn, partial) else getattr(fn, '__name__', str(fn))


# The reference switches between its Triton fp8_gemm and a bf16 round trip on
# USE_FP8GEMM_TRITON_KERNEL (module_utils.py:14-22); here the HIP fp8 GEMM is always present.
USE_FP8GEMM_TRITON_KERNEL = True


def block_wise_fp8_forward_func(x, w, w_scale, block_size, bias):
    """module_utils.py:41-46: act_quant of x (1x128 groups), block-scaled fp8 GEMM, bf16."""
    from .kernel import act_quant, fp8_gemm
    x, scale = act_quant(x.contiguous(), block_size)
    y = fp8_gemm(x, scale, w, w_scale).to(torch.bfloat16)
    if bias is not None:
        y += bias
    return y


class LlmcFp8Linear(nn.Module):
    """module_utils.py:223-285: a DeepSeek-V3-style block-fp8 linear (e4m3 weight, 128x128
    ``weight_scale_inv``) whose forward runs on the fp8 MFMA without a bf16 weight copy."""

    def __init__(self, in_features, out_features, bias, block_size):
        super().__init__()
        self.block_size = block_size
        self.in_features = in_features
        self.out_features = out_features
        if bias:
            self.bias = nn.Parameter(torch.empty(out_features))
        else:
            self.register_parameter('bias', None)
        self.weight = nn.Parameter(
            torch.empty(out_features, in_features, dtype=torch.float8_e4m3fn),
            requires_grad=False)
        so = (out_features + block_size - 1) // block_size
        si = (in_features + block_size - 1) // block_size
        self.weight_scale_inv = nn.Parameter(torch.empty(so, si, dtype=torch.float32),
                                             requires_grad=False)

    def forward(self, x):
        if self.weight.data.dtype == torch.float8_e4m3fn:
            if USE_FP8GEMM_TRITON_KERNEL:
                return block_wise_fp8_forward_func(x, self.weight, self.weight_scale_inv,
                                                   self.block_size, self.bias)
            from .kernel import weight_cast_to_bf16
            self.weight.data = weight_cast_to_bf16(self.weight.data, self.weight_scale_inv.data,
                                                   self.block_size).to(torch.bfloat16)
        return lcq_linear(x, self.weight, self.bias)

    @classmethod
    @torch.no_grad()
    def new(cls, module, block_size):
        return cls(module.in_features, module.out_features, module.bias is not None,
                   block_size)

    def __repr__(self):
        return (f'LlmcFp8Linear(in_features={self.in_features}, '
                f'out_features={self.out_features}, bias={self.bias is not None}, '
                f'weight_shape={self.weight.shape}, weight_dtype={self.weight.dtype}, '
                f'block_size={self.block_size}, '
                f'use_fp8gemm_triton_kernel={USE_FP8GEMM_TRITON_KERNEL})')


class FakeQuantLinear(nn.Module):
    """module_utils.py:679-771 — weight fake-quantised lazily on first forward (w_qdq)."""

    def __init__(self, weight, bias, ori_module, w_qdq, a_qdq):
        super().__init__()
        self.register_buffer('weight', weight)
        if bias is not None:
            self.register_buffer('bias', bias)
        else:
            self.bias = None
        self.a_qdq, self.w_qdq = a_qdq, w_qdq
        for name, buf in list(ori_module.named_buffers()) + list(ori_module.named_parameters()):
            if name.startswith('buf_'):
                self.register_buffer(name, buf.data)
        self.buf_rotate = False
        self.dynamic_quant_weight = False
        self.dynamic_quant_tmp_weight = False

    def forward(self, x):
        if self.a_qdq is not None:
            x = self.a_qdq(x, self)
        if not hasattr(self, 'tmp_weight'):
            self.register_buffer('tmp_weight', self.w_qdq(self), persistent=False)
            self.tmp_bias = self.bias
        elif self.dynamic_quant_weight:
            self.tmp_weight = self.w_qdq(self)
            self.tmp_bias = self.bias
        elif self.dynamic_quant_tmp_weight:
            self.tmp_weight = self.w_qdq(self)
        return lcq_linear(x, self.tmp_weight, self.tmp_bias)

    def _lcq_after_move(self):
        """The block was moved between HBM and the host (residency.BlockStreamer): tmp_bias is
        a plain alias of the bias buffer set by the memoising forward, re-pointed at the
        buffer's new home so it never pins the old copy."""
        if 'tmp_bias' in self.__dict__:
            self.tmp_bias = self.bias

    @classmethod
    @torch.no_grad()
    def new(cls, module, w_qdq, a_qdq):
        bias = module.bias.data if getattr(module, 'bias', None) is not None else None
        m = cls(module.weight.data, bias, ori_module=module, w_qdq=w_qdq, a_qdq=a_qdq)
        m.in_features, m.out_features = module.in_features, module.out_features
        m.w_qdq_name, m.a_qdq_name = _fname(w_qdq), _fname(a_qdq)
        return m

    def __repr__(self):
        return (f'FakeQuantLinear(in_features={self.in_features},out_features={self.out_features},'
                f' bias={self.bias is not None},weight_quant={self.w_qdq_name},'
                f'act_quant={self.a_qdq_name})')


class EffcientFakeQuantLinear(nn.Module):
    """module_utils.py:774-852 — weight fake-quantised once at construction (deploy)."""

    def __init__(self, weight, bias, ori_module, a_qdq):
        super().__init__()
        self.register_buffer('weight', weight)
        if bias is not None:
            self.register_buffer('bias', bias)
        else:
            self.bias = None
        self.a_qdq = a_qdq
        for name, buf in ori_module.named_buffers():
            if name.startswith('buf_'):
                self.register_buffer(name, buf.data)
        self.buf_rotate = False

    @torch.no_grad()
    def forward(self, x):
        if self.a_qdq is not None:
            x = self.a_qdq(x, self)
        return lcq_linear(x, self.weight, self.bias)

    @classmethod
    @torch.no_grad()
    def new(cls, module, w_qdq, a_qdq, debug_print={}):
        weight = w_qdq(module)
        bias = module.bias.data if module.bias is not None else None
        m = cls(weight, bias, ori_module=module, a_qdq=a_qdq)
        m.in_features, m.out_features = module.in_features, module.out_features
        m.w_qdq_name, m.a_qdq_name = _fname(w_qdq), _fname(a_qdq)
        m.debug_print = debug_print
        return m


class OriginFloatLinear(nn.Module):
    """module_utils.py OriginFloatLinear: keeps the float (transformed) weight."""

    def __init__(self, weight, bias, ori_module):
        super().__init__()
        self.register_buffer('weight', weight)
        if bias is not None:
            self.register_buffer('bias', bias)
        else:
            self.bias = None
        for name, buf in ori_module.named_buffers():
            if name.startswith('buf_'):
                self.register_buffer(name, buf.data)

    @torch.no_grad()
    def forward(self, x):
        return lcq_linear(x, self.weight, self.bias)

    @classmethod
    @torch.no_grad()
    def new(cls, module):
        bias = module.bias.data if module.bias is not None else None
        m = cls(module.weight.data, bias, module)
        m.in_features, m.out_features = module.in_features, module.out_features
        return m


_SHELL_PROTO = nn.Module()
_SHELL_PLAIN = {k: v for k, v in _SHELL_PROTO.__dict__.items() if not isinstance(v, (dict, set))}
_SHELL_CONT = [(k, v) for k, v in _SHELL_PROTO.__dict__.items() if isinstance(v, (dict, set))]


def _module_shell(cls, buffers: dict, attrs: dict):
    """An instance of nn.Module subclass `cls` with exactly the state its __init__ +
    register_buffer calls would give (fresh hook / child containers, `buffers` registered
    persistent, `attrs` as plain attributes), built without nn.Module.__setattr__'s per-call
    bookkeeping: a deploy builds hundreds of these per MoE block (new_batch)."""
    m = object.__new__(cls)
    d = m.__dict__
    d.update(_SHELL_PLAIN)
    for k, v in _SHELL_CONT:
        d[k] = v.copy()
    d['_buffers'].update(buffers)
    d.update(attrs)
    return m


class VllmRealQuantLinear(nn.Module):
    """module_utils.py:855-955 — vLLM compressed-tensors int layout."""

    def __init__(self, weight, bias, scales, input_scale, need_pack, scales_name):
        super().__init__()
        self.register_buffer('weight_packed' if need_pack else 'weight', weight)
        if bias is not None:
            self.register_buffer('bias', bias)
        else:
            self.bias = None
        self.register_buffer(scales_name, scales)
        self.register_buffer('input_scale', input_scale)

    @torch.no_grad()
    def forward(self, x):
        raise NotImplementedError

    @classmethod
    @torch.no_grad()
    def new(cls, module, w_q, quant_config):
        weight, scales = cls.quant_pack(module, w_q, quant_config)
        input_scale = getattr(module, 'buf_act_scales_0', None)
        bias = module.bias.data if module.bias is not None else None
        need_pack = quant_config['weight'].get('need_pack', False)
        scales_name = ('weight_scale_inv' if quant_config['weight']['granularity'] == 'per_block'
                       else 'weight_scale')
        m = cls(weight, bias, scales, input_scale, need_pack, scales_name)
        m.in_features, m.out_features = module.in_features, module.out_features
        m.weight_shape, m.weight_dtype = weight.shape, weight.dtype
        m.scales_shape, m.scales_dtype = scales.shape, scales.dtype
        m.zeros_shape = m.zeros_dtype = None
        return m

    @classmethod
    @torch.no_grad()
    def new_batch(cls, modules, w_q, quant_config, prequant=None):
        """new() for every module of a list (a block's linears), the same modules and buffers:
        codes / scales from `prequant` (one batched requant launch pair per block,
        BaseBlockwiseQuantization._prequant_fp8_block) where given, quant_pack otherwise; the
        module objects built as shells (_module_shell) -- for a DeepSeek-V3 MoE block the
        per-linear Python of new() (nn.Module construction, register_buffer and __setattr__
        bookkeeping) cost ~10x the deploy kernels."""
        need_pack = quant_config['weight'].get('need_pack', False)
        scales_name = ('weight_scale_inv' if quant_config['weight']['granularity'] == 'per_block'
                       else 'weight_scale')
        wname = 'weight_packed' if need_pack else 'weight'
        out = []
        for i, module in enumerate(modules):
            pre = prequant[i] if prequant is not None else None
            weight, scales = pre if pre is not None else cls.quant_pack(module, w_q, quant_config)
            b = module.__dict__['_parameters'].get('bias', module.__dict__['_buffers'].get('bias'))
            bufs = {wname: weight}
            attrs = {}
            if b is not None:
                bufs['bias'] = b.data
            else:
                attrs['bias'] = None
            bufs[scales_name] = scales
            bufs['input_scale'] = module.__dict__['_buffers'].get('buf_act_scales_0')
            attrs.update(in_features=module.in_features, out_features=module.out_features,
                         weight_shape=weight.shape, weight_dtype=weight.dtype,
                         scales_shape=scales.shape, scales_dtype=scales.dtype,
                         zeros_shape=None, zeros_dtype=None)
            out.append(_module_shell(cls, bufs, attrs))
        return out

    @classmethod
    @torch.no_grad()
    def quant_pack(cls, module, w_q, quant_config):
        wq = getattr(w_q, 'keywords', {}).get('wquantizer')
        if (module.weight.data.dtype == torch.float8_e4m3fn and wq is not None
                and hasattr(wq, 'real_quant_weight_from_block_fp8')
                and not quant_config['weight'].get('need_pack', False)):
            # fp8 checkpoint -> per-tensor fp8 without materialising the bf16 weight
            weight, scales, _ = wq.real_quant_weight_from_block_fp8(
                module.weight.data, module.weight_scale_inv.data, module.block_size)
            return weight, scales
        if module.weight.data.dtype == torch.float8_e4m3fn:  # module_utils.py:917-922
            from .kernel import weight_cast_to_bf16
            module.weight.data = weight_cast_to_bf16(
                module.weight.data, module.weight_scale_inv.data,
                module.block_size).to(torch.bfloat16)
        weight, scales, zeros = w_q(module)
        if quant_config['weight'].get('need_pack', False):
            weight, scales = cls.pack(weight, scales, quant_config)
        return weight, scales

    @classmethod
    @torch.no_grad()
    def pack(cls, weight, scales, quant_config):
        """Device pack: int32 [rows, ceil(cols*b/32)], scales -> fp16 (module_utils.py:929-955)."""
        bits = quant_config['weight']['bit']
        return ops.pack_vllm(weight.contiguous(), bits), scales.to(torch.float16)


class SglRealQuantLinear(VllmRealQuantLinear):
    pass


class LightllmRealQuantLinear(VllmRealQuantLinear):
    pass


class Lightx2vRealQuantLinear(VllmRealQuantLinear):
    pass


class AutoawqRealQuantLinear(nn.Module):
    """module_utils.py:1025-1158 — AutoAWQ GEMM layout (qweight [IC, OC/8])."""

    def __init__(self, weight, bias, scales, zeros):
        super().__init__()
        self.register_buffer('qweight', weight)
        if bias is not None:
            self.register_buffer('bias', bias)
        else:
            self.bias = None
        self.register_buffer('scales', scales)
        if zeros is not None:
            self.register_buffer('qzeros', zeros)
        else:
            self.qzeros = None

    @torch.no_grad()
    def forward(self, x):
        raise NotImplementedError

    @classmethod
    @torch.no_grad()
    def new(cls, module, w_q, quant_config):
        weight, scales, zeros = cls.quant_pack(module, w_q, quant_config)
        bias = module.bias.data if module.bias is not None else None
        m = cls(weight, bias, scales, zeros)
        m.in_features, m.out_features = module.in_features, module.out_features
        m.weight_shape, m.weight_dtype = weight.shape, weight.dtype
        m.scales_shape, m.scales_dtype = scales.shape, scales.dtype
        m.zeros_shape = zeros.shape if zeros is not None else None
        m.zeros_dtype = zeros.dtype if zeros is not None else None
        return m

    @classmethod
    @torch.no_grad()
    def quant_pack(cls, module, w_q, quant_config):
        if module.weight.data.dtype == torch.float8_e4m3fn:  # module_utils.py:1079-1085
            from .kernel import weight_cast_to_bf16
            module.weight.data = weight_cast_to_bf16(
                module.weight.data, module.weight_scale_inv.data,
                module.block_size).to(torch.bfloat16)
        _, scales, zeros = w_q(module)
        if quant_config['weight']['pack_version'] != 'gemm_pack':
            raise NotImplementedError(f"Not support {quant_config['weight']['pack_version']}.")
        return cls.gemm_pack(module, module.weight.data, scales, zeros, quant_config)

    @classmethod
    @torch.no_grad()
    def gemm_pack(cls, module, weight, scales, zeros, quant_config):
        assert scales is not None and zeros is not None
        bit = quant_config['weight']['bit']
        if bit != 4:
            raise NotImplementedError('Only 4-bit are supported for now.')
        return ops.pack_autoawq_gemm(weight.contiguous(), scales, zeros,
                                     quant_config['weight']['group_size'], bit)


class MlcllmRealQuantLinear(AutoawqRealQuantLinear):
    pass


_REALQUANT_LINEAR_MAP_ = {
    'vllm_quant': VllmRealQuantLinear,
    'lightllm_quant': LightllmRealQuantLinear,
    'sgl_quant': SglRealQuantLinear,
    'autoawq_quant': AutoawqRealQuantLinear,
    'mlcllm_quant': MlcllmRealQuantLinear,
    'lightx2v_quant': Lightx2vRealQuantLinear,
}

_LLMC_LINEAR_TYPES_ = [LlmcFp8Linear, OriginFloatLinear, FakeQuantLinear,
                       EffcientFakeQuantLinear, VllmRealQuantLinear, SglRealQuantLinear,
                       AutoawqRealQuantLinear, MlcllmRealQuantLinear, LightllmRealQuantLinear,
                       Lightx2vRealQuantLinear]
_TRANSFORMERS_LINEAR_TYPES_ = [nn.Linear]
