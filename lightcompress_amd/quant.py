"""Quantizer plugin API (drop-in for ``llmc.compression.quantization.quant``).

``IntegerQuantizer`` / ``FloatQuantizer`` keep the reference constructor, attribute names and
method signatures (quant.py:46-1229) so the reference's algorithms and YAML configs use them
unchanged; the arithmetic runs in the HIP kernels of ``liblcq.so`` (see ``ops.py``), which
reproduce the reference's per-op dtype rounding bit for bit. There is no CPU path: tensors must
live on the GPU.

Supported on the device path (the hot path of SURVEY.md §8a): calib_algo ``minmax``,
granularity per_group / per_channel / per_token / per_tensor / per_head, round_zp=True,
bit 2..8, dynamic and static qparams, fake quant, real quant (+ vLLM / AutoAWQ packing in
``module_utils``). Not yet supported (raise NotImplementedError): mse / hqq / learnable / static
histogram calibration, ``int_indices`` mixed precision, STE rounding, ``rounding`` overrides.
"""
from __future__ import annotations

import torch

from . import ops

__all__ = ['BaseQuantizer', 'IntegerQuantizer', 'FloatQuantizer']


class BaseQuantizer:
    """Mirrors BaseQuantizer.__init__ (quant.py:46-101): same attributes and kwargs."""

    def __init__(self, bit, symmetric, granularity, **kwargs):
        self.bit = bit
        self.sym = symmetric
        self.granularity = granularity
        self.kwargs = kwargs
        self.calib_algo = kwargs.get('calib_algo', 'minmax')
        if granularity == 'per_group':
            self.group_size = kwargs['group_size']
        elif granularity == 'per_head':
            self.head_num = kwargs['head_num']
        elif granularity == 'per_block':
            assert self.calib_algo == 'minmax' and self.sym
            self.block_size = kwargs['block_size']
        self.round_zp = kwargs.get('round_zp', True)
        self.ste = kwargs.get('ste', False)
        self.ste_all = kwargs.get('ste_all', False)
        self.round_func = torch.round
        self.mse_b_num = kwargs.get('mse_b_num', 1)
        self.maxshrink = kwargs.get('maxshrink', 0.8)
        self.mse_grid = kwargs.get('mse_grid', 100)

    # -- layout helpers (quant.py:612-658) --------------------------------------------------
    def reshape_tensor(self, tensor, allow_padding=False):
        if self.granularity == 'per_group':
            if tensor.shape[-1] >= self.group_size:
                if tensor.shape[-1] % self.group_size == 0:
                    return tensor.reshape(-1, self.group_size)
                if allow_padding:
                    pad = self.group_size - tensor.shape[-1] % self.group_size
                    z = torch.zeros((*tensor.shape[:-1], pad), device=tensor.device,
                                    dtype=tensor.dtype)
                    return torch.cat((tensor, z), dim=-1).reshape(-1, self.group_size)
                raise ValueError(f'Dimension {tensor.shape[-1]} '
                                 f'not divisible by group size {self.group_size}')
            return tensor
        if self.granularity == 'per_head':
            return tensor.reshape(self.head_num, -1)
        return tensor

    def restore_tensor(self, tensor, shape):
        if tensor.shape == shape:
            return tensor
        try:
            return tensor.reshape(shape)
        except RuntimeError:
            pad = self.group_size - shape[1] % self.group_size
            return tensor.reshape(*shape[:-1], -1)[..., :-pad]

    def _kernel_view(self, tensor):
        """2-D [rows, cols] view + group length the grouped kernel reduces over."""
        g = self.granularity
        if g == 'per_group':
            if tensor.shape[-1] >= self.group_size:
                if tensor.shape[-1] % self.group_size:
                    raise ValueError(f'Dimension {tensor.shape[-1]} '
                                     f'not divisible by group size {self.group_size}')
                return tensor.reshape(-1, tensor.shape[-1]), self.group_size
            return tensor.reshape(-1, tensor.shape[-1]), tensor.shape[-1]
        if g in ('per_channel', 'per_token'):
            return tensor.reshape(-1, tensor.shape[-1]), tensor.shape[-1]
        if g == 'per_tensor':
            return tensor.reshape(1, -1), tensor.numel()
        if g == 'per_head':
            t = tensor.reshape(self.head_num, -1)
            return t, t.shape[1]
        raise NotImplementedError(f'granularity {g} is not on the device path yet')

    def _check_supported(self, args):
        if self.calib_algo not in ('minmax',):
            raise NotImplementedError(f'calib_algo={self.calib_algo} is not on the device path')
        if not self.round_zp:
            raise NotImplementedError('round_zp=False is not on the device path')
        for k in ('int_indices', 'rounding'):
            if k in args:
                raise NotImplementedError(f'args[{k!r}] is not on the device path')
        if args.get('lowbound_factor') is not None or args.get('upbound_factor') is not None:
            raise NotImplementedError('learnable clip factors (clip v2) are not on the device path')

    # -- API helpers kept for signature parity (quant.py:132-143, 545-559) -----------------
    def get_minmax_range(self, tensor):
        if self.granularity == 'per_tensor':
            return torch.min(tensor), torch.max(tensor)
        return tensor.amin(dim=-1, keepdim=True), tensor.amax(dim=-1, keepdim=True)

    def get_tensor_range(self, tensor, args={}):
        return self.get_minmax_range(tensor)


class IntegerQuantizer(BaseQuantizer):
    """IntegerQuantizer (quant.py:661-960) on the lcq kernels."""

    def __init__(self, bit, symmetric, granularity, **kwargs):
        super().__init__(bit, symmetric, granularity, **kwargs)
        self.quant_type = 'int-quant'
        if 'int_range' in kwargs:
            qmin, qmax = kwargs['int_range']
        elif self.sym:
            qmin, qmax = -(2 ** (bit - 1)), 2 ** (bit - 1) - 1
        else:
            qmin, qmax = 0.0, 2 ** bit - 1
        self.qmin = torch.tensor(qmin)
        self.qmax = torch.tensor(qmax)
        self.dst_nbins = 2 ** bit

    @property
    def _iq(self):
        return int(self.qmin.item()), int(self.qmax.item())

    def get_qparams(self, tensor_range, device):
        """quant.py:545-559 (tiny tensors; kept for API parity)."""
        mn, mx = tensor_range
        qmin, qmax = self.qmin.to(device), self.qmax.to(device)
        if self.sym:
            am = torch.max(mx.abs(), mn.abs()).clamp(min=1e-5)
            return am / qmax, torch.tensor(0.0), qmax, qmin
        s = (mx - mn).clamp(min=1e-5) / (qmax - qmin)
        z = (qmin - torch.round(mn / s)).clamp(qmin, qmax)
        return s, z, qmax, qmin

    def get_tensor_qparams(self, tensor, args={}):
        """quant.py:690-697: (reshaped tensor, scales, zeros, qmax, qmin)."""
        self._check_supported(args)
        x2, group = self._kernel_view(tensor.contiguous())
        qmin, qmax = self._iq
        r = ops.int_quant_dynamic(x2, group, qmin, qmax, self.sym, fq=False)
        dev = tensor.device
        zeros = r['zeros'] if not self.sym else torch.tensor(0.0)
        scales = r['scales']
        if self.granularity == 'per_tensor':
            scales = scales.reshape(())
            zeros = zeros.reshape(()) if not self.sym else zeros
        return (self.reshape_tensor(tensor), scales, zeros, self.qmax.to(dev), self.qmin.to(dev))

    # -- elementwise ops with given qparams (quant.py:699-717) ------------------------------
    def _static(self, tensor, scales, zeros, want):
        t2 = tensor.reshape(-1, tensor.shape[-1]).contiguous()
        s = scales.contiguous()
        ng = s.numel()
        if t2.numel() % ng:
            raise ValueError('scales do not tile the tensor')
        group = t2.numel() // ng
        if group != t2.shape[1] and t2.shape[1] % group:
            raise ValueError('unsupported scales layout')
        zz = None
        if torch.is_tensor(zeros) and zeros.dim() > 0:
            zz = zeros.contiguous()
        elif torch.is_tensor(zeros) and zeros.item() != 0 or (not torch.is_tensor(zeros) and zeros):
            zz = torch.full_like(s, float(zeros), dtype=s.dtype)
        ct = tensor.dtype if s.dim() == 0 else torch.promote_types(tensor.dtype, s.dtype)
        if zz is not None and zz.is_floating_point():
            ct = torch.promote_types(ct, zz.dtype)
        qmin, qmax = self._iq
        if want == 'codes':
            r = ops.int_quant_static(t2, group, s, zz, qmin, qmax, ct_dtype=ct, fq=False,
                                     codes_dtype=torch.int32)
            return r['codes'].to(ct).reshape(tensor.shape)
        r = ops.int_quant_static(t2, group, s, zz, qmin, qmax, ct_dtype=ct, fq=True)
        return r['fq'].reshape(tensor.shape)

    def quant(self, tensor, scales, zeros, qmax, qmin):
        return self._static(tensor, scales, zeros, 'codes')

    def dequant(self, tensor, scales, zeros):
        return (tensor - zeros) * scales  # quant.py:710-712 (single fused-free expression)

    def quant_dequant(self, tensor, scales, zeros, qmax, qmin, output_scale_factor=1):
        if output_scale_factor != 1:
            raise NotImplementedError('output_scale_factor != 1 on the device path')
        return self._static(tensor, scales, zeros, 'fq')

    # -- weights -------------------------------------------------------------------------------
    def _maybe_t(self, weight, args):
        return ('dim' in args and 'ic' in args['dim'])

    def fake_quant_weight_dynamic(self, weight, args={}):
        """quant.py:833-869."""
        self._check_supported(args)
        tr = self._maybe_t(weight, args)
        w = weight.T if tr else weight
        shape = w.shape
        x2, group = self._kernel_view(w.contiguous())
        qmin, qmax = self._iq
        fq = ops.int_quant_dynamic(x2, group, qmin, qmax, self.sym, qparams=False)['fq']
        fq = fq.reshape(shape)
        return fq.T if tr else fq

    def fake_quant_weight_static(self, weight, args):
        """quant.py:785-831."""
        self._check_supported(args)
        if args.get('output_scale_factor', 1) != 1:
            raise NotImplementedError('output_scale_factor != 1 on the device path')
        tr = self._maybe_t(weight, args)
        w = weight.T if tr else weight
        zeros = args['zeros'] if args.get('zeros') is not None else torch.tensor(0.0)
        out = self._static(w, args['scales'], zeros, 'fq').to(w.dtype)
        return out.T if tr else out

    def _codes_dtype(self):
        return ops.code_dtype(self.bit, int(self.qmin.item()))

    def real_quant_weight_dynamic(self, weight, args={}):
        """quant.py:916-953: (codes, scales [rows, -1], zeros [rows, -1] | None)."""
        self._check_supported({k: v for k, v in args.items() if k != 'output_scale_factor'})
        osf = args.pop('output_scale_factor', 1) if 'output_scale_factor' in args else 1
        x2, group = self._kernel_view(weight.contiguous())
        qmin, qmax = self._iq
        cd = self._codes_dtype()
        r = ops.int_quant_dynamic(x2, group, qmin, qmax, self.sym, fq=False, codes_dtype=cd)
        codes = r['codes'].reshape(weight.shape)
        scales = r['scales'] * osf if osf != 1 else r['scales']
        zeros = r['zeros'].to(cd) if not self.sym else None
        qshape = 1 if self.granularity == 'per_tensor' else (codes.shape[0], -1)
        if zeros is not None:
            zeros = zeros.view(qshape)
        return codes, scales.view(qshape), zeros

    def real_quant_weight_static(self, weight, args):
        """quant.py:871-914."""
        osf = args.pop('output_scale_factor', 1) if 'output_scale_factor' in args else 1
        zeros = args['zeros'] if args.get('zeros') is not None else torch.tensor(0.0)
        scales = args['scales']
        codes = self._static(weight, scales, zeros, 'codes')
        if osf != 1:
            scales = scales * osf
        cd = self._codes_dtype()
        codes = codes.to(cd)
        if not self.sym and self.round_zp:
            zeros = zeros.to(cd)
        elif self.sym:
            zeros = None
        qshape = 1 if self.granularity == 'per_tensor' else (codes.shape[0], -1)
        if zeros is not None:
            zeros = zeros.view(qshape)
        return codes, scales.view(qshape), zeros

    # -- activations (quant.py:719-783) ---------------------------------------------------------
    def fake_quant_act_dynamic(self, act, args={}):
        self._check_supported(args)
        x2, group = self._kernel_view(act.contiguous())
        qmin, qmax = self._iq
        fq = ops.int_quant_dynamic(x2, group, qmin, qmax, self.sym, qparams=False)['fq']
        return fq.reshape(act.shape)

    def fake_quant_act_static(self, act, args={}):
        self._check_supported(args)
        zeros = args['zeros'] if args.get('zeros') is not None else torch.tensor(0.0)
        return self._static(act, args['scales'], zeros, 'fq').to(act.dtype)

    def __repr__(self):
        return (f'IntegerQuantizer(bit={self.bit}, sym={self.sym},granularity={self.granularity},'
                f'kwargs={self.kwargs}, qmin={self.qmin}, qmax={self.qmax})')


class FloatQuantizer(BaseQuantizer):
    """FloatQuantizer (quant.py:963-1229). Device path: FP8 e4m3 with native OCP cast
    (``use_qtorch`` semantics; qtorch itself is absent, so that path is parity-unpinned)."""

    def __init__(self, bit, symmetric, granularity, **kwargs):
        super().__init__(bit, symmetric, granularity, **kwargs)
        self.sym = True
        self.quant_type = 'float-quant'
        self.e_bits = int(bit[1])
        self.m_bits = int(bit[-1])
        self.num_bits = self.e_bits + self.m_bits + 1
        self.use_qtorch = kwargs.get('use_qtorch')

    def __repr__(self):
        return (f'FloatQuantizer(bit={self.bit},e_bits={self.e_bits}, m_bits={self.m_bits},'
                f'granularity={self.granularity},kwargs={self.kwargs})')
