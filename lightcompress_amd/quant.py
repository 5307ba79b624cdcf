"""Quantizer plugin API (drop-in for ``llmc.compression.quantization.quant``).

``IntegerQuantizer`` / ``FloatQuantizer`` keep the reference constructor, attribute names and
method signatures (quant.py:46-1229) so the reference's algorithms and YAML configs use them
unchanged; the arithmetic runs in the HIP kernels of ``liblcq.so`` (see ``ops.py``), which
reproduce the reference's per-op dtype rounding bit for bit. There is no CPU path: tensors must
live on the GPU.

Supported on the device path (the hot path of SURVEY.md §8a): calib_algo ``minmax``,
granularity per_group / per_channel / per_token / per_tensor / per_head (+ per_block for FP8),
round_zp=True, bit 2..8, dynamic and static qparams, fake quant, real quant (+ vLLM / AutoAWQ
packing in ``module_utils``); FP8 e4m3 / e5m2 (``FloatQuantizer``); static per-tensor activation
calibration (static_minmax / static_moving_minmax / static_hist). Not yet supported (raise
NotImplementedError): ``int_indices`` mixed precision, STE rounding, ``rounding`` overrides.
calib_algo mse and hqq (the proximal search, ``lcq_hqq_proximal``), round_zp False and
learnable (min/max without clip factors; with the v2 clip factors of AutoClipper the range of
get_learnable_range, ``lcq_int_quant_learnable``) run on the device.
"""
from __future__ import annotations

import torch

from . import ops

__all__ = ['BaseQuantizer', 'IntegerQuantizer', 'FloatQuantizer', 'weight_cast_to_bf16',
           'weight_cast_to_fp8']


def weight_cast_to_bf16(weight, scale, block_size):
    """quant.py:18-31: dequant(weight.float(), scale) per block, then bf16."""
    return ops.fp8_dequant_blocks(weight.contiguous(), scale, block_size,
                                  out_dtype=torch.bfloat16)


def weight_cast_to_fp8(weight, block_size):
    """quant.py:34-43: per_block FloatQuantizer real quant (clamp 1e-5, ``+ zeros``)."""
    if block_size != 128:
        raise NotImplementedError('block-fp8 supports block_size 128')
    r = ops.fp8_quant_blocks(weight, torch.float8_e4m3fn, 128, qmax=448.0, clamp_min=1e-5,
                             add_zero=True)
    return r['codes'], r['scales']


# get_tensor_range (quant.py:122-130) falls back to min/max for the static_* algorithms, which
# only change get_batch_tensors_qparams, and learnable is min/max until clip factors are given
_MINMAX_LIKE = ('minmax', 'static_minmax', 'static_moving_minmax', 'static_hist', 'learnable')


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
        # hqq config (quant.py:87-101)
        self.lp_norm = kwargs.get('lp_norm', 0.7)
        self.beta = kwargs.get('beta', 10)
        self.kappa = kwargs.get('kappa', 1.01)
        self.iters = kwargs.get('iters', 20)

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
        if self.granularity == 'per_block':  # quant.py:636-641 (zero pad to block multiples)
            m, n = tensor.shape
            b = self.block_size
            pm, pn = -(-m // b) * b, -(-n // b) * b
            t = torch.zeros((pm, pn), dtype=tensor.dtype, device=tensor.device)
            t[:m, :n] = tensor
            return t.view(-1, b, pn // b, b)
        return tensor

    def restore_tensor(self, tensor, shape):
        if tensor.shape == shape:
            return tensor
        if self.granularity == 'per_block':  # quant.py:648-652
            try:
                return tensor.reshape(-1, shape[-1])[:shape[0], :]
            except RuntimeError:
                return tensor.reshape(shape[0], -1)[:, :shape[1]]
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
        if self.calib_algo not in _MINMAX_LIKE + ('mse', 'hqq'):
            raise NotImplementedError(f'calib_algo={self.calib_algo} is not on the device path')
        if not self.round_zp and self.calib_algo == 'mse':
            raise NotImplementedError('round_zp=False with mse is not on the device path')
        for k in ('int_indices', 'rounding'):
            if k in args:
                raise NotImplementedError(f'args[{k!r}] is not on the device path')
        if self._factors(args) is not None and (
                getattr(self, 'quant_type', 'int-quant') != 'int-quant' or not self.round_zp):
            raise NotImplementedError('learnable clip factors: integer quantizers, round_zp')

    def _factors(self, args):
        """(up, low | None): the clip factors get_learnable_range applies (quant.py:127-128,
        205-219), or None. Only calib_algo learnable reads them; sym needs the upper factor,
        asym both (one missing leaves the min/max range)."""
        if self.calib_algo != 'learnable' or not args:
            return None
        up, low = args.get('upbound_factor'), args.get('lowbound_factor')
        if up is None or (not self.sym and low is None):
            return None
        return up, (None if self.sym else low)

    # -- API helpers kept for signature parity (quant.py:132-143, 545-559) -----------------
    def get_minmax_range(self, tensor):
        if self.granularity == 'per_tensor':
            return torch.min(tensor), torch.max(tensor)
        return tensor.amin(dim=-1, keepdim=True), tensor.amax(dim=-1, keepdim=True)

    def get_tensor_range(self, tensor, args={}):
        if self.calib_algo == 'mse':
            return self.get_mse_range(tensor)
        if self.calib_algo == 'learnable':
            return self.get_learnable_range(tensor, **args)
        return self.get_minmax_range(tensor)

    def get_learnable_range(self, tensor, lowbound_factor=None, upbound_factor=None):
        """quant.py:205-219 (tiny tensors; kept for API parity -- the fake quant fuses it in
        lcq_int_quant_learnable)."""
        mn, mx = self.get_minmax_range(tensor)
        if self.sym:
            if upbound_factor is not None:
                am = torch.max(mx.abs(), mn.abs()).clamp(min=1e-5)
                am = torch.sigmoid(upbound_factor) * am
                mn, mx = -am, am
        elif upbound_factor is not None and lowbound_factor is not None:
            mn = torch.sigmoid(lowbound_factor) * mn
            mx = torch.sigmoid(upbound_factor) * mx
        return mn, mx

    def _mse_nsteps(self):
        return int(self.maxshrink * self.mse_grid)

    def get_mse_range(self, tensor, norm=2.4, bs=256):
        """quant.py:145-203 on the device (``lcq_mse_qparams``): tensor is the reshaped
        [groups, group] view; returns fp32 (min, max) [groups, 1]."""
        assert self.mse_b_num >= 1 and tensor.shape[0] % self.mse_b_num == 0, \
            'Batch number must be divisible by tensor.shape[0],'
        t = tensor.reshape(tensor.shape[0], -1)
        qmin, qmax = self._iq
        mn, mx, _, _ = ops.mse_qparams(t, t.shape[1], self.sym, qmin, qmax, self._mse_nsteps(),
                                       float(self.mse_grid), norm)
        return mn.view(-1, 1), mx.view(-1, 1)

    # -- static activation calibration (quant.py:103-120, 221-262, 431-450, 561-586) --------
    def reshape_batch_tensors(self, act_tensors):
        """quant.py:103-120 without mutating the caller's list: one list of calibration
        segments per module input (a single entry = one batch of samples, split per sample)."""
        assert len(act_tensors) > 0, (
            'Calibration data is insufficient. Please provide more data to ensure '
            'all experts in the MOE receive an adequate number of tokens.')
        if isinstance(act_tensors[0], tuple):
            return [list(torch.stack(ts)) for ts in zip(*act_tensors)]
        if len(act_tensors) == 1:
            return [[act_tensors[0][i] for i in range(act_tensors[0].size(0))]]
        return [list(act_tensors)]

    def _static_scale_dtype(self, range_dtype):
        qd = self.qmax.dtype if self.sym else torch.promote_types(self.qmax.dtype,
                                                                  self.qmin.dtype)
        if not qd.is_floating_point:
            return range_dtype  # 0-dim float op 0-dim int -> the float dtype
        return torch.promote_types(range_dtype, qd)

    @torch.no_grad()
    def get_batch_tensors_qparams(self, act_tensors, alpha=0.01, args={}):
        """quant.py:561-586 on the device: per-segment torch.min / torch.max in one HBM pass
        (``lcq_minmax_segments``), the range and get_qparams in one tiny kernel
        (``lcq_act_static_qparams``). Returns (scales, zeros, qmin, qmax) lists, one entry per
        module input, as 0-dim tensors with the reference's dtypes."""
        if self.calib_algo == 'static_hist':
            assert self.sym is True and self.granularity == 'per_tensor', \
                'Only support per tensor static symmetric int quantize.'
            if not isinstance(self.bit, int):
                raise NotImplementedError('static_hist is for integer quantizers')
            scales_l, zeros_l, qmin_l, qmax_l = [], [], [], []
            for tensors in self.reshape_batch_tensors(act_tensors):
                dev = tensors[0].device
                mm = ops.minmax_segments(tensors)
                r = ops.act_static_hist_qparams(tensors, mm, self.bit, float(self.qmax))
                scales_l.append(r[0].clone())
                zeros_l.append(torch.tensor(0.0, device=dev))
                qmin_l.append(self.qmin.to(dev))
                qmax_l.append(self.qmax.to(dev))
            return scales_l, zeros_l, qmin_l, qmax_l
        if self.calib_algo not in ops.CALIB_ALGOS:
            raise ValueError(f'Unsupported calibration algorithm: {self.calib_algo}')
        if self.granularity != 'per_tensor':
            raise NotImplementedError('static activation qparams are per_tensor '
                                      '(base_blockwise_quantization.py:181-184)')
        if not self.round_zp:
            raise NotImplementedError('round_zp=False is not on the device path')
        scales_l, zeros_l, qmin_l, qmax_l = [], [], [], []
        for tensors in self.reshape_batch_tensors(act_tensors):
            dev = tensors[0].device
            mm = ops.minmax_segments(tensors)
            rdt = torch.float32 if self.calib_algo == 'static_minmax' else tensors[0].dtype
            sdt = self._static_scale_dtype(rdt)
            r = ops.act_static_qparams(mm, self.calib_algo, alpha, rdt, sdt, self.sym,
                                       float(self.qmin), float(self.qmax))
            scales_l.append(r[0].to(sdt))
            zeros_l.append(torch.tensor(0.0, device=dev) if self.sym else r[1].to(sdt))
            qmin_l.append(self.qmin.to(dev))
            qmax_l.append(self.qmax.to(dev))
        return scales_l, zeros_l, qmin_l, qmax_l


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
        if not self.round_zp:
            return s, qmin - (mn / s), qmax, qmin
        z = (qmin - torch.round(mn / s)).clamp(qmin, qmax)
        return s, z, qmax, qmin

    def _hqq_or_nozp(self, tensor):
        """qparams of the two paths the lane kernel does not fuse: calib_algo hqq
        (get_hqq_qparams, quant.py:680-689: tensor.float(), minmax qparams, the proximal
        search on the device) and minmax with round_zp False. Returns (x2, group, scales [ng],
        zeros [ng] | None, compute dtype)."""
        if self.granularity not in ('per_group', 'per_channel', 'per_token', 'per_head'):
            raise NotImplementedError(f'{self.calib_algo} / round_zp with {self.granularity}')
        qmin, qmax = self._iq
        if self.calib_algo == 'hqq':
            x2, group = self._kernel_view(tensor.float().contiguous())
            s, z = ops.minmax_qparams(x2, group, qmin, qmax, self.sym, self.round_zp)
            if z is None:  # sym: zeros = torch.tensor(0.0) until the first update
                z = torch.zeros_like(s)
            s, z, _ = ops.hqq_proximal(x2, group, s, z, qmin, qmax, self.lp_norm, self.beta,
                                       self.iters)
            return x2, group, s, z, torch.float32
        x2, group = self._kernel_view(tensor.contiguous())
        s, z = ops.minmax_qparams(x2, group, qmin, qmax, self.sym, round_zp=False)
        return x2, group, s, z, tensor.dtype

    def _mse(self, tensor):
        """(x2, group, scales [ng] fp32, zeros [ng] fp32 | None) from the MSE range search."""
        if self.granularity not in ('per_group', 'per_channel', 'per_token', 'per_tensor'):
            raise NotImplementedError(f'mse with {self.granularity}')
        x2, group = self._kernel_view(tensor.contiguous())
        if (x2.numel() // group) % self.mse_b_num:
            raise AssertionError('Batch number must be divisible by tensor.shape[0],')
        qmin, qmax = self._iq
        _, _, s, z = ops.mse_qparams(x2, group, self.sym, qmin, qmax, self._mse_nsteps(),
                                     float(self.mse_grid))
        return x2, group, s, z

    def get_hqq_qparams(self, tensor, args={}):
        """quant.py:680-689: (reshaped tensor.float(), best scales, zeros, qmax, qmin)."""
        _, _, s, z, _ = self._hqq_or_nozp(tensor)
        dev = tensor.device
        return (self.reshape_tensor(tensor.float()), s.view(-1, 1), z.view(-1, 1),
                self.qmax.to(dev), self.qmin.to(dev))

    def get_tensor_qparams(self, tensor, args={}):
        """quant.py:690-697: (reshaped tensor, scales, zeros, qmax, qmin)."""
        self._check_supported(args)
        f = self._factors(args)
        if f is not None:
            x2, group = self._kernel_view(tensor.contiguous())
            r = self._learnable(x2, group, f, tensor.dtype, qparams=True)
            dev = tensor.device
            zeros = r['zeros'] if not self.sym else torch.tensor(0.0)
            return (self.reshape_tensor(tensor), r['scales'], zeros, self.qmax.to(dev),
                    self.qmin.to(dev))
        if self.calib_algo == 'hqq':
            return self.get_hqq_qparams(tensor, args)
        if not self.round_zp and self.calib_algo != 'mse':
            _, _, s, z, _ = self._hqq_or_nozp(tensor)
            dev = tensor.device
            zeros = z.view(-1, 1) if not self.sym else torch.tensor(0.0)
            return (self.reshape_tensor(tensor), s.view(-1, 1), zeros, self.qmax.to(dev),
                    self.qmin.to(dev))
        if self.calib_algo == 'mse':  # fp32 qparams from the search over tensor.float()
            _, _, s, z = self._mse(tensor)
            dev = tensor.device
            zeros = z.view(-1, 1) if not self.sym else torch.tensor(0.0)
            scales = s.view(-1, 1)
            if self.granularity == 'per_tensor':
                scales = scales.reshape(())
                zeros = zeros.reshape(()) if not self.sym else zeros
            return (self.reshape_tensor(tensor), scales, zeros, self.qmax.to(dev),
                    self.qmin.to(dev))
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

    def _learnable(self, x2, group, f, dtype, qparams=False):
        up, low = f
        for t in (up, low):
            if t is not None and t.dtype != x2.dtype:
                raise NotImplementedError('clip factors in a dtype other than the weight\'s')
        qmin, qmax = self._iq
        return ops.int_quant_learnable(x2, group, up, low, qmin, qmax, self.sym, fq_dtype=dtype,
                                       qparams=qparams)

    # -- elementwise ops with given qparams (quant.py:699-717) ------------------------------
    def _static(self, tensor, scales, zeros, want):
        t2 = tensor.reshape(-1, tensor.shape[-1]).contiguous()
        s = scales.contiguous()
        if s.dim() == 0 and (not torch.is_tensor(zeros) or zeros.dim() == 0):
            if not self.round_zp:
                raise NotImplementedError('round_zp=False with 0-dim qparams')
            # per-tensor qparams as 0-dim tensors (static act qparams, per_tensor weights):
            # torch-CPU uses them as scalars at full precision, results in the tensor's dtype
            qmin, qmax = self._iq
            z = None
            if torch.is_tensor(zeros) and zeros.item() != 0 or (not torch.is_tensor(zeros)
                                                                  and zeros):
                z = torch.as_tensor(zeros, dtype=torch.float32, device=t2.device)
            r = ops.int_quant_static_scalar(t2, s.to(t2.device), z, qmin, qmax,
                                            ct_dtype=tensor.dtype, fq=want != 'codes',
                                            codes_dtype=torch.int32 if want == 'codes' else None)
            if want == 'codes':
                return r['codes'].to(tensor.dtype).reshape(tensor.shape)
            return r['fq'].reshape(tensor.shape)
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
        if zz is not None and zz.is_floating_point() and torch.is_tensor(zeros) and zeros.dim() > 0:
            ct = torch.promote_types(ct, zz.dtype)  # a 0-dim zero never promotes (torch rule)
        qmin, qmax = self._iq
        if want == 'codes':
            r = ops.int_quant_static(t2, group, s, zz, qmin, qmax, ct_dtype=ct, fq=False,
                                     codes_dtype=torch.int32, round_zp=self.round_zp)
            return r['codes'].to(ct).reshape(tensor.shape)
        r = ops.int_quant_static(t2, group, s, zz, qmin, qmax, ct_dtype=ct, fq=True,
                                 round_zp=self.round_zp)
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
        qmin, qmax = self._iq
        f = self._factors(args)
        if f is not None:  # calib_algo learnable with the v2 clip factors (w_qdq)
            x2, group = self._kernel_view(w.contiguous())
            fq = self._learnable(x2, group, f, w.dtype)['fq'].reshape(shape)
            return fq.T if tr else fq
        if self.calib_algo == 'mse':  # fp32 scales -> the quant_dequant computes in fp32
            x2, group, s, z = self._mse(w)
            fq = ops.int_quant_static(x2, group, s, z, qmin, qmax, ct_dtype=torch.float32,
                                      fq_dtype=w.dtype)['fq'].reshape(shape)
            return fq.T if tr else fq
        if self.calib_algo == 'hqq' or not self.round_zp:
            # hqq: quant_dequant of tensor.float() with fp32 qparams, then .to(weight dtype)
            x2, group, s, z, ct = self._hqq_or_nozp(w)
            fq = ops.int_quant_static(x2, group, s, z, qmin, qmax, ct_dtype=ct, fq_dtype=w.dtype,
                                      round_zp=self.round_zp)['fq'].reshape(shape)
            return fq.T if tr else fq
        x2, group = self._kernel_view(w.contiguous())
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
        if self.calib_algo == 'mse':
            x2, group, s, z = self._mse(weight)
            r = ops.int_quant_static(x2, group, s, z, qmin, qmax, ct_dtype=torch.float32,
                                     fq=False, codes_dtype=cd)
            r['scales'], r['zeros'] = s, (z if z is not None else None)
        elif self.calib_algo == 'hqq' or not self.round_zp:
            x2, group, s, z, ct = self._hqq_or_nozp(weight)
            r = ops.int_quant_static(x2, group, s, z, qmin, qmax, ct_dtype=ct, fq=False,
                                     codes_dtype=cd, round_zp=self.round_zp)
            r['scales'], r['zeros'] = s, z
        else:
            r = ops.int_quant_dynamic(x2, group, qmin, qmax, self.sym, fq=False,
                                      codes_dtype=cd)
        codes = r['codes'].reshape(weight.shape)
        scales = r['scales'] * osf if osf != 1 else r['scales']
        zeros = None
        if not self.sym:  # quant.py:938-941: float zeros kept when round_zp is False
            zeros = r['zeros'].to(cd) if self.round_zp else r['zeros']
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


_FLOAT_RANGES = {  # quant.py:982-996
    ('e4m3', 8): torch.float8_e4m3fn,
    ('e5m2', 8): torch.float8_e5m2,
    ('e3m2', 6): (-28, 28),
    ('e4m7', 12): (-510, 510),
    ('e2m1', 4): (-6, 6),
}


class FloatQuantizer(BaseQuantizer):
    """FloatQuantizer (quant.py:963-1229) on the lcq FP8 kernels.

    ``use_qtorch=True``: absmax scales in the tensor dtype (fp32 for per_block), then the
    value rounding. qtorch's ``float_quantize`` is not in this image, so the rounding is the
    native cast (torch / c10 ``Float8_e4m3fn`` / ``Float8_e5m2`` RNE) -- exact for the scales
    and every surrounding op, parity-unpinned for qtorch's own rounding.
    Only e4m3 / e5m2 have a native cast; other formats need qtorch and raise.
    ``use_qtorch=False``: ``get_float_qparams`` emulation (per-element power-of-two scales),
    bit-exact for bf16 / fp16 tensors (``lcq_fp_emul_quant``).
    """

    def __init__(self, bit, symmetric, granularity, **kwargs):
        super().__init__(bit, symmetric, granularity, **kwargs)
        self.sym = True
        self.quant_type = 'float-quant'
        self.e_bits = int(self.bit[1])
        self.m_bits = int(self.bit[-1])
        self.sign_bits = 1
        self.num_bits = self.e_bits + self.m_bits + self.sign_bits
        self.default_bias = 2 ** (self.e_bits - 1)
        self.dst_nbins = 2 ** self.num_bits
        self.use_qtorch = self.kwargs.get('use_qtorch')
        self.fp8_dtype = {'e4m3': torch.float8_e4m3fn, 'e5m2': torch.float8_e5m2}.get(bit)
        if self.use_qtorch:
            if 'float_range' in self.kwargs:
                self.qmin, self.qmax = self.kwargs['float_range']
            else:
                key = (self.bit, self.num_bits)
                if key not in _FLOAT_RANGES:
                    raise NotImplementedError('Only 4, 6, 8, and 12-bit quantization is supported.')
                r = _FLOAT_RANGES[key]
                if isinstance(r, tuple):
                    self.qmin, self.qmax = r
                else:
                    fi = torch.finfo(r)
                    self.qmin, self.qmax = fi.min, fi.max
            self.qmax = torch.tensor(self.qmax)
            self.qmin = torch.tensor(self.qmin)

    # -- helpers ---------------------------------------------------------------------------
    def _cast_dtype(self):
        if self.fp8_dtype is None:
            raise NotImplementedError(f'{self.bit}: only e4m3 / e5m2 have a native cast; the '
                                      'qtorch rounding of other formats is not available')
        return self.fp8_dtype

    def _check(self, args):
        if self.calib_algo not in _MINMAX_LIKE:
            raise NotImplementedError(f'calib_algo={self.calib_algo} is not on the device path')
        if 'rounding' in args:
            raise NotImplementedError("args['rounding'] is not on the device path")

    def _qmax_f(self):
        return float(self.qmax.item())

    def _view(self, tensor):
        """(2-D view, group, per_tensor) for the row/group kernels."""
        g = self.granularity
        if g == 'per_tensor':
            return tensor.reshape(1, -1), tensor.numel(), True
        x2, group = self._kernel_view(tensor)
        return x2, group, False

    def _dyn(self, tensor, *, codes, fq, fq_dtype=None):
        """Dynamic FP8 over the quantizer's granularity: dict(codes, fq, scales)."""
        fp8 = self._cast_dtype()
        t = tensor.contiguous()
        if self.granularity == 'per_block':
            if self.block_size != 128:
                raise NotImplementedError('per_block FP8 supports block_size 128')
            r = ops.fp8_quant_blocks(t, fp8, 128, qmax=self._qmax_f(), clamp_min=1e-5,
                                     add_zero=True, codes=codes, fq=fq, fq_dtype=fq_dtype)
            return r
        x2, group, pt = self._view(t)
        r = ops.fp8_quant(x2, group, fp8, qmax=self._qmax_f(), clamp_min=1e-5, add_zero=True,
                          per_tensor=pt, codes=codes, fq=fq, fq_dtype=fq_dtype)
        if codes:
            r['codes'] = r['codes'].reshape(tensor.shape)
        if fq:
            r['fq'] = r['fq'].reshape(tensor.shape)
        return r

    def _emul(self, tensor):
        if self.granularity in ('per_tensor', 'per_block'):
            raise NotImplementedError(f'use_qtorch=False with {self.granularity} (the reference '
                                      'indexes maxval.shape[0] / pads differently here)')
        x2, group, _ = self._view(tensor.contiguous())
        return ops.fp_emul_quant(x2, group, self.e_bits, self.m_bits).reshape(tensor.shape)

    # -- qparams (API parity; quant.py:1005-1059) --------------------------------------------
    def get_float_qparams(self, tensor, tensor_range, device):
        """quant.py:1005-1027 in torch on the tensor's device (API helper)."""
        min_val, max_val = tensor_range
        maxval = torch.max(max_val, -min_val)
        e_bits = torch.tensor(self.e_bits, dtype=torch.float32, device=device)
        m_bits = torch.tensor(self.m_bits, dtype=torch.float32, device=device)
        if maxval.shape[0] != 1 and len(maxval.shape) != len(tensor.shape):
            maxval = maxval.view([-1] + [1] * (len(tensor.shape) - 1))
        if e_bits >= 5:
            maxval = maxval.to(dtype=torch.float32)
        bias = 2 ** e_bits - torch.log2(maxval) + torch.log2(2 - 2 ** (-m_bits)) - 1
        xc = torch.min(torch.max(tensor, -maxval), maxval)
        log_scales = torch.clamp((torch.floor(torch.log2(torch.abs(xc)) + bias)).detach(), 1.0)
        return xc, 2.0 ** (log_scales - m_bits - bias)

    def get_qparams(self, tensor_range, device):
        min_val, max_val = tensor_range
        abs_max = torch.max(max_val.abs(), min_val.abs()).clamp(min=1e-5)
        qmax = self.qmax.to(device)
        return abs_max / qmax, torch.tensor(0.0), qmax, self.qmin.to(device)

    def get_minmax_range(self, tensor):
        if self.granularity == 'per_block':
            return (tensor.abs().float().amin(dim=(1, 3), keepdim=True),
                    tensor.abs().float().amax(dim=(1, 3), keepdim=True))
        return super().get_minmax_range(tensor)

    def get_tensor_qparams(self, tensor, args={}):
        """quant.py:1044-1059: (tensor, scales, zeros, qmax, qmin)."""
        self._check(args)
        if not self.use_qtorch:
            t = self.reshape_tensor(tensor)
            xc, scales = self.get_float_qparams(t, self.get_minmax_range(t), t.device)
            return xc, scales, torch.tensor(0), None, None
        r = self._dyn(tensor, codes=False, fq=False)
        s = r['scales']
        if self.granularity == 'per_tensor':
            s = s.reshape(())
        elif self.granularity == 'per_block':
            s = s.view(s.shape[0], 1, s.shape[1], 1)
        dev = tensor.device
        return (self.reshape_tensor(tensor), s, torch.tensor(0.0), self.qmax.to(dev),
                self.qmin.to(dev))

    # -- elementwise with given qparams (quant.py:1061-1080) ----------------------------------
    def _static(self, tensor, scales, want, fq_dtype=None):
        fp8 = self._cast_dtype()
        s = scales
        s.masked_fill_(s == 0, 1)  # quant.py:1062 mutates the caller's scales
        if self.granularity == 'per_block' and s.dim() == 4:
            raise NotImplementedError('static per_block: use the dynamic path')
        ct = tensor.dtype if s.dim() == 0 else torch.promote_types(tensor.dtype, s.dtype)
        r = ops.fp8_quant_static(tensor.reshape(tensor.shape[0] if tensor.dim() else 1, -1),
                                 s.reshape(-1), fp8, ct_dtype=ct, add_zero=True,
                                 codes=want == 'codes', fq=want == 'fq', fq_dtype=fq_dtype,
                                 saturate=True)
        return r[want].reshape(tensor.shape)

    def quant(self, tensor, scales, zeros, qmax, qmin):
        if not self.use_qtorch:
            scales[scales == 0] = 1
            return self.round_func(tensor / scales + zeros)
        return self._static(tensor, scales, 'codes').float()

    def dequant(self, tensor, scales, zeros):
        return (tensor - zeros) * scales

    def quant_dequant(self, tensor, scales, zeros, qmax, qmin):
        if not self.use_qtorch:
            return self.dequant(self.quant(tensor, scales, zeros, qmax, qmin), scales, zeros)
        return self._static(tensor, scales, 'fq', fq_dtype=torch.float32)

    # -- weights / activations -----------------------------------------------------------------
    @staticmethod
    def _tr(args):
        return 'dim' in args and 'ic' in args['dim']

    def fake_quant_weight_dynamic(self, weight, args={}):
        """quant.py:1119-1139."""
        self._check(args)
        w = weight.T if self._tr(args) else weight
        if self.use_qtorch:
            out = self._dyn(w, codes=False, fq=True, fq_dtype=w.dtype)['fq']
        else:
            out = self._emul(w)
        return out.T if self._tr(args) else out

    def fake_quant_weight_static(self, weight, args):
        """quant.py:1084-1117."""
        self._check(args)
        if not self.use_qtorch:
            raise NotImplementedError('static use_qtorch=False fake quant is not on the device '
                                      'path')
        w = weight.T if self._tr(args) else weight
        out = self._static(w, args['scales'], 'fq', fq_dtype=w.dtype)
        return out.T if self._tr(args) else out

    def fake_quant_act_dynamic(self, act, args={}):
        """quant.py:1072-1081."""
        self._check(args)
        if not self.use_qtorch:
            return self._emul(act)
        return self._dyn(act, codes=False, fq=True, fq_dtype=act.dtype)['fq']

    def fake_quant_act_static(self, act, args={}):
        """quant.py:1058-1070."""
        self._check(args)
        if not self.use_qtorch:
            raise NotImplementedError('static use_qtorch=False fake quant is not on the device '
                                      'path')
        return self._static(act, args['scales'], 'fq', fq_dtype=act.dtype)

    def _qshape(self, codes, scales):
        if self.granularity == 'per_tensor':
            return 1
        if self.granularity == 'per_block':
            return tuple(scales.shape)
        return (codes.shape[0], -1)

    def real_quant_weight_dynamic(self, weight, args={}):
        """quant.py:1191-1221: (fp8 weight, scales, None)."""
        assert self.bit in ['e4m3', 'e5m2'], 'Only FP8 E4M3 and E5M2 support real quant'
        if not self.use_qtorch:
            raise NotImplementedError('use_qtorch=False real quant is not on the device path')
        osf = args.pop('output_scale_factor', 1) if 'output_scale_factor' in args else 1
        self._check(args)
        r = self._dyn(weight, codes=True, fq=False)
        codes, scales = r['codes'], r['scales']
        if osf != 1:
            scales = scales * osf
        return codes, scales.view(self._qshape(codes, scales)), None

    def real_quant_weight_from_block_fp8(self, codes, scale_inv, block_size):
        """The deploy chain of a block-fp8 checkpoint weight: weight_cast_to_bf16 then
        real_quant_weight_dynamic (module_utils.py:917-922). Per-tensor e4m3/e5m2 runs fused
        (lcq_fp8_block_to_tensor, bit-identical, 3 B/element); other granularities compose."""
        if self.granularity == 'per_tensor' and self.use_qtorch and self.fp8_dtype is not None:
            c, s = ops.fp8_block_to_tensor(codes, scale_inv, block_size, self.fp8_dtype,
                                           qmax=self._qmax_f())
            return c, s, None
        w = weight_cast_to_bf16(codes, scale_inv, block_size)
        return self.real_quant_weight_dynamic(w)

    def real_quant_weights_from_block_fp8(self, codes, scales_inv, block_size):
        """Batched real_quant_weight_from_block_fp8 over lists (per-tensor e4m3/e5m2: one
        launch pair for all of them). Returns a list of (codes, scale[1], None)."""
        if self.granularity == 'per_tensor' and self.use_qtorch and self.fp8_dtype is not None:
            cs, ss = ops.fp8_block_to_tensor_many(codes, scales_inv, block_size, self.fp8_dtype,
                                                  qmax=self._qmax_f())
            return [(c, ss[i:i + 1], None) for i, c in enumerate(cs)]
        return [self.real_quant_weight_from_block_fp8(c, s, block_size)
                for c, s in zip(codes, scales_inv)]

    def real_quant_weight_static(self, weight, args):
        """quant.py:1161-1189."""
        assert self.bit in ['e4m3', 'e5m2'], 'Only FP8 E4M3 and E5M2 support real quant'
        if not self.use_qtorch:
            raise NotImplementedError('use_qtorch=False real quant is not on the device path')
        osf = args.pop('output_scale_factor', 1) if 'output_scale_factor' in args else 1
        scales = args['scales']
        codes = self._static(weight, scales, 'codes')
        scales = scales * osf
        if self.granularity == 'per_block':
            return codes, scales.view(scales.shape[0], scales.shape[2]), None
        return codes, scales.view(self._qshape(codes, scales)), None

    def __repr__(self):
        return (f'FloatQuantizer(bit={self.bit},e_bits={self.e_bits}, m_bits={self.m_bits},'
                f'granularity={self.granularity},kwargs={self.kwargs}, '
                f'qmin={getattr(self, "qmin", None)}, qmax={getattr(self, "qmax", None)})')
