"""HQQ (drop-in for llmc ``quantization/hqq.py``): data-free half-quadratic qparam search per
linear. block_opt (hqq.py:64-97): W.float() (transposed when ``special.axis`` is 0, so the
groups run along the output channels), the weight quantizer's qparams of that tensor
(get_tensor_qparams: min/max, usually with ``round_zp: False``), then the proximal loop
(optimize_weights_proximal, hqq.py:36-61) on the device (``lcq_hqq_proximal``: no host sync
per iteration), registered as buf_scales / buf_zeros / buf_qmax / buf_qmin. w_qdq
(hqq.py:99-108) fake-quantizes with those static qparams along the same axis."""
import torch

from . import ops
from .base_blockwise_quantization import BaseBlockwiseQuantization
from .registry import ALGO_REGISTRY


@ALGO_REGISTRY
class HQQ(BaseBlockwiseQuantization):
    def __init__(self, model, quant_config, input, padding_mask, config):
        super().__init__(model, quant_config, input, padding_mask, config)
        self.add_quant_config()

    def add_quant_config(self):
        sp = self.quant_config['special']
        self.lp_norm = sp['lp_norm']
        self.beta = sp['beta']
        self.kappa = sp['kappa']  # the reference's shrink_op reads self.beta, never current_beta
        self.iters = sp['iters']
        self.axis = sp['axis']

    @torch.no_grad()
    def optimize_weights_proximal(self, W_f, scales, zeros, qmax, qmin):
        """hqq.py:36-61 on the device: W_f is the reshaped fp32 group view."""
        q = self.wquantizer
        group = W_f.shape[-1]
        zeros = torch.as_tensor(zeros, dtype=torch.float32, device=W_f.device)
        s, z, _ = ops.hqq_proximal(W_f.reshape(-1, group), group, scales.reshape(-1), zeros,
                                   int(q.qmin.item()), int(q.qmax.item()), self.lp_norm,
                                   self.beta, self.iters)
        return s.view(-1, 1), z.view(-1, 1)

    @torch.no_grad()
    def block_opt(self, block):
        # shard_units (data-free, world > 1): only this rank's linears; deploy publishes
        for name, layer in self.owned_linears(block).items():
            tensor = layer.weight.data.float()
            if self.axis == 0:
                tensor = tensor.T
            tensor, org_scales, org_zeros, qmax, qmin = self.wquantizer.get_tensor_qparams(
                tensor.contiguous())
            best_scales, best_zeros = self.optimize_weights_proximal(tensor, org_scales,
                                                                     org_zeros, qmax, qmin)
            layer.register_buffer('buf_scales', best_scales)
            layer.register_buffer('buf_zeros', best_zeros)
            layer.register_buffer('buf_qmax', torch.as_tensor(qmax).clone())
            layer.register_buffer('buf_qmin', torch.as_tensor(qmin).clone())

    def w_qdq(self, module, wquantizer):
        args = {'scales': module.buf_scales, 'zeros': module.buf_zeros,
                'qmax': module.buf_qmax, 'qmin': module.buf_qmin}
        if self.axis == 0:
            args['dim'] = 'ic'
        return wquantizer.fake_quant_weight_static(module.weight, args)
