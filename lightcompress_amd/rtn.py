"""RTN (drop-in for llmc ``quantization/rtn.py``): no calibration transform; all the work is
the deploy-time fake / real quant (HIP grouped-quant kernels). With static activation
quantization the block loop runs (rtn.py:16-20) only to register the per-tensor act qparams
(``register_act_qparams``, device calibration kernels)."""
import torch

from .base_blockwise_quantization import BaseBlockwiseQuantization
from .registry import ALGO_REGISTRY


@ALGO_REGISTRY
class RTN(BaseBlockwiseQuantization):
    def block_has_work(self):
        return self.act_static

    @torch.no_grad()
    def block_opt(self, block, *opt_kwargs):
        if self.act_static:  # rtn.py:16-20 (kv-cache quant is out of scope)
            super().block_opt(block, *opt_kwargs)

    @torch.no_grad()
    def subset_transform(self, subset, input_feat, subset_kwargs):
        pass
