"""RTN (drop-in for llmc ``quantization/rtn.py``): no calibration transform; all the work is
the deploy-time fake / real quant (HIP grouped-quant kernels)."""
import torch

from .base_blockwise_quantization import BaseBlockwiseQuantization
from .registry import ALGO_REGISTRY


@ALGO_REGISTRY
class RTN(BaseBlockwiseQuantization):
    @torch.no_grad()
    def block_opt(self, block, *opt_kwargs):
        return  # rtn.py:16-20 (no kv-cache / static-act paths on the device path)

    @torch.no_grad()
    def subset_transform(self, subset, input_feat, subset_kwargs):
        pass
