"""Pipeline helpers mirroring llmc/__main__.py:28-177 for the hot path: build the algorithm
from the YAML config, run the block loop, deploy / save."""
from __future__ import annotations

from .registry import ALGO_REGISTRY, MODEL_REGISTRY
from . import awq, gptq, hqq, rtn  # noqa: F401  (register algorithms)
from . import deepseekv3, llama, opt  # noqa: F401  (register model adapters)


def build_model(config, device='cuda'):
    """MODEL_REGISTRY[config.model.type](config) (llmc/__main__.py:31)."""
    return MODEL_REGISTRY[config['model']['type']](config, device=device)


def build_algo(model, config, calib_input, padding_mask=None):
    """ALGO_REGISTRY[method](model, quant_config, input, padding_mask, config)."""
    qc = config['quant']
    qc.setdefault('modality', 'language')
    cls = ALGO_REGISTRY[qc['method']]
    return cls(model, qc, calib_input, padding_mask, config)


def run(model, config, calib_input, deploy_format=None, save_path=None):
    algo = build_algo(model, config, calib_input)
    algo.run_block_loop()
    if deploy_format:
        algo.deploy(deploy_format)
    if save_path:
        algo.save_model(save_path)
    return algo
