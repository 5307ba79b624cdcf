"""Quantized-checkpoint config writers (drop-in for ``llmc/utils/export_vllm.py`` and
``llmc/utils/export_autoawq.py``) and the save flow of ``llmc/__main__.py:96-160``.

The packed tensors themselves come from the deploy path (``VllmRealQuantLinear`` /
``AutoawqRealQuantLinear`` buffers, produced on the device by the pack kernels) and are written
by ``save_model`` (HF ``save_pretrained``: safetensors); these functions add the
``compression_config`` / ``quantization_config`` entry the serving engines read.
"""
from __future__ import annotations

import json
import os


def _get(d, k, default=None):
    return d.get(k, default) if isinstance(d, dict) else getattr(d, k, default)


def _rw_config(path, fn):
    cfg_file = os.path.join(path, 'config.json')
    with open(cfg_file) as f:
        cfg = json.load(f)
    fn(cfg)
    with open(cfg_file, 'w') as f:
        json.dump(cfg, f, indent=4)


def update_vllm_quant_config(model, config, save_quant_path,
                             vllm_quant_method='compressed-tensors'):
    """export_vllm.py:4-125: vLLM compressed-tensors (or fp8) quantization config."""
    q = config['quant']
    w = q['weight']
    act = q.get('act')
    need_pack = w.get('need_pack', False)
    weight_quant_type = w.get('quant_type', 'int-quant')
    act_quant_type = None
    if act is not None:
        act_quant_type = act.get('quant_type', 'int-quant')
        assert act_quant_type == weight_quant_type
    a_num_bits = None
    if act_quant_type == 'float-quant':
        if act.get('static', False):
            qc = {'activation_scheme': 'static', 'ignored_layers': [model.skip_layer_name()],
                  'quant_method': 'fp8'}
            _rw_config(save_quant_path, lambda c: c.__setitem__('quantization_config', qc))
            return
        elif w.get('granularity', 'per_block'):  # (always true in the reference)
            qc = {'activation_scheme': 'dynamic', 'fmt': 'e4m3', 'quant_method': 'fp8',
                  'weight_block_size': [w['block_size'], w['block_size']]}
            _rw_config(save_quant_path, lambda c: c.__setitem__('quantization_config', qc))
            return
    elif need_pack:
        fmt, quant_type, w_num_bits = 'pack-quantized', 'int', w['bit']
    elif weight_quant_type == 'float-quant':
        fmt, quant_type, w_num_bits = 'float-quantized', 'float', 8
    else:
        fmt, quant_type, w_num_bits = 'int-quantized', 'int', w['bit']
        if act is not None:
            a_num_bits = act['bit']
    group_size = w['group_size'] if w['granularity'] == 'per_group' else None
    dynamic = (not act['static']) if (act is not None and 'static' in act) else True
    qc = {
        'config_groups': {
            'group_0': {
                'targets': ['Linear'],
                'input_activations': {
                    'dynamic': dynamic, 'group_size': None, 'num_bits': a_num_bits,
                    'observer': 'minmax', 'observer_kwargs': {},
                    'strategy': 'token' if act['granularity'] == 'per_token' else 'tensor',
                    'symmetric': act['symmetric'], 'type': quant_type,
                } if act is not None else None,
                'weights': {
                    'dynamic': False, 'group_size': group_size, 'num_bits': w_num_bits,
                    'observer': 'minmax', 'observer_kwargs': {},
                    'strategy': 'group' if w['granularity'] == 'per_group' else 'channel',
                    'symmetric': w['symmetric'], 'type': quant_type,
                },
            }
        },
        'format': fmt,
        'ignore': model.skip_layer_name(),
        'quant_method': vllm_quant_method,
    }

    def upd(c):
        if weight_quant_type == 'int-quant' and 'quantization_config' in c:
            del c['quantization_config']
        c['compression_config'] = qc
    _rw_config(save_quant_path, upd)


def update_autoawq_quant_config(config, save_quant_path):
    """export_autoawq.py:4-30: AutoAWQ ``quantization_config``."""
    w = config['quant']['weight']
    qc = {'bits': w['bit'],
          'group_size': w['group_size'] if w['granularity'] == 'per_group' else -1,
          'modules_to_not_convert': None, 'quant_method': 'awq',
          'version': w['pack_version'].split('_')[0],
          'zero_point': not w['symmetric']}

    def upd(c):
        c.pop('quantization_config', None)
        c['quantization_config'] = qc
    _rw_config(save_quant_path, upd)


def save_quantized(algo, config, save_quant_path):
    """The real-quant branch of __main__.py:96-160 for one language modality: checks, deploy,
    save_model (safetensors) and the serving-engine config."""
    save = config.get('save', {}) or {}
    w, a = config['quant']['weight'], config['quant'].get('act')
    os.makedirs(save_quant_path, exist_ok=True)
    if save.get('save_vllm', False) or save.get('save_sgl', False) or \
            save.get('save_lightllm', False):
        if isinstance(w['bit'], str):
            assert w['symmetric'], 'Only symmetric quant is supported.'
            assert w['bit'] in ['e4m3', 'e3m4'], 'Supported quant: w8a16.'
            if a:
                assert w['symmetric'] and a['symmetric'], 'Only symmetric quant is supported.'
                assert (w['bit'] == a['bit'] and w['bit'] in ['e4m3', 'e5m2']
                        and a['bit'] in ['e4m3', 'e5m2']), 'Only WA FP8 quant is supported'
        else:
            assert w['symmetric'], 'Only symmetric quant is supported.'
            assert w['bit'] in [4, 8], 'Supported quant: w4a16, w8a16, w8a8.'
            if a:
                assert a['symmetric'], 'Only symmetric quant is supported.'
                assert a['bit'] == 8, 'Supported quant: w4a16, w8a16, w8a8.'
        fmt = ('vllm_quant' if save.get('save_vllm', False) else
               'lightllm_quant' if save.get('save_lightllm', False) else 'sgl_quant')
        algo.deploy(fmt)
        algo.save_model(save_quant_path)
        update_vllm_quant_config(algo.model, config, save_quant_path)
    elif save.get('save_autoawq', False) or save.get('save_mlcllm', False):
        assert w['bit'] in [4] and a is None, \
            'AutoAWQ supports only 4-bit weight-only quantization.'
        assert not w['symmetric'], 'Only asymmetric quant is supported.'
        algo.deploy('autoawq_quant' if save.get('save_autoawq', False) else 'mlcllm_quant')
        algo.save_model(save_quant_path)
        update_autoawq_quant_config(config, save_quant_path)
    else:
        raise ValueError('no real-quant save target in config.save')
