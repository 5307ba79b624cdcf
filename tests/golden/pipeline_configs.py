"""Configs of the end-to-end pipeline goldens (data only; shared by tests/golden/gen_pipeline.py,
which runs the reference in the build container, and tests/test_pipeline_golden_gpu.py)."""
from pathlib import Path

MODEL_DIR = Path(__file__).resolve().parent / 'pipeline_llama'

# reference configs (configs/quantization/methods/*/..._w_only.yml), calib shrunk to tiny sizes
CONFIGS = {
    'gptq': {'quant': {'method': 'GPTQ',
                       'weight': {'bit': 4, 'symmetric': False, 'granularity': 'per_group',
                                  'group_size': 128},
                       'special': {'actorder': True, 'static_groups': False, 'percdamp': 0.01,
                                   'blocksize': 128, 'true_sequential': True},
                       'quant_out': True},
             'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}},
    # static_groups (gptq.py:224-227); deployed weights only (Hessians pinned by 'gptq')
    'gptq_static': {'quant': {'method': 'GPTQ',
                              'weight': {'bit': 4, 'symmetric': False,
                                         'granularity': 'per_group', 'group_size': 64},
                              'special': {'actorder': True, 'static_groups': True,
                                          'percdamp': 0.01, 'blocksize': 128,
                                          'true_sequential': True},
                              'quant_out': True},
                    'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}, 'diag': False},
    'awq': {'quant': {'method': 'Awq',
                      'weight': {'bit': 4, 'symmetric': True, 'granularity': 'per_group',
                                 'group_size': 128},
                      'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                  'clip_sym': True}},
            'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    'awq_qout_asym': {'quant': {'method': 'Awq',
                                'weight': {'bit': 4, 'symmetric': False,
                                           'granularity': 'per_group', 'group_size': 128},
                                'special': {'trans': True, 'trans_version': 'v2',
                                            'weight_clip': True, 'clip_sym': False},
                                'quant_out': True},
                      'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    # configs/quantization/methods/RTN/rtn_w_a_pertensor_static.yml with calib_algo
    # static_minmax (static_hist is not on the device path); deployed act scales compared too
    'rtn_a8_static': {'quant': {'method': 'RTN',
                                'weight': {'bit': 8, 'symmetric': True,
                                           'granularity': 'per_channel', 'group_size': -1},
                                'act': {'bit': 8, 'symmetric': True, 'granularity': 'per_tensor',
                                        'static': True, 'calib_algo': 'static_minmax'}},
                      'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}, 'diag': False},
    # configs/quantization/methods/RTN/rtn_w_a_pertensor_static.yml as shipped (static_hist)
    'rtn_a8_hist': {'quant': {'method': 'RTN',
                              'weight': {'bit': 8, 'symmetric': True,
                                         'granularity': 'per_channel', 'group_size': -1},
                              'act': {'bit': 8, 'symmetric': True, 'granularity': 'per_tensor',
                                      'static': True, 'calib_algo': 'static_hist'}},
                    'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}, 'diag': False},
    'rtn': {'quant': {'method': 'RTN',
                      'weight': {'bit': 8, 'symmetric': True, 'granularity': 'per_channel'}},
            'calib': None},
}
