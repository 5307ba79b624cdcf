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
    # do_gqa_trans (awq.py:338-351, base_blockwise_quantization.py:591-595, 678-685): the
    # o_proj subset is searched on v_proj's input and its scales move into v_proj's rows
    'awq_gqa': {'quant': {'method': 'Awq',
                          'weight': {'bit': 4, 'symmetric': True, 'granularity': 'per_group',
                                     'group_size': 128},
                          'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                      'clip_sym': True, 'do_gqa_trans': True}},
                'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    'awq_qout_asym': {'quant': {'method': 'Awq',
                                'weight': {'bit': 4, 'symmetric': False,
                                           'granularity': 'per_group', 'group_size': 128},
                                'special': {'trans': True, 'trans_version': 'v2',
                                            'weight_clip': True, 'clip_sym': False},
                                'quant_out': True},
                      'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    # configs/quantization/backend/vllm/awq_w8a8.yml: int8 per_channel weights, int8 dynamic
    # per_token activations (the search and the clip see fake-quantized inputs), per-channel
    # auto-clip, quant_out
    'awq_w8a8': {'quant': {'method': 'Awq',
                           'weight': {'bit': 8, 'symmetric': True, 'granularity': 'per_channel',
                                      'group_size': -1},
                           'act': {'bit': 8, 'symmetric': True, 'granularity': 'per_token'},
                           'special': {'trans': True, 'trans_version': 'v2',
                                       'weight_clip': True},
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
    # configs/quantization/methods/HQQ/hqq_w_only.yml (data-free; axis 0: groups along OC)
    'hqq': {'quant': {'method': 'HQQ',
                      'weight': {'bit': 4, 'symmetric': False, 'granularity': 'per_group',
                                 'group_size': 128, 'round_zp': False},
                      'special': {'axis': 0, 'lp_norm': 0.7, 'beta': 10, 'kappa': 1.01,
                                  'iters': 20}},
            'calib': None},
    'rtn': {'quant': {'method': 'RTN',
                      'weight': {'bit': 8, 'symmetric': True, 'granularity': 'per_channel'}},
            'calib': None},
    # ---- OPT (opt.py:53-89; fc2 do_trans False), fp16 -------------------------------------
    # BASELINE config 1: OPT-125M RTN w8a16 per-channel (data-free)
    'opt_rtn': {'model': 'Opt',
                'quant': {'method': 'RTN',
                          'weight': {'bit': 8, 'symmetric': True, 'granularity': 'per_channel'}},
                'calib': None},
    'opt_awq': {'model': 'Opt',
                'quant': {'method': 'Awq',
                          'weight': {'bit': 4, 'symmetric': True, 'granularity': 'per_group',
                                     'group_size': 128},
                          'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                      'clip_sym': True}},
                'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    'opt_gptq': {'model': 'Opt',
                 'quant': {'method': 'GPTQ',
                           'weight': {'bit': 4, 'symmetric': False, 'granularity': 'per_group',
                                      'group_size': 128},
                           'special': {'actorder': True, 'static_groups': False,
                                       'percdamp': 0.01, 'blocksize': 128,
                                       'true_sequential': True},
                           'quant_out': True},
                 'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}},
    # ---- DeepSeek-V3 (deepseekv3.py:69-167: MLA subsets, MoE + per-expert down subsets) -----
    # configs/quantization/deepseekv3/awq_w_only_dsv3_bf16.yml, calib shrunk
    'dsv3_awq': {'model': 'DeepseekV3',
                 'quant': {'method': 'Awq',
                           'weight': {'bit': 4, 'symmetric': False, 'granularity': 'per_group',
                                      'group_size': 64},
                           'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                       'save_mem': False}},
                 'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    # static per-tensor activation calibration through the expert subsets (each expert's
    # act scale from the tokens routed to it). The FP8 form (e4m3 act, sglang/fp8 configs)
    # needs qtorch in the reference (quant.py:975-978, absent), so the reference runs the
    # int8 form; tests/test_models_gpu.py checks the FP8 run's scales against these.
    'dsv3_rtn_a8_static': {'model': 'DeepseekV3',
                           'quant': {'method': 'RTN',
                                     'weight': {'bit': 8, 'symmetric': True,
                                                'granularity': 'per_channel', 'group_size': -1},
                                     'act': {'bit': 8, 'symmetric': True,
                                             'granularity': 'per_tensor', 'static': True,
                                             'calib_algo': 'static_minmax'}},
                           'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}, 'diag': False},
    # ---- float-quant (FP8 e4m3) weights through AWQ / GPTQ (configs/quantization/backend/
    # vllm/fp8/*.yml). These need qtorch in the reference (quant.py:975-978, absent), so the
    # generator gives the reference's quant module a float_quantize that is the native
    # Float8_e4m3fn RNE cast (the rounding our FloatQuantizer documents); every other op of the
    # search, the clip, the column loop and the deploy is the reference's own ('qtorch_native').
    # awq_fp8_static.yml as shipped omits the act calib_algo, which get_batch_tensors_qparams
    # rejects (quant.py:564-574); static_minmax is the minmax-like choice it needs. Its
    # quant_out forward feeds o_proj / down inputs beyond the act range calibrated on the float
    # inputs (and GPTQ's error-compensated columns exceed their static scales): c10's plain cast
    # maps |x / s| >= 464 to NaN there, hence the saturating stand-in.
    'awq_fp8_static': {'quant': {'method': 'Awq',
                                 'weight': {'quant_type': 'float-quant', 'bit': 'e4m3',
                                            'symmetric': True, 'granularity': 'per_tensor',
                                            'use_qtorch': True},
                                 'act': {'quant_type': 'float-quant', 'bit': 'e4m3',
                                         'symmetric': True, 'granularity': 'per_tensor',
                                         'use_qtorch': True, 'static': True,
                                         'calib_algo': 'static_minmax'},
                                 'special': {'trans': True, 'trans_version': 'v2',
                                             'weight_clip': True},
                                 'quant_out': True},
                       'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128},
                       'qtorch_native': True},
    'awq_fp8': {'quant': {'method': 'Awq',
                          'weight': {'quant_type': 'float-quant', 'bit': 'e4m3',
                                     'symmetric': True, 'granularity': 'per_channel',
                                     'use_qtorch': True},
                          'act': {'quant_type': 'float-quant', 'bit': 'e4m3', 'symmetric': True,
                                  'granularity': 'per_token', 'use_qtorch': True},
                          'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True},
                          'quant_out': True},
                'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}, 'qtorch_native': True},
    'gptq_fp8': {'quant': {'method': 'GPTQ',
                           'weight': {'quant_type': 'float-quant', 'bit': 'e4m3',
                                      'symmetric': True, 'granularity': 'per_channel',
                                      'use_qtorch': True},
                           'act': {'quant_type': 'float-quant', 'bit': 'e4m3', 'symmetric': True,
                                   'granularity': 'per_token', 'use_qtorch': True},
                           'special': {'actorder': True, 'static_groups': False,
                                       'percdamp': 0.01, 'blocksize': 128,
                                       'true_sequential': True},
                           'quant_out': True},
                 'calib': {'bs': 1, 'n_samples': 16, 'seq_len': 128}, 'qtorch_native': True},
    # ---- clip_version v2 (learnable clip factors) -------------------------------------------
    # configs/quantization/combination/awq_comb_omni/{w8a8,w6a6}/step_1_awq.yml: asym
    # per_channel weights with calib_algo learnable, asym per_token activations, the clip
    # searched with learnable-range candidates and kept as logit factors (buf_*bound_factor)
    # that the deploy fake quant applies; scales.pth / clips.pth written (paths filled in by
    # the generator and the test)
    'awq_omni_w8a8': {'quant': {'method': 'Awq',
                                'weight': {'bit': 8, 'symmetric': False,
                                           'granularity': 'per_channel', 'group_size': -1,
                                           'calib_algo': 'learnable'},
                                'act': {'bit': 8, 'symmetric': False,
                                        'granularity': 'per_token', 'calib_algo': 'minmax'},
                                'special': {'trans': True, 'trans_version': 'v2',
                                            'weight_clip': True, 'clip_version': 'v2',
                                            'save_scale': True, 'save_clip': True}},
                      'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
    'awq_omni_w6a6': {'quant': {'method': 'Awq',
                                'weight': {'bit': 6, 'symmetric': False,
                                           'granularity': 'per_channel', 'group_size': -1,
                                           'calib_algo': 'learnable'},
                                'act': {'bit': 6, 'symmetric': False,
                                        'granularity': 'per_token', 'calib_algo': 'minmax'},
                                'special': {'trans': True, 'trans_version': 'v2',
                                            'weight_clip': True, 'clip_version': 'v2',
                                            'save_scale': True, 'save_clip': True}},
                      'calib': {'bs': -1, 'n_samples': 16, 'seq_len': 128}},
}
