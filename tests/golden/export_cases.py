"""Exporter cases (data only) shared by gen_export.py and tests/test_export.py."""
BASE = {'architectures': ['LlamaForCausalLM'], 'hidden_size': 4096, 'torch_dtype': 'bfloat16',
        'quantization_config': {'quant_method': 'fp8', 'weight_block_size': [128, 128]}}

CASES = {
    'vllm_w4a16_g128_pack': ('vllm', {'quant': {'weight': {
        'bit': 4, 'symmetric': True, 'granularity': 'per_group', 'group_size': 128,
        'need_pack': True}}}),
    'vllm_w8a16_channel': ('vllm', {'quant': {'weight': {
        'bit': 8, 'symmetric': True, 'granularity': 'per_channel'}}}),
    'vllm_w8a8_int_token': ('vllm', {'quant': {
        'weight': {'bit': 8, 'symmetric': True, 'granularity': 'per_channel'},
        'act': {'bit': 8, 'symmetric': True, 'granularity': 'per_token'}}}),
    'vllm_w8a8_int_static': ('vllm', {'quant': {
        'weight': {'bit': 8, 'symmetric': True, 'granularity': 'per_channel'},
        'act': {'bit': 8, 'symmetric': True, 'granularity': 'per_tensor', 'static': True}}}),
    'vllm_fp8_weight_only': ('vllm', {'quant': {'weight': {
        'bit': 'e4m3', 'symmetric': True, 'granularity': 'per_channel',
        'quant_type': 'float-quant'}}}),
    'vllm_fp8_block_dynamic': ('vllm', {'quant': {
        'weight': {'bit': 'e4m3', 'symmetric': True, 'granularity': 'per_block',
                   'block_size': 128, 'quant_type': 'float-quant'},
        'act': {'bit': 'e4m3', 'symmetric': True, 'granularity': 'per_token',
                'quant_type': 'float-quant'}}}),
    'vllm_fp8_static': ('vllm', {'quant': {
        'weight': {'bit': 'e4m3', 'symmetric': True, 'granularity': 'per_tensor',
                   'quant_type': 'float-quant'},
        'act': {'bit': 'e4m3', 'symmetric': True, 'granularity': 'per_tensor',
                'quant_type': 'float-quant', 'static': True}}}),
    'autoawq_w4_g128': ('autoawq', {'quant': {'weight': {
        'bit': 4, 'symmetric': False, 'granularity': 'per_group', 'group_size': 128,
        'pack_version': 'gemm_pack'}}}),
    'autoawq_w4_channel': ('autoawq', {'quant': {'weight': {
        'bit': 4, 'symmetric': False, 'granularity': 'per_channel',
        'pack_version': 'gemv_pack'}}}),
}
