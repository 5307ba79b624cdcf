"""End-to-end plugin pipeline on a tiny random Llama (2 blocks) on the GPU: Awq (+clip),
GPTQ (act-order, true_sequential, quant_out) and RTN through run_block_loop + deploy, with the
reference's YAML config schema."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def tiny_model(dev, layers=2):
    from transformers import LlamaConfig
    from lightcompress_amd.llama import Llama
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=layers, vocab_size=128,
                      max_position_embeddings=512, rms_norm_eps=1e-5)
    return Llama.random(cfg, device=dev, seed=1)


def calib(model, n=4, seq=64, seed=0):
    g = torch.Generator(device=model.blocks[0].self_attn.q_proj.weight.device).manual_seed(seed)
    dev = model.blocks[0].self_attn.q_proj.weight.device
    x = torch.randn(n, seq, model.model_config.hidden_size, generator=g, device=dev)
    return {'data': [x.to(torch.bfloat16)], 'kwargs': [model.rotary_kwargs(seq)]}


AWQ_CFG = {'calib': {'seq_len': 64},
           'quant': {'method': 'Awq', 'weight': {'bit': 4, 'symmetric': True,
                                                 'granularity': 'per_group', 'group_size': 128},
                     'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                 'clip_sym': True}, 'quant_out': True}}

GPTQ_CFG = {'quant': {'method': 'GPTQ', 'weight': {'bit': 4, 'symmetric': False,
                                                   'granularity': 'per_group',
                                                   'group_size': 128},
                      'special': {'actorder': True, 'static_groups': False, 'percdamp': 0.01,
                                  'blocksize': 128, 'true_sequential': True},
                      'quant_out': True}}

GPTQ_SG_CFG = copy.deepcopy(GPTQ_CFG)
GPTQ_SG_CFG['quant']['special']['static_groups'] = True
GPTQ_OWQ_CFG = copy.deepcopy(GPTQ_CFG)  # configs/quantization/methods/GPTQ/gptq_owq_w_only.yml
GPTQ_OWQ_CFG['quant']['special'].update(owq=True, actorder=False, n_outs=[6, 6, 6, 6, 2, 2, 6])
AWQ_V1_CFG = copy.deepcopy(AWQ_CFG)  # backend/*/w4a16_combin/step_1_awq.yml
AWQ_V1_CFG['quant']['special']['trans_version'] = 'v1'


@pytest.mark.parametrize('cfg', [AWQ_CFG, GPTQ_CFG, GPTQ_SG_CFG, GPTQ_OWQ_CFG, AWQ_V1_CFG],
                         ids=['awq', 'gptq', 'gptq_static', 'gptq_owq', 'awq_v1'])
def test_pipeline_runs_and_deploys(dev, cfg):
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    model = tiny_model(dev)
    config = load_config(cfg)
    algo = build_algo(model, config, calib(model))
    algo.run_block_loop()
    for b in model.blocks:
        for n, m in model.get_block_linears(b).items():
            assert torch.isfinite(m.weight).all(), n
    algo.deploy('fake_quant')
    x = torch.randn(2, 16, 256, device=dev, dtype=torch.bfloat16)
    kw = model.rotary_kwargs(16)
    y = model.blocks[0](x, **kw)
    y = y[0] if isinstance(y, tuple) else y
    assert torch.isfinite(y).all()
    # deployed fake-quant weights take at most 16 values per 128-group (groups live in the
    # act-order permuted column space for GPTQ, in the original one with static_groups)
    m = model.blocks[0].mlp.down_proj
    w = m.weight.float()
    if getattr(algo, 'owq', False):  # outlier columns stay float: check the others
        w = w[:, m.buf_perm][:, :int(m.buf_n_nonout) // 128 * 128]
    elif hasattr(m, 'buf_perm') and not getattr(algo, 'static_groups', False):
        w = w[:, m.buf_perm]
    w = w.reshape(-1, 128)
    assert max(len(torch.unique(r)) for r in w[:64]) <= 16


def test_awq_vllm_pack_deploy(dev):
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    cfg = {**AWQ_CFG, 'quant': {**AWQ_CFG['quant'],
                                'weight': {**AWQ_CFG['quant']['weight'], 'need_pack': True}}}
    model = tiny_model(dev)
    algo = build_algo(model, load_config(cfg), calib(model))
    algo.run_block_loop()
    algo.deploy('vllm_quant')
    m = model.blocks[0].mlp.gate_proj
    assert m.weight_packed.dtype == torch.int32 and m.weight_packed.shape == (512, 256 // 8)
    assert m.weight_scale.dtype == torch.float16 and m.weight_scale.shape == (512, 2)


def test_rtn_autoawq_deploy(dev):
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    cfg = {'quant': {'method': 'RTN', 'weight': {'bit': 4, 'symmetric': False,
                                                 'granularity': 'per_group', 'group_size': 128,
                                                 'pack_version': 'gemm_pack'}}}
    model = tiny_model(dev)
    algo = build_algo(model, load_config(cfg), None)
    algo.run_block_loop()
    algo.deploy('autoawq_quant')
    m = model.blocks[1].self_attn.o_proj
    assert m.qweight.shape == (256, 256 // 8) and m.scales.dtype == torch.float16


@pytest.mark.parametrize('quant_out', [False, True])
def test_awq_org_output_reuse_is_bit_identical(dev, quant_out):
    """Reusing the capture forward's inspect outputs as the search's original outputs gives
    the same losses, scales and deployed weights as recomputing them (awq.py:204-206)."""
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    import copy
    cfg = copy.deepcopy(AWQ_CFG)
    cfg['quant']['quant_out'] = quant_out
    results = []
    for reuse in (True, False):
        model = tiny_model(dev)
        algo = build_algo(model, load_config(copy.deepcopy(cfg)), calib(model))
        algo.reuse_org = reuse
        losses = []
        orig = algo.search_scale_subset

        def rec(*a, _o=orig, **k):
            r = _o(*a, **k)
            losses.append(list(algo.last_search['losses']))
            return r
        algo.search_scale_subset = rec
        algo.run_block_loop()
        algo.deploy('fake_quant')
        w = [m.weight.detach().clone() for b in model.blocks
             for m in model.get_block_linears(b).values()]
        results.append((losses, w, dict(algo.org_reuse_stats)))
    (l1, w1, st1), (l0, w0, st0) = results
    assert st1['reused'] == 3 * len(w1) // 7 and st0['reused'] == 0
    assert l1 == l0
    assert all(torch.equal(a.view(torch.int16), b.view(torch.int16)) for a, b in zip(w1, w0))


@pytest.mark.parametrize('target', ['save_vllm', 'save_autoawq'])
def test_save_quantized_checkpoint(dev, tmp_path, target):
    """__main__.py:96-160 real-quant save flow: deploy + safetensors + serving config."""
    import json
    from safetensors import safe_open
    from lightcompress_amd.export import save_quantized
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    sym = target == 'save_vllm'
    w = {'bit': 4, 'symmetric': sym, 'granularity': 'per_group', 'group_size': 128}
    if sym:
        w['need_pack'] = True
    else:
        w['pack_version'] = 'gemm_pack'
    cfg = load_config({'quant': {'method': 'RTN', 'weight': w}, 'save': {target: True}})
    model = tiny_model(dev)
    algo = build_algo(model, cfg, None)
    algo.run_block_loop()
    save_quantized(algo, cfg, str(tmp_path))
    conf = json.loads((tmp_path / 'config.json').read_text())
    keys = []
    for f in tmp_path.glob('*.safetensors'):
        with safe_open(str(f), 'pt') as fh:
            keys += list(fh.keys())
    if sym:
        assert conf['compression_config']['format'] == 'pack-quantized'
        assert any(k.endswith('q_proj.weight_packed') for k in keys)
        assert any(k.endswith('q_proj.weight_scale') for k in keys)
    else:
        assert conf['quantization_config']['quant_method'] == 'awq'
        assert any(k.endswith('q_proj.qweight') for k in keys)
        assert any(k.endswith('q_proj.qzeros') for k in keys)


@pytest.mark.parametrize('static', [False, True], ids=['dynamic', 'static_groups'])
def test_gptq_concatenated_rows_bit_identical(dev, static):
    """q/k/v (and gate/up) quantized as one column loop over their concatenated rows give the
    same weights and qparams, bit for bit, as one loop per linear."""
    from lightcompress_amd.gptq import GPTQ
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    out = []
    for concat in (True, False):
        model = tiny_model(dev)
        algo = build_algo(model, load_config(copy.deepcopy(GPTQ_SG_CFG if static else GPTQ_CFG)),
                          calib(model))
        algo.concat_rows = concat
        algo.run_block_loop()
        st = {}
        for bi, b in enumerate(model.blocks):
            for n, m in model.get_block_linears(b).items():
                st[f'{bi}.{n}.w'] = m.weight.detach().clone()
                st[f'{bi}.{n}.s'] = m.buf_scales.detach().clone()
                st[f'{bi}.{n}.z'] = m.buf_zeros.detach().clone()
        out.append(st)
    assert GPTQ.concat_rows  # the default path is the concatenated one
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k
