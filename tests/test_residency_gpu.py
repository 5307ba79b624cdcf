"""Block residency on the GPU (lightcompress_amd/residency.py):

* ``residency: stream`` -- the model stays in pinned host memory and every block passes
  through HBM (upload of block i + 1 on a side stream while block i is transformed): the
  deployed weights are bit-identical to the HBM-resident run for RTN, AWQ, GPTQ (tiny Llama
  goldens) and DeepSeek-V3 AWQ;
* ``shard_units`` (data-free): two ranks on one GPU (gloo over device
  tensors) each real-quant + pack their LPT share of the linears -- DeepSeek-V3 experts
  EP-style -- and publish the packed shards: every block tensor equals one process's, for
  OPT RTN w8 (BASELINE config 1's recipe) and the rtn_w_only_dsv3 recipe on a block-fp8
  DeepSeek-V3 checkpoint;
* ``materialize: owned``: the non-owned units are never allocated on a rank, and the per-rank
  sharded save equals the one-process save."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pipeline_helpers as P
import tiny_models as TM

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', ['rtn', 'awq', 'gptq', 'dsv3_awq'])
def test_stream_bit_identical_to_resident(dev, name):
    _, res, _ = P.run_ours(name, dev, model_override={'residency': 'device'})
    _, got, _, model = P.run_ours(name, dev, model_override={'residency': 'stream'},
                                  return_model=True)
    st = model.streamer
    assert st is not None
    n = len(model.get_blocks())
    # every block went through HBM (deploy at least), uploads were prefetched
    assert st.stats['fetches'] >= n and st.stats['h2d_bytes'] > 0, st.stats
    if name != 'rtn':
        assert st.stats['prefetched'] >= 1, st.stats
    if name == 'gptq':
        # the fake-quant deploy built every block's modules on the host from the
        # FakeQuantLinear memos (no block went through HBM for it): same bits as the resident
        # run's w_qdq at deploy
        assert st.stats['host_deployed_modules'] == 7 * n, st.stats
    # and is back on the host, pinned
    for b in model.get_blocks():
        for t in [*b.parameters(), *b.buffers()]:
            assert t.device.type == 'cpu' and t.is_pinned()
    assert res.keys() == got.keys()
    for k in res:
        assert res[k].dtype == got[k].dtype and torch.equal(res[k], got[k]), k


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fp8_checkpoint(dst):
    """The tiny DeepSeek-V3 golden as a block-fp8 checkpoint (e4m3 block linears with
    128 x 128 weight_scale_inv, kernel.py:57-81 restated by the oracle), the layout of the
    real DeepSeek-V3 checkpoints rtn_w_only_dsv3.yml loads."""
    from safetensors.torch import load_file, save_file

    from oracle import fp8_ref
    src = TM.MODEL_DIRS['DeepseekV3']
    sd = load_file(str(src / 'model.safetensors'))
    out = {}
    for k, t in sd.items():
        if (k.startswith('model.layers.') and k.endswith('.weight') and t.dim() == 2
                and not k.endswith('mlp.gate.weight')):   # every block linear, not the router
            q, s = fp8_ref.weight_cast_to_fp8(t, 128)
            out[k] = q
            out[k.replace('.weight', '.weight_scale_inv')] = s
        else:
            out[k] = t
    os.makedirs(dst, exist_ok=True)
    save_file(out, os.path.join(dst, 'model.safetensors'), metadata={'format': 'pt'})
    cfg = json.load(open(src / 'config.json'))
    cfg['quantization_config'] = {'quant_method': 'fp8', 'fmt': 'e4m3',
                                  'activation_scheme': 'dynamic',
                                  'weight_block_size': [128, 128]}
    json.dump(cfg, open(os.path.join(dst, 'config.json'), 'w'))
    return dst


RECIPES = {
    # BASELINE config 1's quantization on the tiny OPT: w8 per-channel sym, vLLM layout
    'opt_rtn_w8': ({'type': 'Opt', 'path': str(TM.MODEL_DIRS['Opt']), 'torch_dtype': 'float16'},
                   {'method': 'RTN', 'weight': {'bit': 8, 'symmetric': True,
                                                'granularity': 'per_channel'}},
                   'vllm_quant'),
    # configs/quantization/deepseekv3/rtn_w_only_dsv3.yml: block-fp8 checkpoint, int4 asym
    # g64, AutoAWQ gemm pack
    'dsv3_rtn_w_only': ({'type': 'DeepseekV3', 'path': None,
                         'torch_dtype': 'torch.float8_e4m3fn', 'block_wise_quant': True},
                        {'method': 'RTN', 'weight': {'bit': 4, 'symmetric': False,
                                                     'granularity': 'per_group',
                                                     'group_size': 64,
                                                     'pack_version': 'gemm_pack'}},
                        'autoawq_quant'),
    # data-free W8A8 dynamic (per-channel weights, per-token activations) deployed as
    # fake_quant: the published modules must carry a_qdq (forward checked below)
    'opt_rtn_w8a8_fake': ({'type': 'Opt', 'path': str(TM.MODEL_DIRS['Opt']),
                           'torch_dtype': 'float16'},
                          {'method': 'RTN', 'weight': {'bit': 8, 'symmetric': True,
                                                       'granularity': 'per_channel'},
                           'act': {'bit': 8, 'symmetric': True, 'granularity': 'per_token'}},
                          'fake_quant'),
}


def _run_recipe(name, fp8_dir, materialize='all', save=None):
    from lightcompress_amd.pipeline import build_algo, build_model
    from lightcompress_amd.utils import load_config
    mcfg, q, fmt = RECIPES[name]
    mcfg = dict(mcfg, materialize=materialize, residency='device')
    if mcfg['path'] is None:
        mcfg['path'] = fp8_dir
    config = load_config({'model': mcfg, 'quant': q})
    model = build_model(config, device='cuda:0')
    never = []
    if model.ownership is not None:   # what this rank does not own is not allocated
        for bi, b in enumerate(model.get_blocks()):
            lins = set(model.get_block_linears(b))
            for n, t in [*b.named_parameters(), *b.named_buffers()]:
                if not model.ownership.owns_block_tensor(bi, n, lins):
                    assert t.is_meta, n
                    never.append(f'{bi}.{n}')
    algo = build_algo(model, config, None)
    algo.run_block_loop()
    algo.deploy(fmt)
    if save:
        algo.save_model(save)
    out = {f'{i}.{n}': t.detach().cpu() for i, b in enumerate(model.get_blocks())
           for n, t in [*b.named_parameters(), *b.named_buffers()] if not t.is_meta}
    if fmt == 'fake_quant':   # a forward through every deployed linear (act fake quant too)
        g = torch.Generator(device='cuda:0').manual_seed(1)
        for i, b in enumerate(model.get_blocks()):
            for n, m in model.get_block_linears(b).items():
                x = torch.randn(5, m.in_features, generator=g, device='cuda:0').to(m.weight.dtype)
                out[f'fwd.{i}.{n}'] = m(x).detach().cpu()
    return out, never


def _worker(rank, world, port, name, fp8_dir, materialize, save, path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK='0')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        out, never = _run_recipe(name, fp8_dir, materialize, save)
        torch.save({'out': out, 'never': never}, f'{path}.{rank}')
    finally:
        dist.destroy_process_group()


def _two_ranks(name, fp8_dir, tmp_path, materialize='all', save=None):
    ctx = mp.get_context('spawn')
    port = _port()
    path = str(tmp_path / f'{name}_{materialize}')
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, fp8_dir, materialize, save,
                                                path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return [torch.load(f'{path}.{r}', weights_only=True) for r in range(2)]


@pytest.mark.parametrize('name', ['opt_rtn_w8', 'dsv3_rtn_w_only', 'opt_rtn_w8a8_fake'])
def test_shard_units_two_ranks_match_single(dev, name, tmp_path):
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    fp8_dir = _fp8_checkpoint(str(tmp_path / 'dsv3_fp8'))
    single, _ = _run_recipe(name, fp8_dir)
    if name.endswith('_fake'):
        assert any(k.startswith('fwd.') for k in single)
    else:
        assert any(k.endswith(('weight', 'weight_packed', 'qweight')) and
                   v.dtype in (torch.int8, torch.int32) for k, v in single.items())
    for res in _two_ranks(name, fp8_dir, tmp_path):
        multi = res['out']
        assert single.keys() == multi.keys()
        for k in single:
            assert single[k].dtype == multi[k].dtype, k
            assert torch.equal(single[k], multi[k]), k


def test_owned_sharded_save_matches_single(dev, tmp_path):
    from safetensors.torch import load_file
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    fp8_dir = _fp8_checkpoint(str(tmp_path / 'dsv3_fp8'))
    one, two = str(tmp_path / 'one'), str(tmp_path / 'two')
    _run_recipe('dsv3_rtn_w_only', fp8_dir, save=one)
    res = _two_ranks('dsv3_rtn_w_only', fp8_dir, tmp_path, materialize='owned', save=two)
    # each rank skipped the other's units: disjoint, and together every routed expert
    assert res[0]['never'] and res[1]['never']
    assert not set(res[0]['never']) & set(res[1]['never'])
    a = load_file(os.path.join(one, 'model.safetensors'))
    b = {}
    for f in sorted(os.listdir(two)):
        if f.endswith('.safetensors'):
            b.update(load_file(os.path.join(two, f)))
    assert sorted(a) == sorted(b)
    for k in a:
        assert a[k].dtype == b[k].dtype and torch.equal(a[k], b[k]), k


def test_stream_bounds_device_memory(dev):
    """``residency: stream`` keeps at most ~3 blocks in HBM (the one being transformed, the
    next one arriving, the previous one leaving: residency.py), so over the same AWQ run +
    vLLM deploy its device-memory peak above the post-load footprint must undercut the
    HBM-resident run's peak by at least (model bytes - 3 blocks): the reference's
    block.cuda() / block.cpu() bound (base_blockwise_quantization.py:397, 418)."""
    import gc

    from transformers import LlamaConfig

    from lightcompress_amd.llama import Llama
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    cfg = LlamaConfig(hidden_size=512, intermediate_size=2048, num_attention_heads=8,
                      num_key_value_heads=4, num_hidden_layers=12, vocab_size=128,
                      max_position_embeddings=512, rms_norm_eps=1e-5)
    conf = load_config({'calib': {'seq_len': 64},
                        'quant': {'method': 'Awq',
                                  'weight': {'bit': 4, 'symmetric': True,
                                             'granularity': 'per_group', 'group_size': 128,
                                             'need_pack': True},
                                  'special': {'trans': True, 'trans_version': 'v2',
                                              'weight_clip': True, 'clip_sym': True},
                                  'quant_out': False}})

    def run(residency):
        model = Llama.random(cfg, device=dev, seed=3, residency=residency)
        blocks = model.get_blocks()
        block_bytes = sum(t.numel() * t.element_size()
                          for t in [*blocks[0].parameters(), *blocks[0].buffers()])
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        start = torch.cuda.memory_allocated(dev)
        torch.cuda.reset_peak_memory_stats(dev)
        g = torch.Generator(device=dev).manual_seed(9)
        x = torch.randn(4, 64, 512, generator=g, device=dev).to(torch.bfloat16)
        algo = build_algo(model, conf, {'data': [x], 'kwargs': [model.rotary_kwargs(64)]})
        algo.run_block_loop()
        algo.deploy('vllm_quant')
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated(dev)
        algo.release()
        del algo, x
        return start, peak, block_bytes, len(blocks), model

    s_dev, p_dev, bb, n, m_dev = run('device')
    del m_dev
    s_str, p_str, _, _, m_str = run('stream')
    assert m_str.streamer is not None
    model_bytes = n * bb
    assert s_dev - s_str >= model_bytes - bb, (s_dev, s_str, model_bytes)  # blocks on the host
    assert p_str <= p_dev - (model_bytes - 3 * bb), (p_str, p_dev, model_bytes, bb)
