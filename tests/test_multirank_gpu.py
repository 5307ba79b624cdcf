"""Two ranks on one GPU (gloo over device tensors), SURVEY.md §8e: block-sharded AWQ
(quant_out False; deployed to vLLM int4, the other ranks receive the packed shards only),
ratio-grid + clip-row sharded AWQ (quant_out True) and replica GPTQ with a
row-sharded column loop reproduce the single-process result bit for bit (the per-unit math is
identical, only the placement changes); token-sharded GPTQ too (the grouped Hessian sums its
partials in one fixed tree on any world size dividing 8)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model_and_calib(layers, entries=(4,)):
    from transformers import LlamaConfig
    from lightcompress_amd.llama import Llama
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=layers, vocab_size=128,
                      max_position_embeddings=512, rms_norm_eps=1e-5)
    model = Llama.random(cfg, device='cuda:0', seed=3)
    g = torch.Generator(device='cuda:0').manual_seed(9)
    x = torch.randn(sum(entries), 64, 256, generator=g, device='cuda:0').to(torch.bfloat16)
    return model, {'data': list(torch.split(x, list(entries))),
                   'kwargs': [model.rotary_kwargs(64) for _ in entries]}


AWQ = {'calib': {'seq_len': 64},
       'quant': {'method': 'Awq', 'weight': {'bit': 4, 'symmetric': True,
                                             'granularity': 'per_group', 'group_size': 128},
                 'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                             'clip_sym': True}, 'quant_out': False}}
AWQ_OUT = {'calib': {'seq_len': 64},
           'quant': {'method': 'Awq', 'weight': {'bit': 4, 'symmetric': False,
                                                 'granularity': 'per_group', 'group_size': 128},
                     'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                 'clip_sym': False}, 'quant_out': True}}
GPTQ_SPECIAL = {'actorder': True, 'static_groups': False, 'percdamp': 0.01, 'blocksize': 128,
                'true_sequential': True}
GPTQ = {'quant': {'method': 'GPTQ', 'weight': {'bit': 4, 'symmetric': False,
                                               'granularity': 'per_group', 'group_size': 128},
                  'special': dict(GPTQ_SPECIAL, parallel='replicate'), 'quant_out': True}}
GPTQ_TOK = {'quant': {'method': 'GPTQ', 'weight': {'bit': 4, 'symmetric': False,
                                                   'granularity': 'per_group', 'group_size': 128},
                      'special': dict(GPTQ_SPECIAL), 'quant_out': True},
            'deploy': 'fake_quant'}
# token sharding with every Hessian built from float inputs (no quant_out, no
# true_sequential rehooks): each layer's H differs from one GPU only in its fp32 summation order
GPTQ_TOK_FLOAT = {'quant': {'method': 'GPTQ',
                            'weight': {'bit': 4, 'symmetric': False, 'granularity': 'per_group',
                                       'group_size': 128},
                            'special': dict(GPTQ_SPECIAL, true_sequential=False,
                                            parallel='shard_tokens'),
                            'quant_out': False},
                  'deploy': 'fake_quant'}


def _run(cfg_dict, layers):
    from lightcompress_amd import gptq_core
    model, calib = _model_and_calib(layers, cfg_dict.get('entries', (4,)))
    old_min = gptq_core.SHARD_MIN_ROWS
    if 'chain_shard_min' in cfg_dict:   # the tiny Hessians (256, 512) take the split path too
        gptq_core.SHARD_MIN_ROWS = cfg_dict['chain_shard_min']
    try:
        return _run_algo(cfg_dict, model, calib)
    finally:
        gptq_core.SHARD_MIN_ROWS = old_min


def _run_algo(cfg_dict, model, calib):
    from lightcompress_amd import gptq_core
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    split0 = gptq_core.shard_stats['split_products']
    cfg_dict = {k: v for k, v in cfg_dict.items() if k not in ('entries', 'chain_shard_min')}
    algo = build_algo(model, load_config(cfg_dict), calib)
    algo.run_block_loop()
    if cfg_dict.get('deploy'):
        algo.deploy(cfg_dict['deploy'])
    else:  # shard_blocks publishes the transformed float blocks on demand
        algo.materialize_blocks()
    if cfg_dict.get('deploy') == 'vllm_quant':  # every buffer of every block (codes, scales,
        return {f'{i}.{n}': t.detach().cpu()   # norms) as the rank holds it after the gather
                for i, b in enumerate(model.blocks)
                for n, t in [*b.named_parameters(), *b.named_buffers()]}
    out = {f'{i}.{n}': m.weight.detach().float().cpu()
           for i, b in enumerate(model.blocks) for n, m in model.get_block_linears(b).items()}
    out.update({f'{i}.{n}.{bn}': t.detach().float().cpu()   # static act qparams
                for i, b in enumerate(model.blocks) for n, m in model.get_block_linears(b).items()
                for bn, t in m.named_buffers() if bn.startswith('buf_act_')})
    out['_stats.split_products'] = torch.tensor(
        [gptq_core.shard_stats['split_products'] - split0])
    return out


def _worker(rank, world, port, cfg, layers, path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK='0')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        out = _run(cfg, layers)
        if rank == 0:
            torch.save(out, path)
    finally:
        dist.destroy_process_group()


def _two_ranks(cfg, layers, tmp_path):
    ctx = mp.get_context('spawn')
    port = _port()
    path = str(tmp_path / 'rank0.pt')
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, layers, path))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return torch.load(path, weights_only=True)


AWQ_VLLM = dict(AWQ, deploy='vllm_quant')


@pytest.mark.parametrize('name,cfg,layers', [('awq_shard_blocks', AWQ, 4),
                                             ('awq_shard_blocks_vllm', AWQ_VLLM, 4),
                                             ('awq_shard_search', AWQ_OUT, 2),
                                             ('gptq_replicate_rows', GPTQ, 2)])
def test_two_ranks_match_single(dev, name, cfg, layers, tmp_path):
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    single = _run(cfg, layers)
    multi = _two_ranks(cfg, layers, tmp_path)
    assert single.keys() == multi.keys()
    for k in single:
        if k.startswith('_stats.'):
            continue
        assert single[k].dtype == multi[k].dtype, k
        assert torch.equal(single[k], multi[k]), k


def _codes_vs_single(cfg, tmp_path):
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    single = _run(cfg, 2)
    multi = _two_ranks(cfg, 2, tmp_path)
    assert single.keys() == multi.keys()
    eq = {k: (single[k] == multi[k]).float().mean().item() for k in single}
    rel = {k: ((single[k] - multi[k]).norm() / single[k].norm()).item() for k in single}
    for k in single:
        print(f'{k:28s} equal {eq[k] * 100:7.3f} %  rel |dW| {rel[k]:.2e}')
    return eq, rel


@pytest.mark.parametrize('name,cfg', [('float_inputs', GPTQ_TOK_FLOAT), ('quant_out', GPTQ_TOK),
                                      ('quant_out_split_chain', dict(GPTQ_TOK, chain_shard_min=128))])
def test_gptq_token_shards_bit_identical(dev, name, cfg, tmp_path):
    """Each rank forwards its half of the calibration samples (cut on the grouped Hessian's
    group boundaries); every Hessian is the same fixed tree of 8 group partials
    (gptq_core.HessianAccumulator), finished across the ranks, so H -- hence U, the row-sharded
    column loop and every deployed weight -- equals one GPU's bit for bit, with float inputs
    and under quant_out + true_sequential (gptq_w_only.yml) alike. With chain_shard_min the
    factorisation's products of >= 128 rows are row-split over the two ranks
    (gptq_core.chain_sharding): still bit for bit."""
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    single = _run(cfg, 2)
    multi = _two_ranks(cfg, 2, tmp_path)
    assert single.keys() == multi.keys()
    assert int(single['_stats.split_products']) == 0
    if 'chain_shard_min' in cfg:
        assert int(multi['_stats.split_products']) > 0   # the launch list shows the split
    for k in single:
        if not k.startswith('_stats.'):
            assert torch.equal(single[k], multi[k]), k


def _static_act(entries, algo):
    q = {k: dict(v) if isinstance(v, dict) else v for k, v in GPTQ_TOK_FLOAT['quant'].items()}
    q['act'] = {'bit': 8, 'symmetric': algo != 'static_moving_minmax', 'granularity': 'per_tensor',
                'static': True, 'calib_algo': algo}
    return {'quant': q, 'deploy': 'fake_quant', 'entries': entries}


@pytest.mark.parametrize('entries,algo', [((4,), 'static_minmax'),
                                          ((3, 1), 'static_minmax'),
                                          ((1, 2, 1), 'static_moving_minmax')])
def test_static_act_qparams_token_shards_bit_identical(dev, entries, algo, tmp_path):
    """Static per-tensor activation calibration (register_act_qparams,
    base_blockwise_quantization.py:567-588) under shard_tokens: per-sample (min, max) gathered
    in global order and folded into the reference's segments (samples of one batch, or entries
    -- (3, 1) cuts entry 0 between the ranks), so buf_act_* and every GPTQ weight equal one
    GPU's."""
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    cfg = _static_act(entries, algo)
    single = _run(cfg, 2)
    assert any('buf_act_scales_0' in k for k in single)
    multi = _two_ranks(cfg, 2, tmp_path)
    assert single.keys() == multi.keys()
    for k in single:
        if not k.startswith('_stats.'):
            assert torch.equal(single[k], multi[k]), k


def _chain_worker(rank, world, port, n, path, x6):
    from lightcompress_amd import gptq_core, ops
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK='0')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        gptq_core.SHARD_MIN_ROWS = 256
        x6_split = []
        if x6:
            ops.X6_MIN_TILES = 1
            real = ops.gemm_f32x6

            def spy(A, B, out, alpha, beta, b_trans, row0=0, row1=None, **kw):
                if row1 is not None and row1 - row0 < out.shape[0]:
                    x6_split.append((out.shape[0], row0, row1))
                return real(A, B, out, alpha, beta, b_trans, row0, row1, **kw)
            ops.gemm_f32x6 = spy
        H = torch.load(path + '.H', weights_only=True).to('cuda:0')
        with gptq_core.chain_sharding(rank, world):
            U = gptq_core.inverse_cholesky_upper(H)
        torch.save({'U': U.cpu(), 'split': gptq_core.shard_stats['split_products'],
                    'x6_split': len(x6_split)}, f'{path}.{rank}')
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('n,x6', [(1536, False), (2304, True)])
def test_chain_row_split_bit_identical(dev, tmp_path, n, x6):
    """gptq_core.chain_sharding: every product of >= 256 output rows is computed by each rank
    for its rows only (the full shape's kernel plan: lcq_gemm_f32_rows, or with x6 the
    split-plane lcq_gemm_f32x6 row ranges, K split by the full shape and folded per row range)
    and all-gathered in rank order; U equals the one-process chain (same products, unsplit) bit
    for bit on both ranks. n 2304 with X6_MIN_TILES 1 puts the K >= 1024 products on x6."""
    from lightcompress_amd import gptq_core, ops
    g = torch.Generator().manual_seed(3)
    X = torch.randn(n, 2 * n, generator=g)
    H = X @ X.T / (2 * n)
    H.diagonal().add_(0.05)
    path = str(tmp_path / 'chain')
    torch.save(H, path + '.H')
    old = gptq_core.SHARD_MIN_ROWS, ops.X6_MIN_TILES
    try:
        gptq_core.SHARD_MIN_ROWS = 256
        if x6:
            ops.X6_MIN_TILES = 1
        single = gptq_core.inverse_cholesky_upper(H.to(dev)).cpu()
    finally:
        gptq_core.SHARD_MIN_ROWS, ops.X6_MIN_TILES = old
        gptq_core.clear_chain_graphs()   # captured under the probe thresholds
    ctx = mp.get_context('spawn')
    port = _port()
    procs = [ctx.Process(target=_chain_worker, args=(r, 2, port, n, path, x6))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    for r in range(2):
        res = torch.load(f'{path}.{r}', weights_only=True)
        assert res['split'] > 0
        if x6:
            assert res['x6_split'] > 0, 'no row-split product reached lcq_gemm_f32x6'
        assert torch.equal(res['U'], single), r


def _owned_awq_run(materialize):
    from transformers import LlamaConfig

    from lightcompress_amd.llama import Llama
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                      num_key_value_heads=2, num_hidden_layers=4, vocab_size=128,
                      max_position_embeddings=512, rms_norm_eps=1e-5)
    conf = load_config(dict(AWQ, model={'type': 'Llama', 'materialize': materialize}))
    model = Llama(conf, hf_config=cfg, random_init={'seed': 3, 'std': 0.02}, device='cuda:0')
    g = torch.Generator(device='cuda:0').manual_seed(9)
    x = torch.randn(4, 64, 256, generator=g, device='cuda:0').to(torch.bfloat16)
    algo = build_algo(model, conf, {'data': [x], 'kwargs': [model.rotary_kwargs(64)]})
    algo.run_block_loop()
    algo.deploy('vllm_quant')
    return {f'{i}.{n}': t.detach().cpu() for i, b in enumerate(model.get_blocks())
            for n, t in [*b.named_parameters(), *b.named_buffers()] if not t.is_meta}


def _owned_awq_worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK='0')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.save(_owned_awq_run('owned'), f'{path}.{rank}')
    finally:
        dist.destroy_process_group()


def test_awq_shard_blocks_owned_matches_single(dev, tmp_path):
    """bench.py --gpus N's AWQ leg: shard_blocks with materialize: owned (a synthetic
    random_init model whose tensors are seeded by name) -- each rank allocates, transforms and
    vLLM-packs only its own blocks (ring hand-off of the activations, no weight gather); every
    tensor a rank holds equals the one-process run's, and the ranks together hold every block."""
    for k in ('RANK', 'WORLD_SIZE'):
        os.environ.pop(k, None)
    single = _owned_awq_run('all')
    ctx = mp.get_context('spawn')
    port = _port()
    path = str(tmp_path / 'owned')
    procs = [ctx.Process(target=_owned_awq_worker, args=(r, 2, port, path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    held = set()
    for r in range(2):
        res = torch.load(f'{path}.{r}', weights_only=True)
        blocks = {int(k.split('.')[0]) for k in res}
        assert blocks == {i for i in range(4) if i % 2 == r}, (r, blocks)
        for k, v in res.items():
            assert v.dtype == single[k].dtype and torch.equal(v, single[k]), k
        held |= set(res)
    assert held == set(single)
