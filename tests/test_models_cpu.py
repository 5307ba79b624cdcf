"""Model adapters on the CPU (no kernels run): each adapter's contract — subsets of every block
(layers, prev_op, input, inspect, flags), block linears, extra modules, layer norms — equals
the reference adapter's on the same tiny model (tests/golden/subsets_<family>.json, written
by gen_pipeline.py from llmc/models/{llama,opt,deepseekv3}.py), and DeepSeek-V3's per-expert
layout computes what transformers' fused experts compute."""
import json

import pytest
import torch

import tiny_models as TM

FAMILIES = ['Llama', 'Opt', 'DeepseekV3']


def _adapter(family, hf_model):
    from lightcompress_amd.pipeline import MODEL_REGISTRY
    return MODEL_REGISTRY[family](hf_model=hf_model, device='cpu')


def _structure(model, block):
    names = {id(m): n for n, m in block.named_modules()}
    out = []
    for sub in model.get_subsets_in_block(block):
        d = {'layers': list(sub['layers']),
             'prev_op': [None if p is None else names[id(p)] for p in sub['prev_op']],
             'input': list(sub['input']), 'inspect': names[id(sub['inspect'])]}
        for k in ('has_kwargs', 'is_mlp', 'do_trans', 'skip_rotate'):
            if k in sub:
                d[k] = sub[k]
        out.append(d)
    return out


@pytest.mark.parametrize('family', FAMILIES)
def test_adapter_contract_matches_reference(family):
    from transformers import AutoModelForCausalLM
    ref = json.loads((TM.HERE / f'subsets_{family}.json').read_text())
    hf = AutoModelForCausalLM.from_pretrained(TM.MODEL_DIRS[family], local_files_only=True)
    model = _adapter(family, hf)
    assert model.block_name_prefix == ref['block_name_prefix']
    assert model.has_bias() == ref['has_bias']
    assert model.skip_layer_name() == ref['skip_layer_name']
    assert len(model.get_blocks()) == len(ref['blocks'])
    n_lin = 0
    for block, rb in zip(model.get_blocks(), ref['blocks']):
        names = {id(m): n for n, m in block.named_modules()}
        assert _structure(model, block) == rb['subsets']
        assert list(model.get_block_linears(block)) == rb['linears']
        assert {k: names[id(v)] for k, v in model.get_extra_modules(block).items()} == rb['extra']
        assert {k: names[id(v)] for k, v in
                model.get_layernorms_in_block(block).items()} == rb['layernorms']
        n_lin += len(rb['linears'])
    assert n_lin == TM.N_LINEARS[family]


def test_dsv3_per_expert_layout_same_forward():
    """unfuse_experts: ExpertList of per-expert MLPs vs transformers' DeepseekV3Experts on the
    same weights (fp32, so the comparison is not hidden by bf16 rounding)."""
    from lightcompress_amd.deepseekv3 import ExpertList, unfuse_experts
    fused = TM.build('DeepseekV3').float().eval()
    ids = torch.randint(0, 128, (2, 64), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        want = fused(input_ids=ids).logits
        per = unfuse_experts(fused)
        moe = per.model.layers[1].mlp
        assert isinstance(moe.experts, ExpertList) and len(moe.experts) == 4
        assert moe.experts[2].gate_proj.weight.shape == (128, 256)
        got = per(input_ids=ids).logits
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)


def test_dsv3_moe_subsets_cover_every_expert():
    """deepseekv3.py:128-167: one MoE subset holding every expert's gate/up, the shared
    expert's and the router, then one down_proj subset per expert and the shared down."""
    from transformers import AutoModelForCausalLM
    hf = AutoModelForCausalLM.from_pretrained(TM.MODEL_DIRS['DeepseekV3'], local_files_only=True)
    model = _adapter('DeepseekV3', hf)
    subs = model.get_subsets_in_block(model.get_blocks()[1])
    moe = [s for s in subs if s['input'] == ['mlp']]
    assert len(moe) == 1 and moe[0]['inspect'] is model.get_blocks()[1].mlp
    assert len(moe[0]['layers']) == 2 * 4 + 2 + 1 and 'mlp.gate' in moe[0]['layers']
    downs = [s for s in subs if list(s['layers'])[0].endswith('down_proj')]
    assert len(downs) == 5
    assert model.get_moe_gate(model.get_blocks()[1]) is not None
    assert model.get_moe_gate(model.get_blocks()[0]) is None


def test_entry_view_unequal_entries():
    """A token shard can cut a calibration entry part-way (_shard_input_tokens), so the
    entries of one stacked forward may differ in batch size: 2-D linear inputs are split back
    per entry by their own row counts (dense: contiguous blocks; routed: by global row index)."""
    from types import SimpleNamespace
    from lightcompress_amd.base_blockwise_quantization import BaseBlockwiseQuantization as B
    counts = [3 * 4, 1 * 4, 2 * 4]  # entries of batch 3, 1, 2 at 4 tokens each
    ctx = SimpleNamespace(_batch_ctx=counts)
    x = torch.arange(sum(counts) * 2, dtype=torch.float32).view(-1, 2)
    dense = B.entry_view(ctx, SimpleNamespace(), x)
    assert [t.shape[0] for t in dense] == counts
    assert torch.equal(torch.cat(dense), x)
    # equal entries keep the [entries, tokens, C] view
    ctx._batch_ctx = [4, 4, 4]
    assert B.entry_view(ctx, SimpleNamespace(), x[:12]).shape == (3, 4, 2)
    # routed rows: global token indices 0..23 over entries [0,12), [12,16), [16,24)
    ctx._batch_ctx = counts
    rows = torch.tensor([20, 1, 13, 11, 15, 23])
    m = SimpleNamespace(_lcq_rows=rows)
    xr = torch.arange(6, dtype=torch.float32).view(6, 1)
    got = B.entry_view(ctx, m, xr)
    assert [t.flatten().tolist() for t in got] == [[1.0, 3.0], [2.0, 4.0], [0.0, 5.0]]
    # no stacked forward: inputs pass unchanged
    ctx._batch_ctx = None
    assert B.entry_view(ctx, m, xr) is xr


def test_batchable_unequal_batches():
    """Entries of equal sample shape stack into one calibration forward even when their batch
    sizes differ (an unequal calibration set, or a token shard that cut an entry), unless a
    kwarg tensor carries a batch dim (it could not follow the stacked batch); a padding mask
    keeps the per-sample loop."""
    from lightcompress_amd.base_blockwise_quantization import _batchable
    rot = (torch.ones(1, 8, 4), torch.zeros(1, 8, 4))
    xs = [torch.zeros(3, 8, 16), torch.zeros(1, 8, 16)]
    assert _batchable(xs, [{'position_embeddings': rot}] * 2)
    assert not _batchable(xs, [{'position_ids': torch.zeros(3, 8)},
                               {'position_ids': torch.zeros(1, 8)}])
    assert not _batchable([torch.zeros(3, 8, 16), torch.zeros(1, 4, 16)],
                          [{'position_embeddings': rot}] * 2)
    eq = [torch.zeros(2, 8, 16), torch.zeros(2, 8, 16)]
    assert _batchable(eq, [{'position_ids': torch.zeros(1, 8)}] * 2)
    assert not _batchable(eq, [{'attention_mask': torch.ones(2, 8)}] * 2)
    assert not _batchable(xs[:1], [{}])


@pytest.mark.parametrize('scaling', [None, 'llama3', 'dynamic'])
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
def test_rotary_kwargs_equal_module(scaling, dtype):
    """Llama.rotary_kwargs builds cos / sin as an elementwise outer product (no K = 1 GEMM
    launch); the values equal LlamaRotaryEmbedding.forward's bit for bit, rope scaling included."""
    from transformers import LlamaConfig
    from lightcompress_amd.llama import Llama
    rs = None if scaling is None else {'rope_type': 'llama3', 'factor': 8.0,
                                       'low_freq_factor': 1.0, 'high_freq_factor': 4.0,
                                       'original_max_position_embeddings': 8192}
    maxpos = 131072
    if scaling == 'dynamic':  # the table depends on seq_len past the original context
        rs, maxpos = {'rope_type': 'dynamic', 'factor': 2.0}, 1024
    cfg = LlamaConfig(hidden_size=256, intermediate_size=512, num_attention_heads=2,
                      num_key_value_heads=1, num_hidden_layers=1, rope_theta=500000.0,
                      max_position_embeddings=maxpos, rope_scaling=rs, torch_dtype=dtype)
    m = Llama.random(cfg, num_layers=1, device=torch.device('cpu'), seed=0)
    m.torch_dtype = dtype
    for S in (64, 2048):
        kw = m.rotary_kwargs(S)
        pos = kw['position_ids']
        c0, s0 = m.rotary_emb(torch.empty(1, S, 1, dtype=dtype), pos)
        c, s = kw['position_embeddings']
        assert c.dtype == dtype and torch.equal(c, c0) and torch.equal(s, s0)


def test_expert_list_grouped_host_logic_matches_loop(monkeypatch):
    """The grouped block-fp8 expert forward's host logic (sort of the token slots by expert,
    row_off, the per-slot token gather a_rows = order // k, gate + up as a SiLU pair, the
    combine in ascending expert order) against the per-expert loop, on the CPU: every device
    kernel is replaced by the oracle restatement (oracle/fp8_ref.py: act_quant, fp8_gemm), so the
    two paths differ only in how rows are grouped and recombined -- the outputs must be equal."""
    from transformers.models.deepseek_v3 import modeling_deepseek_v3 as md

    from lightcompress_amd import deepseekv3, kernel, module_utils, ops
    from lightcompress_amd.deepseekv3 import ExpertList
    from lightcompress_amd.module_utils import LlmcFp8Linear
    from oracle import fp8_ref as O
    E, H, inter, T, k = 6, 256, 128, 40, 3
    g = torch.Generator().manual_seed(3)
    cfg = md.DeepseekV3Config(hidden_size=H, intermediate_size=inter, hidden_act='silu')
    experts = ExpertList()
    for _ in range(E):
        mlp = md.DeepseekV3MLP(cfg, intermediate_size=inter)
        for p in ('gate_proj', 'up_proj', 'down_proj'):
            lin = getattr(mlp, p)
            m = LlmcFp8Linear.new(lin, 128)
            m.weight.data, m.weight_scale_inv.data = O.weight_cast_to_fp8(
                torch.randn(lin.out_features, lin.in_features, generator=g) * 0.05)
            setattr(mlp, p, m)
        experts.append(mlp)
    idx = torch.stack([torch.randperm(E, generator=g)[:k] for _ in range(T)])
    w = torch.rand(T, k, generator=g)
    x = (torch.randn(T, H, generator=g) * 2).to(torch.bfloat16)

    def gemm_rows(a, a_s, b, b_s):   # oracle GEMM, C rounded to bf16 like the fp32 -> bf16 path
        return O.fp8_gemm(a, a_s, b, b_s).to(torch.bfloat16)

    def grouped(a, a_s, row_off, wtab, n, out_dtype, a_rows=None, silu_mul=False):
        K = a.shape[1]
        a_s = a_s.view(-1, K // 128)
        if a_rows is not None:
            a, a_s = a[a_rows], a_s[a_rows]
        sets = [t for t in tables] if wtab.dim() == 3 else [tables_down]
        outs = []
        for ws in sets:
            c = torch.empty(a.shape[0], n, dtype=torch.bfloat16)
            for gi, (b, b_s) in enumerate(ws):
                r0, r1 = int(row_off[gi]), int(row_off[gi + 1])
                if r1 > r0:
                    c[r0:r1] = gemm_rows(a[r0:r1], a_s[r0:r1], b, b_s)
            outs.append(c)
        if silu_mul:
            return torch.nn.functional.silu(outs[0]) * outs[1]
        return outs[0] if len(outs) == 1 else torch.stack(outs)

    def combine(y, slot_row, expert, weights, T_):
        out = torch.zeros(T_, y.shape[1], dtype=torch.bfloat16)
        sr, ex = slot_row.view(T_, -1), expert.view(T_, -1)
        for e in range(E):
            tok, pos = torch.where(ex == e)
            if tok.numel():
                out.index_add_(0, tok, (y[sr[tok, pos]] * weights[tok, pos, None]).to(
                    torch.bfloat16))
        return out

    tables = [[(getattr(m, p).weight.data, getattr(m, p).weight_scale_inv.data) for m in experts]
              for p in ('gate_proj', 'up_proj')]
    tables_down = [(m.down_proj.weight.data, m.down_proj.weight_scale_inv.data) for m in experts]
    monkeypatch.setattr(kernel, 'act_quant', O.act_quant)
    monkeypatch.setattr(ops, 'fp8_gemm_grouped', grouped)
    monkeypatch.setattr(ops, 'moe_combine', combine)
    monkeypatch.setattr(ExpertList, '_fp8_tables', lambda self, dev: (torch.zeros(2, E, 2),
                                                                     torch.zeros(E, 2)))
    monkeypatch.setattr(module_utils, 'block_wise_fp8_forward_func',
                        lambda xx, wt, ws, bs, bias: gemm_rows(*O.act_quant(xx.contiguous()),
                                                               wt, ws))
    assert deepseekv3._mlp_forward() is md.DeepseekV3MLP.forward
    got = experts._forward_grouped_fp8(x, idx, w)
    monkeypatch.setattr(ExpertList, '_grouped_fp8_ok', lambda self, xx: False)
    want = experts(x, idx, w)
    assert got.dtype == want.dtype == torch.bfloat16
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))
