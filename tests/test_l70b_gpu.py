"""Llama-3-70B shapes (BASELINE.json configs[3]: hidden 8192, MLP 28672, 64q / 8kv heads) on
one GPU, checked through properties that hold at any size:

* the down_proj Hessian (IC 28672) against fp64 on a sample of its rows, exactly symmetric;
* the GPTQ column loop at 8192 x 28672 (act-order, g128): every column within half a step of
  its group's grid and a smaller GPTQ objective tr((W-Q) H (W-Q)^T) than round-to-nearest;
* a whole AWQ block: the fused-GEMM search (projection GEMMs with SiLU / loss epilogues at
  K = 28672) against the same search on torch's GEMMs (hipBLASLt) — same loss curves to the
  bf16-output level, the same ratios (or a near tie), and deployed weights that agree
  (measured: identical, both GEMMs accumulate every output in fp32 in ascending K order).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

H70, I70 = 8192, 28672


def _acts(n, ic, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    mag = torch.exp(torch.randn(ic, generator=g, device=dev))
    return (torch.randn(n, ic, generator=g, device=dev) * mag).to(torch.bfloat16)


def test_l70b_down_proj_hessian_vs_fp64(dev):
    from lightcompress_amd.gptq_core import HessianAccumulator
    acc = HessianAccumulator(I70, dev)
    xs = [_acts(1024, I70, dev, s) for s in (1, 2)]
    for x in xs:
        acc.add_batch(x.unsqueeze(0))
    H = acc.H
    assert acc.nsamples == 2
    assert torch.equal(H, H.t())
    x = torch.cat(xs).double()
    idx = torch.randperm(I70, generator=torch.Generator().manual_seed(0))[:192].to(dev)
    xi = x[:, idx]
    ref = (2.0 / 2) * (xi.t() @ x)            # H = 2/nsamples * sum x x^T (gptq.py:286-295)
    bound = (xi.abs().t() @ x.abs())
    err = (H[idx].double() - ref).abs()
    assert (err <= 2e-6 * bound + 1e-30).all(), (err / bound).max().item()


def test_l70b_down_proj_gptq_column_loop(dev):
    from lightcompress_amd import gptq_core
    from lightcompress_amd.gptq_core import HessianAccumulator
    from lightcompress_amd.quant import IntegerQuantizer
    g = torch.Generator(device=dev).manual_seed(7)
    W = (torch.randn(H70, I70, generator=g, device=dev) * 0.02).to(torch.bfloat16)
    acc = HessianAccumulator(I70, dev)
    acc.add_batch(_acts(4096, I70, dev, 3).unsqueeze(0))
    Hc = acc.H.clone()
    wq = IntegerQuantizer(4, False, 'per_group', group_size=128)
    r = gptq_core.quantize_layer(W, acc.H, wq, actorder=True, percdamp=0.01)
    Wg = r['weight'].float()       # error-compensated weight; deploy quantizes it with (s, z)
    assert Wg.shape == W.shape and torch.isfinite(Wg).all()
    # group of original column j = invperm[j] // 128 (act-order groups, gptq.py:206-214)
    inv = r['invperm']
    s = r['scales'].view(H70, -1)
    z = r['zeros'].view(H70, -1)
    grp = (inv // 128).long()
    sc, zc = s[:, grp], z[:, grp]
    codes = torch.clamp(torch.round(Wg / sc) + zc, 0, 15)
    Q = (codes - zc) * sc
    # a column's own quantization error is at most half a step unless the error feedback of
    # earlier columns pushed it past its group's range (fixed at the group's first column)
    inside = ((Wg - Q).abs() <= 0.5 * sc * (1 + 1e-5) + 1e-7).float().mean().item()
    print(f'within half a step: {inside * 100:.3f} %')
    assert inside > 0.98
    # GPTQ objective vs round-to-nearest of the same weight (rows sampled)
    rows = torch.arange(0, H70, 32, device=dev)
    Wf = W.float()[rows]
    rtn = wq.fake_quant_weight_dynamic(W)[rows].float()

    def obj(D):
        return ((D @ Hc) * D).sum().item()
    e_gptq, e_rtn = obj(Wf - Q[rows]), obj(Wf - rtn)
    print(f'GPTQ objective {e_gptq:.4e} vs RTN {e_rtn:.4e}')
    assert e_gptq < 0.8 * e_rtn


def test_l70b_awq_block_fused_vs_torch_gemm(dev, monkeypatch):
    from transformers import LlamaConfig

    from lightcompress_amd.awq import Awq
    from lightcompress_amd.llama import Llama
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.utils import load_config
    cfg = LlamaConfig(hidden_size=H70, intermediate_size=I70, num_attention_heads=64,
                      num_key_value_heads=8, head_dim=128, rope_theta=500000.0,
                      max_position_embeddings=8192, rms_norm_eps=1e-5, num_hidden_layers=1)
    config = {'quant': {'method': 'Awq',
                        'weight': {'bit': 4, 'symmetric': True, 'granularity': 'per_group',
                                   'group_size': 128},
                        'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                                    'clip_sym': True}},
              'calib': {'seq_len': 512, 'bs': -1, 'n_samples': 32}}
    g = torch.Generator(device=dev).manual_seed(11)
    mag = torch.exp(torch.randn(H70, generator=g, device=dev))
    x = (torch.randn(32, 512, H70, generator=g, device=dev) * mag).to(torch.bfloat16)
    orig = Awq.search_scale_subset
    from lightcompress_amd import ops
    orig_sq = ops.linear_sq_diff

    def run(fused):
        curves = []
        calls = [0]

        def sq(*a, **k):
            calls[0] += 1
            return orig_sq(*a, **k)

        def rec(self, *a, **k):
            best = orig(self, *a, **k)
            curves.append(torch.tensor(self.last_search['losses'], dtype=torch.float64))
            return best
        with monkeypatch.context() as m:
            m.setattr(Awq, 'search_scale_subset', rec)
            m.setattr(ops, 'linear_sq_diff', sq)
            if not fused:
                m.setattr(Awq, 'fused_search', False)
                # every linear back on torch (hipBLASLt): the test-side A/B
                m.setattr(ops, 'gemm_supported', lambda *a, **k: False)
            model = Llama.random(cfg, num_layers=1, device=dev, seed=12)
            algo = build_algo(model, load_config(config),
                              {'data': [x], 'kwargs': [model.rotary_kwargs(512)]})
            algo.run_block_loop()
            w = {n: l.weight.detach().clone()
                 for n, l in model.get_block_linears(model.get_blocks()[0]).items()}
        assert (calls[0] > 0) == fused, calls   # the loss epilogue ran only in the fused run
        return curves, w

    c_f, w_f = run(True)
    c_t, w_t = run(False)
    assert len(c_f) == len(c_t) == 3        # q/k/v, gate/up, down (o_proj: GQA skip)
    same_pick = []
    for i, (a, b) in enumerate(zip(c_f, c_t)):
        rel = ((a - b).abs() / b.abs()).max().item()
        ia, ib = int(a.argmin()), int(b.argmin())
        print(f'subset {i}: max rel loss diff {rel:.2e}, argmin fused {ia} torch {ib}')
        assert rel < 5e-3, i
        assert ia == ib or b[ia].item() <= b[ib].item() * 1.002, i
        same_pick.append(ia == ib)
    for n in w_f:
        eq = (w_f[n].view(torch.int16) == w_t[n].view(torch.int16)).float().mean().item()
        print(f'{n:20s} equal {eq * 100:.3f} %')
        if all(same_pick):
            assert eq >= 0.95, n
