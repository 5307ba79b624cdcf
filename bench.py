"""Benchmark: LightCompress per-layer weight-quantization hot path on MI355X.

Headline (BASELINE.json configs[1]): Llama-3-8B AWQ w4a16 g128 (symmetric, weight_clip,
trans_version v2 -- configs/quantization/methods/Awq/awq_w_only.yml) with 128 calibration
samples x 512 tokens, deployed to vLLM packed int4 (need_pack). One step = one Llama-3-8B
decoder block through the reference's run_block_loop / block_opt (calibration forward with
input capture, AWQ scale search on the qkv / gate-up / down subsets -- o_proj is skipped under
GQA exactly as the reference does -- scale application, auto-clip of v/o/gate/up/down) plus
the real-quant + vLLM pack of its 7 linears. Random-init weights and synthetic activations of
the real shapes (no network: no checkpoints / datasets).

metric: linear layers quantized per second (whole job, all ranks). Multi-GPU: one process per
GPU (torchrun); quant_out=False makes AWQ blocks independent given the float activations
(SURVEY.md §8e), so the timed run is the algorithm's own run_block_loop in shard_blocks mode
over steps x N blocks with materialize: owned: every rank allocates, quantizes and packs only
its own blocks, the float activations pass from the owner of block i to the owner of block i + 1
over a ring edge (the only collective on the data path) -- weak scaling.

Also in the line:
* "gptq" (configs[2]): Llama-3-8B GPTQ w4a16 g128 asym, act-order, true_sequential, quant_out,
  128 x 2048 tokens (bs 1); per-block time; at N > 1 the calibration samples are sharded
  (shard_tokens: partial Hessians summed, row-sharded column loop); roofline = the XᵀX kernel.
* "e2e": MEASURED end-to-end wall-clock of the whole 32-block Llama-3-8B (AWQ and GPTQ):
  run_block_loop + deploy (vllm_quant / fake_quant) -- the reference's llmc_duration_time.
* "l70b" (configs[3] shapes): one Llama-3-70B decoder block through the AWQ and the GPTQ
  recipes (block_opt + deploy), per-block time and the projection-GEMM roofline at 70B shapes.
* "fp8" (configs[4]): DeepSeek-V3 expert linears, block-fp8 -> per-tensor e4m3 deploy, and the
  block-scaled fp8 GEMM of their calibration forward.
* roofline: the dominant kernel of the headline step (k_gemm16: the projection GEMMs of the
  AWQ loss search with their fused epilogues), flops and algorithmic bytes of every launch
  over its device-event time; traffic = PMC HBM bytes per launch from profiles/.
* cpu_baseline: the oracle (the reference algorithm restated on torch-CPU, pinned to the
  reference by tests/golden) on the host cores over a bounded sample, extrapolated; AWQ (the
  headline) and GPTQ.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
PEAK_FP8_TFLOPS = 5000.0    # MI355X dense fp8 (e4m3) MFMA (MI355X_MICROARCH.md)

LLAMA3_8B = dict(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                 num_key_value_heads=8, head_dim=128, rope_theta=500000.0,
                 max_position_embeddings=8192, rms_norm_eps=1e-5, num_hidden_layers=32,
                 vocab_size=128256)
LLAMA3_70B = dict(LLAMA3_8B, hidden_size=8192, intermediate_size=28672,
                  num_attention_heads=64, num_key_value_heads=8, num_hidden_layers=80)
N_LINEARS_PER_BLOCK = 7
GEMM_FAMILY = ('lcq_gemm', 'lcq_gemm_rope', 'lcq_gemm_silu_mul', 'lcq_gemm_sq_diff',
               'lcq_gemm_residual')


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--n-samples', type=int, default=128)
    ap.add_argument('--seq-len', type=int, default=512)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-e2e', action='store_true')
    ap.add_argument('--e2e-blocks', type=int, default=32)
    ap.add_argument('--algo', choices=['awq', 'gptq', 'fp8', 'both', 'all'], default='all')
    ap.add_argument('--fp8-experts', type=int, default=32)
    ap.add_argument('--fp8-tokens', type=int, default=2048,
                    help='calibration tokens routed to each expert in the fp8 forward leg')
    ap.add_argument('--gptq-steps', type=int, default=3)
    ap.add_argument('--gptq-samples', type=int, default=128)
    ap.add_argument('--gptq-seq-len', type=int, default=2048)
    ap.add_argument('--cpu-budget-s', type=float, default=20.0)
    ap.add_argument('--no-stream', action='store_true',
                    help='skip the host-resident (streamed) e2e runs')
    ap.add_argument('--rank-timeout', type=float, default=3000.0,
                    help='bench.py --gpus N without a launcher: kill every rank after this many '
                         'seconds (0: no limit)')
    ap.add_argument('--no-l70b', action='store_true',
                    help='skip the Llama-3-70B-shaped block leg (BASELINE configs[3])')
    return ap.parse_args()


def awq_config(seq_len, n_samples=128):
    from lightcompress_amd.utils import load_config
    return load_config({
        'base': {'seed': 42},
        'calib': {'name': 'pileval', 'n_samples': n_samples, 'bs': -1, 'seq_len': seq_len,
                  'preproc': 'pileval_awq'},
        'quant': {'method': 'Awq',
                  'weight': {'bit': 4, 'symmetric': True, 'granularity': 'per_group',
                             'group_size': 128, 'need_pack': True},
                  'special': {'trans': True, 'trans_version': 'v2', 'weight_clip': True,
                              'clip_sym': True},
                  'quant_out': False},
    })


def gptq_config(seq_len, n_samples):
    from lightcompress_amd.utils import load_config
    return load_config({
        'base': {'seed': 42},
        'calib': {'name': 'wikitext2', 'n_samples': n_samples, 'bs': 1, 'seq_len': seq_len,
                  'preproc': 'wikitext2_gptq'},
        'quant': {'method': 'GPTQ',
                  'weight': {'bit': 4, 'symmetric': False, 'granularity': 'per_group',
                             'group_size': 128},
                  'special': {'actorder': True, 'static_groups': False, 'percdamp': 0.01,
                              'blocksize': 128, 'true_sequential': True},
                  'quant_out': True},
    })


def synthetic_hidden(n, seq, hidden, device, seed):
    """Calibration hidden states with log-normal per-channel magnitudes (outlier channels,
    SURVEY.md §8d), bf16. The same seed on every rank: one global calibration set."""
    g = torch.Generator(device=device).manual_seed(seed)
    mag = torch.exp(torch.randn(hidden, generator=g, device=device))
    x = torch.randn(n, seq, hidden, generator=g, device=device) * mag
    return x.to(torch.bfloat16)


def pmc_traffic(leg, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this
    round (profiles/*_pmc_traffic_<leg>.json, made by scripts/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2 FETCH correction), or None."""
    files = sorted((ROOT / 'profiles').glob(f'*_pmc_traffic_{leg}.json'))
    if not files:
        return None, None
    d = json.loads(files[-1].read_text())
    names = kernel if isinstance(kernel, tuple) else (kernel,)   # a tuple: one call's kernels
    ks = [d.get('kernels', {}).get(k) for k in names]
    if not all(ks):
        return None, str(files[-1].relative_to(ROOT))
    return sum(k['hbm_bytes'] for k in ks), str(files[-1].relative_to(ROOT))


class ClockSampler:
    """The GFX clock over a timed region, read by amdsmi on a host thread every `period` s
    (`amdsmi_get_clock_info(GFX)['clk']`, and the firmware's `average_gfxclk_frequency` from
    the GPU metrics table where present). MI355X lowers its clock under MFMA load (DVFS,
    MI355X_MICROARCH.md 'DVFS give-back'); this puts the clock the chip held next to the
    number, so a box-to-box difference can be told apart from a code regression. It reads
    sysfs-level clocks, which run up to ~10 % above the in-kernel clock of an MFMA loop.
    None when amdsmi is unavailable (never fails the bench)."""

    def __init__(self, dev, period=0.05):
        import threading
        self.period, self.samples, self.avg = period, [], []
        self._stop = threading.Event()
        self._thread = None
        self.handle = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self._smi = amdsmi
            handles = amdsmi.amdsmi_get_processor_handles()
            idx = torch.device(dev).index or 0
            try:
                p = torch.cuda.get_device_properties(idx)
                bdf = f'{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0'
                self.handle = amdsmi.amdsmi_get_processor_handle_from_bdf(bdf)
            except Exception:
                self.handle = handles[idx] if idx < len(handles) else None
        except Exception:
            self.handle = None

    def _run(self):
        smi = self._smi
        while not self._stop.is_set():
            try:
                self.samples.append(float(smi.amdsmi_get_clock_info(
                    self.handle, smi.AmdSmiClkType.GFX)['clk']))
            except Exception:
                pass
            try:
                v = smi.amdsmi_get_gpu_metrics_info(self.handle).get('average_gfxclk_frequency')
                if isinstance(v, (int, float)) and 0 < v < 10000:
                    self.avg.append(float(v))
            except Exception:
                pass
            self._stop.wait(self.period)

    def __enter__(self):
        if self.handle is not None:
            import threading
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=5)
        return False

    def summary(self):
        if not self.samples:
            return None
        xs = sorted(self.samples)
        out = {'mean': round(sum(xs) / len(xs), 1), 'median': xs[len(xs) // 2],
               'min': xs[0], 'max': xs[-1], 'samples': len(xs),
               'source': 'amdsmi GFX clock (MHz), sampled every 50 ms over the timed region'}
        if self.avg:
            out['fw_average_gfxclk_mean'] = round(sum(self.avg) / len(self.avg), 1)
        return out


class CollectiveMeter:
    """Bytes this rank hands to torch.distributed collectives / P2P inside the context (the
    algorithms call them as dist.<op>, so the module attributes are wrapped): the payload
    tensor's bytes per call -- the input of a reduce / broadcast / send, the gathered output of
    an all-gather / all-to-all -- by op. Measures the data-path volume per block the N-GPU
    scaling model needs; 0 at N = 1."""
    OPS = {'all_reduce': 0, 'broadcast': 0, 'send': 0, 'isend': 0, 'recv': 0, 'irecv': 0,
           'all_gather': 1, 'all_gather_into_tensor': 0, 'all_to_all_single': 0}

    def __init__(self, world):
        self.world = world
        self.bytes = {}
        self.calls = {}
        self._orig = {}

    def __enter__(self):
        if self.world <= 1:
            return self
        for name, arg in self.OPS.items():
            fn = getattr(dist, name, None)
            if fn is None:
                continue
            self._orig[name] = fn

            def wrapped(*a, _fn=fn, _name=name, _arg=arg, **kw):
                t = a[_arg] if len(a) > _arg else None
                ts = t if isinstance(t, (list, tuple)) else [t]
                n = sum(x.numel() * x.element_size() for x in ts if torch.is_tensor(x))
                self.bytes[_name] = self.bytes.get(_name, 0) + n
                self.calls[_name] = self.calls.get(_name, 0) + 1
                return _fn(*a, **kw)
            setattr(dist, name, wrapped)
        return self

    def __exit__(self, *exc):
        for name, fn in self._orig.items():
            setattr(dist, name, fn)

    def per_block(self, blocks):
        """{op: MB per block} (+ total), or None at N = 1."""
        if self.world <= 1:
            return None
        out = {k: round(v / blocks / 2 ** 20, 2) for k, v in sorted(self.bytes.items())}
        out['total'] = round(sum(self.bytes.values()) / blocks / 2 ** 20, 2)
        out['calls_per_block'] = round(sum(self.calls.values()) / blocks, 1)
        return out


def sync_barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def free_device():
    """After a leg: collect the algorithm <-> model cycles (deployed modules hold the quant
    callables) and return the allocator's free blocks, so the next leg starts from its own
    model + calibration only (e2e's hbm_at_start_gb)."""
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def max_over_ranks(v, world, dev):
    if world > 1:
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        v = t.item()
    return v


def take_linear_fallbacks():
    """lcq_linear calls since the last call that took torch's F.linear instead of the lcq GEMM
    (module_utils.LINEAR_FALLBACKS), as {"dtype x / w K->N": count}; resets the counter."""
    from lightcompress_amd import module_utils as mu
    got = {f'{a}/{b} {k}->{n}': c for (a, b, k, n), c in mu.LINEAR_FALLBACKS.items()}
    mu.LINEAR_FALLBACKS.clear()
    return got


def kernel_table(kern, elapsed):
    return {k: {'launches': v['launches'], 'avg_ms': round(v['avg_ms'], 4),
                'share_of_step': round(v['total_ms'] / (elapsed * 1e3), 4)}
            for k, v in sorted(kern.items(), key=lambda kv: -kv[1]['total_ms'])}


def gemm_roofline(kern, elapsed):
    """The projection-GEMM family (all k_gemm16 launches: lcq_gemm / _silu_mul / _sq_diff):
    algorithmic flops and bytes of every launch (noted by ops.py) over the device-event time
    of those launches."""
    fam = [kern[n] for n in GEMM_FAMILY if n in kern]
    if not fam:
        return None
    ms = sum(f['total_ms'] for f in fam)
    n = sum(f['launches'] for f in fam)
    fl = sum(f.get('flops', 0.0) for f in fam)
    by = sum(f.get('bytes', 0.0) for f in fam)
    tf = fl / (ms * 1e-3) / 1e12
    traffic, src = pmc_traffic('awq', 'k_gemm16')
    return {'kernel': 'k_gemm16h (csrc/gemm256.hip): bf16 MFMA projection GEMMs of the AWQ loss '
                      'search + calibration forwards, epilogues fused (q/k/v, SiLU*up, loss)',
            'bound': 'mfma', 'achieved': round(tf, 1), 'peak': PEAK_BF16_TFLOPS,
            'unit': 'TFLOP/s', 'frac': round(tf / PEAK_BF16_TFLOPS, 4), 'traffic': traffic,
            'traffic_source': src, 'algorithmic_bytes_per_launch': by / n,
            'flops_per_launch': fl / n, 'avg_launch_ms': round(ms / n, 4), 'launches': n,
            'share_of_step': round(ms / (elapsed * 1e3), 3)}


# ---------------------------------------------------------------------------------------
# CPU baselines (oracle = the reference algorithm on torch-CPU; bounded samples, extrapolated)
# ---------------------------------------------------------------------------------------
# auto-clip's VALU issue bound: each SIMD issues one wave64 vector instruction per 2 cycles
# (MI355X_MICROARCH.md, wave scheduling), and a DT-rounded product costs at least 1/32 of one
# (v_pk_mul_f32 and v_pk_add_f32 cover 128 products, v_cvt_pk_bf16_f32 64): 1024 SIMDs x
# 2.4 GHz / 2 x 32 products
PEAK_CLIP_GPRODUCTS = 1024 * 2.4 / 2 * 32   # 3.93e4 G products/s


def clip_roofline(kern):
    """The auto-clip search (AutoClipper.auto_clip_layer, auto_clip.py:83-191) against its
    VALU issue bound: products per second over the launches' HIP-event time, both entries
    together (lcq_auto_clip_search_ws runs every layer of the headline on k_clip_qtable +
    k_auto_clip_tw while the sampled tokens fit 512 lanes; lcq_auto_clip_search_act is the
    lane-pair k_auto_clip for the other configurations)."""
    ts = [kern[k] for k in ('lcq_auto_clip_search_ws', 'lcq_auto_clip_search_act')
          if kern.get(k) and kern[k].get('flops')]
    if not ts:
        return None
    flops = sum(t['flops'] for t in ts)
    ms = sum(t['total_ms'] for t in ts)
    launches = sum(t['launches'] for t in ts)
    gp = flops / (ms * 1e-3) / 1e9
    return {'kernel': ('k_clip_qtable + k_auto_clip_tw (one lane per sampled token, all 512 '
                       'in one 8-wave workgroup, candidate rows staged in LDS by LDS-DMA)'),
            'bound': 'valu', 'achieved': round(gp, 1), 'peak': PEAK_CLIP_GPRODUCTS,
            'unit': 'G products/s', 'frac': round(gp / PEAK_CLIP_GPRODUCTS, 4),
            'avg_launch_ms': round(ms / launches, 4), 'launches': launches,
            'products_per_launch': flops / launches,
            'pmc_source': 'profiles/r6_clip_tw_pmc.txt'}


def cpu_baseline_awq(args, budget_s):
    """One AWQ block step on the host cores: as many calibration samples x (org + one ratio)
    per subset as fit in ~60% of the budget, auto-clip on as many 64-row chunks of gate_proj
    as fit in the next ~25%, the real-quant + vLLM pack of one gate_proj; extrapolated
    linearly to the full step."""
    from transformers import LlamaConfig
    from transformers.models.llama import modeling_llama as ml
    from oracle import awq_ref as A
    from oracle import quant_ref as Q
    torch.manual_seed(0)
    threads = torch.get_num_threads()
    cfg = LlamaConfig(**LLAMA3_8B)
    cfg._attn_implementation = 'sdpa'
    layer = ml.LlamaDecoderLayer(cfg, layer_idx=0).to(torch.bfloat16).eval()
    with torch.no_grad():
        for p in layer.parameters():
            if p.dim() == 2:
                p.normal_(0, 0.02)
    rot = ml.LlamaRotaryEmbedding(cfg)
    seq = args.seq_len
    pos = torch.arange(seq).unsqueeze(0)
    t_start = time.perf_counter()
    fwd_t, org_t, ratio_t = [], {}, {}
    n_done = 0
    with torch.no_grad():
        while True:
            x = synthetic_hidden(1, seq, cfg.hidden_size, 'cpu', 7 + n_done)
            kw = {'position_embeddings': rot(x, pos), 'attention_mask': None, 'position_ids': pos}
            t0 = time.perf_counter()
            xq = layer.input_layernorm(x)
            h = x + layer.self_attn(xq, **kw)[0]
            xm = layer.post_attention_layernorm(h)
            xd = layer.mlp.act_fn(layer.mlp.gate_proj(xm)) * layer.mlp.up_proj(xm)
            h + layer.mlp.down_proj(xd)
            fwd_t.append(time.perf_counter() - t0)
            subsets = {
                'qkv': (xq, [layer.self_attn.q_proj, layer.self_attn.k_proj,
                             layer.self_attn.v_proj], lambda t: layer.self_attn(t, **kw)[0]),
                'mlp': (xm, [layer.mlp.gate_proj, layer.mlp.up_proj], layer.mlp),
                'down': (xd, [layer.mlp.down_proj], layer.mlp.down_proj),
            }
            for name, (xin, mods, fwd) in subsets.items():
                t0 = time.perf_counter()
                org = fwd(xin)
                t1 = time.perf_counter()
                ratio = ((n_done % 20) + 1) / 20
                s = A.scales_v2(A.act_scale(xin), ratio)
                saved = [m.weight.data for m in mods]
                for m in mods:
                    m.weight.data = A.fake_quant_scaled(m.weight.data, s, 4, True, 128)
                out = fwd(xin / s.view(1, -1))
                A.loss(org, out)
                for m, w in zip(mods, saved):
                    m.weight.data = w
                t2 = time.perf_counter()
                org_t.setdefault(name, []).append(t1 - t0)
                ratio_t.setdefault(name, []).append(t2 - t1)
            n_done += 1
            if time.perf_counter() - t_start > 0.6 * budget_s or n_done >= args.n_samples:
                break
        parts = {'block_forward': sum(fwd_t) / len(fwd_t) * args.n_samples}
        for name in org_t:
            per_sample = (sum(org_t[name]) / len(org_t[name])
                          + 20 * sum(ratio_t[name]) / len(ratio_t[name]))
            parts[f'search_{name}'] = per_sample * args.n_samples  # linear in tokens
        xs = xm.reshape(-1, cfg.hidden_size)[: seq]
        t_clip, rows = 0.0, 0
        while rows < cfg.intermediate_size:
            w = layer.mlp.gate_proj.weight.data[rows:rows + 64].clone()
            t0 = time.perf_counter()
            A.clip_layer(w, xs, 4, True, 128, True, n_sample_token=seq)
            t_clip += time.perf_counter() - t0
            rows += 64
            if time.perf_counter() - t_start > 0.85 * budget_s:
                break
        clipped = (cfg.num_key_value_heads * cfg.head_dim * cfg.hidden_size
                   + cfg.hidden_size ** 2 + 3 * cfg.intermediate_size * cfg.hidden_size)
        parts['auto_clip'] = t_clip * clipped / (rows * cfg.hidden_size)
        t0 = time.perf_counter()
        codes, sc, _ = Q.real_quant_dynamic(layer.mlp.gate_proj.weight.data, 4, True)
        Q.pack_vllm(codes, 4)
        t_dep = time.perf_counter() - t0
        all_params = clipped + (cfg.hidden_size + cfg.num_key_value_heads * cfg.head_dim) * cfg.hidden_size
        parts['deploy'] = t_dep * all_params / layer.mlp.gate_proj.weight.numel()
    t_total_est = sum(parts.values())
    wall = time.perf_counter() - t_start
    return {'value': N_LINEARS_PER_BLOCK / t_total_est, 'unit': 'linears/s', 'cores': threads,
            'kind': 'port',
            'sample': (f'oracle (torch-CPU restatement of awq.py/auto_clip.py/quant.py, pinned to '
                       f'the reference by tests/golden) on one Llama-3-8B block: {n_done} of '
                       f'{args.n_samples} calibration samples x (org + 1 of 20 ratios) per '
                       f'subset, auto-clip of {rows} gate_proj rows, real-quant+pack of one '
                       f'gate_proj; {wall:.1f} s measured, extrapolated linearly to '
                       f'{t_total_est:.0f} s per block step'),
            'est_s_per_block': round(t_total_est, 1),
            'parts_s': {k: round(v, 1) for k, v in parts.items()}}


def cpu_baseline_gptq(args, budget_s):
    """One GPTQ block step on the host cores, the reference's own work per block: 11 Hessians
    (7 in block_init + 4 recomputed by true_sequential, gptq.py / base_blockwise_quantization
    .py:498-526) over 128 x 2048 tokens, the Cholesky chain per linear and the column loop of
    each linear. Sampled: the 4096-wide Hessian over as many 2048-token samples as fit in
    ~45% of the budget, one Cholesky chain at IC 4096, the column loop of a row slice of a
    4096^2 linear; extrapolated by IC^2 (Hessian), IC^3 (Cholesky), OC*IC^2 (column loop)."""
    from oracle import gptq_ref as Gr
    threads = torch.get_num_threads()
    H, I = 4096, 14336
    seq, ns = args.gptq_seq_len, args.gptq_samples
    t_start = time.perf_counter()
    samples, t_h = [], 0.0
    while True:
        x = synthetic_hidden(1, seq, H, 'cpu', 100 + len(samples))
        samples.append(x)
        t0 = time.perf_counter()
        Hm, _ = Gr.hessian(samples[-1:], H)
        t_h += time.perf_counter() - t0
        if time.perf_counter() - t_start > 0.45 * budget_s or len(samples) >= ns:
            break
    per_sample_4096 = t_h / len(samples)
    hess_units = 9 + 2 * (I / H) ** 2          # 9 Hessians at IC 4096, 2 at IC 14336
    t_hess = per_sample_4096 * ns * hess_units
    g = torch.Generator().manual_seed(1)
    W = (torch.randn(H, H, generator=g) * 0.02)
    Hm = Hm + torch.eye(H)
    t0 = time.perf_counter()
    Wp, U, perm = Gr.prepare(W.clone(), Hm.clone(), True, 0.01)
    t_chol = time.perf_counter() - t0
    rows = 64
    t0 = time.perf_counter()
    while True:
        Gr.column_loop(Wp[:rows].clone(), U, 4, False, 128)
        if time.perf_counter() - t_start > 0.9 * budget_s or rows >= H:
            break
        rows *= 2
    t_col_rows = time.perf_counter() - t0
    # the last call covered `rows` rows (the doublings before it cost as much again)
    per_row_4096 = t_col_rows / (2 * rows - 64)
    oc_ic2 = (H * H * H * 2 + 2 * 1024 * H * H + 2 * I * H * H + H * I * I) / (H * H)  # rows x (IC/4096)^2
    t_col = per_row_4096 * oc_ic2
    t_chol_all = t_chol * (6 + (I / H) ** 3)   # 6 linears at IC 4096 (q,k,v,o,gate,up), down
    t_total = t_hess + t_chol_all + t_col
    wall = time.perf_counter() - t_start
    return {'value': N_LINEARS_PER_BLOCK / t_total, 'unit': 'linears/s', 'cores': threads,
            'kind': 'port',
            'sample': (f'oracle (gptq_ref: gptq.py restated on torch-CPU, pinned by tests/golden) '
                       f'on Llama-3-8B block shapes: Hessian of {len(samples)} of {ns} 2048-token '
                       f'samples at IC 4096, one Cholesky chain at IC 4096, column loop of '
                       f'{rows} rows x 4096; {wall:.1f} s measured, extrapolated to '
                       f'{t_total:.0f} s per block (11 Hessians, 7 chains, 7 column loops)'),
            'est_s_per_block': round(t_total, 1),
            'parts_s': {'hessian': round(t_hess, 1), 'cholesky': round(t_chol_all, 1),
                        'column_loop': round(t_col, 1)}}


# ---------------------------------------------------------------------------------------
# legs
# ---------------------------------------------------------------------------------------
def bench_awq(args, rank, world, dev):
    """Headline: AWQ block steps through the algorithm's run_block_loop (shard_blocks at N > 1)
    + the vLLM real-quant deploy of this rank's blocks."""
    from transformers import LlamaConfig
    from lightcompress_amd import _native
    from lightcompress_amd.llama import Llama
    from lightcompress_amd.pipeline import build_algo
    from lightcompress_amd.module_utils import VllmRealQuantLinear
    cfg = LlamaConfig(**LLAMA3_8B)
    config = awq_config(args.seq_len, args.n_samples)
    # warmup on blocks of its own model (no collectives: every rank warms its kernels)
    if args.warmup:
        wm = Llama.random(cfg, num_layers=args.warmup, device=dev, seed=999)
        wx = synthetic_hidden(args.n_samples, args.seq_len, cfg.hidden_size, dev, 5)
        walgo = build_algo(wm, config, {'data': [wx], 'kwargs': [wm.rotary_kwargs(args.seq_len)]})
        for i, b in enumerate(wm.get_blocks()):
            walgo.block_idx = i
            walgo.block_opt(b)
            wm.replace_module_block(VllmRealQuantLinear, b, i,
                                    walgo.get_replacement_params('vllm_quant', walgo.w_only))
        walgo.release()
        del walgo, wm, wx
        free_device()
    nblk = args.steps * world
    if world == 1:
        model = Llama.random(cfg, num_layers=nblk, device=dev, seed=1000)
    else:
        # shard_blocks: each rank materialises only its own blocks (materialize: owned; the
        # other blocks stay on the meta device, every tensor seeded by its name so a block is
        # the same whichever rank builds it); the deploy packs each rank's blocks in place
        from lightcompress_amd.utils import load_config
        config = load_config(dict(config, model={'type': 'Llama', 'materialize': 'owned'}))
        model = Llama(config, hf_config=LlamaConfig(**dict(LLAMA3_8B, num_hidden_layers=nblk)),
                      random_init={'seed': 1000, 'std': 0.02}, device=dev)
    hidden = synthetic_hidden(args.n_samples, args.seq_len, cfg.hidden_size, dev, 17)
    algo = build_algo(model, config, {'data': [hidden], 'kwargs': [model.rotary_kwargs(args.seq_len)]})
    timer = _native.KernelTimer()
    clock = ClockSampler(dev)
    meter = CollectiveMeter(world)
    sync_barrier(world)
    t0 = time.perf_counter()
    with timer, clock, meter:
        algo.run_block_loop()
        # deploy: real-quant + vLLM pack; under shard_blocks each rank packs its own blocks and
        # the packed shards are gathered, so every rank ends with the whole deployed model
        algo.deploy('vllm_quant')
    sync_barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    kern = timer.summary()
    mode = algo.parallel_mode()
    algo.release()
    del algo, model, hidden
    free_device()
    return elapsed, kern, mode, clock.summary(), meter.per_block(nblk)


def bench_gptq(args, rank, world, dev):
    """GPTQ leg: per-block wall-clock (block_opt; token-sharded at N > 1) and the Hessian
    kernel's roofline."""
    from transformers import LlamaConfig
    from lightcompress_amd import _native
    from lightcompress_amd.llama import Llama
    from lightcompress_amd.pipeline import build_algo
    cfg = LlamaConfig(**LLAMA3_8B)
    warm, steps = 1, args.gptq_steps
    model = Llama.random(cfg, num_layers=warm + steps, device=dev, seed=2000)
    seq = args.gptq_seq_len
    hidden = synthetic_hidden(args.gptq_samples, seq, cfg.hidden_size, dev, 31)
    kw = model.rotary_kwargs(seq)
    calib = {'data': [hidden[i:i + 1] for i in range(args.gptq_samples)],
             'kwargs': [kw] * args.gptq_samples}
    algo = build_algo(model, gptq_config(seq, args.gptq_samples), calib)
    blocks = model.get_blocks()

    def step(i):
        algo.block_idx = i
        algo.block_opt(blocks[i])

    for i in range(warm):
        step(i)
    timer = _native.KernelTimer()
    meter = CollectiveMeter(world)
    sync_barrier(world)
    t0 = time.perf_counter()
    with timer, meter:
        for i in range(warm, warm + steps):
            step(i)
    sync_barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    kern = timer.summary()
    ms = elapsed / steps * 1e3
    out = {'linears_per_s': round(N_LINEARS_PER_BLOCK * steps / elapsed, 3),
           'parallelism': ('single GPU' if world == 1 else
                           f'{world} ranks, {algo.parallel_mode()} (calibration samples sharded, '
                           'partial Hessians summed, row-sharded column loop)'),
           'ms_per_block': round(ms, 1), 'steps': steps, 'warmup': warm,
           'workload': (f'Llama-3-8B GPTQ w4a16 g128 asym act-order true_sequential quant_out, '
                        f'{args.gptq_samples}x{seq} calib tokens (bs 1)'),
           'collective_mb_per_block': meter.per_block(steps),
           'lcq_kernels': kernel_table(kern, elapsed)}
    h = kern.get('lcq_hessian_grouped') or kern.get('lcq_hessian_accum')
    if h:
        # algorithmic: symmetric rank-n update n*ic*(ic+1) flops per launch
        tf = h['flops'] / (h['total_ms'] * 1e-3) / 1e12
        traffic, src = pmc_traffic('gptq', ('k_syrk_x', 'k_syrk_reduce'))
        out['roofline'] = {'kernel': 'lcq_hessian_grouped (k_syrk_x: bf16 MFMA XᵀX read from '
                                     'token-major X through transposed LDS reads, all 8 '
                                     'calibration-sample groups in one launch; k_syrk_reduce: '
                                     'per-group fold + fixed group tree)',
                           'bound': 'mfma', 'achieved': round(tf, 1), 'peak': PEAK_BF16_TFLOPS,
                           'unit': 'TFLOP/s', 'frac': round(tf / PEAK_BF16_TFLOPS, 4),
                           'traffic': traffic, 'traffic_source': src,
                           'avg_launch_ms': round(h['avg_ms'], 4),
                           'flops_per_launch': h['flops'] / h['launches']}
    algo.release()   # block_opt driven directly: the chain graphs go with the algorithm
    del algo, model, hidden, calib, blocks
    free_device()
    return out


def bench_e2e(args, rank, world, dev, which, residency='device'):
    """Whole-model wall-clock (MEASURED, not extrapolated): a random-init 32-block Llama-3-8B
    through build_algo -> run_block_loop -> deploy, the span the reference times as
    llmc_duration_time (llmc/__main__.py:182, 265-267) minus model loading / dataset / eval.
    residency 'stream': the blocks live in pinned host memory and pass through HBM one at a
    time (the reference's block.cuda() / block.cpu() scheme, base_blockwise_quantization.py:397,
    418, with the uploads and write-backs on side streams)."""
    from transformers import LlamaConfig
    from lightcompress_amd.llama import Llama
    from lightcompress_amd.pipeline import build_algo
    cfg = LlamaConfig(**LLAMA3_8B)
    nb = args.e2e_blocks
    free_device()   # whatever an earlier leg left to the cyclic collector goes first
    model = Llama.random(cfg, num_layers=nb, device=dev, seed=3000 if which == 'awq' else 4000,
                         residency=residency)
    torch.cuda.empty_cache()
    hbm0 = torch.cuda.memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    if which == 'awq':
        hidden = synthetic_hidden(args.n_samples, args.seq_len, cfg.hidden_size, dev, 41)
        calib = {'data': [hidden], 'kwargs': [model.rotary_kwargs(args.seq_len)]}
        config, fmt = awq_config(args.seq_len, args.n_samples), 'vllm_quant'
    else:
        seq = args.gptq_seq_len
        hidden = synthetic_hidden(args.gptq_samples, seq, cfg.hidden_size, dev, 43)
        kw = model.rotary_kwargs(seq)
        calib = {'data': [hidden[i:i + 1] for i in range(args.gptq_samples)],
                 'kwargs': [kw] * args.gptq_samples}
        config, fmt = gptq_config(seq, args.gptq_samples), 'fake_quant'
    meter = CollectiveMeter(world)
    sync_barrier(world)
    t0 = time.perf_counter()
    with meter:
        algo = build_algo(model, config, calib)
        algo.run_block_loop()
        t_loop = time.perf_counter() - t0
        algo.deploy(fmt)
    sync_barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    t_loop = max_over_ranks(t_loop, world, dev)
    mode = algo.parallel_mode()
    out = {'wall_s': round(elapsed, 2), 'block_loop_s': round(t_loop, 2),
           'blocks': nb, 'linears': N_LINEARS_PER_BLOCK * nb,
           'linears_per_s': round(N_LINEARS_PER_BLOCK * nb / elapsed, 3),
           'deploy': fmt, 'parallel_mode': mode, 'residency': residency,
           'hbm_at_start_gb': round(hbm0 / 2 ** 30, 2),
           'hbm_peak_gb': round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
           'collective_mb_per_block': meter.per_block(nb)}
    if model.streamer is not None:
        st = model.streamer.stats
        out['streamed'] = {'h2d_gb': round(st['h2d_bytes'] / 2 ** 30, 2),
                           'd2h_gb': round(st['d2h_bytes'] / 2 ** 30, 2),
                           'fetches': st['fetches'], 'prefetched': st['prefetched'],
                           'pin_alloc_gb': round(st['pin_alloc_bytes'] / 2 ** 30, 2),
                           'pin_alloc_s': round(st['pin_alloc_s'], 3),
                           'pin_ahead_gb': round(st['pin_ahead_bytes'] / 2 ** 30, 2),
                           'pin_recycled_gb': round(st['pin_recycled_bytes'] / 2 ** 30, 2),
                           'evict_host_s': round(st['evict_host_s'], 3),
                           'deploy_s': round(elapsed - t_loop, 3)}
    algo.release()
    del algo, model, hidden, calib
    free_device()
    return out


def bench_l70b(args, rank, world, dev):
    """Llama-3-70B shapes (BASELINE.json configs[3]: hidden 8192, MLP 28672, 64q/8kv heads):
    one decoder block through the AWQ headline config (128 x 512 tokens, vLLM int4 deploy) and
    one through the GPTQ config (128 x 2048 tokens: the IC-28672 down_proj Hessian and column
    loop), each timed as block_opt + deploy after one warm-up block of the same shapes. The
    80-block model is 80 such blocks (per-block time x 80 / N GPUs under shard_blocks)."""
    from transformers import LlamaConfig
    from lightcompress_amd import _native
    from lightcompress_amd.llama import Llama
    from lightcompress_amd.module_utils import VllmRealQuantLinear
    from lightcompress_amd.pipeline import build_algo
    cfg = LlamaConfig(**LLAMA3_70B)
    out = {}
    for which in ('awq', 'gptq'):
        model = Llama.random(cfg, num_layers=2, device=dev, seed=5000)
        if which == 'awq':
            seq, n = args.seq_len, args.n_samples
            hidden = synthetic_hidden(n, seq, cfg.hidden_size, dev, 51)
            calib = {'data': [hidden], 'kwargs': [model.rotary_kwargs(seq)]}
            config = awq_config(seq, n)
        else:
            seq, n = args.gptq_seq_len, args.gptq_samples
            hidden = synthetic_hidden(n, seq, cfg.hidden_size, dev, 53)
            kw = model.rotary_kwargs(seq)
            calib = {'data': [hidden[i:i + 1] for i in range(n)], 'kwargs': [kw] * n}
            config = gptq_config(seq, n)
        algo = build_algo(model, config, calib)
        blocks = model.get_blocks()

        def step(i):
            algo.block_idx = i
            algo.block_opt(blocks[i])
            if which == 'awq':
                model.replace_module_block(VllmRealQuantLinear, blocks[i], i,
                                           algo.get_replacement_params('vllm_quant',
                                                                       algo.w_only))
        step(0)
        timer = _native.KernelTimer()
        sync_barrier(world)
        t0 = time.perf_counter()
        with timer:
            step(1)
        sync_barrier(world)
        el = max_over_ranks(time.perf_counter() - t0, world, dev)
        kern = timer.summary()
        top = dict(list(kernel_table(kern, el).items())[:6])
        out[which] = {'ms_per_block': round(el * 1e3, 1),
                      'linears_per_s': round(N_LINEARS_PER_BLOCK * world / el, 3),
                      'est_80_blocks_s': round(80 * el / world, 1),
                      'calib': f'{n}x{seq} tokens' + (' (bs 1)' if which == 'gptq' else ''),
                      'lcq_kernels': top}
        if which == 'awq':
            out[which]['roofline'] = gemm_roofline(kern, el)
        algo.release()
        del algo, model, hidden, calib, blocks
        free_device()
    out['workload'] = ('Llama-3-70B decoder block (8192 / 28672, 64q/8kv): AWQ w4a16 g128 '
                       '(configs[1] recipe) and GPTQ w4a16 g128 act-order (configs[2] recipe); '
                       'per-GPU replicas at N > 1')
    return out


DSV3_EXPERT = dict(hidden=7168, moe_inter=2048, block=128)


def dsv3_config(n_layers, n_experts):
    """DeepSeek-V3's layer shapes (public config: hidden 7168, MLA q_lora 1536 / kv_lora 512 /
    128 heads of 128 + 64 rope, routed experts 2048 wide, one shared expert) with every layer
    an MoE layer; the vocabulary is cut to 1024 (embeddings are not on the deploy path)."""
    from transformers import DeepseekV3Config
    cfg = DeepseekV3Config(hidden_size=7168, intermediate_size=18432, moe_intermediate_size=2048,
                           num_hidden_layers=n_layers, num_attention_heads=128,
                           num_key_value_heads=128, n_shared_experts=1,
                           n_routed_experts=n_experts, num_experts_per_tok=8, n_group=1,
                           topk_group=1, first_k_dense_replace=0, q_lora_rank=1536,
                           kv_lora_rank=512, qk_nope_head_dim=128, qk_rope_head_dim=64,
                           v_head_dim=128, vocab_size=1024, max_position_embeddings=4096,
                           tie_word_embeddings=False)
    cfg._attn_implementation = 'sdpa'
    return cfg


def fp8_rtn_config(world):
    """BASELINE configs[4]'s quantization (configs/quantization/backend/vllm/fp8/rtn_fp8.yml
    with per-tensor granularity): RTN, e4m3 weights + e4m3 activations per tensor, data-free,
    deployed as vllm_quant; each rank materialises only its LPT share of the units (a routed
    expert's three linears are one unit: EP-style), so N ranks hold N x the experts."""
    from lightcompress_amd.utils import load_config
    return load_config({
        'model': {'type': 'DeepseekV3', 'torch_dtype': 'torch.float8_e4m3fn',
                  'block_wise_quant': True, 'materialize': 'owned' if world > 1 else 'all'},
        'quant': {'method': 'RTN',
                  'weight': {'quant_type': 'float-quant', 'bit': 'e4m3', 'symmetric': True,
                             'granularity': 'per_tensor', 'use_qtorch': True},
                  'act': {'quant_type': 'float-quant', 'bit': 'e4m3', 'symmetric': True,
                          'granularity': 'per_tensor', 'use_qtorch': True}}})


def bench_fp8(args, rank, world, dev):
    """FP8 leg (BASELINE.json configs[4]): DeepSeek-V3 MoE layers stored block-fp8 (128x128,
    fp32 weight_scale_inv) as in the checkpoints, through the reference's data-free RTN
    pipeline: build_algo -> run_block_loop -> algo.deploy('vllm_quant') (per-tensor e4m3 real
    quant of every block linear: module_utils.py:914-927 + quant.py:1191-1221; each block's
    fp8 linears requantized in one batched launch pair). One step = one MoE layer: MLA (5
    linears), shared expert (3), args.fp8_experts routed experts per rank (x 3); at N > 1 the
    units are LPT-sharded with materialize: owned (no collective), weak scaling."""
    from lightcompress_amd import _native
    from lightcompress_amd.deepseekv3 import DeepseekV3
    from lightcompress_amd.pipeline import build_algo
    E = args.fp8_experts * world
    config = fp8_rtn_config(world)

    def build(n_layers, seed):
        return DeepseekV3(config, device=dev, dtype=torch.float8_e4m3fn,
                          hf_config=dsv3_config(n_layers, E),
                          random_init={'seed': seed, 'std': 0.02})

    wm = build(1, 7)   # warm-up: one layer through the same path
    walgo = build_algo(wm, config, None)
    walgo.deploy('vllm_quant')
    walgo.release()
    del wm, walgo
    free_device()
    model = build(args.steps, 77)
    algo = build_algo(model, config, None)
    mine = [(m.weight.numel()) for b in model.get_blocks()
            for m in model.get_block_linears(b).values() if not m.weight.is_meta]
    n_units, elems = len(mine), float(sum(mine))
    fwd_w = [(m.weight.data, m.weight_scale_inv.data)
             for n, m in model.get_block_linears(model.get_blocks()[0]).items()
             if '.experts.' in n and not m.weight.is_meta]   # this rank's routed experts
    fwd_w = [(c.clone(), s.clone()) for c, s in fwd_w]
    timer = _native.KernelTimer()
    sync_barrier(world)
    t0 = time.perf_counter()
    with timer:
        algo.run_block_loop()
        torch.cuda.synchronize(dev)
        t_loop = time.perf_counter() - t0
        algo.deploy('vllm_quant')
    sync_barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    kern = timer.summary()
    units = torch.tensor([n_units], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(units)
    out = {'linears_per_s': round(units.item() / elapsed, 1),
           'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'steps': args.steps,
           'block_loop_ms_per_step': round(t_loop / args.steps * 1e3, 3),
           'deploy_ms_per_step': round((elapsed - t_loop) / args.steps * 1e3, 3),
           'warmup': 1, 'mode': algo.parallel_mode(),
           'workload': (f'DeepSeek-V3 MoE layers (MLA + shared expert + {E} routed experts of '
                        f'2048x7168 / 7168x2048), block-fp8 checkpoint layout, data-free RTN '
                        f'e4m3 per-tensor W+A (rtn_fp8.yml per_tensor) through algo.deploy('
                        f"'vllm_quant'); {args.fp8_experts} experts x 3 linears per rank per "
                        f'layer, 1 layer per step'),
           'linears_per_rank': n_units,
           'lcq_kernels': kernel_table(kern, elapsed)}
    t = kern.get('lcq_fp8_block_to_tensor_many')
    if t:
        # algorithmic bytes: 1 B fp8 read + 1 B fp8 written per weight element
        gbs = elems * 2.0 / (t['total_ms'] * 1e-3) / 1e9
        traffic, src = pmc_traffic('fp8', ('k_bmax16_many', 'k_requant16_many'))
        out['roofline'] = {'kernel': 'lcq_fp8_block_to_tensor_many (k_bmax16_many + '
                                     'k_requant16_many)', 'bound': 'hbm',
                           'achieved': round(gbs, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                           'frac': round(gbs / PEAK_HBM_GBS, 4), 'traffic': traffic,
                           'traffic_source': src, 'avg_launch_ms': round(t['avg_ms'], 4),
                           'algorithmic_bytes_per_launch': elems * 2.0 / t['launches']}
    algo.release()
    del algo, model
    free_device()
    out['calib_forward'] = bench_fp8_forward(args, fwd_w, dev, world)
    return out


def _fp8_expert_list(weights, dev):
    """An ExpertList (deepseekv3.py) of DeepseekV3MLP experts whose gate / up / down are
    LlmcFp8Linear modules holding `weights` (consecutive (w, scale_inv) triples)."""
    from transformers.models.deepseek_v3 import modeling_deepseek_v3 as md

    from lightcompress_amd.deepseekv3 import ExpertList
    from lightcompress_amd.module_utils import LlmcFp8Linear
    inter, H = weights[0][0].shape
    cfg = md.DeepseekV3Config(hidden_size=H, intermediate_size=inter, hidden_act='silu')
    experts = ExpertList()
    for e in range(len(weights) // 3):
        with torch.device('meta'):
            mlp = md.DeepseekV3MLP(cfg, intermediate_size=inter)
        for p, (w, s) in zip(('gate_proj', 'up_proj', 'down_proj'), weights[3 * e:3 * e + 3]):
            m = LlmcFp8Linear(w.shape[1], w.shape[0], False, 128)
            m.weight = torch.nn.Parameter(w, requires_grad=False)
            m.weight_scale_inv = torch.nn.Parameter(s, requires_grad=False)
            setattr(mlp, p, m)
        experts.append(mlp)
    return experts.to(dev)


def bench_fp8_forward(args, weights, dev, world):
    """Calibration forward of the routed block-fp8 experts of a DeepSeek-V3 MoE layer
    (the experts call of DeepseekV3MoE.forward -> per expert LlmcFp8Linear.forward =
    block_wise_fp8_forward_func, module_utils.py:41-46, 244-262: act_quant + the block-scaled
    fp8 GEMM, kernel.py:141-242): the rank's args.fp8_experts routed experts (32: DSv3's 256
    over 8 ranks, EP-style), args.fp8_tokens x E / 8 tokens routed top-8 (args.fp8_tokens
    = 2048 tokens per expert on average, ragged: a 128 x 512-token calibration batch over
    256 experts), through ExpertList's grouped path (one lcq_fp8_gemm_grouped launch per
    projection). The reference's per-expert loop over the same
    routing is timed beside it (`loop`). Every rank runs its own experts (weak scaling);
    linears_per_s is the job total over ranks.
    Roofline: 2 * rows * N * K flops per lcq_fp8_gemm_grouped launch (rows = tokens x top-k)
    over its HIP-event time vs the fp8 dense peak."""
    from lightcompress_amd import _native
    E = len(weights) // 3
    k = min(8, E)
    T = args.fp8_tokens * E // k
    experts = _fp8_expert_list(weights, dev)
    inter, H = weights[0][0].shape
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(T, H, device=dev, generator=g).to(torch.bfloat16)
    idx = torch.argsort(torch.rand(T, E, device=dev, generator=g), dim=1)[:, :k].contiguous()
    w = torch.softmax(torch.randn(T, k, device=dev, generator=g), dim=1)
    assert experts._grouped_fp8_ok(x), 'grouped fp8 expert path not taken'

    def run(grouped):
        if not grouped:
            experts._grouped_fp8_ok = lambda x: False   # the reference's per-expert loop
        try:
            experts(x, idx, w)
            timer = _native.KernelTimer()
            sync_barrier(world)
            t0 = time.perf_counter()
            with timer:
                for _ in range(args.steps):
                    experts(x, idx, w)
            sync_barrier(world)
            return max_over_ranks(time.perf_counter() - t0, world, dev), timer.summary()
        finally:
            experts.__dict__.pop('_grouped_fp8_ok', None)

    loop_elapsed, _ = run(False)
    elapsed, kern = run(True)
    flops = 2.0 * T * k * 3 * inter * H   # per step: gate, up, down over all routed rows
    out = {'linears_per_s': round(3 * E * args.steps * world / elapsed, 1),
           'ms_per_step': round(elapsed / args.steps * 1e3, 3),
           'loop_ms_per_step': round(loop_elapsed / args.steps * 1e3, 3),
           'workload': (f'{E} DSv3 block-fp8 routed experts (gate/up {inter}x{H}, down '
                        f'{H}x{inter}) per rank, {T} bf16 tokens routed top-{k} '
                        f'(~{T * k // E} per expert): ExpertList forward, grouped (loop = the '
                        'per-expert act_quant + fp8 GEMM loop)'),
           'lcq_kernels': kernel_table(kern, elapsed)}
    t = kern.get('lcq_fp8_gemm_grouped')
    if t:
        tf = flops * args.steps / (t['total_ms'] * 1e-3) / 1e12
        traffic, src = pmc_traffic('fp8', 'k_fp8_gemm2_grouped')
        out['roofline'] = {'kernel': 'lcq_fp8_gemm_grouped (k_fp8_gemm2_grouped: 256x256 '
                                     'tiles of every expert in one launch)', 'bound': 'mfma',
                           'achieved': round(tf, 1), 'peak': PEAK_FP8_TFLOPS, 'unit': 'TFLOP/s',
                           'frac': round(tf / PEAK_FP8_TFLOPS, 4), 'traffic': traffic,
                           'traffic_source': src,
                           'flops_per_launch': flops * args.steps / t['launches'],
                           'avg_launch_ms': round(t['avg_ms'], 4)}
    return out


def launch_ranks(n: int, limit_s: float = 0.0) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1 rendezvous) and wait. This
    process never touches the GPU (children are fresh interpreters, no exec of a GPU process);
    rank 0 prints the JSON line. Returns the first non-zero child exit code (others killed), or
    124 when ranks are still running after `limit_s` seconds (all killed, the stragglers
    named)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = {}
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs[r] = subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__),
                                     *sys.argv[1:]], env=env)
    rc = 0
    t0 = time.time()
    try:
        while procs:
            if limit_s and time.time() - t0 > limit_s:
                print(f'bench.py: ranks {sorted(procs)} still running after {limit_s:.0f} s: '
                      'killing every rank', file=sys.stderr, flush=True)
                return 124
            for r, p in list(procs.items()):
                code = p.poll()
                if code is None:
                    continue
                del procs[r]
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs.values():
                        q.terminate()
            time.sleep(0.2)
    finally:
        for q in procs.values():
            q.kill()
        for q in procs.values():
            q.wait()
    return rc


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus, args.rank_timeout))
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    if world != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}: launch with torchrun '
                         f'--nproc-per-node {args.gpus}, or without a launcher (bench.py starts '
                         'the ranks itself)')
    # one process per GPU (RCCL). LCQ_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
    # (ranks then share devices round-robin); the driver's runs use the default.
    backend = os.environ.get('LCQ_DIST_BACKEND', 'nccl')
    ndev = torch.cuda.device_count()
    if backend == 'nccl' and world > ndev:
        raise SystemExit(f'{world} ranks need {world} GPUs ({ndev} visible)')
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)
    from lightcompress_amd import _native
    _native.load()

    # the headline first, on a cold chip (the side legs heat it: a warm MI355X holds a lower
    # MFMA clock, measured ~4 % on this step after the FP8 and GPTQ legs)
    awq_first = args.algo in ('awq', 'both', 'all')
    fallbacks = {}
    take_linear_fallbacks()
    if awq_first:
        elapsed, kern, mode, clock, coll = bench_awq(args, rank, world, dev)
        fallbacks['awq'] = take_linear_fallbacks()
    fp8 = bench_fp8(args, rank, world, dev) if args.algo in ('fp8', 'all') else None
    if fp8 is not None:
        fallbacks['fp8'] = take_linear_fallbacks()
    if args.algo == 'fp8':
        if rank == 0:
            print(json.dumps({'metric': 'FP8 expert linears quantized/sec (DSv3 MoE, e4m3 '
                              'per-tensor)', 'value': fp8['linears_per_s'], 'unit': 'linears/s',
                              'n_gpus': world, 'fp8': fp8}))
        if world > 1:
            dist.destroy_process_group()
        return
    gptq = bench_gptq(args, rank, world, dev) if args.algo in ('gptq', 'both', 'all') else None
    if gptq is not None:
        fallbacks['gptq'] = take_linear_fallbacks()
    if args.algo == 'gptq':
        if rank == 0:
            print(json.dumps({'metric': 'linear-layers quantized/sec (Llama-3-8B GPTQ w4a16 '
                              'g128 act-order)', 'value': gptq['linears_per_s'],
                              'unit': 'linears/s', 'n_gpus': world, 'gptq': gptq}))
        if world > 1:
            dist.destroy_process_group()
        return

    if not awq_first:
        elapsed, kern, mode, clock, coll = bench_awq(args, rank, world, dev)
        fallbacks['awq'] = take_linear_fallbacks()
    linears = N_LINEARS_PER_BLOCK * args.steps * world
    value = linears / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    l70b = None
    if not args.no_l70b and args.algo == 'all':
        l70b = bench_l70b(args, rank, world, dev)
        fallbacks['l70b'] = take_linear_fallbacks()

    e2e = None
    if not args.no_e2e and args.algo == 'all':
        e2e = {'awq': bench_e2e(args, rank, world, dev, 'awq'),
               'gptq': bench_e2e(args, rank, world, dev, 'gptq')}
        if not args.no_stream:
            # the same two runs with the model host-resident, streamed block by block
            e2e['awq_stream'] = bench_e2e(args, rank, world, dev, 'awq', 'stream')
            e2e['gptq_stream'] = bench_e2e(args, rank, world, dev, 'gptq', 'stream')
        fallbacks['e2e'] = take_linear_fallbacks()

    if rank == 0:
        roofline = gemm_roofline(kern, elapsed)
        if roofline and clock and clock.get('mean'):
            # informative: the dense peak scaled to the GFX clock held over the timed region
            # (MI355X_MICROARCH.md's 2.5 PF is quoted at 2.4 GHz); `frac` stays against 2.5 PF
            at_clk = PEAK_BF16_TFLOPS * clock['mean'] / 2400.0
            roofline['peak_at_sampled_clock'] = round(at_clk, 1)
            roofline['frac_at_sampled_clock'] = round(roofline['achieved'] / at_clk, 4)
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            cpu = cpu_baseline_awq(args, args.cpu_budget_s)
            if gptq is not None:
                gptq['cpu_baseline'] = cpu_baseline_gptq(args, args.cpu_budget_s * 0.75)
        line = {
            'metric': 'linear-layers quantized/sec (Llama-3-8B AWQ w4a16 g128)',
            'value': round(value, 3), 'unit': 'linears/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 2),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'bf16',
            'data': 'synthetic (random-init Llama-3-8B blocks, log-normal-channel activations)',
            'config': {'workload': 'Llama-3-8B AWQ w4a16 g128 sym, weight_clip, v2, '
                                   f'{args.n_samples}x{args.seq_len} calib tokens, vLLM int4 '
                                   'pack; 1 step = 1 decoder block (7 linears) per GPU',
                       'model': 'Llama-3-8B (4096/14336, 32q/8kv heads)',
                       'global_batch': args.n_samples, 'seq_len': args.seq_len,
                       'parallelism': (f'run_block_loop {mode}: {args.steps} blocks per GPU '
                                       f'x {world} GPU(s)' + ('' if world == 1 else
                                       '; materialize: owned (each rank allocates and packs '
                                       'its own blocks only), ring hand-off of the block '
                                       'activations over the edge pairs'))},
            'e2e': e2e,
            'l70b': l70b,
            'gptq': gptq,
            'fp8': fp8,
            'roofline': roofline,
            'auto_clip_roofline': clip_roofline(kern),
            'gpu_sclk_mhz': clock,
            'collective_mb_per_block': coll,
            'lcq_kernels': kernel_table(kern, elapsed),
            'cpu_baseline': cpu,
            # lcq_linear calls per leg that fell back to torch's F.linear (vendor BLAS): {}
            # means every projection of every leg ran on the lcq GEMM
            'linear_fallbacks': fallbacks,
        }
        try:
            import psutil
            line['child_processes_at_exit'] = len(psutil.Process().children(recursive=True))
        except ImportError:
            pass
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
