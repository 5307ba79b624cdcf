"""Run our block driver on a golden config (tests/golden/pipeline_configs.py) the way
tests/golden/gen_pipeline.py ran the reference's: the same tiny model files, the same
calibration token ids through our Catcher, run_block_loop + deploy('fake_quant'). Returns the
reference's fixture, our deployed weights and our diagnostics (GPTQ Hessians, AWQ loss curves
and chosen scales, static act scales, v2 clip factors, saved scales.pth / clips.pth) under the
fixture's key names."""
import copy
import shutil
import tempfile

import torch

import fixtures as F
import tiny_models as TM
from pipeline_configs import CONFIGS


def run_ours(name, dev, monkeypatch=None, config_override=None, model_override=None,
             return_model=False):
    from lightcompress_amd.pipeline import build_algo, build_model
    from lightcompress_amd.utils import load_config
    spec = CONFIGS[name]
    family = spec.get('model', 'Llama')
    ref = F.load(f'pipe_{name}')
    diag = {}
    if monkeypatch is not None and spec['quant']['method'] == 'GPTQ':
        from lightcompress_amd.gptq import GPTQ
        orig = GPTQ.layer_transform

        def lt(self, layer, lname):
            diag[f'H_b{self.block_idx}__{lname.replace(".", "__")}'] = \
                self.layers_cache[lname]['acc'].H.detach().cpu().clone()
            return orig(self, layer, lname)
        orig_g = GPTQ.group_transform

        def gt(self, grp):
            for lname, _ in grp:
                diag[f'H_b{self.block_idx}__{lname.replace(".", "__")}'] = \
                    self.layers_cache[lname]['acc'].H.detach().cpu().clone()
            return orig_g(self, grp)
        monkeypatch.setattr(GPTQ, 'layer_transform', lt)
        monkeypatch.setattr(GPTQ, 'group_transform', gt)
    elif monkeypatch is not None and spec['quant']['method'] == 'Awq':
        from lightcompress_amd.awq import Awq
        orig = Awq.search_scale_subset

        def ss(self, *a, **k):
            best = orig(self, *a, **k)
            n = len([d for d in diag if d.startswith(f'S_b{self.block_idx}')])
            diag[f'S_b{self.block_idx}__{n}'] = best.detach().cpu().clone()
            diag[f'L_b{self.block_idx}__{n}'] = torch.tensor(self.last_search['losses'],
                                                             dtype=torch.float64)
            return best
        monkeypatch.setattr(Awq, 'search_scale_subset', ss)
    dtype = 'float16' if family == 'Opt' else 'bfloat16'
    quant = copy.deepcopy(spec['quant'])
    if config_override:
        quant = config_override(quant)
    sp = quant.get('special', {})
    tmp = tempfile.mkdtemp()
    if sp.get('save_scale'):
        sp['scale_path'] = f'{tmp}/scale'
    if sp.get('save_clip'):
        sp['clip_path'] = f'{tmp}/clip'
    cfg = {'model': {'type': family, 'path': str(TM.MODEL_DIRS[family]), 'torch_dtype': dtype},
           'quant': quant}
    if model_override:
        cfg['model'].update(model_override)
    if spec['calib']:
        cfg['calib'] = dict(spec['calib'])
    config = load_config(cfg)
    model = build_model(config, device=dev)
    calib = spec['calib']
    if calib is None:
        first = None
    else:
        ids = ref['ids']
        batches = ([{'input_ids': ids}] if calib['bs'] == -1 else
                   [{'input_ids': ids[i:i + 1]} for i in range(ids.shape[0])])
        first = model.collect_first_block_input(batches)
    algo = build_algo(model, config, first)
    algo.run_block_loop()
    for bi, block in enumerate(model.get_blocks()):  # v2 clip factors, before the deploy
        for ln, lin in model.get_block_linears(block).items():
            for k in ('upbound', 'lowbound'):
                f = getattr(lin, f'buf_{k}_factor', None)
                if f is not None:
                    diag[f'{k[:2]}_b{bi}__{ln.replace(".", "__")}'] = f.detach().cpu().clone()
    if sp.get('save_scale'):
        for k, v in torch.load(f'{tmp}/scale/scales.pth', weights_only=True).items():
            diag[f'sc__{k.replace(".", "__")}'] = v.cpu()
    if sp.get('save_clip'):
        for bi, d in torch.load(f'{tmp}/clip/clips.pth', weights_only=True).items():
            for k, v in d.items():
                if v is not None:
                    diag[f'cl{bi}__{k.replace(".", "__")}'] = v
    shutil.rmtree(tmp, ignore_errors=True)
    algo.deploy('fake_quant')
    got = {}
    for bi, block in enumerate(model.get_blocks()):
        for ln, lin in model.get_block_linears(block).items():
            got[f'b{bi}__{ln.replace(".", "__")}'] = lin.weight.data.detach().cpu()
            if hasattr(lin, 'buf_act_scales_0'):  # static act qparams
                diag[f'a_b{bi}__{ln.replace(".", "__")}'] = lin.buf_act_scales_0.detach().cpu()
    if return_model:
        return ref, got, diag, model
    return ref, got, diag


def compare(ref, got, n):
    """Per deployed linear: the fraction of bit-equal weight elements."""
    res = {}
    for k, w in got.items():
        r = ref[k]
        assert r.shape == w.shape and r.dtype == w.dtype, k
        eq = (r.view(torch.int16) == w.view(torch.int16)).float().mean().item()
        res[k] = eq
        print(f'{k:40s} equal {eq * 100:8.4f} %  max|dw| '
              f'{(r.float() - w.float()).abs().max().item():.3e}')
    assert len(res) == n
    return res
