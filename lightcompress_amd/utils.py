"""Config plumbing for the YAML-driven pipeline (llmc/__main__.py:180-268, utils/utils.py).

``AttrDict`` plays the role of the reference's EasyDict: nested dict with attribute access,
so algorithm code can use ``cfg.quant.special`` and ``cfg['quant']['special']`` alike.
"""
from __future__ import annotations

import os
import random

import yaml


class AttrDict(dict):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        for k, v in list(self.items()):
            self[k] = _wrap(v)

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = _wrap(v)

    def __setitem__(self, k, v):
        super().__setitem__(k, _wrap(v))

    def __deepcopy__(self, memo):
        import copy
        return AttrDict({k: copy.deepcopy(v, memo) for k, v in self.items()})


def _wrap(v):
    if isinstance(v, dict) and not isinstance(v, AttrDict):
        return AttrDict(v)
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


def load_config(path_or_dict) -> AttrDict:
    if isinstance(path_or_dict, (dict, AttrDict)):
        cfg = AttrDict(path_or_dict)
    else:
        with open(path_or_dict) as f:
            cfg = AttrDict(yaml.safe_load(f))
    check_config(cfg)
    return cfg


def check_config(cfg: AttrDict):
    """The hot-path subset of llmc/utils/utils.py:21-53 (check_config)."""
    q = cfg.get('quant', {})
    if 'method' in q and 'weight' in q:
        w = q['weight']
        if w.get('granularity') == 'per_group':
            assert 'group_size' in w, 'per_group weight quantization needs group_size'
        q.setdefault('modality', 'language')
    return cfg


def seed_all(seed: int):
    import numpy as np
    import torch
    random.seed(seed)
    os.environ['PYTHONHASHSEED'] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def world():
    """(rank, world_size, local_rank) from torchrun env (defaults for a single process)."""
    return (int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)),
            int(os.environ.get('LOCAL_RANK', 0)))
