"""Load/save golden fixtures (inputs + expected outputs) as .npz with dtype tags.

bf16 / fp8 tensors are stored as raw uint16 / uint8 views; the key suffix ``@dtype`` restores
them. Pure data — no reference code is stored here.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

GOLDEN_DIR = Path(__file__).resolve().parent

_VIEW = {torch.bfloat16: (torch.int16, 'bfloat16'),
         torch.float8_e4m3fn: (torch.uint8, 'float8_e4m3fn'),
         torch.float8_e5m2: (torch.uint8, 'float8_e5m2')}
_BACK = {'bfloat16': torch.bfloat16, 'float8_e4m3fn': torch.float8_e4m3fn,
         'float8_e5m2': torch.float8_e5m2}


def _to_np(t):
    if isinstance(t, np.ndarray):
        return t, None
    if isinstance(t, (int, float, bool)):
        return np.asarray(t), None
    t = t.detach().cpu().contiguous()
    if t.dtype in _VIEW:
        vdt, tag = _VIEW[t.dtype]
        return t.view(vdt).numpy(), tag
    return t.numpy(), None


def save(name: str, **tensors):
    arrays = {}
    for k, v in tensors.items():
        if v is None:
            continue
        a, tag = _to_np(v)
        arrays[f'{k}@{tag}' if tag else k] = a
    np.savez_compressed(GOLDEN_DIR / f'{name}.npz', **arrays)


def load(name: str) -> dict:
    out = {}
    with np.load(GOLDEN_DIR / f'{name}.npz', allow_pickle=False) as z:
        for k in z.files:
            a = z[k]
            if '@' in k:
                key, tag = k.split('@')
                out[key] = torch.from_numpy(a.copy()).view(_BACK[tag])
            else:
                out[k] = torch.from_numpy(a.copy()) if a.ndim else torch.tensor(a.item())
    return out


def names(prefix: str = '') -> list[str]:
    return sorted(p.stem for p in GOLDEN_DIR.glob(f'{prefix}*.npz'))
