"""Import the reference ``llmc`` package from /root/reference, CPU-only, for fixture generation.

Used ONLY by ``tests/golden/gen_golden.py`` in the build container (the reference does not
exist on the GPU box and nothing under tests/ imports this module at test time).

Recipe: stub ``loguru``; install a meta-path finder for ``llmc.*`` that
(i) creates package modules without executing their ``__init__.py`` (which import every
algorithm) and (ii) applies in memory the same text substitutions ci_check/change_files.py
writes to disk (.cuda() -> cpu, nccl -> gloo, guarded cache calls). ``n_grid`` stays 20.
No reference source is copied anywhere.
"""
from __future__ import annotations

import importlib.abc
import importlib.machinery
import importlib.util
import os
import sys
import types
from pathlib import Path

REF_ROOT = Path(os.environ.get('LCQ_REFERENCE', '/root/reference'))

_SUBS = [
    ('.cuda()', ".to('cpu')"),
    ("torch.device('cuda')", "torch.device('cpu')"),
    ('torch.device("cuda")', 'torch.device("cpu")'),
    ("device='cuda'", "device='cpu'"),
    ("move_embed_to_device('cuda')", "move_embed_to_device('cpu')"),
    ('torch.cuda.empty_cache()', 'None'),
    ('torch.cuda.synchronize()', 'None'),
    ("backend='nccl'", "backend='gloo'"),
]


class _Logger:
    def __getattr__(self, name):
        return lambda *a, **k: None


def _stub_loguru():
    if 'loguru' not in sys.modules:
        m = types.ModuleType('loguru')
        m.logger = _Logger()
        sys.modules['loguru'] = m


class _PatchedLoader(importlib.abc.SourceLoader):
    def __init__(self, path: Path):
        self.path = path

    def get_filename(self, fullname):
        return str(self.path)

    def get_data(self, path):
        src = Path(path).read_text()
        for a, b in _SUBS:
            src = src.replace(a, b)
        return src.encode()


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path, target=None):
        if fullname != 'llmc' and not fullname.startswith('llmc.'):
            return None
        rel = Path(*fullname.split('.'))
        pkg_dir = REF_ROOT / rel
        if pkg_dir.is_dir():
            spec = importlib.machinery.ModuleSpec(fullname, None, is_package=True)
            spec.submodule_search_locations = [str(pkg_dir)]
            return spec
        file = REF_ROOT / rel.with_suffix('.py')
        if file.exists():
            return importlib.util.spec_from_loader(fullname, _PatchedLoader(file))
        return None


class _EmptyPkgLoader(importlib.abc.Loader):
    def create_module(self, spec):
        return None

    def exec_module(self, module):
        module.__path__ = list(module.__spec__.submodule_search_locations or [])


def install():
    if not REF_ROOT.exists():
        raise RuntimeError(f'reference not found at {REF_ROOT}')
    _stub_loguru()
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.insert(0, _Finder())
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('LOCAL_RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')


# package specs above have loader=None; give them an empty loader so __init__ is skipped
_orig_find = _Finder.find_spec


def _find_with_loader(self, fullname, path, target=None):
    spec = _orig_find(self, fullname, path, target)
    if spec is not None and spec.loader is None:
        locs = spec.submodule_search_locations
        spec = importlib.machinery.ModuleSpec(fullname, _EmptyPkgLoader(), is_package=True)
        spec.submodule_search_locations = locs
    return spec


_Finder.find_spec = _find_with_loader


def init_dist():
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group('gloo', rank=0, world_size=1)


def quant_module():
    install()
    import llmc.compression.quantization.quant as q
    return q


def module_utils():
    install()
    import llmc.compression.quantization.module_utils as mu
    return mu


def native_float_quantize():
    """qtorch is absent: give the reference's quant module a ``float_quantize``
    that is the native OCP Float8 RNE cast, saturating at +-finfo.max (NaN kept) -- the
    rounding lightcompress_amd's FloatQuantizer documents for use_qtorch=True.
    Everything around that one step stays the reference's own, so fixtures made this way pin
    the scales, the algorithms' control flow and every other op; the rounding step itself is
    parity-unpinned against qtorch."""
    import torch
    q = quant_module()
    fmts = {(4, 3): torch.float8_e4m3fn, (5, 2): torch.float8_e5m2}

    def float_quantize(x, exp, man, rounding='stochastic'):
        assert rounding == 'nearest', rounding
        dt = fmts[(int(exp), int(man))]
        m = torch.finfo(dt).max
        x = x.float()
        return torch.where(x.isnan(), x, x.clamp(-m, m)).to(dt).float()
    q.float_quantize = float_quantize
