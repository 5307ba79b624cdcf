"""In-tree build of the HIP C-ABI library ``lightcompress_amd/_lib/liblcq.so`` for gfx950.

Plain ``hipcc`` (no cmake, no torch JIT cache): every ``csrc/*.hip`` is compiled to an object
under ``build/`` and linked into one shared library that travels with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / 'csrc'
INCLUDE = ROOT / 'include'
BUILD = ROOT / 'build' / 'lcq'
LIB_DIR = PKG / '_lib'
LIB = LIB_DIR / 'liblcq.so'

HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
CFLAGS = ['-O3', '-fPIC', '-std=c++17', f'--offload-arch={ARCH}', '-Wall',
          '-Wno-unused-function', '-Wno-unused-variable', '-ffp-contract=off',
          f'-I{INCLUDE}', f'-I{CSRC}']


def _needs(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _compile(src: Path, headers, build_dir: Path = BUILD, defines=()) -> Path:
    obj = build_dir / (src.stem + '.o')
    if _needs(obj, [src, *headers]):
        cmd = [HIPCC, *CFLAGS, *[f'-D{d}' for d in defines], '-c', str(src), '-o', str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}')
    return obj


def build(verbose: bool = False, defines=(), lib: Path = LIB, build_dir: Path = BUILD) -> Path:
    """Compile every csrc/*.hip and link ``lib``. ``defines`` (``NAME=VALUE`` strings) are for
    probe builds only (scripts/probe_build.py: a separate build_dir and library, loaded through
    LCQ_LIB_PATH); the product library is always built without them."""
    build_dir.mkdir(parents=True, exist_ok=True)
    lib.parent.mkdir(parents=True, exist_ok=True)
    sources = sorted(CSRC.glob('*.hip'))
    headers = sorted(CSRC.glob('*.h')) + sorted(INCLUDE.glob('*.h'))
    jobs = min(len(sources), int(os.environ.get('MAX_JOBS', '8')))
    with cf.ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, headers, build_dir, defines), sources))
    if _needs(lib, objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', str(lib), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
    if verbose:
        print(f'built {lib}')
    return lib


if __name__ == '__main__':
    build(verbose=True)
    sys.exit(0)
