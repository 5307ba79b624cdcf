"""A/B launcher: run bench.py with module switches set first (python scripts/bench_with.py
X6=0 -- <bench args>). Switches: X6 (ops.X6, the split-plane chain products)."""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from lightcompress_amd import ops  # noqa: E402

args = sys.argv[1:]
cut = args.index('--') if '--' in args else len(args)
for kv in args[:cut]:
    k, v = kv.split('=')
    if k == 'X6':
        ops.X6 = v != '0'
    else:
        raise SystemExit(f'unknown switch {k}')
sys.argv = [str(ROOT / 'bench.py')] + args[cut + 1:]
runpy.run_path(str(ROOT / 'bench.py'), run_name='__main__')
