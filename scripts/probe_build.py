"""Build a PROBE variant of liblcq.so with compile-time knobs that the product library never
reads at run time (they change tile orders or fp32 fold orders):

  LCQ_PROBE_SYRK_NS=<n>    force lcq_hessian_accum's split-K count     (csrc/hessian.hip)
  LCQ_PROBE_SYRK_GNS=<n>   force lcq_hessian_grouped's per-group splits (csrc/hessian.hip)
  LCQ_PROBE_GEMM_ORDER=1   k_gemm16b N-band-major tile order           (csrc/gemm256.hip)
  LCQ_PROBE_GEMM_PP=0      the round-4 4-barrier k_gemm16b body         (csrc/gemm256.hip)
  LCQ_PROBE_GEMM_CM=<m>    k_gemm16h XCD chunk of m x (32/m) tiles      (csrc/gemm256.hip)
  LCQ_PROBE_CHOL_IEEE_RSQ=1  IEEE sqrtf / division in the tile's S1      (csrc/chol.hip)

usage: python scripts/probe_build.py <tag> NAME=VALUE [NAME=VALUE ...]
writes scripts/_lib/liblcq_<tag>.so (objects under build/probe_<tag>/); load it in a probe
process with LCQ_LIB_PATH=scripts/_lib/liblcq_<tag>.so. Build here (CPU), run on the GPU box."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from lightcompress_amd import _build  # noqa: E402

if __name__ == '__main__':
    tag, defs = sys.argv[1], sys.argv[2:]
    assert all('=' in d and d.startswith('LCQ_PROBE_') for d in defs), defs
    _build.build(verbose=True, defines=defs, lib=ROOT / 'scripts' / '_lib' / f'liblcq_{tag}.so',
                 build_dir=ROOT / 'build' / f'probe_{tag}')
