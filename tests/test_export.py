"""Exporter configs (lightcompress_amd/export.py) vs the reference's (export_vllm.py,
export_autoawq.py) on the cases in tests/golden/export_cases.py; goldens made by
tests/golden/gen_export.py from the real reference."""
import json

import pytest

from export_cases import BASE, CASES
from fixtures import GOLDEN_DIR

GOLD = json.loads((GOLDEN_DIR / 'export_configs.json').read_text())


class _Model:
    def skip_layer_name(self):
        return ['lm_head']


@pytest.mark.parametrize('name', sorted(CASES))
def test_export_config_matches_reference(tmp_path, name):
    from lightcompress_amd import export
    from lightcompress_amd.utils import load_config
    kind, cfg = CASES[name]
    (tmp_path / 'config.json').write_text(json.dumps(BASE))
    c = load_config(json.loads(json.dumps(cfg)))
    if kind == 'vllm':
        export.update_vllm_quant_config(_Model(), c, str(tmp_path))
    else:
        export.update_autoawq_quant_config(c, str(tmp_path))
    assert json.loads((tmp_path / 'config.json').read_text()) == GOLD[name]
