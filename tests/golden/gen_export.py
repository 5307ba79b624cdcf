"""Golden quantization configs from the REAL reference's exporters
(llmc/utils/export_vllm.py, export_autoawq.py), build container only:

    python tests/golden/gen_export.py

Writes tests/golden/export_configs.json: for each case, the config.json the reference leaves
after updating a base HF config.
"""
import json
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import _ref_import as R  # noqa: E402
from export_cases import BASE, CASES  # noqa: E402
from gen_pipeline import ED  # noqa: E402


class _Model:
    def skip_layer_name(self):
        return ['lm_head']


def main():
    R.install()
    import llmc.utils.export_autoawq as ea
    import llmc.utils.export_vllm as ev
    out = {}
    for name, (kind, cfg) in CASES.items():
        with tempfile.TemporaryDirectory() as d:
            (Path(d) / 'config.json').write_text(json.dumps(BASE))
            if kind == 'vllm':
                ev.update_vllm_quant_config(_Model(), ED(cfg), d)
            else:
                ea.update_autoawq_quant_config(ED(cfg), d)
            out[name] = json.loads((Path(d) / 'config.json').read_text())
    (HERE / 'export_configs.json').write_text(json.dumps(out, indent=1, sort_keys=True))
    print(f'{len(out)} export configs written')


if __name__ == '__main__':
    main()
