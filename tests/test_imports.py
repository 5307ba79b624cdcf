"""Every module of the package and the oracle imports on CPU (no GPU, no compute calls)."""
import importlib
import pkgutil

import lightcompress_amd


def test_import_all_package_modules():
    names = [m.name for m in pkgutil.walk_packages(lightcompress_amd.__path__, 'lightcompress_amd.')]
    assert names
    for n in names:
        importlib.import_module(n)


def test_import_oracle_and_bench():
    for n in ('oracle.quant_ref', 'oracle.gptq_ref', 'oracle.awq_ref', 'oracle.fp8_ref', 'bench',
              '__graft_entry__'):
        importlib.import_module(n)
