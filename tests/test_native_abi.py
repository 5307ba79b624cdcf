"""CPU checks of the C-ABI boundary: the library loads, exports every symbol include/lcq.h
declares, the ctypes signatures cover exactly that set, and host tensors are refused."""
import ctypes

import pytest
import torch

from lightcompress_amd import _native as N


@pytest.fixture(scope='module')
def lib():
    if not N.lib_path().exists():
        import __graft_entry__
        __graft_entry__.build()
    return N.load()


def test_exports_every_declared_symbol(lib):
    declared = N.header_symbols()
    assert declared, 'no symbols parsed from include/lcq.h'
    for name in declared:
        assert hasattr(lib, name), f'{name} declared in lcq.h but not exported'


def test_signatures_match_header(lib):
    assert sorted(N.SIGNATURES) == N.header_symbols()


def test_version_and_error(lib):
    assert lib.lcq_version() >= 1
    assert isinstance(lib.lcq_last_error(), bytes)


def test_bad_arguments_return_einval(lib):
    # validation happens on the host before any launch, so it is testable without a GPU
    rc = lib.lcq_int_quant_dynamic(None, N.BF16, 4, 100, 128, None, None, None, 0, 15, 0,
                                   None, 0, None, 0, None, 0, None, None, None)
    assert rc == -1
    assert b'divisible' in lib.lcq_last_error()
    rc = lib.lcq_pack_autoawq_gemm(None, N.BF16, 8, 256, 128, None, N.BF16, None, 8, None,
                                   None, None, None)
    assert rc == -1 and b'4-bit' in lib.lcq_last_error()


def test_cpu_tensor_raises():
    """No silent CPU fallback: the product path refuses host tensors."""
    from lightcompress_amd.quant import IntegerQuantizer
    wq = IntegerQuantizer(4, True, 'per_group', group_size=128)
    with pytest.raises(N.LcqError):
        wq.fake_quant_weight_dynamic(torch.zeros(8, 128, dtype=torch.bfloat16))
