"""lightcompress_amd — MI355X-native weight-quantization hot path of LightCompress (llmc).

Drop-in for ``llmc.compression.quantization`` quantizers / algorithms / packers, backed by
hand-written gfx950 HIP kernels behind the C ABI in ``include/lcq.h``.
"""
from . import _native  # noqa: F401
from .quant import FloatQuantizer, IntegerQuantizer  # noqa: F401

__version__ = '0.1.0'
