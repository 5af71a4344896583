"""onebit_asr — MI355X-native BitLinear (1.58-bit QuantizedLinear) hot path for the
1.58-bit Conformer ASR training step of y00njaekim/CMU-11785-IDL-1.58bit-ASR.

Import path mirrors the reference (``from onebit_asr.conformer import ConformerASR``,
train.py:18). The BitLinear kernels live in ``libonebit_hip.so`` (C ABI:
include/onebit_hip.h), bound by ``onebit_asr._lib``.
"""
from .quant import BitLinear, QuantizedLinear, quantize_weight  # noqa: F401

__version__ = "0.1.0"
