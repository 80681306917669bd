"""Abstract quantizer API (reference: quantizers/base.py:4-32).

Like the reference this is a plain ABC, not an nn.Module: the nn.Module level is
`QuantizationManager` / `FakeQuantize`.  Concrete quantizers are built
positionally as ``Quantizer(num_bits, symmetric)`` (quantization_manager.py:41).
"""
from abc import ABC, abstractmethod


class BaseQuantizer(ABC):
    @abstractmethod
    def quantize(self, x, scale, zero_point):
        """Fake-quantize ``x``: ``(clamp(round(x/scale + zp)) - zp) * scale``."""
