"""LSQQuantizer — the name README.md:70-71,126 advertises but the reference never
registers.  It is UniformQuantizer's learnable path
(uniform.py:47-56) with a WORKING learnable asymmetric zero point: the manager
gives it a float64 zero-point Parameter (QuantizationManager.make_learn_qparameter
checks ``learns_zero_point``) instead of the int 0 that makes the reference raise.

Forward / backward arithmetic is identical to UniformQuantizer's (same HIP
kernels K1/K4); only the zero-point handling differs.
"""
from __future__ import annotations

from ..utils.registry import register_class
from .uniform import UniformQuantizer


@register_class
class LSQQuantizer(UniformQuantizer):
    def __init__(self, num_bits=8, symmetric=True):
        super().__init__(num_bits, symmetric)
        self.learns_zero_point = not symmetric

    def _int_zero_point_learnable(self, zero_point):
        # a plain number zero point is used as a fixed value (no gradient) instead of raising,
        # with the reference's clamp(round(zp), qmin, qmax) applied (uniform.py:98-102)
        return float(min(max(round(float(zero_point)), self.qmin), self.qmax))
