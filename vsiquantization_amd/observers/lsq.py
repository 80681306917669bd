"""LSQObserver — the observer name README.md:131 advertises but the reference never
registers.  In the reference's QAT flow an observer only feeds the
calibration statistics; the LSQ step size itself is initialised from mean(|x|)
(QuantizationManager.init_scaling_factor_for_learning, qm.py:105-112).  So
LSQObserver is MinMaxObserver's K2 pass under the README's name.
"""
from ..utils.registry import register_class
from .minmax import MinMaxObserver


@register_class
class LSQObserver(MinMaxObserver):
    pass
