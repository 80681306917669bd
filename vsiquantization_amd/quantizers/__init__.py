from .base import BaseQuantizer  # noqa: F401
from .uniform import UniformQuantizer, ScaleGradient, RoundStraightThrough  # noqa: F401
from .lsq import LSQQuantizer  # noqa: F401
from .per_channel import PerChannelUniformQuantizer  # noqa: F401
from .quantization_manager import QuantizationManager  # noqa: F401
from .fake_quantize import FakeQuantize  # noqa: F401
from .lsq_module import LSQFakeQuantize  # noqa: F401
