"""vsiquantization_amd — MI355X-native (gfx950) fake-quantization hot path of
tranngocduvnvp/VSIQuantization behind the reference's own plugin API.

Importing the package registers the quantizer/observer classes by name in
``vsiquantization_amd.utils.registry.CLASS_REGISTRY``:

  UniformQuantizer, MinMaxObserver                  (reference names, same behaviour)
  LSQQuantizer, LSQObserver                         (names the reference README advertises)
  PerChannelUniformQuantizer, PerChannelMinMaxObserver  (per-channel, axis 0)

plus ``LSQFakeQuantize`` (quantizers/lsq_module.py, the torch.ao-based LSQ module).
All fake-quant arithmetic runs in the HIP kernels of ``csrc/`` through the C ABI of
``include/vsiq.h``; CPU float32 tensors run the same
library's native host loops (``host.py``, ``vsiq_host_*``), never the test oracle.
"""
import torch  # noqa: F401  (must be imported before the HIP library is loaded)

from .utils.registry import CLASS_REGISTRY, register_class  # noqa: F401
from .quantizers.base import BaseQuantizer  # noqa: F401
from .observers.base import BaseObserver  # noqa: F401
from .quantizers.uniform import UniformQuantizer, ScaleGradient, RoundStraightThrough  # noqa: F401
from .quantizers.lsq import LSQQuantizer  # noqa: F401
from .quantizers.per_channel import PerChannelUniformQuantizer  # noqa: F401
from .observers.minmax import MinMaxObserver  # noqa: F401
from .observers.minmax import LSQObserver  # noqa: F401
from .observers.per_channel import PerChannelMinMaxObserver  # noqa: F401
from .quantizers.quantization_manager import QuantizationManager  # noqa: F401
from .quantizers.fake_quantize import FakeQuantize  # noqa: F401
from .quantizers.lsq_module import LSQFakeQuantize  # noqa: F401
from .quantizers.foreach import enable_multi_tensor_weights, quantize_weights_multi  # noqa: F401
from .quantizers.deferred import bundle_qparams, enable_deferred_qparam_grads  # noqa: F401
from .utils.quantize_manager import (disable_model_launches, enable_model_launches,  # noqa: F401
                                     model_launches_enabled)

__version__ = "0.1.0"
