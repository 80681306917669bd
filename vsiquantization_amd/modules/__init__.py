from .fused import (ConvBnReLU, ConvBn, ConvReLU, Conv, LinearBnReLU, LinearBn,  # noqa: F401
                    LinearReLU, Linear)
from .fuse import fuse_modules_unified, PATTERN_TO_FUSED  # noqa: F401
from .fuse_config import (FuseConfig, FuseConfigManager, load_fuse_config_from_yaml,  # noqa: F401
                          create_fuse_config_manager)
