"""Per-layer quantizer/observer selection (reference: modules/fuse_config.py:6-244).

``FuseConfig`` carries the registry NAMES of the observer/quantizer for weights
and activations plus symmetry, BN folding and bit widths; the MI355X kernels are
selected purely through those names (no schema change).  ``FuseConfigManager``
resolves a layer name against regex patterns in insertion order (``re.search``,
substring fallback for invalid patterns) and falls back to the default config.
"""
import re
from typing import Dict, Optional, Union

import yaml

_FIELDS = ("observer_w_name", "quantizer_w_name", "observer_a_name", "quantizer_a_name",
           "w_symmetric", "a_symmetric", "is_fuse_bn", "bits_w", "bits_a")


class FuseConfig:
    def __init__(self, observer_w_name: str = "MinMaxObserver", quantizer_w_name: str = "UniformQuantizer",
                 observer_a_name: str = "MinMaxObserver", quantizer_a_name: str = "UniformQuantizer",
                 w_symmetric: bool = True, a_symmetric: bool = True, is_fuse_bn: bool = True,
                 bits_w: int = 8, bits_a: int = 8):
        self.observer_w_name = observer_w_name
        self.quantizer_w_name = quantizer_w_name
        self.observer_a_name = observer_a_name
        self.quantizer_a_name = quantizer_a_name
        self.w_symmetric = w_symmetric
        self.a_symmetric = a_symmetric
        self.is_fuse_bn = is_fuse_bn
        self.bits_w = bits_w
        self.bits_a = bits_a

    def __repr__(self):
        return (f"FuseConfig(observer_w='{self.observer_w_name}', quantizer_w='{self.quantizer_w_name}', "
                f"observer_a='{self.observer_a_name}', quantizer_a='{self.quantizer_a_name}', "
                f"w_symmetric={self.w_symmetric}, a_symmetric={self.a_symmetric}, "
                f"is_fuse_bn={self.is_fuse_bn}, bits_w={self.bits_w}, bits_a={self.bits_a})")

    def as_dict(self):
        return {k: getattr(self, k) for k in _FIELDS}


class FuseConfigManager:
    def __init__(self, default_config: Optional[FuseConfig] = None):
        self.default_config = default_config or FuseConfig()
        self.layer_configs: Dict[str, FuseConfig] = {}

    def add_layer_config(self, layer_pattern: str, config: FuseConfig):
        self.layer_configs[layer_pattern] = config

    def get_config_for_layer(self, layer_name: str) -> FuseConfig:
        """First pattern (insertion order) matching ``layer_name``, else the default."""
        return next((cfg for pat, cfg in self.layer_configs.items()
                     if self._match_pattern(layer_name, pat)), self.default_config)

    @staticmethod
    def _match_pattern(layer_name: str, pattern: str) -> bool:
        try:
            return re.search(pattern, layer_name) is not None
        except re.error:
            return pattern in layer_name

    def set_default_config(self, config: FuseConfig):
        self.default_config = config

    def clear_layer_configs(self):
        self.layer_configs.clear()

    def get_all_patterns(self) -> list:
        return list(self.layer_configs)

    def __repr__(self):
        return f"FuseConfigManager(default={self.default_config}, patterns={list(self.layer_configs)})"


def load_fuse_config_from_yaml(yaml_path: str) -> FuseConfigManager:
    """YAML with optional ``default:`` and ``layers: {pattern: {...}}`` sections."""
    try:
        with open(yaml_path, "r", encoding="utf-8") as f:
            data = yaml.safe_load(f)
    except FileNotFoundError:
        raise FileNotFoundError(f"Configuration file not found: {yaml_path}")
    except yaml.YAMLError as e:
        raise ValueError(f"Invalid YAML format in {yaml_path}: {e}")
    mgr = FuseConfigManager()
    if "default" in data:
        mgr.default_config = FuseConfig(**data["default"])
    for pattern, cfg in (data.get("layers") or {}).items():
        mgr.add_layer_config(pattern, FuseConfig(**cfg))
    return mgr


def create_fuse_config_manager(default_config: Optional[FuseConfig] = None,
                               layer_configs: Optional[Dict[str, Union[FuseConfig, Dict]]] = None
                               ) -> FuseConfigManager:
    mgr = FuseConfigManager(default_config)
    for pattern, cfg in (layer_configs or {}).items():
        if isinstance(cfg, dict):
            cfg = FuseConfig(**cfg)
        elif not isinstance(cfg, FuseConfig):
            raise ValueError(f"Config for pattern '{pattern}' must be FuseConfig or dict")
        mgr.add_layer_config(pattern, cfg)
    return mgr
