from .registry import CLASS_REGISTRY, register_class  # noqa: F401
