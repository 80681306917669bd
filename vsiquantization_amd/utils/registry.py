"""Name -> class plugin registry (reference: utils/registry.py:2-27).

`QuantizationManager` instantiates quantizers/observers purely by these names
(quantizers/quantization_manager.py:41-42), so registering the MI355X classes
under the reference's names is the whole drop-in mechanism.
"""
CLASS_REGISTRY = {}


def register_class(cls):
    """Class decorator: ``CLASS_REGISTRY[cls.__name__] = cls`` and return the class unchanged."""
    CLASS_REGISTRY[cls.__name__] = cls
    return cls
