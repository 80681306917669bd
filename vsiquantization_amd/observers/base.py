"""Abstract observer API (reference: observers/base.py:5-41).

Plain ABC (not an nn.Module).  Observers are built positionally as
``Observer(symmetric)`` (quantization_manager.py:42).
"""
from abc import ABC, abstractmethod


class BaseObserver(ABC):
    @abstractmethod
    def observe(self, x):
        """Update the running statistics from ``x``."""

    @abstractmethod
    def get_scale_zero_point(self):
        """Return ``(scale, zero_point)`` from the collected statistics."""
