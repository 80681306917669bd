from .base import BaseObserver  # noqa: F401
from .minmax import LSQObserver, MinMaxObserver  # noqa: F401
from .per_channel import PerChannelMinMaxObserver  # noqa: F401
