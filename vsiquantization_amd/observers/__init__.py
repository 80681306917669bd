from .base import BaseObserver  # noqa: F401
from .minmax import MinMaxObserver  # noqa: F401
from .lsq import LSQObserver  # noqa: F401
from .per_channel import PerChannelMinMaxObserver  # noqa: F401
