"""ROS layer: message types, in-process topic bus, rospy-compatible API, bags."""
from . import bag, bus, compat, msgs  # noqa: F401
from .bag import Bag  # noqa: F401
from .bus import TopicBus, default_bus, reset_default_bus  # noqa: F401
