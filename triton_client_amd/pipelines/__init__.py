"""Device-resident per-frame pipelines (one per sensor family) and the
hipGraph runner that replays a whole step with one launch."""
from .camera import CameraPipeline  # noqa: F401
from .lidar import LidarPipeline  # noqa: F401
from .graph import GraphRunner  # noqa: F401
from .centerpoint import CenterPointPipeline  # noqa: F401,E402
from .detectron import DetectronPipeline  # noqa: F401,E402
from .yolov4 import Yolov4Pipeline  # noqa: F401,E402
from .second import SecondPipeline  # noqa: F401,E402
