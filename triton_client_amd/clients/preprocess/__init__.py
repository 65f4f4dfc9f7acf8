"""Preprocessors (re-exported; implementations live next to their clients)."""
from ..detectron_client import FCOSpreprocess  # noqa: F401
from ..detector_3d_client import PointpillarPreprocess, det3DPreprocess  # noqa: F401
from ..yolov5_client import Yolov5preprocess  # noqa: F401
