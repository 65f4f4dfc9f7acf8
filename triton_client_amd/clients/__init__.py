"""Model-family clients (reference clients/__init__.py)."""
from .base_client import Client, client_for_model  # noqa: F401
from .detectron_client import FCOS_client, FCOSpostprocess, FCOSpreprocess  # noqa: F401
from .detector_3d_client import (Pointpillars_client, PointPillarPostprocess, PointpillarPreprocess,  # noqa: F401
                                 det3DPreprocess)
from .yolov5_client import Yolov5client, Yolov5postprocess, Yolov5preprocess  # noqa: F401
from .yolov4_client import Yolov4client, Yolov4postprocess, Yolov4preprocess  # noqa: F401
