"""Inference drivers (reference ``communicator/``): live ROS 2D/3D, bag
replay, evaluation — over pluggable local (MI355X) / remote (KServe) engines."""
from .bag_inference import BagInference2D, BagInference3D  # noqa: F401
from .base_inference import BaseInference  # noqa: F401
from .engines import (Detector2D, Detector3D, LocalDetector2D, LocalDetector3D, RemoteDetector2D,  # noqa: F401
                      RemoteDetector3D)
from .evaluate_inference import EvaluateInference, gt_from_msg  # noqa: F401
from .ros_inference import RosInference, decode_image_msg, detections_to_msg  # noqa: F401
from .ros_inference3d import RosInference3D, boxes_to_detection3d, boxes_to_jsk, select_boxes  # noqa: F401
