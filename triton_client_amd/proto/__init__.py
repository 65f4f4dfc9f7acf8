"""KServe-v2 protocol (runtime-built Triton-compatible protobuf types)."""
from .kserve import (KSERVE_TO_NP, NP_TO_KSERVE, SERVICE, SERVICE_METHODS, config_dtype_to_kserve,  # noqa: F401
                     model_config_pb2, parse_config_pbtxt, service_pb2)
