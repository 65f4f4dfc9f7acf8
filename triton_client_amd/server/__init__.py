"""In-process KServe-v2 server hosting the MI355X detectors."""
from .kserve_server import FaultInjector, GRPCInferenceServicer, KServeServer  # noqa: F401
from .model import EchoModel, InferError, ServedModel, tensor_spec  # noqa: F401
from .repository import FACTORIES, ModelRepository, register_factory  # noqa: F401
