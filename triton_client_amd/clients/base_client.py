"""Client ABC (reference ``clients/base_client.py:5-104``).

A client bundles a model family's preprocess and postprocess and knows how
to read the model's tensor contract from ``ModelMetadata`` + ``ModelConfig``.
``parse_model`` keeps the reference's image-model semantics (exactly one
3-D input in NCHW or NHWC, the batch dim ignored) and return tuple
``(input_name, [output_names], c, h, w, format, datatype)``.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

from ..proto import model_config_pb2 as mc


class Client(ABC):
    def __init__(self):
        self._clients = {}

    def register_client(self, clienttype, client):
        self._clients[clienttype] = client

    @abstractmethod
    def get_preprocess(self):
        ...

    @abstractmethod
    def get_postprocess(self):
        ...

    def parse_model(self, model_metadata, model_config):
        if len(model_metadata.inputs) != 1:
            raise Exception(f"expecting 1 input, got {len(model_metadata.inputs)}")
        if len(model_config.input) != 1:
            raise Exception(f"expecting 1 input in model configuration, got {len(model_config.input)}")
        input_metadata = model_metadata.inputs[0]
        input_config = model_config.input[0]
        shape = list(input_metadata.shape)
        if len(shape) == 4 and shape[0] in (1, -1):  # explicit batch dim (max_batch_size > 0 or reshape)
            shape = shape[1:]
        if len(shape) != 3:
            raise Exception(f"expecting input to have 3 dimensions, model '{model_metadata.name}' input has "
                            f"{len(input_metadata.shape)}")
        fmt = input_config.format
        if fmt not in (mc.ModelInput.FORMAT_NCHW, mc.ModelInput.FORMAT_NHWC):
            raise Exception("unexpected input format " + mc.ModelInput.Format.Name(fmt) + ", expecting "
                            + mc.ModelInput.Format.Name(mc.ModelInput.FORMAT_NCHW) + " or "
                            + mc.ModelInput.Format.Name(mc.ModelInput.FORMAT_NHWC))
        if fmt == mc.ModelInput.FORMAT_NHWC:
            h, w, c = shape
        else:
            c, h, w = shape
        return (input_metadata.name, [o.name for o in model_metadata.outputs], c, h, w, fmt,
                input_metadata.datatype)


def client_for_model(model_name: str, model_config=None, device="cpu") -> Client:
    """Pick the client by model family (fixes SURVEY Appendix A1: the
    reference hard-codes Yolov5client regardless of ``-m``).  ``device``: where the
    client's pre/postprocess runs (a GPU: the HIP kernels; "cpu": config 1)."""
    n = model_name.lower()
    outs = len(model_config.output) if model_config is not None else 0
    if "pointpillar" in n or "second" in n or "centerpoint" in n or (model_config is not None and len(model_config.input) == 3):
        from .detector_3d_client import Pointpillars_client
        return Pointpillars_client(device)
    if "fcos" in n or "retina" in n or "detectron" in n or n == "test_model" or outs == 4:
        from .detectron_client import FCOS_client
        return FCOS_client(device)
    if "yolov4" in n or outs == 2:
        from .yolov4_client import Yolov4client
        return Yolov4client(device)
    from .yolov5_client import Yolov5client
    return Yolov5client(device)
