"""KServe-v2 / Triton gRPC protocol messages, built at run time.

The reference imports ``tritonclient.grpc.service_pb2`` / ``model_config_pb2``
(``communicator/channel/grpc_channel.py:3-5``, ``clients/base_client.py:3``);
neither ``tritonclient`` nor ``protoc`` exists here, so the message types are
declared as ``FileDescriptorProto``s and materialised with the protobuf
runtime.  Package, message names and field numbers follow Triton's
``grpc_service.proto`` and ``model_config.proto`` so the bytes on the wire are
interchangeable with a real Triton server/client.  Only the subset the
framework uses is declared; unknown fields from a real server are preserved
by protobuf.

Usage mirrors the generated modules::

    from triton_client_amd.proto import service_pb2 as pb, model_config_pb2 as mc
    req = pb.ModelInferRequest(model_name="YOLOv5nCOCO")
    mc.ModelInput.FORMAT_NCHW
"""
from __future__ import annotations

import types
from typing import Dict, List, Optional, Sequence, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
T_DOUBLE, T_FLOAT, T_INT64, T_UINT64, T_INT32 = F.TYPE_DOUBLE, F.TYPE_FLOAT, F.TYPE_INT64, F.TYPE_UINT64, F.TYPE_INT32
T_BOOL, T_STRING, T_MSG, T_BYTES, T_UINT32, T_ENUM = F.TYPE_BOOL, F.TYPE_STRING, F.TYPE_MESSAGE, F.TYPE_BYTES, F.TYPE_UINT32, F.TYPE_ENUM
OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
PKG = "inference"

_POOL = descriptor_pool.DescriptorPool()


def _field(m, name, num, typ, label=OPT, type_name=None, oneof=None):
    f = m.field.add()
    f.name, f.number, f.type, f.label = name, num, typ, label
    if type_name:
        f.type_name = type_name if type_name.startswith(".") else f".{PKG}.{type_name}"
    if oneof is not None:
        f.oneof_index = oneof
    return f


def _map(m, name, num, key_type, value_type, value_type_name=None):
    entry = m.nested_type.add()
    entry.name = "".join(p.capitalize() for p in name.split("_")) + "Entry"
    entry.options.map_entry = True
    _field(entry, "key", 1, key_type)
    _field(entry, "value", 2, value_type, type_name=value_type_name)
    _field(m, name, num, T_MSG, REP, type_name=f"{m.name}.{entry.name}" if "." not in m.name else None)
    return entry


def _enum(parent, name, values: Sequence[Tuple[str, int]]):
    e = parent.enum_type.add()
    e.name = name
    for n, v in values:
        ev = e.value.add()
        ev.name, ev.number = n, v
    return e


def _model_config_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="model_config.proto", package=PKG, syntax="proto3")
    _enum(fd, "DataType", [("TYPE_INVALID", 0), ("TYPE_BOOL", 1), ("TYPE_UINT8", 2), ("TYPE_UINT16", 3),
                           ("TYPE_UINT32", 4), ("TYPE_UINT64", 5), ("TYPE_INT8", 6), ("TYPE_INT16", 7),
                           ("TYPE_INT32", 8), ("TYPE_INT64", 9), ("TYPE_FP16", 10), ("TYPE_FP32", 11),
                           ("TYPE_FP64", 12), ("TYPE_STRING", 13), ("TYPE_BF16", 14)])
    m = fd.message_type.add(name="ModelTensorReshape")
    _field(m, "shape", 1, T_INT64, REP)

    m = fd.message_type.add(name="ModelInput")
    _enum(m, "Format", [("FORMAT_NONE", 0), ("FORMAT_NHWC", 1), ("FORMAT_NCHW", 2)])
    _field(m, "name", 1, T_STRING)
    _field(m, "data_type", 2, T_ENUM, type_name="DataType")
    _field(m, "format", 3, T_ENUM, type_name="ModelInput.Format")
    _field(m, "dims", 4, T_INT64, REP)
    _field(m, "reshape", 5, T_MSG, type_name="ModelTensorReshape")
    _field(m, "is_shape_tensor", 6, T_BOOL)
    _field(m, "allow_ragged_batch", 7, T_BOOL)
    _field(m, "optional", 8, T_BOOL)

    m = fd.message_type.add(name="ModelOutput")
    _field(m, "name", 1, T_STRING)
    _field(m, "data_type", 2, T_ENUM, type_name="DataType")
    _field(m, "dims", 3, T_INT64, REP)
    _field(m, "label_filename", 4, T_STRING)
    _field(m, "reshape", 5, T_MSG, type_name="ModelTensorReshape")
    _field(m, "is_shape_tensor", 6, T_BOOL)

    m = fd.message_type.add(name="ModelInstanceGroup")
    _enum(m, "Kind", [("KIND_AUTO", 0), ("KIND_GPU", 1), ("KIND_CPU", 2), ("KIND_MODEL", 3)])
    _field(m, "name", 1, T_STRING)
    _field(m, "count", 2, T_INT32)
    _field(m, "gpus", 3, T_INT32, REP)
    _field(m, "kind", 4, T_ENUM, type_name="ModelInstanceGroup.Kind")
    _field(m, "profile", 5, T_STRING, REP)
    _field(m, "passive", 7, T_BOOL)

    m = fd.message_type.add(name="ModelDynamicBatching")
    _field(m, "preferred_batch_size", 1, T_INT32, REP)
    _field(m, "max_queue_delay_microseconds", 2, T_UINT64)
    _field(m, "preserve_ordering", 3, T_BOOL)

    m = fd.message_type.add(name="ModelParameter")
    _field(m, "string_value", 1, T_STRING)

    m = fd.message_type.add(name="ModelEnsembling")
    step = m.nested_type.add(name="Step")
    _field(step, "model_name", 1, T_STRING)
    _field(step, "model_version", 2, T_INT64)
    e = step.nested_type.add(name="InputMapEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_STRING)
    _field(step, "input_map", 3, T_MSG, REP, type_name="ModelEnsembling.Step.InputMapEntry")
    e = step.nested_type.add(name="OutputMapEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_STRING)
    _field(step, "output_map", 4, T_MSG, REP, type_name="ModelEnsembling.Step.OutputMapEntry")
    _field(m, "step", 1, T_MSG, REP, type_name="ModelEnsembling.Step")

    m = fd.message_type.add(name="ModelConfig")
    _field(m, "name", 1, T_STRING)
    _field(m, "platform", 2, T_STRING)
    _field(m, "max_batch_size", 4, T_INT32)
    _field(m, "input", 5, T_MSG, REP, type_name="ModelInput")
    _field(m, "output", 6, T_MSG, REP, type_name="ModelOutput")
    _field(m, "instance_group", 7, T_MSG, REP, type_name="ModelInstanceGroup")
    _field(m, "default_model_filename", 8, T_STRING)
    m.oneof_decl.add(name="scheduling_choice")
    _field(m, "dynamic_batching", 11, T_MSG, type_name="ModelDynamicBatching", oneof=0)
    _field(m, "ensemble_scheduling", 15, T_MSG, type_name="ModelEnsembling", oneof=0)
    e = m.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="ModelParameter")
    _field(m, "parameters", 14, T_MSG, REP, type_name="ModelConfig.ParametersEntry")
    _field(m, "backend", 17, T_STRING)
    return fd


def _param_map(m, num):
    e = m.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="InferParameter")
    full = m.name
    return _field(m, "parameters", num, T_MSG, REP, type_name=f"{_PARENT.get(id(m), '')}{full}.ParametersEntry")


_PARENT: Dict[int, str] = {}


def _service_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="grpc_service.proto", package=PKG, syntax="proto3",
                                            dependency=["model_config.proto"])
    add = fd.message_type.add
    add(name="ServerLiveRequest")
    _field(add(name="ServerLiveResponse"), "live", 1, T_BOOL)
    add(name="ServerReadyRequest")
    _field(add(name="ServerReadyResponse"), "ready", 1, T_BOOL)
    m = add(name="ModelReadyRequest")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_STRING)
    _field(add(name="ModelReadyResponse"), "ready", 1, T_BOOL)
    add(name="ServerMetadataRequest")
    m = add(name="ServerMetadataResponse")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_STRING)
    _field(m, "extensions", 3, T_STRING, REP)
    m = add(name="ModelMetadataRequest")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_STRING)
    m = add(name="ModelMetadataResponse")
    tm = m.nested_type.add(name="TensorMetadata")
    _field(tm, "name", 1, T_STRING)
    _field(tm, "datatype", 2, T_STRING)
    _field(tm, "shape", 3, T_INT64, REP)
    _field(m, "name", 1, T_STRING)
    _field(m, "versions", 2, T_STRING, REP)
    _field(m, "platform", 3, T_STRING)
    _field(m, "inputs", 4, T_MSG, REP, type_name="ModelMetadataResponse.TensorMetadata")
    _field(m, "outputs", 5, T_MSG, REP, type_name="ModelMetadataResponse.TensorMetadata")

    m = add(name="InferParameter")
    m.oneof_decl.add(name="parameter_choice")
    _field(m, "bool_param", 1, T_BOOL, oneof=0)
    _field(m, "int64_param", 2, T_INT64, oneof=0)
    _field(m, "string_param", 3, T_STRING, oneof=0)
    _field(m, "double_param", 4, T_DOUBLE, oneof=0)
    _field(m, "uint64_param", 5, T_UINT64, oneof=0)

    m = add(name="InferTensorContents")
    _field(m, "bool_contents", 1, T_BOOL, REP)
    _field(m, "int_contents", 2, T_INT32, REP)
    _field(m, "int64_contents", 3, T_INT64, REP)
    _field(m, "uint_contents", 4, T_UINT32, REP)
    _field(m, "uint64_contents", 5, T_UINT64, REP)
    _field(m, "fp32_contents", 6, T_FLOAT, REP)
    _field(m, "fp64_contents", 7, T_DOUBLE, REP)
    _field(m, "bytes_contents", 8, T_BYTES, REP)

    def tensor_msg(parent, name, parent_full):
        t = parent.nested_type.add(name=name)
        _field(t, "name", 1, T_STRING)
        return t

    m = add(name="ModelInferRequest")
    t = m.nested_type.add(name="InferInputTensor")
    _field(t, "name", 1, T_STRING)
    _field(t, "datatype", 2, T_STRING)
    _field(t, "shape", 3, T_INT64, REP)
    e = t.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="InferParameter")
    _field(t, "parameters", 4, T_MSG, REP, type_name="ModelInferRequest.InferInputTensor.ParametersEntry")
    _field(t, "contents", 5, T_MSG, type_name="InferTensorContents")
    t = m.nested_type.add(name="InferRequestedOutputTensor")
    _field(t, "name", 1, T_STRING)
    e = t.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="InferParameter")
    _field(t, "parameters", 2, T_MSG, REP, type_name="ModelInferRequest.InferRequestedOutputTensor.ParametersEntry")
    e = m.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="InferParameter")
    _field(m, "model_name", 1, T_STRING)
    _field(m, "model_version", 2, T_STRING)
    _field(m, "id", 3, T_STRING)
    _field(m, "parameters", 4, T_MSG, REP, type_name="ModelInferRequest.ParametersEntry")
    _field(m, "inputs", 5, T_MSG, REP, type_name="ModelInferRequest.InferInputTensor")
    _field(m, "outputs", 6, T_MSG, REP, type_name="ModelInferRequest.InferRequestedOutputTensor")
    _field(m, "raw_input_contents", 7, T_BYTES, REP)

    m = add(name="ModelInferResponse")
    t = m.nested_type.add(name="InferOutputTensor")
    _field(t, "name", 1, T_STRING)
    _field(t, "datatype", 2, T_STRING)
    _field(t, "shape", 3, T_INT64, REP)
    e = t.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="InferParameter")
    _field(t, "parameters", 4, T_MSG, REP, type_name="ModelInferResponse.InferOutputTensor.ParametersEntry")
    _field(t, "contents", 5, T_MSG, type_name="InferTensorContents")
    e = m.nested_type.add(name="ParametersEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="InferParameter")
    _field(m, "model_name", 1, T_STRING)
    _field(m, "model_version", 2, T_STRING)
    _field(m, "id", 3, T_STRING)
    _field(m, "parameters", 4, T_MSG, REP, type_name="ModelInferResponse.ParametersEntry")
    _field(m, "outputs", 5, T_MSG, REP, type_name="ModelInferResponse.InferOutputTensor")
    _field(m, "raw_output_contents", 6, T_BYTES, REP)

    m = add(name="ModelStreamInferResponse")
    _field(m, "error_message", 1, T_STRING)
    _field(m, "infer_response", 2, T_MSG, type_name="ModelInferResponse")

    m = add(name="ModelConfigRequest")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_STRING)
    _field(add(name="ModelConfigResponse"), "config", 1, T_MSG, type_name="ModelConfig")

    m = add(name="StatisticDuration")
    _field(m, "count", 1, T_UINT64)
    _field(m, "ns", 2, T_UINT64)
    m = add(name="InferStatistics")
    for i, n in enumerate(("success", "fail", "queue", "compute_input", "compute_infer", "compute_output"), 1):
        _field(m, n, i, T_MSG, type_name="StatisticDuration")
    m = add(name="ModelStatistics")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_STRING)
    _field(m, "last_inference", 3, T_UINT64)
    _field(m, "inference_count", 4, T_UINT64)
    _field(m, "execution_count", 5, T_UINT64)
    _field(m, "inference_stats", 6, T_MSG, type_name="InferStatistics")
    m = add(name="ModelStatisticsRequest")
    _field(m, "name", 1, T_STRING)
    _field(m, "version", 2, T_STRING)
    _field(add(name="ModelStatisticsResponse"), "model_stats", 1, T_MSG, REP, type_name="ModelStatistics")

    m = add(name="RepositoryIndexRequest")
    _field(m, "repository_name", 1, T_STRING)
    _field(m, "ready", 2, T_BOOL)
    m = add(name="RepositoryIndexResponse")
    mi = m.nested_type.add(name="ModelIndex")
    for i, n in enumerate(("name", "version", "state", "reason"), 1):
        _field(mi, n, i, T_STRING)
    _field(m, "models", 1, T_MSG, REP, type_name="RepositoryIndexResponse.ModelIndex")
    for name in ("RepositoryModelLoadRequest", "RepositoryModelUnloadRequest"):
        m = add(name=name)
        _field(m, "repository_name", 1, T_STRING)
        _field(m, "model_name", 2, T_STRING)
    add(name="RepositoryModelLoadResponse")
    add(name="RepositoryModelUnloadResponse")

    # system shared-memory extension (Triton grpc_service.proto SystemSharedMemory*)
    m = add(name="SystemSharedMemoryStatusRequest")
    _field(m, "name", 1, T_STRING)
    m = add(name="SystemSharedMemoryStatusResponse")
    rs = m.nested_type.add(name="RegionStatus")
    _field(rs, "name", 1, T_STRING)
    _field(rs, "key", 2, T_STRING)
    _field(rs, "offset", 3, T_UINT64)
    _field(rs, "byte_size", 4, T_UINT64)
    e = m.nested_type.add(name="RegionsEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="SystemSharedMemoryStatusResponse.RegionStatus")
    _field(m, "regions", 1, T_MSG, REP, type_name="SystemSharedMemoryStatusResponse.RegionsEntry")
    m = add(name="SystemSharedMemoryRegisterRequest")
    _field(m, "name", 1, T_STRING)
    _field(m, "key", 2, T_STRING)
    _field(m, "offset", 3, T_UINT64)
    _field(m, "byte_size", 4, T_UINT64)
    add(name="SystemSharedMemoryRegisterResponse")
    m = add(name="SystemSharedMemoryUnregisterRequest")
    _field(m, "name", 1, T_STRING)
    add(name="SystemSharedMemoryUnregisterResponse")

    # device shared-memory extension (Triton grpc_service.proto CudaSharedMemory*; on this
    # framework the handle is a HIP IPC memory handle of a device allocation, server/shm.py)
    m = add(name="CudaSharedMemoryStatusRequest")
    _field(m, "name", 1, T_STRING)
    m = add(name="CudaSharedMemoryStatusResponse")
    rs = m.nested_type.add(name="RegionStatus")
    _field(rs, "name", 1, T_STRING)
    _field(rs, "device_id", 2, T_UINT64)
    _field(rs, "byte_size", 3, T_UINT64)
    e = m.nested_type.add(name="RegionsEntry")
    e.options.map_entry = True
    _field(e, "key", 1, T_STRING)
    _field(e, "value", 2, T_MSG, type_name="CudaSharedMemoryStatusResponse.RegionStatus")
    _field(m, "regions", 1, T_MSG, REP, type_name="CudaSharedMemoryStatusResponse.RegionsEntry")
    m = add(name="CudaSharedMemoryRegisterRequest")
    _field(m, "name", 1, T_STRING)
    _field(m, "raw_handle", 2, T_BYTES)
    _field(m, "device_id", 3, T_INT64)
    _field(m, "byte_size", 4, T_UINT64)
    add(name="CudaSharedMemoryRegisterResponse")
    m = add(name="CudaSharedMemoryUnregisterRequest")
    _field(m, "name", 1, T_STRING)
    add(name="CudaSharedMemoryUnregisterResponse")

    svc = fd.service.add(name="GRPCInferenceService")
    for rpc, req, resp, cs, ss in SERVICE_METHODS:
        mth = svc.method.add(name=rpc, input_type=f".{PKG}.{req}", output_type=f".{PKG}.{resp}")
        mth.client_streaming, mth.server_streaming = cs, ss
    return fd


SERVICE = f"{PKG}.GRPCInferenceService"
SERVICE_METHODS = [
    # rpc, request, response, client_streaming, server_streaming
    ("ServerLive", "ServerLiveRequest", "ServerLiveResponse", False, False),
    ("ServerReady", "ServerReadyRequest", "ServerReadyResponse", False, False),
    ("ModelReady", "ModelReadyRequest", "ModelReadyResponse", False, False),
    ("ServerMetadata", "ServerMetadataRequest", "ServerMetadataResponse", False, False),
    ("ModelMetadata", "ModelMetadataRequest", "ModelMetadataResponse", False, False),
    ("ModelInfer", "ModelInferRequest", "ModelInferResponse", False, False),
    ("ModelStreamInfer", "ModelInferRequest", "ModelStreamInferResponse", True, True),
    ("ModelConfig", "ModelConfigRequest", "ModelConfigResponse", False, False),
    ("ModelStatistics", "ModelStatisticsRequest", "ModelStatisticsResponse", False, False),
    ("RepositoryIndex", "RepositoryIndexRequest", "RepositoryIndexResponse", False, False),
    ("RepositoryModelLoad", "RepositoryModelLoadRequest", "RepositoryModelLoadResponse", False, False),
    ("RepositoryModelUnload", "RepositoryModelUnloadRequest", "RepositoryModelUnloadResponse", False, False),
    ("SystemSharedMemoryStatus", "SystemSharedMemoryStatusRequest", "SystemSharedMemoryStatusResponse", False, False),
    ("SystemSharedMemoryRegister", "SystemSharedMemoryRegisterRequest", "SystemSharedMemoryRegisterResponse", False,
     False),
    ("SystemSharedMemoryUnregister", "SystemSharedMemoryUnregisterRequest", "SystemSharedMemoryUnregisterResponse",
     False, False),
    ("CudaSharedMemoryStatus", "CudaSharedMemoryStatusRequest", "CudaSharedMemoryStatusResponse", False, False),
    ("CudaSharedMemoryRegister", "CudaSharedMemoryRegisterRequest", "CudaSharedMemoryRegisterResponse", False, False),
    ("CudaSharedMemoryUnregister", "CudaSharedMemoryUnregisterRequest", "CudaSharedMemoryUnregisterResponse", False,
     False),
]


def _materialise():
    mc_fd = _model_config_file()
    sv_fd = _service_file()
    _POOL.Add(mc_fd)
    _POOL.Add(sv_fd)
    mc = types.ModuleType("model_config_pb2")
    sv = types.ModuleType("service_pb2")
    for mod, fd in ((mc, mc_fd), (sv, sv_fd)):
        for m in fd.message_type:
            desc = _POOL.FindMessageTypeByName(f"{PKG}.{m.name}")
            cls = message_factory.GetMessageClass(desc)
            setattr(mod, m.name, cls)
        for e in fd.enum_type:
            ed = _POOL.FindEnumTypeByName(f"{PKG}.{e.name}")
            setattr(mod, e.name, ed)
            for v in ed.values:
                setattr(mod, v.name, v.number)
    return mc, sv


model_config_pb2, service_pb2 = _materialise()
mc = model_config_pb2

# KServe datatype strings <-> numpy
KSERVE_TO_NP = {"BOOL": "bool", "UINT8": "uint8", "UINT16": "uint16", "UINT32": "uint32", "UINT64": "uint64",
                "INT8": "int8", "INT16": "int16", "INT32": "int32", "INT64": "int64", "FP16": "float16",
                "FP32": "float32", "FP64": "float64", "BYTES": "object"}
NP_TO_KSERVE = {v: k for k, v in KSERVE_TO_NP.items()}
CONFIG_TO_KSERVE = {"TYPE_BOOL": "BOOL", "TYPE_UINT8": "UINT8", "TYPE_UINT16": "UINT16", "TYPE_UINT32": "UINT32",
                    "TYPE_UINT64": "UINT64", "TYPE_INT8": "INT8", "TYPE_INT16": "INT16", "TYPE_INT32": "INT32",
                    "TYPE_INT64": "INT64", "TYPE_FP16": "FP16", "TYPE_FP32": "FP32", "TYPE_FP64": "FP64",
                    "TYPE_STRING": "BYTES", "TYPE_BF16": "BF16"}


def config_dtype_to_kserve(data_type: int) -> str:
    name = model_config_pb2.DataType.values_by_number[data_type].name
    return CONFIG_TO_KSERVE[name]


def parse_config_pbtxt(text: str):
    """Parse a Triton ``config.pbtxt`` (protobuf text format) into ModelConfig."""
    from google.protobuf import text_format

    cfg = model_config_pb2.ModelConfig()
    text_format.Parse(text, cfg, allow_unknown_field=True)
    return cfg
