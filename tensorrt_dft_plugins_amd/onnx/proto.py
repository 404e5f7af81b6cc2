"""Minimal ONNX protobuf schema, built at runtime with ``google.protobuf`` descriptors.

The ``onnx`` package is not available (and not needed): the reference relies on TensorRT's
ONNX parser (/root/reference/tests/test_dft.py:89-101); here the ModelProto messages are
declared from the public ONNX IR field numbers (onnx.proto, proto2 syntax) so exported models
can be written and parsed byte-compatibly.  Only the fields this library reads or writes are
declared; unknown fields are preserved by protobuf on round trips.  Enum-typed fields are
declared as int32 (identical varint wire encoding).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_PKG = "amd_dft_onnx"

F = descriptor_pb2.FieldDescriptorProto

# (name, number, type, label, type_name, packed)
_T_INT64, _T_INT32, _T_FLOAT, _T_DOUBLE = F.TYPE_INT64, F.TYPE_INT32, F.TYPE_FLOAT, F.TYPE_DOUBLE
_T_STRING, _T_BYTES, _T_MSG, _T_UINT64 = F.TYPE_STRING, F.TYPE_BYTES, F.TYPE_MESSAGE, F.TYPE_UINT64
_OPT, _REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

_MESSAGES = {
    "StringStringEntryProto": [("key", 1, _T_STRING, _OPT, None, False), ("value", 2, _T_STRING, _OPT, None, False)],
    "OperatorSetIdProto": [("domain", 1, _T_STRING, _OPT, None, False), ("version", 2, _T_INT64, _OPT, None, False)],
    "TensorShapeProto.Dimension": [
        ("dim_value", 1, _T_INT64, _OPT, None, False),
        ("dim_param", 2, _T_STRING, _OPT, None, False),
        ("denotation", 3, _T_STRING, _OPT, None, False),
    ],
    "TensorShapeProto": [("dim", 1, _T_MSG, _REP, "TensorShapeProto.Dimension", False)],
    "TypeProto.Tensor": [
        ("elem_type", 1, _T_INT32, _OPT, None, False),
        ("shape", 2, _T_MSG, _OPT, "TensorShapeProto", False),
    ],
    "TypeProto": [
        ("tensor_type", 1, _T_MSG, _OPT, "TypeProto.Tensor", False),
        ("denotation", 6, _T_STRING, _OPT, None, False),
    ],
    "TensorProto.Segment": [("begin", 1, _T_INT64, _OPT, None, False), ("end", 2, _T_INT64, _OPT, None, False)],
    "TensorProto": [
        ("dims", 1, _T_INT64, _REP, None, False),
        ("data_type", 2, _T_INT32, _OPT, None, False),
        ("segment", 3, _T_MSG, _OPT, "TensorProto.Segment", False),
        ("float_data", 4, _T_FLOAT, _REP, None, True),
        ("int32_data", 5, _T_INT32, _REP, None, True),
        ("string_data", 6, _T_BYTES, _REP, None, False),
        ("int64_data", 7, _T_INT64, _REP, None, True),
        ("name", 8, _T_STRING, _OPT, None, False),
        ("raw_data", 9, _T_BYTES, _OPT, None, False),
        ("double_data", 10, _T_DOUBLE, _REP, None, True),
        ("uint64_data", 11, _T_UINT64, _REP, None, True),
        ("doc_string", 12, _T_STRING, _OPT, None, False),
        ("external_data", 13, _T_MSG, _REP, "StringStringEntryProto", False),
        ("data_location", 14, _T_INT32, _OPT, None, False),
    ],
    "AttributeProto": [
        ("name", 1, _T_STRING, _OPT, None, False),
        ("f", 2, _T_FLOAT, _OPT, None, False),
        ("i", 3, _T_INT64, _OPT, None, False),
        ("s", 4, _T_BYTES, _OPT, None, False),
        ("t", 5, _T_MSG, _OPT, "TensorProto", False),
        ("g", 6, _T_MSG, _OPT, "GraphProto", False),
        ("floats", 7, _T_FLOAT, _REP, None, False),
        ("ints", 8, _T_INT64, _REP, None, False),
        ("strings", 9, _T_BYTES, _REP, None, False),
        ("tensors", 10, _T_MSG, _REP, "TensorProto", False),
        ("graphs", 11, _T_MSG, _REP, "GraphProto", False),
        ("doc_string", 13, _T_STRING, _OPT, None, False),
        ("tp", 14, _T_MSG, _OPT, "TypeProto", False),
        ("type", 20, _T_INT32, _OPT, None, False),
        ("ref_attr_name", 21, _T_STRING, _OPT, None, False),
    ],
    "ValueInfoProto": [
        ("name", 1, _T_STRING, _OPT, None, False),
        ("type", 2, _T_MSG, _OPT, "TypeProto", False),
        ("doc_string", 3, _T_STRING, _OPT, None, False),
    ],
    "NodeProto": [
        ("input", 1, _T_STRING, _REP, None, False),
        ("output", 2, _T_STRING, _REP, None, False),
        ("name", 3, _T_STRING, _OPT, None, False),
        ("op_type", 4, _T_STRING, _OPT, None, False),
        ("attribute", 5, _T_MSG, _REP, "AttributeProto", False),
        ("doc_string", 6, _T_STRING, _OPT, None, False),
        ("domain", 7, _T_STRING, _OPT, None, False),
    ],
    "GraphProto": [
        ("node", 1, _T_MSG, _REP, "NodeProto", False),
        ("name", 2, _T_STRING, _OPT, None, False),
        ("initializer", 5, _T_MSG, _REP, "TensorProto", False),
        ("doc_string", 10, _T_STRING, _OPT, None, False),
        ("input", 11, _T_MSG, _REP, "ValueInfoProto", False),
        ("output", 12, _T_MSG, _REP, "ValueInfoProto", False),
        ("value_info", 13, _T_MSG, _REP, "ValueInfoProto", False),
    ],
    "ModelProto": [
        ("ir_version", 1, _T_INT64, _OPT, None, False),
        ("producer_name", 2, _T_STRING, _OPT, None, False),
        ("producer_version", 3, _T_STRING, _OPT, None, False),
        ("domain", 4, _T_STRING, _OPT, None, False),
        ("model_version", 5, _T_INT64, _OPT, None, False),
        ("doc_string", 6, _T_STRING, _OPT, None, False),
        ("graph", 7, _T_MSG, _OPT, "GraphProto", False),
        ("opset_import", 8, _T_MSG, _REP, "OperatorSetIdProto", False),
        ("metadata_props", 14, _T_MSG, _REP, "StringStringEntryProto", False),
    ],
}

# TensorProto.DataType
UNDEFINED, FLOAT, UINT8, INT8, UINT16, INT16, INT32, INT64, STRING, BOOL = range(10)
FLOAT16, DOUBLE, UINT32, UINT64, COMPLEX64, COMPLEX128, BFLOAT16 = 10, 11, 12, 13, 14, 15, 16

# AttributeProto.AttributeType
ATTR_UNDEFINED, ATTR_FLOAT, ATTR_INT, ATTR_STRING, ATTR_TENSOR, ATTR_GRAPH = 0, 1, 2, 3, 4, 5
ATTR_FLOATS, ATTR_INTS, ATTR_STRINGS, ATTR_TENSORS, ATTR_GRAPHS = 6, 7, 8, 9, 10


def _build():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "amd_dft_onnx.proto"
    fdp.package = _PKG
    fdp.syntax = "proto2"
    msgs = {}
    # top-level first, nested after
    for full in sorted(_MESSAGES, key=lambda n: n.count(".")):
        parts = full.split(".")
        if len(parts) == 1:
            m = fdp.message_type.add()
        else:
            m = msgs[parts[0]].nested_type.add()
        m.name = parts[-1]
        msgs[full] = m
    for full, fields in _MESSAGES.items():
        m = msgs[full]
        for name, num, typ, label, tname, packed in fields:
            f = m.field.add()
            f.name, f.number, f.type, f.label = name, num, typ, label
            if tname:
                f.type_name = f".{_PKG}.{tname}"
            if packed:
                f.options.packed = True
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    out = {}
    for full in _MESSAGES:
        out[full] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{full}"))
    return out


_CLASSES = _build()
ModelProto = _CLASSES["ModelProto"]
GraphProto = _CLASSES["GraphProto"]
NodeProto = _CLASSES["NodeProto"]
AttributeProto = _CLASSES["AttributeProto"]
TensorProto = _CLASSES["TensorProto"]
ValueInfoProto = _CLASSES["ValueInfoProto"]
TypeProto = _CLASSES["TypeProto"]
TensorShapeProto = _CLASSES["TensorShapeProto"]
OperatorSetIdProto = _CLASSES["OperatorSetIdProto"]
StringStringEntryProto = _CLASSES["StringStringEntryProto"]


def load_model(data: bytes | str) -> "ModelProto":
    """Parse serialized ModelProto bytes (or a file path)."""
    if isinstance(data, str):
        with open(data, "rb") as f:
            data = f.read()
    m = ModelProto()
    m.ParseFromString(data)
    return m


# ----------------------------------------------------------------- tensor conversion
def _torch_dtype_map():
    import torch

    return {
        FLOAT: torch.float32, DOUBLE: torch.float64, FLOAT16: torch.float16, BFLOAT16: torch.bfloat16,
        INT8: torch.int8, UINT8: torch.uint8, INT16: torch.int16, INT32: torch.int32, INT64: torch.int64,
        BOOL: torch.bool, COMPLEX64: torch.complex64, COMPLEX128: torch.complex128,
    }


def onnx_dtype_to_torch(t: int):
    return _torch_dtype_map()[t]


def torch_dtype_to_onnx(dt) -> int:
    for k, v in _torch_dtype_map().items():
        if v == dt:
            return k
    raise TypeError(f"unsupported dtype {dt}")


def tensor_to_torch(t: "TensorProto"):
    """TensorProto -> torch.Tensor (CPU)."""
    import numpy as np
    import torch

    dt = onnx_dtype_to_torch(t.data_type)
    shape = list(t.dims)
    if t.raw_data:
        buf = bytearray(t.raw_data)
        if dt == torch.bfloat16:
            x = torch.frombuffer(buf, dtype=torch.int16).view(torch.bfloat16)
        else:
            x = torch.frombuffer(buf, dtype=dt) if len(buf) else torch.empty(0, dtype=dt)
        return x.reshape(shape).clone()
    if t.data_type in (FLOAT, COMPLEX64):
        arr = np.asarray(t.float_data, dtype=np.float32)
    elif t.data_type in (DOUBLE, COMPLEX128):
        arr = np.asarray(t.double_data, dtype=np.float64)
    elif t.data_type == INT64:
        arr = np.asarray(t.int64_data, dtype=np.int64)
    elif t.data_type in (INT32, INT16, INT8, UINT8, BOOL, UINT16):
        arr = np.asarray(t.int32_data, dtype=np.int32)
    elif t.data_type in (FLOAT16, BFLOAT16):
        arr = np.asarray(t.int32_data, dtype=np.int32).astype(np.uint16).view(np.int16)
        x = torch.from_numpy(arr.copy()).view(dt)
        return x.reshape(shape)
    else:
        raise TypeError(f"unsupported TensorProto data_type {t.data_type}")
    x = torch.from_numpy(arr.copy())
    if t.data_type in (COMPLEX64, COMPLEX128):
        x = torch.view_as_complex(x.reshape(-1, 2))
    return x.to(dt).reshape(shape)


def torch_to_tensor(x, name: str = "") -> "TensorProto":
    import torch

    t = TensorProto()
    t.name = name
    t.data_type = torch_dtype_to_onnx(x.dtype)
    t.dims.extend(list(x.shape))
    xc = x.detach().contiguous().cpu()
    if xc.dtype == torch.bfloat16:
        t.raw_data = xc.view(torch.int16).numpy().tobytes()
    else:
        t.raw_data = xc.numpy().tobytes()
    return t
