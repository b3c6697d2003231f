"""The reference's program / tensor file formats.

* ``framework.proto`` (paddle/fluid/framework/framework.proto:50 OpDesc, :212 BlockDesc, :236
  ProgramDesc): the message classes are built at import time from a ``FileDescriptorProto`` with
  the same package, message names, field numbers and types, so ``.pdmodel`` files are the
  reference's protobuf wire format (``ProgramDesc.SerializeToString()``). No protoc is needed.
* The LoDTensor stream (paddle/fluid/framework/lod_tensor.cc:205 SerializeToStream,
  tensor_util.cc:1046 TensorToStream): ``uint32 version=0 | uint64 lod_level | (uint64 bytes,
  size_t offsets)* | uint32 version=0 | int32 desc_size | VarType.TensorDesc | raw data``;
  ``save_combine`` (``.pdiparams``) is the concatenation of these streams in variable order.
"""
from __future__ import annotations

import struct

import numpy as np
import torch
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
_OPT, _REQ, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REQUIRED, _F.LABEL_REPEATED


def _field(msg, name, number, ftype, label=_OPT, type_name=None, default=None):
    f = msg.field.add()
    f.name, f.number, f.type, f.label = name, number, ftype, label
    if type_name:
        f.type_name = type_name
    if default is not None:
        f.default_value = default
    return f


def _build_file():
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "paddle_hackathon_amd/framework.proto"
    fd.package = "paddle.framework.proto"
    fd.syntax = "proto2"
    P = ".paddle.framework.proto."

    m = fd.message_type.add()
    m.name = "Version"
    _field(m, "version", 1, _F.TYPE_INT64, default="0")

    e = fd.enum_type.add()
    e.name = "AttrType"
    for i, n in enumerate(["INT", "FLOAT", "STRING", "INTS", "FLOATS", "STRINGS", "BOOLEAN", "BOOLEANS", "BLOCK",
                           "LONG", "BLOCKS", "LONGS", "FLOAT64S"]):
        v = e.value.add()
        v.name, v.number = n, i

    op = fd.message_type.add()
    op.name = "OpDesc"
    at = op.nested_type.add()
    at.name = "Attr"
    _field(at, "name", 1, _F.TYPE_STRING, _REQ)
    _field(at, "type", 2, _F.TYPE_ENUM, _REQ, P + "AttrType")
    _field(at, "i", 3, _F.TYPE_INT32)
    _field(at, "f", 4, _F.TYPE_FLOAT)
    _field(at, "s", 5, _F.TYPE_STRING)
    _field(at, "ints", 6, _F.TYPE_INT32, _REP)
    _field(at, "floats", 7, _F.TYPE_FLOAT, _REP)
    _field(at, "strings", 8, _F.TYPE_STRING, _REP)
    _field(at, "b", 10, _F.TYPE_BOOL)
    _field(at, "bools", 11, _F.TYPE_BOOL, _REP)
    _field(at, "block_idx", 12, _F.TYPE_INT32)
    _field(at, "l", 13, _F.TYPE_INT64)
    _field(at, "blocks_idx", 14, _F.TYPE_INT32, _REP)
    _field(at, "longs", 15, _F.TYPE_INT64, _REP)
    _field(at, "float64s", 16, _F.TYPE_DOUBLE, _REP)
    var = op.nested_type.add()
    var.name = "Var"
    _field(var, "parameter", 1, _F.TYPE_STRING, _REQ)
    _field(var, "arguments", 2, _F.TYPE_STRING, _REP)
    _field(op, "type", 3, _F.TYPE_STRING, _REQ)
    _field(op, "inputs", 1, _F.TYPE_MESSAGE, _REP, P + "OpDesc.Var")
    _field(op, "outputs", 2, _F.TYPE_MESSAGE, _REP, P + "OpDesc.Var")
    _field(op, "attrs", 4, _F.TYPE_MESSAGE, _REP, P + "OpDesc.Attr")
    _field(op, "is_target", 5, _F.TYPE_BOOL, default="false")

    vt = fd.message_type.add()
    vt.name = "VarType"
    te = vt.enum_type.add()
    te.name = "Type"
    for n, i in [("BOOL", 0), ("INT16", 1), ("INT32", 2), ("INT64", 3), ("FP16", 4), ("FP32", 5), ("FP64", 6),
                 ("SIZE_T", 19), ("UINT8", 20), ("INT8", 21), ("BF16", 22), ("COMPLEX64", 23), ("COMPLEX128", 24),
                 ("LOD_TENSOR", 7), ("SELECTED_ROWS", 8), ("FEED_MINIBATCH", 9), ("FETCH_LIST", 10),
                 ("STEP_SCOPES", 11), ("LOD_RANK_TABLE", 12), ("LOD_TENSOR_ARRAY", 13), ("PLACE_LIST", 14),
                 ("READER", 15), ("RAW", 17), ("TUPLE", 18), ("STRING", 25), ("STRINGS", 26), ("VOCAB", 27),
                 ("FEED_LIST", 28), ("PSTRING", 29)]:
        v = te.value.add()
        v.name, v.number = n, i
    td = vt.nested_type.add()
    td.name = "TensorDesc"
    _field(td, "data_type", 1, _F.TYPE_ENUM, _REQ, P + "VarType.Type")
    _field(td, "dims", 2, _F.TYPE_INT64, _REP)
    ld = vt.nested_type.add()
    ld.name = "LoDTensorDesc"
    _field(ld, "tensor", 1, _F.TYPE_MESSAGE, _REQ, P + "VarType.TensorDesc")
    _field(ld, "lod_level", 2, _F.TYPE_INT32, default="0")
    la = vt.nested_type.add()
    la.name = "LoDTensorArrayDesc"
    _field(la, "tensor", 1, _F.TYPE_MESSAGE, _REQ, P + "VarType.TensorDesc")
    _field(la, "lod_level", 2, _F.TYPE_INT32, default="0")
    rd = vt.nested_type.add()
    rd.name = "ReaderDesc"
    _field(rd, "lod_tensor", 1, _F.TYPE_MESSAGE, _REP, P + "VarType.LoDTensorDesc")
    tu = vt.nested_type.add()
    tu.name = "Tuple"
    _field(tu, "element_type", 1, _F.TYPE_ENUM, _REP, P + "VarType.Type")
    _field(vt, "type", 1, _F.TYPE_ENUM, _REQ, P + "VarType.Type")
    _field(vt, "selected_rows", 2, _F.TYPE_MESSAGE, type_name=P + "VarType.TensorDesc")
    _field(vt, "lod_tensor", 3, _F.TYPE_MESSAGE, type_name=P + "VarType.LoDTensorDesc")
    _field(vt, "tensor_array", 4, _F.TYPE_MESSAGE, type_name=P + "VarType.LoDTensorArrayDesc")
    _field(vt, "reader", 5, _F.TYPE_MESSAGE, type_name=P + "VarType.ReaderDesc")
    _field(vt, "tuple", 7, _F.TYPE_MESSAGE, type_name=P + "VarType.Tuple")
    _field(vt, "string", 8, _F.TYPE_MESSAGE, type_name=P + "VarType.TensorDesc")
    _field(vt, "strings", 9, _F.TYPE_MESSAGE, type_name=P + "VarType.TensorDesc")
    _field(vt, "vocab", 10, _F.TYPE_MESSAGE, type_name=P + "VarType.TensorDesc")

    vd = fd.message_type.add()
    vd.name = "VarDesc"
    va = vd.nested_type.add()
    va.name = "Attr"
    _field(va, "name", 1, _F.TYPE_STRING, _REQ)
    _field(va, "type", 2, _F.TYPE_ENUM, _REQ, P + "AttrType")
    _field(va, "i", 3, _F.TYPE_INT32)
    _field(va, "s", 4, _F.TYPE_STRING)
    _field(va, "ints", 5, _F.TYPE_INT32, _REP)
    _field(vd, "name", 1, _F.TYPE_STRING, _REQ)
    _field(vd, "type", 2, _F.TYPE_MESSAGE, _REQ, P + "VarType")
    _field(vd, "persistable", 3, _F.TYPE_BOOL, default="false")
    _field(vd, "need_check_feed", 4, _F.TYPE_BOOL, default="false")
    _field(vd, "is_parameter", 5, _F.TYPE_BOOL, default="false")
    _field(vd, "stop_gradient", 6, _F.TYPE_BOOL, default="false")
    _field(vd, "attrs", 7, _F.TYPE_MESSAGE, _REP, P + "VarDesc.Attr")

    bd = fd.message_type.add()
    bd.name = "BlockDesc"
    _field(bd, "idx", 1, _F.TYPE_INT32, _REQ)
    _field(bd, "parent_idx", 2, _F.TYPE_INT32, _REQ)
    _field(bd, "vars", 3, _F.TYPE_MESSAGE, _REP, P + "VarDesc")
    _field(bd, "ops", 4, _F.TYPE_MESSAGE, _REP, P + "OpDesc")
    _field(bd, "forward_block_idx", 5, _F.TYPE_INT32, default="-1")

    ov = fd.message_type.add()
    ov.name = "OpVersion"
    _field(ov, "version", 1, _F.TYPE_INT32, _REQ)
    om = fd.message_type.add()
    om.name = "OpVersionMap"
    pr = om.nested_type.add()
    pr.name = "OpVersionPair"
    _field(pr, "op_name", 1, _F.TYPE_STRING, _REQ)
    _field(pr, "op_version", 2, _F.TYPE_MESSAGE, _REQ, P + "OpVersion")
    _field(om, "pair", 1, _F.TYPE_MESSAGE, _REP, P + "OpVersionMap.OpVersionPair")

    pd = fd.message_type.add()
    pd.name = "ProgramDesc"
    rr = pd.reserved_range.add()
    rr.start, rr.end = 2, 4
    _field(pd, "blocks", 1, _F.TYPE_MESSAGE, _REP, P + "BlockDesc")
    _field(pd, "version", 4, _F.TYPE_MESSAGE, type_name=P + "Version")
    _field(pd, "op_version_map", 5, _F.TYPE_MESSAGE, type_name=P + "OpVersionMap")
    return fd


_pool = descriptor_pool.DescriptorPool()
_pool.Add(_build_file())


def _cls(name):
    d = _pool.FindMessageTypeByName("paddle.framework.proto." + name)
    return message_factory.GetMessageClass(d)


ProgramDesc = _cls("ProgramDesc")
BlockDesc = _cls("BlockDesc")
OpDesc = _cls("OpDesc")
VarDesc = _cls("VarDesc")
VarType = _cls("VarType")
TensorDesc = _cls("VarType.TensorDesc")
Version = _cls("Version")

# AttrType values
INT, FLOAT, STRING, INTS, FLOATS, STRINGS, BOOLEAN, BOOLEANS, BLOCK, LONG, BLOCKS, LONGS, FLOAT64S = range(13)

# VarType.Type <-> torch dtype
_DT2VT = {torch.bool: 0, torch.int16: 1, torch.int32: 2, torch.int64: 3, torch.float16: 4, torch.float32: 5,
          torch.float64: 6, torch.uint8: 20, torch.int8: 21, torch.bfloat16: 22, torch.complex64: 23,
          torch.complex128: 24}
_VT2DT = {v: k for k, v in _DT2VT.items()}
LOD_TENSOR, FEED_MINIBATCH, FETCH_LIST = 7, 9, 10


def vartype_of(dtype):
    return _DT2VT[dtype]


def dtype_of(vt):
    return _VT2DT[vt]


# ---- LoDTensor stream / save_combine --------------------------------------------------------------
def tensor_to_stream(t, lod=()):
    """bytes of one LoDTensor in the reference's stream layout (host copy of ``t``)."""
    t = t.detach().contiguous().cpu()
    out = [struct.pack("<I", 0), struct.pack("<Q", len(lod))]
    for level in lod:
        arr = np.asarray(level, dtype=np.uint64)
        out += [struct.pack("<Q", arr.nbytes), arr.tobytes()]
    desc = TensorDesc()
    desc.data_type = vartype_of(t.dtype)
    desc.dims.extend(list(t.shape))
    db = desc.SerializeToString()
    out += [struct.pack("<I", 0), struct.pack("<i", len(db)), db]
    if t.dtype == torch.bfloat16:
        raw = t.view(torch.int16).numpy().tobytes()
    else:
        raw = t.numpy().tobytes()
    out.append(raw)
    return b"".join(out)


def tensor_from_stream(buf, off=0):
    """-> (torch tensor, lod, new offset)"""
    (ver,) = struct.unpack_from("<I", buf, off)
    off += 4
    if ver != 0:
        raise ValueError(f"unsupported LoDTensor version {ver}")
    (nlod,) = struct.unpack_from("<Q", buf, off)
    off += 8
    lod = []
    for _ in range(nlod):
        (nb,) = struct.unpack_from("<Q", buf, off)
        off += 8
        lod.append(np.frombuffer(buf, dtype=np.uint64, count=nb // 8, offset=off).tolist())
        off += nb
    (tver,) = struct.unpack_from("<I", buf, off)
    off += 4
    if tver != 0:
        raise ValueError(f"unsupported Tensor version {tver}")
    (dsz,) = struct.unpack_from("<i", buf, off)
    off += 4
    desc = TensorDesc()
    desc.ParseFromString(bytes(buf[off:off + dsz]))
    off += dsz
    dt = dtype_of(desc.data_type)
    shape = list(desc.dims)
    n = int(np.prod(shape)) if shape else 1
    esize = torch.empty(0, dtype=dt).element_size()
    raw = bytes(buf[off:off + n * esize])
    if len(raw) != n * esize:
        raise ValueError(f"truncated LoDTensor stream: {len(raw)} of {n * esize} data bytes")
    off += n * esize
    if dt == torch.bfloat16:
        t = torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16)
    else:
        npdt = torch.empty(0, dtype=dt).numpy().dtype
        t = torch.from_numpy(np.frombuffer(raw, dtype=npdt).copy())
    return t.reshape(shape), lod, off


def save_combine(tensors, path):
    """``tensors``: ordered list of torch tensors -> one file of concatenated LoDTensor streams"""
    with open(path, "wb") as f:
        for t in tensors:
            f.write(tensor_to_stream(t))


def load_combine(path):
    """-> list of torch tensors, in file order"""
    with open(path, "rb") as f:
        buf = f.read()
    out, off = [], 0
    while off < len(buf):
        t, _, off = tensor_from_stream(buf, off)
        out.append(t)
    return out
