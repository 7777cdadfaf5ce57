"""KServe V2 / Triton ``GRPCInferenceService`` over grpcio (S6 / S7 / N14).

The reference's FasterTransformer client talks gRPC too: ``--protocol grpc``
opens a bidirectional ``ModelStreamInfer`` stream with tritonclient
(``start_stream`` + ``async_stream_infer``,
online-inference/fastertransformer/client/example.py:126-140) and reads
``output_ids`` from the streamed ``ModelInferResponse`` (:100-116). This module
serves that protocol for the same ``Model`` objects the REST server hosts:

* message types are built at import time from a ``FileDescriptorProto``
  written in code (package ``inference``, the field numbers of Triton's
  ``grpc_service.proto``) -- no protoc / codegen step;
* ``ServerLive`` / ``ServerReady`` / ``ModelReady`` / ``ServerMetadata`` /
  ``ModelMetadata`` / ``ModelInfer`` / ``ModelStreamInfer``;
* input tensors from ``raw_input_contents`` (tritonclient's default) or typed
  ``contents``; outputs always as ``raw_output_contents``;
* on the stream, a request whose parameters carry ``"streaming": true`` (or a
  model configured decoupled) gets one response per generation step from
  ``Model.infer_stream`` (FT's ``decoupled: True``), the last one marked with
  ``triton_final_response``; otherwise one response per request.
"""
from __future__ import annotations

import logging
import struct
from concurrent import futures

import numpy as np
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

log = logging.getLogger("kca.serving")

SERVICE = "inference.GRPCInferenceService"
_F = descriptor_pb2.FieldDescriptorProto


def _field(msg, name, number, ftype, label=_F.LABEL_OPTIONAL, type_name=None, oneof=None):
    f = msg.field.add(name=name, number=number, type=ftype, label=label)
    if type_name:
        f.type_name = type_name
    if oneof is not None:
        f.oneof_index = oneof
    return f


def _map(msg, name, number, value_type_name):
    """map<string, Message> field: a nested *Entry message with map_entry set."""
    entry = msg.nested_type.add(name="".join(p.capitalize() for p in name.split("_")) + "Entry")
    entry.options.map_entry = True
    _field(entry, "key", 1, _F.TYPE_STRING)
    _field(entry, "value", 2, _F.TYPE_MESSAGE, type_name=value_type_name)
    _field(msg, name, number, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, type_name=entry.name)
    # relative type names resolve inside the enclosing message
    msg.field[-1].type_name = entry.name


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="kca_grpc_service.proto", package="inference", syntax="proto3")
    R = _F.LABEL_REPEATED
    S, B, I64, U64, D, I32, U32, FL, BY = (_F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT64, _F.TYPE_UINT64,
                                          _F.TYPE_DOUBLE, _F.TYPE_INT32, _F.TYPE_UINT32, _F.TYPE_FLOAT,
                                          _F.TYPE_BYTES)
    M = _F.TYPE_MESSAGE

    def msg(name):
        return fd.message_type.add(name=name)
    for n in ("ServerLiveRequest", "ServerReadyRequest", "ServerMetadataRequest"):
        msg(n)
    _field(msg("ServerLiveResponse"), "live", 1, B)
    _field(msg("ServerReadyResponse"), "ready", 1, B)
    m = msg("ModelReadyRequest")
    _field(m, "name", 1, S)
    _field(m, "version", 2, S)
    _field(msg("ModelReadyResponse"), "ready", 1, B)
    m = msg("ServerMetadataResponse")
    _field(m, "name", 1, S)
    _field(m, "version", 2, S)
    _field(m, "extensions", 3, S, R)
    m = msg("ModelMetadataRequest")
    _field(m, "name", 1, S)
    _field(m, "version", 2, S)
    m = msg("ModelMetadataResponse")
    tm = m.nested_type.add(name="TensorMetadata")
    _field(tm, "name", 1, S)
    _field(tm, "datatype", 2, S)
    _field(tm, "shape", 3, I64, R)
    _field(m, "name", 1, S)
    _field(m, "versions", 2, S, R)
    _field(m, "platform", 3, S)
    _field(m, "inputs", 4, M, R, ".inference.ModelMetadataResponse.TensorMetadata")
    _field(m, "outputs", 5, M, R, ".inference.ModelMetadataResponse.TensorMetadata")
    m = msg("InferParameter")
    m.oneof_decl.add(name="parameter_choice")
    for name, num, t in (("bool_param", 1, B), ("int64_param", 2, I64), ("string_param", 3, S),
                         ("double_param", 4, D), ("uint64_param", 5, U64)):
        _field(m, name, num, t, oneof=0)
    m = msg("InferTensorContents")
    for name, num, t in (("bool_contents", 1, B), ("int_contents", 2, I32), ("int64_contents", 3, I64),
                         ("uint_contents", 4, U32), ("uint64_contents", 5, U64), ("fp32_contents", 6, FL),
                         ("fp64_contents", 7, D), ("bytes_contents", 8, BY)):
        _field(m, name, num, t, R)
    P, C = ".inference.InferParameter", ".inference.InferTensorContents"
    m = msg("ModelInferRequest")
    it = m.nested_type.add(name="InferInputTensor")
    _field(it, "name", 1, S)
    _field(it, "datatype", 2, S)
    _field(it, "shape", 3, I64, R)
    _map(it, "parameters", 4, P)
    _field(it, "contents", 5, M, type_name=C)
    ro = m.nested_type.add(name="InferRequestedOutputTensor")
    _field(ro, "name", 1, S)
    _map(ro, "parameters", 2, P)
    _field(m, "model_name", 1, S)
    _field(m, "model_version", 2, S)
    _field(m, "id", 3, S)
    _map(m, "parameters", 4, P)
    _field(m, "inputs", 5, M, R, ".inference.ModelInferRequest.InferInputTensor")
    _field(m, "outputs", 6, M, R, ".inference.ModelInferRequest.InferRequestedOutputTensor")
    _field(m, "raw_input_contents", 7, BY, R)
    m = msg("ModelInferResponse")
    ot = m.nested_type.add(name="InferOutputTensor")
    _field(ot, "name", 1, S)
    _field(ot, "datatype", 2, S)
    _field(ot, "shape", 3, I64, R)
    _map(ot, "parameters", 4, P)
    _field(ot, "contents", 5, M, type_name=C)
    _field(m, "model_name", 1, S)
    _field(m, "model_version", 2, S)
    _field(m, "id", 3, S)
    _map(m, "parameters", 4, P)
    _field(m, "outputs", 5, M, R, ".inference.ModelInferResponse.InferOutputTensor")
    _field(m, "raw_output_contents", 6, BY, R)
    m = msg("ModelStreamInferResponse")
    _field(m, "error_message", 1, S)
    _field(m, "infer_response", 2, M, type_name=".inference.ModelInferResponse")
    svc = fd.service.add(name="GRPCInferenceService")
    for name, req, resp, cs, ss in (
            ("ServerLive", "ServerLiveRequest", "ServerLiveResponse", False, False),
            ("ServerReady", "ServerReadyRequest", "ServerReadyResponse", False, False),
            ("ModelReady", "ModelReadyRequest", "ModelReadyResponse", False, False),
            ("ServerMetadata", "ServerMetadataRequest", "ServerMetadataResponse", False, False),
            ("ModelMetadata", "ModelMetadataRequest", "ModelMetadataResponse", False, False),
            ("ModelInfer", "ModelInferRequest", "ModelInferResponse", False, False),
            ("ModelStreamInfer", "ModelInferRequest", "ModelStreamInferResponse", True, True)):
        svc.method.add(name=name, input_type=".inference." + req, output_type=".inference." + resp,
                       client_streaming=cs, server_streaming=ss)
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_build_file())
pb = type("pb", (), {})  # namespace of message classes: pb.ModelInferRequest, ...
for _name in _FILE.message_types_by_name:
    setattr(pb, _name, message_factory.GetMessageClass(_FILE.message_types_by_name[_name]))

_NP = {"BOOL": np.bool_, "UINT8": np.uint8, "UINT16": np.uint16, "UINT32": np.uint32, "UINT64": np.uint64,
       "INT8": np.int8, "INT16": np.int16, "INT32": np.int32, "INT64": np.int64, "FP16": np.float16,
       "FP32": np.float32, "FP64": np.float64}
_CONTENTS = {"BOOL": "bool_contents", "INT8": "int_contents", "INT16": "int_contents", "INT32": "int_contents",
             "INT64": "int64_contents", "UINT8": "uint_contents", "UINT16": "uint_contents",
             "UINT32": "uint_contents", "UINT64": "uint64_contents", "FP32": "fp32_contents",
             "FP64": "fp64_contents", "BYTES": "bytes_contents"}


def _param_value(p):
    which = p.WhichOneof("parameter_choice")
    return getattr(p, which) if which else None


def _bytes_decode(raw: bytes) -> list:
    out, i = [], 0
    while i < len(raw):
        (n,) = struct.unpack_from("<I", raw, i)
        out.append(raw[i + 4:i + 4 + n])
        i += 4 + n
    return out


def decode_inputs(req) -> dict:
    """ModelInferRequest -> {name: ndarray}."""
    out = {}
    raw = list(req.raw_input_contents)
    for i, t in enumerate(req.inputs):
        shape = [int(s) for s in t.shape]
        dt = t.datatype
        if raw:
            if i >= len(raw):
                raise ValueError(f"raw_input_contents has no entry for input {t.name}")
            if dt == "BYTES":
                a = np.array(_bytes_decode(raw[i]), dtype=np.object_).reshape(shape)
            else:
                a = np.frombuffer(raw[i], dtype=_NP[dt]).reshape(shape).copy()
        else:
            vals = list(getattr(t.contents, _CONTENTS[dt]))
            a = (np.array(vals, dtype=np.object_) if dt == "BYTES" else np.array(vals, dtype=_NP[dt])).reshape(shape)
        out[t.name] = a
    return out


def encode_response(model_name: str, outputs: dict, req, version: str = "1", params: dict | None = None):
    from .v2 import triton_dtype
    resp = pb.ModelInferResponse(model_name=model_name, model_version=version or "1", id=req.id)
    wanted = [o.name for o in req.outputs] or list(outputs)
    for name in wanted:
        if name not in outputs:
            continue
        a = np.asarray(outputs[name])
        dt = triton_dtype(a)
        o = resp.outputs.add(name=name, datatype=dt)
        o.shape.extend(int(s) for s in a.shape)
        if dt == "BYTES":
            resp.raw_output_contents.append(b"".join(struct.pack("<I", len(x)) + x for x in
                                                     (v if isinstance(v, bytes) else str(v).encode()
                                                      for v in a.reshape(-1))))
        else:
            resp.raw_output_contents.append(np.ascontiguousarray(a).tobytes())
    for k, v in (params or {}).items():
        if isinstance(v, bool):
            resp.parameters[k].bool_param = v
        elif isinstance(v, int):
            resp.parameters[k].int64_param = v
        else:
            resp.parameters[k].string_param = str(v)
    return resp


class InferenceServicer:
    def __init__(self, models: dict, server_name: str = "kubernetes-cloud-amd", version: str = "0.1"):
        self.models, self.server_name, self.version = models, server_name, version

    def _model(self, name, context):
        import grpc
        m = self.models.get(name)
        if m is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"Request for unknown model: '{name}' is not found")
        if not m.ready:
            context.abort(grpc.StatusCode.UNAVAILABLE, f"Model '{name}' is not ready")
        return m

    def ServerLive(self, request, context):
        return pb.ServerLiveResponse(live=True)

    def ServerReady(self, request, context):
        return pb.ServerReadyResponse(ready=all(m.ready for m in self.models.values()))

    def ModelReady(self, request, context):
        m = self.models.get(request.name)
        return pb.ModelReadyResponse(ready=bool(m is not None and m.ready))

    def ServerMetadata(self, request, context):
        return pb.ServerMetadataResponse(name=self.server_name, version=self.version,
                                         extensions=["binary_tensor_data", "model_repository", "streaming"])

    def ModelMetadata(self, request, context):
        import grpc
        m = self.models.get(request.name)
        if m is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"Request for unknown model: '{request.name}' is not found")
        md = m.metadata()
        resp = pb.ModelMetadataResponse(name=md.get("name", request.name), versions=md.get("versions", ["1"]),
                                        platform=md.get("platform", ""))
        for key in ("inputs", "outputs"):
            for t in md.get(key, []):
                e = getattr(resp, key).add(name=t["name"], datatype=t["datatype"])
                e.shape.extend(int(s) for s in t["shape"])
        return resp

    def _infer(self, m, req):
        inputs = decode_inputs(req)
        js = {"id": req.id, "parameters": {k: _param_value(v) for k, v in req.parameters.items()}}
        return m.infer(inputs, js)

    def ModelInfer(self, request, context):
        import grpc
        m = self._model(request.model_name, context)
        try:
            outs = self._infer(m, request)
        except (ValueError, KeyError, TypeError) as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        except Exception as e:  # noqa: BLE001
            log.exception("gRPC infer failed")
            context.abort(grpc.StatusCode.INTERNAL, str(e))
        return encode_response(request.model_name, outs, request, request.model_version)

    def ModelStreamInfer(self, request_iterator, context):
        for req in request_iterator:
            m = self.models.get(req.model_name)
            if m is None or not m.ready:
                yield pb.ModelStreamInferResponse(
                    error_message=f"Request for unknown or unready model: '{req.model_name}'")
                continue
            params = {k: _param_value(v) for k, v in req.parameters.items()}
            decoupled = bool(params.get("streaming", getattr(m, "decoupled", False)))
            try:
                if decoupled and hasattr(m, "infer_stream"):
                    inputs = decode_inputs(req)
                    last = None
                    for outs in m.infer_stream(inputs, {"id": req.id, "parameters": params}):
                        if last is not None:
                            yield pb.ModelStreamInferResponse(infer_response=encode_response(
                                req.model_name, last, req, req.model_version, {"triton_final_response": False}))
                        last = outs
                    yield pb.ModelStreamInferResponse(infer_response=encode_response(
                        req.model_name, last, req, req.model_version, {"triton_final_response": True}))
                else:
                    outs = self._infer(m, req)
                    yield pb.ModelStreamInferResponse(
                        infer_response=encode_response(req.model_name, outs, req, req.model_version))
            except Exception as e:  # noqa: BLE001 -- errors travel in-band on the stream (Triton semantics)
                log.exception("gRPC stream infer failed")
                yield pb.ModelStreamInferResponse(error_message=str(e))


def make_handler(servicer: InferenceServicer):
    import grpc
    unary = [("ServerLive", pb.ServerLiveRequest, pb.ServerLiveResponse),
             ("ServerReady", pb.ServerReadyRequest, pb.ServerReadyResponse),
             ("ModelReady", pb.ModelReadyRequest, pb.ModelReadyResponse),
             ("ServerMetadata", pb.ServerMetadataRequest, pb.ServerMetadataResponse),
             ("ModelMetadata", pb.ModelMetadataRequest, pb.ModelMetadataResponse),
             ("ModelInfer", pb.ModelInferRequest, pb.ModelInferResponse)]
    handlers = {n: grpc.unary_unary_rpc_method_handler(getattr(servicer, n), request_deserializer=rq.FromString,
                                                       response_serializer=rs.SerializeToString)
                for n, rq, rs in unary}
    handlers["ModelStreamInfer"] = grpc.stream_stream_rpc_method_handler(
        servicer.ModelStreamInfer, request_deserializer=pb.ModelInferRequest.FromString,
        response_serializer=pb.ModelStreamInferResponse.SerializeToString)
    return grpc.method_handlers_generic_handler(SERVICE, handlers)


def serve(models: dict, port: int, host: str = "0.0.0.0", workers: int = 16, block: bool = False):
    """Start the gRPC server (returns it; ``block`` waits for termination)."""
    import grpc
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                         options=[("grpc.max_send_message_length", 1 << 30),
                                  ("grpc.max_receive_message_length", 1 << 30)])
    server.add_generic_rpc_handlers((make_handler(InferenceServicer(models)),))
    bound = server.add_insecure_port(f"{host}:{port}")
    server.start()
    server.bound_port = bound
    log.info("gRPC V2 (%s) on %s:%d", SERVICE, host, bound)
    if block:
        server.wait_for_termination()
    return server


__all__ = ["pb", "serve", "InferenceServicer", "decode_inputs", "encode_response", "SERVICE"]
