"""KServe V2 / Triton gRPC (serving/grpc_v2.py) against the FasterTransformer
model, driven through a raw grpc channel with the tensor names and values of
the reference's client/sample_request.json: unary ModelInfer, the
bidirectional ModelStreamInfer the FT client uses (example.py:126-140), and
token streaming (decoupled mode) whose final response equals the unary one."""
import json
import os

import grpc
import numpy as np
import pytest

from kubernetes_cloud_amd.serving.grpc_v2 import SERVICE, pb, serve

from .helpers import make_model_dir

SAMPLE = "/root/reference/online-inference/fastertransformer/client/sample_request.json"


@pytest.fixture(scope="module")
def ft_server(tmp_path_factory):
    from kubernetes_cloud_amd.serving.triton_ft import FasterTransformerModel, write_model_store
    d = make_model_dir(str(tmp_path_factory.mktemp("gptj")), "gpt-j-6b")
    store = str(tmp_path_factory.mktemp("store"))
    write_model_store(d, store, data_type="fp32")
    ft = FasterTransformerModel(store_dir=store)
    ft.load()
    srv = serve({ft.name: ft}, 0, host="127.0.0.1")
    ch = grpc.insecure_channel(f"127.0.0.1:{srv.bound_port}")
    yield ch, ft
    ch.close()
    srv.stop(0)
    ft.generator.close()


def _sample_request(prompt_ids, out_len=8):
    """sample_request.json's tensors (reference file when present, else its
    documented values), prompt filled in like example.py's generate_parameters."""
    if os.path.exists(SAMPLE):
        fields = json.load(open(SAMPLE))["request"]
    else:
        fields = [{"name": "request_output_len", "data": [[64]], "dtype": "int32"},
                  {"name": "runtime_top_k", "data": [[10]], "dtype": "int32"},
                  {"name": "random_seed", "data": [[0]], "dtype": "uint64"}]
    req = pb.ModelInferRequest(model_name="fastertransformer", id="r1")
    for f in fields:
        data = f["data"]
        if f["name"] == "input_ids":
            data = [prompt_ids]
        elif f["name"] == "input_lengths":
            data = [[len(prompt_ids)]]
        elif f["name"] == "request_output_len":
            data = [[out_len]]
        elif f["name"] == "runtime_top_k":
            data = [[0]]  # greedy (top_k == top_p == 0) so streamed == unary
        a = np.array(data, dtype=np.dtype({"int32": np.int32, "float32": np.float32, "uint64": np.uint64,
                                           "bool": np.bool_}[f["dtype"]]))
        t = req.inputs.add(name=f["name"], datatype={"int32": "INT32", "float32": "FP32", "uint64": "UINT64",
                                                      "bool": "BOOL"}[f["dtype"]])
        t.shape.extend(a.shape)
        req.raw_input_contents.append(a.tobytes())  # tritonclient's wire form
    return req


def _outputs(resp):
    return {o.name: np.frombuffer(raw, dtype={"INT32": np.int32, "FP32": np.float32}[o.datatype]).reshape(
        list(o.shape)) for o, raw in zip(resp.outputs, resp.raw_output_contents)}


def _rpc(ch, name, req_cls, resp_cls, stream=False):
    path = f"/{SERVICE}/{name}"
    if stream:
        return ch.stream_stream(path, request_serializer=req_cls.SerializeToString,
                                response_deserializer=resp_cls.FromString)
    return ch.unary_unary(path, request_serializer=req_cls.SerializeToString, response_deserializer=resp_cls.FromString)


def test_health_and_metadata(ft_server):
    ch, _ = ft_server
    assert _rpc(ch, "ServerLive", pb.ServerLiveRequest, pb.ServerLiveResponse)(pb.ServerLiveRequest()).live
    assert _rpc(ch, "ServerReady", pb.ServerReadyRequest, pb.ServerReadyResponse)(pb.ServerReadyRequest()).ready
    mr = _rpc(ch, "ModelReady", pb.ModelReadyRequest, pb.ModelReadyResponse)
    assert mr(pb.ModelReadyRequest(name="fastertransformer")).ready
    assert not mr(pb.ModelReadyRequest(name="nope")).ready
    md = _rpc(ch, "ModelMetadata", pb.ModelMetadataRequest, pb.ModelMetadataResponse)(
        pb.ModelMetadataRequest(name="fastertransformer"))
    assert {t.name for t in md.inputs} >= {"input_ids", "request_output_len", "bad_words_list"}
    assert {t.name for t in md.outputs} >= {"output_ids", "sequence_length"}
    with pytest.raises(grpc.RpcError) as e:
        _rpc(ch, "ModelMetadata", pb.ModelMetadataRequest, pb.ModelMetadataResponse)(pb.ModelMetadataRequest(name="x"))
    assert e.value.code() == grpc.StatusCode.NOT_FOUND


def test_model_infer_and_stream_infer(ft_server):
    ch, _ = ft_server
    prompt = [5, 6, 7, 8, 9]
    unary = _rpc(ch, "ModelInfer", pb.ModelInferRequest, pb.ModelInferResponse)(_sample_request(prompt))
    out = _outputs(unary)
    assert unary.id == "r1" and out["output_ids"].shape[:2] == (1, 1)
    assert out["output_ids"][0, 0, :5].tolist() == prompt and int(out["sequence_length"][0, 0]) == 13
    # bidirectional stream, two requests on one stream (one response each)
    call = _rpc(ch, "ModelStreamInfer", pb.ModelInferRequest, pb.ModelStreamInferResponse, stream=True)
    resps = list(call(iter([_sample_request(prompt), _sample_request([11, 12], 4)])))
    assert len(resps) == 2 and not resps[0].error_message
    assert _outputs(resps[0].infer_response)["output_ids"].tolist() == out["output_ids"].tolist()
    assert int(_outputs(resps[1].infer_response)["sequence_length"][0, 0]) == 6
    # decoupled token streaming: several responses, lengths grow, last is final and == unary
    req = _sample_request(prompt)
    req.parameters["streaming"].bool_param = True
    resps = list(call(iter([req])))
    assert len(resps) >= 3
    lens = [int(_outputs(r.infer_response)["sequence_length"][0, 0]) for r in resps]
    assert lens == sorted(lens) and lens[-1] == 13
    assert resps[-1].infer_response.parameters["triton_final_response"].bool_param
    assert not resps[0].infer_response.parameters["triton_final_response"].bool_param
    assert _outputs(resps[-1].infer_response)["output_ids"].tolist() == out["output_ids"].tolist()
    # errors travel in-band on the stream
    bad = pb.ModelInferRequest(model_name="missing")
    r = list(call(iter([bad])))
    assert r[0].error_message
