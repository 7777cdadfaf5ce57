"""VirtualServer client (P5) against a mock Kubernetes API: create -> Ready ->
stop -> Stopped -> update -> start -> delete, plus kubeconfig parsing."""
import json

import httpx
import yaml

from kubernetes_cloud_amd.platform.virtual_server import K8sREST, VirtualServerClient


def test_virtual_server_lifecycle(tmp_path):
    store, calls = {}, []

    def handler(req: httpx.Request):
        calls.append((req.method, req.url.path))
        p = req.url.path
        base = "/apis/virtualservers.coreweave.com/v1alpha1/namespaces/ns/virtualservers"
        if req.method == "POST" and p == base:
            obj = json.loads(req.content)
            obj["status"] = {"conditions": [{"type": "Ready", "reason": "VirtualServerReady", "status": "True"}],
                             "network": {"externalIP": "1.2.3.4", "internalIP": "10.0.0.2"}}
            store[obj["metadata"]["name"]] = obj
            return httpx.Response(201, json=obj)
        if p.startswith(base + "/"):
            name = p.rsplit("/", 1)[1]
            if name not in store:
                return httpx.Response(404, json={"reason": "NotFound"})
            if req.method == "GET":
                return httpx.Response(200, json=store[name])
            if req.method == "PATCH":
                store[name]["spec"].update(json.loads(req.content)["spec"])
                return httpx.Response(200, json=store[name])
            if req.method == "DELETE":
                del store[name]
                return httpx.Response(200, json={"status": "Success"})
        if "/subresources.kubevirt.io/" in p and req.method == "PUT":
            name, verb = p.split("/")[-2:]
            reason = {"stop": ("VirtualServerStopped", "False"), "start": ("VirtualServerReady", "True")}[verb]
            store[name]["status"]["conditions"] = [{"type": "Ready", "reason": reason[0], "status": reason[1]}]
            return httpx.Response(202)
        return httpx.Response(400)

    c = VirtualServerClient(K8sREST("https://k8s.example", "tok", transport=httpx.MockTransport(handler)))
    man = {"apiVersion": "virtualservers.coreweave.com/v1alpha1", "kind": "VirtualServer",
           "metadata": {"name": "vs1", "namespace": "ns"}, "spec": {"resources": {"cpu": {"count": 4}}}}
    c.create(man)
    st, ips = c.ready("ns", "vs1", poll_s=0.01)
    assert st == "Ready" and ips["externalIP"] == "1.2.3.4"
    c.stop("ns", "vs1")
    assert c.ready("ns", "vs1", "Stopped", poll_s=0.01)[0] == "Stopped"
    man["spec"]["resources"]["cpu"]["count"] = 8
    assert c.update(man)["spec"]["resources"]["cpu"]["count"] == 8
    c.start("ns", "vs1")
    assert c.ready("ns", "vs1", poll_s=0.01)[0] == "Ready"
    c.delete("ns", "vs1")
    assert c.ready("ns", "vs1", poll_s=0.01)[0] == "Deleted"
    assert ("PUT", "/apis/subresources.kubevirt.io/v1/namespaces/ns/virtualmachines/vs1/stop") in calls


def test_kubeconfig_parsing(tmp_path):
    kc = {"current-context": "c", "contexts": [{"name": "c", "context": {"cluster": "k", "user": "u"}}],
          "clusters": [{"name": "k", "cluster": {"server": "https://api.example:6443",
                                                  "insecure-skip-tls-verify": True}}],
          "users": [{"name": "u", "user": {"token": "abc"}}]}
    p = tmp_path / "kubeconfig"
    p.write_text(yaml.safe_dump(kc))
    api = K8sREST.from_kubeconfig(str(p))
    assert str(api.http.base_url).startswith("https://api.example:6443")
    assert api.http.headers["Authorization"] == "Bearer abc"
