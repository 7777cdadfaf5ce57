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


def test_workstation_bootstrap_offline_mirror(tmp_path, monkeypatch):
    """P6 (getting-started/k8ctl_setup.ps1): plan per OS/arch, install the
    three CLIs from a file:// mirror (helm out of its archive), import the
    kubeconfig, uninstall."""
    import io
    import json
    import tarfile
    import zipfile

    from kubernetes_cloud_amd.platform import workstation as ws

    assert ws.host_target("Windows", "AMD64") == ("windows", "amd64")
    assert ws.host_target("Linux", "aarch64") == ("linux", "arm64")
    p = {e["tool"]: e for e in ws.plan("windows", "amd64", ws.PINNED)}
    assert p["kubectl"]["url"].endswith("/bin/windows/amd64/kubectl.exe")
    assert p["helm"]["url"].endswith(".zip") and p["helm"]["member"] == "windows-amd64/helm.exe"
    assert p["virtctl"]["binary"] == "virtctl.exe"

    mirror = tmp_path / "mirror"
    for e in ws.plan("linux", "amd64", ws.PINNED, f"file://{mirror}"):
        f = mirror / e["tool"] / e["version"]
        f.mkdir(parents=True)
        asset = e["url"].rsplit("/", 1)[1]
        if e["member"]:
            with tarfile.open(f / asset, "w:gz") as t:
                data = b"#!/bin/sh\necho helm\n"
                info = tarfile.TarInfo(e["member"])
                info.size = len(data)
                t.addfile(info, io.BytesIO(data))
        else:
            (f / asset).write_bytes(b"#!/bin/sh\necho " + e["tool"].encode() + b"\n")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    monkeypatch.setattr(ws.shutil, "which", lambda name: None)
    kc = tmp_path / "cw-kubeconfig"
    kc.write_text("apiVersion: v1\nkind: Config\n")
    dest = tmp_path / "k8s"
    rc = ws.main(["--dest", str(dest), "--os", "linux", "--arch", "amd64", "--mirror", f"file://{mirror}",
                  "--kubeconfig", str(kc)])
    assert rc == 0
    for b in ("kubectl", "virtctl", "helm"):
        assert (dest / b).exists() and (dest / b).stat().st_mode & 0o111
    assert (tmp_path / "home" / ".kube" / "config").read_text().startswith("apiVersion")
    assert ws.main(["--dest", str(dest), "--uninstall"]) == 0 and not dest.exists()
    # the zip layout used on Windows
    z = tmp_path / "h.zip"
    with zipfile.ZipFile(z, "w") as zz:
        zz.writestr("windows-amd64/helm.exe", b"MZ")
    ent = [{"tool": "helm", "version": "v0", "url": f"file://{z}", "member": "windows-amd64/helm.exe",
            "binary": "helm.exe"}]
    assert ws.install(ent, str(tmp_path / "w"))[0].endswith("helm.exe")
    assert json.loads(json.dumps(ws.plan("darwin", "arm64", ws.PINNED)))[2]["url"].endswith("darwin-arm64.tar.gz")
