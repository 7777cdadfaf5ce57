"""VirtualServer (KubeVirt) control-plane client (P5) without the kubernetes SDK.

Covers the lifecycle the reference's examples drive
(virtual-server/examples/python/vsclient.py + kubevirtclient.py + main.py):
create -> wait Ready -> stop -> wait Stopped -> update -> start -> delete,
against the ``virtualservers.coreweave.com/v1alpha1`` CRD and KubeVirt's
``subresources.kubevirt.io/v1`` start/stop/restart endpoints. It talks plain
REST (httpx) with the kubeconfig's bearer token / client certificate or the
in-cluster service account, and waits by polling the object's first
``Ready`` condition (reason VirtualServerReady / VirtualServerStopped /
Terminating) rather than holding a watch stream open.

    python -m kubernetes_cloud_amd.platform.virtual_server --namespace ns \
        create manifest.yaml | ready NAME | stop NAME | start NAME | delete NAME | list
"""
from __future__ import annotations

import argparse
import base64
import json
import os
import tempfile
import time

GROUP, VERSION, PLURAL = "virtualservers.coreweave.com", "v1alpha1", "virtualservers"
CONDITIONS = {
    "Ready": ("VirtualServerReady", "True"),
    "Stopped": ("VirtualServerStopped", "False"),
    "Terminating": ("Terminating", "False"),
}


class K8sREST:
    def __init__(self, server: str, token: str | None = None, verify=True, cert=None, transport=None):
        import httpx
        headers = {"Authorization": f"Bearer {token}"} if token else {}
        kw = {"transport": transport} if transport is not None else {}
        self.http = httpx.Client(base_url=server.rstrip("/"), headers=headers, verify=verify, cert=cert,
                                 timeout=60.0, **kw)

    @classmethod
    def in_cluster(cls):
        sa = "/var/run/secrets/kubernetes.io/serviceaccount"
        with open(os.path.join(sa, "token")) as f:
            token = f.read().strip()
        host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ["KUBERNETES_SERVICE_PORT"]
        return cls(f"https://{host}:{port}", token, verify=os.path.join(sa, "ca.crt"))

    @classmethod
    def from_kubeconfig(cls, path: str | None = None):
        import yaml
        path = path or os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))
        with open(path) as f:
            kc = yaml.safe_load(f)
        ctx_name = kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        user = next(u["user"] for u in kc["users"] if u["name"] == ctx["user"])

        def materialise(data_key, file_key, src):
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp()
                with os.fdopen(fd, "wb") as f:
                    f.write(base64.b64decode(src[data_key]))
                return p
            return None
        ca = materialise("certificate-authority-data", "certificate-authority", cluster)
        verify = False if cluster.get("insecure-skip-tls-verify") else (ca or True)
        cert = None
        crt = materialise("client-certificate-data", "client-certificate", user)
        key = materialise("client-key-data", "client-key", user)
        if crt and key:
            cert = (crt, key)
        return cls(cluster["server"], user.get("token"), verify=verify, cert=cert)

    def request(self, method: str, path: str, body=None, content_type="application/json"):
        headers = {"Content-Type": content_type} if body is not None else {}
        r = self.http.request(method, path, content=json.dumps(body) if body is not None else None, headers=headers)
        if r.status_code >= 400:
            raise RuntimeError(f"{method} {path}: {r.status_code} {r.text[:500]}")
        return r.json() if r.content else {}


class VirtualServerClient:
    def __init__(self, api: K8sREST):
        self.api = api

    def _base(self, ns):
        return f"/apis/{GROUP}/{VERSION}/namespaces/{ns}/{PLURAL}"

    def create(self, manifest: dict):
        ns = manifest["metadata"].get("namespace", "default")
        return self.api.request("POST", self._base(ns), manifest)

    def update(self, manifest: dict):
        ns = manifest["metadata"].get("namespace", "default")
        name = manifest["metadata"]["name"]
        return self.api.request("PATCH", f"{self._base(ns)}/{name}", manifest, "application/merge-patch+json")

    def get(self, ns: str, name: str):
        return self.api.request("GET", f"{self._base(ns)}/{name}")

    def list(self, ns: str):
        return self.api.request("GET", self._base(ns))

    def delete(self, ns: str, name: str):
        return self.api.request("DELETE", f"{self._base(ns)}/{name}")

    def _vm(self, ns, name, verb):
        return self.api.request("PUT", f"/apis/subresources.kubevirt.io/v1/namespaces/{ns}/virtualmachines/{name}/{verb}",
                                {})

    def start(self, ns, name):
        return self._vm(ns, name, "start")

    def stop(self, ns, name):
        return self._vm(ns, name, "stop")

    def restart(self, ns, name):
        return self._vm(ns, name, "restart")

    @staticmethod
    def state_of(obj: dict) -> str | None:
        conds = (obj.get("status") or {}).get("conditions") or []
        if not conds:
            return None
        c = conds[0]
        for st, (reason, status) in CONDITIONS.items():
            if c.get("type") == "Ready" and c.get("reason") == reason and c.get("status") == status:
                return st
        return None

    def ready(self, ns: str, name: str, expected: str = "Ready", timeout_s: float = 1800, poll_s: float = 5.0):
        """Block until the first Ready-type condition matches ``expected``
        (or the object is gone -> "Deleted"); returns the state and, when
        Ready, the external/internal IPs."""
        t0 = time.time()
        while True:
            try:
                obj = self.get(ns, name)
            except RuntimeError as e:
                if " 404 " in str(e):
                    return "Deleted", {}
                raise
            st = self.state_of(obj)
            if st == expected or (st in ("Stopped", "Terminating") and expected != "Ready"):
                net = (obj.get("status") or {}).get("network") or {}
                return st, {"externalIP": net.get("externalIP", ""), "internalIP": net.get("internalIP", "")}
            if time.time() - t0 > timeout_s:
                raise TimeoutError(f"{name} not {expected} after {timeout_s}s (state {st})")
            time.sleep(poll_s)


def main(argv=None):
    import yaml
    ap = argparse.ArgumentParser(description="VirtualServer lifecycle client")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--namespace", "-n", default=os.environ.get("NAMESPACE", "default"))
    ap.add_argument("op", choices=["create", "update", "get", "list", "delete", "ready", "start", "stop", "restart"])
    ap.add_argument("arg", nargs="?", help="manifest file (create/update) or name")
    a = ap.parse_args(argv)
    api = K8sREST.in_cluster() if os.environ.get("KUBERNETES_SERVICE_HOST") and not a.kubeconfig \
        else K8sREST.from_kubeconfig(a.kubeconfig)
    c = VirtualServerClient(api)
    if a.op in ("create", "update"):
        with open(a.arg) as f:
            man = yaml.safe_load(f)
        man["metadata"].setdefault("namespace", a.namespace)
        out = getattr(c, a.op)(man)
    elif a.op == "list":
        out = c.list(a.namespace)
    elif a.op == "ready":
        out = c.ready(a.namespace, a.arg)
    else:
        out = getattr(c, a.op)(a.namespace, a.arg)
    print(json.dumps(out, indent=2, default=str))
    return out


if __name__ == "__main__":
    main()
