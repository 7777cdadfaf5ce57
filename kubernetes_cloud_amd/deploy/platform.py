"""Platform / dev-environment manifests for MI355X nodes.

* ``dev_ssh``  -- persistent GPU dev box over SSH (cuda-ssh/sshd-deployment.yaml:
  1-131): the root filesystem is copied once onto a PVC by an init container
  and sub-path mounted back, so installed packages survive restarts; a
  LoadBalancer service exposes port 22. ROCm/RCCL image instead of CUDA/NCCL,
  ``amd.com/gpu`` instead of ``nvidia.com/gpu`` (6 GPUs as in the reference).
* ``jupyter``  -- notebook pod (tensorflow-jupyter/*.yaml, 2 GPUs) running
  JupyterLab on the framework's PyTorch-ROCm image.
* ``spark``    -- Spark-on-K8s img2dataset job plumbing (spark/spark-role.yaml,
  spark-pvc.yaml, cpu-pod-template.yaml, jupyter/jupyter-service.yaml): service
  account + role, a CPU pod template for driver/executors, the data PVC and an
  interactive Jupyter driver. The job itself is ``kubernetes_cloud_amd.data.
  img2dataset`` (CPU only; no GPU content, as in the reference).
"""
from __future__ import annotations

from .k8s import affinity, image, pvc, pvc_volume, resources, shm_volume

ROOT_DIRS = ["bin", "boot", "etc", "home", "lib", "lib64", "opt", "root", "sbin", "srv", "usr", "var"]


def _deployment(name: str, pod_spec: dict, labels: dict | None = None) -> dict:
    labels = labels or {"app.kubernetes.io/name": name}
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name},
            "spec": {"strategy": {"type": "Recreate"}, "replicas": 1, "selector": {"matchLabels": labels},
                     "template": {"metadata": {"labels": labels}, "spec": pod_spec}}}


def _service(name: str, port: int, target: int, svc_type: str = "LoadBalancer", selector: dict | None = None) -> dict:
    spec = {"type": svc_type}
    if svc_type == "LoadBalancer":
        spec["externalTrafficPolicy"] = "Local"
    spec["ports"] = [{"name": name, "port": port, "targetPort": target, "protocol": "TCP"}]
    spec["selector"] = selector or {"app.kubernetes.io/name": name}
    return {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name}, "spec": spec}


def dev_ssh(gpus: int = 6) -> dict:
    init = {"name": "init", "image": image(dev=True), "command": ["/bin/bash", "-c"],
            "args": ["if [ ! -f /target/initialized ]; then dpkg-reconfigure openssh-server && cp -ax / /target && "
                     "echo 'Initialization complete' && touch /target/initialized; fi"],
            "resources": {"requests": {"cpu": 1, "memory": "1Gi"}},
            "volumeMounts": [{"name": "root-storage", "mountPath": "/target"}]}
    mounts = [{"name": "data-storage", "mountPath": "/mnt/data"}, {"name": "dshm", "mountPath": "/dev/shm"}]
    mounts += [{"name": "root-storage", "mountPath": f"/{d}", "subPath": d} for d in ROOT_DIRS]
    main = {"name": "sshd", "image": image(dev=True), "command": ["/usr/bin/tini", "--"],
            "args": ["service", "ssh", "start", "-D"], "tty": True,
            "ports": [{"name": "sshd", "containerPort": 22, "protocol": "TCP"}],
            "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
            "volumeMounts": mounts, "resources": resources(gpus=gpus, cpu=30, memory="512Gi", limits_only=True)}
    spec = {"terminationGracePeriodSeconds": 10, "initContainers": [init], "containers": [main],
            "volumes": [pvc_volume("sshd-root-pv-claim") | {"name": "root-storage"},
                        pvc_volume("sshd-data-pv-claim") | {"name": "data-storage"}, shm_volume("256Gi")],
            "affinity": affinity("MI355X", "ORD1")}
    return {
        "sshd-root-pvc.yaml": pvc("sshd-root-pv-claim", "100Gi", access="ReadWriteOnce", storage_class="block-nvme"),
        "sshd-data-pvc.yaml": pvc("sshd-data-pv-claim", "1000Gi"),
        "sshd-deployment.yaml": _deployment("sshd", spec),
        "sshd-service.yaml": _service("sshd", 22, 22),
    }


def jupyter(gpus: int = 2) -> dict:
    c = {"name": "jupyter", "image": image(dev=True), "command": ["jupyter", "lab"],
         "args": ["--ip=0.0.0.0", "--port=8888", "--no-browser", "--allow-root",
                  "--ServerApp.token=$(JUPYTER_TOKEN)", "--notebook-dir=/mnt/pvc"],
         "env": [{"name": "JUPYTER_TOKEN", "valueFrom": {"secretKeyRef": {"name": "jupyter-token", "key": "token"}}}],
         "ports": [{"name": "notebook", "containerPort": 8888, "protocol": "TCP"}],
         "readinessProbe": {"tcpSocket": {"port": "notebook"}, "initialDelaySeconds": 5, "periodSeconds": 10},
         "volumeMounts": [{"name": "jupyter-data", "mountPath": "/mnt/pvc"}, {"name": "dshm", "mountPath": "/dev/shm"}],
         "resources": resources(gpus=gpus, cpu=8, memory="64Gi", limits_only=True)}
    spec = {"containers": [c], "volumes": [pvc_volume("jupyter-pv-claim") | {"name": "jupyter-data"}, shm_volume()],
            "affinity": affinity("MI355X", "ORD1")}
    return {
        "jupyter-pvc.yaml": pvc("jupyter-pv-claim", "300Gi"),
        "jupyter-deployment.yaml": _deployment("jupyter", spec),
        "jupyter-service.yaml": _service("jupyter", 80, 8888),
    }


def spark() -> dict:
    sa = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "spark-sa"}}
    role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": "spark-role"},
            "rules": [{"apiGroups": [""], "resources": ["pods", "services", "configmaps", "persistentvolumeclaims"],
                       "verbs": ["create", "get", "list", "watch", "delete", "deletecollection", "patch", "update"]}]}
    rb = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding", "metadata": {"name": "spark-rb"},
          "subjects": [{"kind": "ServiceAccount", "name": "spark-sa"}],
          "roleRef": {"kind": "Role", "name": "spark-role", "apiGroup": "rbac.authorization.k8s.io"}}
    template = {"apiVersion": "v1", "kind": "Pod", "spec": {
        "containers": [{"name": "spark", "volumeMounts": [{"name": "spark-pvc", "mountPath": "/mnt/pvc"}]}],
        "volumes": [pvc_volume("spark-pvc") | {"name": "spark-pvc"}],
        "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
            {"matchExpressions": [{"key": "node.coreweave.cloud/cpu", "operator": "In",
                                   "values": ["amd-epyc-genoa", "amd-epyc-turin"]},
                                  {"key": "topology.kubernetes.io/region", "operator": "In",
                                   "values": ["ORD1"]}]}]}}}}}
    drv = {"name": "jupyter", "image": image(dev=True), "command": ["jupyter", "lab"],
           "args": ["--ip=0.0.0.0", "--port=8888", "--no-browser", "--allow-root", "--notebook-dir=/mnt/pvc"],
           "ports": [{"containerPort": 8888}, {"containerPort": 7078, "name": "driver-rpc"},
                     {"containerPort": 7079, "name": "blockmanager"}],
           "volumeMounts": [{"name": "spark-pvc", "mountPath": "/mnt/pvc"}],
           "resources": resources(cpu=16, memory="64Gi")}
    jspec = {"serviceAccountName": "spark-sa", "containers": [drv],
             "volumes": [pvc_volume("spark-pvc") | {"name": "spark-pvc"}]}
    headless = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "spark-jupyter-driver"},
                "spec": {"clusterIP": "None", "selector": {"app.kubernetes.io/name": "spark-jupyter"},
                         "ports": [{"name": "driver-rpc", "port": 7078}, {"name": "blockmanager", "port": 7079}]}}
    return {
        "spark-role.yaml": [sa, role, rb],
        "spark-pvc.yaml": pvc("spark-pvc", "400Gi"),
        "cpu-pod-template.yaml": template,
        "jupyter/jupyter-service.yaml": [_deployment("spark-jupyter", jspec), headless,
                                         _service("spark-jupyter", 80, 8888, selector={
                                             "app.kubernetes.io/name": "spark-jupyter"})],
    }
