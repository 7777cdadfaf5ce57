"""Kubernetes building blocks for MI355X nodes.

SURVEY §2.6 item 14: ``nvidia.com/gpu`` becomes the AMD device-plugin resource
``amd.com/gpu``; the ``gpu.nvidia.com/class`` node label becomes an MI355X
class label; shared memory stays an ``emptyDir: Memory`` on /dev/shm (RCCL and
the data loaders use it). Every manifest in ``deploy/`` is rendered from these
helpers (``python -m kubernetes_cloud_amd.deploy.render``) so resource names,
labels and the image are defined once.
"""
from __future__ import annotations

GPU_RESOURCE = "amd.com/gpu"
GPU_CLASS_LABEL = "gpu.amd.com/class"
REGION_LABEL = "topology.kubernetes.io/region"
# built by deploy/images/Dockerfile (targets: kubernetes_cloud_amd/deploy/images.py)
IMAGE = "ghcr.io/kubernetes-cloud-amd/kca"
DEV_IMAGE = "ghcr.io/kubernetes-cloud-amd/kca-dev"  # + sshd, tini, JupyterLab (dev-ssh, Jupyter)
TAG = "rocm7.2-gfx950"


def image(tag_param: str | None = None, image_param: str | None = None, dev: bool = False) -> str:
    if tag_param:
        return f"{{{{workflow.parameters.{image_param}}}}}:{{{{workflow.parameters.{tag_param}}}}}"
    return f"{DEV_IMAGE if dev else IMAGE}:{TAG}"


def affinity(gpu_class: str | None, region: str | None) -> dict:
    exprs = []
    if gpu_class:
        exprs.append({"key": GPU_CLASS_LABEL, "operator": "In", "values": [gpu_class]})
    if region:
        exprs.append({"key": REGION_LABEL, "operator": "In", "values": [region]})
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": exprs}]}}}


def resources(gpus=None, cpu=None, memory=None, ephemeral=None, limits_only=False) -> dict:
    r = {}
    if gpus is not None:
        r[GPU_RESOURCE] = gpus
    if cpu is not None:
        r["cpu"] = cpu
    if memory is not None:
        r["memory"] = memory
    if ephemeral is not None:
        r["ephemeral-storage"] = ephemeral
    return {"limits": dict(r)} if limits_only else {"requests": dict(r), "limits": dict(r)}


def pvc_volume(name: str) -> dict:
    return {"name": name, "persistentVolumeClaim": {"claimName": name}}


def shm_volume(size: str | None = None) -> dict:
    ed = {"medium": "Memory"}
    if size:
        ed["sizeLimit"] = size
    return {"name": "dshm", "emptyDir": ed}


def pvc(name: str, size: str, access: str = "ReadWriteMany", storage_class: str = "shared-nvme") -> dict:
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name},
            "spec": {"accessModes": [access], "storageClassName": storage_class,
                     "resources": {"requests": {"storage": size}}}}


def secret(name: str, key: str, placeholder: str = "<base64-encoded-value>") -> dict:
    return {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name}, "type": "Opaque",
            "data": {key: placeholder}}


def role_binding(name: str, sa: str = "inference") -> list[dict]:
    """Argo steps that create InferenceServices need RBAC on the ISVC CRD."""
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": sa}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": {"name": name},
         "rules": [{"apiGroups": ["serving.kubeflow.org", "serving.kserve.io"],
                    "resources": ["inferenceservices"],
                    "verbs": ["create", "delete", "get", "list", "watch", "patch", "update"]},
                   {"apiGroups": [""], "resources": ["pods", "pods/log"], "verbs": ["get", "list", "watch", "patch"]},
                   {"apiGroups": ["argoproj.io"], "resources": ["workflowtaskresults"],
                    "verbs": ["create", "patch"]}]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding", "metadata": {"name": name},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": name},
         "subjects": [{"kind": "ServiceAccount", "name": sa}]},
    ]


def wp(name: str) -> str:
    """Argo workflow-parameter reference."""
    return f"{{{{workflow.parameters.{name}}}}}"


def ip(name: str) -> str:
    return f"{{{{inputs.parameters.{name}}}}}"


ROCM_ENV = [
    {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},  # dmabuf IPC for RCCL / tensor sharing
    {"name": "NCCL_MIN_NCHANNELS", "value": "32"},          # use all xGMI links for large collectives
    {"name": "PYTHONUNBUFFERED", "value": "1"},
]
