"""Training jobs outside Argo (T13): ResNet-50 ImageNet data-parallel.

The reference ran the same script two ways -- a PyTorchJob with torchrun + DDP
(k8s/imagenet-pytorchjob.yaml) and an MPIJob with Horovod
(k8s/imagenet-mpijob.yaml). Here both are one PyTorchJob running
``train.resnet`` (DDP over RCCL); the Horovod knobs (``--fp16-allreduce``,
``--gradient-predivide-factor``, ``--use-mixed-precision``) are flags of the
same trainer, so the MPI launcher, SSH keys and sleep hack are gone.
"""
from __future__ import annotations

from .k8s import ROCM_ENV, affinity, image, pvc, resources, shm_volume


def resnet50(nodes: int = 2) -> dict:
    def job(name, extra):
        return {
            "apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": name},
            "spec": {"pytorchReplicaSpecs": {
                role: {"replicas": n, "restartPolicy": "OnFailure", "template": {"spec": {
                    "affinity": affinity("MI355X", None),
                    "containers": [{
                        "name": "pytorch", "image": image(),
                        "command": ["torchrun", "--nproc_per_node=8", "--nnodes=$(WORLD_SIZE)",
                                    "--node_rank=$(RANK)", "--master_addr=$(MASTER_ADDR)",
                                    "--master_port=$(MASTER_PORT)", "-m", "kubernetes_cloud_amd.train.resnet"],
                        "args": ["--backend", "nccl", "--log-dir", "/mnt/pvc/pytorch/logs",
                                 "--data-dir", "/mnt/pvc/dataset/ILSVRC/Data/CLS-LOC",
                                 "--model-dir", "/mnt/pvc/pytorch/checkpoints", "--epochs", "10",
                                 "--batch-size", "256", "--wandb-project", "resnet50-imagenet-pytorch",
                                 "--wandb-run", f"mi355x-{8 * nodes}gpu"] + extra,
                        "env": [{"name": "WANDB_API_KEY", "valueFrom": {"secretKeyRef": {
                            "name": "wandb-token-secret", "key": "token", "optional": True}}}] + list(ROCM_ENV),
                        "resources": resources(gpus=8, cpu=96, memory="700G"),
                        "volumeMounts": [{"name": "kubeflow-resnet50", "mountPath": "/mnt/pvc"},
                                         {"name": "dshm", "mountPath": "/dev/shm"}]}],
                    "volumes": [{"name": "kubeflow-resnet50",
                                 "persistentVolumeClaim": {"claimName": "kubeflow-resnet50"}}, shm_volume()]}}}
                for role, n in (("Master", 1), ("Worker", nodes - 1)) if n > 0}}}
    download = {
        "apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "imagenet-download"},
        "spec": {"template": {"spec": {
            "restartPolicy": "Never",
            "containers": [{"name": "download", "image": image(), "command": ["bash", "-c"],
                            "args": ["mkdir -p /mnt/pvc/dataset && cd /mnt/pvc/dataset && "
                                     "kaggle competitions download -c imagenet-object-localization-challenge && "
                                     "unzip -q imagenet-object-localization-challenge.zip && "
                                     "python3 -m kubernetes_cloud_amd.train.resnet --prepare-val "
                                     "--data-dir /mnt/pvc/dataset/ILSVRC/Data/CLS-LOC "
                                     "--val-labels /mnt/pvc/dataset/LOC_val_solution.csv"],
                            "env": [{"name": "KAGGLE_USERNAME", "valueFrom": {"secretKeyRef": {
                                "name": "kaggle-token-secret", "key": "username"}}},
                                {"name": "KAGGLE_KEY", "valueFrom": {"secretKeyRef": {
                                    "name": "kaggle-token-secret", "key": "key"}}}],
                            "resources": resources(cpu=16, memory="32Gi"),
                            "volumeMounts": [{"name": "kubeflow-resnet50", "mountPath": "/mnt/pvc"}]}],
            "volumes": [{"name": "kubeflow-resnet50", "persistentVolumeClaim": {"claimName": "kubeflow-resnet50"}}]}}}}
    return {
        "model-pvc.yaml": pvc("kubeflow-resnet50", "400Gi"),
        "imagenet-download-job.yaml": download,
        "imagenet-pytorchjob.yaml": job("resnet50-ddp", []),
        "imagenet-pytorchjob-fp16-allreduce.yaml": job("resnet50-ddp-fp16ar", ["--fp16-allreduce",
                                                                              "--use-mixed-precision"]),
    }


__all__ = ["resnet50"]
