"""kubernetes_cloud_amd -- an MI355X-native (gfx950 / CDNA4) GPU-workflow stack.

Same capabilities and external contracts as the CoreWeave ``kubernetes-cloud``
examples (finetuner / SD finetuner / online-inference / kubeflow jobs), rebuilt
on PyTorch-ROCm + hand-written HIP kernels + RCCL over xGMI.
"""
__version__ = "0.1.0"
