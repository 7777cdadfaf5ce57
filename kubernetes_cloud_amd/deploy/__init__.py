"""Kubernetes manifests (Argo workflows, KServe ISVCs, Jobs) for MI355X nodes, rendered from Python."""
