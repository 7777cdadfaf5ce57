"""Control-plane helpers (no GPU code): VirtualServer / KubeVirt client."""
