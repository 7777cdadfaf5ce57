"""HF hub snapshot downloader into ``$HF_HOME`` (the BLOOM DeepSpeed example's
downloader: online-inference/bloom-176b-deepspeed/downloader/download.py:1-10,
``--model-id`` / ``--revision`` -> ``huggingface_hub.snapshot_download``).

The serving side resolves the result read-only through the hub cache layout
``hub/models--{org}--{name}/refs/{revision}`` -> ``snapshots/{sha}``
(``serving.bloom_server.resolve_hf_cache_path``, isvc-patch.txt:55-77).
``KCA_HF_MIRROR=<dir>`` populates the same layout from a local mirror
(air-gapped clusters, tests) instead of the network.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import sys


def _mirror(src: str, model_id: str, revision: str, hf_home: str) -> str:
    org_name = "models--" + model_id.replace("/", "--")
    root = os.path.join(hf_home, "hub", org_name)
    sha = hashlib.sha1(f"{model_id}@{revision}".encode()).hexdigest()
    snap = os.path.join(root, "snapshots", sha)
    if os.path.isdir(snap):
        shutil.rmtree(snap)
    shutil.copytree(src, snap)
    os.makedirs(os.path.join(root, "refs"), exist_ok=True)
    with open(os.path.join(root, "refs", revision), "w") as f:
        f.write(sha)
    return snap


def main(argv=None):
    ap = argparse.ArgumentParser(description="snapshot an HF hub repo into $HF_HOME")
    ap.add_argument("--model-id", required=True)
    ap.add_argument("--revision", default="main")
    a = ap.parse_args(argv)
    hf_home = os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface"))
    mirror = os.environ.get("KCA_HF_MIRROR")
    if mirror:
        path = _mirror(mirror, a.model_id, a.revision, hf_home)
    else:
        from huggingface_hub import snapshot_download
        path = snapshot_download(repo_id=a.model_id, revision=a.revision)
    print(path)
    return path


if __name__ == "__main__":
    main()
    sys.exit(0)
