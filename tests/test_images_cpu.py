"""Container images vs the manifests (deploy/images/Dockerfile, kubernetes_cloud_amd/deploy/images.py):
every image a manifest names is built by a Dockerfile target (or is a listed third-party image),
every package entry point a manifest starts is in the image, and the build context keeps what the
Dockerfile copies."""
import os
import shutil

import yaml

from kubernetes_cloud_amd.deploy import images as I


def test_manifests_and_images_consistent():
    assert I.check() == []


def test_every_manifest_image_is_built_or_external():
    seen = set()
    for p in I.manifest_files():
        for ref in I.images_in(p):
            assert ref in I.BUILD_TARGETS or ref in I.EXTERNAL, (p, ref)
            seen.add(ref)
    # both build targets are used, and the templated workflow images resolve to the runtime image
    assert set(I.BUILD_TARGETS) <= seen


def test_entrypoints_resolve_to_package_modules():
    mods = set()
    for p in I.manifest_files():
        mods |= set(I.modules_in(p))
    for must in ("kubernetes_cloud_amd.train.finetuner", "kubernetes_cloud_amd.serving.tp_server",
                 "kubernetes_cloud_amd.serving.triton_ft", "kubernetes_cloud_amd.serving.sd_service",
                 "kubernetes_cloud_amd.train.sd_finetuner", "kubernetes_cloud_amd.data.downloader"):
        assert must in mods
    for m in mods:
        assert I.module_file(m) is not None, m


def test_dev_tools_only_on_dev_image():
    """sshd / tini / jupyter are installed in the dev target only: containers that start them must
    name the dev image."""
    dev = [r for r, t in I.BUILD_TARGETS.items() if t == "dev"][0]

    def containers(o):
        if isinstance(o, dict):
            if "image" in o and ("command" in o or "args" in o):
                yield o
            for v in o.values():
                yield from containers(v)
        elif isinstance(o, list):
            for v in o:
                yield from containers(v)

    n = 0
    for p in I.manifest_files():
        for doc in yaml.safe_load_all(open(p)):
            for c in containers(doc):
                cmd = " ".join(map(str, (c.get("command") or []) + (c.get("args") or [])))
                if any(t in cmd for t in ("tini", "jupyter", "openssh", "service ssh")):
                    assert c["image"] == dev, (p, c["image"])
                    n += 1
    assert n >= 3


def test_check_catches_breakage(tmp_path):
    root = tmp_path / "repo"
    for d in ("deploy", "kubernetes_cloud_amd", "csrc", "tools", "tuning", "bench"):
        shutil.copytree(os.path.join(I.ROOT, d), root / d, ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    for f in (".dockerignore", "bench.py", "__graft_entry__.py"):
        shutil.copy(os.path.join(I.ROOT, f), root / f)
    assert I.check(str(root)) == []
    # an unknown image in a manifest
    bad = root / "deploy" / "argo-workflow" / "extra.yaml"
    bad.write_text("kind: Pod\nspec:\n  containers:\n  - name: x\n    image: example.com/nope:1\n")
    assert any("no build target" in p for p in I.check(str(root)))
    bad.unlink()
    # the build context dropping the package
    with open(root / ".dockerignore", "a") as f:
        f.write("kubernetes_cloud_amd/serving\n")
    probs = I.check(str(root))
    assert any("excluded from the build context" in p for p in probs)
