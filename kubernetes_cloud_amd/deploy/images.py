"""Container images of the deploy plane and the checks that tie them to the manifests.

``deploy/images/Dockerfile`` builds two images (reference: 24 per-component Dockerfiles, e.g.
``finetuner-workflow/finetuner/Dockerfile:1-50`` with its native-op builder stage,
``online-inference/bloom-176b-deepspeed/Dockerfile:1-15``, ``online-inference/stable-diffusion/
Dockerfile``): every trainer, predictor and workflow step of this tree is one Python package, so one
runtime image (the package, its gfx950 libraries built in a builder stage, ``tuning/``) serves them
all, and a dev image adds sshd / tini / JupyterLab for the interactive deployments.

    python -m kubernetes_cloud_amd.deploy.images            # the docker build commands
    python -m kubernetes_cloud_amd.deploy.images --check    # manifests <-> images consistency
    python -m kubernetes_cloud_amd.deploy.images --build    # run the builds (needs docker buildx)
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys

import yaml

from .k8s import DEV_IMAGE, IMAGE, TAG

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
DOCKERFILE = os.path.join("deploy", "images", "Dockerfile")

# image reference -> Dockerfile target
BUILD_TARGETS = {f"{IMAGE}:{TAG}": "runtime", f"{DEV_IMAGE}:{TAG}": "dev"}
# third-party images a manifest may name as-is (the reference's own choices for these steps)
EXTERNAL = {
    "ghcr.io/coreweave/dataset-downloader/smashwords-downloader:cd6408a",  # finetune-workflow.yaml default
    "cirrusci/wget:latest",  # gpt-neox 04-finetune-workflow.yaml downloader
    "alpine:3.19",
}

_PARAM = re.compile(r"\{\{\s*workflow\.parameters\.([A-Za-z0-9_]+)\s*\}\}")
_IMAGE_LINE = re.compile(r"""image:\s*['"]?([^\s'"\\,]+)""")
_MODULE = re.compile(r"kubernetes_cloud_amd(?:\.[A-Za-z0-9_]+)+")


def manifest_files(root: str = ROOT) -> list[str]:
    out = []
    for d, _, fs in os.walk(os.path.join(root, "deploy")):
        if os.path.relpath(d, root).startswith(os.path.join("deploy", "images")):
            continue
        out += [os.path.join(d, f) for f in fs if f.endswith((".yaml", ".yml"))]
    return sorted(out)


def _param_defaults(text: str) -> dict:
    vals = {}

    def walk(o):
        if isinstance(o, dict):
            if "name" in o and "value" in o and isinstance(o.get("value"), (str, int, float)):
                vals.setdefault(str(o["name"]), str(o["value"]))
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            for v in o:
                walk(v)

    for doc in yaml.safe_load_all(text):
        walk(doc)
    return vals


def images_in(path: str) -> list[str]:
    """Every image a manifest names, workflow parameters resolved to their defaults."""
    text = open(path).read()
    params = _param_defaults(text)
    out = []
    for m in _IMAGE_LINE.finditer(text.replace("\\n", "\n")):
        ref = m.group(1)
        full = text[m.start():text.find("\n", m.start())]
        if "{{" in full:  # re-read the whole templated value
            tmpl = re.search(r"image:\s*['\"]?(\{\{[^'\"\n]*\}\}(?::\{\{[^'\"\n]*\}\})?)", full)
            ref = tmpl.group(1) if tmpl else ref
        ref = _PARAM.sub(lambda p: params.get(p.group(1), p.group(0)), ref)
        out.append(ref)
    return out


def modules_in(path: str) -> list[str]:
    """Package modules a manifest starts or imports (``python3 -m kubernetes_cloud_amd.X`` in a
    command list, ``from kubernetes_cloud_amd.X import main`` in a ``-c`` one-liner)."""
    return sorted(set(_MODULE.findall(open(path).read())))


def module_file(mod: str, root: str = ROOT) -> str | None:
    """The file a dotted reference resolves to (its longest module prefix: ``pkg.mod.attr`` ->
    ``pkg/mod.py``)."""
    parts = mod.split(".")
    for n in range(len(parts), 1, -1):
        rel = os.path.join(root, *parts[:n])
        for cand in (rel + ".py", os.path.join(rel, "__init__.py")):
            if os.path.exists(cand):
                return cand
    return None


def dockerfile_targets(root: str = ROOT) -> dict:
    """stage name -> list of COPY sources (build context paths)."""
    stages, cur = {}, None
    for line in open(os.path.join(root, DOCKERFILE)):
        s = line.strip()
        m = re.match(r"FROM\s+\S+(?:\s+AS\s+(\S+))?", s, re.I)
        if m:
            cur = m.group(1) or f"stage{len(stages)}"
            stages[cur] = []
            continue
        m = re.match(r"COPY\s+(.*)", s, re.I)
        if m and cur:
            toks = [t for t in m.group(1).split() if not t.startswith("--")]
            if "--from" not in m.group(1):
                stages[cur] += toks[:-1]
    return stages


def dockerignore(root: str = ROOT) -> list[str]:
    p = os.path.join(root, ".dockerignore")
    if not os.path.exists(p):
        return []
    return [ln.strip() for ln in open(p) if ln.strip() and not ln.startswith("#")]


def _ignored(rel: str, patterns: list[str]) -> bool:
    import fnmatch
    rel = rel.replace(os.sep, "/")
    for pat in patterns:
        pat = pat.rstrip("/")
        if pat.startswith("**/"):
            if fnmatch.fnmatch(os.path.basename(rel), pat[3:]) or fnmatch.fnmatch(rel, pat[3:]):
                return True
        elif rel == pat or rel.startswith(pat + "/") or fnmatch.fnmatch(rel, pat):
            return True
    return False


def check(root: str = ROOT) -> list[str]:
    """Problems (empty = consistent): unbuilt images, entry points missing from the package or the
    image, build-context exclusions of what the images copy."""
    problems = []
    stages = dockerfile_targets(root)
    for ref, target in BUILD_TARGETS.items():
        if target not in stages:
            problems.append(f"{ref}: target {target!r} not in {DOCKERFILE}")
    ign = dockerignore(root)
    for st, srcs in stages.items():
        for src in srcs:
            if _ignored(src, ign):
                problems.append(f"{DOCKERFILE} stage {st} copies {src}, which .dockerignore excludes")
            if not os.path.exists(os.path.join(root, src)):
                problems.append(f"{DOCKERFILE} stage {st} copies {src}, which does not exist")
    # the runtime image carries the package (built in `build`, copied --from) and tuning/
    build_srcs = stages.get("build", [])
    if "kubernetes_cloud_amd" not in build_srcs or "csrc" not in build_srcs:
        problems.append("build stage must copy kubernetes_cloud_amd and csrc")
    for path in manifest_files(root):
        rel = os.path.relpath(path, root)
        for ref in images_in(path):
            if ref not in BUILD_TARGETS and ref not in EXTERNAL:
                problems.append(f"{rel}: image {ref} has no build target")
        for mod in modules_in(path):
            f = module_file(mod, root)
            if f is None:
                problems.append(f"{rel}: entry point {mod} not in the package")
            elif _ignored(os.path.relpath(f, root), ign):
                problems.append(f"{rel}: entry point {mod} excluded from the build context")
    return problems


def build_commands(push: bool = False) -> list[list[str]]:
    cmds = []
    for ref, target in BUILD_TARGETS.items():
        c = ["docker", "buildx", "build", "-f", DOCKERFILE, "--target", target, "-t", ref, "."]
        if push:
            c.insert(3, "--push")
        cmds.append(c)
    return cmds


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--push", action="store_true")
    a = ap.parse_args(argv)
    if a.check:
        probs = check()
        for p in probs:
            print(p)
        sys.exit(1 if probs else 0)
    for c in build_commands(a.push):
        print(" ".join(c))
        if a.build:
            subprocess.run(c, check=True, cwd=ROOT)


if __name__ == "__main__":
    main()
