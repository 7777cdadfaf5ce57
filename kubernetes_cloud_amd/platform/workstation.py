"""Workstation bootstrap (P6): install kubectl, virtctl and helm for the host
OS/arch, put them on PATH and import the cluster kubeconfig.

Reference behaviour: ``getting-started/k8ctl_setup.ps1`` (Windows-only
PowerShell: pinned or ``-UseLatest`` versions of the three CLIs under
``%ProgramData%\\k8s`` (:32-46), PATH update (:50-55), kubeconfig import
into ``~/.kube/config`` (:230-252), ``-Uninstall`` (:260-275)). This is one
portable CLI instead (Windows, Linux, macOS; amd64/arm64) so the same
getting-started step works from the Linux hosts an MI355X cluster is usually
driven from:

    python -m kubernetes_cloud_amd.platform.workstation [--dest DIR]
        [--use-latest] [--kubeconfig FILE] [--mirror URL] [--dry-run] [--uninstall]

``--mirror`` replaces every download origin with one base URL (an internal
artifact mirror, or ``file://`` for air-gapped installs): the files are then
looked up as ``<mirror>/<tool>/<version>/<asset>``.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import shutil
import stat
import sys
import tarfile
import urllib.request
import zipfile

PINNED = {"kubectl": "v1.30.2", "virtctl": "v1.2.2", "helm": "v3.15.2"}


def host_target(system: str | None = None, machine: str | None = None) -> tuple[str, str]:
    s = (system or platform.system()).lower()
    m = (machine or platform.machine()).lower()
    os_ = {"windows": "windows", "linux": "linux", "darwin": "darwin"}.get(s)
    arch = {"x86_64": "amd64", "amd64": "amd64", "aarch64": "arm64", "arm64": "arm64"}.get(m)
    if os_ is None or arch is None:
        raise SystemExit(f"unsupported host {s}/{m}")
    return os_, arch


def _latest(tool: str) -> str:
    if tool == "kubectl":
        with urllib.request.urlopen("https://dl.k8s.io/release/stable.txt", timeout=30) as r:
            return r.read().decode().strip()
    repo = {"virtctl": "kubevirt/kubevirt", "helm": "helm/helm"}[tool]
    with urllib.request.urlopen(f"https://api.github.com/repos/{repo}/releases/latest", timeout=30) as r:
        return json.load(r)["tag_name"]


def plan(os_: str, arch: str, versions: dict, mirror: str | None = None) -> list[dict]:
    """One entry per tool: download URL, archive member (helm) and binary name."""
    exe = ".exe" if os_ == "windows" else ""
    out = []
    for tool in ("kubectl", "virtctl", "helm"):
        v = versions[tool]
        if tool == "kubectl":
            asset, url = f"kubectl{exe}", f"https://dl.k8s.io/release/{v}/bin/{os_}/{arch}/kubectl{exe}"
            member = None
        elif tool == "virtctl":
            asset = f"virtctl-{v}-{os_}-{arch}{exe}"
            url = f"https://github.com/kubevirt/kubevirt/releases/download/{v}/{asset}"
            member = None
        else:
            asset = f"helm-{v}-{os_}-{arch}." + ("zip" if os_ == "windows" else "tar.gz")
            url = f"https://get.helm.sh/{asset}"
            member = f"{os_}-{arch}/helm{exe}"
        if mirror:
            url = f"{mirror.rstrip('/')}/{tool}/{v}/{asset}"
        out.append({"tool": tool, "version": v, "url": url, "member": member, "binary": f"{tool}{exe}"})
    return out


def _fetch(url: str, dst: str) -> None:
    with urllib.request.urlopen(url, timeout=120) as r, open(dst, "wb") as f:
        shutil.copyfileobj(r, f)


def install(entries: list[dict], dest: str) -> list[str]:
    os.makedirs(dest, exist_ok=True)
    done = []
    for e in entries:
        target = os.path.join(dest, e["binary"])
        tmp = target + ".download"
        _fetch(e["url"], tmp)
        if e["member"]:  # helm ships in an archive
            if e["url"].endswith(".zip"):
                with zipfile.ZipFile(tmp) as z, z.open(e["member"]) as src, open(target, "wb") as f:
                    shutil.copyfileobj(src, f)
            else:
                with tarfile.open(tmp) as t:
                    src = t.extractfile(e["member"])
                    with open(target, "wb") as f:
                        shutil.copyfileobj(src, f)
            os.remove(tmp)
        else:
            os.replace(tmp, target)
        os.chmod(target, os.stat(target).st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)
        done.append(target)
    return done


def import_kubeconfig(src: str, home: str | None = None) -> str:
    home = home or os.path.expanduser("~")
    kdir = os.path.join(home, ".kube")
    os.makedirs(kdir, exist_ok=True)
    dst = os.path.join(kdir, "config")
    if os.path.exists(dst):
        shutil.copy2(dst, dst + ".bak")
    shutil.copy2(src, dst)
    os.chmod(dst, 0o600)
    return dst


def path_hint(dest: str, os_: str) -> str | None:
    if dest in os.environ.get("PATH", "").split(os.pathsep):
        return None
    if os_ == "windows":
        return f'setx PATH "%PATH%;{dest}"'
    return f'export PATH="$PATH:{dest}"   # add to ~/.bashrc or ~/.zshrc'


def uninstall(dest: str, home: str | None = None, remove_kubeconfig: bool = False) -> list[str]:
    removed = []
    if os.path.isdir(dest):
        shutil.rmtree(dest)
        removed.append(dest)
    if remove_kubeconfig:
        kdir = os.path.join(home or os.path.expanduser("~"), ".kube")
        if os.path.isdir(kdir):
            shutil.rmtree(kdir)
            removed.append(kdir)
    return removed


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    default_dest = (os.path.join(os.environ.get("ProgramData", "C:\\ProgramData"), "k8s")
                    if os.name == "nt" else os.path.expanduser("~/.local/k8s/bin"))
    ap.add_argument("--dest", default=default_dest)
    ap.add_argument("--use-latest", action="store_true", help="resolve the newest releases instead of the pins")
    ap.add_argument("--tools", default="kubectl,virtctl,helm")
    ap.add_argument("--kubeconfig", help="cluster kubeconfig to import into ~/.kube/config")
    ap.add_argument("--mirror", help="base URL replacing the public download origins")
    ap.add_argument("--os", dest="os_", help="override the detected OS (windows/linux/darwin)")
    ap.add_argument("--arch", help="override the detected arch (amd64/arm64)")
    ap.add_argument("--dry-run", action="store_true", help="print the plan as JSON, change nothing")
    ap.add_argument("--uninstall", action="store_true")
    ap.add_argument("--remove-kubeconfig", action="store_true", help="with --uninstall: also remove ~/.kube")
    a = ap.parse_args(argv)
    if a.uninstall:
        print(json.dumps({"removed": uninstall(a.dest, remove_kubeconfig=a.remove_kubeconfig)}))
        return 0
    os_, arch = host_target(a.os_, a.arch)
    versions = {t: (_latest(t) if a.use_latest else PINNED[t]) for t in PINNED}
    wanted = set(a.tools.split(","))
    entries = [e for e in plan(os_, arch, versions, a.mirror) if e["tool"] in wanted]
    if a.dry_run:
        print(json.dumps({"os": os_, "arch": arch, "dest": a.dest, "tools": entries}, indent=1))
        return 0
    installed = [e for e in entries if shutil.which(e["binary"]) is None
                 and not os.path.exists(os.path.join(a.dest, e["binary"]))]
    out = {"installed": install(installed, a.dest)}
    if a.kubeconfig:
        out["kubeconfig"] = import_kubeconfig(a.kubeconfig)
    elif not os.path.exists(os.path.expanduser("~/.kube/config")):
        print("warning: no kubeconfig at ~/.kube/config; pass --kubeconfig FILE", file=sys.stderr)
    hint = path_hint(a.dest, os_)
    if hint:
        out["path_hint"] = hint
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
