"""Single-node launcher: one process per GPU (the deepspeed.launcher.runner /
accelerate launch / torchrun role).

    python -m kubernetes_cloud_amd.launch --num_gpus 8 /app/finetuner.py --run-name ...
    python -m kubernetes_cloud_amd.launch --num_processes 2 -m kubernetes_cloud_amd.train.sd_finetuner ...

Children get RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR /
MASTER_PORT (torchrun's env contract) plus ``--local_rank=i`` like DeepSpeed's
runner (finetune-workflow.yaml:507). If any rank fails, the others are
terminated and the launcher exits with that rank's code (Argo / Kubeflow see
the failure and apply their retry policy).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _count_gpus() -> int:
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
        or os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis:
        return len([v for v in vis.split(",") if v.strip()])
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def rank_env(i: int, n: int, master_addr: str, port: int, base=None) -> dict:
    """torchrun's env contract for rank ``i`` of ``n`` on one node."""
    return dict(os.environ if base is None else base, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), MASTER_ADDR=master_addr, MASTER_PORT=str(port),
                HSA_ENABLE_IPC_MODE_LEGACY="0")


def spawn(cmds, envs) -> int:
    """Run one child per rank (own process group each) and wait. If a rank
    fails, the others are terminated; returns the first non-zero exit code."""
    procs = [subprocess.Popen(c, env=e, start_new_session=True) for c, e in zip(cmds, envs)]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in procs:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.2)
    except KeyboardInterrupt:
        for q in procs:
            try:
                os.killpg(q.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        rc = 130
    return rc


def self_launch_argv(script: str, argv, n: int, master_addr: str = "127.0.0.1", port: int = 0):
    """(cmds, envs) to re-run ``script argv`` as ``n`` ranks -- used by entry
    points (bench.py) invoked with ``--gpus N`` outside torchrun. Must be
    called before anything initialises the GPU in the parent."""
    port = port or _free_port()
    cmds = [[sys.executable, "-u", script] + list(argv) for _ in range(n)]
    envs = [rank_env(i, n, master_addr, port) for i in range(n)]
    return cmds, envs


def main(argv=None):
    ap = argparse.ArgumentParser(description="kubernetes_cloud_amd single-node launcher")
    ap.add_argument("--num_gpus", "--num-gpus", "--num_processes", "--num-processes", "--nproc_per_node",
                    "--nproc-per-node", dest="n", type=int, default=-1)
    ap.add_argument("--master_addr", "--master-addr", default="127.0.0.1")
    ap.add_argument("--master_port", "--master-port", type=int, default=0)
    ap.add_argument("--no_local_rank", "--no-local-rank", action="store_true",
                    help="do not append --local_rank=i to the child's argv")
    argv = list(sys.argv[1:] if argv is None else argv)
    # launcher flags end at `-m MODULE` or at the first non-flag token (the script)
    split = len(argv)
    i = 0
    while i < len(argv):
        tok = argv[i]
        if tok == "-m" or not tok.startswith("-"):
            split = i
            break
        i += 1 if ("=" in tok or tok == "--no_local_rank" or tok == "--no-local-rank") else 2
    a = ap.parse_args(argv[:split])
    rest = argv[split:]
    if not rest:
        ap.error("script or -m module required")
    n = a.n if a.n > 0 else max(1, _count_gpus())
    port = a.master_port or _free_port()
    if rest[0] == "-m":
        base = [sys.executable, "-u", "-m", rest[1]]
        child_args = rest[2:]
    else:
        base = [sys.executable, "-u", rest[0]]
        child_args = rest[1:]
    cmds = [base + list(child_args) + ([] if a.no_local_rank else [f"--local_rank={i}"]) for i in range(n)]
    envs = [rank_env(i, n, a.master_addr, port) for i in range(n)]
    return spawn(cmds, envs)


if __name__ == "__main__":
    sys.exit(main())
