"""Launcher contract: `bench.py --gpus N` outside torchrun re-runs itself as N
ranks with torchrun's env (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), and the
generic launcher appends DeepSpeed's --local_rank (finetune-workflow.yaml:507)."""
import json
import os
import subprocess
import sys

from kubernetes_cloud_amd.launch import main as launch_main
from kubernetes_cloud_amd.launch import rank_env, self_launch_argv, spawn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import json, os, sys
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "HSA_ENABLE_IPC_MODE_LEGACY")
with open(os.path.join(sys.argv[1], "r%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({"env": {k: os.environ.get(k) for k in keys}, "argv": sys.argv[2:]}, f)
"""


def test_self_launch_argv_env():
    cmds, envs = self_launch_argv("/x/bench.py", ["--gpus", "4", "--steps", "3"], 4, port=29511)
    assert len(cmds) == 4 and all(c[-5:] == ["/x/bench.py", "--gpus", "4", "--steps", "3"] for c in cmds)
    assert all(c[0] == sys.executable for c in cmds)
    for i, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(i)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_spawn_runs_every_rank_and_propagates_failure(tmp_path):
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    cmds, envs = self_launch_argv(str(probe), [str(tmp_path), "--k", "v"], 3)
    assert spawn(cmds, envs) == 0
    for r in range(3):
        rec = json.loads((tmp_path / f"r{r}.json").read_text())
        assert rec["env"]["RANK"] == str(r) and rec["env"]["WORLD_SIZE"] == "3"
        assert rec["argv"] == ["--k", "v"]
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(30)\n")
    cmds, envs = self_launch_argv(str(bad), [], 2)
    assert spawn(cmds, envs) == 3  # rank 1's code; rank 0 is terminated, not waited 30 s for


def test_launcher_appends_local_rank(tmp_path):
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    assert launch_main(["--num_gpus", "2", str(probe), str(tmp_path)]) == 0
    for r in range(2):
        rec = json.loads((tmp_path / f"r{r}.json").read_text())
        assert rec["argv"] == [f"--local_rank={r}"]


def test_bench_self_launches_without_world_size(tmp_path):
    """bench.py --gpus 2 with no WORLD_SIZE spawns 2 ranks of itself; each
    child sees WORLD_SIZE=2 and (no GPU here) exits non-zero at the device
    check -- proving the children ran as ranks, not as another launcher."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["KCA_BENCH_DRYRUN"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert '"world_size": 2' in out, out[-2000:]
    assert out.count("[bench] dryrun rank") == 2, out[-2000:]


def test_rank_env_base():
    e = rank_env(1, 2, "127.0.0.1", 1234, base={"FOO": "1"})
    assert e == {"FOO": "1", "RANK": "1", "LOCAL_RANK": "1", "WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2",
                 "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1234", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
