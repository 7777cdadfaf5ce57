"""Debug: the TP=2 engine worker of tests/test_tp_engine_gpu.py with stack dumps
on a hang and progress lines (run on the GPU box)."""
import faulthandler
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_tp_engine_gpu import PROMPTS, _model, _port  # noqa: E402


def w(rank, port):
    faulthandler.dump_traceback_later(40, exit=True)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    from kubernetes_cloud_amd.engine.llm_engine import LLMEngine, SamplingParams
    from kubernetes_cloud_amd.engine.runner import ModelRunner
    from kubernetes_cloud_amd.engine.tp_driver import CollectiveRunner, follower_loop
    from kubernetes_cloud_amd.parallel import custom_ar
    from kubernetes_cloud_amd.parallel.tensor_parallel import shard_model_from_full
    full = _model("bloom-560m")
    group = dist.new_group(backend="gloo")
    ar = custom_ar.register(group, max_bytes=4 << 20)
    tp = shard_model_from_full(full, rank, 2, group)
    ctrl = dist.new_group(backend="gloo")
    runner = ModelRunner(tp, max_slots=8, max_len=128, use_graphs=False, page_size=16)
    print(f"[{rank}] ready {time.time():.1f}", flush=True)
    if rank == 0:
        eng = LLMEngine(tp, runner=CollectiveRunner(runner, ctrl))
        sp = SamplingParams(max_new_tokens=12, do_sample=False)
        r = eng.generate(PROMPTS, sp)
        print("[0] gen", [x.output for x in r], flush=True)
        eng.runner.shutdown()
    else:
        follower_loop(runner, ctrl)
    dist.barrier()
    print(f"[{rank}] done calls={ar.calls}", flush=True)
    faulthandler.cancel_dump_traceback_later()
    dist.destroy_process_group()


if __name__ == "__main__":
    port = _port()
    mp.spawn(w, args=(port,), nprocs=2)
