"""Native shared-memory control channel (csrc/runtime/ctrl_channel.cpp,
engine/ctrl_channel.py): one writer, several reader processes; messages
larger than the ring (fragments streamed through 4 slots), back-pressure on a
slow reader, ordering, and close -> readers drain then see "closed"."""
import os
import time
import uuid

import multiprocessing as mp

import pytest


def _reader(name, idx, n, slow, q):
    from kubernetes_cloud_amd.engine.ctrl_channel import ChannelError, ShmChannel
    ch = ShmChannel(name, idx, timeout_s=60)
    got = []
    for _ in range(n):
        got.append(ch.recv())
        if slow:
            time.sleep(0.002)
    try:
        ch.recv()
        closed = False
    except ChannelError as e:
        closed = "closed" in str(e)
    ch.close()
    q.put((idx, got, closed))


def test_shm_channel_fragments_backpressure_close():
    from kubernetes_cloud_amd.engine.ctrl_channel import ShmChannel
    name = f"/kca_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    w = ShmChannel(name, -1, readers=3, slots=4, slot_bytes=4096, timeout_s=60)
    msgs = [("decode", list(range(i % 7)), i) for i in range(200)]
    msgs[50] = ("prefill", bytes(range(256)) * 200, 50)  # 51 KB: 13 fragments through a 4-slot ring
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_reader, args=(name, i, len(msgs), i == 2, q)) for i in range(3)]
    for p in ps:
        p.start()
    for m in msgs:
        w.send(m)
    time.sleep(0.5)
    w.close()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for idx, got, closed in res:
        assert got == msgs, idx
        assert closed, idx


def test_shm_channel_bad_args():
    from kubernetes_cloud_amd.engine.ctrl_channel import ChannelError, ShmChannel
    with pytest.raises(ChannelError):
        ShmChannel("/kca_missing_" + uuid.uuid4().hex[:8], 0, timeout_s=0.2)._lib  # open of a missing ring


def test_as_channel_wraps_process_groups():
    """A ProcessGroup has .send/.recv of its own: it must still be wrapped."""
    import socket as _s

    import torch.distributed as dist

    from kubernetes_cloud_amd.engine.ctrl_channel import GlooChannel
    from kubernetes_cloud_amd.engine.tp_driver import as_channel
    with _s.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        g = dist.new_group(backend="gloo")
        assert isinstance(as_channel(g), GlooChannel)
        assert isinstance(as_channel(None), GlooChannel)
        ch = GlooChannel(g)
        assert as_channel(ch) is ch
    finally:
        dist.destroy_process_group()


def _doomed_writer(name, q):
    from kubernetes_cloud_amd.engine.ctrl_channel import ShmChannel
    w = ShmChannel(name, -1, readers=1, slots=4, slot_bytes=4096)
    w.send("hello")
    q.put("sent")
    time.sleep(600)  # killed by the test without closing the channel


def test_blocking_reader_raises_when_writer_dies():
    """a blocking follower (timeout_s=None) must not spin forever when rank 0 is
    SIGKILLed / OOM-killed without closing -- recv sees the writer pid gone and raises."""
    from kubernetes_cloud_amd.engine.ctrl_channel import ChannelError, ShmChannel
    name = f"/kca_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_doomed_writer, args=(name, q))
    p.start()
    assert q.get(timeout=120) == "sent"
    r = ShmChannel(name, 0)  # blocking reader
    assert r.recv() == "hello"
    p.kill()
    p.join(timeout=30)
    t0 = time.monotonic()
    with pytest.raises(ChannelError, match="writer died"):
        r.recv()
    assert time.monotonic() - t0 < 30
    r.close()
    try:
        os.unlink("/dev/shm" + name)  # the killed writer never unlinked it
    except OSError:
        pass
