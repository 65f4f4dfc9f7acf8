"""Live micro-batching (inference/batching.py) and the batched live drivers:
latest-wins window, one engine call per micro-batch, and a re-published
stream whose header.seq is strictly increasing under out-of-order batch
completion — in-process and with the engine sharded over 2 gloo ranks."""
import os
import random
import threading
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from triton_client_amd.inference.batching import LatestWinsWindow, MicroBatchRunner, OrderedRepublisher
from triton_client_amd.ros import msgs
from triton_client_amd.ros.bus import TopicBus


class _M:
    def __init__(self, seq):
        self.header = msgs.Header(seq=seq)


def test_window_drops_oldest():
    w = LatestWinsWindow(3)
    for i in range(5):
        w.put(i)
    assert w.dropped == 2 and w.take_locked(10) == [2, 3, 4]


def test_republisher_orders_tickets_and_drops_stale():
    out = []
    r = OrderedRepublisher(out.append)
    r.submit(1, [(3, "c"), (4, "d")])
    assert out == []
    r.submit(0, [(1, "a"), (2, "b")])
    assert out == ["a", "b", "c", "d"]
    r.submit(2, [(4, "dup"), (5, "e")])  # seq 4 already published
    assert out[-1] == "e" and r.stale == 1


def test_runner_out_of_order_completion_is_published_in_order():
    rnd = random.Random(0)
    published, sizes = [], []
    lock = threading.Lock()

    def process(ms):
        with lock:
            sizes.append(len(ms))
        time.sleep(rnd.uniform(0, 0.02))  # batches finish out of order across the 4 workers
        return [m.header.seq for m in ms]

    run = MicroBatchRunner(process, published.append, batch=4, capacity=1000, workers=4)
    for s in range(200):
        run.push(_M(s))
        if s % 7 == 0:
            time.sleep(0.002)
    run.close(drain=True)
    assert published == sorted(published) and len(set(published)) == len(published)
    assert published == list(range(200))  # nothing dropped with a large window
    assert max(sizes) > 1 and not run.errors


class _FakeEngine:
    names = ["a", "b"]

    def __init__(self):
        self.calls = []

    def detect(self, frames):
        self.calls.append(len(frames))
        time.sleep(0.005)
        return [np.array([[1, 2, 10, 20, float(f[0, 0, 0]) / 255, 1]], np.float32) for f in frames]


def _frame_msg(seq):
    from triton_client_amd.ros import compat
    img = np.full((16, 16, 3), seq % 256, np.uint8)
    return compat.numpy_to_imgmsg(img, "rgb8", header=msgs.Header(seq=seq, frame_id="cam"))


def _run_driver(engine, n=60, batch=4, workers=2):
    from triton_client_amd.inference import RosInference

    bus = TopicBus()
    params = {"sub_topic": "/cam", "pub_topic": "/det"}
    got = []
    bus.subscribe("/det/detections", lambda m: got.append((m.header.seq, [d.results[0].score for d in m.detections])))
    drv = RosInference(engine=engine, params=params, bus=bus, draw=False, batch=batch, workers=workers)
    drv.start_inference(spin=False)
    for s in range(n):
        bus.publish("/cam", _frame_msg(s))
    bus.wait_idle(30)
    drv.stop(drain=True)
    bus.wait_idle(30)
    bus.close()
    return got


def test_batched_live_driver_in_process():
    eng = _FakeEngine()
    got = _run_driver(eng, n=60, batch=4, workers=2)
    seqs = [s for s, _ in got]
    assert seqs == sorted(seqs) and len(seqs) >= 8  # latest-wins may drop, never reorders
    for s, scores in got:
        assert scores == pytest.approx([(s % 256) / 255], abs=1e-6)  # each result belongs to its frame
    assert max(eng.calls) > 1  # micro-batched engine calls


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=True)
    try:
        from triton_client_amd.parallel.dp import DataParallelDetector2D, init_distributed

        class SlowOnRank1(_FakeEngine):
            def detect(self, frames):
                if rank == 1:
                    time.sleep(0.03)  # the peer shard completes after rank 0's own shard
                return super().detect(frames)

        info = init_distributed("gloo")
        dp = DataParallelDetector2D(SlowOnRank1(), info, max_det=4)
        if info.is_main:
            got = _run_driver(dp, n=80, batch=6, workers=3)
            dp.close()
            seqs = [s for s, _ in got]
            assert seqs == sorted(seqs) and len(set(seqs)) == len(seqs) and len(seqs) >= 10, seqs
            for s, scores in got:
                assert scores == pytest.approx([(s % 256) / 255], abs=1e-6)
            q.put((0, "ok"))
        else:
            dp.serve()
            q.put((rank, "ok"))
        q.close()
        q.join_thread()
        os._exit(0)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


def test_batched_live_driver_data_parallel_gloo():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert res == {0: "ok", 1: "ok"}, res
