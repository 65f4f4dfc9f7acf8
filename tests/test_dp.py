"""Data parallelism on the CPU: gloo, world_size 2 and 3, 127.0.0.1 rendezvous.

The same code paths run over RCCL on GPUs (FrameExchange's grouped p2p,
parameter broadcast, the DP detectors used by the bag drivers)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeDetector:
    """Deterministic, rank-independent: one box per frame from its pixel stats."""
    names = ["x"]

    def detect(self, frames):
        out = []
        for f in frames:
            m = float(f.mean())
            k = int(f[0, 0, 0]) % 4
            out.append(np.array([[m, m, m + 10, m + 10, 0.5, j] for j in range(k)], np.float32).reshape(-1, 6))
        return out


class FakeDetector3D:
    names = ["a"]

    def detect(self, clouds):
        from triton_client_amd.ros.compat import cloud_to_numpy
        out = []
        for c in clouds:
            p = cloud_to_numpy(c)
            k = len(p) % 5
            out.append({"pred_boxes": np.tile(p[:1, [0, 1, 2, 3, 0, 1, 2]], (k, 1)).astype(np.float32),
                        "pred_scores": np.full(k, p[:, 3].mean(), np.float32),
                        "pred_labels": np.arange(k, dtype=np.int64)})
        return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(int(os.environ.get("TCA_DP_TEST_DUMP", "150")), exit=True)
    try:
        from triton_client_amd.models.common import broadcast_parameters
        from triton_client_amd.parallel.dp import (DataParallelDetector2D, DataParallelDetector3D, FrameExchange,
                                                   allreduce_max, barrier, init_distributed, shutdown)
        from triton_client_amd.ros import compat, msgs

        info = init_distributed("gloo")
        assert dist.get_backend() == "gloo"
        # scatter / gather of tensor sets
        ex = FrameExchange(info)
        src = [[torch.full((3, 4), float(r)), torch.arange(5) + r] for r in range(world)] if info.is_main else None
        dst = [torch.empty(3, 4), torch.empty(5, dtype=torch.int64)]
        ex.scatter(src, dst)
        assert torch.equal(dst[0], torch.full((3, 4), float(rank))) and torch.equal(dst[1], torch.arange(5) + rank)
        g = [[torch.empty(2), torch.empty(1, dtype=torch.int32)] for _ in range(world)] if info.is_main else None
        ex.gather([torch.full((2,), 10.0 * rank), torch.tensor([rank], dtype=torch.int32)], g)
        if info.is_main:
            for r in range(world):
                assert torch.equal(g[r][0], torch.full((2,), 10.0 * r)) and int(g[r][1]) == r
        # parameter broadcast
        lin = torch.nn.Linear(4, 3)
        torch.nn.init.constant_(lin.weight, float(rank))
        broadcast_parameters(lin)
        assert float(lin.weight.detach().abs().sum()) == 0.0
        assert allreduce_max(info, float(rank)) == world - 1
        # DP 2D detector: rank 0 drives, others serve
        frames = [np.full((8, 12, 3), 7 * i, np.uint8) for i in range(7)]
        dp = DataParallelDetector2D(FakeDetector(), info, max_det=8)
        clouds = [compat.create_cloud_xyzi(np.random.default_rng(i).random((20 + 3 * i, 4)).astype(np.float32),
                                           msgs.Header(seq=i)) for i in range(5)]
        dp3 = DataParallelDetector3D(FakeDetector3D(), info, max_out=8)
        if info.is_main:
            got = dp.detect(frames)
            want = FakeDetector().detect(frames)
            assert len(got) == len(want)
            for a, b in zip(got, want):
                np.testing.assert_array_equal(a, b)
            mixed = dp.detect([frames[1], np.full((4, 4, 3), 9, np.uint8)])
            np.testing.assert_array_equal(mixed[1], FakeDetector().detect([np.full((4, 4, 3), 9, np.uint8)])[0])
            dp.close()
            got3 = dp3.detect(clouds)
            want3 = FakeDetector3D().detect(clouds)
            for a, b in zip(got3, want3):
                for k in a:
                    np.testing.assert_allclose(a[k], b[k], rtol=1e-6)
            dp3.close()
        else:
            # the 7-frame batch; the mixed batch's single-frame steps run on rank 0 alone
            assert dp.serve() == 1
            assert dp3.serve() == 1
        barrier(info)
        shutdown(info)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_dp_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def _fault_worker(rank, world, port, q):
    """Rank 2 serves one batch, then its process dies without any cleanup; rank
    0's HealthMonitor notices the stalled heartbeat and the next batches are
    re-sharded over ranks {0, 1} with unchanged results."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    import time
    faulthandler.dump_traceback_later(150, exit=True)
    try:
        from triton_client_amd.parallel.dp import DataParallelDetector2D, HealthMonitor, init_distributed

        info = init_distributed("gloo")
        # a 2 s heartbeat timeout: a loaded CI host can hold a healthy rank's 0.1 s beat past 1 s
        mon = HealthMonitor(info, interval=0.1, timeout=2.0)
        dp = DataParallelDetector2D(FakeDetector(), info, max_det=8, monitor=mon)
        frames = [np.full((8, 12, 3), 7 * i, np.uint8) for i in range(9)]
        want = FakeDetector().detect(frames)
        if info.is_main:
            got = dp.detect(frames)
            assert all(np.array_equal(a, b) for a, b in zip(got, want))
            assert mon.alive() == [0, 1, 2]
            q.put((2, "wait"))  # let rank 2 die before the next batch
            time.sleep(4.5)
            for _ in range(2):
                got = dp.detect(frames)
                assert all(np.array_equal(a, b) for a, b in zip(got, want))
            assert mon.alive() == [0, 1] and mon.dead == {2}
            dp.close()
            q.put((0, "ok"))
        elif rank == 1:
            assert dp.serve() == 3
            q.put((1, "ok"))
        else:
            assert dp.serve(max_steps=1) == 1
            mon.stop()
            os._exit(0)  # simulated crash: no close, no heartbeat, sockets drop
        mon.stop()
        q.close()
        q.join_thread()  # flush the result before the hard exit
        os._exit(0)
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


def test_dp_rank_failure_resharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fault_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert res == {0: "ok", 1: "ok", 2: "wait"}, res


class _DiesMidStep(FakeDetector):
    """Rank 2's engine: the process dies inside its second shard, i.e. after
    the step's scatter and before its gather (the case a header-less protocol
    would answer with a stale payload on retry)."""

    def __init__(self):
        self.calls = 0

    def detect(self, frames):
        self.calls += 1
        if self.calls == 2:
            os._exit(0)
        return super().detect(frames)


def _midstep_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=True)
    try:
        from triton_client_amd.parallel.dp import DataParallelDetector2D, HealthMonitor, init_distributed

        info = init_distributed("gloo")
        mon = HealthMonitor(info, interval=0.1, timeout=1.0)
        local = _DiesMidStep() if rank == 2 else FakeDetector()
        dp = DataParallelDetector2D(local, info, max_det=8, monitor=mon)
        if info.is_main:
            for b in range(3):
                frames = [np.full((8, 12, 3), 5 * i + 40 * b, np.uint8) for i in range(9)]
                want = FakeDetector().detect(frames)
                got = dp.detect(frames)
                assert len(got) == len(want)
                for a, w in zip(got, want):
                    assert np.array_equal(a, w), (b, a, w)
            assert dp.retries == 1 and mon.dead == {2}, (dp.retries, mon.dead)
            dp.close()
            q.put((0, "ok"))
        else:
            n = dp.serve()
            q.put((rank, f"served {n}"))
        mon.stop()
        q.close()
        q.join_thread()
        os._exit(0)
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


def test_dp_rank_dies_between_scatter_and_gather():
    """rank 0 drains every op of the failed step, the survivor's payload is
    consumed in that step (so the retry cannot read it), the retry runs with a
    new sequence number over the survivors and every batch's results are exact."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_midstep_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    # rank 1: batch 0, the failed batch 1, its retry, batch 2
    assert res == {0: "ok", 1: "served 4"}, res
