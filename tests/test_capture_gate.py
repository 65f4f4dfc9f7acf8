"""CaptureGate (pipelines/graph.py): submissions share the gate, a capture window
is exclusive, writers are not starved, and a first-use capture inside a submission
(shared -> exclusive on one thread) does not deadlock."""
import threading
import time

import pytest

from triton_client_amd.pipelines.graph import CaptureGate


def test_shared_holders_run_together():
    g = CaptureGate()
    inside, peak, lock = [0], [0], threading.Lock()

    def sub():
        with g.shared():
            with lock:
                inside[0] += 1
                peak[0] = max(peak[0], inside[0])
            time.sleep(0.05)
            with lock:
                inside[0] -= 1
    ts = [threading.Thread(target=sub) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(5)
    assert peak[0] >= 2  # submissions of different engines do not serialise


def test_exclusive_excludes_shared_and_is_not_starved():
    g = CaptureGate()
    log, stop = [], threading.Event()

    def streamer():
        while not stop.is_set():
            with g.shared():
                log.append(("s", time.monotonic()))
                time.sleep(0.002)

    ts = [threading.Thread(target=streamer) for _ in range(3)]
    for t in ts:
        t.start()
    time.sleep(0.02)
    t0 = time.monotonic()
    with g.exclusive():
        win = (time.monotonic(), None)
        n_before = len(log)
        time.sleep(0.05)
        assert len(log) == n_before  # nobody submits inside the capture window
        win = (win[0], time.monotonic())
    waited = win[0] - t0
    time.sleep(0.02)
    stop.set()
    for t in ts:
        t.join(5)
    assert waited < 1.0  # writer preference: the capture got in despite continuous submissions
    assert any(ts_ > win[1] for k, ts_ in log)  # streaming resumed after the window


def test_reentrant_and_upgrade_inside_shared():
    g = CaptureGate()
    done = []

    def worker():
        with g.shared():
            with g.shared():
                with g.exclusive():  # first-use capture inside a submission
                    with g.shared():
                        with g.exclusive():
                            done.append(1)
    t = threading.Thread(target=worker)
    t.start()
    t.join(5)
    assert done == [1] and not t.is_alive()
    with g.exclusive():  # the gate is free again
        pass
    assert g._readers == 0 and g._writer is None


@pytest.mark.gpu
def test_two_threads_submit_to_executor_with_lazy_capture(cuda):
    """Both sets' graphs dropped, so the first submissions capture inside ``submit``
    (shared -> exclusive while holding the executor lock) while a second thread submits
    to the same executor: with the lock taken before the gate, neither blocks forever."""
    import torch

    from triton_client_amd.pipelines.stream import StreamExecutor

    class Owner:
        x = torch.zeros(1024, device=cuda)

    own = Owner()
    ex = StreamExecutor(lambda: own.x * 2 + 1, [(own, "x")], cuda)
    for r in ex.runners:
        r.graph = None  # the next call of each set re-captures inside submit
    host = [torch.full((1024,), float(i), pin_memory=True) for i in range(4)]
    got, errs = {}, []

    def worker(i):
        try:
            t = ex.submit(lambda k, i=i: [(ex.inputs[k][0], host[i])]).wait()
            got[i] = float(t.host[0][0])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts), "submission deadlocked"
    assert not errs and got == {i: 2.0 * i + 1 for i in range(4)}
