"""Thread-safety of the in-process topic bus (the reference relies on
rospy's one-thread-per-subscriber serialisation, ros_inference.py:138-147, and has
a two-subscriber evaluator, evaluate_inference.py:114-118).  Concurrent
publishers, serialised callbacks, latest-wins queues, and churn of subscribers
while publishing."""
import threading
import time

from triton_client_amd.ros import TopicBus


def test_concurrent_publishers_reach_every_subscriber_in_order():
    bus = TopicBus()
    P, N = 8, 500
    got = [[], []]
    inside = [0, 0]
    overlap = []

    def make_cb(k):
        def cb(msg):
            inside[k] += 1
            if inside[k] != 1:  # a second callback of this subscriber is running
                overlap.append(msg)
            got[k].append(msg)
            inside[k] -= 1
        return cb

    for k in range(2):
        bus.subscribe("/t", make_cb(k))

    def pub(p):
        for i in range(N):
            bus.publish("/t", (p, i))

    ts = [threading.Thread(target=pub, args=(p,)) for p in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert bus.wait_idle(30)
    bus.close()
    assert not overlap
    assert bus.published["/t"] == P * N
    for k in range(2):
        assert len(got[k]) == P * N
        for p in range(P):  # each publisher's messages arrive in its publish order
            assert [i for q, i in got[k] if q == p] == list(range(N))


def test_bounded_queue_drops_oldest_and_keeps_latest():
    bus = TopicBus()
    seen = []
    gate = threading.Event()

    def slow(msg):
        gate.wait(5)
        seen.append(msg)

    sq = bus.subscribe("/cam", slow, queue_size=1)
    for i in range(200):
        bus.publish("/cam", i)
    gate.set()
    assert bus.wait_idle(30)
    bus.close()
    assert sq.dropped + sq.delivered == 200
    assert seen[-1] == 199 and sq.dropped >= 190  # latest wins under back-pressure


def test_subscriber_churn_while_publishing():
    bus = TopicBus()
    stop = threading.Event()
    errors = []
    counts = []

    def publisher():
        i = 0
        while not stop.is_set():
            try:
                bus.publish("/x", i)
            except Exception as e:  # pragma: no cover
                errors.append(e)
            i += 1

    def churn():
        for _ in range(50):
            box = []
            sq = bus.subscribe("/x", box.append, queue_size=4)
            time.sleep(0.001)
            bus.unsubscribe("/x", sq)
            counts.append(sq.delivered)

    tp = threading.Thread(target=publisher)
    tp.start()
    tc = [threading.Thread(target=churn) for _ in range(4)]
    for t in tc:
        t.start()
    for t in tc:
        t.join()
    stop.set()
    tp.join()
    bus.close()
    assert not errors and len(counts) == 200
    assert bus.num_subscribers("/x") == 0
