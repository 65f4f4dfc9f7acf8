"""In-process topic bus with rospy-like semantics (no ROS master needed).

* ``Subscriber`` gets its own dispatch thread and a bounded queue; when the
  queue is full the OLDEST message is dropped (rospy ``queue_size``
  behaviour — latest-wins back-pressure).
* Callbacks of one subscriber are serialised (one thread), as in rospy —
  the reference relies on this for its mutable per-channel request
  (``communicator/ros_inference.py:138-147``).
* ``Publisher.publish`` fans out to every subscriber of the topic.
"""
from __future__ import annotations

import collections
import threading
from typing import Callable, Dict, List, Optional


class _SubQueue:
    def __init__(self, callback: Callable, queue_size: Optional[int]):
        self.callback = callback
        self.maxlen = queue_size if queue_size and queue_size > 0 else None
        self.q = collections.deque()
        self.cv = threading.Condition()
        self.dropped = 0
        self.delivered = 0
        self.closed = False
        self.errors: List[BaseException] = []
        self.idle = threading.Event()
        self.idle.set()
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def put(self, msg):
        with self.cv:
            if self.maxlen is not None and len(self.q) >= self.maxlen:
                self.q.popleft()
                self.dropped += 1
            self.q.append(msg)
            self.idle.clear()
            self.cv.notify()

    def _run(self):
        while True:
            with self.cv:
                while not self.q and not self.closed:
                    self.idle.set()
                    self.cv.wait()
                if self.closed and not self.q:
                    self.idle.set()
                    return
                msg = self.q.popleft()
            try:
                self.callback(msg)
            except BaseException as e:  # keep the bus alive; surface in tests
                self.errors.append(e)
            self.delivered += 1

    def close(self):
        with self.cv:
            self.closed = True
            self.cv.notify()
        self.t.join(timeout=5)


class TopicBus:
    def __init__(self):
        self._subs: Dict[str, List[_SubQueue]] = collections.defaultdict(list)
        self._lock = threading.Lock()
        self.shutdown_event = threading.Event()
        self.published: Dict[str, int] = collections.defaultdict(int)

    def subscribe(self, topic: str, callback: Callable, queue_size: Optional[int] = None) -> _SubQueue:
        sq = _SubQueue(callback, queue_size)
        with self._lock:
            self._subs[topic].append(sq)
        return sq

    def unsubscribe(self, topic: str, sq: _SubQueue) -> None:
        with self._lock:
            if sq in self._subs.get(topic, []):
                self._subs[topic].remove(sq)
        sq.close()

    def publish(self, topic: str, msg) -> None:
        with self._lock:
            subs = list(self._subs.get(topic, []))
            self.published[topic] += 1
        for s in subs:
            s.put(msg)

    def num_subscribers(self, topic: str) -> int:
        with self._lock:
            return len(self._subs.get(topic, []))

    def wait_idle(self, timeout: float = 30.0) -> bool:
        """Block until every subscriber queue is drained."""
        with self._lock:
            subs = [s for lst in self._subs.values() for s in lst]
        return all(s.idle.wait(timeout) for s in subs)

    def close(self) -> None:
        with self._lock:
            subs = [s for lst in self._subs.values() for s in lst]
            self._subs.clear()
        for s in subs:
            s.close()
        self.shutdown_event.set()


_DEFAULT = TopicBus()


def default_bus() -> TopicBus:
    return _DEFAULT


def reset_default_bus() -> TopicBus:
    global _DEFAULT
    _DEFAULT.close()
    _DEFAULT = TopicBus()
    return _DEFAULT
