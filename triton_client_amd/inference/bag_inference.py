"""Offline bag replay (reference ``communicator/bag_inference2d.py:22-160`` and
``communicator/bag_inference3d.py:46-184``).

Reads the sensor topic from a bag and runs the same per-frame body as the
live drivers, but ``batch`` frames at a time (one local graph replay or a
window of remote RPCs per micro-batch) instead of one blocking RPC per frame.
2D: annotated PNGs to ``out_dir/NNNN.png`` and, if ``out_bag`` is given, the
input image + annotated image + Detection2DArray written to it (the
reference opened ``output.bag`` but never wrote).  3D: the input cloud and
the BoundingBoxArray are written to ``<bag>_output.bag`` like the
reference.  Bag path and output dir are arguments (fixes A14);
``start_seq`` resumes a replay.
"""
from __future__ import annotations

import os
import time
from typing import Optional

from ..ros.bag import Bag
from .ros_inference import RosInference
from .ros_inference3d import RosInference3D


def _ingest(engine):
    """The data-parallel engine's ingest arena allocator (payloads deserialised
    straight into the node's host ring), or None."""
    return getattr(engine, "ingest_buffer", None)


def _readers(engine) -> int:
    """Threads reading the bag's chunks ahead into the ingest arena (with an arena only)."""
    return 8 if getattr(engine, "ingest_buffer", None) is not None else 0


def _read_kw(engine) -> dict:
    """How the bag is read for this engine: a data-parallel engine that shards by file
    (``ring_dp.file_sharding``) gets messages whose payloads stay in the mapped bag -- rank 0
    reads record headers and message prefixes, every rank reads its own shard's payloads --
    else payloads are deserialised into the ingest arena by reader threads."""
    if getattr(engine, "file_sharding", False):
        return {"mapped": True}
    return {"alloc": _ingest(engine), "readers": _readers(engine)}


def _batches(it, n):
    buf = []
    for item in it:
        buf.append(item)
        if len(buf) == n:
            yield buf
            buf = []
    if buf:
        yield buf


class BagInference2D(RosInference):
    def __init__(self, channel=None, client=None, bagfile: str = "", out_dir: Optional[str] = "./output_data",
                 out_bag: Optional[str] = None, batch: int = 8, save_png: bool = True, start_seq: int = 0,
                 max_frames: Optional[int] = None, **kw):
        super().__init__(channel, client, **kw)
        self.bagfile, self.out_dir, self.out_bag = bagfile, out_dir, out_bag
        self.batch, self.save_png, self.start_seq, self.max_frames = batch, save_png, start_seq, max_frames
        self.results = []
        self.elapsed = 0.0

    def start_inference(self, spin: bool = False, timeout: Optional[float] = None):
        if self.save_png and self.out_dir:
            os.makedirs(self.out_dir, exist_ok=True)
        ob = Bag(self.out_bag, "w") if self.out_bag else None
        p = self.params
        count = 0
        t0 = time.perf_counter()
        with Bag(self.bagfile) as bag:
            it = (m for _, m, _ in bag.read_messages(topics=[p["sub_topic"]], start_seq=self.start_seq,
                                                     **_read_kw(self.engine)))
            for chunk in _batches(it, self.batch):
                if self.max_frames is not None:
                    chunk = chunk[: max(0, self.max_frames - count)]
                    if not chunk:
                        break
                for m, (im, det, d) in zip(chunk, self.process(chunk)):
                    if self.save_png and self.out_dir:
                        _save_png(os.path.join(self.out_dir, f"{count:04}.png"), im)
                    if ob is not None:
                        ob.write(p["sub_topic"], m)
                        ob.write(p["pub_topic"], im)
                        ob.write(p["pub_topic"] + "/detections", det)
                    self.results.append((m.header.seq, d))
                    count += 1
        self.elapsed = time.perf_counter() - t0
        if ob is not None:
            ob.close()
        return count


def _save_png(path, im) -> None:
    from PIL import Image as PILImage

    from ..ros.compat import imgmsg_to_numpy

    PILImage.fromarray(imgmsg_to_numpy(im, "rgb8")).save(path)


class BagInference3D(RosInference3D):
    def __init__(self, channel=None, client=None, bagfile: str = "", out_bag: Optional[str] = "", batch: int = 8,
                 start_seq: int = 0, max_frames: Optional[int] = None, verbose: bool = False, **kw):
        super().__init__(channel, client, **kw)
        self.bagfile, self.batch, self.start_seq, self.max_frames = bagfile, batch, start_seq, max_frames
        self.out_bag = (os.path.splitext(bagfile)[0] + "_output.bag") if out_bag == "" else out_bag
        self.verbose = verbose
        self.results = []
        self.elapsed = 0.0

    def start_inference(self, spin: bool = False, timeout: Optional[float] = None):
        p = self.params
        ob = Bag(self.out_bag, "w") if self.out_bag else None
        count = 0
        t0 = time.perf_counter()
        with Bag(self.bagfile) as bag:
            it = (m for _, m, _ in bag.read_messages(topics=[p["sub_topic"]], start_seq=self.start_seq,
                                                     **_read_kw(self.engine)))
            for chunk in _batches(it, self.batch):
                if self.max_frames is not None:
                    chunk = chunk[: max(0, self.max_frames - count)]
                    if not chunk:
                        break
                for m, (out, pred) in zip(chunk, self.process(chunk)):
                    if ob is not None:
                        ob.write(p["sub_topic"], m)
                        ob.write(p["pub_topic"], out)
                    if self.verbose:
                        print(m.header.seq)
                    self.results.append((m.header.seq, pred))
                    count += 1
        self.elapsed = time.perf_counter() - t0
        if ob is not None:
            ob.close()
        return count
