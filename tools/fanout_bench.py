"""How many GPUs can rank 0 feed through the shared host ring?

In the data-parallel live drivers (``parallel/ring_dp.py``) rank 0 copies every
payload of a node step into the ring slot itself (``tca_host_gather_copy`` on
C++ threads, ``_write_step``).  At the one-GPU rate of the headline (32 camera
frames + 32 LiDAR sweeps per ~7.3 ms step) a node of G GPUs needs
G x 32 x (2.76 MB raw 1280x720 frame + 1.92 MB 120k-point cloud) per step.
This measures the copy rate into a ring data area (a /dev/shm mapping, as in
production) for 32 x 2.76 MB frames and 32 x 1.92 MB clouds at several thread
counts, and from it the largest G whose copy still fits in one step.

    python tools/fanout_bench.py --threads 4,8,16,32 --json out.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FRAME = 720 * 1280 * 3      # raw rgb8 frame
CLOUD = 64 * 1875 * 16      # 120k points x 16 B (x, y, z, intensity)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--threads", default="4,8,16,32")
    ap.add_argument("--items", type=int, default=32, help="frames and clouds per GPU per step")
    ap.add_argument("--step-ms", type=float, default=7.3, help="one-GPU step time to feed")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--gpus", type=int, default=8, help="node size for the feed estimate")
    ap.add_argument("--frame-bytes", type=int, default=FRAME,
                    help="camera payload bytes (default a raw rgb8 1280x720 frame; a JPEG CompressedImage, the "
                         "reference's camera topic, is ~220 KB at quality 90)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--bag", action="store_true",
                    help="also measure replaying a ROS bag (in /dev/shm) of one GPU-step of frames + clouds: "
                         "messages read into bytes vs uncompressed chunks read straight into the ingest arena")
    ap.add_argument("--deserialize", action="store_true",
                    help="also measure deserialising the node batch's wire messages into bytes (the copy path: the "
                         "ring copy comes on top) vs into the ring's ingest arena (the only copy)")
    a = ap.parse_args(argv)

    from triton_client_amd.inference.live import gather_copy
    from triton_client_amd.parallel.host_ring import HostRing

    rng = np.random.default_rng(0)
    n = a.items
    # sources: bytes objects, like deserialised ROS message payloads
    srcs = [rng.integers(0, 255, a.frame_bytes, np.uint8).tobytes() for _ in range(n)] + \
        [rng.integers(0, 255, CLOUD, np.uint8).tobytes() for _ in range(n)]
    sizes = [len(s) for s in srcs]
    total = sum(sizes)
    ring = HostRing(f"tca_fanout_{os.getpid()}", nslots=1, world=1, create=True, pin=False)
    try:
        data = ring.new_generation(total + 4096 * len(srcs))
        offs, o = [], 0
        for z in sizes:
            offs.append(o)
            o += (z + 4095) // 4096 * 4096
        dst = [data.base + x for x in offs]
        rows = []
        for t in [int(v) for v in a.threads.split(",")]:
            for _ in range(3):  # first touch of the mapping, thread pool warm-up
                gather_copy(dst, srcs, sizes, t)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                gather_copy(dst, srcs, sizes, t)
                ts.append(time.perf_counter() - t0)
            med = float(np.median(ts))
            gbs = total / med / 1e9
            feed = (a.step_ms / 1e3) / med  # GPUs whose per-step payload rank 0 copies within one step
            rows.append({"threads": t, "bytes_per_gpu_step": total, "median_ms": med * 1e3,
                         "min_ms": min(ts) * 1e3, "GBps": gbs, "gpus_fed_at_1gpu_rate": feed})
            print(f"threads {t:3d}: {med * 1e3:7.2f} ms per GPU-step of {total / 1e6:.1f} MB = {gbs:6.1f} GB/s "
                  f"-> rank 0 feeds {feed:4.1f} GPUs at {a.step_ms} ms/step", flush=True)
        best = max(rows, key=lambda r: r["GBps"])
        deser = _deserialize_rows(a, srcs, total) if a.deserialize else None
        bag = _bag_rows(a, srcs, total) if a.bag else None
        out = {"tool": "tools/fanout_bench.py", "items_per_gpu": n, "frame_bytes": a.frame_bytes, "cloud_bytes": CLOUD,
               "step_ms": a.step_ms, "cpus_allowed": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
               "rows": rows, "best": best, "node_gpus": a.gpus,
               "node_step_copy_ms_at_best": best["median_ms"] * a.gpus,
               "feeds_node": best["gpus_fed_at_1gpu_rate"] >= a.gpus, "deserialize": deser, "bag": bag}
        print(json.dumps({"best_GBps": best["GBps"], "gpus_fed": best["gpus_fed_at_1gpu_rate"],
                          "cpus_allowed": out["cpus_allowed"]}))
        if a.json:
            with open(a.json, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        ring.close()
    return 0


def _deserialize_rows(a, srcs, total):
    """Rank 0's ingest with the arena: each wire message (a serialised Image / PointCloud2)
    deserialised once, its payload written into the arena (``rosmsg.deserialize(.., alloc)``,
    numpy copies outside the GIL), and nothing copied by the ring step -- against
    deserialising into ``bytes`` (the copy path, before its ring copy)."""
    from concurrent.futures import ThreadPoolExecutor

    from triton_client_amd.parallel.host_ring import IngestArena
    from triton_client_amd.ros import msgs, rosmsg

    n = a.items
    wire = []
    for i, s in enumerate(srcs):
        if i < n:
            m = msgs.Image(height=1, width=len(s) // 3, encoding="rgb8", step=len(s), data=s)
            wire.append((rosmsg.serialize(m), "sensor_msgs/Image"))
        else:
            m = msgs.PointCloud2(height=1, width=len(s) // 16, point_step=16, row_step=len(s), data=s)
            wire.append((rosmsg.serialize(m), "sensor_msgs/PointCloud2"))
    arena = IngestArena(f"/dev/shm/tca_fanout_in_{os.getpid()}", 3 * (total + 256 * len(srcs)), True, pin=False)
    rows = []
    by_type = {}
    for w, typ in wire:
        by_type.setdefault(typ, []).append(w)
    try:
        for t in [int(v) for v in a.threads.split(",")]:
            with ThreadPoolExecutor(t) as pool:
                # bytes / arena: one deserialize() per message on a pool of t threads (the native parse
                # for these types); arena_py: the same with the per-field Python reader (round 5's path);
                # arena_batch: one deserialize_many() per message type, its payload copy on t threads
                for mode in ("bytes", "arena", "arena_py", "arena_batch"):
                    alloc = arena.alloc if mode != "bytes" else None
                    fn = rosmsg.deserialize_py if mode == "arena_py" else rosmsg.deserialize

                    def one(w, alloc=alloc, fn=fn):
                        return fn(w[0], w[1], alloc)
                    ts = []
                    for r in range(a.reps + 3):
                        t0 = time.perf_counter()
                        if mode == "arena_batch":
                            out = [m for typ, ws in by_type.items()
                                   for m in rosmsg.deserialize_many(ws, typ, alloc=alloc, threads=t)]
                        else:
                            out = list(pool.map(one, wire))
                        dt = time.perf_counter() - t0
                        if mode == "arena":
                            assert all(isinstance(m.data, memoryview) for m in out)
                        del out
                        if r >= 3:
                            ts.append(dt)
                    med = float(np.median(ts))
                    rows.append({"threads": t, "mode": mode, "median_ms": med * 1e3, "GBps": total / med / 1e9,
                                 "gpus_fed_at_1gpu_rate": (a.step_ms / 1e3) / med})
                    print(f"deserialise into {mode:11s}, {t:3d} threads: {med * 1e3:7.2f} ms per GPU-step = "
                          f"{total / med / 1e9:6.1f} GB/s", flush=True)
    finally:
        arena.close(unlink=True)
    return rows


def _bag_rows(a, srcs, total):
    """Bag replay on rank 0 (``Bag.read_messages``): one GPU-step of messages (a.items raw
    frames + a.items clouds) from a ROS bag v2 in /dev/shm, into bytes vs with ``alloc`` = the
    ingest arena (uncompressed chunks ``readinto`` the arena, payloads views of them), and with
    4 / 8 / 16 threads reading chunks ahead (``readers``)."""
    from triton_client_amd.parallel.host_ring import IngestArena
    from triton_client_amd.ros import msgs
    from triton_client_amd.ros.bag import Bag, RosBag

    n = a.items
    path = f"/dev/shm/tca_fanout_{os.getpid()}.bag"
    w = RosBag(path, "w")
    for i, s in enumerate(srcs):
        if i < n:
            w.write("/cam", msgs.Image(header=msgs.Header(seq=i), height=1, width=len(s) // 3, encoding="rgb8",
                                       step=len(s), data=s))
        else:
            w.write("/pc", msgs.PointCloud2(header=msgs.Header(seq=i), height=1, width=len(s) // 16, point_step=16,
                                            row_step=len(s), data=s))
    w.close()
    arena = IngestArena(f"/dev/shm/tca_fanout_bag_{os.getpid()}", 2 * (total + (64 << 20)), True, pin=False)
    rows = []
    try:
        for mode in ("bytes", "arena", "arena_r4", "arena_r8", "arena_r16"):
            readers = int(mode.split("_r")[1]) if "_r" in mode else 0
            ts = []
            for r in range(a.reps + 2):
                t0 = time.perf_counter()
                with Bag(path) as b:
                    out = [m for _, m, _ in b.read_messages(alloc=arena.alloc if mode != "bytes" else None,
                                                            readers=readers)]
                dt = time.perf_counter() - t0
                assert len(out) == 2 * n
                del out
                if r >= 2:
                    ts.append(dt)
            med = float(np.median(ts))
            rows.append({"mode": mode, "median_ms": med * 1e3, "GBps": total / med / 1e9, "us_per_msg": med / (2 * n) * 1e6,
                         "gpus_fed_at_1gpu_rate": (a.step_ms / 1e3) / med})
            print(f"bag replay into {mode:9s}: {med * 1e3:7.2f} ms per GPU-step = {total / med / 1e9:6.1f} GB/s, "
                  f"{med / (2 * n) * 1e6:.0f} us per message", flush=True)
        rows.append(_sharded_row(a, path, total, n))
    finally:
        arena.close(unlink=True)
        os.unlink(path)
    return rows


def _sharded_row(a, path, total, n):
    """Sharded replay (``Bag.read_messages(mapped=True)`` + ``ring_dp`` file-sourced items):
    rank 0's part per GPU-step is reading the record headers and message prefixes of the mapped
    bag, building the messages and locating each payload in the file (``FileMaps.locate``, what
    ``_write_step`` does per item) -- no payload byte.  Each rank's part is gathering its own
    shard's payloads from its own mapping into its pinned staging (``gather_copy``, as the live
    engines do), on its own cores.  GPUs fed = step time / rank 0's time per GPU-step; the
    per-rank read must fit in one step on that rank's cores."""
    from triton_client_amd.inference.live import gather_copy
    from triton_client_amd.parallel.host_ring import FileMaps
    from triton_client_amd.ros.bag import Bag

    ts = []
    for r in range(a.reps + 2):
        t0 = time.perf_counter()
        with Bag(path) as b:
            ms = [m for _, m, _ in b.read_messages(mapped=True)]
            locs = [FileMaps.locate(memoryview(m.data), len(m.data)) for m in ms]
        dt = time.perf_counter() - t0
        assert len(ms) == 2 * n and all(x is not None for x in locs)
        if r >= 2:
            ts.append(dt)
        del ms, locs
    med = float(np.median(ts))
    # one rank's shard read: its GPU-step of payloads from the file into pinned staging
    view = FileMaps.view(path)
    with Bag(path) as b:
        ms = [m for _, m, _ in b.read_messages(mapped=True)]
        sizes = [len(m.data) for m in ms]
        offs = [FileMaps.locate(memoryview(m.data), len(m.data))[1] for m in ms]
    del ms
    try:
        import torch
        pinned = torch.cuda.is_available()
        dst = torch.empty(sum(sizes) + 4096 * len(sizes), dtype=torch.uint8, pin_memory=pinned)
        base = dst.data_ptr()
    except Exception:  # noqa: BLE001
        pinned = False
        dst = np.empty(sum(sizes) + 4096 * len(sizes), np.uint8)
        base = dst.ctypes.data
    dptr, o = [], 0
    for z in sizes:
        dptr.append(base + o)
        o += (z + 4095) // 4096 * 4096
    rt = {}
    for th in (4, 8, 16):
        tt = []
        for r in range(a.reps + 2):
            t0 = time.perf_counter()
            gather_copy(dptr, [view[x:x + z] for x, z in zip(offs, sizes)], sizes, th)
            if r >= 2:
                tt.append(time.perf_counter() - t0)
        rt[th] = float(np.median(tt))
    best_th = min(rt, key=rt.get)
    row = {"mode": "sharded", "rank0_ms_per_gpu_step": med * 1e3, "us_per_msg_rank0": med / (2 * n) * 1e6,
           "gpus_fed_by_rank0": (a.step_ms / 1e3) / med,
           "rank_shard_read_ms": {str(k): v * 1e3 for k, v in rt.items()},
           "rank_shard_read_GBps": total / rt[best_th] / 1e9, "rank_read_fits_step": rt[best_th] * 1e3 <= a.step_ms,
           "pinned_staging": pinned, "median_ms": med * 1e3, "GBps": None,
           "gpus_fed_at_1gpu_rate": (a.step_ms / 1e3) / med}
    print(f"sharded replay: rank 0 {med * 1e3:7.2f} ms per GPU-step ({med / (2 * n) * 1e6:.1f} us per message) -> "
          f"feeds {row['gpus_fed_by_rank0']:.1f} GPUs; one rank's shard read {rt[best_th] * 1e3:.2f} ms "
          f"({total / rt[best_th] / 1e9:.1f} GB/s, {best_th} threads)", flush=True)
    return row


if __name__ == "__main__":
    sys.exit(main())
