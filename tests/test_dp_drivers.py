"""The data-parallel live drivers over the node's shared host ring
(parallel/host_ring.py, parallel/ring_dp.py, csrc/runtime/host_ring.cpp):
cross-process signalling, NUMA binding, and 2-rank replays of the fixture bag
whose outputs must be bit-identical to a single rank's (CPU here; on the GPU
box the same replays run two ranks on the one card over gloo)."""
import multiprocessing as mp
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "fixtures", "ros1_sensors.bag")


def _runtime_or_skip():
    from triton_client_amd import _native
    try:
        return _native.runtime()
    except _native.NativeError:
        pytest.skip("runtime library not built")


# ------------------------------------------------------------------ host ring signalling
def _peer(name, q):
    from triton_client_amd.parallel.host_ring import HostRing

    ring = HostRing(name)
    for seq in range(1, 7):
        s = seq % ring.nslots
        assert ring.wait_ready(s, seq, 10000)
        hdr = ring.header(s)
        data = ring.use_generation(int(hdr[1]), int(hdr[2]))
        v = data.slot(s)[:8].copy()
        data.slot(s)[8:16] = v[::-1]  # an "output"
        ring.ack(s, 1, seq)
    q.put("ok")


def test_host_ring_cross_process():
    _runtime_or_skip()
    from triton_client_amd.parallel.host_ring import HostRing

    name = f"tca_test_ring_{os.getpid()}"
    ring = HostRing(name, nslots=3, world=2, create=True, pin=False)
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_peer, args=(name, q))
    p.start()
    try:
        for seq in range(1, 7):
            s = seq % 3
            if seq > 3:
                assert ring.wait_acks(s, [1], seq - 3, 10000) == []
            if seq in (1, 4):  # a new data generation mid-stream
                ring.new_generation(4096 * seq)
            data = ring.data
            data.slot(s)[:8] = np.arange(seq, seq + 8, dtype=np.uint8)
            hdr = ring.header(s)
            hdr[1], hdr[2] = ring.gen, data.slot_bytes
            ring.publish(s, seq)
        for seq in range(4, 7):
            s = seq % 3
            assert ring.wait_acks(s, [1], seq, 10000) == []
            np.testing.assert_array_equal(ring.data.slot(s)[8:16], np.arange(seq, seq + 8, dtype=np.uint8)[::-1])
        assert q.get(timeout=30) == "ok"
        # a rank that never acks: the wait times out and names it
        assert ring.wait_acks(0, [1, 2], 100, 50) == [1, 2]
        assert not ring.wait_ready(0, 99, 20)
    finally:
        p.join(10)
        ring.close()
    assert not os.path.exists(ring.ctl_path) and not os.path.exists(ring.data_path(1))


def _fake_sysfs(tmp_path, devices, kfd_nodes=()):
    pci = tmp_path / "pci"
    for bdf, vendor, cls, cpus, node in devices:
        d = pci / bdf
        d.mkdir(parents=True)
        (d / "vendor").write_text(vendor + "\n")
        (d / "class").write_text(cls + "\n")
        (d / "local_cpulist").write_text(cpus + "\n")
        (d / "numa_node").write_text(f"{node}\n")
    kfd = tmp_path / "kfd"
    kfd.mkdir()
    for i, props in enumerate(kfd_nodes):
        n = kfd / str(i)
        n.mkdir()
        (n / "properties").write_text("".join(f"{k} {v}\n" for k, v in props.items()))
    return str(pci), str(kfd)


def test_numa_binding_from_sysfs(tmp_path, monkeypatch):
    from triton_client_amd.parallel import numa

    assert numa.parse_cpulist("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    root, kfd = _fake_sysfs(tmp_path, (
        ("0000:05:00.0", "0x1002", "0x038000", "0-1", 0),
        ("0000:15:00.0", "0x1002", "0x120000", "2-3", 1),   # Instinct: processing accelerator
        ("0000:16:00.0", "0x8086", "0x038000", "4-5", 0),   # not AMD
        ("0000:17:00.0", "0x1002", "0x020000", "6-7", 0)))  # not a GPU
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    # no KFD topology: PCI class order
    assert [os.path.basename(d) for d in numa.gpu_devices(root, kfd)] == ["0000:05:00.0", "0000:15:00.0"]
    assert numa.gpu_cpus(1, root, kfd) == {2, 3}
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert numa.gpu_cpus(0, root, kfd) == {2, 3}
    info = numa.describe(0, root, kfd)
    assert info["gpu_pci"] == "0000:15:00.0" and info["numa_node"] == 1 and info["local_cpus"] == 2
    monkeypatch.setenv("TCA_NUMA_BIND", "0")
    assert numa.bind_to_gpu(0, root, kfd) is None


def test_numa_kfd_topology_order(tmp_path, monkeypatch):
    """KFD GPU nodes (simd_count > 0) name the PCI functions in HSA agent order, which
    need not be bus order; CPU nodes are skipped."""
    from triton_client_amd.parallel import numa

    root, kfd = _fake_sysfs(tmp_path, (
        ("0000:05:00.0", "0x1002", "0x120000", "0-1", 0),
        ("0000:85:00.0", "0x1002", "0x120000", "2-3", 1)),
        kfd_nodes=({"cpu_cores_count": 64, "simd_count": 0},
                   {"simd_count": 1024, "location_id": 0x8500, "domain": 0},
                   {"simd_count": 1024, "location_id": 0x0500, "domain": 0}))
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert [os.path.basename(d) for d in numa.gpu_devices(root, kfd)] == ["0000:85:00.0", "0000:05:00.0"]
    assert numa.gpu_cpus(0, root, kfd) == {2, 3}


_BIND_CHILD = r"""
import os, sys, threading, json
from triton_client_amd.parallel import numa
root, kfd = sys.argv[1], sys.argv[2]
seen = {}
go, done = threading.Event(), threading.Event()
def early():
    go.wait()
    seen["early"] = sorted(os.sched_getaffinity(0))
    done.set()
t = threading.Thread(target=early)
t.start()                      # started before the binding
before = sorted(os.sched_getaffinity(0))
got = numa.bind_to_gpu(0, root, kfd)
go.set(); done.wait(10); t.join()
print(json.dumps({"before": before, "got": sorted(got) if got else None, "main": sorted(os.sched_getaffinity(0)),
                  "early": seen["early"]}))
"""


def test_numa_binding_covers_existing_threads(tmp_path):
    """bind_to_gpu binds every thread of the process, including one started earlier
    (run in a child process so the test runner keeps its CPU set)."""
    import json
    import subprocess
    import sys

    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs 2 CPUs")
    local = f"{cpus[0]}"
    root, kfd = _fake_sysfs(tmp_path, (("0000:05:00.0", "0x1002", "0x120000", local, 0),))
    env = {k: v for k, v in os.environ.items() if k not in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                           "CUDA_VISIBLE_DEVICES", "TCA_NUMA_BIND")}
    env["PYTHONPATH"] = ROOT
    out = subprocess.run([sys.executable, "-c", _BIND_CHILD, root, kfd], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["got"] == [cpus[0]] and r["main"] == [cpus[0]] and r["early"] == [cpus[0]], r


# ------------------------------------------------------------------ bag replays, 1 rank vs 2 ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, ranks, device, extra_env=None):
    env = dict(os.environ, OMP_NUM_THREADS="2", TCA_DP_HEARTBEAT="0")
    if extra_env:
        env.update(extra_env)
    if ranks == 1:
        cmd = [sys.executable, "-m"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]


def _bag_messages(path, topic):
    from triton_client_amd.ros.bag import Bag
    with Bag(path) as b:
        return [m for _, m, _ in b.read_messages(topics=[topic])]


def _replay_pair(tmp_path, device, env=None):
    """One rank calibrates the random-init heads on its first frame and exports the
    weights; the two-rank run loads them (--weights) -- the way a deployment pins a
    model across launches: head calibration on the GPU is not bit-reproducible from one
    process to the next (MIOpen / PyTorch reductions), so two separate launches would
    otherwise each calibrate their own prior."""
    out = {}
    w2, w3 = str(tmp_path / "w2.pt"), str(tmp_path / "w3.pt")
    for ranks in (1, 2):
        ob2, ob3 = str(tmp_path / f"cam{ranks}.bag"), str(tmp_path / f"pc{ranks}.bag")
        wflag2 = ["--export-weights", w2] if ranks == 1 else ["--weights", w2]
        wflag3 = ["--export-weights", w3] if ranks == 1 else ["--weights", w3]
        _run(["triton_client_amd.cli.bag2d", "--bag", FIX, "--engine", "local", "--device", device, "--out", "",
              "--out-bag", ob2, "--frames-per-step", "2"] + wflag2, ranks, device, env)
        _run(["triton_client_amd.cli.bag3d", "--bag", FIX, "--engine", "local", "--device", device, "--out-bag", ob3,
              "--labels", "all", "--score-thresh", "0", "--frames-per-step", "1"] + wflag3, ranks, device, env)
        out[ranks] = (_bag_messages(ob2, "/aver_01/camera_color/detection/detections"),
                      _bag_messages(ob2, "/aver_01/camera_color/detection"),
                      _bag_messages(ob3, "/detections_3d"))
    return out


def _assert_identical(out):
    from triton_client_amd.ros import rosmsg

    d1, im1, b1 = out[1]
    d2, im2, b2 = out[2]
    assert len(d1) == len(d2) == 3 and len(b1) == len(b2) == 2
    assert [m.header.seq for m in d2] == [m.header.seq for m in d1]
    for a, b in zip(d1 + im1 + b1, d2 + im2 + b2):  # byte-identical messages
        assert rosmsg.serialize(a) == rosmsg.serialize(b)
    assert sum(len(m.boxes) for m in b1) > 0


def test_bag_replays_two_ranks_identical_cpu(tmp_path):
    _runtime_or_skip()
    _assert_identical(_replay_pair(tmp_path, "cpu"))


@pytest.mark.gpu
def test_bag_replays_two_ranks_identical_gpu(cuda, tmp_path):
    """The verdict's rehearsal: bag2d / bag3d --engine local on the GPU, two ranks on the
    one card (gloo), the node batch through the host ring; outputs == one rank's."""
    _assert_identical(_replay_pair(tmp_path, "cuda", {"TCA_DIST_BACKEND": "gloo"}))


def _dp_camera_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(280, exit=True)
    try:
        import io

        import torch
        from PIL import Image

        from triton_client_amd.inference.engines import LocalDetector2D
        from triton_client_amd.parallel.dp import DataParallelDetector2D, init_distributed
        from triton_client_amd.ros import msgs
        from triton_client_amd.utils.synthetic import camera_frame

        info = init_distributed("gloo")
        det = LocalDetector2D(batch=3, device=info.device, letterbox=True, names=[f"c{i}" for i in range(80)])
        dp = DataParallelDetector2D(det, info)  # rank 0 calibrates on the first frame and broadcasts
        if info.is_main:
            jp = []
            for i in range(7):
                buf = io.BytesIO()
                Image.fromarray(camera_frame(240, 320, 30 + i)).save(buf, format="JPEG", quality=85)
                jp.append(buf.getvalue())
            ms = [msgs.CompressedImage(header=msgs.Header(seq=i + 1), format="jpeg", data=d) for i, d in enumerate(jp)]
            got = dp.live().process(ms, draw=True, names=det.names)
            held = [im for im, _ in got]  # published messages still viewing the ring
            again = dp.live().process(ms, draw=True, names=det.names)  # slots in use: a new data generation
            dp.close()
            want = det.live().process(ms, draw=True, names=det.names)
            assert sum(len(d) for _, d in want) > 0
            for res in (got, again):
                for (im, d), (wim, wd), m in zip(res, want, ms):
                    np.testing.assert_array_equal(d, wd)
                    assert im.header is m.header and bytes(im.data) == bytes(wim.data)
            assert held[0].data.obj is not None
            q.put((0, "ok"))
        else:
            q.put((rank, f"served {dp.serve()}"))
        torch.cuda.synchronize()
        q.close()
        q.join_thread()
        os._exit(0)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


@pytest.mark.gpu
def test_dp_camera_jpeg_annotated_two_ranks(cuda):
    """JPEG messages through the ring on two ranks (each decodes its own shard on the
    device, annotated frames DMA'd into the ring): detections and published images
    equal one rank's live path bit for bit."""
    import torch.multiprocessing as tmp

    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_camera_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    # 7 frames, batch 3 per rank: steps of 6 (3 + 3) and 1 (rank 0 alone), twice
    assert res == {0: "ok", 1: "served 2"}, res


# ------------------------------------------------------------------ slot reuse vs a slow non-participant
class _NullEngine:
    names = []

    def detect(self, frames):
        return [np.zeros((0, 6), np.float32) for _ in frames]


def _slow_peer_worker(rank, world, port, q, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TCA_NUMA_BIND="0")
    try:
        import time

        from triton_client_amd.parallel.dp import init_distributed
        from triton_client_amd.parallel.ring_dp import DataParallelDetector2D
        from triton_client_amd.ros import compat, msgs

        info = init_distributed("gloo")
        dp = DataParallelDetector2D(_NullEngine(), info, nslots=3)
        if info.is_main:
            frame = np.zeros((8, 8, 3), np.uint8)
            for i in range(steps):  # one message per step: rank 0 is the only participant
                m = compat.numpy_to_imgmsg(frame, "rgb8", header=msgs.Header(seq=i))
                assert len(dp.process([m], draw=False)) == 1
            dp.close()
            q.put((0, dp.steps))
        else:
            orig = dp.ring.wait_ready

            def slow(s, seq, timeout_ms):  # a peer that reads every header late
                time.sleep(0.02)
                return orig(s, seq, timeout_ms)
            dp.ring.wait_ready = slow
            q.put((rank, dp.serve()))
            dp.ring.close()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_ring_slot_reuse_waits_for_slow_non_participant():
    """Single-message steps have only rank 0 as participant, but every peer reads every
    slot header: rank 0 must not rewrite a slot a slow peer has not acked yet (it would
    read a newer header and end its serve loop with a RingStepError)."""
    _runtime_or_skip()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 15
    procs = [ctx.Process(target=_slow_peer_worker, args=(r, 2, port, q, steps)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res == {0: steps, 1: 0}, res


def test_ring_data_area_reserved_or_clear_error(monkeypatch):
    """Ring files are fully backed when created (no SIGBUS later on a full /dev/shm);
    when /dev/shm cannot hold one, creation fails with RingSpaceError and leaves no file."""
    import errno

    from triton_client_amd.parallel import host_ring

    name = f"tca_test_space_{os.getpid()}"
    ring = host_ring.HostRing(name, nslots=2, world=1, create=True, pin=False)
    try:
        d = ring.new_generation(1 << 20)
        assert os.stat(d.path).st_blocks * 512 >= 2 << 20  # allocated, not sparse
        def full(fd, off, size):
            raise OSError(errno.ENOSPC, "No space left on device")
        monkeypatch.setattr(host_ring.os, "posix_fallocate", full)
        with pytest.raises(host_ring.RingSpaceError, match="shm-size"):
            ring.new_generation(4 << 20)
        assert not os.path.exists(ring.data_path(ring.gen + 1)) and ring.data is d and os.path.exists(d.path)
    finally:
        monkeypatch.undo()
        ring.close()


# ------------------------------------------------------------------ ingest arena: payloads deserialised into the ring
def test_ingest_arena_fifo_allocator():
    """Blocks are handed out in order, freed out of order (the tail advances over freed
    blocks only), wrap at the end, and a full arena returns None instead of blocking."""
    import gc

    from triton_client_amd.parallel.host_ring import IngestArena

    path = f"/dev/shm/tca_test_arena_{os.getpid()}"
    ar = IngestArena(path, 4096, True, pin=False)
    try:
        a = ar.alloc(1000)  # 1024 B blocks
        b = ar.alloc(1000)
        c = ar.alloc(1000)
        assert [ar.offset_of(x, 1000) for x in (a, b, c)] == [0, 1024, 2048]
        a[:] = 1
        view = memoryview(b)[10:20]  # a view keeps its block alive
        del b
        gc.collect()
        assert ar.in_use() == 3072
        d = ar.alloc(1000)
        assert ar.offset_of(d, 1000) == 3072 and ar.alloc(100) is None and ar.stats["full"] == 1
        del a
        gc.collect()
        e = ar.alloc(1000)  # wraps into a's block
        assert ar.offset_of(e, 1000) == 0
        del view, c
        gc.collect()
        f = ar.alloc(2000)  # b and c freed behind e: the tail moved past them
        assert ar.offset_of(f, 2000) == 1024
        assert ar.offset_of(np.zeros(10, np.uint8), 10) is None and ar.offset_of(b"xy", 2) is None
        del d, e, f
        gc.collect()
        assert ar.in_use() == 0
    finally:
        ar.close(unlink=True)
    assert not os.path.exists(path)


def test_bag_read_ahead_threads_match_sequential(tmp_path):
    """ROS bag replay with chunks read ahead by threads into alloc buffers: every message in
    order and equal to the sequential read, a full arena (alloc -> None) falling back."""
    from triton_client_amd.ros import compat, msgs
    from triton_client_amd.ros.bag import Bag, RosBag

    rng = np.random.default_rng(3)
    path = str(tmp_path / "multi.bag")
    w = RosBag(path, "w")
    frames = [rng.integers(0, 255, (100, 300, 3), np.uint8) for _ in range(12)]
    for i, f in enumerate(frames):
        w.write("/cam", compat.numpy_to_imgmsg(f, "rgb8", header=msgs.Header(seq=i)))
        w.write("/other", msgs.Header(seq=1000 + i))
    w.close()
    with Bag(path) as b:
        want = [(t, m) for t, m, _ in b.read_messages()]
    calls = []

    def alloc(n):
        calls.append(n)
        return np.empty(n, np.uint8) if len(calls) % 3 else None  # every third: "full"
    with Bag(path) as b:
        got = [(t, m) for t, m, _ in b.read_messages(alloc=alloc, readers=4)]
    assert calls and [t for t, _ in got] == [t for t, _ in want]
    for (_, a), (_, c) in zip(got, want):
        if hasattr(c, "data"):
            assert bytes(a.data) == bytes(c.data) and a.header.seq == c.header.seq
        else:
            assert a.seq == c.seq


def test_deserialize_into_caller_buffers(tmp_path):
    """rosmsg.deserialize / Bag.read_messages put large byte arrays into alloc() buffers
    (the ring's ingest arena) and leave small ones as bytes; the messages are unchanged."""
    from triton_client_amd.ros import compat, msgs, rosmsg
    from triton_client_amd.ros.bag import Bag

    frame = np.random.default_rng(0).integers(0, 255, (120, 200, 3), np.uint8)
    m = compat.numpy_to_imgmsg(frame, "rgb8", header=msgs.Header(seq=3))
    small = compat.numpy_to_imgmsg(frame[:4, :4], "rgb8")
    got, bufs = [], []

    def alloc(n):
        got.append(n)
        bufs.append(np.zeros(n, np.uint8))
        return bufs[-1]
    for msg in (m, small):
        back = rosmsg.deserialize(rosmsg.serialize(msg), "sensor_msgs/Image", alloc)
        assert bytes(back.data) == bytes(msg.data) and back.header.seq == msg.header.seq
    assert got == [frame.nbytes]
    assert isinstance(rosmsg.deserialize(rosmsg.serialize(m), "sensor_msgs/Image").data, bytes)
    for kind in ("rosbag", "tca"):
        path = str(tmp_path / f"x_{kind}.bag")
        if kind == "rosbag":
            from triton_client_amd.ros.bag import RosBag
            w = RosBag(path, "w")
        else:
            w = Bag(path, "w")
        w.write("/cam", m)
        w.close()
        got.clear()
        bufs.clear()
        with Bag(path) as b:
            (_, back, _), = list(b.read_messages(topics=["/cam"], alloc=alloc))
        with Bag(path) as b:  # chunks read ahead by reader threads: the same message
            (_, back2, _), = list(b.read_messages(topics=["/cam"], alloc=alloc, readers=3))
        assert bytes(back2.data) == bytes(back.data) and back2.header.seq == back.header.seq
        got.pop()
        bufs.pop()
        assert isinstance(back.data, memoryview), kind
        # ROS bags: the whole uncompressed chunk is read into the buffer and the payload is a view
        # of it; msgpack bags: the payload is copied into a buffer of its own size
        assert len(got) == 1 and got[0] >= frame.nbytes, (kind, got)
        a0 = bufs[0].ctypes.data
        addr = np.frombuffer(back.data, np.uint8).ctypes.data
        assert a0 <= addr and addr + frame.nbytes <= a0 + got[0]
        np.testing.assert_array_equal(compat.imgmsg_to_numpy(back, "rgb8"), frame)


class _SumEngine:
    """Host engine whose 'detection' is a checksum of the frame: a peer that read the
    wrong bytes shows up in the result."""
    names = []

    def detect(self, frames):
        return [np.array([[float(f.sum() % 100003), float(f[0, 0, 0]), 0, 0, 1, 0]], np.float32) for f in frames]


def _arena_worker(rank, world, port, q, arena_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TCA_NUMA_BIND="0")
    try:
        from triton_client_amd.parallel.dp import init_distributed
        from triton_client_amd.parallel.ring_dp import DataParallelDetector2D
        from triton_client_amd.ros import compat, msgs, rosmsg

        info = init_distributed("gloo")
        dp = DataParallelDetector2D(_SumEngine(), info, nslots=2, arena_mb=arena_mb)
        if info.is_main:
            rng = np.random.default_rng(1)
            wire = [rosmsg.serialize(compat.numpy_to_imgmsg(rng.integers(0, 255, (160, 256, 3), np.uint8), "rgb8",
                                                            header=msgs.Header(seq=i))) for i in range(9)]
            res = []
            for rep in range(3):  # more steps than slots: blocks are freed and reused
                # rep 1 mixes arena payloads with copied ones in the same steps
                ms = [rosmsg.deserialize(w, "sensor_msgs/Image", dp.ingest_buffer if (rep != 1 or i % 2) else None)
                      for i, w in enumerate(wire)]
                res.append([d for _, d in dp.process(ms, draw=False)])
                want = _SumEngine().detect([compat.imgmsg_to_numpy(x, "rgb8") for x in ms])
                for d, w in zip(res[-1], want):
                    np.testing.assert_array_equal(d, w)
                del ms
            q.put((0, (dp.arena_items, dp.copied_items, dp.steps)))
            dp.close()
        else:
            q.put((rank, dp.serve()))
            dp.ring.close()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("arena_mb", [4, 0])
def test_ring_payloads_from_ingest_arena_two_ranks(arena_mb):
    """Frames deserialised into rank 0's ingest arena reach rank 1 without a slot copy
    (those items read from the arena; one round mixes arena and copied payloads in the same
    steps) and give the same results as the copy path (arena off)."""
    _runtime_or_skip()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_arena_worker, args=(r, 2, port, q, arena_mb)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res[1] == 3, res
    assert res[0] == ((22, 5, 3) if arena_mb else (0, 27, 3)), res


def _file_worker(rank, world, port, q, path, shard):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TCA_NUMA_BIND="0", TCA_RING_FILE_SHARD=str(int(shard)))
    try:
        from triton_client_amd.parallel.dp import init_distributed
        from triton_client_amd.parallel.ring_dp import DataParallelDetector2D
        from triton_client_amd.ros.bag import Bag

        info = init_distributed("gloo")
        dp = DataParallelDetector2D(_SumEngine(), info, nslots=2, arena_mb=0)
        if info.is_main:
            assert dp.file_sharding == shard
            seqs, dets = [], []
            with Bag(path) as b:
                ms = [m for _, m, _ in b.read_messages(topics=["/cam"], mapped=dp.file_sharding)]
                for k in range(0, len(ms), 4):  # steps of 4 frames over the two ranks
                    chunk = ms[k:k + 4]
                    for m, (im, d) in zip(chunk, dp.process(chunk, draw=False)):
                        seqs.append(im.header.seq)
                        dets.append(d.tolist())
                del ms
            q.put((0, (seqs, dets, dp.file_items, dp.copied_items)))
            dp.close()
        else:
            q.put((rank, dp.serve()))
            dp.ring.close()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_sharded_bag_replay_reads_payloads_per_rank(tmp_path):
    """Sharded replay: rank 0 reads the bag mapped (record headers + message prefixes only)
    and publishes file offsets; rank 1 reads its shard's payloads from its own mapping of the
    bag.  Same messages, same order and same results as the copy path and as one engine."""
    _runtime_or_skip()
    from triton_client_amd.ros import compat, msgs
    from triton_client_amd.ros.bag import Bag, RosBag

    rng = np.random.default_rng(5)
    path = str(tmp_path / "cams.bag")
    w = RosBag(path, "w")
    frames = []
    for i in range(10):
        f = rng.integers(0, 255, (120, 200, 3), np.uint8)
        frames.append(f)
        w.write("/cam", compat.numpy_to_imgmsg(f, "rgb8", header=msgs.Header(seq=100 + i)))
        if i % 3 == 0:  # a non-sensor message type between the frames (flushes the native parse run)
            w.write("/other", msgs.BoundingBoxArray(header=msgs.Header(seq=i)))
    w.close()
    want = [d.tolist() for d in _SumEngine().detect(frames)]
    out = {}
    for shard in (True, False):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_file_worker, args=(r, 2, port, q, path, shard)) for r in range(2)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=180) for _ in range(2))
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
        assert isinstance(res[1], int) and res[1] == 3, res
        out[shard] = res[0]
    seqs, dets, nfile, ncopy = out[True]
    assert seqs == list(range(100, 110)) and dets == want
    assert (nfile, ncopy) == (10, 0)
    assert out[False][:2] == (seqs, dets) and out[False][2:] == (0, 10)
    # the mapped reader yields the same messages as the ordinary one
    with Bag(path) as a, Bag(path) as b:
        ra, rb = list(a.read_messages()), list(b.read_messages(mapped=True))
        assert len(ra) == len(rb) == 14
        for (t1, m1, s1), (t2, m2, s2) in zip(ra, rb):
            assert (t1, s1) == (t2, s2) and m1.header == m2.header
            if t1 == "/cam":
                assert bytes(m1.data) == bytes(m2.data) and isinstance(m2.data, memoryview)
