"""Native ROS wire parse (csrc/runtime/ros_wire.cpp) against the schema-driven Python reader
(``rosmsg.deserialize_py``): Image / CompressedImage / PointCloud2 with random headers,
strings and payload sizes, into bytes, into caller buffers (the ingest arena) and as
zero-copy views; malformed and truncated buffers are rejected; the bag chunk record scan
finds what the Python chunk walker finds."""
import numpy as np
import pytest

from triton_client_amd.ros import msgs, rosmsg


def _rt():
    rt = rosmsg._native_rt()
    if rt is None or not hasattr(rt, "tca_ros_parse"):
        pytest.skip("runtime library not built")
    return rt


def _messages(rng, n):
    out = []
    for i in range(n):
        hdr = msgs.Header(int(rng.integers(0, 2**32)), msgs.Time(int(rng.integers(0, 2**31)), int(rng.integers(0, 10**9))),
                          "frame_%d" % rng.integers(0, 5) + "é" * int(rng.integers(0, 2)))
        k = int(rng.choice([0, 17, 65536, 200_003]))
        data = rng.integers(0, 256, k, dtype=np.uint8).tobytes()
        t = i % 3
        if t == 0:
            out.append(("sensor_msgs/Image", msgs.Image(hdr, int(rng.integers(1, 1000)), int(rng.integers(1, 1000)),
                                                        rng.choice(["rgb8", "bgr8", "mono8"]), int(rng.integers(0, 2)),
                                                        int(rng.integers(0, 5000)), data)))
        elif t == 1:
            out.append(("sensor_msgs/CompressedImage", msgs.CompressedImage(hdr, rng.choice(["jpeg", "png"]), data)))
        else:
            fields = [msgs.PointField(nm, 4 * j, 7, 1) for j, nm in enumerate(["x", "y", "z", "intensity"][:int(rng.integers(1, 5))])]
            out.append(("sensor_msgs/PointCloud2", msgs.PointCloud2(hdr, 1, k // 16, fields, bool(rng.integers(0, 2)), 16,
                                                                    k, data, bool(rng.integers(0, 2)))))
    return out


def _same(a, b):
    assert type(a) is type(b)
    for f in a.__dataclass_fields__:
        va, vb = getattr(a, f), getattr(b, f)
        if f == "data":
            assert bytes(va) == bytes(vb)
        else:
            assert va == vb, f


@pytest.mark.parametrize("mode", ["bytes", "alloc", "zero_copy"])
def test_native_parse_matches_python_reader(mode):
    _rt()
    rng = np.random.default_rng(0)
    bufs = []
    alloc = (lambda n: bufs.append(np.empty(n, np.uint8)) or bufs[-1]) if mode == "alloc" else None
    for typ, m in _messages(rng, 30):
        wire = rosmsg.serialize(m, typ)
        want = rosmsg.deserialize_py(wire, typ)
        got = rosmsg.deserialize_many([wire], typ, alloc=alloc, zero_copy=mode == "zero_copy")[0]
        _same(want, got)
        _same(m, got) if typ != "sensor_msgs/PointCloud2" else None
        big = len(m.data) >= rosmsg.ALLOC_MIN
        if mode == "alloc" and big:
            assert isinstance(got.data, memoryview) and got.data.obj is bufs[-1]
        if mode == "zero_copy" and big:
            assert isinstance(got.data, memoryview)
        if not big or mode == "bytes":
            assert isinstance(got.data, bytes)
        # the single-message entry point takes the native path for these types
        _same(want, rosmsg.deserialize(wire, typ))


def test_native_batch_of_mixed_sizes_one_call():
    _rt()
    rng = np.random.default_rng(1)
    ms = [m for t, m in _messages(rng, 60) if t == "sensor_msgs/Image"]
    wires = [rosmsg.serialize(m) for m in ms]
    arena = np.empty(sum(len(w) for w in wires) + 4096 * len(wires), np.uint8)
    pos = [0]

    def alloc(n):
        o = pos[0]
        pos[0] += (n + 4095) // 4096 * 4096
        return arena[o:o + n]
    got = rosmsg.deserialize_many(wires, "sensor_msgs/Image", alloc=alloc, threads=4)
    for m, g in zip(ms, got):
        _same(m, g)


def test_native_parse_rejects_malformed():
    _rt()
    m = msgs.Image(msgs.Header(1, msgs.Time(2, 3), "f"), 2, 2, "rgb8", 0, 6, bytes(range(12)))
    wire = rosmsg.serialize(m)
    for bad in (wire[:-1], wire + b"\0", wire[:10], b""):
        with pytest.raises(Exception):
            rosmsg.deserialize_many([wire, bad], "sensor_msgs/Image")
    # a string length past the end
    evil = bytearray(wire)
    evil[12:16] = (1 << 30).to_bytes(4, "little")
    with pytest.raises(Exception):
        rosmsg.deserialize_many([bytes(evil)], "sensor_msgs/Image")


def test_bag_scan_matches_python_walker(tmp_path):
    rt = _rt()
    from triton_client_amd.ros import rosbag_v2
    rng = np.random.default_rng(2)
    path = str(tmp_path / "x.bag")
    w = rosbag_v2.RosBagWriter(path, chunk_threshold=1 << 30)  # one chunk
    for typ, m in _messages(rng, 9):
        w.write("/t/" + typ.split("/")[1], m)
    w.close()
    r = rosbag_v2.RosBagReader(path)
    blob = None
    for h, off, dl in r._records():
        if h["op"][0] == rosbag_v2.OP_CHUNK:
            r.f.seek(off)
            blob = r.f.read(dl)
            break
    want = list(r._iter_payload(blob))
    cap = len(blob) // 8
    arr = {k: np.empty(cap, dt) for k, dt in (("op", np.int32), ("conn", np.int32), ("sec", np.uint32),
                                              ("nsec", np.uint32), ("hoff", np.int64), ("hlen", np.int64),
                                              ("doff", np.int64), ("dlen", np.int64))}
    b = np.frombuffer(blob, np.uint8)
    k = rt.tca_bag_scan(b.ctypes.data, len(blob), cap, *[arr[n].ctypes.data for n in
                                                         ("op", "conn", "sec", "nsec", "hoff", "hlen", "doff", "dlen")])
    msgs_ = [i for i in range(k) if arr["op"][i] == rosbag_v2.OP_MSG]
    assert len(msgs_) == len(want) == 9
    for i, (c, t, data) in zip(msgs_, want):
        assert arr["conn"][i] == c.id and (arr["sec"][i], arr["nsec"][i]) == (t.secs, t.nsecs)
        assert blob[arr["doff"][i]:arr["doff"][i] + arr["dlen"][i]] == bytes(data)
    assert rt.tca_bag_scan(b.ctypes.data, len(blob) - 3, cap, *[arr[n].ctypes.data for n in arr]) == -1


def test_rospy_anymsg_ingest_into_arena(monkeypatch):
    """With a real ROS master (faked here: rospy is not installed), a data-parallel driver's
    subscriber takes the raw wire bytes (``rospy.AnyMsg``) and deserialises them natively with
    the payload in the ingest arena; other types / no arena keep the typed subscription."""
    _rt()
    from triton_client_amd.ros import compat

    subs = []

    class AnyMsg:
        pass

    class _Sub:
        def __init__(self, topic, t, cb, queue_size=None):
            subs.append((topic, t, cb))

    FakeRospy = type("FakeRospy", (), {"AnyMsg": AnyMsg, "Subscriber": _Sub})

    monkeypatch.setattr(compat, "HAVE_ROSPY", True)
    monkeypatch.setattr(compat, "_rospy", FakeRospy)
    arena = np.zeros(1 << 22, np.uint8)
    used = []

    def ingest(n):
        used.append(n)
        return arena[:n]
    got = []
    compat.Subscriber("/cam", msgs.CompressedImage, got.append, ingest=ingest)
    compat.Subscriber("/dets", msgs.Detection2DArray, got.append, ingest=ingest)
    compat.Subscriber("/cam2", msgs.CompressedImage, got.append)
    assert [t for _, t, _ in subs] == [AnyMsg, msgs.Detection2DArray, msgs.CompressedImage]
    payload = bytes(range(256)) * 600  # >= ALLOC_MIN
    raw = AnyMsg()
    raw._buff = rosmsg.serialize(msgs.Image(msgs.Header(7, msgs.Time(1, 2), "cam"), 200, 256, "rgb8", 0, 768,
                                            payload))
    raw._connection_header = {"type": "sensor_msgs/Image"}
    subs[0][2](raw)
    m = got[-1]
    assert isinstance(m, msgs.Image) and m.header.seq == 7 and bytes(m.data) == payload
    assert used == [len(payload)] and np.frombuffer(m.data, np.uint8).ctypes.data == arena.ctypes.data
