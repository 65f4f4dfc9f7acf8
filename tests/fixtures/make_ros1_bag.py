"""Builds tests/fixtures/ros1_sensors.bag byte by byte, independently of
triton_client_amd.ros.rosbag_v2 / rosmsg: the ROS bag 2.0 record layout and
the genpy wire format of sensor_msgs/{CompressedImage, Image, PointCloud2}
written by hand, with the md5sums the ROS message packages publish.

    python tests/fixtures/make_ros1_bag.py   # rewrites the fixture (deterministic)

Contents (what tests/test_rosbag_v2.py checks):
  /camera/color/image_raw                      3 x sensor_msgs/CompressedImage (JPEG 64x48)
  /camera/color/image_raw_rgb                  2 x sensor_msgs/Image rgb8 32x24
  /ai_test_field/sensors/os_cloud_node/points  2 x sensor_msgs/PointCloud2 (x,y,z,intensity f32, 1500 pts)
  /diagnostics_raw                             1 x acme_msgs/Opaque (no schema: read back raw)
chunk 1 uncompressed, chunk 2 bz2.
"""
import bz2
import io
import os
import struct

import numpy as np

MD5 = {"sensor_msgs/CompressedImage": "8f7a12909da2c9d3332d540a0977563f",
       "sensor_msgs/Image": "060021388200f6f0f447d0fcd9c64743",
       "sensor_msgs/PointCloud2": "1158d486dd51d683ce2f1be655c3c181",
       "acme_msgs/Opaque": "0123456789abcdef0123456789abcdef"}


def u32(v):
    return struct.pack("<I", v)


def string(s):
    b = s.encode()
    return u32(len(b)) + b


def header(seq, secs, nsecs, frame):
    return u32(seq) + u32(secs) + u32(nsecs) + string(frame)


def fields(d):
    out = b""
    for k, v in d.items():
        f = k.encode() + b"=" + v
        out += u32(len(f)) + f
    return out


def record(h, data):
    hb = fields(h)
    return u32(len(hb)) + hb + u32(len(data)) + data


def jpeg(seed):
    from PIL import Image
    rng = np.random.default_rng(seed)
    img = (rng.integers(0, 255, (48, 64, 3))).astype(np.uint8)
    img[10:30, 20:50] = (200, 30, 30)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=90)
    return b.getvalue()


def cloud(seed, n=1500):
    rng = np.random.default_rng(seed)
    p = np.zeros((n, 4), np.float32)
    p[:, 0] = rng.uniform(2, 40, n)
    p[:, 1] = rng.uniform(-20, 20, n)
    p[:, 2] = rng.uniform(-2, 1, n)
    p[:, 3] = rng.uniform(0, 100, n)
    p[::97, 0] = np.nan
    return p


def msgs_():
    out = []
    for i in range(3):
        data = jpeg(i)
        out.append(("/camera/color/image_raw", "sensor_msgs/CompressedImage", (100 + i, 0),
                    header(i, 100 + i, 0, "camera") + string("jpeg") + u32(len(data)) + data))
    for i in range(2):
        px = np.full((24, 32, 3), 40 * i + 7, np.uint8).tobytes()
        out.append(("/camera/color/image_raw_rgb", "sensor_msgs/Image", (110 + i, 5),
                    header(i, 110 + i, 5, "camera") + u32(24) + u32(32) + string("rgb8") + b"\x00" + u32(96)
                    + u32(len(px)) + px))
    for i in range(2):
        p = cloud(10 + i)
        flds = u32(4) + b"".join(string(nm) + u32(off) + b"\x07" + u32(1)
                                 for nm, off in (("x", 0), ("y", 4), ("z", 8), ("intensity", 12)))
        data = p.tobytes()
        out.append(("/ai_test_field/sensors/os_cloud_node/points", "sensor_msgs/PointCloud2", (120 + i, 0),
                    header(i, 120 + i, 0, "os_sensor") + u32(1) + u32(len(p)) + flds + b"\x00" + u32(16)
                    + u32(16 * len(p)) + u32(len(data)) + data + b"\x00"))
    out.append(("/diagnostics_raw", "acme_msgs/Opaque", (130, 0), b"\x01\x02\x03\x04"))
    return out


def main(path):
    ms = msgs_()
    conns = {}
    for topic, typ, _, _ in ms:
        conns.setdefault((topic, typ), len(conns))

    def conn_rec(topic, typ):
        cid = conns[(topic, typ)]
        return record({"op": b"\x07", "conn": u32(cid), "topic": topic.encode()},
                      fields({"topic": topic.encode(), "type": typ.encode(), "md5sum": MD5[typ].encode(),
                              "message_definition": b""}))

    body = bytearray()
    chunk_infos = []
    for ci, (part, comp) in enumerate(((ms[:4], "none"), (ms[4:], "bz2"))):
        raw = bytearray()
        seen = set()
        index = {}
        for topic, typ, (s, ns), data in part:
            cid = conns[(topic, typ)]
            if cid not in seen:
                raw += conn_rec(topic, typ)
                seen.add(cid)
            index.setdefault(cid, []).append((s, ns, len(raw)))
            raw += record({"op": b"\x02", "conn": u32(cid), "time": u32(s) + u32(ns)}, data)
        blob = bytes(raw) if comp == "none" else bz2.compress(bytes(raw))
        pos = len(b"#ROSBAG V2.0\n") + 4096 + len(body)
        body += record({"op": b"\x05", "compression": comp.encode(), "size": u32(len(raw))}, blob)
        for cid, ents in sorted(index.items()):
            body += record({"op": b"\x04", "ver": u32(1), "conn": u32(cid), "count": u32(len(ents))},
                           b"".join(u32(s) + u32(ns) + u32(o) for s, ns, o in ents))
        ts = [(s, ns) for _, _, (s, ns), _ in part]
        chunk_infos.append((pos, min(ts), max(ts), {c: len(e) for c, e in index.items()}))
    index_pos = len(b"#ROSBAG V2.0\n") + 4096 + len(body)
    for (topic, typ) in sorted(conns, key=lambda k: conns[k]):
        body += conn_rec(topic, typ)
    for pos, t0, t1, counts in chunk_infos:
        body += record({"op": b"\x06", "ver": u32(1), "chunk_pos": struct.pack("<Q", pos),
                        "start_time": u32(t0[0]) + u32(t0[1]), "end_time": u32(t1[0]) + u32(t1[1]),
                        "count": u32(len(counts))}, b"".join(u32(c) + u32(n) for c, n in sorted(counts.items())))
    hb = fields({"op": b"\x03", "index_pos": struct.pack("<Q", index_pos), "conn_count": u32(len(conns)),
                 "chunk_count": u32(len(chunk_infos))})
    pad = 4096 - 4 - len(hb) - 4
    with open(path, "wb") as f:
        f.write(b"#ROSBAG V2.0\n" + u32(len(hb)) + hb + u32(pad) + b" " * pad + bytes(body))


if __name__ == "__main__":
    main(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ros1_sensors.bag"))
