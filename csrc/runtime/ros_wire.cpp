// ROS1 wire parsing for the sensor messages the drivers ingest, and the record scan of a ROS
// bag v2.0 chunk: the per-field Python deserialiser (triton_client_amd/ros/rosmsg.py) costs
// ~100 us of GIL-held interpreter time per message, which caps rank 0 of the data-parallel
// drivers at ~2 GPUs of ingest (profiles/r5/fanout/fanout_arena.json).  Here a batch of
// messages is parsed in one ctypes call (the GIL is released for the whole call); the
// payloads stay where they are -- the caller copies them into the ingest arena with
// tca_host_gather_copy (csrc/runtime/host_copy.cpp) or hands them on as views of a mapped
// bag file.
//
// Wire format (genpy, little-endian): uint32 length prefixes for strings and variable arrays,
// uint8[] as raw bytes, time as (uint32 secs, uint32 nsecs); field order from the .msg files:
//   sensor_msgs/Image:           Header, u32 height, u32 width, string encoding, u8 is_bigendian,
//                                u32 step, uint8[] data
//   sensor_msgs/CompressedImage: Header, string format, uint8[] data
//   sensor_msgs/PointCloud2:     Header, u32 height, u32 width, PointField[] fields, bool
//                                is_bigendian, u32 point_step, u32 row_step, uint8[] data, bool is_dense
//   std_msgs/Header:             u32 seq, time stamp, string frame_id
//   sensor_msgs/PointField:      string name, u32 offset, u8 datatype, u32 count
// Reference: the messages the reference subscribes to and replays
// (communicator/ros_inference.py:93, ros_inference3d.py:96, bag_inference2d.py:34-35,
// bag_inference3d.py:62-63), deserialised there by genpy / rosbag.
#include <cstdint>
#include <cstring>

#define TCA_API extern "C" __attribute__((visibility("default")))

namespace {

struct Cursor {
  const uint8_t* p;
  int64_t n, off;
  bool ok = true;
  bool need(int64_t k) {
    if (!ok || k < 0 || off + k > n) ok = false;
    return ok;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t v;
    std::memcpy(&v, p + off, 4);
    off += 4;
    return v;
  }
  uint8_t u8() {
    if (!need(1)) return 0;
    return p[off++];
  }
  // a length-prefixed byte run: its offset and length
  void run(int64_t& o, int64_t& len) {
    const uint32_t k = u32();
    o = off;
    len = k;
    if (need((int64_t)k)) off += k;
  }
};

enum { kImage = 1, kCompressed = 2, kCloud = 3 };
enum {
  MI_SEQ, MI_SEC, MI_NSEC, MI_FRAME_OFF, MI_FRAME_LEN,
  MI_A, MI_B, MI_C, MI_D, MI_E, MI_F,  // type-specific, see tca_ros_parse
  MI_DATA_OFF, MI_DATA_LEN, MI_G, MI_H, MI_END, MI_INTS
};
static_assert(MI_INTS == 16, "meta row");

bool parse_one(int type, const uint8_t* p, int64_t n, int64_t* m) {
  Cursor c{p, n, 0};
  for (int k = 0; k < MI_INTS; ++k) m[k] = 0;
  m[MI_SEQ] = c.u32();
  m[MI_SEC] = c.u32();
  m[MI_NSEC] = c.u32();
  c.run(m[MI_FRAME_OFF], m[MI_FRAME_LEN]);
  if (type == kImage) {
    m[MI_A] = c.u32();              // height
    m[MI_B] = c.u32();              // width
    c.run(m[MI_C], m[MI_D]);         // encoding
    m[MI_E] = c.u8();               // is_bigendian
    m[MI_F] = c.u32();              // step
    c.run(m[MI_DATA_OFF], m[MI_DATA_LEN]);
  } else if (type == kCompressed) {
    c.run(m[MI_A], m[MI_B]);         // format
    c.run(m[MI_DATA_OFF], m[MI_DATA_LEN]);
  } else if (type == kCloud) {
    m[MI_A] = c.u32();              // height
    m[MI_B] = c.u32();              // width
    m[MI_C] = c.off;                // fields block: [MI_C, MI_D) incl. its count prefix
    const uint32_t nf = c.u32();
    for (uint32_t f = 0; f < nf && c.ok; ++f) {
      int64_t o, l;
      c.run(o, l);                 // name
      c.u32();                     // offset
      c.u8();                      // datatype
      c.u32();                     // count
    }
    m[MI_D] = c.off;
    m[MI_E] = c.u8();               // is_bigendian
    m[MI_F] = c.u32();              // point_step
    m[MI_G] = c.u32();              // row_step
    c.run(m[MI_DATA_OFF], m[MI_DATA_LEN]);
    m[MI_H] = c.u8();               // is_dense
  } else {
    return false;
  }
  m[MI_END] = c.off;
  return c.ok;
}

// a bag record header: <u32 len>name=value fields; picks op, conn, time
bool record_header(const uint8_t* h, int64_t hl, int32_t& op, int32_t& conn, uint32_t& sec, uint32_t& nsec) {
  op = -1;
  conn = -1;
  sec = nsec = 0;
  int64_t o = 0;
  while (o + 4 <= hl) {
    uint32_t fl;
    std::memcpy(&fl, h + o, 4);
    o += 4;
    if (o + fl > (uint64_t)hl) return false;
    const uint8_t* f = h + o;
    const uint8_t* eq = static_cast<const uint8_t*>(std::memchr(f, '=', fl));
    if (eq) {
      const int64_t kl = eq - f, vl = (int64_t)fl - kl - 1;
      const uint8_t* v = eq + 1;
      if (kl == 2 && std::memcmp(f, "op", 2) == 0 && vl >= 1) op = v[0];
      else if (kl == 4 && std::memcmp(f, "conn", 4) == 0 && vl >= 4) std::memcpy(&conn, v, 4);
      else if (kl == 4 && std::memcmp(f, "time", 4) == 0 && vl >= 8) {
        std::memcpy(&sec, v, 4);
        std::memcpy(&nsec, v + 4, 4);
      }
    }
    o += fl;
  }
  return o == hl;
}

}  // namespace

// Parse n messages of one type (1 Image, 2 CompressedImage, 3 PointCloud2).  meta: [n][16]
// int64, offsets relative to each message's first byte:
//   0 seq, 1 stamp secs, 2 stamp nsecs, 3 / 4 frame_id offset / length,
//   Image:           5 height, 6 width, 7 / 8 encoding offset / length, 9 is_bigendian, 10 step
//   CompressedImage: 5 / 6 format offset / length
//   PointCloud2:     5 height, 6 width, 7 / 8 fields block [start, end) (count prefix included),
//                    9 is_bigendian, 10 point_step, 13 row_step, 14 is_dense
//   11 / 12 data offset / length, 15 bytes consumed (== the message length for a well-formed one).
// Returns 0, -1 on a bad argument, or i + 1 for the first message that does not parse.
TCA_API int tca_ros_parse(int type, int n, const uint8_t* const* msgs, const int64_t* lens, int64_t* meta) {
  if (n < 0 || (n > 0 && (!msgs || !lens || !meta)) || type < kImage || type > kCloud) return -1;
  for (int i = 0; i < n; ++i) {
    if (!msgs[i] || lens[i] < 0) return -1;
    int64_t* m = meta + (int64_t)i * MI_INTS;
    if (!parse_one(type, msgs[i], lens[i], m) || m[MI_END] != lens[i]) return i + 1;
  }
  return 0;
}

// Scan the records of a bag v2.0 chunk's (uncompressed) data: per record its op, conn, time
// and the [offset, length) of its header and data inside ``blob``.  Returns the record count
// (<= cap; cap reached: the caller scans on from the last record's end), or -1 on a truncated
// or malformed record.
TCA_API int64_t tca_bag_scan(const uint8_t* blob, int64_t n, int64_t cap, int32_t* op, int32_t* conn, uint32_t* sec,
                             uint32_t* nsec, int64_t* hoff, int64_t* hlen, int64_t* doff, int64_t* dlen) {
  if (!blob || n < 0 || cap < 0) return -1;
  int64_t off = 0, k = 0;
  while (off + 8 <= n && k < cap) {
    uint32_t hl, dl;
    std::memcpy(&hl, blob + off, 4);
    if (off + 4 + (int64_t)hl + 4 > n) return -1;
    std::memcpy(&dl, blob + off + 4 + hl, 4);
    if (off + 8 + (int64_t)hl + (int64_t)dl > n) return -1;
    if (!record_header(blob + off + 4, hl, op[k], conn[k], sec[k], nsec[k])) return -1;
    hoff[k] = off + 4;
    hlen[k] = hl;
    doff[k] = off + 8 + hl;
    dlen[k] = dl;
    off += 8 + (int64_t)hl + dl;
    ++k;
  }
  return k;
}

namespace {
// the value of header field ``key`` ([vo, vo + vl) inside h), false if absent
bool header_field(const uint8_t* h, int64_t hl, const char* key, int64_t kl, int64_t& vo, int64_t& vl) {
  int64_t o = 0;
  while (o + 4 <= hl) {
    uint32_t fl;
    std::memcpy(&fl, h + o, 4);
    o += 4;
    if (o + (int64_t)fl > hl) return false;
    if ((int64_t)fl > kl && h[o + kl] == '=' && std::memcmp(h + o, key, (size_t)kl) == 0) {
      vo = o + kl + 1;
      vl = (int64_t)fl - kl - 1;
      return true;
    }
    o += fl;
  }
  return false;
}
}  // namespace

// Index a mapped ROS bag v2.0 file in one pass: top-level records from state[0], descending into
// uncompressed chunks (state[1] = the offset inside the current chunk's data, 0 at top level).
// Emits message (op 2) and connection (op 7) records with ABSOLUTE offsets, and compressed
// chunks as op 5 records (the caller decompresses those); bag header, index data and chunk info
// records are skipped.  Writes at most cap records and returns their count; state is advanced
// so the next call resumes after the last emitted record (0 records: end of file).  -1: a
// truncated or malformed record.
TCA_API int64_t tca_bag_index(const uint8_t* file, int64_t n, int64_t* state, int64_t cap, int32_t* op, int32_t* conn,
                              uint32_t* sec, uint32_t* nsec, int64_t* hoff, int64_t* hlen, int64_t* doff,
                              int64_t* dlen) {
  if (!file || n < 0 || !state || cap < 0) return -1;
  int64_t top = state[0], inner = state[1], k = 0;
  while (k < cap && top + 8 <= n) {
    uint32_t hl, dl;
    std::memcpy(&hl, file + top, 4);
    if (top + 4 + (int64_t)hl + 4 > n) return -1;
    std::memcpy(&dl, file + top + 4 + hl, 4);
    const int64_t d0 = top + 8 + hl;
    if (d0 + (int64_t)dl > n) return -1;
    int32_t o, c;
    uint32_t s, ns;
    if (!record_header(file + top + 4, hl, o, c, s, ns)) return -1;
    const int64_t next = d0 + dl;
    if (o == 5) {  // chunk
      int64_t vo, vl;
      const bool plain = !header_field(file + top + 4, hl, "compression", 11, vo, vl) ||
                         (vl == 4 && std::memcmp(file + top + 4 + vo, "none", 4) == 0);
      if (!plain) {
        if (inner == 0) {
          op[k] = 5; conn[k] = -1; sec[k] = nsec[k] = 0;
          hoff[k] = top + 4; hlen[k] = hl; doff[k] = d0; dlen[k] = dl;
          ++k;
        }
        top = next;
        inner = 0;
        continue;
      }
      // inner records of the chunk's data [d0, next)
      int64_t p = d0 + inner;
      while (k < cap && p + 8 <= next) {
        uint32_t ihl, idl;
        std::memcpy(&ihl, file + p, 4);
        if (p + 4 + (int64_t)ihl + 4 > next) return -1;
        std::memcpy(&idl, file + p + 4 + ihl, 4);
        const int64_t id0 = p + 8 + ihl;
        if (id0 + (int64_t)idl > next) return -1;
        int32_t io, ic;
        uint32_t is, ins;
        if (!record_header(file + p + 4, ihl, io, ic, is, ins)) return -1;
        if (io == 2 || io == 7) {
          op[k] = io; conn[k] = ic; sec[k] = is; nsec[k] = ins;
          hoff[k] = p + 4; hlen[k] = ihl; doff[k] = id0; dlen[k] = idl;
          ++k;
        }
        p = id0 + idl;
      }
      if (p + 8 <= next) {  // cap reached inside the chunk: resume there
        inner = p - d0;
        break;
      }
      top = next;
      inner = 0;
      continue;
    }
    if (o == 2 || o == 7) {
      op[k] = o; conn[k] = c; sec[k] = s; nsec[k] = ns;
      hoff[k] = top + 4; hlen[k] = hl; doff[k] = d0; dlen[k] = dl;
      ++k;
    }
    top = next;
    inner = 0;
  }
  state[0] = top;
  state[1] = inner;
  return k;
}
