// Baseline JPEG entropy decoder: marker parsing + Huffman decode to quantised
// DCT coefficients, no pixel reconstruction.  The pixel half (dequantise,
// 8x8 IDCT, chroma upsampling, YCbCr -> RGB) runs on the GPU
// (csrc/kernels/jpeg.hip), so the host does only the serial part of a JPEG
// decode and writes coefficients straight into pinned staging.
//
// Reference parity: the camera node decodes CompressedImage JPEGs with
// cv2.imdecode on one thread per message (communicator/ros_inference.py:124-131).
//
// Supported: SOF0 / SOF1 (8-bit sequential Huffman), 1 or 3 components in one
// interleaved scan, any sampling factors up to 2x2, DRI restart intervals.
// Progressive / arithmetic / 12-bit / multi-scan files return an error code
// and the caller decodes them on the host instead.
//
// Output of one frame (geometry from tca_jpeg_probe):
//   coef  int16 [sum_c bh_c*bw_c][64], natural (row-major) order, component
//         planes back to back, blocks in raster order of each component's
//         MCU-padded block grid;
//   q     float [3][64] dequantisation table of each component, natural order;
//   geom  int32 [16] = W, H, nc, hmax, vmax, mcux, mcuy,
//                      h0, v0, h1, v1, h2, v2, nblocks, 0, 0.
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

enum Err {
  OK = 0,
  E_NOT_JPEG = -1,
  E_UNSUPPORTED = -2,
  E_CORRUPT = -3,
  E_CAPACITY = -4,
  E_TRUNCATED = -5,
};

constexpr int kFastBits = 11;

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

struct Huffman {
  bool present = false;
  uint8_t fast_len[1 << kFastBits];  // 0: code longer than kFastBits
  uint8_t fast_val[1 << kFastBits];
  // AC tables only: symbol + magnitude bits resolved in one lookup when both
  // fit in kFastBits: (value << 16) | (run << 8) | total bits; 0 = slow path
  int32_t fast_ac[1 << kFastBits];
  int32_t maxcode[18];  // largest code of each length, -1 if none
  int32_t valptr[17];   // index into vals of the first code of each length
  int32_t mincode[17];
  uint8_t vals[256];

  bool build(const uint8_t* counts, const uint8_t* symbols, int nsym) {
    if (nsym > 256) return false;
    std::memcpy(vals, symbols, nsym);
    std::memset(fast_len, 0, sizeof(fast_len));
    int code = 0, k = 0;
    for (int len = 1; len <= 16; ++len) {
      const int n = counts[len - 1];
      // over-subscribed table (a crafted DHT): reject before any fast-table write, whose
      // index (code << shift) | j must stay below 1 << kFastBits
      if (code + n > (1 << len) || k + n > nsym) return false;
      valptr[len] = k;
      mincode[len] = code;
      for (int i = 0; i < n; ++i, ++k, ++code) {
        if (len <= kFastBits) {
          const int shift = kFastBits - len;
          for (int j = 0; j < (1 << shift); ++j) {
            fast_len[(code << shift) | j] = uint8_t(len);
            fast_val[(code << shift) | j] = symbols[k];
          }
        }
      }
      maxcode[len] = n ? code - 1 : -1;
      code <<= 1;
    }
    maxcode[17] = 0x7fffffff;
    for (int i = 0; i < (1 << kFastBits); ++i) {
      fast_ac[i] = 0;
      const int len = fast_len[i];
      if (!len) continue;
      const int rs = fast_val[i], run = rs >> 4, sz = rs & 15;
      if (sz == 0 || len + sz > kFastBits) continue;  // EOB / ZRL / long: slow path
      const int bits = (i >> (kFastBits - len - sz)) & ((1 << sz) - 1);
      fast_ac[i] = int32_t(uint32_t(extend(bits, sz)) << 16) | (run << 8) | (len + sz);
    }
    present = true;
    return true;
  }
};

// MSB-first bit reader over the entropy-coded segment.  Byte stuffing
// (FF 00) is removed; on any other marker the reader stops consuming and
// feeds zero bits, leaving `pos` at the marker.
struct BitReader {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t acc = 0;
  int nbits = 0;
  int marker = 0;

  void fill() {
    // fast path: the next bytes hold no 0xFF (no stuffing, no marker): load them at once
    if (!marker && end - p >= 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      const int take = (63 - nbits) >> 3;  // whole bytes that fit
      const uint64_t mask = take >= 8 ? ~0ull : ((1ull << (8 * take)) - 1);
      const uint64_t x = ~w & mask;  // 0xFF bytes become 0x00
      const bool has_ff = ((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull & mask) != 0;
      if (!has_ff && take > 0) {
        const uint64_t be = __builtin_bswap64(w) >> (64 - 8 * take);  // first byte most significant
        acc |= be << (64 - nbits - 8 * take);
        nbits += 8 * take;
        p += take;
        return;
      }
    }
    while (nbits <= 56) {
      uint32_t b = 0;
      if (!marker) {
        if (p >= end) {
          marker = 0xD9;  // ran off the data: treat as EOI
        } else if (p[0] != 0xFF) {
          b = *p++;
        } else if (p + 1 < end && p[1] == 0x00) {
          b = 0xFF;
          p += 2;
        } else if (p + 1 < end && p[1] == 0xFF) {
          ++p;  // fill byte before a marker
          continue;
        } else {
          marker = p + 1 < end ? p[1] : 0xD9;
        }
      }
      acc |= uint64_t(b) << (56 - nbits);
      nbits += 8;
    }
  }
  uint32_t peek(int k) const { return uint32_t(acc >> (64 - k)); }
  void skip(int k) {
    acc <<= k;
    nbits -= k;
  }
  void reset() {
    acc = 0;
    nbits = 0;
  }

  int decode(const Huffman& h) {
    if (nbits < 16) fill();
    const uint32_t look = peek(kFastBits);
    if (const int len = h.fast_len[look]) {
      skip(len);
      return h.fast_val[look];
    }
    for (int len = kFastBits + 1; len <= 16; ++len) {
      const int32_t code = int32_t(peek(len));
      if (code <= h.maxcode[len]) {
        skip(len);
        const int idx = h.valptr[len] + code - h.mincode[len];
        return idx < 256 ? h.vals[idx] : -1;
      }
    }
    return -1;
  }
  // magnitude category s -> signed value (JPEG F.2.2.1 EXTEND)
  int receive_extend(int s) {
    if (s == 0) return 0;
    if (nbits < s) fill();
    const int v = int(peek(s));
    skip(s);
    return extend(v, s);
  }
};

struct Component {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int bw = 0, bh = 0;   // MCU-padded block grid
  int64_t offset = 0;   // first block of this component in the output
};

struct Frame {
  int width = 0, height = 0, nc = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
  int restart = 0;
  Component comp[3];
  uint16_t q[4][64];
  bool q_present[4] = {false, false, false, false};
  Huffman dc[4], ac[4];
  int64_t nblocks = 0;
  const uint8_t* scan = nullptr;  // first entropy-coded byte
  int scan_order[3] = {0, 1, 2};
  int ns = 0;
};

inline int be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// Parse every marker up to the (single) scan's entropy-coded data.
int parse(const uint8_t* data, int64_t len, Frame& f) {
  if (len < 4 || data[0] != 0xFF || data[1] != 0xD8) return E_NOT_JPEG;
  int64_t pos = 2;
  bool have_sof = false;
  while (pos + 4 <= len) {
    if (data[pos] != 0xFF) return E_CORRUPT;
    while (pos < len && data[pos] == 0xFF) ++pos;
    if (pos >= len) return E_TRUNCATED;
    const int m = data[pos++];
    if (m == 0xD9) return E_CORRUPT;  // EOI before any scan
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (pos + 2 > len) return E_TRUNCATED;
    const int seglen = be16(data + pos);
    if (seglen < 2 || pos + seglen > len) return E_TRUNCATED;
    const uint8_t* s = data + pos + 2;
    const int n = seglen - 2;
    switch (m) {
      case 0xDB: {  // DQT
        int i = 0;
        while (i < n) {
          const int pq = s[i] >> 4, tq = s[i] & 15;
          ++i;
          if (tq > 3 || i + 64 * (pq ? 2 : 1) > n) return E_CORRUPT;
          for (int k = 0; k < 64; ++k) {
            f.q[tq][kZigzag[k]] = pq ? uint16_t(be16(s + i + 2 * k)) : s[i + k];
          }
          i += 64 * (pq ? 2 : 1);
          f.q_present[tq] = true;
        }
        break;
      }
      case 0xC0:
      case 0xC1: {  // SOF0 / SOF1: sequential Huffman
        if (n < 6 || s[0] != 8) return E_UNSUPPORTED;
        f.height = be16(s + 1);
        f.width = be16(s + 3);
        f.nc = s[5];
        if (f.width <= 0 || f.height <= 0) return E_UNSUPPORTED;  // DNL height not supported
        if (!(f.nc == 1 || f.nc == 3) || n < 6 + 3 * f.nc) return E_UNSUPPORTED;
        for (int c = 0; c < f.nc; ++c) {
          Component& k = f.comp[c];
          k.id = s[6 + 3 * c];
          k.h = s[7 + 3 * c] >> 4;
          k.v = s[7 + 3 * c] & 15;
          k.tq = s[8 + 3 * c];
          if (k.h < 1 || k.h > 2 || k.v < 1 || k.v > 2 || k.tq > 3) return E_UNSUPPORTED;
          f.hmax = k.h > f.hmax ? k.h : f.hmax;
          f.vmax = k.v > f.vmax ? k.v : f.vmax;
        }
        if (f.nc == 1) {  // a single component is never interleaved: 8x8 MCUs
          f.comp[0].h = f.comp[0].v = f.hmax = f.vmax = 1;
        }
        f.mcux = (f.width + 8 * f.hmax - 1) / (8 * f.hmax);
        f.mcuy = (f.height + 8 * f.vmax - 1) / (8 * f.vmax);
        int64_t off = 0;
        for (int c = 0; c < f.nc; ++c) {
          Component& k = f.comp[c];
          k.bw = f.mcux * k.h;
          k.bh = f.mcuy * k.v;
          k.offset = off;
          off += int64_t(k.bw) * k.bh;
        }
        f.nblocks = off;
        have_sof = true;
        break;
      }
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
      case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        return E_UNSUPPORTED;  // progressive, lossless, hierarchical, arithmetic
      case 0xC4: {  // DHT
        int i = 0;
        while (i < n) {
          if (i + 17 > n) return E_CORRUPT;
          const int tc = s[i] >> 4, th = s[i] & 15;
          const uint8_t* counts = s + i + 1;
          int nsym = 0;
          for (int k = 0; k < 16; ++k) nsym += counts[k];
          if (tc > 1 || th > 3 || i + 17 + nsym > n) return E_CORRUPT;
          Huffman& h = tc ? f.ac[th] : f.dc[th];
          if (!h.build(counts, s + i + 17, nsym)) return E_CORRUPT;
          i += 17 + nsym;
        }
        break;
      }
      case 0xDD:  // DRI
        if (n < 2) return E_CORRUPT;
        f.restart = be16(s);
        break;
      case 0xDA: {  // SOS
        if (!have_sof) return E_CORRUPT;
        f.ns = s[0];
        if (f.ns != f.nc || n < 1 + 2 * f.ns + 3) return E_UNSUPPORTED;  // one interleaved scan only
        for (int j = 0; j < f.ns; ++j) {
          const int cid = s[1 + 2 * j];
          int c = 0;
          while (c < f.nc && f.comp[c].id != cid) ++c;
          if (c == f.nc) return E_CORRUPT;
          f.scan_order[j] = c;
          f.comp[c].td = s[2 + 2 * j] >> 4;
          f.comp[c].ta = s[2 + 2 * j] & 15;
          if (f.comp[c].td > 3 || f.comp[c].ta > 3) return E_CORRUPT;
          if (!f.dc[f.comp[c].td].present || !f.ac[f.comp[c].ta].present) return E_CORRUPT;
          if (!f.q_present[f.comp[c].tq]) return E_CORRUPT;
        }
        const int ss = s[1 + 2 * f.ns], se = s[2 + 2 * f.ns];
        if (ss != 0 || se != 63) return E_UNSUPPORTED;
        f.scan = s + n;
        return OK;
      }
      default:  // APPn, COM, ...: skip
        break;
    }
    pos += seglen;
  }
  return E_TRUNCATED;
}

// Decode one block into `blk` (zeroed here); returns false on corrupt data.
inline bool decode_block(BitReader& br, const Huffman& dc, const Huffman& ac, int& pred, int16_t* blk) {
  std::memset(blk, 0, 64 * sizeof(int16_t));
  if (br.nbits < 32) br.fill();
  const int t = br.decode(dc);
  if (t < 0 || t > 11) return false;
  pred += br.receive_extend(t);
  blk[0] = int16_t(pred);
  for (int k = 1; k < 64;) {
    if (br.nbits < 32) br.fill();
    const int32_t e = ac.fast_ac[br.peek(kFastBits)];
    if (e) {
      k += (e >> 8) & 15;
      if (k > 63) return false;
      blk[kZigzag[k]] = int16_t(e >> 16);
      br.skip(e & 255);
      ++k;
      continue;
    }
    const int rs = br.decode(ac);
    if (rs < 0) return false;
    const int r = rs >> 4, sz = rs & 15;
    if (sz == 0) {
      if (r != 15) break;  // EOB
      k += 16;             // ZRL
      continue;
    }
    k += r;
    if (k > 63) return false;
    blk[kZigzag[k]] = int16_t(br.receive_extend(sz));
    ++k;
  }
  return true;
}

int decode_scan(const uint8_t* data, int64_t len, const Frame& f, int16_t* coef) {
  BitReader br{f.scan, data + len};
  int pred[3] = {0, 0, 0};
  const int64_t nmcu = int64_t(f.mcux) * f.mcuy;
  int todo = f.restart;
  for (int64_t m = 0; m < nmcu; ++m) {
    if (f.restart && todo == 0) {
      // expect RSTn: drop the partial byte, step over the marker, reset predictors
      br.reset();
      if (br.marker >= 0xD0 && br.marker <= 0xD7) {
        br.p += 2;
        br.marker = 0;
      } else {  // lost sync: scan forward for the next RSTn
        while (br.p + 1 < br.end && !(br.p[0] == 0xFF && br.p[1] >= 0xD0 && br.p[1] <= 0xD7)) ++br.p;
        if (br.p + 1 >= br.end) return E_CORRUPT;
        br.p += 2;
        br.marker = 0;
      }
      pred[0] = pred[1] = pred[2] = 0;
      todo = f.restart;
    }
    const int mx = int(m % f.mcux), my = int(m / f.mcux);
    for (int j = 0; j < f.ns; ++j) {
      const int c = f.scan_order[j];
      const Component& k = f.comp[c];
      for (int v = 0; v < k.v; ++v) {
        for (int h = 0; h < k.h; ++h) {
          const int by = my * k.v + v, bx = mx * k.h + h;
          int16_t* blk = coef + (k.offset + int64_t(by) * k.bw + bx) * 64;
          if (!decode_block(br, f.dc[k.td], f.ac[k.ta], pred[c], blk)) return E_CORRUPT;
        }
      }
    }
    if (f.restart) --todo;
  }
  return OK;
}

void fill_geom(const Frame& f, int32_t* g) {
  std::memset(g, 0, 16 * sizeof(int32_t));
  g[0] = f.width;
  g[1] = f.height;
  g[2] = f.nc;
  g[3] = f.hmax;
  g[4] = f.vmax;
  g[5] = f.mcux;
  g[6] = f.mcuy;
  for (int c = 0; c < f.nc; ++c) {
    g[7 + 2 * c] = f.comp[c].h;
    g[8 + 2 * c] = f.comp[c].v;
  }
  g[13] = int32_t(f.nblocks);
}

int decode_one(const uint8_t* data, int64_t len, int16_t* coef, int64_t capacity_blocks, float* q, int32_t* geom) {
  Frame f;
  int rc = parse(data, len, f);
  if (rc != OK) return rc;
  fill_geom(f, geom);
  if (f.nblocks > capacity_blocks) return E_CAPACITY;
  for (int c = 0; c < 3; ++c) {
    const int t = f.comp[c < f.nc ? c : 0].tq;
    for (int k = 0; k < 64; ++k) q[c * 64 + k] = float(f.q[t][k]);
  }
  return decode_scan(data, len, f, coef);
}

}  // namespace

extern "C" {

// Header only: geometry of a JPEG (see the layout above).  0 or an error code.
int tca_jpeg_probe(const uint8_t* data, int64_t len, int32_t* geom) {
  Frame f;
  const int rc = parse(data, len, f);
  if (rc == OK) fill_geom(f, geom);
  return rc;
}

// One frame: coefficients into `coef` (room for `capacity_blocks` blocks).
int tca_jpeg_decode_coefs(const uint8_t* data, int64_t len, int16_t* coef, int64_t capacity_blocks, float* q,
                          int32_t* geom) {
  return decode_one(data, len, coef, capacity_blocks, q, geom);
}

// A batch on `nthreads` host threads: frame i goes to coef + i*stride_blocks*64,
// q + i*192, geom + i*16; status[i] = 0 or its error code.  Returns the number
// of frames that failed.
int tca_jpeg_decode_batch(const uint8_t* const* data, const int64_t* lens, int n, int16_t* coef,
                          int64_t stride_blocks, float* q, int32_t* geom, int32_t* status, int nthreads) {
  std::atomic<int> next{0};
  std::atomic<int> failed{0};
  auto work = [&]() {
    for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) {
      const int rc = decode_one(data[i], lens[i], coef + int64_t(i) * stride_blocks * 64, stride_blocks,
                                q + int64_t(i) * 192, geom + int64_t(i) * 16);
      status[i] = rc;
      if (rc != OK) failed.fetch_add(1);
    }
  };
  nthreads = nthreads < 1 ? 1 : (nthreads > n ? n : nthreads);
  std::vector<std::thread> pool;
  pool.reserve(nthreads > 0 ? nthreads - 1 : 0);
  for (int t = 1; t < nthreads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return failed.load();
}

}  // extern "C"
