// Host-side fuzz / round-trip driver for the KServe wire codec, built with
// -fsanitize=address,undefined by tests/test_native_sanitizers.py (SURVEY §5.2:
// sanitizers on the host code; GPU ASan is not available on this pool).
//
//   1. round trip: random requests encoded by tca_kserve_encode_request, then
//      re-read as a *response-shaped* message (same field layout for names /
//      datatypes / shapes when fields 5/7 are renumbered) — checks every offset
//      the parser returns lies inside the buffer;
//   2. mutation fuzz: random byte flips / truncations / length-prefix inflation
//      of valid responses must return 0, -1 or -2 without touching memory
//      outside the buffer (ASan aborts the process if they do).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

extern "C" {
long tca_kserve_request_size(const char*, const char*, const char*, int, const char**, const char**, const int64_t*,
                             const int*, const long*, int, const char**);
long tca_kserve_encode_request(const char*, const char*, const char*, int, const char**, const char**,
                               const int64_t*, const int*, const void**, const long*, int, const char**, uint8_t*,
                               long);
int tca_kserve_parse_response(const uint8_t*, long, int, long*, int64_t*, int, long*, long*);
}

static void put_varint(std::vector<uint8_t>& b, uint64_t v) {
  while (v >= 0x80) { b.push_back((uint8_t)(v | 0x80)); v >>= 7; }
  b.push_back((uint8_t)v);
}
static void put_bytes(std::vector<uint8_t>& b, int field, const void* d, size_t n) {
  put_varint(b, ((uint64_t)field << 3) | 2);
  put_varint(b, n);
  const uint8_t* p = (const uint8_t*)d;
  b.insert(b.end(), p, p + n);
}

// A ModelInferResponse: 1 model_name, 5 outputs{1 name, 2 datatype, 3 shape}, 6 raw contents.
static std::vector<uint8_t> make_response(std::mt19937& rng) {
  std::vector<uint8_t> b;
  put_bytes(b, 1, "model", 5);
  const int n = 1 + rng() % 4;
  std::vector<std::vector<uint8_t>> raws;
  for (int i = 0; i < n; ++i) {
    std::vector<uint8_t> t;
    std::string name = "out" + std::to_string(i);
    put_bytes(t, 1, name.data(), name.size());
    put_bytes(t, 2, "FP32", 4);
    std::vector<uint8_t> sh;
    const int nd = rng() % 4;
    size_t elems = 1;
    for (int d = 0; d < nd; ++d) { const int v = 1 + rng() % 7; elems *= v; put_varint(sh, v); }
    if (nd) put_bytes(t, 3, sh.data(), sh.size());
    put_bytes(b, 5, t.data(), t.size());
    raws.emplace_back(elems * 4, (uint8_t)i);
  }
  for (auto& r : raws) put_bytes(b, 6, r.data(), r.size());
  return b;
}

static int check(const std::vector<uint8_t>& buf, bool expect_ok) {
  // parse from an exact-size heap copy so any over-read hits ASan's redzone
  uint8_t* p = (uint8_t*)malloc(buf.size() ? buf.size() : 1);
  if (!buf.empty()) memcpy(p, buf.data(), buf.size());
  long meta[8 * 8], raw[8 * 2], counts[4];
  int64_t shapes[32];
  const int rc = tca_kserve_parse_response(p, (long)buf.size(), 8, meta, shapes, 32, raw, counts);
  if (rc == 0) {
    const long n = (long)buf.size();
    for (int k = 0; k < counts[0]; ++k) {
      const long* m = meta + 8 * k;
      if (m[0] < 0 || m[0] + m[1] > n || m[2] < 0 || m[2] + m[3] > n) { free(p); return 10; }
    }
    for (int k = 0; k < counts[1]; ++k)
      if (raw[2 * k] < 0 || raw[2 * k] + raw[2 * k + 1] > n) { free(p); return 11; }
    if (counts[2] < 0 || counts[2] + counts[3] > n) { free(p); return 12; }
  }
  free(p);
  if (expect_ok && rc != 0) return 13;
  if (rc != 0 && rc != -1 && rc != -2) return 14;
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937 rng(1234);
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> b = make_response(rng);
    if (int e = check(b, true)) { fprintf(stderr, "valid response failed: %d (iter %d)\n", e, it); return e; }
    // mutations
    std::vector<uint8_t> m = b;
    switch (rng() % 4) {
      case 0: m.resize(rng() % (m.size() + 1)); break;                               // truncate
      case 1: for (int k = 0; k < 4; ++k) m[rng() % m.size()] ^= (uint8_t)(1u << (rng() % 8)); break;  // bit flips
      case 2: m[rng() % m.size()] = 0xff; break;                                       // inflate a length / varint
      case 3: { size_t at = rng() % m.size(); m.insert(m.begin() + at, 0x80 | (rng() & 0x7f)); } break;
    }
    if (int e = check(m, false)) { fprintf(stderr, "mutated response: %d (iter %d)\n", e, it); return e; }
  }
  // encoder: size query == bytes written, tiny caps refused
  for (int it = 0; it < 2000; ++it) {
    const int n_in = 1 + rng() % 3;
    std::vector<std::string> names, dts;
    std::vector<const char*> np, dp;
    std::vector<int64_t> shapes;
    std::vector<int> nds;
    std::vector<std::vector<uint8_t>> data;
    std::vector<const void*> ptrs;
    std::vector<long> nbytes;
    for (int i = 0; i < n_in; ++i) {
      names.push_back("in" + std::to_string(i));
      dts.push_back("FP32");
      const int nd = 1 + rng() % 3;
      nds.push_back(nd);
      long e = 1;
      for (int d = 0; d < nd; ++d) { const int v = 1 + rng() % 300; shapes.push_back(v); e *= v; }
      data.emplace_back(e * 4, 7);
      nbytes.push_back(e * 4);
    }
    for (int i = 0; i < n_in; ++i) { np.push_back(names[i].c_str()); dp.push_back(dts[i].c_str()); ptrs.push_back(data[i].data()); }
    const char* outs[2] = {"o1", "o2"};
    const long need = tca_kserve_request_size("m", "1", "id", n_in, np.data(), dp.data(), shapes.data(), nds.data(),
                                              nbytes.data(), 2, outs);
    std::vector<uint8_t> buf(need);
    const long w = tca_kserve_encode_request("m", "1", "id", n_in, np.data(), dp.data(), shapes.data(), nds.data(),
                                             ptrs.data(), nbytes.data(), 2, outs, buf.data(), need);
    if (w != need) { fprintf(stderr, "encode size mismatch %ld != %ld\n", w, need); return 20; }
    if (tca_kserve_encode_request("m", "1", "id", n_in, np.data(), dp.data(), shapes.data(), nds.data(), ptrs.data(),
                                  nbytes.data(), 2, outs, buf.data(), need - 1) != -need) return 21;
  }
  printf("wire fuzz ok\n");
  return 0;
}
