// Sanitizer driver for the host JPEG entropy decoder and the host preprocess
// (csrc/runtime/jpeg_entropy.cpp, cpu_image.cpp): decode the given JPEG files,
// then feed truncated / byte-flipped variants (seeded) through the single and
// threaded batch entry points, and run the preprocess on random geometries.
// Built with -fsanitize=address,undefined (or thread) by tests/test_native_sanitizers.py.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

extern "C" {
int tca_jpeg_probe(const uint8_t* data, int64_t len, int32_t* geom);
int tca_jpeg_decode_coefs(const uint8_t* data, int64_t len, int16_t* coef, int64_t capacity_blocks, float* q,
                          int32_t* geom);
int tca_jpeg_decode_batch(const uint8_t* const* data, const int64_t* lens, int n, int16_t* coef,
                          int64_t stride_blocks, float* q, int32_t* geom, int32_t* status, int nthreads);
int tca_cpu_preprocess(const uint8_t* src, int h0, int w0, int c0, int swap_rb, float* out, int layout, int H, int W,
                       int top, int left, int nh, int nw, float pad, int quantize, const float* scale,
                       const float* bias, int nthreads);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: jpeg_fuzz <iterations> <file.jpg>...\n");
    return 2;
  }
  const int iters = std::atoi(argv[1]);
  std::vector<std::vector<uint8_t>> files;
  for (int i = 2; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    files.emplace_back(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  const int64_t cap = 1 << 14;  // blocks per frame slot
  std::vector<int16_t> coef(cap * 64 * 4);
  std::vector<float> q(192 * 4);
  std::vector<int32_t> geom(16 * 4), status(4);
  int ok = 0;
  for (auto& f : files) {
    int32_t g[16];
    if (tca_jpeg_probe(f.data(), (int64_t)f.size(), g) != 0) return 3;
    if (tca_jpeg_decode_coefs(f.data(), (int64_t)f.size(), coef.data(), cap, q.data(), geom.data()) != 0) return 4;
    ++ok;
  }
  // crafted over-subscribed DHT tables: every table of every file gets all its
  // symbols moved to code length 1 (counts[0] = nsym, the rest 0; the segment
  // length stays consistent) or 3 of them (counts[0] = 3).  Both must be rejected
  // before the fast lookup table is written.
  int crafted = 0;
  for (auto& f : files) {
    for (size_t p = 2; p + 4 < f.size(); ++p) {
      if (f[p] != 0xFF || f[p + 1] != 0xC4) continue;
      const size_t seg_end = p + 2 + ((size_t)f[p + 2] << 8 | f[p + 3]);
      for (size_t t = p + 4; t + 17 <= seg_end && t + 17 <= f.size();) {
        int nsym = 0;
        for (int l = 0; l < 16; ++l) nsym += f[t + 1 + l];
        for (int variant = 0; variant < 2; ++variant) {
          if (variant == 1 && nsym < 4) continue;
          std::vector<uint8_t> v = f;
          if (variant == 0) {
            for (int l = 0; l < 16; ++l) v[t + 1 + l] = 0;
            v[t + 1] = (uint8_t)nsym;
          } else {
            // 3 codes of length 1, the remaining symbols at the longest used length
            int last = 15;
            while (last > 0 && f[t + 1 + last] == 0) --last;
            for (int l = 0; l < 16; ++l) v[t + 1 + l] = 0;
            v[t + 1] = 3;
            v[t + 1 + last] = (uint8_t)(nsym - 3);
          }
          int32_t g[16];
          if (tca_jpeg_probe(v.data(), (int64_t)v.size(), g) == 0) return 5;
          if (tca_jpeg_decode_coefs(v.data(), (int64_t)v.size(), coef.data(), cap, q.data(), geom.data()) == 0)
            return 6;
          ++crafted;
        }
        t += 17 + nsym;
      }
    }
  }
  if (crafted == 0) return 7;
  std::mt19937 rng(1234);
  int rejected = 0;
  for (int it = 0; it < iters; ++it) {
    std::vector<std::vector<uint8_t>> batch;
    for (int b = 0; b < 4; ++b) {
      std::vector<uint8_t> v = files[rng() % files.size()];
      if (rng() & 1) v.resize(2 + rng() % (v.size() - 2));
      const int flips = rng() % 8;
      for (int k = 0; k < flips; ++k) v[rng() % v.size()] = (uint8_t)rng();
      batch.push_back(std::move(v));
    }
    const uint8_t* ptrs[4];
    int64_t lens[4];
    for (int b = 0; b < 4; ++b) {
      ptrs[b] = batch[b].data();
      lens[b] = (int64_t)batch[b].size();
    }
    rejected += tca_jpeg_decode_batch(ptrs, lens, 4, coef.data(), cap, q.data(), geom.data(), status.data(), 3);
  }
  // preprocess on random geometries (letterbox regions inside the destination)
  std::vector<uint8_t> img(97 * 131 * 4);
  for (auto& p : img) p = (uint8_t)rng();
  std::vector<float> out(3 * 80 * 96);
  const float sc[3] = {1 / 255.f, 1 / 255.f, 1 / 255.f}, bi[3] = {0, 0, 0};
  for (int it = 0; it < 200; ++it) {
    const int h0 = 1 + rng() % 97, w0 = 1 + rng() % 131, c0 = 3 + rng() % 2;
    const int H = 1 + rng() % 80, W = 1 + rng() % 96;
    const int nh = 1 + rng() % H, nw = 1 + rng() % W;
    const int top = rng() % (H - nh + 1), left = rng() % (W - nw + 1);
    tca_cpu_preprocess(img.data(), h0, w0, c0, rng() & 1, out.data(), rng() & 1, H, W, top, left, nh, nw, 114.f,
                       rng() & 1, sc, bi, 1 + rng() % 3);
  }
  std::printf("jpeg fuzz ok: %d files, %d crafted DHT tables rejected, %d iterations, %d corrupt frames rejected\n",
              ok, crafted, iters, rejected);
  return 0;
}
