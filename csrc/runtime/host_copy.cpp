// Host staging copies for the live drivers: a batch of sensor payloads
// (PointCloud2 data, raw Image rows) gathered into one pinned slot.
//
// Reference: the per-message path turns each payload into Python objects
// (point_cloud2.read_points, ros_inference3d.py:125; cv_bridge,
// ros_inference.py:131).  Here a batch of payloads is copied, as bytes, into
// the pinned slot the H2D DMA reads — split into ~1 MiB chunks over a few
// std::threads so one batch (32 x 1.9 MB clouds) is not one core's memcpy,
// and called through ctypes, i.e. without the GIL.
//
// Large pieces are copied with non-temporal (streaming) stores: the destination is
// a page-locked staging slot that only the DMA engine reads next, so filling the CPU
// caches with it (and reading every destination line first, the write-allocate of an
// ordinary store) only costs memory bandwidth -- the budget rank 0 spends feeding the
// node's GPUs through the shared host ring (tools/fanout_bench.py).  TCA_HOST_COPY_NT=0
// turns it off (plain memcpy) for A/B runs.
#if defined(__x86_64__) || defined(__i386__)
#include <immintrin.h>
#define TCA_HAVE_NT_COPY 1
#else
#define TCA_HAVE_NT_COPY 0  // other hosts: plain memcpy
#endif

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define TCA_API extern "C" __attribute__((visibility("default")))

namespace {
constexpr int64_t kChunk = 1 << 20;
constexpr int64_t kStreamMin = 64 << 10;  // pieces below this keep memcpy

#if TCA_HAVE_NT_COPY
__attribute__((target("avx2"))) void copy_stream(char* d, const char* s, int64_t n) {
  int64_t head = (int64_t)((32 - ((uintptr_t)d & 31)) & 31);
  if (head > n) head = n;
  std::memcpy(d, s, (size_t)head);
  d += head;
  s += head;
  n -= head;
  const int64_t body = n & ~(int64_t)127;
  for (int64_t i = 0; i < body; i += 128) {
    const __m256i a0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i a1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i a2 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i a3 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a0);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), a1);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), a2);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), a3);
  }
  std::memcpy(d + body, s + body, (size_t)(n - body));
}

void store_fence() { _mm_sfence(); }

bool use_stream() {
  static const bool on = [] {
    const char* e = std::getenv("TCA_HOST_COPY_NT");
    return !(e && e[0] == '0') && __builtin_cpu_supports("avx2");
  }();
  return on;
}
#else
void copy_stream(char* d, const char* s, int64_t n) { std::memcpy(d, s, (size_t)n); }
void store_fence() {}
bool use_stream() { return false; }
#endif
}  // namespace

// n copies dst[i] <- src[i] of nbytes[i]; returns 0, or -1 on a bad argument.
TCA_API int tca_host_gather_copy(int n, void* const* dst, const void* const* src, const int64_t* nbytes,
                                 int nthreads) {
  if (n < 0 || (n > 0 && (!dst || !src || !nbytes))) return -1;
  struct Piece {
    char* d;
    const char* s;
    int64_t len;
  };
  std::vector<Piece> pieces;
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (nbytes[i] < 0 || (nbytes[i] > 0 && (!dst[i] || !src[i]))) return -1;
    for (int64_t o = 0; o < nbytes[i]; o += kChunk)
      pieces.push_back({(char*)dst[i] + o, (const char*)src[i] + o, std::min(kChunk, nbytes[i] - o)});
    total += nbytes[i];
  }
  const int t = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::max(nthreads, 1),
                                                              (int64_t)pieces.size(), total / (4 * kChunk) + 1}));
  std::atomic<size_t> next{0};
  const bool nt = use_stream();
  auto work = [&] {
    bool streamed = false;
    for (size_t k; (k = next.fetch_add(1)) < pieces.size();) {
      if (nt && pieces[k].len >= kStreamMin) {
        copy_stream(pieces[k].d, pieces[k].s, pieces[k].len);
        streamed = true;
      } else {
        std::memcpy(pieces[k].d, pieces[k].s, pieces[k].len);
      }
    }
    if (streamed) store_fence();  // this thread's streaming stores are globally visible before it joins
  };
  std::vector<std::thread> pool;
  pool.reserve(t - 1);
  for (int i = 1; i < t; ++i) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}
