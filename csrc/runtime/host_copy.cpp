// Host staging copies for the live drivers: a batch of sensor payloads
// (PointCloud2 data, raw Image rows) gathered into one pinned slot.
//
// Reference: the per-message path turns each payload into Python objects
// (point_cloud2.read_points, ros_inference3d.py:125; cv_bridge,
// ros_inference.py:131).  Here a batch of payloads is copied, as bytes, into
// the pinned slot the H2D DMA reads — split into ~1 MiB chunks over a few
// std::threads so one batch (32 x 1.9 MB clouds) is not one core's memcpy,
// and called through ctypes, i.e. without the GIL.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#define TCA_API extern "C" __attribute__((visibility("default")))

namespace {
constexpr int64_t kChunk = 1 << 20;
}

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
  auto work = [&] {
    for (size_t k; (k = next.fetch_add(1)) < pieces.size();) std::memcpy(pieces[k].d, pieces[k].s, pieces[k].len);
  };
  std::vector<std::thread> pool;
  pool.reserve(t - 1);
  for (int i = 1; i < t; ++i) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return 0;
}
