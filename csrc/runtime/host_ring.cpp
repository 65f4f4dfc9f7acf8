// Cross-process signalling for the node's shared host ring (parallel/host_ring.py).
//
// The data-parallel drivers run one process per GPU.  Rank 0 (the ROS
// subscriber) writes each node batch into a slot of a POSIX shared-memory
// ring and publishes the slot's sequence number; every rank then DMAs its own
// shard out of the ring over its own PCIe link and acknowledges.  This file
// is the part Python cannot do safely: 32-bit sequence words in the shared
// mapping with release/acquire ordering (payload writes become visible before
// the sequence number that announces them) and futex sleep/wake on them, so
// an idle rank blocks in the kernel instead of polling, and a wait releases
// the GIL (ctypes).
//
// Sequence comparisons are wrap-safe: a word "has reached" v when
// (int32_t)(word - v) >= 0.
#include <linux/futex.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>

#define TCA_API extern "C" __attribute__((visibility("default")))

namespace {

inline std::atomic<uint32_t>* word(void* p) { return reinterpret_cast<std::atomic<uint32_t>*>(p); }

inline bool reached(uint32_t w, uint32_t v) { return (int32_t)(w - v) >= 0; }

long futex(void* addr, int op, uint32_t val, const timespec* ts) {
  // shared (not FUTEX_PRIVATE): the word lives in a mapping of several processes
  return syscall(SYS_futex, addr, op, val, ts, nullptr, 0);
}

int64_t now_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000000000LL + t.tv_nsec;
}

// Wait until *p has reached v; 0 = reached, 1 = timed out (timeout_ms < 0: forever).
int wait_word(void* p, uint32_t v, int64_t timeout_ms) {
  auto* w = word(p);
  const int64_t end = timeout_ms < 0 ? INT64_MAX : now_ns() + timeout_ms * 1000000LL;
  for (int spin = 0; spin < 2000; ++spin) {  // a few us of spinning for the common short wait
    if (reached(w->load(std::memory_order_acquire), v)) return 0;
  }
  for (;;) {
    const uint32_t cur = w->load(std::memory_order_acquire);
    if (reached(cur, v)) return 0;
    const int64_t left = end - now_ns();
    if (left <= 0) return 1;
    const int64_t slice = left < 50000000LL ? left : 50000000LL;  // re-check at least every 50 ms
    timespec ts{(time_t)(slice / 1000000000LL), (long)(slice % 1000000000LL)};
    futex(p, FUTEX_WAIT, cur, &ts);  // returns on wake, value change (EAGAIN), timeout or signal
  }
}

}  // namespace

// *p = v (release), then wake every waiter on p.
TCA_API int tca_ring_publish(void* p, uint32_t v) {
  if (!p || ((uintptr_t)p & 3)) return -1;
  word(p)->store(v, std::memory_order_release);
  futex(p, FUTEX_WAKE, 0x7fffffff, nullptr);
  return 0;
}

// Acquire-load of a sequence word.
TCA_API uint32_t tca_ring_load(void* p) { return word(p)->load(std::memory_order_acquire); }

// Block until *p has reached v.  0: reached, 1: timed out, -1: bad argument.
TCA_API int tca_ring_wait(void* p, uint32_t v, int64_t timeout_ms) {
  if (!p || ((uintptr_t)p & 3)) return -1;
  return wait_word(p, v, timeout_ms);
}

// Block until every word base[i * stride_words] with bit i of mask set has
// reached v (the ranks' acknowledgements of one slot).  Returns 0, 1 on
// timeout (then *missing gets the mask of the words that had not), -1.
TCA_API int tca_ring_wait_all(void* base, int stride_words, uint64_t mask, uint32_t v, int64_t timeout_ms,
                              uint64_t* missing) {
  if (!base || ((uintptr_t)base & 3) || stride_words <= 0) return -1;
  const int64_t end = timeout_ms < 0 ? INT64_MAX : now_ns() + timeout_ms * 1000000LL;
  for (int i = 0; i < 64; ++i) {
    if (!((mask >> i) & 1)) continue;
    void* p = (uint32_t*)base + (int64_t)i * stride_words;
    const int64_t left = timeout_ms < 0 ? -1 : (end - now_ns()) / 1000000LL;
    if (timeout_ms >= 0 && left < 0) {
      if (!reached(word(p)->load(std::memory_order_acquire), v)) goto timed_out;
      continue;
    }
    if (wait_word(p, v, left) != 0) goto timed_out;
  }
  if (missing) *missing = 0;
  return 0;
timed_out:
  if (missing) {
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i)
      if (((mask >> i) & 1) && !reached(word((uint32_t*)base + (int64_t)i * stride_words)->load(), v))
        m |= 1ULL << i;
    *missing = m;
  }
  return 1;
}
