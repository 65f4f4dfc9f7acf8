// Served-path helpers.  Batched device-to-device copies: the request tensors of a
// dynamic batch (device shared-memory slots of several client processes, mapped
// by HIP IPC handle) into the plan's input buffers, and the outputs back into the
// clients' slots, as ONE kernel launch.  hipMemcpy on an IPC-mapped pointer takes
// the peer path (an SDMA engine at PCIe-class rates: 86 MB of YOLO outputs in
// 2.3 ms, profiles/r3/served); this is a plain vector load/store kernel at HBM rate.
#include "tca_common.h"

namespace {

constexpr int kMaxSeg = 64;
constexpr int kChunk = 64 * 1024;  // bytes per workgroup

struct Segs {
  const unsigned char* src[kMaxSeg];
  unsigned char* dst[kMaxSeg];
  long nbytes[kMaxSeg];
};

__global__ void __launch_bounds__(256) copy_segments_kernel(Segs s) {
  const int g = blockIdx.y;
  const long n = s.nbytes[g];
  const long base = (long)blockIdx.x * kChunk;
  if (base >= n) return;
  const long end = base + kChunk < n ? base + kChunk : n;
  const unsigned char* src = s.src[g];
  unsigned char* dst = s.dst[g];
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  if (vec) {
    const long v_end = base + ((end - base) & ~15L);
    for (long o = base + threadIdx.x * 16; o < v_end; o += 256 * 16)
      *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(src + o);
    for (long o = v_end + threadIdx.x; o < end; o += 256) dst[o] = src[o];
  } else {
    for (long o = base + threadIdx.x; o < end; o += 256) dst[o] = src[o];
  }
}

}  // namespace

// n segments: dst[i] <- src[i], nbytes[i] bytes (device pointers, same device; any
// alignment).  Segments of zero bytes are skipped.
TCA_API int tca_copy_segments(int n, void* const* dst, const void* const* src, const long* nbytes,
                              hipStream_t stream) {
  for (int s0 = 0; s0 < n; s0 += kMaxSeg) {
    Segs s;
    const int k = n - s0 < kMaxSeg ? n - s0 : kMaxSeg;
    long mx = 0;
    for (int i = 0; i < kMaxSeg; ++i) {
      const bool on = i < k;
      s.src[i] = on ? static_cast<const unsigned char*>(src[s0 + i]) : nullptr;
      s.dst[i] = on ? static_cast<unsigned char*>(dst[s0 + i]) : nullptr;
      s.nbytes[i] = on ? nbytes[s0 + i] : 0;
      if (s.nbytes[i] < 0) return (int)hipErrorInvalidValue;
      mx = s.nbytes[i] > mx ? s.nbytes[i] : mx;
    }
    if (mx == 0) continue;
    const long gx = (mx + kChunk - 1) / kChunk;
    if (gx > 0x7fffffffL) return (int)hipErrorInvalidValue;
    copy_segments_kernel<<<dim3((unsigned)gx, (unsigned)k), 256, 0, stream>>>(s);
  }
  TCA_LAUNCH_CHECK();
}

// ---- served PointPillars: range check of the received voxel coordinates / counts of a
// dynamic batch, on the device, after they were copied into the plan's buffers and before
// its graph runs.  Slot b (rows < vcount[b]) is bad when a (z, y, x) cell lies outside
// the grid or a point count outside [1, P]: its vcount is zeroed (the graph then scatters
// nothing for it: no out-of-range canvas write) and flags[b] = 1 (host-visible; the server
// answers that request INVALID_ARGUMENT after the batch), else flags[b] = 0.
namespace {

__global__ void __launch_bounds__(256) voxel_check_kernel(const int* __restrict__ coords,
                                                          const int* __restrict__ nump, int* __restrict__ vcount,
                                                          int V, int P, int nz, int ny, int nx,
                                                          int* __restrict__ flags) {
  __shared__ int bad;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const int n = min(vcount[b], V);
  int my = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int4 c = *reinterpret_cast<const int4*>(coords + ((long)b * V + i) * 4);
    const int k = nump[(long)b * V + i];
    my |= (unsigned)c.y >= (unsigned)nz || (unsigned)c.z >= (unsigned)ny || (unsigned)c.w >= (unsigned)nx ||
          k < 1 || k > P;
  }
  if (my) atomicOr(&bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    flags[b] = bad;
    if (bad) vcount[b] = 0;
  }
}

}  // namespace

// coords int32 [B, V, 4] (b, z, y, x), nump int32 [B, V], vcount int32 [B] (device);
// flags int32 [B] (device or pinned host).
TCA_API int tca_voxel_check(const int* coords, const int* nump, int* vcount, int B, int V, int P, int nz, int ny,
                            int nx, int* flags, hipStream_t stream) {
  if (B <= 0) return 0;
  if (V < 0 || P < 1) return (int)hipErrorInvalidValue;
  voxel_check_kernel<<<B, 256, 0, stream>>>(coords, nump, vcount, V, P, nz, ny, nx, flags);
  TCA_LAUNCH_CHECK();
}
