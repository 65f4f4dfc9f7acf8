// K6 — PointCloud2 unpack (reference: communicator/ros_inference3d.py:125-128 —
// `np.array(list(point_cloud2.read_points(msg, ("x","y","z","intensity"), skip_nans=True)))`,
// then intensity /= max(intensity) and z += 1.5).  In the reference this
// per-point Python loop costs 138 ms for a 120k-point cloud.
//
// Batched over B clouds that share one field layout (one sensor).  Raw
// PointCloud2 bytes are read in place (per-frame byte offset + point count
// in device arrays).  Two launches:
//   pass 1: per 1024-point block — count NaN-free points, block max of
//           intensity (LDS reduce) -> one atomicMax per block on an
//           order-preserving uint encoding of the float;
//   pass 2: per block — prefix of the earlier blocks' counts of the same frame
//           (a wave-strided sum; <= a few hundred ints), in-block ordered
//           compaction with a block scan, intensity scaling and z offset.
// Output order == input order (skip_nans semantics).
#include <cstdlib>

#include "tca_common.h"

using namespace tca;

namespace {

constexpr int kPtsPerThread = 4;
constexpr int kBlock = 256;
constexpr int kPtsPerBlock = kPtsPerThread * kBlock;

struct FieldDesc {
  int off[4];    // byte offset of x, y, z, intensity inside a point record
  int dtype[4];  // sensor_msgs/PointField datatype codes (1..8)
  // 1: every field float32 at a 4-B aligned offset and step % 4 == 0 (dword loads, not byte loads);
  // 2: in addition x, y, z, intensity are the 16 B at offsets 0 / 4 / 8 / 12 and step % 16 == 0 (one
  // 16-B load per point: the Ouster / Velodyne xyzi record).  The frame's byte offset must be as
  // aligned, checked per block.
  int fast;
};

__device__ __forceinline__ float load_field(const uint8_t* rec, int off, int dt) {
  const uint8_t* p = rec + off;
  switch (dt) {
    case 1: return (float)*(const int8_t*)p;
    case 2: return (float)*(const uint8_t*)p;
    case 3: { int16_t v; __builtin_memcpy(&v, p, 2); return (float)v; }
    case 4: { uint16_t v; __builtin_memcpy(&v, p, 2); return (float)v; }
    case 5: { int32_t v; __builtin_memcpy(&v, p, 4); return (float)v; }
    case 6: { uint32_t v; __builtin_memcpy(&v, p, 4); return (float)v; }
    case 8: { double v; __builtin_memcpy(&v, p, 8); return (float)v; }
    default: { float v; __builtin_memcpy(&v, p, 4); return v; }
  }
}

typedef float nt_f4 __attribute__((ext_vector_type(4)));

// NT: the payload's last read (pc2_compact, TCA_VOX_NT=1) as a non-temporal load, so the streamed
// records do not displace the L2 lines of the BEV convs running beside the front
template <bool NT = false>
__device__ __forceinline__ bool load_point(const uint8_t* base, int i, int step, const FieldDesc& fd, float* v,
                                           int fast) {
  const uint8_t* rec = base + (long)i * step;
  if (fast == 2) {
    const nt_f4 q = NT ? __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(rec))
                       : *reinterpret_cast<const nt_f4*>(rec);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else if (fast == 1) {
#pragma unroll
    for (int f = 0; f < 4; ++f) v[f] = *reinterpret_cast<const float*>(rec + fd.off[f]);
  } else {
#pragma unroll
    for (int f = 0; f < 4; ++f) v[f] = load_field(rec, fd.off[f], fd.dtype[f]);
  }
  return !(isnan(v[0]) || isnan(v[1]) || isnan(v[2]) || isnan(v[3]));
}

// the fast path this frame can take: its byte offset must keep the records aligned
__device__ __forceinline__ int frame_fast(const FieldDesc& fd, long off) {
  if (fd.fast == 2 && (off & 15) == 0) return 2;
  if (fd.fast >= 1 && (off & 3) == 0) return 1;
  return 0;
}

__global__ void __launch_bounds__(kBlock) pc2_count_kernel(const uint8_t* __restrict__ data,
                                                           const long* __restrict__ frame_off,
                                                           const int* __restrict__ frame_n, int step, FieldDesc fd,
                                                           int blocks_per_frame, int* __restrict__ block_count,
                                                           uint32_t* __restrict__ frame_imax) {
  __shared__ int s_cnt[kBlock / 64];
  __shared__ float s_max[kBlock / 64];
  const int b = blockIdx.y, blk = blockIdx.x;
  const int n = frame_n[b];
  const uint8_t* base = data + frame_off[b];
  const int fast = frame_fast(fd, frame_off[b]);
  int cnt = 0;
  float mx = -INFINITY;
  // consecutive lanes read consecutive points (coalesced): point i = first + k * kBlock
  const int first = blk * kPtsPerBlock + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kPtsPerThread; ++k) {
    const int i = first + k * kBlock;
    if (i < n) {
      float v[4];
      if (load_point(base, i, step, fd, v, fast)) { ++cnt; mx = fmaxf(mx, v[3]); }
    }
  }
  cnt = wave_sum(cnt);
  mx = wave_maxf(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { s_cnt[w] = cnt; s_max[w] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0;
    float m = -INFINITY;
    for (int k = 0; k < kBlock / 64; ++k) { c += s_cnt[k]; m = fmaxf(m, s_max[k]); }
    block_count[b * blocks_per_frame + blk] = c;
    if (c > 0) atomicMax(&frame_imax[b], float_to_ordered(m));
  }
}

template <bool NT>
__global__ void __launch_bounds__(kBlock) pc2_compact_kernel(const uint8_t* __restrict__ data,
                                                             const long* __restrict__ frame_off,
                                                             const int* __restrict__ frame_n, int step, FieldDesc fd,
                                                             int blocks_per_frame, const int* __restrict__ block_count,
                                                             const uint32_t* __restrict__ frame_imax, int normalize,
                                                             float z_offset, float* __restrict__ out, int out_stride,
                                                             int max_points, int* __restrict__ out_count) {
  __shared__ int s_scan[kBlock / 64 + 1];
  __shared__ int s_prefix;
  const int b = blockIdx.y, blk = blockIdx.x;
  const int n = frame_n[b];
  const uint8_t* base = data + frame_off[b];
  // prefix over earlier blocks (first wave)
  if (threadIdx.x < 64) {
    int acc = 0;
    for (int k = threadIdx.x; k < blk; k += 64) acc += block_count[b * blocks_per_frame + k];
    acc = wave_sum(acc);
    if (threadIdx.x == 0) s_prefix = acc;
    if (blk == blocks_per_frame - 1) {  // last block publishes the frame's total
      int tot = 0;
      for (int k = threadIdx.x; k < blocks_per_frame; k += 64) tot += block_count[b * blocks_per_frame + k];
      tot = wave_sum(tot);
      if (threadIdx.x == 0) out_count[b] = min(tot, max_points);
    }
  }
  float inv = 1.f;
  if (normalize) {
    const float m = ordered_to_float(frame_imax[b]);
    inv = (m > 0.f && !isinf(m)) ? 1.f / m : 1.f;
  }
  float v[kPtsPerThread][4];
  bool ok[kPtsPerThread];
  int cnt = 0;
  const int fast = frame_fast(fd, frame_off[b]);
  const int first = blk * kPtsPerBlock + threadIdx.x * kPtsPerThread;
#pragma unroll
  for (int k = 0; k < kPtsPerThread; ++k) {
    const int i = first + k;
    ok[k] = i < n && load_point<NT>(base, i, step, fd, v[k], fast);
    cnt += ok[k];
  }
  int total;
  int pos = block_excl_scan(cnt, s_scan, &total);
  pos += s_prefix;
  float* ob = out + (long)b * max_points * out_stride;
#pragma unroll
  for (int k = 0; k < kPtsPerThread; ++k) {
    if (!ok[k]) continue;
    if (pos < max_points) {
      float* o = ob + (long)pos * out_stride;
      if (out_stride == 4) {  // one 16-B store
        *reinterpret_cast<float4*>(o) = make_float4(v[k][0], v[k][1], v[k][2] + z_offset, v[k][3] * inv);
      } else {
        o[0] = v[k][0];
        o[1] = v[k][1];
        o[2] = v[k][2] + z_offset;
        o[3] = v[k][3] * inv;
        for (int f = 4; f < out_stride; ++f) o[f] = 0.f;  // e.g. zero time-lag column (voxelize.py:38-39)
      }
    }
    ++pos;
  }
}

}  // namespace

// data: device bytes; frame_off/frame_n: device [B]; offsets/dtypes host [4].
// work: block_count int[B*blocks_per_frame], frame_imax uint[B].
TCA_API int tca_pc2_unpack(const void* data, const long* frame_off, const int* frame_n, int batch, int max_points,
                           int point_step, const int* field_off, const int* field_dtype, int normalize_intensity,
                           float z_offset, float* out, int out_stride, int* out_count, int* block_count,
                           uint32_t* frame_imax, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (out_stride < 4) return (int)hipErrorInvalidValue;
  FieldDesc fd;
  bool f32 = (point_step & 3) == 0;
  for (int f = 0; f < 4; ++f) {
    fd.off[f] = field_off[f];
    fd.dtype[f] = field_dtype[f];
    f32 = f32 && field_dtype[f] == 7 && (field_off[f] & 3) == 0 && field_off[f] + 4 <= point_step;
  }
  fd.fast = !f32 ? 0
            : (field_off[0] == 0 && field_off[1] == 4 && field_off[2] == 8 && field_off[3] == 12 &&
               (point_step & 15) == 0) ? 2 : 1;
  if (((uintptr_t)out & 15) != 0 && out_stride == 4) return (int)hipErrorInvalidValue;  // 16-B stores
  const int bpf = (max_points + kPtsPerBlock - 1) / kPtsPerBlock;
  int e = zero_i32_async((int*)frame_imax, batch, stream);
  if (e) return e;
  dim3 grid(bpf, batch);
  const uint8_t* d = (const uint8_t*)data;
  pc2_count_kernel<<<grid, kBlock, 0, stream>>>(d, frame_off, frame_n, point_step, fd, bpf, block_count, frame_imax);
  static const bool nt = getenv("TCA_VOX_NT") && atoi(getenv("TCA_VOX_NT")) != 0;
  (nt ? pc2_compact_kernel<true> : pc2_compact_kernel<false>)<<<grid, kBlock, 0, stream>>>(d, frame_off, frame_n, point_step, fd, bpf, block_count, frame_imax,
                                                  normalize_intensity, z_offset, out, out_stride, max_points, out_count);
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_pc2_blocks_per_frame(int max_points) { return (max_points + kPtsPerBlock - 1) / kPtsPerBlock; }
