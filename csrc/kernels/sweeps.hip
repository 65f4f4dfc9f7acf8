// K7s — multi-sweep LiDAR accumulation for CenterPoint's nuScenes "10sweep"
// input (data/nusc_centerpoint_pp_02voxel_two_pfn_10sweep.py: nsweeps, 5 point
// features with the time lag as the 5th; the reference client only zero-fills
// that column for one sweep, clients/preprocess/voxelize.py:38-39).
//
// A device ring keeps the last R = nsweeps - 1 unpacked sweeps of every frame
// slot (xyz + intensity, their count, timestamp and sensor pose).  Each step:
//   merge   — [current sweep | sweep t-1 | ... | sweep t-R] -> one point list per
//             frame, stride 5: (x, y, z, intensity, time lag).  Older sweeps are
//             moved into the current sensor frame with the relative pose
//             inv(T_cur) * T_k (rigid 3x4 poses, row-major [R | t]) and get
//             lag = t_cur - t_k, the det3d sweep convention (current sweep first);
//   push    — the current sweep into the ring slot `head` (the oldest, consumed);
//   advance — head = (head + 1) % R, and the clock += dt when auto-clocked.
// The ring position lives in device memory, so the three kernels replay inside a
// captured step graph: every replay consumes and advances the ring.
#include "tca_common.h"

using namespace tca;

namespace {

struct SweepRing {
  float* ring;        // [R][B][maxp][4]
  int* ring_n;        // [R][B]
  double* ring_t;     // [R][B] timestamps (fp64: epoch-second stamps / hours of auto-clock keep ms lags)
  float* ring_pose;   // [R][B][12]
  int* head;          // [1]
  double* clock;      // [B] current timestamps (fp64)
  float* pose;        // [B][12] current poses
  int R, B, maxp;
};

__device__ __forceinline__ int ring_slot(int head, int k, int R) { return ((head - k) % R + R) % R; }

__global__ void __launch_bounds__(256) sweep_merge_kernel(const float* __restrict__ cur, int cs,
                                                          const int* __restrict__ cur_n, SweepRing r,
                                                          float* __restrict__ out, int* __restrict__ out_n) {
  const int b = blockIdx.z, k = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int S = r.R + 1, h = *r.head;
  // offsets: counts of sweeps 0..k-1 of this frame (S <= 32: a short serial sum per thread)
  int off = 0, nk = 0, total = 0;
  for (int j = 0; j < S; ++j) {
    const int n = j == 0 ? min(cur_n[b], r.maxp) : r.ring_n[ring_slot(h, j, r.R) * r.B + b];
    if (j < k) off += n;
    if (j == k) nk = n;
    total += n;
  }
  if (k == 0 && i == 0) out_n[b] = total;
  if (i >= nk) return;
  float* o = out + ((long)b * S * r.maxp + off + i) * 5;
  if (k == 0) {
    const float* p = cur + ((long)b * r.maxp + i) * cs;
    o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = p[3]; o[4] = 0.f;
    return;
  }
  const int slot = ring_slot(h, k, r.R);
  const float* p = r.ring + (((long)slot * r.B + b) * r.maxp + i) * 4;
  const float* Tk = r.ring_pose + ((long)slot * r.B + b) * 12;
  const float* Tc = r.pose + (long)b * 12;
  // q = R_k p + t_k - t_c ; p' = R_c^T q
  float q[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) q[a] = Tk[4 * a] * p[0] + Tk[4 * a + 1] * p[1] + Tk[4 * a + 2] * p[2] + Tk[4 * a + 3] - Tc[4 * a + 3];
#pragma unroll
  for (int a = 0; a < 3; ++a) o[a] = Tc[a] * q[0] + Tc[4 + a] * q[1] + Tc[8 + a] * q[2];
  o[3] = p[3];
  o[4] = (float)(r.clock[b] - r.ring_t[slot * r.B + b]);
}

__global__ void __launch_bounds__(256) sweep_push_kernel(const float* __restrict__ cur, int cs,
                                                         const int* __restrict__ cur_n, SweepRing r) {
  const int b = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  const int slot = *r.head, n = min(cur_n[b], r.maxp);
  if (blockIdx.x == 0 && threadIdx.x < 12) {
    if (threadIdx.x == 0) {
      r.ring_n[slot * r.B + b] = n;
      r.ring_t[slot * r.B + b] = r.clock[b];
    }
    r.ring_pose[((long)slot * r.B + b) * 12 + threadIdx.x] = r.pose[(long)b * 12 + threadIdx.x];
  }
  if (i >= n) return;
  const float* p = cur + ((long)b * r.maxp + i) * cs;
  *reinterpret_cast<float4*>(r.ring + (((long)slot * r.B + b) * r.maxp + i) * 4) = make_float4(p[0], p[1], p[2], p[3]);
}

__global__ void sweep_advance_kernel(SweepRing r, double dt) {
  const int t = threadIdx.x;
  if (t == 0) *r.head = (*r.head + 1) % r.R;
  if (dt != 0.0)
    for (int b = t; b < r.B; b += blockDim.x) r.clock[b] += dt;
}

}  // namespace

// cur [B, maxp, cs] (cs >= 4) unpacked points with counts cur_n [B]; ring state as in
// SweepRing; out [B, (R + 1) * maxp, 5], out_n [B].  dt: seconds added to every
// clock after the step (0: the caller sets the clock from message stamps).
// ring_t [R, B] and clock [B] are fp64 seconds.
TCA_API int tca_sweep_step(const float* cur, int cs, const int* cur_n, int B, int maxp, int R, float* ring, int* ring_n,
                           double* ring_t, float* ring_pose, int* head, double* clock, float* pose, double dt,
                           float* out, int* out_n, hipStream_t stream) {
  if (B <= 0) return 0;
  if (R < 1 || R > 31 || cs < 4 || maxp <= 0) return (int)hipErrorInvalidValue;
  SweepRing r{ring, ring_n, ring_t, ring_pose, head, clock, pose, R, B, maxp};
  const unsigned gx = (unsigned)((maxp + 255) / 256);
  sweep_merge_kernel<<<dim3(gx, R + 1, B), 256, 0, stream>>>(cur, cs, cur_n, r, out, out_n);
  sweep_push_kernel<<<dim3(gx, B), 256, 0, stream>>>(cur, cs, cur_n, r);
  sweep_advance_kernel<<<1, 64, 0, stream>>>(r, dt);
  TCA_LAUNCH_CHECK();
}
