// K8 + K9 — PillarVFE fused with PointPillarScatter, on MFMA
// (reference: server-side OpenPCDet PillarVFE/PointPillarScatter behind
// examples/pointpillar_kitti/1/model.py:163; config data/pointpillar.yaml:53-62).
//
// One wave64 per pillar, grid-stride over (frame, pillar):
//   * lanes l and l+32 own slot r = l & 31 of the pillar (P <= 32): they
//     gather the point (straight from the voxeliser's sorted slot list — no
//     [V,P,4] voxel tensor is materialised on the fused path — or from a
//     materialised voxel tensor on the server path);
//   * pillar mean of xyz: 32-lane shuffle reduction;
//   * 10-d decorated feature row per slot (x,y,z,i, xyz-mean, xyz-centre),
//     zero for padded slots exactly like OpenPCDet (so padded slots still
//     contribute relu(bias) to the max);
//   * Linear(10->64) with BN folded, as mfma_f32_32x32x16_bf16 (K padded to
//     16, two 32-column tiles).  Absolute coordinates (up to ~70 m) do not
//     survive a single bf16 rounding, so operands are split hi+lo and three
//     MFMAs (hi*hi + hi*lo + lo*hi) give ~fp32 accuracy — still 6 MFMAs per
//     pillar;
//   * max over slots: 16 accumulator registers, then lane l <-> l+32;
//     relu(max + bias) == max(relu(x + bias));
//   * scatter: lanes write the 64 channels of canvas[b][y][x][:] as one
//     128-byte (bf16) or 256-byte (fp32 mode) line (NHWC canvas, the layout
//     the BEV convs consume).
// tca_pillar_canvas_clear zeroes exactly the cells the previous frame wrote,
// so the 27 MB/frame canvas is never memset.
#include <type_traits>

#include "tca_common.h"

using namespace tca;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct PillarGeom {
  float r0, r1, r2, vx, vy, vz;
  int nx, ny;
};

__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

template <bool FROM_SLOTS, typename CT, int PFIX = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) pillar_vfe_kernel(
    const float* __restrict__ pts, int pstride, int max_pts,               // FROM_SLOTS source
    const int* __restrict__ slots, const int* __restrict__ vcount,        // FROM_SLOTS source
    const float* __restrict__ voxels, const int* __restrict__ num_points,  // materialised source [V][P][4]
    const int* __restrict__ coords, const int* __restrict__ voxel_count, int batch, int max_voxels, int P_arg,
    const float* __restrict__ W /*[64][10]*/, const float* __restrict__ bias /*[64]*/, PillarGeom g,
    CT* __restrict__ canvas, float* __restrict__ feat_out, uint8_t* __restrict__ occ) {
  // PFIX = 32 (every PointPillars config here): the slot bounds and the per-row
  // masks of the point max are compile-time
  const int P = PFIX ? PFIX : P_arg;
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;

  // B fragments (weights), hi/lo, two 32-column tiles: lane holds W[c][k=8h+j].  They stay in
  // LDS ([t][hi|lo][64 lanes][16 B], 4 KiB, read per pillar, conflict-free) rather than 16 VGPRs:
  // the kernel then fits 64 VGPRs, 8 waves per SIMD alone and 2 beside the BEV neck.
  __shared__ bf16x8 wfrag[2][2][64];
  if (threadIdx.x < 64) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int c = 32 * t + r;
      bf16x8 hv, lv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * h + j;
        const float w = k < 10 ? W[c * 10 + k] : 0.f;
        __bf16 hi, lo;
        split_bf16(w, hi, lo);
        hv[j] = hi;
        lv[j] = lo;
      }
      wfrag[t][0][lane] = hv;
      wfrag[t][1][lane] = lv;
    }
  }
  __syncthreads();
  const float b_my0 = bias[r], b_my1 = bias[32 + r];

  // 32-bit pillar indices (B * max_voxels < 2^31): 64-bit div/mod is ~150 VALU.
  // The pillar walk is wave-uniform (readfirstlane), so counts, coords and the
  // frame's voxel_count are scalar loads, and the two per-lane vector loads
  // (slot row, point) are issued unconditionally from clamped addresses: hipcc
  // can then wait for just the current point (vmcnt(1)) while the next
  // pillar's slot row is in flight, instead of draining with vmcnt(0).
  const int nv = batch * max_voxels;
  const int step = __builtin_amdgcn_readfirstlane((int)nwaves);
  auto next_valid = [&](int vv) {
    while (vv < nv) {
      const int bb = (unsigned)vv / (unsigned)max_voxels;
      if (vv - bb * max_voxels < voxel_count[bb]) break;
      vv += step;
    }
    return vv;
  };
  const bool vec4 = (pstride & 3) == 0;
  const int rs = min(r, P - 1);
  auto slot_of = [&](int vv) { return FROM_SLOTS ? slots[(long)min(vv, nv - 1) * P + rs] : 0; };
  auto gather = [&](int vv, int id, float (&q)[4]) {
    const int vc_ = vv < nv ? (FROM_SLOTS ? vcount[vv] : num_points[vv]) : 0;
    const bool real_ = r < min(vc_, P);
    const int bb = (unsigned)min(vv, nv - 1) / (unsigned)max_voxels;
    const float* src = FROM_SLOTS ? pts + ((long)bb * max_pts + (real_ ? id : 0)) * pstride
                                  : voxels + ((long)min(vv, nv - 1) * P + rs) * 4;
    if (!FROM_SLOTS || vec4) {
      const float4 t = *reinterpret_cast<const float4*>(src);
      q[0] = t.x; q[1] = t.y; q[2] = t.z; q[3] = t.w;
    } else {
      q[0] = src[0]; q[1] = src[1]; q[2] = src[2]; q[3] = src[3];
    }
  };
  // Three-deep: slot rows three pillars ahead, points two ahead, the pillar's count and
  // coordinates one ahead (each dependent load has two pillars of compute to land).
  auto meta = [&](int vv, int& vc_, int4& co_) {
    const int vq = min(vv, nv - 1);
    vc_ = FROM_SLOTS ? vcount[vq] : num_points[vq];
    co_ = *reinterpret_cast<const int4*>(coords + (long)vq * 4);
  };
  int v = next_valid(__builtin_amdgcn_readfirstlane((int)wave));
  int vn = v < nv ? next_valid(v + step) : nv;
  int vnn = vn < nv ? next_valid(vn + step) : nv;
  float pc[4], pn[4];
  gather(v, slot_of(v), pc);
  gather(vn, slot_of(vn), pn);
  int idx_nn = slot_of(vnn);
  int vc;
  int4 co;
  meta(v, vc, co);
  while (v < nv) {
    const int b = (unsigned)v / (unsigned)max_voxels;
    const int n = min(vc, P);
    const bool real = r < n;
    const int v3 = vnn < nv ? next_valid(vnn + step) : nv;
    const int idx_3 = slot_of(v3);     // three ahead
    float pnn[4];
    gather(vnn, idx_nn, pnn);          // two ahead
    int vc_n;
    int4 co_n;
    meta(vn, vc_n, co_n);              // one ahead
    float p[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = real ? pc[k] : 0.f;
    // pillar mean over the n real points (sum within each 32-lane half)
    float sx = p[0], sy = p[1], sz = p[2];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      sx += __shfl_xor(sx, o, 64);
      sy += __shfl_xor(sy, o, 64);
      sz += __shfl_xor(sz, o, 64);
    }
    const float inv_n = 1.f / (float)max(n, 1);
    const float mx = sx * inv_n, my = sy * inv_n, mz = sz * inv_n;
    const float xc = (float)co.w * g.vx + (g.vx * 0.5f + g.r0);
    const float yc = (float)co.z * g.vy + (g.vy * 0.5f + g.r1);
    const float zc = (float)co.y * g.vz + (g.vz * 0.5f + g.r2);
    float f[8];
    if (h == 0) {
      f[0] = p[0]; f[1] = p[1]; f[2] = p[2]; f[3] = p[3];
      f[4] = p[0] - mx; f[5] = p[1] - my; f[6] = p[2] - mz; f[7] = p[0] - xc;
    } else {
      f[0] = p[1] - yc; f[1] = p[2] - zc;
#pragma unroll
      for (int j = 2; j < 8; ++j) f[j] = 0.f;
    }
    bf16x8 ah, al;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float val = real ? f[j] : 0.f;
      __bf16 hi, lo;
      split_bf16(val, hi, lo);
      ah[j] = hi;
      al[j] = lo;
    }
    float m[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16x8 bh = wfrag[t][0][lane], bl = wfrag[t][1][lane];
      f32x16 acc = {};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
      float mm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * h;
        if (row < P) mm = fmaxf(mm, acc[j]);
      }
      mm = fmaxf(mm, __shfl_xor(mm, 32, 64));
      m[t] = mm;
      __builtin_amdgcn_sched_barrier(0);  // one tile's 16 accumulators live at a time
    }
    // lanes 0-31 -> channel r (tile 0), lanes 32-63 -> channel 32 + r (tile 1)
    const float val = fmaxf((h == 0 ? m[0] + b_my0 : m[1] + b_my1), 0.f);
    const int ch = 32 * h + r;
    if (canvas) {
      const long cell = ((long)b * g.ny + co.z) * g.nx + co.w;
      if constexpr (std::is_same<CT, PairTag>::value) {
        // pair storage: channel ch -> hi at 16*(ch/8) + ch%8, lo 8 bf16 later
        __bf16* c2 = reinterpret_cast<__bf16*>(canvas) + cell * 128 + (ch >> 3) * 16 + (ch & 7);
        const __bf16 h = (__bf16)val;
        c2[0] = h;
        c2[8] = (__bf16)(val - (float)h);
      } else {
        canvas[cell * 64 + ch] = from_f32<CT>(val);
      }
    }
    if (feat_out) feat_out[(long)v * 64 + ch] = val;
    // occupancy byte per written cell: the first BEV conv gates its reads on it
    if (occ && lane == 0) occ[((long)b * g.ny + co.z) * g.nx + co.w] = 1;
    v = vn;
    vn = vnn;
    vnn = v3;
    idx_nn = idx_3;
    vc = vc_n;
    co = co_n;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pc[k] = pn[k];
      pn[k] = pnn[k];
    }
  }
}

// The same PillarVFE + scatter, with the Linear(10->64) folded by linearity so it runs on the
// VALU in plain fp32 (more accurate than the split-bf16 MFMA above, and ~5x fewer VALU ops
// per pillar: no operand splits, no accumulator scan).  The ten features are
// [p, p - mean, p_xyz - centre], so with W = [W1 | W2 | W3]:
//   W f(p) = A p + d,   A = W1 + [W2 | 0] + [W3 | 0]   (64 x 4, per channel),
//                       d = -(W2 mean + W3 centre)     (per pillar and channel).
// max over the real points of (A p) + d, then the padded slots' zero row when n < P, then
// relu(+ bias) -- exactly OpenPCDet's masked features (padded rows give relu(bias)).
// One wave per pillar; lane c owns channel c; the pillar's points are staged in LDS
// (one float4 per slot, broadcast reads) and the per-point loop runs over the n real points
// only (n is wave-uniform): 3 FMA + 1 MUL + 1 MAX + 3 ADD (the xyz sums for the mean).
template <bool FROM_SLOTS, typename CT, int PFIX = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) pillar_vfe_lin_kernel(
    const float* __restrict__ pts, int pstride, int max_pts, const int* __restrict__ slots,
    const int* __restrict__ vcount, const float* __restrict__ voxels, const int* __restrict__ num_points,
    const int* __restrict__ coords, const int* __restrict__ voxel_count, int batch, int max_voxels, int P_arg,
    const float* __restrict__ W /*[64][10]*/, const float* __restrict__ bias /*[64]*/, PillarGeom g,
    CT* __restrict__ canvas, float* __restrict__ feat_out, uint8_t* __restrict__ occ) {
  const int P = PFIX ? PFIX : P_arg;
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wid = threadIdx.x >> 6;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  __shared__ float4 spts[4][32];

  const float* w = W + lane * 10;
  const float a0 = w[0] + w[4] + w[7], a1 = w[1] + w[5] + w[8], a2 = w[2] + w[6] + w[9], a3 = w[3];
  const float u0 = w[4], u1 = w[5], u2 = w[6], t0 = w[7], t1 = w[8], t2 = w[9];
  const float bc = bias[lane];

  const int nv = batch * max_voxels;
  const int step = __builtin_amdgcn_readfirstlane((int)nwaves);
  // Waves are spread over the frames (waves_per_frame of them each, frames b, b + fstep, ...), and
  // a wave walks its frame's real pillars with a fixed stride: the scalar unit (one per CU, shared
  // by the CU's 32 waves) no longer steps over the empty tail of every frame's max_voxels rows with
  // an integer division per row -- that scalar work bounded the kernel (PMC: 2x the VALU count in
  // SALU instructions, profiles/r6/vfe_pmc/).
  const int wave_u = __builtin_amdgcn_readfirstlane((int)wave);
  const int wpf = max(1, step / batch);
  const int fstep = max(1, step / wpf);
  const int loc0 = wave_u % wpf;
  auto first_at = [&](int bb) {
    while (bb < batch && loc0 >= voxel_count[bb]) bb += fstep;
    return bb;
  };
  int cb = first_at(wave_u / wpf), cl = loc0;  // the next pillar this wave takes
  auto take = [&](int& bb) {
    bb = min(cb, batch - 1);
    if (cb >= batch) return nv;
    const int row = cb * max_voxels + cl;
    cl += wpf;
    if (cl >= voxel_count[cb]) {
      cb = first_at(cb + fstep);
      cl = loc0;
    }
    return row;
  };
  const bool vec4 = (pstride & 3) == 0;
  const int rs = min(r, P - 1);
  auto slot_of = [&](int vv) { return FROM_SLOTS ? slots[min(vv, nv - 1) * P + rs] : 0; };
  auto gather = [&](int vv, int bb, int id, float (&q)[4]) {
    const int vc_ = vv < nv ? (FROM_SLOTS ? vcount[vv] : num_points[vv]) : 0;
    const bool real_ = r < min(vc_, P);
    const float* src = FROM_SLOTS ? pts + ((long)bb * max_pts + (real_ ? id : 0)) * pstride
                                  : voxels + ((long)min(vv, nv - 1) * P + rs) * 4;
    if (!FROM_SLOTS || vec4) {
      const float4 t = *reinterpret_cast<const float4*>(src);
      q[0] = t.x; q[1] = t.y; q[2] = t.z; q[3] = t.w;
    } else {
      q[0] = src[0]; q[1] = src[1]; q[2] = src[2]; q[3] = src[3];
    }
  };
  auto meta = [&](int vv, int& vc_, int4& co_) {
    const int vq = min(vv, nv - 1);
    vc_ = FROM_SLOTS ? vcount[vq] : num_points[vq];
    co_ = *reinterpret_cast<const int4*>(coords + vq * 4);
  };
  // the same three-deep load pipeline as the MFMA kernel
  int b, bn, bnn;
  int v = take(b);
  int vn = take(bn);
  int vnn = take(bnn);
  float pc[4], pn[4];
  gather(v, b, slot_of(v), pc);
  gather(vn, bn, slot_of(vn), pn);
  int idx_nn = slot_of(vnn);
  int vc;
  int4 co;
  meta(v, vc, co);
  while (v < nv) {
    const int n = __builtin_amdgcn_readfirstlane(min(vc, P));
    int b3;
    const int v3 = take(b3);
    const int idx_3 = slot_of(v3);
    float pnn[4];
    gather(vnn, bnn, idx_nn, pnn);
    int vc_n;
    int4 co_n;
    meta(vn, vc_n, co_n);
    if (h == 0) spts[wid][r] = make_float4(pc[0], pc[1], pc[2], pc[3]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float acc = -INFINITY, sx = 0.f, sy = 0.f, sz = 0.f;
#pragma unroll 4
    for (int j = 0; j < n; ++j) {
      const float4 q = spts[wid][j];
      acc = fmaxf(acc, fmaf(a0, q.x, fmaf(a1, q.y, fmaf(a2, q.z, a3 * q.w))));
      sx += q.x;
      sy += q.y;
      sz += q.z;
    }
    __builtin_amdgcn_wave_barrier();  // this pillar's reads before the next pillar's LDS writes
    const float inv_n = 1.f / (float)max(n, 1);
    const float xc = (float)co.w * g.vx + (g.vx * 0.5f + g.r0);
    const float yc = (float)co.z * g.vy + (g.vy * 0.5f + g.r1);
    const float zc = (float)co.y * g.vz + (g.vz * 0.5f + g.r2);
    const float d = -(u0 * (sx * inv_n) + u1 * (sy * inv_n) + u2 * (sz * inv_n) + t0 * xc + t1 * yc + t2 * zc);
    float mval = acc + d;
    if (n < P) mval = fmaxf(mval, 0.f);  // a padded slot's all-zero feature row
    const float val = fmaxf(mval + bc, 0.f);
    const int ch = lane;
    if (canvas) {
      const long cell = ((long)b * g.ny + co.z) * g.nx + co.w;
      if constexpr (std::is_same<CT, PairTag>::value) {
        __bf16* c2 = reinterpret_cast<__bf16*>(canvas) + cell * 128 + (ch >> 3) * 16 + (ch & 7);
        const __bf16 hv = (__bf16)val;
        c2[0] = hv;
        c2[8] = (__bf16)(val - (float)hv);
      } else {
        canvas[cell * 64 + ch] = from_f32<CT>(val);
      }
    }
    if (feat_out) feat_out[(long)v * 64 + ch] = val;
    if (occ && lane == 0) occ[((long)b * g.ny + co.z) * g.nx + co.w] = 1;
    v = vn;
    vn = vnn;
    vnn = v3;
    b = bn;
    bn = bnn;
    bnn = b3;
    idx_nn = idx_3;
    vc = vc_n;
    co = co_n;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pc[k] = pn[k];
      pn[k] = pnn[k];
    }
  }
}

// pillar_vfe_lin_kernel, two pillars per wave iteration: lanes 0-31 gather pillar A's slots and
// lanes 32-63 pillar B's (the one-pillar kernel loads the same 32 points into both halves), so a
// wave walks its chain of dependent loads (take -> slot index -> point gather) half as many times.
// That chain is what the one-pillar kernel waits on (PMC: 53% of wave time waiting,
// profiles/r6/vfe/).  Per pillar the expressions are those of the one-pillar kernel (the same
// values to fp32 rounding: the compiler may contract them into FMAs differently).
template <bool FROM_SLOTS, typename CT, int PFIX = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) pillar_vfe_lin2_kernel(
    const float* __restrict__ pts, int pstride, int max_pts, const int* __restrict__ slots,
    const int* __restrict__ vcount, const float* __restrict__ voxels, const int* __restrict__ num_points,
    const int* __restrict__ coords, const int* __restrict__ voxel_count, int batch, int max_voxels, int P_arg,
    const float* __restrict__ W /*[64][10]*/, const float* __restrict__ bias /*[64]*/, PillarGeom g,
    CT* __restrict__ canvas, float* __restrict__ feat_out, uint8_t* __restrict__ occ) {
  const int P = PFIX ? PFIX : P_arg;
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wid = threadIdx.x >> 6;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  __shared__ float4 spts[4][64];  // [wave][half * 32 + slot]

  const float* w = W + lane * 10;
  const float a0 = w[0] + w[4] + w[7], a1 = w[1] + w[5] + w[8], a2 = w[2] + w[6] + w[9], a3 = w[3];
  const float u0 = w[4], u1 = w[5], u2 = w[6], t0 = w[7], t1 = w[8], t2 = w[9];
  const float bc = bias[lane];

  const int nv = batch * max_voxels;
  const int step = __builtin_amdgcn_readfirstlane((int)nwaves);
  // the one-pillar kernel's per-frame walk: consecutive takes are this wave's next pillars
  const int wave_u = __builtin_amdgcn_readfirstlane((int)wave);
  const int wpf = max(1, step / batch);
  const int fstep = max(1, step / wpf);
  const int loc0 = wave_u % wpf;
  auto first_at = [&](int bb) {
    while (bb < batch && loc0 >= voxel_count[bb]) bb += fstep;
    return bb;
  };
  int cb = first_at(wave_u / wpf), cl = loc0;
  auto take = [&](int& bb) {
    bb = min(cb, batch - 1);
    if (cb >= batch) return nv;
    const int row = cb * max_voxels + cl;
    cl += wpf;
    if (cl >= voxel_count[cb]) {
      cb = first_at(cb + fstep);
      cl = loc0;
    }
    return row;
  };
  const bool vec4 = (pstride & 3) == 0;
  const int rs = min(r, P - 1);
  // lane half h works on pillar h of the pair (vA, vB)
  auto slot_of = [&](int vA, int vB) {
    const int vv = h ? vB : vA;
    return FROM_SLOTS ? slots[min(vv, nv - 1) * P + rs] : 0;
  };
  auto gather = [&](int vA, int vB, int bA, int bB, int id, float (&q)[4]) {
    const int vv = h ? vB : vA, bb = h ? bB : bA;
    const int vc_ = vv < nv ? (FROM_SLOTS ? vcount[vv] : num_points[vv]) : 0;
    const bool real_ = r < min(vc_, P);
    const float* src = FROM_SLOTS ? pts + ((long)bb * max_pts + (real_ ? id : 0)) * pstride
                                  : voxels + ((long)min(vv, nv - 1) * P + rs) * 4;
    if (!FROM_SLOTS || vec4) {
      const float4 t = *reinterpret_cast<const float4*>(src);
      q[0] = t.x; q[1] = t.y; q[2] = t.z; q[3] = t.w;
    } else {
      q[0] = src[0]; q[1] = src[1]; q[2] = src[2]; q[3] = src[3];
    }
  };
  auto meta = [&](int vA, int vB, int& vc_, int4& co_) {
    const int vq = min(h ? vB : vA, nv - 1);
    vc_ = FROM_SLOTS ? vcount[vq] : num_points[vq];
    co_ = *reinterpret_cast<const int4*>(coords + vq * 4);
  };
  // one pillar's output: the one-pillar kernel's expressions
  auto emit = [&](int n, float acc, float sx, float sy, float sz, int b, int cz, int cy, int cx, int v) {
    const float inv_n = 1.f / (float)max(n, 1);
    const float xc = (float)cx * g.vx + (g.vx * 0.5f + g.r0);
    const float yc = (float)cy * g.vy + (g.vy * 0.5f + g.r1);
    const float zc = (float)cz * g.vz + (g.vz * 0.5f + g.r2);
    const float d = -(u0 * (sx * inv_n) + u1 * (sy * inv_n) + u2 * (sz * inv_n) + t0 * xc + t1 * yc + t2 * zc);
    float mval = acc + d;
    if (n < P) mval = fmaxf(mval, 0.f);
    const float val = fmaxf(mval + bc, 0.f);
    const int ch = lane;
    const long cell = ((long)b * g.ny + cy) * g.nx + cx;
    if (canvas) {
      if constexpr (std::is_same<CT, PairTag>::value) {
        __bf16* c2 = reinterpret_cast<__bf16*>(canvas) + cell * 128 + (ch >> 3) * 16 + (ch & 7);
        const __bf16 hv = (__bf16)val;
        c2[0] = hv;
        c2[8] = (__bf16)(val - (float)hv);
      } else {
        canvas[cell * 64 + ch] = from_f32<CT>(val);
      }
    }
    if (feat_out) feat_out[(long)v * 64 + ch] = val;
    if (occ && lane == 0) occ[cell] = 1;
  };
  auto points_max = [&](const float4* sp, int n, float& acc, float& sx, float& sy, float& sz) {
    acc = -INFINITY;
    sx = sy = sz = 0.f;
#pragma unroll 4
    for (int j = 0; j < n; ++j) {
      const float4 q = sp[j];
      acc = fmaxf(acc, fmaf(a0, q.x, fmaf(a1, q.y, fmaf(a2, q.z, a3 * q.w))));
      sx += q.x;
      sy += q.y;
      sz += q.z;
    }
  };
  int bA, bB, bAn, bBn, bAnn, bBnn;
  int vA = take(bA), vB = take(bB);
  int vAn = take(bAn), vBn = take(bBn);
  int vAnn = take(bAnn), vBnn = take(bBnn);
  float pc[4], pn[4];
  gather(vA, vB, bA, bB, slot_of(vA, vB), pc);
  gather(vAn, vBn, bAn, bBn, slot_of(vAn, vBn), pn);
  int idx_nn = slot_of(vAnn, vBnn);
  int vc;
  int4 co;
  meta(vA, vB, vc, co);
  while (vA < nv) {
    const int mv = min(vc, P);
    const int nA = __builtin_amdgcn_readlane(mv, 0);
    const int nB = vB < nv ? __builtin_amdgcn_readlane(mv, 32) : 0;
    const int zA = __builtin_amdgcn_readlane(co.y, 0), yA = __builtin_amdgcn_readlane(co.z, 0),
              xA = __builtin_amdgcn_readlane(co.w, 0);
    const int zB = __builtin_amdgcn_readlane(co.y, 32), yB = __builtin_amdgcn_readlane(co.z, 32),
              xB = __builtin_amdgcn_readlane(co.w, 32);
    int bA3, bB3;
    const int vA3 = take(bA3), vB3 = take(bB3);
    const int idx_3 = slot_of(vA3, vB3);
    float pnn[4];
    gather(vAnn, vBnn, bAnn, bBnn, idx_nn, pnn);
    int vc_n;
    int4 co_n;
    meta(vAn, vBn, vc_n, co_n);
    spts[wid][lane] = make_float4(pc[0], pc[1], pc[2], pc[3]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float accA, sxA, syA, szA, accB, sxB, syB, szB;
    points_max(&spts[wid][0], nA, accA, sxA, syA, szA);
    points_max(&spts[wid][32], nB, accB, sxB, syB, szB);
    __builtin_amdgcn_wave_barrier();  // this pair's reads before the next pair's LDS writes
    emit(nA, accA, sxA, syA, szA, bA, zA, yA, xA, vA);
    if (nB > 0) emit(nB, accB, sxB, syB, szB, bB, zB, yB, xB, vB);
    vA = vAn; vB = vBn;
    vAn = vAnn; vBn = vBnn;
    vAnn = vA3; vBnn = vB3;
    bA = bAn; bB = bBn;
    bAn = bAnn; bBn = bBnn;
    bAnn = bA3; bBnn = bB3;
    idx_nn = idx_3;
    vc = vc_n;
    co = co_n;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pc[k] = pn[k];
      pn[k] = pnn[k];
    }
  }
}

// Zero exactly the cells the previous frame scattered: one thread per 16-B
// chunk of a pillar's C channels (C * esize % 16 == 0), frame per grid row.
// A bounded grid walks each frame's pillars (grid-stride): dispatching B x max_voxels worth of
// mostly early-exit workgroups (80 k for KITTI's 40 k pillars at batch 32) cost more than the stores.
__global__ void __launch_bounds__(256) canvas_clear_kernel(const int* __restrict__ coords,
                                                           const int* __restrict__ voxel_count, int max_voxels, int nx,
                                                           int ny, int C, int esize, uint4* __restrict__ canvas,
                                                           uint8_t* __restrict__ occ) {
  const int b = blockIdx.y;
  const int cpp = C * esize >> 4;
  const int sh = __builtin_ctz(cpp);  // cpp is a power of two (checked by the launcher): no division
  const int n = voxel_count[b] * cpp;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
    const int vid = t >> sh, c = t & (cpp - 1);
    const int* co = coords + ((long)b * max_voxels + vid) * 4;
    const long cell = ((long)b * ny + co[2]) * nx + co[3];
    canvas[cell * cpp + c] = make_uint4(0u, 0u, 0u, 0u);
    if (occ && c == 0) occ[cell] = 0;
  }
}

}  // namespace

namespace {
template <bool FROM_SLOTS, int PFIX>
int launch_vfe_t(const float* pts, int pstride, int max_pts, const int* slots, const int* vcount, const float* voxels,
                 const int* num_points, const int* coords, const int* voxel_count, int batch, int max_voxels, int P,
                 const float* W, const float* bias, const PillarGeom& g, void* canvas, float* feat_out, int dt,
                 uint8_t* occ, hipStream_t stream);

template <bool FROM_SLOTS>
int launch_vfe(const float* pts, int pstride, int max_pts, const int* slots, const int* vcount, const float* voxels,
               const int* num_points, const int* coords, const int* voxel_count, int batch, int max_voxels, int P,
               const float* W, const float* bias, const PillarGeom& g, void* canvas, float* feat_out, int dt,
               uint8_t* occ, hipStream_t stream) {
  if (P > 32 || (dt != kBF16 && dt != kF32 && dt != kPair)) return (int)hipErrorInvalidValue;
  if (P == 32) return launch_vfe_t<FROM_SLOTS, 32>(pts, pstride, max_pts, slots, vcount, voxels, num_points, coords,
                                                    voxel_count, batch, max_voxels, P, W, bias, g, canvas, feat_out,
                                                    dt, occ, stream);
  return launch_vfe_t<FROM_SLOTS, 0>(pts, pstride, max_pts, slots, vcount, voxels, num_points, coords, voxel_count,
                                     batch, max_voxels, P, W, bias, g, canvas, feat_out, dt, occ, stream);
}

// 0: the fp32 VALU kernel, one pillar per wave iteration (TCA_VFE_LIN2=0); 1: the split-bf16 MFMA
// kernel (TCA_VFE_MFMA=1; kept for A/B and its tests); 2 (default since round 6): the fp32 VALU kernel,
// two pillars per wave iteration -- bit-identical to 0, 119 vs 141 us alone at the headline batch and
// +0.4 / +0.5% on the headline in two same-box sweeps of the final tree (profiles/r6/knobs/).
// tca_pillar_vfe_set_variant switches at run time.
int g_vfe_variant = -1;

// workgroups of the encoder launch: 2048 (8 per CU), TCA_VFE_GRID overrides for sweeps
int vfe_grid() {
  static int g = 0;
  if (!g) {
    const char* e = getenv("TCA_VFE_GRID");
    g = e ? atoi(e) : 0;
    g = g >= 64 && g <= 65536 ? g : 2048;
  }
  return g;
}

int vfe_variant() {
  if (g_vfe_variant < 0) {
    const char* e = getenv("TCA_VFE_MFMA");
    const char* e2 = getenv("TCA_VFE_LIN2");
    g_vfe_variant = (e && e[0] == '1') ? 1 : (e2 && e2[0] == '0') ? 0 : 2;
  }
  return g_vfe_variant;
}

template <bool FROM_SLOTS, int PFIX>
int launch_vfe_t(const float* pts, int pstride, int max_pts, const int* slots, const int* vcount, const float* voxels,
                 const int* num_points, const int* coords, const int* voxel_count, int batch, int max_voxels, int P,
                 const float* W, const float* bias, const PillarGeom& g, void* canvas, float* feat_out, int dt,
                 uint8_t* occ, hipStream_t stream) {
#define TCA_VFE_LAUNCH(KERNEL, CT)                                                                                 \
  KERNEL<FROM_SLOTS, CT, PFIX><<<vfe_grid(), 256, 0, stream>>>(pts, pstride, max_pts, slots, vcount, voxels, num_points, \
                                                        coords, voxel_count, batch, max_voxels, P, W, bias, g,      \
                                                        (CT*)canvas, feat_out, occ)
  const int var = vfe_variant();
  if (dt == kF32) {
    if (var == 1) TCA_VFE_LAUNCH(pillar_vfe_kernel, float);
    else if (var == 2) TCA_VFE_LAUNCH(pillar_vfe_lin2_kernel, float);
    else TCA_VFE_LAUNCH(pillar_vfe_lin_kernel, float);
  } else if (dt == kPair) {
    if (var == 1) TCA_VFE_LAUNCH(pillar_vfe_kernel, PairTag);
    else if (var == 2) TCA_VFE_LAUNCH(pillar_vfe_lin2_kernel, PairTag);
    else TCA_VFE_LAUNCH(pillar_vfe_lin_kernel, PairTag);
  } else {
    if (var == 1) TCA_VFE_LAUNCH(pillar_vfe_kernel, __hip_bfloat16);
    else if (var == 2) TCA_VFE_LAUNCH(pillar_vfe_lin2_kernel, __hip_bfloat16);
    else TCA_VFE_LAUNCH(pillar_vfe_lin_kernel, __hip_bfloat16);
  }
#undef TCA_VFE_LAUNCH
  TCA_LAUNCH_CHECK();
}
}  // namespace

// VFE kernel selection: 0 = fp32 VALU, 1 = split-bf16 MFMA, 2 = fp32 VALU two pillars per wave
// iteration; returns the previous one.
TCA_API int tca_pillar_vfe_set_variant(int v) {
  const int old = vfe_variant();
  g_vfe_variant = (v == 1 || v == 2) ? v : 0;
  return old;
}

// Fused path: source = voxeliser slots + unpacked points.  canvas_dtype: kBF16,
// kF32 or kPair (fp32 mode's pair storage, see tca_common.h).
TCA_API int tca_pillar_vfe_slots(const float* pts, int pstride, int max_pts, const int* slots, const int* vcount,
                                 const int* coords, const int* voxel_count, int batch, int max_voxels, int P,
                                 const float* W, const float* bias, const float* range, const float* vsize, int nx,
                                 int ny, void* canvas, float* feat_out, int canvas_dtype, hipStream_t stream) {
  if (batch <= 0) return 0;
  PillarGeom g{range[0], range[1], range[2], vsize[0], vsize[1], vsize[2], nx, ny};
  return launch_vfe<true>(pts, pstride, max_pts, slots, vcount, nullptr, nullptr, coords, voxel_count, batch,
                          max_voxels, P, W, bias, g, canvas, feat_out, canvas_dtype, nullptr, stream);
}

// Same, also marking occ[b, y, x] = 1 (uint8 [B, ny, nx]) for every written cell.
TCA_API int tca_pillar_vfe_slots_occ(const float* pts, int pstride, int max_pts, const int* slots, const int* vcount,
                                     const int* coords, const int* voxel_count, int batch, int max_voxels, int P,
                                     const float* W, const float* bias, const float* range, const float* vsize,
                                     int nx, int ny, void* canvas, float* feat_out, int canvas_dtype, uint8_t* occ,
                                     hipStream_t stream) {
  if (batch <= 0) return 0;
  PillarGeom g{range[0], range[1], range[2], vsize[0], vsize[1], vsize[2], nx, ny};
  return launch_vfe<true>(pts, pstride, max_pts, slots, vcount, nullptr, nullptr, coords, voxel_count, batch,
                          max_voxels, P, W, bias, g, canvas, feat_out, canvas_dtype, occ, stream);
}

// Server path: source = materialised voxels [B*V][P][4] + num_points (KServe inputs).
TCA_API int tca_pillar_vfe_voxels(const float* voxels, const int* num_points, const int* coords,
                                  const int* voxel_count, int batch, int max_voxels, int P, const float* W,
                                  const float* bias, const float* range, const float* vsize, int nx, int ny,
                                  void* canvas, float* feat_out, int canvas_dtype, hipStream_t stream) {
  if (batch <= 0) return 0;
  PillarGeom g{range[0], range[1], range[2], vsize[0], vsize[1], vsize[2], nx, ny};
  return launch_vfe<false>(nullptr, 4, 0, nullptr, nullptr, voxels, num_points, coords, voxel_count, batch,
                           max_voxels, P, W, bias, g, canvas, feat_out, canvas_dtype, nullptr, stream);
}

TCA_API int tca_pillar_vfe_voxels_occ(const float* voxels, const int* num_points, const int* coords,
                                      const int* voxel_count, int batch, int max_voxels, int P, const float* W,
                                      const float* bias, const float* range, const float* vsize, int nx, int ny,
                                      void* canvas, float* feat_out, int canvas_dtype, uint8_t* occ,
                                      hipStream_t stream) {
  if (batch <= 0) return 0;
  PillarGeom g{range[0], range[1], range[2], vsize[0], vsize[1], vsize[2], nx, ny};
  return launch_vfe<false>(nullptr, 4, 0, nullptr, nullptr, voxels, num_points, coords, voxel_count, batch,
                           max_voxels, P, W, bias, g, canvas, feat_out, canvas_dtype, occ, stream);
}

namespace {
int canvas_clear(const int* coords, const int* voxel_count, int batch, int max_voxels, int nx, int ny, int C,
                 void* canvas, int canvas_dtype, uint8_t* occ, hipStream_t stream) {
  if (batch <= 0) return 0;
  const int esize = (canvas_dtype == kF32 || canvas_dtype == kPair) ? 4 : 2;
  if ((C * esize) & 15 || (canvas_dtype != kBF16 && canvas_dtype != kF32 && canvas_dtype != kPair))
    return (int)hipErrorInvalidValue;
  const int cpp = C * esize / 16;
  if (cpp & (cpp - 1)) return (int)hipErrorInvalidValue;  // 16-B chunks per pillar: a power of two
  const int need = (max_voxels * (C * esize / 16) + 255) / 256;
  canvas_clear_kernel<<<dim3(need < 64 ? need : 64, batch), 256, 0, stream>>>(
      coords, voxel_count, max_voxels, nx, ny, C, esize, (uint4*)canvas, occ);
  TCA_LAUNCH_CHECK();
}
// Occupancy-gated canvas (every reader of the features skips unoccupied cells: the first BEV conv
// gates its loads on occ): the previous frame's features may stay, only its occupancy bytes go.
// One thread per pillar, a bounded grid per frame.
__global__ void __launch_bounds__(256) occ_clear_kernel(const int* __restrict__ coords,
                                                        const int* __restrict__ voxel_count, int max_voxels, int nx,
                                                        int ny, uint8_t* __restrict__ occ) {
  const int b = blockIdx.y;
  const int n = voxel_count[b];
  for (int vid = blockIdx.x * 256 + threadIdx.x; vid < n; vid += gridDim.x * 256) {
    const int4 co = *reinterpret_cast<const int4*>(coords + ((long)b * max_voxels + vid) * 4);
    occ[((long)b * ny + co.z) * nx + co.w] = 0;
  }
}
}  // namespace

// Clear only the occupancy bytes of the cells the previous frame wrote (see occ_clear_kernel).
TCA_API int tca_pillar_occ_clear(const int* coords, const int* voxel_count, int batch, int max_voxels, int nx, int ny,
                                 uint8_t* occ, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (!occ) return (int)hipErrorInvalidValue;
  const int need = (max_voxels + 255) / 256;
  occ_clear_kernel<<<dim3(need < 16 ? need : 16, batch), 256, 0, stream>>>(coords, voxel_count, max_voxels, nx, ny,
                                                                           occ);
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_pillar_canvas_clear(const int* coords, const int* voxel_count, int batch, int max_voxels, int nx,
                                    int ny, int C, void* canvas, int canvas_dtype, hipStream_t stream) {
  return canvas_clear(coords, voxel_count, batch, max_voxels, nx, ny, C, canvas, canvas_dtype, nullptr, stream);
}

// Same, also clearing those cells' occupancy bytes.
TCA_API int tca_pillar_canvas_clear_occ(const int* coords, const int* voxel_count, int batch, int max_voxels, int nx,
                                        int ny, int C, void* canvas, int canvas_dtype, uint8_t* occ,
                                        hipStream_t stream) {
  return canvas_clear(coords, voxel_count, batch, max_voxels, nx, ny, C, canvas, canvas_dtype, occ, stream);
}
