// CenterPoint-PointPillars (det3d, nuScenes) device ops:
//   K8b + K9  pfn2: two-layer PillarFeatureNet fused with PointPillarsScatter
//   K12 + K13 centerhead_decode: heatmap sigmoid/argmax + box assembly +
//             score / per-class threshold + post-centre-range filter + compaction
// Reference: data/nusc_centerpoint_pp_02voxel_two_pfn_10sweep.py:24-56 (model),
// :69-81 (test_cfg); voxel input clients/preprocess/voxelize.py:11-49 (5 point
// features, zero time lag); per-class score thresholds
// clients/postprocess/detector_3d_postprocess.py:98-133.
//
// pfn2 — one wave64 per pillar (P <= 32 slots; lanes l and l+32 own slot l&31):
//   features (x, y, z, r, t=0, xyz - mean, xy - centre), zero for padded slots;
//   layer 1: Linear(10->32) with BN folded on MFMA 32x32x16 (hi/lo bf16 split ->
//   3 MFMAs, because absolute coordinates of ~50 m do not survive one bf16
//   rounding), + bias, ReLU; max over the P slots;
//   layer 2: [y1 | max1] (64) -> Linear(64->64) on MFMA (y1 re-laid out through
//   a 2 KiB per-wave LDS tile so lanes own rows), + bias, ReLU, max over slots;
//   scatter: one 128-B NHWC canvas line per pillar.
//   F32 (the fp32 precision mode): layer 2 also runs as split products (y1 / max1
//   and W2 as hi + lo bf16 halves, 3 MFMAs per step, fp32 accumulation) and the
//   canvas is fp32 (256-B lines).
//
// centerhead_decode — one thread per (frame, task, pixel); the merged head
// output is NHWC with each task's channels [reg 2 | height 1 | dim 3 | rot 2 |
// vel 2 | hm nc] at a per-task channel offset.  Candidates are compacted per
// (frame, task) segment with a (score, ~pixel) key, so the following top-k /
// rotated NMS (nms.hip, segments = frame x task) is deterministic.  Box layout
// [x, y, z, w, l, h, yaw, vx, vy] keeps the NMS fields at 0..6.
#include "tca_common.h"

using namespace tca;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct PfnGeom {
  float r0, r1, vx, vy;
  int nx, ny;
};

__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

template <bool FROM_SLOTS, bool F32>
__global__ void __launch_bounds__(256) pfn2_kernel(
    const float* __restrict__ pts, int pstride, int max_pts,                // FROM_SLOTS source
    const int* __restrict__ slots, const int* __restrict__ vcount,
    const float* __restrict__ voxels, int vfeat, const int* __restrict__ num_points,  // materialised [V][P][vfeat]
    const int* __restrict__ coords, const int* __restrict__ voxel_count, int batch, int max_voxels, int P,
    const float* __restrict__ W1 /*[32][10]*/, const float* __restrict__ b1 /*[32]*/,
    const float* __restrict__ W2 /*[64][64]*/, const float* __restrict__ b2 /*[64]*/, PfnGeom g,
    void* __restrict__ canvas, float* __restrict__ feat_out) {
  constexpr int Y1 = 32 * 32 + 32;  // per wave: y1 rows + max1 (F32: hi tile, then lo tile)
  __shared__ __attribute__((aligned(16))) __hip_bfloat16 s_y1[4][F32 ? 2 * Y1 : Y1];
  const int lane = threadIdx.x & 63, wl = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  __hip_bfloat16* y1s = s_y1[wl];

  // layer-1 weights (hi/lo): lane holds W1[c=r][k=8h+j]
  bf16x8 w1h, w1l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * h + j;
    const float w = k < 10 ? W1[r * 10 + k] : 0.f;
    __bf16 hi, lo;
    split_bf16(w, hi, lo);
    w1h[j] = hi;
    w1l[j] = lo;
  }
  // layer-2 weights: tile t (cols 32t..32t+31), k-step s: W2[32t + r][16s + 8h + j]
  bf16x8 w2[2][4], w2l[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 hi, lo;
        split_bf16(W2[(32 * t + r) * 64 + 16 * s + 8 * h + j], hi, lo);
        w2[t][s][j] = hi;
        w2l[t][s][j] = F32 ? lo : (__bf16)0.f;
      }
  const float bias1 = b1[r];
  const float bias2_0 = b2[r], bias2_1 = b2[32 + r];

  const int nv = batch * max_voxels;  // 32-bit: 64-bit div/mod is ~150 VALU per use
  for (int v = (int)wave; v < nv; v += (int)nwaves) {
    const int b = (int)((unsigned)v / (unsigned)max_voxels), vid = v - b * max_voxels;
    if (vid >= voxel_count[b]) continue;
    int n;
    float p[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (FROM_SLOTS) {
      n = min(vcount[v], P);
      if (r < n) {
        const float* src = pts + ((long)b * max_pts + slots[v * P + r]) * pstride;
        p[0] = src[0]; p[1] = src[1]; p[2] = src[2]; p[3] = src[3];
        if (pstride >= 5) p[4] = src[4];
      }
    } else {
      n = min(num_points[v], P);
      if (r < n) {
        const float* src = voxels + (v * P + r) * vfeat;
        p[0] = src[0]; p[1] = src[1]; p[2] = src[2]; p[3] = src[3];
        if (vfeat >= 5) p[4] = src[4];
      }
    }
    float sx = p[0], sy = p[1], sz = p[2];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      sx += __shfl_xor(sx, o, 64);
      sy += __shfl_xor(sy, o, 64);
      sz += __shfl_xor(sz, o, 64);
    }
    const float inv_n = 1.f / (float)max(n, 1);
    const int* co = coords + v * 4;
    const float xc = (float)co[3] * g.vx + (g.vx * 0.5f + g.r0);
    const float yc = (float)co[2] * g.vy + (g.vy * 0.5f + g.r1);
    float f[8];
    if (h == 0) {
      f[0] = p[0]; f[1] = p[1]; f[2] = p[2]; f[3] = p[3]; f[4] = p[4];
      f[5] = p[0] - sx * inv_n; f[6] = p[1] - sy * inv_n; f[7] = p[2] - sz * inv_n;
    } else {
      f[0] = p[0] - xc; f[1] = p[1] - yc;
#pragma unroll
      for (int j = 2; j < 8; ++j) f[j] = 0.f;
    }
    const bool real = r < n;
    bf16x8 ah, al;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 hi, lo;
      split_bf16(real ? f[j] : 0.f, hi, lo);
      ah[j] = hi;
      al[j] = lo;
    }
    // ---- layer 1: rows = slots, cols = 32 units
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, w1h, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, w1l, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, w1h, acc, 0, 0, 0);
    float m1 = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int row = (j & 3) + 8 * (j >> 2) + 4 * h;
      const float y = fmaxf(acc[j] + bias1, 0.f);
      if constexpr (F32) {
        __bf16 hi, lo;
        split_bf16(y, hi, lo);
        reinterpret_cast<__bf16*>(y1s)[row * 32 + r] = hi;
        reinterpret_cast<__bf16*>(y1s)[Y1 + row * 32 + r] = lo;
      } else {
        y1s[row * 32 + r] = __float2bfloat16(y);
      }
      if (row < P) m1 = fmaxf(m1, y);
    }
    m1 = fmaxf(m1, __shfl_xor(m1, 32, 64));
    if (h == 0) {
      if constexpr (F32) {
        __bf16 hi, lo;
        split_bf16(m1, hi, lo);
        reinterpret_cast<__bf16*>(y1s)[32 * 32 + r] = hi;
        reinterpret_cast<__bf16*>(y1s)[Y1 + 32 * 32 + r] = lo;
      } else {
        y1s[32 * 32 + r] = __float2bfloat16(m1);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    // ---- layer 2: A rows = slots, k = [y1 (32) | max1 (32)]
    f32x16 a2[2] = {{}, {}};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const __hip_bfloat16* src = s < 2 ? y1s + r * 32 + 16 * s + 8 * h : y1s + 32 * 32 + 16 * (s - 2) + 8 * h;
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(src);
      if constexpr (F32) {
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(src + Y1);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          a2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, w2l[t][s], a2[t], 0, 0, 0);
          a2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, w2[t][s], a2[t], 0, 0, 0);
          a2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, w2[t][s], a2[t], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) a2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, w2[t][s], a2[t], 0, 0, 0);
      }
    }
    float m2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float mm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * h;
        if (row < P) mm = fmaxf(mm, a2[t][j]);
      }
      m2[t] = fmaxf(mm, __shfl_xor(mm, 32, 64));
    }
    __builtin_amdgcn_wave_barrier();  // LDS reads done before the next pillar overwrites y1s
    const float val = fmaxf(h == 0 ? m2[0] + bias2_0 : m2[1] + bias2_1, 0.f);
    const int ch = 32 * h + r;
    if (canvas) {
      const long cell = ((long)b * g.ny + co[2]) * g.nx + co[3];
      if constexpr (F32)
        reinterpret_cast<float*>(canvas)[cell * 64 + ch] = val;
      else
        reinterpret_cast<__hip_bfloat16*>(canvas)[cell * 64 + ch] = __float2bfloat16(val);
    }
    if (feat_out) feat_out[v * 64 + ch] = val;
  }
}

constexpr int kMaxTasks = 8;
constexpr int kMaxClasses = 32;

struct DecodeParams {
  int ntask;
  int toff[kMaxTasks];    // channel offset of task t in the merged head output
  int tnc[kMaxTasks];     // classes of task t
  int tcls0[kMaxTasks];   // global label of task t's first class
  float cls_thresh[kMaxClasses];  // per-class score threshold (K13); <= score_thresh disables
  float score_thresh;
  float r0, r1, vx, vy;
  int osf;
  float pcr[6];
};

template <typename T>
__global__ void __launch_bounds__(256) centerhead_decode_kernel(
    const T* __restrict__ head, int ldc, int H, int W, DecodeParams dp, float* __restrict__ cand_box,
    float* __restrict__ cand_score, int* __restrict__ cand_label, uint64_t* __restrict__ cand_key,
    int* __restrict__ cand_count, int cap) {
  const int t = blockIdx.y, b = blockIdx.z;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = b * dp.ntask + t;
  bool pass = false;
  float score = 0.f, bx[9];
  int label = 0;
  if (pix < H * W) {
    const int y = pix / W, x = pix - y * W;
    const T* c = head + ((long)b * H * W + pix) * ldc + dp.toff[t];
    float best = -INFINITY;
    int bc = 0;
    for (int k = 0; k < dp.tnc[t]; ++k) {
      const float v = to_f32(c[10 + k]);
      if (v > best) { best = v; bc = k; }
    }
    score = sigmoidf_(best);
    label = dp.tcls0[t] + bc;
    const float thr = fmaxf(dp.score_thresh, label < kMaxClasses ? dp.cls_thresh[label] : dp.score_thresh);
    if (score > thr) {
      bx[0] = ((float)x + to_f32(c[0])) * (float)dp.osf * dp.vx + dp.r0;
      bx[1] = ((float)y + to_f32(c[1])) * (float)dp.osf * dp.vy + dp.r1;
      bx[2] = to_f32(c[2]);
      bx[3] = __expf(to_f32(c[3]));
      bx[4] = __expf(to_f32(c[4]));
      bx[5] = __expf(to_f32(c[5]));
      bx[6] = atan2f(to_f32(c[6]), to_f32(c[7]));
      bx[7] = to_f32(c[8]);
      bx[8] = to_f32(c[9]);
      pass = bx[0] >= dp.pcr[0] && bx[1] >= dp.pcr[1] && bx[2] >= dp.pcr[2] && bx[0] <= dp.pcr[3] &&
             bx[1] <= dp.pcr[4] && bx[2] <= dp.pcr[5];
    }
  }
  // wave-level compaction: one atomic per wave
  const unsigned long long m = __ballot(pass);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (m) {
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&cand_count[seg], __popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1, 64);
  }
  if (pass) {
    const int o = base + __popcll(m & ((1ull << lane) - 1ull));
    if (o < cap) {
      const long q = (long)seg * cap + o;
#pragma unroll
      for (int k = 0; k < 9; ++k) cand_box[q * 9 + k] = bx[k];
      cand_score[q] = score;
      cand_label[q] = label;
      cand_key[q] = make_score_key(score, (uint32_t)pix);
    }
  }
}

}  // namespace

TCA_API int tca_pfn2_slots(const float* pts, int pstride, int max_pts, const int* slots, const int* vcount,
                           const int* coords, const int* voxel_count, int batch, int max_voxels, int P,
                           const float* W1, const float* b1, const float* W2, const float* b2, const float* range,
                           const float* vsize, int nx, int ny, void* canvas, float* feat_out, int f32,
                           hipStream_t stream) {
  if (batch <= 0) return 0;
  if (P > 32) return (int)hipErrorInvalidValue;
  PfnGeom g{range[0], range[1], vsize[0], vsize[1], nx, ny};
  if (f32)
    pfn2_kernel<true, true><<<2048, 256, 0, stream>>>(pts, pstride, max_pts, slots, vcount, nullptr, 5, nullptr, coords,
                                                      voxel_count, batch, max_voxels, P, W1, b1, W2, b2, g, canvas,
                                                      feat_out);
  else
    pfn2_kernel<true, false><<<2048, 256, 0, stream>>>(pts, pstride, max_pts, slots, vcount, nullptr, 5, nullptr,
                                                       coords, voxel_count, batch, max_voxels, P, W1, b1, W2, b2, g,
                                                       canvas, feat_out);
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_pfn2_voxels(const float* voxels, int vfeat, const int* num_points, const int* coords,
                            const int* voxel_count, int batch, int max_voxels, int P, const float* W1,
                            const float* b1, const float* W2, const float* b2, const float* range, const float* vsize,
                            int nx, int ny, void* canvas, float* feat_out, int f32, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (P > 32 || vfeat < 4) return (int)hipErrorInvalidValue;
  PfnGeom g{range[0], range[1], vsize[0], vsize[1], nx, ny};
  if (f32)
    pfn2_kernel<false, true><<<2048, 256, 0, stream>>>(nullptr, 4, 0, nullptr, nullptr, voxels, vfeat, num_points,
                                                       coords, voxel_count, batch, max_voxels, P, W1, b1, W2, b2, g,
                                                       canvas, feat_out);
  else
    pfn2_kernel<false, false><<<2048, 256, 0, stream>>>(nullptr, 4, 0, nullptr, nullptr, voxels, vfeat, num_points,
                                                        coords, voxel_count, batch, max_voxels, P, W1, b1, W2, b2, g,
                                                        canvas, feat_out);
  TCA_LAUNCH_CHECK();
}

// head: merged NHWC head output [B, H, W, ldc] (dtype: tca DType code);
// task_info: ntask x {channel offset, classes, first global label};
// cls_thresh: per global class (nullable); pcr: post-centre range [6].
// Candidate buffers are per segment (frame x task): box [B*T, cap, 9], ...
TCA_API int tca_centerhead_decode(const void* head, int dtype, int ldc, int batch, int H, int W, int ntask,
                                  const int* task_info, const float* cls_thresh, int ncls, float score_thresh,
                                  const float* range, const float* vsize, int osf, const float* pcr, float* cand_box,
                                  float* cand_score, int* cand_label, void* cand_key, int* cand_count, int cap,
                                  hipStream_t stream) {
  if (batch <= 0) return 0;
  if (ntask > kMaxTasks || ncls > kMaxClasses) return (int)hipErrorInvalidValue;
  DecodeParams dp{};
  dp.ntask = ntask;
  for (int t = 0; t < ntask; ++t) {
    dp.toff[t] = task_info[3 * t];
    dp.tnc[t] = task_info[3 * t + 1];
    dp.tcls0[t] = task_info[3 * t + 2];
  }
  for (int c = 0; c < kMaxClasses; ++c) dp.cls_thresh[c] = (cls_thresh && c < ncls) ? cls_thresh[c] : score_thresh;
  dp.score_thresh = score_thresh;
  dp.r0 = range[0]; dp.r1 = range[1]; dp.vx = vsize[0]; dp.vy = vsize[1]; dp.osf = osf;
  for (int k = 0; k < 6; ++k) dp.pcr[k] = pcr[k];
  int rc = zero_i32_async(cand_count, batch * ntask, stream);
  if (rc) return rc;
  dim3 grid((H * W + 255) / 256, ntask, batch);
  uint64_t* key = (uint64_t*)cand_key;
  switch (dtype) {
    case kF32: centerhead_decode_kernel<float><<<grid, 256, 0, stream>>>((const float*)head, ldc, H, W, dp, cand_box,
                                                                      cand_score, cand_label, key, cand_count, cap); break;
    case kBF16: centerhead_decode_kernel<__hip_bfloat16><<<grid, 256, 0, stream>>>((const __hip_bfloat16*)head, ldc, H, W,
                                                                               dp, cand_box, cand_score, cand_label,
                                                                               key, cand_count, cap); break;
    case kF16: centerhead_decode_kernel<__half><<<grid, 256, 0, stream>>>((const __half*)head, ldc, H, W, dp, cand_box,
                                                                       cand_score, cand_label, key, cand_count, cap); break;
    default: return (int)hipErrorInvalidValue;
  }
  TCA_LAUNCH_CHECK();
}
