// K11 — anchor-head decode fused with sigmoid / score filter / compaction
// (reference: OpenPCDet AnchorHeadSingle + ResidualCoder + generate_predicted_boxes +
// class_agnostic_nms' score mask, configured by data/pointpillar.yaml:72-142; the
// client-side intent to decode anchors is at clients/postprocess/detector_3d_postprocess.py:13-19).
//
// One thread per anchor (frame, y, x, a), anchors evaluated analytically
// (x = x0 + ix*dx, y = y0 + iy*dy, per-anchor size/height/rotation from a
// small table) so the 321,408 x 7 anchor tensor never exists.  Channel
// layout of the three head maps: cls a*C + c, box a*7 + k, dir a*bins + d —
// the order AnchorHeadSingle's permute/view produces.  Passing anchors
// (max sigmoid >= score_thresh) are compacted per frame; a 64-bit
// (score, ~anchor index) key makes the following top-k/NMS deterministic.
#include "tca_common.h"

using namespace tca;

namespace {

struct AnchorTable {
  float v[8][6];  // dxa, dya, dza, za(centre), rot, diag
};

constexpr int kAnchorsPerBlock = 4096;  // 16 per thread
constexpr int kStage = 2048;            // LDS-staged passing anchors per block

template <typename T>
__device__ __forceinline__ float head_at(const T* base, int layout, int b, int H, int W, int nch, int ld, int y, int x,
                                         int ch) {
  const long off = layout == 0 ? (((long)b * nch + ch) * H + y) * W + x : (((long)b * H + y) * W + x) * ld + ch;
  return to_f32(base[off]);
}

// Decode one passing anchor (ResidualCoder + direction classifier) into candidate slot o.
template <typename T>
__device__ void decode_write(const T* __restrict__ box, const T* __restrict__ dir, int layout, int H, int W, int A,
                             int bins, int ld_box, int ld_dir, const AnchorTable& tb, float x0, float xs, float y0,
                             float ys, float dir_offset, float dir_limit_offset, int b, int aidx, float score,
                             int label, long o, float* __restrict__ cand_box, float* __restrict__ cand_score,
                             int* __restrict__ cand_label, uint64_t* __restrict__ cand_key) {
  const int a = aidx % A, yx = aidx / A, y = yx / W, x = yx - y * W;
  const float* t = tb.v[a];
  const float xa = x0 + x * xs, ya = y0 + y * ys, za = t[3];
  const float dxa = t[0], dya = t[1], dza = t[2], ra = t[4], diag = t[5];
  float e[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) e[q] = head_at(box, layout, b, H, W, A * 7, ld_box, y, x, a * 7 + q);
  float out[7];
  out[0] = e[0] * diag + xa;
  out[1] = e[1] * diag + ya;
  out[2] = e[2] * dza + za;
  out[3] = __expf(e[3]) * dxa;
  out[4] = __expf(e[4]) * dya;
  out[5] = __expf(e[5]) * dza;
  float rg = e[6] + ra;
  if (dir && bins > 0) {
    float bd = -INFINITY;
    int dl = 0;
    for (int d = 0; d < bins; ++d) {
      const float v = head_at(dir, layout, b, H, W, A * bins, ld_dir, y, x, a * bins + d);
      if (v > bd) { bd = v; dl = d; }
    }
    const float period = 2.f * 3.14159265358979f / (float)bins;
    const float val = rg - dir_offset;
    const float lim = val - floorf(val / period + dir_limit_offset) * period;
    rg = lim + dir_offset + period * (float)dl;
  }
  out[6] = rg;
#pragma unroll
  for (int q = 0; q < 7; ++q) cand_box[o * 7 + q] = out[q];
  cand_score[o] = score;
  cand_label[o] = label;
  cand_key[o] = make_score_key(score, (uint32_t)aidx);
}

// One block covers kAnchorsPerBlock consecutive anchors of one frame: the
// class max / sigmoid / threshold runs over all of them (loads of 4
// iterations in flight per thread), passing anchors are staged in LDS, and
// the block takes ONE global slot range (a single atomic per block instead of
// one per 256 anchors), then decodes the staged boxes in parallel.
template <typename T>
__global__ void __launch_bounds__(256) anchor_decode_kernel(
    const T* __restrict__ cls, const T* __restrict__ box, const T* __restrict__ dir, int layout, int H, int W, int A,
    int C, int bins, int ld_cls, int ld_box, int ld_dir, AnchorTable tb, float x0, float xs, float y0, float ys,
    float dir_offset, float dir_limit_offset, float score_thresh, const uint32_t* __restrict__ key_thr,
    float* __restrict__ cand_box, float* __restrict__ cand_score, int* __restrict__ cand_label,
    uint64_t* __restrict__ cand_key, int* __restrict__ cand_count, int cap) {
  __shared__ int s_idx[kStage];
  __shared__ float s_score[kStage];
  __shared__ int s_label[kStage];
  __shared__ int s_cnt, s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int b = blockIdx.y;
  const int total = H * W * A;
  const uint32_t kthr = key_thr ? key_thr[2 * b + 1] : 0u;  // sel layout [B][2]
  const int a0 = blockIdx.x * kAnchorsPerBlock;
  const int a1 = min(a0 + kAnchorsPerBlock, total);
  for (int base = a0 + threadIdx.x; base < a1; base += 4 * 256) {
    float best[4];
    int bc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int aidx = base + u * 256;
      best[u] = -INFINITY;
      bc[u] = 0;
      if (aidx < a1) {
        const int a = aidx % A, yx = aidx / A, y = yx / W, x = yx - y * W;
        for (int c = 0; c < C; ++c) {
          const float v = head_at(cls, layout, b, H, W, A * C, ld_cls, y, x, a * C + c);
          if (v > best[u]) { best[u] = v; bc[u] = c; }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int aidx = base + u * 256;
      if (aidx >= a1) continue;
      const float score = sigmoidf_(best[u]);
      if (key_thr ? float_to_ordered(best[u]) < kthr : score < score_thresh) continue;
      const int slot = atomicAdd(&s_cnt, 1);
      if (slot < kStage) {
        s_idx[slot] = aidx;
        s_score[slot] = score;
        s_label[slot] = bc[u] + 1;
      } else {  // stage full (a dense block): take a global slot directly
        const int g = atomicAdd(&cand_count[b], 1);
        if (g < cap)
          decode_write(box, dir, layout, H, W, A, bins, ld_box, ld_dir, tb, x0, xs, y0, ys, dir_offset,
                       dir_limit_offset, b, aidx, score, bc[u] + 1, (long)b * cap + g, cand_box, cand_score,
                       cand_label, cand_key);
      }
    }
  }
  __syncthreads();
  const int n = min(s_cnt, kStage);
  if (threadIdx.x == 0) s_base = n ? atomicAdd(&cand_count[b], n) : 0;
  __syncthreads();
  const int base_slot = s_base;
  for (int k = threadIdx.x; k < n; k += 256) {
    const int slot = base_slot + k;
    if (slot >= cap) break;
    decode_write(box, dir, layout, H, W, A, bins, ld_box, ld_dir, tb, x0, xs, y0, ys, dir_offset, dir_limit_offset,
                 b, s_idx[k], s_score[k], s_label[k], (long)b * cap + slot, cand_box, cand_score, cand_label,
                 cand_key);
  }
}

// Pixel-major form of the same filter for an fp32 NHWC head (the fused neck's output):
// one thread per BEV pixel loads all A * C class logits of the pixel with 16-B loads
// (A * C = 18 for KITTI's 3 classes x 2 rotations: four float4 + one float2), so each
// thread has every load of its pixel in flight at once instead of a dependent chain of
// C scalar loads per anchor; the per-anchor max / sigmoid / threshold and the LDS-staged
// compaction + decode are the anchor kernel's, so the candidate set is identical.
template <int A, int C>
__global__ void __launch_bounds__(256) anchor_decode_px_kernel(
    const float* __restrict__ cls, const float* __restrict__ box, const float* __restrict__ dir, int H, int W,
    int bins, int ld_cls, int ld_box, int ld_dir, AnchorTable tb, float x0, float xs, float y0, float ys,
    float dir_offset, float dir_limit_offset, float score_thresh, float* __restrict__ cand_box,
    float* __restrict__ cand_score, int* __restrict__ cand_label, uint64_t* __restrict__ cand_key,
    int* __restrict__ cand_count, int cap) {
  constexpr int N = A * C, NV = N / 4;
  static_assert(256 * A <= kStage, "stage");
  __shared__ int s_idx[256 * A];
  __shared__ float s_score[256 * A];
  __shared__ int s_label[256 * A];
  __shared__ int s_cnt, s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int b = blockIdx.y;
  const int px = blockIdx.x * 256 + threadIdx.x;
  if (px < H * W) {
    const float* src = cls + ((long)b * H * W + px) * ld_cls;
    float v[N];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const float4 t = reinterpret_cast<const float4*>(src)[q];
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
#pragma unroll
    for (int q = 4 * NV; q < N; ++q) v[q] = src[q];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      float best = -INFINITY;
      int bc = 0;
#pragma unroll
      for (int c = 0; c < C; ++c)
        if (v[a * C + c] > best) { best = v[a * C + c]; bc = c; }
      const float score = sigmoidf_(best);
      if (score < score_thresh) continue;
      const int slot = atomicAdd(&s_cnt, 1);  // < 256 * A: every anchor of the block fits
      s_idx[slot] = px * A + a;
      s_score[slot] = score;
      s_label[slot] = bc + 1;
    }
  }
  __syncthreads();
  const int n = s_cnt;
  if (threadIdx.x == 0) s_base = n ? atomicAdd(&cand_count[b], n) : 0;
  __syncthreads();
  const int base_slot = s_base;
  for (int k = threadIdx.x; k < n; k += 256) {
    const int slot = base_slot + k;
    if (slot >= cap) break;
    decode_write(box, dir, 1, H, W, A, bins, ld_box, ld_dir, tb, x0, xs, y0, ys, dir_offset, dir_limit_offset, b,
                 s_idx[k], s_score[k], s_label[k], (long)b * cap + slot, cand_box, cand_score, cand_label, cand_key);
  }
}

// ---- exact top-k threshold over all anchors (proposal layers) -------------------
// SECONDHead's proposal layer keeps the top NMS_PRE_MAXSIZE (1024) of all
// 211,200 anchors by max class logit, with no score threshold.  Decoding and
// radix-selecting every anchor (one block per frame) cost ~0.9 ms per batch;
// instead two histogram passes over the ordered-u32 max-logit key (12 bits,
// then the next 12 bits inside the boundary bin) find a per-frame key
// threshold that admits the top k plus at most one 256-key bucket, and the
// decode kernel compacts only those.  Histograms are LDS-privatised per
// block, with the wave's dominant bins aggregated (the high bits of a
// narrow score band are all equal), and self-resetting.
constexpr int kHistBins = 4096;

template <typename T>
__global__ void __launch_bounds__(256) anchor_hist_kernel(const T* __restrict__ cls, int layout, int H, int W, int A,
                                                          int C, int ld_cls, int level, const uint32_t* __restrict__ sel,
                                                          unsigned* __restrict__ hist) {
  __shared__ unsigned sh[kHistBins];
  for (int i = threadIdx.x; i < kHistBins; i += 256) sh[i] = 0;
  __syncthreads();
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int total = H * W * A;
  const int a0 = blockIdx.x * kAnchorsPerBlock, a1 = min(a0 + kAnchorsPerBlock, total);
  const uint32_t pre = level == 2 ? sel[b * 2] : 0u;
  if (level == 2 && pre == 0xffffffffu) return;  // fewer than k anchors: nothing to refine
  for (int aidx = a0 + threadIdx.x; aidx < a0 + kAnchorsPerBlock; aidx += 256) {
    bool m = false;
    int d = 0;
    if (aidx < a1) {
      const int a = aidx % A, yx = aidx / A, y = yx / W, x = yx - y * W;
      float best = -INFINITY;
      for (int c = 0; c < C; ++c) best = fmaxf(best, head_at(cls, layout, b, H, W, A * C, ld_cls, y, x, a * C + c));
      const uint32_t u = float_to_ordered(best);
      if (level == 1) {
        m = true;
        d = (int)(u >> 20);
      } else {
        m = (u >> 20) == pre;
        d = (int)((u >> 8) & (kHistBins - 1));
      }
    }
    for (int round = 0; round < 2; ++round) {
      const unsigned long long mm = __ballot(m);
      if (!mm) break;
      const int leader = __ffsll(mm) - 1;
      const int dl = __shfl(d, leader, 64);
      const unsigned long long same = __ballot(m && d == dl);
      if (lane == leader) atomicAdd(&sh[dl], (unsigned)__popcll(same));
      if (d == dl) m = false;
    }
    if (m) atomicAdd(&sh[d], 1u);
  }
  __syncthreads();
  unsigned* hb = hist + (long)b * kHistBins;
  for (int i = threadIdx.x; i < kHistBins; i += 256)
    if (sh[i]) atomicAdd(&hb[i], sh[i]);
}

// One block per frame.  Level 1: sel[2b] = boundary bin (0xffffffff: all
// anchors pass), sel[2b+1] = count strictly above it.  Level 2: sel[2b+1] =
// the final ordered-key threshold.  Each level zeroes the histogram it read.
__global__ void __launch_bounds__(256) anchor_select_kernel(unsigned* __restrict__ hist, int level, int k,
                                                            uint32_t* __restrict__ sel) {
  __shared__ unsigned s_sum[256];
  __shared__ int s_pick;
  const int b = blockIdx.x, t = threadIdx.x;
  unsigned* hb = hist + (long)b * kHistBins;
  constexpr int PER = kHistBins / 256;  // 16 bins per thread, thread 0 owns the top bins
  unsigned v[PER], sum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    v[j] = hb[kHistBins - 1 - (t * PER + j)];
    sum += v[j];
  }
  s_sum[t] = sum;
  if (t == 0) s_pick = -1;
  __syncthreads();
  const bool all = level == 2 && sel[b * 2] == 0xffffffffu;
  const unsigned need = level == 1 ? (unsigned)k : (unsigned)k - sel[b * 2 + 1];
  if (t == 0 && !all) {  // 256 partial sums, serial from the top
    unsigned cum = 0;
    for (int i = 0; i < 256; ++i) {
      if (cum + s_sum[i] >= need) { s_pick = i; break; }
      cum += s_sum[i];
    }
    s_sum[0] = cum;  // count above the picked thread's range (thread 0 re-reads it below)
  }
  __syncthreads();
  const int pick = s_pick;
  if (t == pick) {
    unsigned cum = s_sum[0];  // count above this thread's bins (written by thread 0's scan)
    int bin = 0;
    for (int j = 0; j < PER; ++j) {
      if (cum + v[j] >= need) { bin = kHistBins - 1 - (t * PER + j); break; }
      cum += v[j];
    }
    if (level == 1) {
      sel[b * 2] = (uint32_t)bin;
      sel[b * 2 + 1] = cum;
    } else {
      sel[b * 2 + 1] = (sel[b * 2] << 20) | ((uint32_t)bin << 8);
    }
  }
  if (t == 0 && (pick < 0 || all)) {  // fewer than k keys: every anchor passes
    if (level == 1) { sel[b * 2] = 0xffffffffu; sel[b * 2 + 1] = 0; }
    else sel[b * 2 + 1] = 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) hb[kHistBins - 1 - (t * PER + j)] = 0;
}

}  // namespace

// sel: [B][2] uint32 scratch, hist: [B][4096] uint32 zero-initialised once
// (self-resetting).  On return sel[b][1] is frame b's ordered max-logit key
// threshold admitting its top k anchors (pass it to tca_anchor_decode_filter_keyed).
TCA_API int tca_anchor_topk_threshold(const void* cls, int dtype, int layout, int batch, int H, int W, int A, int C,
                                      int ld_cls, int k, unsigned* hist, uint32_t* sel, hipStream_t stream) {
  if (batch <= 0) return 0;
  dim3 grid((H * W * A + kAnchorsPerBlock - 1) / kAnchorsPerBlock, batch);
  const int ldc = ld_cls > 0 ? ld_cls : A * C;
  for (int level = 1; level <= 2; ++level) {
    switch (dtype) {
      case kF32: anchor_hist_kernel<float><<<grid, 256, 0, stream>>>((const float*)cls, layout, H, W, A, C, ldc, level,
                                                                      sel, hist); break;
      case kF16: anchor_hist_kernel<__half><<<grid, 256, 0, stream>>>((const __half*)cls, layout, H, W, A, C, ldc,
                                                                       level, sel, hist); break;
      case kBF16: anchor_hist_kernel<__hip_bfloat16><<<grid, 256, 0, stream>>>((const __hip_bfloat16*)cls, layout, H,
                                                                               W, A, C, ldc, level, sel, hist); break;
      default: return (int)hipErrorInvalidValue;
    }
    anchor_select_kernel<<<batch, 256, 0, stream>>>(hist, level, k, sel);
  }
  TCA_LAUNCH_CHECK();
}

// table: host [A][6] (dxa, dya, dza, za, rot, diag).
static int anchor_decode_launch(const void* cls, const void* box, const void* dir, int dtype, int layout, int batch,
                                int H, int W, int A, int C, int bins, int ld_cls, int ld_box, int ld_dir,
                                const float* table, float x0, float xs, float y0, float ys, float dir_offset,
                                float dir_limit_offset, float score_thresh, const uint32_t* key_thr, float* cand_box,
                                float* cand_score, int* cand_label, uint64_t* cand_key, int* cand_count, int cap,
                                hipStream_t stream) {
  if (batch <= 0) return 0;
  if (A > 8) return (int)hipErrorInvalidValue;
  AnchorTable tb;
  for (int a = 0; a < 8; ++a)
    for (int k = 0; k < 6; ++k) tb.v[a][k] = a < A ? table[a * 6 + k] : 0.f;
  int e = zero_i32_async(cand_count, batch, stream);
  if (e) return e;
  const int ldc = ld_cls > 0 ? ld_cls : A * C;
  if (dtype == kF32 && layout == 1 && !key_thr && A == 6 && C == 3 && (ldc & 3) == 0 &&
      ((uintptr_t)cls & 15) == 0) {  // KITTI PointPillars / SECOND head, fp32 NHWC
    anchor_decode_px_kernel<6, 3><<<dim3((H * W + 255) / 256, batch), 256, 0, stream>>>(
        (const float*)cls, (const float*)box, (const float*)dir, H, W, bins, ldc, ld_box > 0 ? ld_box : A * 7,
        ld_dir > 0 ? ld_dir : A * bins, tb, x0, xs, y0, ys, dir_offset, dir_limit_offset, score_thresh, cand_box,
        cand_score, cand_label, cand_key, cand_count, cap);
    TCA_LAUNCH_CHECK();
  }
  dim3 grid((H * W * A + kAnchorsPerBlock - 1) / kAnchorsPerBlock, batch);
#define LAUNCH(T)                                                                                              \
  anchor_decode_kernel<T><<<grid, 256, 0, stream>>>((const T*)cls, (const T*)box, (const T*)dir, layout, H, W, A, C, \
                                                    bins, ld_cls > 0 ? ld_cls : A * C, ld_box > 0 ? ld_box : A * 7,  \
                                                    ld_dir > 0 ? ld_dir : A * bins, tb, x0, xs, y0, ys, dir_offset, dir_limit_offset,          \
                                                    score_thresh, key_thr, cand_box, cand_score, cand_label, cand_key, \
                                                    cand_count, cap)
  switch (dtype) {
    case kF32: LAUNCH(float); break;
    case kF16: LAUNCH(__half); break;
    case kBF16: LAUNCH(__hip_bfloat16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LAUNCH
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_anchor_decode_filter(const void* cls, const void* box, const void* dir, int dtype, int layout, int batch,
                                     int H, int W, int A, int C, int bins, int ld_cls, int ld_box, int ld_dir,
                                     const float* table, float x0, float xs,
                                     float y0, float ys, float dir_offset, float dir_limit_offset, float score_thresh,
                                     float* cand_box, float* cand_score, int* cand_label, uint64_t* cand_key,
                                     int* cand_count, int cap, hipStream_t stream) {
  return anchor_decode_launch(cls, box, dir, dtype, layout, batch, H, W, A, C, bins, ld_cls, ld_box, ld_dir, table, x0,
                              xs, y0, ys, dir_offset, dir_limit_offset, score_thresh, nullptr, cand_box, cand_score,
                              cand_label, cand_key, cand_count, cap, stream);
}

// Same, but an anchor passes iff its ordered max-logit key >= key_thr[b]
// (device array from tca_anchor_topk_threshold; sel + 1 with stride 2).
TCA_API int tca_anchor_decode_filter_keyed(const void* cls, const void* box, const void* dir, int dtype, int layout,
                                           int batch, int H, int W, int A, int C, int bins, int ld_cls, int ld_box,
                                           int ld_dir, const float* table, float x0, float xs, float y0, float ys,
                                           float dir_offset, float dir_limit_offset, const uint32_t* sel,
                                           float* cand_box, float* cand_score, int* cand_label, uint64_t* cand_key,
                                           int* cand_count, int cap, hipStream_t stream) {
  return anchor_decode_launch(cls, box, dir, dtype, layout, batch, H, W, A, C, bins, ld_cls, ld_box, ld_dir, table, x0,
                              xs, y0, ys, dir_offset, dir_limit_offset, 0.f, sel, cand_box, cand_score, cand_label,
                              cand_key, cand_count, cap, stream);
}
