// K4 / K10 — top-k + sort + bitmask NMS, axis-aligned (2D, class-aware) and
// rotated-BEV (3D), with the output formatting fused into the reduce.
//
// Reference semantics:
//  * 2D: clients/postprocess/yolov5_postprocess.py:100-110 — keep top max_nms by
//    conf, class-offset batched torchvision.ops.nms(iou > 0.45), cap max_det.
//    The class offset (+cls*4096) is implemented as "only same-class boxes
//    suppress each other" (identical kept set for coords < 4096 px, and
//    without the fp32 precision loss the offset causes).
//  * 3D: OpenPCDet class_agnostic_nms + iou3d_nms nms_gpu (data/pointpillar.yaml:130-142):
//    score >= thresh, top NMS_PRE_MAXSIZE, suppress iou_bev > thresh, keep
//    NMS_POST_MAXSIZE.  Rotated BEV IoU via Green's theorem over clipped edges.
//
// Pipeline per image (all launch shapes static, counts read on device):
//  1. tca_topk_sort     one 1024-thread block / image: exact radix-select of the
//                       k largest 64-bit keys (8 passes of 8-bit digits, LDS
//                       histogram) when n > k, then an LDS bitonic sort.
//  2. tca_nms_mask_*    64x64 tiles of the upper triangle, one 64-bit
//                       suppression word per (row, 64-column block): a wave64
//                       lane owns one row and one uint64 word per tile.
//  3. tca_nms_reduce    one block / image: 64-row blocks are resolved
//                       serially on LDS words, kept rows' masks are OR-ed
//                       into the removed set in parallel, then the kept boxes
//                       are written out (2D: undo letterbox/stretch + clip).
#include "tca_common.h"

using namespace tca;

namespace {

constexpr int kSortCap = 8192;  // 8192 x (8 B key + 4 B slot) = 96 KiB of LDS

__global__ void __launch_bounds__(1024) topk_sort_kernel(const uint64_t* __restrict__ keys, const int* __restrict__ count,
                                                         int cap, int pre_max, int* __restrict__ order,
                                                         int* __restrict__ sorted_n) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* skey = (uint64_t*)smem;
  int* sslot = (int*)(smem + sizeof(uint64_t) * kSortCap);
  int* hist = sslot + kSortCap;  // 256
  int* misc = hist + 256;        // [0] counter, [1] digit, [2] remaining
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const uint64_t* kb = keys + (long)b * cap;
  const int n = min(count[b], cap);
  const int k = min(min(n, pre_max), kSortCap);
  if (tid == 0) misc[0] = 0;
  __syncthreads();
  if (n > k) {
    uint64_t prefix = 0, pmask = 0;
    int remaining = k;
    for (int pass = 0; pass < 8; ++pass) {
      const int shift = 56 - 8 * pass;
      for (int i = tid; i < 256; i += nt) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < n; i += nt) {
        uint64_t key = kb[i];
        if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int cum = 0, d = 255;
        for (; d >= 0; --d) {
          if (cum + hist[d] >= remaining) break;
          cum += hist[d];
        }
        misc[1] = d < 0 ? 0 : d;
        misc[2] = remaining - cum;
      }
      __syncthreads();
      prefix |= (uint64_t)misc[1] << shift;
      pmask |= (uint64_t)255 << shift;
      remaining = misc[2];
      __syncthreads();
    }
    // keys are unique: exactly k keys are >= the k-th largest (prefix).
    for (int i = tid; i < n; i += nt) {
      uint64_t key = kb[i];
      if (key >= prefix) {
        int p = atomicAdd(&misc[0], 1);
        if (p < k) { skey[p] = key; sslot[p] = i; }
      }
    }
  } else {
    for (int i = tid; i < n; i += nt) { skey[i] = kb[i]; sslot[i] = i; }
  }
  __syncthreads();
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = k + tid; i < P; i += nt) { skey[i] = 0; sslot[i] = -1; }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (P >> 1); i += nt) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint64_t a = skey[lo], c = skey[hi];
        if ((a < c) == desc) {
          skey[lo] = c; skey[hi] = a;
          int t = sslot[lo]; sslot[lo] = sslot[hi]; sslot[hi] = t;
        }
      }
      __syncthreads();
    }
  }
  int* ob = order + (long)b * pre_max;
  for (int i = tid; i < k; i += nt) ob[i] = sslot[i];
  if (tid == 0) sorted_n[b] = k;
}

__device__ __forceinline__ float iou_aa(const float* a, const float* c) {
  const float ix1 = fmaxf(a[0], c[0]), iy1 = fmaxf(a[1], c[1]);
  const float ix2 = fminf(a[2], c[2]), iy2 = fminf(a[3], c[3]);
  const float iw = fmaxf(ix2 - ix1, 0.f), ih = fmaxf(iy2 - iy1, 0.f);
  const float inter = iw * ih;
  const float aa = (a[2] - a[0]) * (a[3] - a[1]);
  const float ac = (c[2] - c[0]) * (c[3] - c[1]);
  return inter / (aa + ac - inter);
}

// ---- rotated BEV IoU ----------------------------------------------------------
// Intersection area of two rotated rectangles without any polygon buffer
// (a dynamically indexed vertex array would live in scratch memory): by
// Green's theorem the CCW boundary of A∩B is the part of A's edges inside B
// plus the part of B's edges inside A, so
//     2·area = Σ_{edges of A} cross(clip_B(e)) + Σ_{edges of B} cross(clip_A(e))
// with cross(p0,p1) = p0.x·p1.y − p0.y·p1.x over the clipped sub-segment.
// Work in A's frame (A axis-aligned, centred at 0): B's edges are clipped to
// A's box by Liang–Barsky; A's edges are clipped by B's four half-planes by
// Cyrus–Beck.  Boundary convention: A's edges use closed half-planes, B's
// edges open ones, so coincident edges (e.g. identical boxes) count once.
// Everything is fully unrolled with static indices: ~150 FLOPs, no branches
// that diverge beyond the early-outs.
__device__ __forceinline__ float cross2(float ax, float ay, float bx, float by) { return ax * by - ay * bx; }

// ca/sa, cb/sb: cos/sin of each box's heading (computed once per box).
__device__ float rotated_overlap(const float* A, const float* B, float ca, float sa, float cb, float sb) {
  const float ra = 0.5f * sqrtf(A[3] * A[3] + A[4] * A[4]), rb = 0.5f * sqrtf(B[3] * B[3] + B[4] * B[4]);
  const float ddx = B[0] - A[0], ddy = B[1] - A[1];
  if (ddx * ddx + ddy * ddy > (ra + rb) * (ra + rb)) return 0.f;
  const float cr = cb * ca + sb * sa, sr = sb * ca - cb * sa;  // rotation of B relative to A
  const float bx = ca * ddx + sa * ddy, by = -sa * ddx + ca * ddy;
  const float ahx = 0.5f * A[3], ahy = 0.5f * A[4], bhx = 0.5f * B[3], bhy = 0.5f * B[4];
  // B's corners in A's frame, CCW
  float qx[4], qy[4];
  {
    const float ox[4] = {-bhx, bhx, bhx, -bhx}, oy[4] = {-bhy, -bhy, bhy, bhy};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      qx[i] = bx + cr * ox[i] - sr * oy[i];
      qy[i] = by + sr * ox[i] + cr * oy[i];
    }
  }
  float area2 = 0.f;
  // B's edges clipped to A's box (open): Liang–Barsky
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float px = qx[i], py = qy[i], dx = qx[(i + 1) & 3] - px, dy = qy[(i + 1) & 3] - py;
    float t0 = 0.f, t1 = 1.f;
    // four constraints  -dx*t < px + ahx, dx*t < ahx - px, ... (strict)
    const float pp[4] = {-dx, dx, -dy, dy};
    const float qq[4] = {px + ahx, ahx - px, py + ahy, ahy - py};
    bool empty = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (pp[j] == 0.f) {
        if (qq[j] <= 0.f) empty = true;
      } else {
        const float r = qq[j] / pp[j];
        if (pp[j] < 0.f) t0 = fmaxf(t0, r);
        else t1 = fminf(t1, r);
      }
    }
    if (!empty && t0 < t1)
      area2 += cross2(px + t0 * dx, py + t0 * dy, px + t1 * dx, py + t1 * dy);
  }
  // A's edges clipped by B's half-planes (closed): Cyrus–Beck
  const float ax_[4] = {-ahx, ahx, ahx, -ahx}, ay_[4] = {-ahy, -ahy, ahy, ahy};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float px = ax_[i], py = ay_[i], qx2 = ax_[(i + 1) & 3], qy2 = ay_[(i + 1) & 3];
    float t0 = 0.f, t1 = 1.f;
    bool empty = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float ex = qx[(j + 1) & 3] - qx[j], ey = qy[(j + 1) & 3] - qy[j];
      const float sp = cross2(ex, ey, px - qx[j], py - qy[j]);
      const float sq = cross2(ex, ey, qx2 - qx[j], qy2 - qy[j]);
      if (sp < 0.f && sq < 0.f) empty = true;
      else if (sp == 0.f && sq == 0.f) {
        // collinear with B's edge j: part of A∩B's boundary only if both edges
        // run the same way (A, B on the same side); touching from outside -> 0
        if (ex * (qx2 - px) + ey * (qy2 - py) < 0.f) empty = true;
      } else if (sp < 0.f) t0 = fmaxf(t0, sp / (sp - sq));
      else if (sq < 0.f) t1 = fminf(t1, sp / (sp - sq));
    }
    if (!empty && t0 < t1) {
      const float dx = qx2 - px, dy = qy2 - py;
      area2 += cross2(px + t0 * dx, py + t0 * dy, px + t1 * dx, py + t1 * dy);
    }
  }
  return fmaxf(0.5f * area2, 0.f);
}

__device__ __forceinline__ float iou_bev(const float* a, const float* c, float cos_a, float sin_a, float cos_c, float sin_c) {
  const float ov = rotated_overlap(a, c, cos_a, sin_a, cos_c, sin_c);
  const float sa = a[3] * a[4], sc = c[3] * c[4];
  return ov / fmaxf(sa + sc - ov, 1e-8f);
}

template <int MODE>  // 0 = axis-aligned 2D (box dim 4), 1 = rotated BEV (box dim >= 7)
__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ boxes, int box_dim,
                                                      const int* __restrict__ cls, const int* __restrict__ order,
                                                      const int* __restrict__ sorted_n, int cap, int pre_max,
                                                      int mask_words, float thr, int agnostic,
                                                      uint64_t* __restrict__ mask) {
  // one wave per block; tiles of 64 rows x 64 columns of the sorted list
  __shared__ float sbox[64][8];   // column boxes (+ [7] = circumradius for MODE 1)
  __shared__ float rbox[64][8];   // row boxes (MODE 1)
  __shared__ float scs[64][2], rcs[64][2];
  __shared__ int scls[64];
  __shared__ unsigned short pairs[64 * 64];
  __shared__ unsigned long long rowbits[64];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int n = sorted_n[b];
  const int nb = (n + 63) >> 6;
  const int* ob = order + (long)b * pre_max;
  const float* bb = boxes + (long)b * cap * box_dim;
  const int* cb_ = cls + (long)b * cap;
  uint64_t* mb = mask + (long)b * pre_max * mask_words;
  const int nbox = MODE == 0 ? 4 : 7;
  for (int t = blockIdx.x; t < nb * nb; t += gridDim.x) {
    const int rb = t / nb, cbk = t - rb * nb;
    if (cbk < rb) continue;
    const int j = cbk * 64 + tid;
    if (j < n) {
      const int s = ob[j];
      for (int d = 0; d < nbox; ++d) sbox[tid][d] = bb[(long)s * box_dim + d];
      scls[tid] = cb_[s];
      if (MODE == 1) {
        sincosf(sbox[tid][6], &scs[tid][1], &scs[tid][0]);
        sbox[tid][7] = 0.5f * sqrtf(sbox[tid][3] * sbox[tid][3] + sbox[tid][4] * sbox[tid][4]);
      }
    }
    const int i = rb * 64 + tid;
    if (MODE == 0) {
      __syncthreads();
      if (i < n) {
        const int s = ob[i];
        float me[4];
        for (int d = 0; d < 4; ++d) me[d] = bb[(long)s * box_dim + d];
        const int mc = cb_[s];
        uint64_t bits = 0;
        const int jmax = min(64, n - cbk * 64);
        for (int jj = 0; jj < jmax; ++jj) {
          const int jg = cbk * 64 + jj;
          if (jg <= i) continue;
          if (!agnostic && scls[jj] != mc) continue;
          if (iou_aa(me, sbox[jj]) > thr) bits |= (1ull << jj);
        }
        mb[(long)i * mask_words + cbk] = bits;
      }
      __syncthreads();
      continue;
    }
    // MODE 1: cheap circumcircle test over all 64x64 pairs, compact the
    // candidates (wave ballot + popcount), then evaluate only those densely.
    float rx = 0.f, ry = 0.f, rr = -1.f;
    int rc = 0;
    if (i < n) {
      const int s = ob[i];
      for (int d = 0; d < 7; ++d) rbox[tid][d] = bb[(long)s * box_dim + d];
      sincosf(rbox[tid][6], &rcs[tid][1], &rcs[tid][0]);
      rx = rbox[tid][0];
      ry = rbox[tid][1];
      rr = 0.5f * sqrtf(rbox[tid][3] * rbox[tid][3] + rbox[tid][4] * rbox[tid][4]);
      rc = cb_[s];
    }
    rowbits[tid] = 0ull;
    __syncthreads();
    int cnt = 0;  // wave-uniform
    const int jmax = min(64, n - cbk * 64);
    const unsigned long long lt = (tid == 0) ? 0ull : (~0ull >> (64 - tid));
    for (int jj = 0; jj < jmax; ++jj) {
      const int jg = cbk * 64 + jj;
      bool c = false;
      if (i < n && jg > i && (agnostic || scls[jj] == rc)) {
        const float dx = sbox[jj][0] - rx, dy = sbox[jj][1] - ry, rs = sbox[jj][7] + rr;
        c = dx * dx + dy * dy <= rs * rs;
      }
      const unsigned long long bal = __ballot(c);
      if (c) pairs[cnt + __popcll(bal & lt)] = (unsigned short)((tid << 6) | jj);
      cnt += __popcll(bal);
    }
    __syncthreads();
    for (int p = tid; p < cnt; p += 64) {
      const int r = pairs[p] >> 6, cc = pairs[p] & 63;
      const float v = iou_bev(rbox[r], sbox[cc], rcs[r][0], rcs[r][1], scs[cc][0], scs[cc][1]);
      if (v > thr) atomicOr(&rowbits[r], 1ull << cc);
    }
    __syncthreads();
    if (i < n) mb[(long)i * mask_words + cbk] = rowbits[tid];
    __syncthreads();
  }
}

struct OutXform {  // 2D: x' = (x - pad_x) / gain_x, clamp to [0, clip_w]
  float gain_x, gain_y, pad_x, pad_y, clip_w, clip_h;
  int enable;
};

__global__ void __launch_bounds__(256) nms_reduce_kernel(const int* __restrict__ order, const int* __restrict__ sorted_n,
                                                         const uint64_t* __restrict__ mask, int pre_max, int mask_words,
                                                         const float* __restrict__ boxes, int box_dim,
                                                         const float* __restrict__ scores, const int* __restrict__ cls,
                                                         int cap, int max_out, OutXform xf,
                                                         float* __restrict__ out_box, float* __restrict__ out_score,
                                                         int* __restrict__ out_cls, int* __restrict__ out_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* removed = (uint64_t*)smem;         // mask_words
  uint64_t* diag = removed + mask_words;       // 64
  int* kept = (int*)(diag + 64);               // 64
  int* s_cnt = kept + 64;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int n = sorted_n[b];
  const int nb = (n + 63) >> 6;
  const int* ob = order + (long)b * pre_max;
  const uint64_t* mb = mask + (long)b * pre_max * mask_words;
  for (int w = tid; w < mask_words; w += nt) removed[w] = 0;
  __syncthreads();
  int nkeep = 0;
  for (int rb = 0; rb < nb && nkeep < max_out; ++rb) {
    if (tid < 64) {
      const int i = rb * 64 + tid;
      diag[tid] = i < n ? mb[(long)i * mask_words + rb] : 0ull;
    }
    __syncthreads();
    if (tid == 0) {
      uint64_t word = removed[rb];
      int c = 0;
      const int lim = min(64, n - rb * 64);
      for (int k = 0; k < lim && nkeep + c < max_out; ++k) {
        if (!((word >> k) & 1ull)) {
          kept[c++] = rb * 64 + k;
          word |= diag[k];
        }
      }
      *s_cnt = c;
    }
    __syncthreads();
    const int c = *s_cnt;
    if (tid < c) {
      const int s = ob[kept[tid]];
      const long src = (long)b * cap + s;
      const long dst = (long)b * max_out + nkeep + tid;
      const float* bx = boxes + src * box_dim;
      float* ox = out_box + dst * box_dim;
      for (int d = 0; d < box_dim; ++d) ox[d] = bx[d];
      if (xf.enable) {
        ox[0] = fminf(fmaxf((bx[0] - xf.pad_x) / xf.gain_x, 0.f), xf.clip_w);
        ox[1] = fminf(fmaxf((bx[1] - xf.pad_y) / xf.gain_y, 0.f), xf.clip_h);
        ox[2] = fminf(fmaxf((bx[2] - xf.pad_x) / xf.gain_x, 0.f), xf.clip_w);
        ox[3] = fminf(fmaxf((bx[3] - xf.pad_y) / xf.gain_y, 0.f), xf.clip_h);
      }
      out_score[dst] = scores[src];
      out_cls[dst] = cls[src];
    }
    // OR the kept rows' masks into the removed set: all (row, word) loads in
    // flight at once, combined with LDS 64-bit atomics.
    const int words_left = nb - rb - 1;
    for (int t = tid; t < c * words_left; t += nt) {
      const int k = t / words_left, w = rb + 1 + t % words_left;
      const uint64_t v = mb[(long)kept[k] * mask_words + w];
      if (v) atomicOr((unsigned long long*)&removed[w], (unsigned long long)v);
    }
    nkeep += c;
    __syncthreads();
  }
  if (tid == 0) out_count[b] = nkeep;
}

}  // namespace

TCA_API int tca_topk_sort(const uint64_t* keys, const int* count, int batch, int cap, int pre_max, int* order,
                          int* sorted_n, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (pre_max > kSortCap) return (int)hipErrorInvalidValue;
  const size_t lds = sizeof(uint64_t) * kSortCap + sizeof(int) * (kSortCap + 256 + 4);
  topk_sort_kernel<<<batch, 1024, lds, stream>>>(keys, count, cap, pre_max, order, sorted_n);
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_nms_mask(int mode, const float* boxes, int box_dim, const int* cls, const int* order,
                         const int* sorted_n, int batch, int cap, int pre_max, float thr, int agnostic,
                         uint64_t* mask, int grid_per_image, hipStream_t stream) {
  if (batch <= 0) return 0;
  const int mask_words = (pre_max + 63) / 64;
  dim3 grid(grid_per_image > 0 ? grid_per_image : 256, batch);
  if (mode == 0)
    nms_mask_kernel<0><<<grid, 64, 0, stream>>>(boxes, box_dim, cls, order, sorted_n, cap, pre_max, mask_words, thr,
                                                agnostic, mask);
  else
    nms_mask_kernel<1><<<grid, 64, 0, stream>>>(boxes, box_dim, cls, order, sorted_n, cap, pre_max, mask_words, thr,
                                                agnostic, mask);
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_nms_reduce(const int* order, const int* sorted_n, const uint64_t* mask, int batch, int pre_max,
                           const float* boxes, int box_dim, const float* scores, const int* cls, int cap, int max_out,
                           const float* xform /*host [6] or null*/, float* out_box, float* out_score, int* out_cls,
                           int* out_count, hipStream_t stream) {
  if (batch <= 0) return 0;
  const int mask_words = (pre_max + 63) / 64;
  OutXform xf{1.f, 1.f, 0.f, 0.f, 0.f, 0.f, 0};
  if (xform) { xf = OutXform{xform[0], xform[1], xform[2], xform[3], xform[4], xform[5], 1}; }
  const size_t lds = sizeof(uint64_t) * (mask_words + 64) + sizeof(int) * (64 + 4);
  nms_reduce_kernel<<<batch, 256, lds, stream>>>(order, sorted_n, mask, pre_max, mask_words, boxes, box_dim, scores, cls,
                                                 cap, max_out, xf, out_box, out_score, out_cls, out_count);
  TCA_LAUNCH_CHECK();
}

// Pairwise IoU matrix for evaluation (K14, reference evaluate_inference.py:408-410,
// base_postprocess.py:48-70): iou[i][j] for a [N,4] x b [M,4] xyxy.
namespace {
__global__ void box_iou_kernel(const float* __restrict__ a, int n, const float* __restrict__ c, int m,
                               float* __restrict__ out) {
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long)n * m) return;
  const int i = (int)(g / m), j = (int)(g - (long)i * m);
  out[g] = iou_aa(a + 4 * i, c + 4 * j);
}
}  // namespace

TCA_API int tca_box_iou(const float* a, int n, const float* b, int m, float* out, hipStream_t stream) {
  if (n <= 0 || m <= 0) return 0;
  const long t = (long)n * m;
  box_iou_kernel<<<(unsigned)((t + 255) / 256), 256, 0, stream>>>(a, n, b, m, out);
  TCA_LAUNCH_CHECK();
}
