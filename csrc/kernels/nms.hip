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

#include <cstdlib>

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
      // In the high passes nearly every key shares one digit (scores in a
      // narrow band), and 64 lanes adding to one LDS word serialise: fold each
      // wave's dominant digits into one atomic each, the rest go direct.
      const int lane = tid & 63;
      for (int i0 = 0; i0 < n; i0 += nt) {  // uniform trip count: every lane reaches the ballots
        const int i = i0 + tid;
        bool m = false;
        int d = 0;
        if (i < n) {
          const uint64_t key = kb[i];
          m = (key & pmask) == prefix;
          d = (int)((key >> shift) & 255);
        }
        for (int round = 0; round < 2; ++round) {
          const unsigned long long mm = __ballot(m);
          if (!mm) break;
          const int leader = __ffsll(mm) - 1;
          const int dl = __shfl(d, leader, 64);
          const unsigned long long same = __ballot(m && d == dl);
          if (lane == leader) atomicAdd(&hist[dl], __popcll(same));
          if (d == dl) m = false;
        }
        if (m) atomicAdd(&hist[d], 1);
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
__device__ __forceinline__ float rotated_overlap(const float* A, const float* B, float ca, float sa, float cb, float sb) {
  const float ra = 0.5f * sqrtf(A[3] * A[3] + A[4] * A[4]), rb = 0.5f * sqrtf(B[3] * B[3] + B[4] * B[4]);
  const float ddx = B[0] - A[0], ddy = B[1] - A[1];
  if (ddx * ddx + ddy * ddy > (ra + rb) * (ra + rb)) return 0.f;
  const float cr = cb * ca + sb * sa, sr = sb * ca - cb * sa;  // rotation of B relative to A
  const float bx = ca * ddx + sa * ddy, by = -sa * ddx + ca * ddy;
  const float ahx = 0.5f * A[3], ahy = 0.5f * A[4], bhx = 0.5f * B[3], bhy = 0.5f * B[4];
  {  // separating-axis test on the four box axes: a strict separation means zero overlap (exact early-out)
    const float acr = fabsf(cr), asr = fabsf(sr);
    const float dxb = cb * ddx + sb * ddy, dyb = -sb * ddx + cb * ddy;
    if (fabsf(bx) > ahx + bhx * acr + bhy * asr || fabsf(by) > ahy + bhx * asr + bhy * acr ||
        fabsf(dxb) > bhx + ahx * acr + ahy * asr || fabsf(dyb) > bhy + ahx * asr + ahy * acr)
      return 0.f;
  }
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
        const float r = __fdividef(qq[j], pp[j]);
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
      } else if (sp < 0.f) t0 = fmaxf(t0, __fdividef(sp, sp - sq));
      else if (sq < 0.f) t1 = fminf(t1, __fdividef(sp, sp - sq));
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

// ---- rotated BEV mask, v2 ----------------------------------------------------
// A prepass writes each sorted candidate once, packed: P0 = (x, y, aabb
// half-extents ex, ey), P1 = (w, l, cos, sin), and its class, so the tile
// kernel's loads are coalesced and no tile recomputes a sincos or chases
// order -> box.  One wave per upper-triangle 64x64 tile: lane = row; each
// column is one broadcast ds_read_b128 and an AABB-overlap test (~8 VALU),
// ballot-compacted in quarters of 16 columns into an LDS pair list; only the
// surviving pairs run the exact rotated IoU (itself SAT-gated).
// soa layout per image (st = pre_max rounded up to 4): float4 P0[st], float4 P1[st], int cls[st].
__global__ void __launch_bounds__(256) nms_prep_rot_kernel(const float* __restrict__ boxes, int box_dim,
                                                           const int* __restrict__ cls, const int* __restrict__ order,
                                                           const int* __restrict__ sorted_n, int cap, int pre_max,
                                                           int st, float* __restrict__ soa) {
  const int b = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  if (i >= sorted_n[b]) return;
  const int s = order[(long)b * pre_max + i];
  const float* bx = boxes + ((long)b * cap + s) * box_dim;
  float* base = soa + (long)b * 9 * st;
  const float w = bx[3], l = bx[4];
  float sn, cs;
  sincosf(bx[6], &sn, &cs);
  reinterpret_cast<float4*>(base)[i] =
      make_float4(bx[0], bx[1], 0.5f * (fabsf(cs) * w + fabsf(sn) * l), 0.5f * (fabsf(sn) * w + fabsf(cs) * l));
  reinterpret_cast<float4*>(base + 4 * st)[i] = make_float4(w, l, cs, sn);
  reinterpret_cast<int*>(base + 8 * st)[i] = cls[(long)b * cap + s];
}

template <bool AGN>
__global__ void __launch_bounds__(256) nms_mask_rot_kernel(const float* __restrict__ soa,
                                                           const int* __restrict__ sorted_n, int pre_max, int st,
                                                           int mask_words, float thr, uint64_t* __restrict__ mask) {
  __shared__ float4 s_r0[4][64], s_r1[4][64], s_c0[4][64], s_c1[4][64];
  __shared__ int s_ccls[4][64];
  __shared__ unsigned short s_pairs[4][64 * 16];
  __shared__ unsigned long long s_bits[4][64];
  const int b = blockIdx.y, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = sorted_n[b], nb = (n + 63) >> 6;
  const int t = blockIdx.x * 4 + wid;
  if (t >= nb * (nb + 1) / 2) return;  // wave-uniform; the kernel has no block-wide barrier
  int rb = 0, rem = t;
  while (rem >= nb - rb) { rem -= nb - rb; ++rb; }
  const int cbk = rb + rem;
  const float* base = soa + (long)b * 9 * st;
  const float4* P0 = reinterpret_cast<const float4*>(base);
  const float4* P1 = reinterpret_cast<const float4*>(base + 4 * st);
  const int* PC = reinterpret_cast<const int*>(base + 8 * st);
  const int i = rb * 64 + lane, j = cbk * 64 + lane;
  const bool rok = i < n;
  // (branches, not selects: `c ? p[i] : zero` makes hipcc spill the zero and select a pointer)
  float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, c0 = r0, c1 = r0;
  int rcls = -1, ccls = -2;
  if (rok) { r0 = P0[i]; r1 = P1[i]; rcls = PC[i]; }
  if (j < n) { c0 = P0[j]; c1 = P1[j]; ccls = PC[j]; }
  s_r0[wid][lane] = r0;
  s_r1[wid][lane] = r1;
  s_c0[wid][lane] = c0;
  s_c1[wid][lane] = c1;
  if (!AGN) s_ccls[wid][lane] = ccls;
  s_bits[wid][lane] = 0ull;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  const int jmax = min(64, n - cbk * 64);
  const int jlo = cbk == rb ? lane : -1;  // diagonal tile: only columns after the row
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  unsigned short* pairs = s_pairs[wid];
  const float4* C0 = s_c0[wid];
  for (int q0 = 0; q0 < jmax; q0 += 16) {
    int cnt = 0;  // wave-uniform
    const int qe = min(q0 + 16, jmax);
    for (int jj = q0; jj < qe; ++jj) {
      const float4 c = C0[jj];
      bool hit = rok && jj > jlo && fabsf(c.x - r0.x) < c.z + r0.z && fabsf(c.y - r0.y) < c.w + r0.w;
      if (!AGN) hit = hit && s_ccls[wid][jj] == rcls;
      const unsigned long long bal = __ballot(hit);
      if (hit) pairs[cnt + __popcll(bal & lt)] = (unsigned short)((lane << 6) | jj);
      cnt += __popcll(bal);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    for (int p = lane; p < cnt; p += 64) {
      const int r = pairs[p] >> 6, cc = pairs[p] & 63;
      const float4 a0 = s_r0[wid][r], a1 = s_r1[wid][r], b0 = C0[cc], b1 = s_c1[wid][cc];
      const float A[5] = {a0.x, a0.y, 0.f, a1.x, a1.y};
      const float Bx[5] = {b0.x, b0.y, 0.f, b1.x, b1.y};
      const float ov = rotated_overlap(A, Bx, a1.z, a1.w, b1.z, b1.w);
      if (ov > 0.f && ov / fmaxf(a1.x * a1.y + b1.x * b1.y - ov, 1e-8f) > thr) atomicOr(&s_bits[wid][r], 1ull << cc);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  if (rok) mask[((long)b * pre_max + i) * mask_words + cbk] = s_bits[wid][lane];
}

struct OutXform {  // 2D: x' = (x - pad_x) / gain_x, clamp to [0, clip_w]
  float gain_x, gain_y, pad_x, pad_y, clip_w, clip_h;
  int enable;
};

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int k) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, k);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), k);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, o), hi = __shfl_xor((int)(uint32_t)(v >> 32), o);
    v |= ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Greedy reduce over the suppression bitmask, one wave per image, RB 64-row
// blocks per memory round.  Round r loads (a) for each of its RB row blocks,
// the rows' own words of the round's blocks (lane k = row k of the block;
// upper triangle only) and (b) the round's words of every row kept so far,
// OR-reduced over the wave.  The blocks are then resolved in order entirely
// in registers: the next kept row is ctz(~removed), and its suppression words
// for the rest of the round come from its lane by readlane.  One dependent
// memory round per RB*64 candidates instead of one per 64 with block barriers.
template <int RB>
__global__ void __launch_bounds__(64) nms_reduce_wave_kernel(const int* __restrict__ order,
                                                             const int* __restrict__ sorted_n,
                                                             const uint64_t* __restrict__ mask, int pre_max,
                                                             int mask_words, const float* __restrict__ boxes,
                                                             int box_dim, const float* __restrict__ scores,
                                                             const int* __restrict__ cls, int cap, int max_out,
                                                             OutXform xf, float* __restrict__ out_box,
                                                             float* __restrict__ out_score, int* __restrict__ out_cls,
                                                             int* __restrict__ out_count) {
  __shared__ int s_kept[kSortCap];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = sorted_n[b], nb = (n + 63) >> 6;
  const uint64_t* mb = mask + (long)b * pre_max * mask_words;
  int nkeep = 0;
  for (int rb0 = 0; rb0 < nb && nkeep < max_out; rb0 += RB) {
    uint64_t M[RB][RB], P[RB];
#pragma unroll
    for (int c = 0; c < RB; ++c) {
      P[c] = 0ull;
      const int row = (rb0 + c) * 64 + lane;
#pragma unroll
      for (int w = 0; w < RB; ++w) {
        M[c][w] = 0ull;
        if (w >= c && rb0 + w < nb && row < n) M[c][w] = mb[(long)row * mask_words + rb0 + w];
      }
    }
    for (int j = lane; j < nkeep; j += 64) {
      const long row = s_kept[j];
#pragma unroll
      for (int w = 0; w < RB; ++w)
        if (rb0 + w < nb) P[w] |= mb[row * mask_words + rb0 + w];
    }
#pragma unroll
    for (int w = 0; w < RB; ++w) P[w] = wave_or64(P[w]);
#pragma unroll
    for (int c = 0; c < RB; ++c) {
      if (rb0 + c >= nb || nkeep >= max_out) break;
      const int lim = min(64, n - (rb0 + c) * 64);
      const uint64_t valid = lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
      uint64_t word = P[c];
      uint64_t avail = ~word & valid;
      while (avail != 0ull && nkeep < max_out) {
        const int k = __builtin_amdgcn_readfirstlane(__builtin_ctzll(avail));
        if (lane == 0) s_kept[nkeep] = (rb0 + c) * 64 + k;
        ++nkeep;
        word |= readlane64(M[c][c], k) | (1ull << k);
#pragma unroll
        for (int w = c + 1; w < RB; ++w) P[w] |= readlane64(M[c][w], k);
        avail = ~word & valid;
      }
    }
    __syncthreads();  // s_kept (lane 0's writes) visible to the next round's loads
  }
  __syncthreads();
  for (int t = lane; t < nkeep; t += 64) {
    const int s = order[(long)b * pre_max + s_kept[t]];
    const long src = (long)b * cap + s;
    const long dst = (long)b * max_out + t;
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
  if (lane == 0) out_count[b] = nkeep;
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

// Rotated-BEV suppression mask, v2: soa is scratch [batch, 9, ceil4(pre_max)] fp32 (16-B aligned).
TCA_API int tca_nms_mask_rot(const float* boxes, int box_dim, const int* cls, const int* order, const int* sorted_n,
                             int batch, int cap, int pre_max, float thr, int agnostic, float* soa, uint64_t* mask,
                             hipStream_t stream) {
  if (batch <= 0) return 0;
  if (box_dim < 7) return (int)hipErrorInvalidValue;
  const int mask_words = (pre_max + 63) / 64;
  const int st = (pre_max + 3) & ~3;
  nms_prep_rot_kernel<<<dim3((pre_max + 255) / 256, batch), 256, 0, stream>>>(boxes, box_dim, cls, order, sorted_n,
                                                                             cap, pre_max, st, soa);
  const int tiles = mask_words * (mask_words + 1) / 2;
  const dim3 grid((tiles + 3) / 4, batch);
  if (agnostic) nms_mask_rot_kernel<true><<<grid, 256, 0, stream>>>(soa, sorted_n, pre_max, st, mask_words, thr, mask);
  else nms_mask_rot_kernel<false><<<grid, 256, 0, stream>>>(soa, sorted_n, pre_max, st, mask_words, thr, mask);
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
  if (max_out > kSortCap) return (int)hipErrorInvalidValue;
  // 4 64-row blocks per memory round (8 measured within noise: profiles/r3/lpipe/README.md)
  nms_reduce_wave_kernel<4><<<batch, 64, 0, stream>>>(order, sorted_n, mask, pre_max, mask_words, boxes, box_dim,
                                                      scores, cls, cap, max_out, xf, out_box, out_score, out_cls,
                                                      out_count);
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

// ---- merge-NMS (K4m; reference clients/postprocess/yolov5_postprocess.py:111-117,
// `merge = True`): every kept box becomes the score-weighted mean of all the
// image's candidates of its class with IoU > thr (itself included), and with
// `redundant` a kept box that overlaps no other candidate is dropped.  Applied
// only when 1 < n < 3000 candidates, as in the reference.  Runs after
// tca_nms_reduce (called without an output transform): one workgroup per image,
// one wave per kept box, candidates streamed 64 at a time; kept results are then
// compacted in score order and mapped to the original frame.
namespace {
constexpr int kMergeMaxKept = 1024;

__global__ void __launch_bounds__(256) nms_merge_kernel(const float* __restrict__ kbox, const float* __restrict__ kscore,
                                                        const int* __restrict__ kcls, const int* __restrict__ kcount,
                                                        const float* __restrict__ cbox, const float* __restrict__ cscore,
                                                        const int* __restrict__ ccls, const int* __restrict__ ccount,
                                                        int cap, int max_out, float thr, int agnostic, int redundant,
                                                        OutXform xf, float* __restrict__ out_box,
                                                        float* __restrict__ out_score, int* __restrict__ out_cls,
                                                        int* __restrict__ out_count) {
  __shared__ float mbox[kMergeMaxKept][4];
  __shared__ int keep_flag[kMergeMaxKept];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int nk = min(kcount[b], max_out);
  const int n = min(ccount[b], cap);
  const bool merge = ccount[b] > 1 && ccount[b] < 3000;  // the reference's 1 < n < 3E3
  const float* kb = kbox + (long)b * max_out * 4;
  const float* cb = cbox + (long)b * cap * 4;
  for (int k = wid; k < nk; k += nw) {
    float me[4] = {kb[4 * k], kb[4 * k + 1], kb[4 * k + 2], kb[4 * k + 3]};
    const int mc = kcls[(long)b * max_out + k];
    float sw = 0.f, sx1 = 0.f, sy1 = 0.f, sx2 = 0.f, sy2 = 0.f;
    int hits = 0;
    if (merge) {
      for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        if (j < n && (agnostic || ccls[(long)b * cap + j] == mc)) {
          const float* c = cb + 4 * (long)j;
          if (iou_aa(me, c) > thr) {
            const float w = cscore[(long)b * cap + j];
            sw += w;
            sx1 += w * c[0]; sy1 += w * c[1]; sx2 += w * c[2]; sy2 += w * c[3];
            ++hits;
          }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        sw += __shfl_xor(sw, o); sx1 += __shfl_xor(sx1, o); sy1 += __shfl_xor(sy1, o);
        sx2 += __shfl_xor(sx2, o); sy2 += __shfl_xor(sy2, o); hits += __shfl_xor(hits, o);
      }
    }
    if (lane == 0) {
      if (merge && sw > 0.f) {
        me[0] = sx1 / sw; me[1] = sy1 / sw; me[2] = sx2 / sw; me[3] = sy2 / sw;
      }
      mbox[k][0] = me[0]; mbox[k][1] = me[1]; mbox[k][2] = me[2]; mbox[k][3] = me[3];
      keep_flag[k] = !(merge && redundant && hits <= 1);
    }
  }
  __syncthreads();
  if (wid != 0) return;
  // compaction in score order: wave 0, 64 kept boxes per round, ballot prefix
  int base = 0;
  for (int k0 = 0; k0 < nk; k0 += 64) {
    const int k = k0 + lane;
    const bool f = k < nk && keep_flag[k];
    const uint64_t bal = __ballot(f);
    const int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
    if (f) {
      float x1 = mbox[k][0], y1 = mbox[k][1], x2 = mbox[k][2], y2 = mbox[k][3];
      if (xf.enable) {
        x1 = fminf(fmaxf((x1 - xf.pad_x) / xf.gain_x, 0.f), xf.clip_w);
        x2 = fminf(fmaxf((x2 - xf.pad_x) / xf.gain_x, 0.f), xf.clip_w);
        y1 = fminf(fmaxf((y1 - xf.pad_y) / xf.gain_y, 0.f), xf.clip_h);
        y2 = fminf(fmaxf((y2 - xf.pad_y) / xf.gain_y, 0.f), xf.clip_h);
      }
      float* o = out_box + ((long)b * max_out + pos) * 4;
      o[0] = x1; o[1] = y1; o[2] = x2; o[3] = y2;
      out_score[(long)b * max_out + pos] = kscore[(long)b * max_out + k];
      out_cls[(long)b * max_out + pos] = kcls[(long)b * max_out + k];
    }
    base += __popcll(bal);
  }
  if (lane == 0) out_count[b] = base;
}
}  // namespace

// kbox/kscore/kcls/kcount: tca_nms_reduce output (model coordinates, xform
// null); cbox/cscore/ccls/ccount: the candidates it ran on (xyxy, box_dim 4).
// Outputs must not alias the kept inputs.
TCA_API int tca_nms_merge(const float* kbox, const float* kscore, const int* kcls, const int* kcount,
                          const float* cbox, const float* cscore, const int* ccls, const int* ccount, int batch,
                          int cap, int max_out, float thr, int agnostic, int redundant,
                          const float* xform /*host [6] or null*/, float* out_box, float* out_score, int* out_cls,
                          int* out_count, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (max_out > kMergeMaxKept) return (int)hipErrorInvalidValue;
  OutXform xf{1.f, 1.f, 0.f, 0.f, 0.f, 0.f, 0};
  if (xform) { xf = OutXform{xform[0], xform[1], xform[2], xform[3], xform[4], xform[5], 1}; }
  nms_merge_kernel<<<batch, 256, 0, stream>>>(kbox, kscore, kcls, kcount, cbox, cscore, ccls, ccount, cap, max_out,
                                              thr, agnostic, redundant, xf, out_box, out_score, out_cls, out_count);
  TCA_LAUNCH_CHECK();
}
