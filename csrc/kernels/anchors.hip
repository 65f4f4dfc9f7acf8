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

template <typename T>
__global__ void __launch_bounds__(256) anchor_decode_kernel(
    const T* __restrict__ cls, const T* __restrict__ box, const T* __restrict__ dir, int layout, int H, int W, int A,
    int C, int bins, int ld_cls, int ld_box, int ld_dir, AnchorTable tb, float x0, float xs, float y0, float ys, float dir_offset, float dir_limit_offset,
    float score_thresh, float* __restrict__ cand_box, float* __restrict__ cand_score, int* __restrict__ cand_label,
    uint64_t* __restrict__ cand_key, int* __restrict__ cand_count, int cap) {
  __shared__ int s_cnt, s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int b = blockIdx.y;
  const int aidx = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = H * W * A;
  bool pass = false;
  float score = 0.f;
  int label = 0;
  float out[7];
  if (aidx < total) {
    const int a = aidx % A;
    const int yx = aidx / A;
    const int y = yx / W, x = yx - y * W;
    // NCHW: nch channels; NHWC: channel stride ld (a slice of a wider tensor)
    auto at = [&](const T* base, int nch, int ld, int ch) -> float {
      long off = layout == 0 ? (((long)b * nch + ch) * H + y) * W + x : (((long)b * H + y) * W + x) * ld + ch;
      return to_f32(base[off]);
    };
    float best = -INFINITY;
    int bc = 0;
    for (int c = 0; c < C; ++c) {
      const float v = at(cls, A * C, ld_cls, a * C + c);
      if (v > best) { best = v; bc = c; }
    }
    score = sigmoidf_(best);
    label = bc + 1;
    if (score >= score_thresh) {
      pass = true;
      const float* t = tb.v[a];
      const float xa = x0 + x * xs, ya = y0 + y * ys, za = t[3];
      const float dxa = t[0], dya = t[1], dza = t[2], ra = t[4], diag = t[5];
      float e[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) e[k] = at(box, A * 7, ld_box, a * 7 + k);
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
          const float v = at(dir, A * bins, ld_dir, a * bins + d);
          if (v > bd) { bd = v; dl = d; }
        }
        const float period = 2.f * 3.14159265358979f / (float)bins;
        const float val = rg - dir_offset;
        const float lim = val - floorf(val / period + dir_limit_offset) * period;
        rg = lim + dir_offset + period * (float)dl;
      }
      out[6] = rg;
    }
  }
  int my = -1;
  if (pass) my = atomicAdd(&s_cnt, 1);
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&cand_count[b], s_cnt) : 0;
  __syncthreads();
  if (pass) {
    const int slot = s_base + my;
    if (slot < cap) {
      const long o = (long)b * cap + slot;
#pragma unroll
      for (int k = 0; k < 7; ++k) cand_box[o * 7 + k] = out[k];
      cand_score[o] = score;
      cand_label[o] = label;
      cand_key[o] = make_score_key(score, (uint32_t)aidx);
    }
  }
}

}  // namespace

// table: host [A][6] (dxa, dya, dza, za, rot, diag).
TCA_API int tca_anchor_decode_filter(const void* cls, const void* box, const void* dir, int dtype, int layout, int batch,
                                     int H, int W, int A, int C, int bins, int ld_cls, int ld_box, int ld_dir,
                                     const float* table, float x0, float xs,
                                     float y0, float ys, float dir_offset, float dir_limit_offset, float score_thresh,
                                     float* cand_box, float* cand_score, int* cand_label, uint64_t* cand_key,
                                     int* cand_count, int cap, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (A > 8) return (int)hipErrorInvalidValue;
  AnchorTable tb;
  for (int a = 0; a < 8; ++a)
    for (int k = 0; k < 6; ++k) tb.v[a][k] = a < A ? table[a * 6 + k] : 0.f;
  int e = zero_i32_async(cand_count, batch, stream);
  if (e) return e;
  dim3 grid((H * W * A + 255) / 256, batch);
#define LAUNCH(T)                                                                                              \
  anchor_decode_kernel<T><<<grid, 256, 0, stream>>>((const T*)cls, (const T*)box, (const T*)dir, layout, H, W, A, C, \
                                                    bins, ld_cls > 0 ? ld_cls : A * C, ld_box > 0 ? ld_box : A * 7,  \
                                                    ld_dir > 0 ? ld_dir : A * bins, tb, x0, xs, y0, ys, dir_offset, dir_limit_offset,          \
                                                    score_thresh, cand_box, cand_score, cand_label, cand_key,        \
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
