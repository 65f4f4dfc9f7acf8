// K3 — YOLOv5 Detect decode fused with the candidate filter
// (reference: clients/postprocess/yolov5_postprocess.py:36-92 — obj > conf_thres,
// cls *= obj, xywh2xyxy, best class (or multi-label), conf > conf_thres, class filter;
// the decode itself is what the exported ONNX model does inside the server).
//
// Reads the three raw head maps (NCHW or NHWC, fp32/fp16/bf16) directly, so
// the 25200 x 85 decoded tensor never has to exist on the hot path.  One
// thread per (image, level, anchor, y, x): objectness is read first and the
// 80 class logits only for the few cells that pass — argmax over logits is
// argmax over sigmoids, so only one extra sigmoid per passing cell.
// Passing candidates are stream-compacted per image with one LDS counter and
// one global atomic per block; a 64-bit key (score, ~anchor index) makes the
// later sort deterministic although slot order is not.
//
// Optionally (decoded != nullptr) every cell's full decoded row is written
// as fp32 [B, N, 5+nc] — the KServe output contract of the reference's ONNX
// YOLOv5 (examples/YOLOv5/config.pbtxt:13-18) served by our own server.
#include "tca_common.h"

using namespace tca;

namespace {

struct YoloHeads {
  const void* head[3];
  int h[3], w[3], stride[3];
  int ldc[3];  // NHWC channel stride per level (>= na*(5+nc)); ignored for NCHW
  float anchor[3][4][2];  // up to 4 anchors per level
};

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i) { return to_f32(p[i]); }

template <typename T>
__global__ void __launch_bounds__(256) yolo_filter_kernel(YoloHeads hd, int layout, int batch, int na, int nc,
                                                          float conf_thres, int multi_label,
                                                          const uint32_t* __restrict__ class_mask,
                                                          float* __restrict__ cand_box, float* __restrict__ cand_score,
                                                          int* __restrict__ cand_cls, uint64_t* __restrict__ cand_key,
                                                          int* __restrict__ cand_count, int cap,
                                                          float* __restrict__ decoded) {
  __shared__ int s_cnt, s_base;
  const int no = nc + 5;
  const int C = na * no;
  const int n0 = na * hd.h[0] * hd.w[0], n1 = na * hd.h[1] * hd.w[1], n2 = na * hd.h[2] * hd.w[2];
  const int N = n0 + n1 + n2;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int b = blockIdx.y;
  const int aidx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = aidx < N;

  // Candidate production: up to nc per thread in multi-label mode, 1 otherwise.
  float box[4] = {0.f, 0.f, 0.f, 0.f};
  float best = -1.f;
  int best_c = 0;
  bool pass = false;
  int l = 0, rem = live ? aidx : 0;
  if (rem >= n0) { rem -= n0; l = 1; if (rem >= n1) { rem -= n1; l = 2; } }
  const int H = hd.h[l], W = hd.w[l];
  const int a = rem / (H * W);
  const int yx = rem - a * H * W;
  const int y = yx / W, x = yx - y * W;
  const T* hp = (const T*)hd.head[l];
  long base, cstride;
  if (layout == 0) {  // NCHW
    base = ((long)b * C + (long)a * no) * H * W + yx;
    cstride = (long)H * W;
  } else {  // NHWC
    base = ((long)b * H * W + yx) * hd.ldc[l] + (long)a * no;
    cstride = 1;
  }
  float obj = 0.f;
  if (live) {
    obj = sigmoidf_(ld(hp, base + 4 * cstride));
    const bool need_full = decoded != nullptr;
    if (obj > conf_thres || need_full) {
      const float sx = sigmoidf_(ld(hp, base)), sy = sigmoidf_(ld(hp, base + cstride));
      const float sw = sigmoidf_(ld(hp, base + 2 * cstride)), sh = sigmoidf_(ld(hp, base + 3 * cstride));
      const float st = (float)hd.stride[l];
      const float cx = (sx * 2.f - 0.5f + (float)x) * st;
      const float cy = (sy * 2.f - 0.5f + (float)y) * st;
      const float bw = (sw * 2.f) * (sw * 2.f) * hd.anchor[l][a][0];
      const float bh = (sh * 2.f) * (sh * 2.f) * hd.anchor[l][a][1];
      box[0] = cx - bw * 0.5f; box[1] = cy - bh * 0.5f; box[2] = cx + bw * 0.5f; box[3] = cy + bh * 0.5f;
      if (need_full) {
        float* drow = decoded + ((long)b * N + aidx) * no;
        drow[0] = cx; drow[1] = cy; drow[2] = bw; drow[3] = bh; drow[4] = obj;
        for (int c = 0; c < nc; ++c) drow[5 + c] = sigmoidf_(ld(hp, base + (5 + c) * cstride));
      }
      if (obj > conf_thres && !multi_label) {
        float m = -INFINITY;
        int mc = 0;
        // best over ALL classes, then the class filter drops the row (reference
        // yolov5_postprocess.py:87-92: max first, `classes` filter after)
        for (int c = 0; c < nc; ++c) {
          float v = ld(hp, base + (5 + c) * cstride);
          if (v > m) { m = v; mc = c; }
        }
        if (m > -INFINITY) {
          best = sigmoidf_(m) * obj;
          best_c = mc;
          pass = best > conf_thres && !(class_mask && !((class_mask[mc >> 5] >> (mc & 31)) & 1u));
        }
      }
    }
  }

  if (!multi_label) {
    // block-level compaction: one LDS atomic per passing thread, one global per block
    int my = -1;
    if (pass) my = atomicAdd(&s_cnt, 1);
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&cand_count[b], s_cnt) : 0;
    __syncthreads();
    if (pass) {
      int slot = s_base + my;
      if (slot < cap) {
        long o = (long)b * cap + slot;
        cand_box[o * 4 + 0] = box[0]; cand_box[o * 4 + 1] = box[1];
        cand_box[o * 4 + 2] = box[2]; cand_box[o * 4 + 3] = box[3];
        cand_score[o] = best; cand_cls[o] = best_c; cand_key[o] = make_score_key(best, (uint32_t)aidx);
      }
    }
  } else if (live && obj > conf_thres) {
    for (int c = 0; c < nc; ++c) {
      if (class_mask && !((class_mask[c >> 5] >> (c & 31)) & 1u)) continue;
      float s = sigmoidf_(ld(hp, base + (5 + c) * cstride)) * obj;
      if (s > conf_thres) {
        int slot = atomicAdd(&cand_count[b], 1);
        if (slot < cap) {
          long o = (long)b * cap + slot;
          cand_box[o * 4 + 0] = box[0]; cand_box[o * 4 + 1] = box[1];
          cand_box[o * 4 + 2] = box[2]; cand_box[o * 4 + 3] = box[3];
          cand_score[o] = s; cand_cls[o] = c; cand_key[o] = make_score_key(s, (uint32_t)(aidx * nc + c));
        }
      }
    }
  }
}

// Decode only (the ONNX YOLOv5 output [B, N, 5 + nc], what a served YOLOv5 returns): every
// output element is a function of one head element, so thread = 4 consecutive output floats
// (one 16-B store; consecutive threads write consecutive bytes) and the reads walk each row's
// channels in order.  yolo_filter_kernel's decoded path (thread = row) wrote 85 floats per
// thread at a 340-B stride across the wave, one cache line per lane per store.
// The last thread of an output whose size is not a multiple of 4 (e.g. img 416 / 608 at batch 1:
// N = 10647 / 22743 rows of 85) writes its 1-3 leftover floats with scalar stores.
template <typename T>
__global__ void __launch_bounds__(256) yolo_decode_kernel(YoloHeads hd, int layout, int na, int nc, long total,
                                                          float* __restrict__ decoded) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q * 4 >= total) return;
  const int no = nc + 5, C = na * no;
  const int n0 = na * hd.h[0] * hd.w[0], n1 = na * hd.h[1] * hd.w[1], n2 = na * hd.h[2] * hd.w[2];
  const long N = (long)n0 + n1 + n2;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long f = q * 4 + e;
    if (f >= total) { v[e] = 0.f; continue; }
    const long row = f / no;
    const int c = (int)(f - row * no);
    const int b = (int)(row / N);
    int rem = (int)(row - (long)b * N), l = 0;
    if (rem >= n0) { rem -= n0; l = 1; if (rem >= n1) { rem -= n1; l = 2; } }
    const int H = hd.h[l], W = hd.w[l];
    const int a = rem / (H * W), yx = rem - a * (H * W);
    const T* hp = (const T*)hd.head[l];
    const long idx = layout == 0 ? ((long)b * C + (long)a * no + c) * H * W + yx
                                 : ((long)b * H * W + yx) * hd.ldc[l] + (long)a * no + c;
    const float s = sigmoidf_(ld(hp, idx));
    const float st = (float)hd.stride[l];
    const int y = yx / W, x = yx - y * W;
    switch (c) {
      case 0: v[e] = (s * 2.f - 0.5f + (float)x) * st; break;
      case 1: v[e] = (s * 2.f - 0.5f + (float)y) * st; break;
      case 2: v[e] = (s * 2.f) * (s * 2.f) * hd.anchor[l][a][0]; break;
      case 3: v[e] = (s * 2.f) * (s * 2.f) * hd.anchor[l][a][1]; break;
      default: v[e] = s;
    }
  }
  if (q * 4 + 4 <= total) {
    *reinterpret_cast<float4*>(decoded + q * 4) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int e = 0; q * 4 + e < total; ++e) decoded[q * 4 + e] = v[e];
  }
}

}  // namespace

TCA_API int tca_yolo_decode(const void* head0, const void* head1, const void* head2, int dtype, int layout, int batch,
                            int na, int nc, const int* hw /*[6]*/, const int* strides /*[3]*/,
                            const int* ldc /*[3] or null*/, const float* anchors /*[3][na][2] host*/, float* decoded,
                            hipStream_t stream) {
  if (batch <= 0) return 0;
  if (na > 4 || na <= 0) return (int)hipErrorInvalidValue;
  YoloHeads hd;
  hd.head[0] = head0; hd.head[1] = head1; hd.head[2] = head2;
  long N = 0;
  for (int l = 0; l < 3; ++l) {
    hd.h[l] = hw[2 * l]; hd.w[l] = hw[2 * l + 1]; hd.stride[l] = strides[l];
    hd.ldc[l] = ldc ? ldc[l] : na * (nc + 5);
    for (int a = 0; a < 4; ++a) {
      hd.anchor[l][a][0] = a < na ? anchors[(l * na + a) * 2] : 0.f;
      hd.anchor[l][a][1] = a < na ? anchors[(l * na + a) * 2 + 1] : 0.f;
    }
    N += (long)na * hd.h[l] * hd.w[l];
  }
  const long total = (long)batch * N * (nc + 5);
  if (((uintptr_t)decoded & 15) != 0) return (int)hipErrorInvalidValue;  // 16-B stores
  const long total4 = (total + 3) / 4;
  const int bs = 256;
  const unsigned grid = (unsigned)((total4 + bs - 1) / bs);
  switch (dtype) {
    case kF32: yolo_decode_kernel<float><<<grid, bs, 0, stream>>>(hd, layout, na, nc, total, decoded); break;
    case kF16: yolo_decode_kernel<__half><<<grid, bs, 0, stream>>>(hd, layout, na, nc, total, decoded); break;
    case kBF16:
      yolo_decode_kernel<__hip_bfloat16><<<grid, bs, 0, stream>>>(hd, layout, na, nc, total, decoded);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_yolo_decode_filter(const void* head0, const void* head1, const void* head2, int dtype, int layout,
                                   int batch, int na, int nc, const int* hw /*[6]*/, const int* strides /*[3]*/,
                                   const int* ldc /*[3] or null*/,
                                   const float* anchors /*[3][na][2] host*/, float conf_thres, int multi_label,
                                   const uint32_t* class_mask, float* cand_box, float* cand_score, int* cand_cls,
                                   uint64_t* cand_key, int* cand_count, int cap, float* decoded,
                                   hipStream_t stream) {
  if (batch <= 0) return 0;
  if (na > 4 || na <= 0) return (int)hipErrorInvalidValue;
  YoloHeads hd;
  hd.head[0] = head0; hd.head[1] = head1; hd.head[2] = head2;
  for (int l = 0; l < 3; ++l) {
    hd.h[l] = hw[2 * l]; hd.w[l] = hw[2 * l + 1]; hd.stride[l] = strides[l];
    hd.ldc[l] = ldc ? ldc[l] : na * (nc + 5);
    for (int a = 0; a < 4; ++a) {
      hd.anchor[l][a][0] = a < na ? anchors[(l * na + a) * 2] : 0.f;
      hd.anchor[l][a][1] = a < na ? anchors[(l * na + a) * 2 + 1] : 0.f;
    }
  }
  int e = zero_i32_async(cand_count, batch, stream);
  if (e) return e;
  long N = 0;
  for (int l = 0; l < 3; ++l) N += (long)na * hd.h[l] * hd.w[l];
  const int bs = 256;
  dim3 grid((unsigned)((N + bs - 1) / bs), (unsigned)batch);
  switch (dtype) {
    case kF32:
      yolo_filter_kernel<float><<<grid, bs, 0, stream>>>(hd, layout, batch, na, nc, conf_thres, multi_label, class_mask,
                                                         cand_box, cand_score, cand_cls, cand_key, cand_count, cap, decoded);
      break;
    case kF16:
      yolo_filter_kernel<__half><<<grid, bs, 0, stream>>>(hd, layout, batch, na, nc, conf_thres, multi_label, class_mask,
                                                          cand_box, cand_score, cand_cls, cand_key, cand_count, cap, decoded);
      break;
    case kBF16:
      yolo_filter_kernel<__hip_bfloat16><<<grid, bs, 0, stream>>>(hd, layout, batch, na, nc, conf_thres, multi_label,
                                                                  class_mask, cand_box, cand_score, cand_cls, cand_key,
                                                                  cand_count, cap, decoded);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  TCA_LAUNCH_CHECK();
}

// ============================================================================
// K3 on a *decoded* prediction — the remote client's postprocess
// (reference clients/postprocess/yolov5_postprocess.py:36-92 applied to the
// ModelInfer response, communicator/ros_inference.py:148).  The server's output
// lands in device memory by one H2D of the response bytes and is filtered here;
// candidates feed the same sort + bitmask NMS as the local pipeline.
//   kind 0 (YOLOv5 ONNX): pred [B, N, ld] rows (cx, cy, w, h, obj, cls[nc]) in
//          model-input pixels; obj > t, then best (cls * obj) > t, or every
//          class with cls * obj > t (multi_label); tie key = row (* nc + class).
//   kind 1 (YOLOv4 ONNX, examples/YOLOv4/config.pbtxt): boxes [B, N, 4]
//          normalised x1y1x2y2 (pred) + confs [B, N, nc] (conf); best conf > t
//          (tools/utils.py:166-233), boxes scaled to img_w x img_h.
// One thread per row: the row's first gate is one load (obj, kind 0), the
// class scan only runs for rows that pass it.  A class filter drops a row whose
// best class is masked (it never promotes a lower-scoring allowed class).  The products are fp32 like the
// reference's NumPy float32 ``x[:, 5:] *= x[:, 4:5]``, so the kept sets match.
// ============================================================================
namespace {

__global__ void __launch_bounds__(256) yolo_filter_decoded_kernel(
    const float* __restrict__ pred, const float* __restrict__ confs, int kind, int N, int ld, int nc,
    float conf_thres, int multi_label, const uint32_t* __restrict__ class_mask, float img_w, float img_h,
    float* __restrict__ cand_box, float* __restrict__ cand_score, int* __restrict__ cand_cls,
    uint64_t* __restrict__ cand_key, int* __restrict__ cand_count, int cap) {
  __shared__ int s_cnt, s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int b = blockIdx.y;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  bool pass = false;
  float box[4] = {0.f, 0.f, 0.f, 0.f}, best = 0.f;
  int best_c = 0;
  if (r < N) {
    if (kind == 0) {
      const float* row = pred + ((long)b * N + r) * ld;
      const float obj = row[4];
      if (obj > conf_thres) {
        const float cx = row[0], cy = row[1], hw = row[2] * 0.5f, hh = row[3] * 0.5f;
        box[0] = cx - hw; box[1] = cy - hh; box[2] = cx + hw; box[3] = cy + hh;
        if (!multi_label) {
          float m = -INFINITY;
          for (int c = 0; c < nc; ++c) {  // best over all classes, class filter after (see K3)
            const float v = row[5 + c] * obj;
            if (v > m) { m = v; best_c = c; }
          }
          best = m;
          pass = m > conf_thres && !(class_mask && !((class_mask[best_c >> 5] >> (best_c & 31)) & 1u));
        } else {
          for (int c = 0; c < nc; ++c) {
            if (class_mask && !((class_mask[c >> 5] >> (c & 31)) & 1u)) continue;
            const float s = row[5 + c] * obj;
            if (s > conf_thres) {
              const int slot = atomicAdd(&cand_count[b], 1);
              if (slot < cap) {
                const long o = (long)b * cap + slot;
                cand_box[o * 4 + 0] = box[0]; cand_box[o * 4 + 1] = box[1];
                cand_box[o * 4 + 2] = box[2]; cand_box[o * 4 + 3] = box[3];
                cand_score[o] = s; cand_cls[o] = c; cand_key[o] = make_score_key(s, (uint32_t)(r * nc + c));
              }
            }
          }
        }
      }
    } else {
      const float* cf = confs + ((long)b * N + r) * nc;
      float m = -INFINITY;
      for (int c = 0; c < nc; ++c) {
        const float v = cf[c];
        if (v > m) { m = v; best_c = c; }
      }
      if (m > conf_thres) {
        const float* bx = pred + ((long)b * N + r) * 4;
        box[0] = bx[0] * img_w; box[1] = bx[1] * img_h; box[2] = bx[2] * img_w; box[3] = bx[3] * img_h;
        best = m;
        pass = true;
      }
    }
  }
  if (multi_label && kind == 0) return;  // compacted above, one atomic per candidate
  int my = -1;
  if (pass) my = atomicAdd(&s_cnt, 1);
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&cand_count[b], s_cnt) : 0;
  __syncthreads();
  if (pass) {
    const int slot = s_base + my;
    if (slot < cap) {
      const long o = (long)b * cap + slot;
      cand_box[o * 4 + 0] = box[0]; cand_box[o * 4 + 1] = box[1];
      cand_box[o * 4 + 2] = box[2]; cand_box[o * 4 + 3] = box[3];
      cand_score[o] = best; cand_cls[o] = best_c; cand_key[o] = make_score_key(best, (uint32_t)r);
    }
  }
}

}  // namespace

TCA_API int tca_yolo_filter_decoded(const float* pred, const float* confs, int kind, int batch, int N, int ld, int nc,
                                    float conf_thres, int multi_label, const uint32_t* class_mask, float img_w,
                                    float img_h, float* cand_box, float* cand_score, int* cand_cls, uint64_t* cand_key,
                                    int* cand_count, int cap, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (N <= 0 || nc <= 0 || (kind == 0 && ld < nc + 5) || (kind == 1 && confs == nullptr) || kind < 0 || kind > 1)
    return (int)hipErrorInvalidValue;
  int e = zero_i32_async(cand_count, batch, stream);
  if (e) return e;
  dim3 grid((unsigned)((N + 255) / 256), (unsigned)batch);
  yolo_filter_decoded_kernel<<<grid, 256, 0, stream>>>(pred, confs, kind, N, ld, nc, conf_thres, multi_label,
                                                       class_mask, img_w, img_h, cand_box, cand_score, cand_cls,
                                                       cand_key, cand_count, cap);
  TCA_LAUNCH_CHECK();
}

// ============================================================================
// K5 — YOLOv4 head decode (reference tools/yolo_layer.py:148-288,
// yolo_forward_dynamic) fused with the post-processing filter
// (tools/utils.py:166-233: max/argmax over conf = sigmoid(cls) * sigmoid(obj),
// conf > thresh).  One thread per (image, row) with rows anchor-major (a, y, x)
// per level, levels at strides 8/16/32 — the [B, N, ...] order of the
// reference's ONNX outputs.  Writes:
//   * optional full outputs: boxes [B, N, 4] normalised x1y1x2y2 and confs
//     [B, N, nc] (examples/YOLOv4/config.pbtxt outputs `boxes` / `confs`);
//   * candidates (max conf > thresh) in model-input pixels, compacted per image.
// ============================================================================
namespace {

template <typename T>
__global__ void __launch_bounds__(256) yolov4_decode_kernel(YoloHeads hd, int batch, int nc, float sxy,
                                                            float conf_thres, int img_h, int img_w,
                                                            float* __restrict__ out_boxes, float* __restrict__ out_confs,
                                                            float* __restrict__ cand_box, float* __restrict__ cand_score,
                                                            int* __restrict__ cand_cls, uint64_t* __restrict__ cand_key,
                                                            int* __restrict__ cand_count, int cap) {
  __shared__ int s_cnt, s_base;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int b = blockIdx.y;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int n0 = 3 * hd.h[0] * hd.w[0], n1 = n0 + 3 * hd.h[1] * hd.w[1], N = n1 + 3 * hd.h[2] * hd.w[2];
  bool pass = false;
  float best = 0.f, box[4];
  int best_c = 0;
  if (n < N) {
    const int l = n < n0 ? 0 : (n < n1 ? 1 : 2);
    const int r = n - (l == 0 ? 0 : (l == 1 ? n0 : n1));
    const int H = hd.h[l], W = hd.w[l], HW = H * W;
    const int a = r / HW, yx = r - a * HW, y = yx / W, x = yx - y * W;
    const T* hp = reinterpret_cast<const T*>(hd.head[l]) + ((long)b * HW + yx) * hd.ldc[l] + a * (5 + nc);
    const float bx = (sigmoidf_(to_f32(hp[0])) * sxy - 0.5f * (sxy - 1.f) + (float)x) / (float)W;
    const float by = (sigmoidf_(to_f32(hp[1])) * sxy - 0.5f * (sxy - 1.f) + (float)y) / (float)H;
    const float bw = __expf(to_f32(hp[2])) * hd.anchor[l][a][0] / (float)W;
    const float bh = __expf(to_f32(hp[3])) * hd.anchor[l][a][1] / (float)H;
    box[0] = bx - 0.5f * bw;
    box[1] = by - 0.5f * bh;
    box[2] = box[0] + bw;
    box[3] = box[1] + bh;
    const float obj = sigmoidf_(to_f32(hp[4]));
    const long row = (long)b * N + n;
    if (out_boxes) {
#pragma unroll
      for (int k = 0; k < 4; ++k) out_boxes[row * 4 + k] = box[k];
    }
    float m = -INFINITY;
    for (int c = 0; c < nc; ++c) {
      const float v = to_f32(hp[5 + c]);
      if (out_confs) out_confs[row * nc + c] = sigmoidf_(v) * obj;
      if (v > m) { m = v; best_c = c; }
    }
    best = sigmoidf_(m) * obj;
    pass = best > conf_thres;
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
      cand_box[o * 4 + 0] = box[0] * img_w; cand_box[o * 4 + 1] = box[1] * img_h;
      cand_box[o * 4 + 2] = box[2] * img_w; cand_box[o * 4 + 3] = box[3] * img_h;
      cand_score[o] = best;
      cand_cls[o] = best_c;
      cand_key[o] = make_score_key(best, (uint32_t)n);
    }
  }
}

}  // namespace

// heads: three NHWC slices with channel strides ldc[3] (>= 3*(5+nc)); anchors [3][3][2]
// already divided by the level stride (masked anchors / stride, yolo_layer.py:318).
TCA_API int tca_yolov4_decode(const void* head0, const void* head1, const void* head2, int dtype, int batch, int nc,
                              const int* hw /*[6]*/, const int* ldc /*[3]*/, const float* anchors /*[3][3][2]*/,
                              float scale_x_y, float conf_thres, int img_h, int img_w, float* out_boxes,
                              float* out_confs, float* cand_box, float* cand_score, int* cand_cls, uint64_t* cand_key,
                              int* cand_count, int cap, hipStream_t stream) {
  if (batch <= 0) return 0;
  YoloHeads hd;
  hd.head[0] = head0; hd.head[1] = head1; hd.head[2] = head2;
  for (int l = 0; l < 3; ++l) {
    hd.h[l] = hw[2 * l]; hd.w[l] = hw[2 * l + 1]; hd.stride[l] = 0; hd.ldc[l] = ldc[l];
    for (int a = 0; a < 4; ++a) {
      hd.anchor[l][a][0] = a < 3 ? anchors[(l * 3 + a) * 2] : 0.f;
      hd.anchor[l][a][1] = a < 3 ? anchors[(l * 3 + a) * 2 + 1] : 0.f;
    }
  }
  int e = zero_i32_async(cand_count, batch, stream);
  if (e) return e;
  long N = 0;
  for (int l = 0; l < 3; ++l) N += 3L * hd.h[l] * hd.w[l];
  dim3 grid((unsigned)((N + 255) / 256), (unsigned)batch);
  switch (dtype) {
    case kF32:
      yolov4_decode_kernel<float><<<grid, 256, 0, stream>>>(hd, batch, nc, scale_x_y, conf_thres, img_h, img_w,
                                                            out_boxes, out_confs, cand_box, cand_score, cand_cls,
                                                            cand_key, cand_count, cap);
      break;
    case kBF16:
      yolov4_decode_kernel<__hip_bfloat16><<<grid, 256, 0, stream>>>(hd, batch, nc, scale_x_y, conf_thres, img_h,
                                                                     img_w, out_boxes, out_confs, cand_box, cand_score,
                                                                     cand_cls, cand_key, cand_count, cap);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  TCA_LAUNCH_CHECK();
}
