// K1 — fused camera-frame preprocessing (reference: communicator/ros_inference.py:131,140-141
// cv2.resize + clients/preprocess/yolov5_preprocess.py:20-24 transpose/astype//255,
// detectron_preprocess.py:20-24 (no /255), utils/preprocess.py:147-157 INCEPTION/VGG/COCO).
//
// One pass: uint8 HWC (RGB or BGR) -> bilinear resize (OpenCV INTER_LINEAR
// pixel-centre convention, optional uint8 re-quantisation like cv2's u8
// output) -> optional letterbox (YOLOv5 style, pad value 114) -> per-channel
// affine (x*scale+bias) -> NCHW or NHWC(4-padded) in fp32/fp16/bf16.
//
// Each thread produces 4 horizontally adjacent output pixels so that the
// stores are 8-16 B per lane per plane (vectorised, cdna_hip_programming.md
// Guideline 13).  Source reads go through L1/L2 (each source pixel is re-read
// by ~1-4 output pixels); the kernel is store-bound.
#include "tca_common.h"

using namespace tca;

namespace {

struct PrepParams {
  int src_h, src_w, src_row_stride, src_c;
  long src_batch_stride;
  int swap_rb;
  int dst_h, dst_w, dst_c, dst_layout;  // layout 0 = NCHW, 1 = NHWC
  int reg_top, reg_left, reg_h, reg_w;  // resized region inside dst
  float pad_value;
  int quantize_u8;
  float sc0, sc1, sc2, b0, b1, b2;
};

__device__ __forceinline__ void coord(float dst, float scale, int src_n, int& i0, int& i1, float& a) {
  float f = (dst + 0.5f) * scale - 0.5f;
  int s = (int)floorf(f);
  a = f - (float)s;
  if (s < 0) { s = 0; a = 0.f; }
  if (s >= src_n - 1) { s = src_n - 1; a = 0.f; }
  i0 = s;
  i1 = min(s + 1, src_n - 1);
}

template <typename T>
__global__ void __launch_bounds__(256) prep_kernel(const uint8_t* __restrict__ src, T* __restrict__ dst, PrepParams p,
                                                   int batch) {
  const int qw = (p.dst_w + 3) >> 2;
  // 32-bit index math (total < 2^31, host-checked): 64-bit div/mod is ~150 VALU each
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned total = (unsigned)batch * p.dst_h * qw;
  if (gid >= total) return;
  const unsigned row = gid / (unsigned)qw;
  const int q = (int)(gid - row * qw);
  const int b = (int)(row / (unsigned)p.dst_h);
  const int y = (int)(row - (unsigned)b * p.dst_h);
  const uint8_t* s = src + (long)b * p.src_batch_stride;
  const float sx_scale = (float)p.src_w / (float)p.reg_w;
  const float sy_scale = (float)p.src_h / (float)p.reg_h;

  float out[4][3];
  const int ly = y - p.reg_top;
  const bool row_in = ly >= 0 && ly < p.reg_h;
  int y0 = 0, y1 = 0;
  float ay = 0.f;
  if (row_in) coord((float)ly, sy_scale, p.src_h, y0, y1, ay);
  const uint8_t* r0 = s + (long)y0 * p.src_row_stride;
  const uint8_t* r1 = s + (long)y1 * p.src_row_stride;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = q * 4 + k;
    const int lx = x - p.reg_left;
    if (!row_in || lx < 0 || lx >= p.reg_w || x >= p.dst_w) {
      out[k][0] = out[k][1] = out[k][2] = p.pad_value;
      continue;
    }
    int x0, x1;
    float ax;
    coord((float)lx, sx_scale, p.src_w, x0, x1, ax);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float v00 = r0[x0 * p.src_c + c], v01 = r0[x1 * p.src_c + c];
      float v10 = r1[x0 * p.src_c + c], v11 = r1[x1 * p.src_c + c];
      float top = v00 + ax * (v01 - v00);
      float bot = v10 + ax * (v11 - v10);
      float v = top + ay * (bot - top);
      if (p.quantize_u8) v = fminf(fmaxf(rintf(v), 0.f), 255.f);
      out[k][c] = v;
    }
  }
  const float sc[3] = {p.sc0, p.sc1, p.sc2};
  const float bi[3] = {p.b0, p.b1, p.b2};
  T* d = dst;
  if (p.dst_layout == 0) {  // NCHW
    const long plane = (long)p.dst_h * p.dst_w;
    const long base = (long)b * p.dst_c * plane + (long)y * p.dst_w + q * 4;
    const bool full = q * 4 + 3 < p.dst_w && ((p.dst_w & 3) == 0);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int sc_c = p.swap_rb ? 2 - c : c;
      T v4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v4[k] = from_f32<T>(out[k][sc_c] * sc[c] + bi[c]);
      T* o = d + base + (long)c * plane;
      if (full) {
        if constexpr (sizeof(T) == 4) {
          *reinterpret_cast<float4*>(o) = *reinterpret_cast<float4*>(v4);
        } else {
          *reinterpret_cast<uint2*>(o) = *reinterpret_cast<uint2*>(v4);
        }
      } else {
        for (int k = 0; k < 4; ++k)
          if (q * 4 + k < p.dst_w) o[k] = v4[k];
      }
    }
    if (p.dst_c == 4) {
      T* o = d + base + 3 * plane;
      for (int k = 0; k < 4; ++k)
        if (q * 4 + k < p.dst_w) o[k] = from_f32<T>(0.f);
    }
  } else if (p.dst_c == 8) {  // NHWC, 3 channels + 5 zero pad: 16-B stores per pixel
    const long base = (((long)b * p.dst_h + y) * p.dst_w + q * 4) * 8;
    for (int k = 0; k < 4; ++k) {
      if (q * 4 + k >= p.dst_w) break;
      T px[8];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int sc_c = p.swap_rb ? 2 - c : c;
        px[c] = from_f32<T>(out[k][sc_c] * sc[c] + bi[c]);
      }
#pragma unroll
      for (int c = 3; c < 8; ++c) px[c] = from_f32<T>(0.f);
#pragma unroll
      for (int v = 0; v < (int)(8 * sizeof(T) / 16); ++v)
        reinterpret_cast<uint4*>(d + base + (long)k * 8)[v] = reinterpret_cast<uint4*>(px)[v];
    }
  } else {  // NHWC with dst_c in {3, 4}
    const long base = (((long)b * p.dst_h + y) * p.dst_w + q * 4) * p.dst_c;
    for (int k = 0; k < 4; ++k) {
      if (q * 4 + k >= p.dst_w) break;
      T px[4];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int sc_c = p.swap_rb ? 2 - c : c;
        px[c] = from_f32<T>(out[k][sc_c] * sc[c] + bi[c]);
      }
      px[3] = from_f32<T>(0.f);
      T* o = d + base + (long)k * p.dst_c;
      if (p.dst_c == 4 && sizeof(T) == 2) {
        *reinterpret_cast<uint2*>(o) = *reinterpret_cast<uint2*>(px);
      } else {
        for (int c = 0; c < p.dst_c; ++c) o[c] = px[c];
      }
    }
  }
}

// One resized / letterboxed / quantised RGB sample of destination pixel (y, x)
// (before the affine), channel order of the source (swap handled by the caller).
__device__ __forceinline__ void sample_px(const PrepParams& p, const uint8_t* s, int y, int x, float (&o)[3]) {
  const int ly = y - p.reg_top, lx = x - p.reg_left;
  if (ly < 0 || ly >= p.reg_h || lx < 0 || lx >= p.reg_w) {
    o[0] = o[1] = o[2] = p.pad_value;
    return;
  }
  int y0, y1, x0, x1;
  float ay, ax;
  coord((float)ly, (float)p.src_h / (float)p.reg_h, p.src_h, y0, y1, ay);
  coord((float)lx, (float)p.src_w / (float)p.reg_w, p.src_w, x0, x1, ax);
  const uint8_t* r0 = s + (long)y0 * p.src_row_stride;
  const uint8_t* r1 = s + (long)y1 * p.src_row_stride;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v00 = r0[x0 * p.src_c + c], v01 = r0[x1 * p.src_c + c];
    const float v10 = r1[x0 * p.src_c + c], v11 = r1[x1 * p.src_c + c];
    const float top = v00 + ax * (v01 - v00);
    const float bot = v10 + ax * (v11 - v10);
    float v = top + ay * (bot - top);
    if (p.quantize_u8) v = fminf(fmaxf(rintf(v), 0.f), 255.f);
    o[c] = v;
  }
}

// Layout 2: space-to-depth 2x2, bf16 or fp32 [B, H/2, W/2, 16]: channel
// (dy*2 + dx)*3 + c holds pixel (2Y + dy, 2X + dx), channels 12..15 zero.  A
// k=6 s=2 p=2 stem conv (YOLOv5 v6+) is exactly a 3x3 s=1 p=1 conv over this
// tensor with rearranged weights (models/fast.py), with 12 of 16 input
// channels real instead of 3 of 8 and half the input bytes.  One thread per
// 2x2 block, 32 B (bf16) or 64 B (fp32) of 16-B stores.
template <typename T>
__global__ void __launch_bounds__(256) prep_s2d_kernel(const uint8_t* __restrict__ src, T* __restrict__ dst,
                                                       PrepParams p, int batch) {
  const int h2 = p.dst_h >> 1, w2 = p.dst_w >> 1;
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned total = (unsigned)batch * h2 * w2;
  if (gid >= total) return;
  const unsigned row = gid / (unsigned)w2;
  const int X = (int)(gid - row * w2);
  const int b = (int)(row / (unsigned)h2);
  const int Y = (int)(row - (unsigned)b * h2);
  const uint8_t* s = src + (long)b * p.src_batch_stride;
  const float sc[3] = {p.sc0, p.sc1, p.sc2};
  const float bi[3] = {p.b0, p.b1, p.b2};
  T px[16];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    float o[3];
    sample_px(p, s, 2 * Y + (d >> 1), 2 * X + (d & 1), o);
#pragma unroll
    for (int c = 0; c < 3; ++c) px[d * 3 + c] = from_f32<T>(o[p.swap_rb ? 2 - c : c] * sc[c] + bi[c]);
  }
#pragma unroll
  for (int c = 12; c < 16; ++c) px[c] = from_f32<T>(0.f);
  constexpr int NV = 16 * sizeof(T) / 16;
  uint4* o = reinterpret_cast<uint4*>(dst + (long)gid * 16);
#pragma unroll
  for (int v = 0; v < NV; ++v) o[v] = reinterpret_cast<uint4*>(px)[v];
}

// Served-model input path: a request tensor that is already model-sized fp32 NCHW
// RGB (the reference's contracts: examples/YOLOv5/config.pbtxt "images" [3, H, W],
// examples/RetinaNet_detectron/config.pbtxt "input__00" [3, 640, 480], 0..255 un-
// normalised) -> per-channel affine (x * scale + bias, e.g. Detectron2's (x - mean) / std
// folded in) -> the plans' input layouts: NHWC x 8 (3 channels + 5 zeros, 16-B stores) or
// space-to-depth 2x2 x 16 (YOLOv5 S2D stem).  One thread per pixel / 2x2 block.
template <typename T, int LAYOUT>
__global__ void __launch_bounds__(256) planar_affine_kernel(const float* __restrict__ src, T* __restrict__ dst,
                                                            int B, int H, int W, float sc0, float sc1, float sc2,
                                                            float b0, float b1, float b2) {
  const float sc[3] = {sc0, sc1, sc2}, bi[3] = {b0, b1, b2};
  const long plane = (long)H * W;
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (LAYOUT == 1) {
    if (gid >= (unsigned)(B * plane)) return;
    const long b = gid / plane, pix = gid - b * plane;
    const float* s = src + b * 3 * plane + pix;
    T px[8];
#pragma unroll
    for (int c = 0; c < 3; ++c) px[c] = from_f32<T>(s[c * plane] * sc[c] + bi[c]);
#pragma unroll
    for (int c = 3; c < 8; ++c) px[c] = from_f32<T>(0.f);
    uint4* o = reinterpret_cast<uint4*>(dst + (long)gid * 8);
#pragma unroll
    for (int v = 0; v < (int)(8 * sizeof(T) / 16); ++v) o[v] = reinterpret_cast<uint4*>(px)[v];
  } else {
    const int h2 = H >> 1, w2 = W >> 1;
    if (gid >= (unsigned)(B * h2 * w2)) return;
    const int X = gid % w2, Y = (gid / w2) % h2, b = gid / (w2 * h2);
    const float* s = src + (long)b * 3 * plane;
    T px[16];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const long pix = (long)(2 * Y + (d >> 1)) * W + 2 * X + (d & 1);
#pragma unroll
      for (int c = 0; c < 3; ++c) px[d * 3 + c] = from_f32<T>(s[c * plane + pix] * sc[c] + bi[c]);
    }
#pragma unroll
    for (int c = 12; c < 16; ++c) px[c] = from_f32<T>(0.f);
    uint4* o = reinterpret_cast<uint4*>(dst + (long)gid * 16);
#pragma unroll
    for (int v = 0; v < (int)(16 * sizeof(T) / 16); ++v) o[v] = reinterpret_cast<uint4*>(px)[v];
  }
}

}  // namespace

// fp32 NCHW [B, 3, H, W] -> dst NHWC x 8 (layout 1) or space-to-depth [B, H/2, W/2, 16]
// (layout 2), fp32 or bf16, x * scale[c] + bias[c].
TCA_API int tca_planar_affine(const float* src, int B, int H, int W, void* dst, int dst_dtype, int dst_layout,
                              float sc0, float sc1, float sc2, float b0, float b1, float b2, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((dst_layout != 1 && dst_layout != 2) || (dst_layout == 2 && ((H & 1) || (W & 1))) ||
      (dst_dtype != kF32 && dst_dtype != kBF16))
    return (int)hipErrorInvalidValue;
  const long n = dst_layout == 1 ? (long)B * H * W : (long)B * (H / 2) * (W / 2);
  if (n >= (1L << 31)) return (int)hipErrorInvalidValue;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (dst_layout == 1) {
    if (dst_dtype == kF32)
      planar_affine_kernel<float, 1><<<g, 256, 0, stream>>>(src, (float*)dst, B, H, W, sc0, sc1, sc2, b0, b1, b2);
    else
      planar_affine_kernel<__hip_bfloat16, 1><<<g, 256, 0, stream>>>(src, (__hip_bfloat16*)dst, B, H, W, sc0, sc1,
                                                                      sc2, b0, b1, b2);
  } else {
    if (dst_dtype == kF32)
      planar_affine_kernel<float, 2><<<g, 256, 0, stream>>>(src, (float*)dst, B, H, W, sc0, sc1, sc2, b0, b1, b2);
    else
      planar_affine_kernel<__hip_bfloat16, 2><<<g, 256, 0, stream>>>(src, (__hip_bfloat16*)dst, B, H, W, sc0, sc1,
                                                                      sc2, b0, b1, b2);
  }
  TCA_LAUNCH_CHECK();
}

// Preprocess `batch` frames of identical geometry.
TCA_API int tca_image_preprocess(const void* src, long src_batch_stride, int src_h, int src_w, int src_row_stride,
                                 int src_c, int swap_rb, void* dst, int dst_dtype, int dst_layout, int dst_c,
                                 int dst_h, int dst_w, int batch, int reg_top, int reg_left, int reg_h, int reg_w,
                                 float pad_value, int quantize_u8, float sc0, float sc1, float sc2, float b0,
                                 float b1, float b2, hipStream_t stream) {
  if (batch <= 0) return 0;
  PrepParams p{src_h, src_w, src_row_stride, src_c, src_batch_stride, swap_rb, dst_h, dst_w, dst_c, dst_layout,
               reg_top, reg_left, reg_h, reg_w, pad_value, quantize_u8, sc0, sc1, sc2, b0, b1, b2};
  if (dst_layout == 2) {  // space-to-depth 2x2, bf16 or fp32, 16 channels
    if (src_c < 3 || dst_c != 16 || (dst_dtype != kBF16 && dst_dtype != kF32) || (dst_h & 1) || (dst_w & 1) ||
        reg_h <= 0 || reg_w <= 0)
      return (int)hipErrorInvalidValue;
    const long t2 = (long)batch * (dst_h / 2) * (dst_w / 2);
    if (t2 >= (1L << 31)) return (int)hipErrorInvalidValue;
    const unsigned g = (unsigned)((t2 + 255) / 256);
    if (dst_dtype == kF32)
      prep_s2d_kernel<float><<<g, 256, 0, stream>>>((const uint8_t*)src, (float*)dst, p, batch);
    else
      prep_s2d_kernel<__hip_bfloat16><<<g, 256, 0, stream>>>((const uint8_t*)src, (__hip_bfloat16*)dst, p, batch);
    TCA_LAUNCH_CHECK();
  }
  if (src_c < 3 || (dst_c != 3 && dst_c != 4 && !(dst_c == 8 && dst_layout == 1)) || reg_h <= 0 ||
      reg_w <= 0)
    return (int)hipErrorInvalidValue;
  const long total = (long)batch * dst_h * ((dst_w + 3) / 4);
  if (total >= (1L << 31)) return (int)hipErrorInvalidValue;  // the kernel's 32-bit index math
  const int bs = 256;
  dim3 grid((unsigned)((total + bs - 1) / bs));
  const uint8_t* s = (const uint8_t*)src;
  switch (dst_dtype) {
    case kF32: prep_kernel<float><<<grid, bs, 0, stream>>>(s, (float*)dst, p, batch); break;
    case kF16: prep_kernel<__half><<<grid, bs, 0, stream>>>(s, (__half*)dst, p, batch); break;
    case kBF16: prep_kernel<__hip_bfloat16><<<grid, bs, 0, stream>>>(s, (__hip_bfloat16*)dst, p, batch); break;
    default: return (int)hipErrorInvalidValue;
  }
  TCA_LAUNCH_CHECK();
}
