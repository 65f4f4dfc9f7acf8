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

#include <cstdlib>

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

// Channel c of a 3-channel sample, red and blue swapped when `swap`: two constant-index reads and a
// select (o[swap ? 2 - c : c] is a run-time index, which puts the whole array in scratch memory).
__device__ __forceinline__ float rgb_at(const float (&o)[3], int c, bool swap) { return swap ? o[2 - c] : o[c]; }

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
      T v4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v4[k] = from_f32<T>(rgb_at(out[k], c, p.swap_rb) * sc[c] + bi[c]);
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
        px[c] = from_f32<T>(rgb_at(out[k], c, p.swap_rb) * sc[c] + bi[c]);
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
        px[c] = from_f32<T>(rgb_at(out[k], c, p.swap_rb) * sc[c] + bi[c]);
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
    for (int c = 0; c < 3; ++c) px[d * 3 + c] = from_f32<T>(rgb_at(o, c, p.swap_rb) * sc[c] + bi[c]);
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


// ---- K1 fused into the YOLOv5 stem and its first stride-2 conv (fp32 mode).
//
// Unfused, the camera branch writes the space-to-depth input [B, 320, 320, 16] fp32
// (210 MB at batch 32), the s2d stem reads it and writes [B, 320, 320, 16] (210 MB), and
// the 3x3 stride-2 conv b1 reads that back: ~840 MB of HBM traffic for ~0.6 GFLOP per frame.
// Here one workgroup owns an 8 x 16 tile of b1's output (160 x 160 grid) and builds
// everything it needs in LDS: the 19 x 35 s2d input pixels are sampled straight from the
// uint8 frame (sample_px: the same resize / letterbox / affine arithmetic as
// prep_s2d_kernel, so the same fp32 values) and split to bf16 hi / lo; the stem (3x3 over
// 16 s2d channels, 16 outputs) runs on the 17 x 33 pixels b1 reads, its bias + activation
// outputs (zero outside the 320 x 320 image: b1's padding) are split into a second LDS image
// that overlays the first, and b1 (16 -> 32, stride 2) reads it.  Products and K-step order
// are those of conv_small_halo_x3 / conv_nhwc_x3 (bf16 x3, fp32 accumulation), so the
// output matches the unfused chain.  Only the frames are read and only b1's output written.
// LDS 44 KiB (3 workgroups per CU).  Weights: split_pairs images [N, 2 * 160] of the
// FusedConvs (K = 9 taps x 16 channels, padded to 160), read as MFMA fragments from L2.
struct StemArgs {
  const uint8_t* src;
  PrepParams p;
  const __hip_bfloat16* w0;  // stem [16, 2 * 160]
  const float* b0;
  const __hip_bfloat16* w1;  // b1 [32, 2 * 160]
  const float* b1;
  int act0, act1;
  float* out;  // [B, H1, W1, ldo], channels [co_off, co_off + 32)
  int ldo, co_off;
  int B, H0, W0, H1, W1;  // stem grid (s2d, dst / 2) and b1 grid
};

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float stem_act(float v, int act) {  // conv_mfma.hip act_fn (same expressions)
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return v / (1.f + __expf(-v));
    case 3: return v > 0.f ? v : 0.1f * v;
    default: return v;
  }
}

__device__ __forceinline__ void stem_mfma3(f32x4_t& acc, const bf16x8_t& bh, const bf16x8_t& bl, const bf16x8_t& ah,
                                           const bf16x8_t& al) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc, 0, 0, 0);
}

template <int TY>
__global__ void __launch_bounds__(256) yolo_stem_fused_kernel(StemArgs a) {
  constexpr int TX = 16, RW = TY / 4;                // b1 output tile TY x 16; RW rows per wave
  static_assert(TY % 4 == 0, "tile rows");
  constexpr int SH = 2 * TY + 1, SW = 2 * TX + 1;    // stem pixels b1 reads (17 x 33)
  constexpr int IH = SH + 2, IW = SW + 2;            // s2d input pixels the stem reads (19 x 35)
  constexpr int NS = SH * SW, NMS = (NS + 15) / 16;  // stem pixels, 16-pixel M tiles (36)
  constexpr int IMG = IH * IW * 32;                  // one input image (hi or lo): 32 B per pixel
  constexpr int SPB = 80;                            // stem pixel: hi 32 B | lo 32 B | 16 B pad (conflict-free stride-2 reads)
  constexpr int LDS = (2 * IMG > NS * SPB) ? 2 * IMG : NS * SPB;
  constexpr int KP = 160;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  unsigned char* const himg = smem;
  unsigned char* const limg = smem + IMG;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  const int ntx = (a.W1 + TX - 1) / TX, nty = (a.H1 + TY - 1) / TY;
  const int tile = blockIdx.x;
  const int b = tile / (nty * ntx), rem = tile - b * nty * ntx;
  const int oy0 = (rem / ntx) * TY, ox0 = (rem - (rem / ntx) * ntx) * TX;
  const int sy0 = 2 * oy0 - 1, sx0 = 2 * ox0 - 1;  // stem region origin
  const int iy0 = sy0 - 1, ix0 = sx0 - 1;          // input region origin

  // phase A: s2d input pixels from the frame, split into the hi / lo images
  const uint8_t* s = a.src + (long)b * a.p.src_batch_stride;
  const float sc[3] = {a.p.sc0, a.p.sc1, a.p.sc2}, bi[3] = {a.p.b0, a.p.b1, a.p.b2};
  // exact 2:1 downscale of a 3-channel frame into an even-aligned region (1280 x 720 -> 640 x 360
  // letterboxed): coord() gives s = 2 dst, a = 0.5 everywhere, so an s2d pixel's 2 x 2 block reads
  // one 4 x 4 source block -- 4 rows of 12 aligned bytes (3 dword loads each) instead of 48 byte loads
  const bool half = a.p.src_c == 3 && a.p.reg_h * 2 == a.p.src_h && a.p.reg_w * 2 == a.p.src_w &&
                    !(a.p.reg_top & 1) && !(a.p.reg_left & 1) && !(a.p.reg_h & 1) && !(a.p.reg_w & 1) &&
                    !(a.p.src_row_stride & 3) && !(a.p.src_batch_stride & 3);
  auto put = [&](int g, const float (&v)[16]) {
    // hi / lo bf16 of the 16 channels packed straight into 32-bit words (no private arrays: a
    // run-time choice between halves of an array kept it in scratch memory, 80 B per lane
    // written and read back per pixel)
    unsigned hw[8], lw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const __bf16 h0 = (__bf16)v[2 * c], h1 = (__bf16)v[2 * c + 1];
      const __bf16 l0 = (__bf16)(v[2 * c] - (float)h0), l1 = (__bf16)(v[2 * c + 1] - (float)h1);
      hw[c] = (unsigned)__builtin_bit_cast(unsigned short, h0) | ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
      lw[c] = (unsigned)__builtin_bit_cast(unsigned short, l0) | ((unsigned)__builtin_bit_cast(unsigned short, l1) << 16);
    }
    const uint4 hA = make_uint4(hw[0], hw[1], hw[2], hw[3]), hB = make_uint4(hw[4], hw[5], hw[6], hw[7]);
    const uint4 lA = make_uint4(lw[0], lw[1], lw[2], lw[3]), lB = make_uint4(lw[4], lw[5], lw[6], lw[7]);
    // 32-B pixel stride: the two 16-B halves go in an order alternating every 4 pixels, so each
    // 8-lane ds_write_b128 group covers the 32 banks once (in one order: 2-way)
    const bool q0 = (g >> 2) & 1;
    uint4 f, s2;
    f.x = q0 ? hB.x : hA.x; f.y = q0 ? hB.y : hA.y; f.z = q0 ? hB.z : hA.z; f.w = q0 ? hB.w : hA.w;
    s2.x = q0 ? hA.x : hB.x; s2.y = q0 ? hA.y : hB.y; s2.z = q0 ? hA.z : hB.z; s2.w = q0 ? hA.w : hB.w;
    *reinterpret_cast<uint4*>(himg + g * 32 + q0 * 16) = f;
    *reinterpret_cast<uint4*>(himg + g * 32 + (!q0) * 16) = s2;
    f.x = q0 ? lB.x : lA.x; f.y = q0 ? lB.y : lA.y; f.z = q0 ? lB.z : lA.z; f.w = q0 ? lB.w : lA.w;
    s2.x = q0 ? lA.x : lB.x; s2.y = q0 ? lA.y : lB.y; s2.z = q0 ? lA.z : lB.z; s2.w = q0 ? lA.w : lB.w;
    *reinterpret_cast<uint4*>(limg + g * 32 + q0 * 16) = f;
    *reinterpret_cast<uint4*>(limg + g * 32 + (!q0) * 16) = s2;
  };
  if (half) {
    // all of this thread's source blocks are requested before any is used (one memory latency
    // per workgroup, not one per pixel)
    constexpr int NPT = (IH * IW + 255) / 256;
    unsigned w[NPT][4][3];
    int state[NPT];  // 0 outside the s2d image (zeros), 1 letterbox pad, 2 frame block
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int g = tid + u * 256;
      const int hy = g / IW, hx = g - (g / IW) * IW;
      const int Y = iy0 + hy, X = ix0 + hx;
      const int ly = 2 * Y - a.p.reg_top, lx = 2 * X - a.p.reg_left;
      state[u] = 0;
      if (g < IH * IW && (unsigned)Y < (unsigned)a.H0 && (unsigned)X < (unsigned)a.W0)
        state[u] = (ly >= 0 && ly < a.p.reg_h && lx >= 0 && lx < a.p.reg_w) ? 2 : 1;
      const uint8_t* r = s + (state[u] == 2 ? (long)(2 * ly) * a.p.src_row_stride + 6 * lx : 0);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          w[u][k][j] = state[u] == 2 ? reinterpret_cast<const unsigned*>(r + (long)k * a.p.src_row_stride)[j] : 0u;
    }
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int g = tid + u * 256;
      if (g >= IH * IW) break;
      float o[4][3], v[16];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int dy = d >> 1, dx = d & 1;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int b0 = (2 * dx) * 3 + c, b1 = b0 + 3;  // bytes of source columns 2 dx, 2 dx + 1
          const float v00 = (float)((w[u][2 * dy][b0 >> 2] >> (8 * (b0 & 3))) & 255u);
          const float v01 = (float)((w[u][2 * dy][b1 >> 2] >> (8 * (b1 & 3))) & 255u);
          const float v10 = (float)((w[u][2 * dy + 1][b0 >> 2] >> (8 * (b0 & 3))) & 255u);
          const float v11 = (float)((w[u][2 * dy + 1][b1 >> 2] >> (8 * (b1 & 3))) & 255u);
          const float top = v00 + 0.5f * (v01 - v00);
          const float bot = v10 + 0.5f * (v11 - v10);
          float q = top + 0.5f * (bot - top);
          if (a.p.quantize_u8) q = fminf(fmaxf(rintf(q), 0.f), 255.f);
          o[d][c] = state[u] == 2 ? q : a.p.pad_value;
        }
      }
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          v[d * 3 + c] = state[u] ? rgb_at(o[d], c, a.p.swap_rb) * sc[c] + bi[c] : 0.f;
#pragma unroll
      for (int c = 12; c < 16; ++c) v[c] = 0.f;
      put(g, v);
    }
  } else {
    for (int g = tid; g < IH * IW; g += 256) {
      const int hy = g / IW, hx = g - (g / IW) * IW;
      const int Y = iy0 + hy, X = ix0 + hx;
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = 0.f;
      if ((unsigned)Y < (unsigned)a.H0 && (unsigned)X < (unsigned)a.W0) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          float o[3];
          sample_px(a.p, s, 2 * Y + (d >> 1), 2 * X + (d & 1), o);
#pragma unroll
          for (int c = 0; c < 3; ++c) v[d * 3 + c] = rgb_at(o, c, a.p.swap_rb) * sc[c] + bi[c];
        }
      }
      put(g, v);
    }
  }
  __syncthreads();

  // phase B: stem, M tiles wid, wid + 4, ... of the 17 x 33 stem pixels (row-major), 16 outputs
  constexpr int MW = (NMS + 3) / 4;  // M tiles per wave (9)
  f32x4_t acc0[MW];
  int hbase[MW];
#pragma unroll
  for (int i = 0; i < MW; ++i) {
    acc0[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int p = (wid + 4 * i) * 16 + fr;
    const int py = p / SW, px = p - (p / SW) * SW;
    hbase[i] = p < NS ? py * IW + px : -1;
  }
#pragma unroll
  for (int st = 0; st < KP / 32; ++st) {
    const int k0 = st * 32 + fq * 8, tap = k0 >> 4, ci0 = k0 & 15;
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    const __hip_bfloat16* wp = a.w0 + fr * 2 * KP + (k0 >> 3) * 16;
    const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(wp);
    const bf16x8_t bl = *reinterpret_cast<const bf16x8_t*>(wp + 8);
#pragma unroll
    for (int i = 0; i < MW; ++i) {
      if (wid + 4 * i >= NMS) continue;
      bf16x8_t ah = bf16x8_t{}, al = bf16x8_t{};
      if (tap < 9 && hbase[i] >= 0) {
        const int hp = hbase[i] + ky * IW + kx;
        ah = *reinterpret_cast<const bf16x8_t*>(himg + hp * 32 + ci0 * 2);
        al = *reinterpret_cast<const bf16x8_t*>(limg + hp * 32 + ci0 * 2);
      }
      stem_mfma3(acc0[i], bh, bl, ah, al);
    }
  }
  __syncthreads();  // every wave done reading the input images: the stem image overlays them
  {
    float bb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bb[r] = a.b0 ? a.b0[fq * 4 + r] : 0.f;
#pragma unroll
    for (int i = 0; i < MW; ++i) {
      if (wid + 4 * i >= NMS) continue;
      const int p = (wid + 4 * i) * 16 + fr;
      if (p >= NS) continue;
      const int py = p / SW, px = p - (p / SW) * SW;
      const bool in = (unsigned)(sy0 + py) < (unsigned)a.H0 && (unsigned)(sx0 + px) < (unsigned)a.W0;
      __bf16 h[4], l[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = in ? stem_act(acc0[i][r] + bb[r], a.act0) : 0.f;
        h[r] = (__bf16)v;
        l[r] = (__bf16)(v - (float)h[r]);
      }
      *reinterpret_cast<uint2*>(smem + p * SPB + fq * 8) = *reinterpret_cast<const uint2*>(h);
      *reinterpret_cast<uint2*>(smem + p * SPB + 32 + fq * 8) = *reinterpret_cast<const uint2*>(l);
    }
  }
  __syncthreads();

  // phase C: b1 (3x3 stride 2, 16 -> 32): wave wid owns output rows 2 wid, 2 wid + 1 of the tile
  f32x4_t acc1[RW][2];
#pragma unroll
  for (int i = 0; i < RW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc1[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < KP / 32; ++st) {
    const int k0 = st * 32 + fq * 8, tap = k0 >> 4, ci0 = k0 & 15;
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    bf16x8_t bh[2], bl[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const __hip_bfloat16* wp = a.w1 + (j * 16 + fr) * 2 * KP + (k0 >> 3) * 16;
      bh[j] = *reinterpret_cast<const bf16x8_t*>(wp);
      bl[j] = *reinterpret_cast<const bf16x8_t*>(wp + 8);
    }
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      bf16x8_t ah = bf16x8_t{}, al = bf16x8_t{};
      if (tap < 9) {
        const int sp = (2 * (RW * wid + i) + ky) * SW + 2 * fr + kx;
        ah = *reinterpret_cast<const bf16x8_t*>(smem + sp * SPB + ci0 * 2);
        al = *reinterpret_cast<const bf16x8_t*>(smem + sp * SPB + 32 + ci0 * 2);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) stem_mfma3(acc1[i][j], bh[j], bl[j], ah, al);
    }
  }
  const int ox = ox0 + fr;
  if (ox >= a.W1) return;
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int oy = oy0 + RW * wid + i;
    if (oy >= a.H1) break;
    float* o = a.out + (((long)b * a.H1 + oy) * a.W1 + ox) * a.ldo + a.co_off;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = j * 16 + fq * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = stem_act(acc1[i][j][r] + (a.b1 ? a.b1[n + r] : 0.f), a.act1);
      *reinterpret_cast<float4*>(o + n) = make_float4(v[0], v[1], v[2], v[3]);
    }
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

// K1 + YOLOv5 s2d stem + b1 in one kernel (yolo_stem_fused_kernel): uint8 frames [B, src_h,
// src_w, src_c] -> b1's output fp32 [B, dst_h / 4, dst_w / 4, ldo] channels [co_off, co_off + 32).
// Geometry / affine arguments as tca_image_preprocess (letterbox region, pad value, quantize);
// w0 / w1: split_pairs weight images (stem 16 x 2*160 over the s2d channels, b1 32 x 2*160).
TCA_API int tca_yolo_stem_fused(const void* src, long src_batch_stride, int src_h, int src_w, int src_row_stride,
                                int src_c, int swap_rb, int dst_h, int dst_w, int batch, int reg_top, int reg_left,
                                int reg_h, int reg_w, float pad_value, int quantize_u8, float sc0, float sc1,
                                float sc2, float b0, float b1, float b2, const void* w0, const float* bias0, int act0,
                                const void* w1, const float* bias1, int act1, float* out, int ldo, int co_off,
                                hipStream_t stream) {
  if (batch <= 0) return 0;
  if (src_c < 3 || (dst_h & 3) || (dst_w & 3) || reg_h <= 0 || reg_w <= 0 || (ldo & 3) || (co_off & 3) ||
      ldo < co_off + 32 || !w0 || !w1 || !out)
    return (int)hipErrorInvalidValue;
  StemArgs a;
  a.src = (const uint8_t*)src;
  a.p = PrepParams{src_h, src_w, src_row_stride, src_c, src_batch_stride, swap_rb, dst_h, dst_w, 16, 2,
                   reg_top, reg_left, reg_h, reg_w, pad_value, quantize_u8, sc0, sc1, sc2, b0, b1, b2};
  a.w0 = (const __hip_bfloat16*)w0; a.b0 = bias0; a.w1 = (const __hip_bfloat16*)w1; a.b1 = bias1;
  a.act0 = act0; a.act1 = act1; a.out = out; a.ldo = ldo; a.co_off = co_off;
  a.B = batch; a.H0 = dst_h / 2; a.W0 = dst_w / 2; a.H1 = dst_h / 4; a.W1 = dst_w / 4;
  // 8-row tiles (44 KiB LDS, three workgroups per CU; 4-row tiles measured 244 vs 204 us: more
  // workgroups per CU but 11 / 4 instead of 19 / 8 sampled rows per output row)
  constexpr int ty = 8;
  const long tiles = (long)batch * ((a.H1 + ty - 1) / ty) * ((a.W1 + 15) / 16);
  if (tiles >= (1L << 31)) return (int)hipErrorInvalidValue;
  yolo_stem_fused_kernel<ty><<<(unsigned)tiles, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}
