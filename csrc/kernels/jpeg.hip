// JPEG pixel reconstruction on the GPU: dequantise + 8x8 inverse DCT, then
// chroma upsampling + YCbCr -> RGB into the camera pipeline's uint8 NHWC
// frame buffer.  The host half (marker parsing + Huffman decode to quantised
// coefficients) is csrc/runtime/jpeg_entropy.cpp; together they replace the
// reference camera node's per-message cv2.imdecode
// (communicator/ros_inference.py:124-131).
//
// Kernel 1 (jpeg_idct_kernel): one wave64 per 8x8 block, lane = (row, col).
//   The coefficient block (128 B) is one coalesced load; dequantised values go
//   to LDS; the separable IDCT is a column pass then a row pass, 8 FMAs each
//   per lane, against a 64-entry basis table kept in LDS.  Output: one uint8
//   plane per component (MCU-padded), rounded and clamped like libjpeg.
// Kernel 2 (jpeg_color_kernel<HS,VS>): one thread per chroma sample writes
//   its HSxVS luma pixels.  Chroma is upsampled with libjpeg's "fancy"
//   triangular filter (h2v1: 3:1 taps, h2v2: 9:3:3:1 with the 8/7 rounding
//   bias), edges replicated, and converted with libjpeg's fixed-point
//   YCbCr -> RGB constants, so output matches a libjpeg decode to within the
//   IDCT's float-vs-integer rounding (+-1 on a few pixels).
#include "tca_common.h"

namespace {

struct JpegGeom {
  int W, H, nc, HS, VS;
  int nblocks;                // blocks per frame (all components)
  int bw[3], bh[3];           // MCU-padded block grid per component
  int boff[3];                // first block of each component within a frame
  long long poff[3];          // plane offset of each component within a frame
  int pw[3];                  // plane row pitch (= bw*8)
};

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coef,
                                                         const float* __restrict__ q,
                                                         uint8_t* __restrict__ planes, JpegGeom g,
                                                         long long coef_stride_blocks, long long plane_stride,
                                                         long long total_blocks) {
  __shared__ float basis[64];      // basis[n*8 + k] = C(k)/2 * cos((2n+1) k pi / 16)
  __shared__ float tile[4][8][9];  // one 8x8 tile per wave, +1 pad
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int y = lane >> 3, x = lane & 7;
  if (threadIdx.x < 64) {
    const int n = threadIdx.x >> 3, k = threadIdx.x & 7;
    basis[threadIdx.x] = 0.5f * (k ? 1.0f : 0.70710678118654752f) * cosf((2 * n + 1) * k * 0.19634954084936207f);
  }
  const long long gb = (long long)blockIdx.x * 4 + w;
  const bool valid = gb < total_blocks;
  int f = 0, c = 0, r = 0;
  if (valid) {
    f = (int)(gb / g.nblocks);
    r = (int)(gb - (long long)f * g.nblocks);
    c = (g.nc > 1 && r >= g.boff[1]) ? ((g.nc > 2 && r >= g.boff[2]) ? 2 : 1) : 0;
  }
  float v = 0.0f;
  if (valid) {
    v = (float)coef[((long long)f * coef_stride_blocks + r) * 64 + lane] * q[(long long)f * 192 + c * 64 + lane];
  }
  tile[w][y][x] = v;
  __syncthreads();
  // column pass: t[y][x] = sum_v basis[y][v] * F[v][x]
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) t = fmaf(basis[y * 8 + k], tile[w][k][x], t);
  __syncthreads();
  tile[w][y][x] = t;
  __syncthreads();
  // row pass: o[y][x] = sum_u basis[x][u] * t[y][u]
  float o = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) o = fmaf(basis[x * 8 + k], tile[w][y][k], o);
  if (valid) {
    const int rb = r - g.boff[c];
    const int by = rb / g.bw[c], bx = rb - by * g.bw[c];
    const int px = min(255, max(0, (int)floorf(o + 128.5f)));
    planes[(long long)f * plane_stride + g.poff[c] + (long long)(by * 8 + y) * g.pw[c] + bx * 8 + x] = (uint8_t)px;
  }
}

// libjpeg fixed-point YCbCr -> RGB (16 fraction bits, round half up)
__device__ __forceinline__ void ycc_to_rgb(int Y, int cb, int cr, uint8_t* o) {
  cb -= 128;
  cr -= 128;
  const int r = Y + ((91881 * cr + 32768) >> 16);
  const int g = Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
  const int b = Y + ((116130 * cb + 32768) >> 16);
  o[0] = (uint8_t)min(255, max(0, r));
  o[1] = (uint8_t)min(255, max(0, g));
  o[2] = (uint8_t)min(255, max(0, b));
}

// Upsampled chroma at output offset (dx, dy) within chroma sample (cx, cy).
template <int HS, int VS>
__device__ __forceinline__ int chroma(const uint8_t* __restrict__ p, int pw, int cw, int ch, int cx, int cy, int dx,
                                      int dy) {
  if constexpr (HS == 1 && VS == 1) {
    return p[cy * pw + cx];
  } else if constexpr (HS == 2 && VS == 1) {
    const uint8_t* row = p + cy * pw;
    const int c0 = row[cx];
    if (dx == 0) return cx == 0 ? c0 : (3 * c0 + row[cx - 1] + 1) >> 2;
    return cx == cw - 1 ? c0 : (3 * c0 + row[cx + 1] + 2) >> 2;
  } else {  // h2v2
    const int far_y = dy == 0 ? max(cy - 1, 0) : min(cy + 1, ch - 1);
    const uint8_t* near_row = p + cy * pw;
    const uint8_t* far_row = p + far_y * pw;
    auto colsum = [&](int xx) { return 3 * near_row[xx] + far_row[xx]; };
    const int s0 = colsum(cx);
    if (dx == 0) return cx == 0 ? (4 * s0 + 8) >> 4 : (3 * s0 + colsum(cx - 1) + 8) >> 4;
    return cx == cw - 1 ? (4 * s0 + 7) >> 4 : (3 * s0 + colsum(cx + 1) + 7) >> 4;
  }
}

template <int HS, int VS>
__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t* __restrict__ planes,
                                                          uint8_t* __restrict__ out, JpegGeom g,
                                                          long long plane_stride, long long out_stride, int B) {
  const int cw = (g.W + HS - 1) / HS, ch = (g.H + VS - 1) / VS;
  const long long per = (long long)cw * ch;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per * B) return;
  const int f = (int)(i / per);
  const int rr = (int)(i - (long long)f * per);
  const int cy = rr / cw, cx = rr - cy * cw;
  const uint8_t* base = planes + (long long)f * plane_stride;
  const uint8_t* Yp = base + g.poff[0];
  uint8_t* dst = out + (long long)f * out_stride;
#pragma unroll
  for (int dy = 0; dy < VS; ++dy) {
    const int yy = cy * VS + dy;
    if (yy >= g.H) break;
#pragma unroll
    for (int dx = 0; dx < HS; ++dx) {
      const int xx = cx * HS + dx;
      if (xx >= g.W) break;
      const int Y = Yp[(long long)yy * g.pw[0] + xx];
      uint8_t* o = dst + ((long long)yy * g.W + xx) * 3;
      if (g.nc == 1) {
        o[0] = o[1] = o[2] = (uint8_t)Y;
      } else {
        const int cb = chroma<HS, VS>(base + g.poff[1], g.pw[1], cw, ch, cx, cy, dx, dy);
        const int cr = chroma<HS, VS>(base + g.poff[2], g.pw[2], cw, ch, cx, cy, dx, dy);
        ycc_to_rgb(Y, cb, cr, o);
      }
    }
  }
}

// geom: the int32[16] record of csrc/runtime/jpeg_entropy.cpp
//   (W, H, nc, hmax, vmax, mcux, mcuy, h0, v0, h1, v1, h2, v2, nblocks).
// Returns false for layouts the colour kernel does not handle.
bool make_geom(const int32_t* s, JpegGeom& g) {
  g.W = s[0];
  g.H = s[1];
  g.nc = s[2];
  const int hmax = s[3], vmax = s[4], mcux = s[5], mcuy = s[6];
  if (g.nc != 1 && g.nc != 3) return false;
  int boff = 0;
  long long poff = 0;
  for (int c = 0; c < 3; ++c) {
    const int cc = c < g.nc ? c : 0;
    const int h = s[7 + 2 * cc], v = s[8 + 2 * cc];
    g.bw[c] = mcux * h;
    g.bh[c] = mcuy * v;
    g.pw[c] = g.bw[c] * 8;
    if (c < g.nc) {
      g.boff[c] = boff;
      g.poff[c] = poff;
      boff += g.bw[c] * g.bh[c];
      poff += (long long)g.pw[c] * g.bh[c] * 8;
    } else {
      g.boff[c] = 0x7fffffff;
      g.poff[c] = 0;
    }
  }
  g.nblocks = boff;
  if (g.nc == 1) {
    g.HS = g.VS = 1;
    return true;
  }
  // luma at full resolution, both chroma planes sampled alike
  if (s[7] != hmax || s[8] != vmax || s[9] != s[11] || s[10] != s[12]) return false;
  g.HS = hmax / s[9];
  g.VS = vmax / s[10];
  return (g.HS == 1 && g.VS == 1) || (g.HS == 2 && g.VS == 1) || (g.HS == 2 && g.VS == 2);
}

}  // namespace

// Bytes of the per-frame plane workspace for this geometry (0: unsupported).
TCA_API long long tca_jpeg_plane_bytes(const int32_t* geom) {
  JpegGeom g;
  if (!make_geom(geom, g)) return 0;
  long long n = 0;
  for (int c = 0; c < g.nc; ++c) n += (long long)g.pw[c] * g.bh[c] * 8;
  return n;
}

// B frames of one geometry: coef int16 [B][coef_stride_blocks][64], q float
// [B][3][64] (device), planes uint8 [B][plane_stride] (workspace).
TCA_API int tca_jpeg_idct(const int16_t* coef, const float* q, uint8_t* planes, const int32_t* geom,
                          long long coef_stride_blocks, long long plane_stride, int B, hipStream_t stream) {
  JpegGeom g;
  if (!make_geom(geom, g) || B <= 0) return (int)hipErrorInvalidValue;
  if (coef_stride_blocks < g.nblocks || plane_stride < tca_jpeg_plane_bytes(geom)) return (int)hipErrorInvalidValue;
  const long long total = (long long)B * g.nblocks;
  const long long grid = (total + 3) / 4;
  jpeg_idct_kernel<<<(unsigned)grid, 256, 0, stream>>>(coef, q, planes, g, coef_stride_blocks, plane_stride, total);
  TCA_LAUNCH_CHECK();
}

// planes -> uint8 RGB NHWC: frame b at out + b*out_stride, rows of W*3 bytes.
TCA_API int tca_jpeg_color(const uint8_t* planes, uint8_t* out, const int32_t* geom, long long plane_stride,
                           long long out_stride, int B, hipStream_t stream) {
  JpegGeom g;
  if (!make_geom(geom, g) || B <= 0 || out_stride < (long long)g.W * g.H * 3) return (int)hipErrorInvalidValue;
  const long long n = (long long)B * ((g.W + g.HS - 1) / g.HS) * ((g.H + g.VS - 1) / g.VS);
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (g.HS == 1 && g.VS == 1) {
    jpeg_color_kernel<1, 1><<<grid, 256, 0, stream>>>(planes, out, g, plane_stride, out_stride, B);
  } else if (g.VS == 1) {
    jpeg_color_kernel<2, 1><<<grid, 256, 0, stream>>>(planes, out, g, plane_stride, out_stride, B);
  } else {
    jpeg_color_kernel<2, 2><<<grid, 256, 0, stream>>>(planes, out, g, plane_stride, out_stride, B);
  }
  TCA_LAUNCH_CHECK();
}
