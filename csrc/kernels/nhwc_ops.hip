// Small NHWC bf16 data-movement kernels for the concat-free detector plans:
//  * max-pool k x k, stride 1, pad k/2 (YOLOv5 SPPF) or strided (ResNet stem), slice in -> slice out
//  * nearest 2x upsample (YOLOv5 PANet), channel slice in -> slice out
// Both move 16 B (8 channels) per thread; slices are ci_off/ldi, co_off/ldo.
#include "tca_common.h"

using namespace tca;

namespace {

__device__ __forceinline__ void bf16x8_max(uint4& acc, const uint4& v) {
  __hip_bfloat16* a = reinterpret_cast<__hip_bfloat16*>(&acc);
  const __hip_bfloat16* b = reinterpret_cast<const __hip_bfloat16*>(&v);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = __float2bfloat16(fmaxf(__bfloat162float(a[e]), __bfloat162float(b[e])));
}

// k x k max-pool, stride s, pad p (out-of-image taps ignored, as nn.MaxPool2d's -inf padding)
__global__ void __launch_bounds__(256) maxpool_kernel(const __hip_bfloat16* __restrict__ in, int B, int H, int W,
                                                      int C, int ldi, int ci_off, int k, int s, int p, int Ho, int Wo,
                                                      __hip_bfloat16* __restrict__ out, int ldo, int co_off) {
  // 32-bit index math (host guarantees total < 2^31): 64-bit div/mod is ~150 VALU each
  const unsigned c8 = C / 8;
  const unsigned total = (unsigned)B * Ho * Wo * c8;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int cv = (int)(t % c8);
    const unsigned pix = t / c8;
    const unsigned yx = pix % ((unsigned)Wo * Ho);
    const int x = (int)(yx % (unsigned)Wo), y = (int)(yx / (unsigned)Wo), b = (int)(pix / ((unsigned)Wo * Ho));
    uint4 acc = make_uint4(0, 0, 0, 0);
    bool first = true;
    for (int dy = 0; dy < k; ++dy) {
      const int yy = y * s - p + dy;
      if (yy < 0 || yy >= H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int xx = x * s - p + dx;
        if (xx < 0 || xx >= W) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(in + (((long)b * H + yy) * W + xx) * ldi + ci_off + cv * 8);
        if (first) { acc = v; first = false; } else bf16x8_max(acc, v);
      }
    }
    *reinterpret_cast<uint4*>(out + (long)pix * ldo + co_off + cv * 8) = acc;
  }
}

__global__ void __launch_bounds__(256) upsample2x_kernel(const __hip_bfloat16* __restrict__ in, int B, int H, int W,
                                                         int C, int ldi, int ci_off,
                                                         __hip_bfloat16* __restrict__ out, int ldo, int co_off) {
  const unsigned c8 = C / 8;
  const int Ho = 2 * H, Wo = 2 * W;
  const unsigned total = (unsigned)B * Ho * Wo * c8;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int cv = (int)(t % c8);
    const unsigned pix = t / c8;
    const unsigned yx = pix % ((unsigned)Wo * Ho);
    const int x = (int)(yx % (unsigned)Wo), y = (int)(yx / (unsigned)Wo), b = (int)(pix / ((unsigned)Wo * Ho));
    const uint4 v = *reinterpret_cast<const uint4*>(in + (((long)b * H + y / 2) * W + x / 2) * ldi + ci_off + cv * 8);
    *reinterpret_cast<uint4*>(out + (long)pix * ldo + co_off + cv * 8) = v;
  }
}

int grid_for(long work) { return (int)min((work + 255) / 256, (long)4096); }

}  // namespace

TCA_API int tca_maxpool_nhwc(const void* in, int B, int H, int W, int C, int ldi, int ci_off, int k, void* out,
                             int ldo, int co_off, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((C & 7) || (ldi & 7) || (ci_off & 7) || (ldo & 7) || (co_off & 7)) return (int)hipErrorInvalidValue;
  if ((long)B * H * W * (C / 8) >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit index math
  maxpool_kernel<<<grid_for((long)B * H * W * (C / 8)), 256, 0, stream>>>(
      (const __hip_bfloat16*)in, B, H, W, C, ldi, ci_off, k, 1, k / 2, H, W, (__hip_bfloat16*)out, ldo, co_off);
  TCA_LAUNCH_CHECK();
}

// strided max-pool (ResNet stem: k 3, s 2, p 1); output Ho x Wo given by the caller
TCA_API int tca_maxpool2d_nhwc(const void* in, int B, int H, int W, int C, int ldi, int ci_off, int k, int s, int p,
                               void* out, int Ho, int Wo, int ldo, int co_off, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((C & 7) || (ldi & 7) || (ci_off & 7) || (ldo & 7) || (co_off & 7) || s < 1 || k < 1) return (int)hipErrorInvalidValue;
  if ((long)B * Ho * Wo * (C / 8) >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit index math
  maxpool_kernel<<<grid_for((long)B * Ho * Wo * (C / 8)), 256, 0, stream>>>(
      (const __hip_bfloat16*)in, B, H, W, C, ldi, ci_off, k, s, p, Ho, Wo, (__hip_bfloat16*)out, ldo, co_off);
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_upsample2x_nhwc(const void* in, int B, int H, int W, int C, int ldi, int ci_off, void* out, int ldo,
                                int co_off, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((C & 7) || (ldi & 7) || (ci_off & 7) || (ldo & 7) || (co_off & 7)) return (int)hipErrorInvalidValue;
  if ((long)B * 4 * H * W * (C / 8) >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit index math
  upsample2x_kernel<<<grid_for((long)B * 4 * H * W * (C / 8)), 256, 0, stream>>>(
      (const __hip_bfloat16*)in, B, H, W, C, ldi, ci_off, (__hip_bfloat16*)out, ldo, co_off);
  TCA_LAUNCH_CHECK();
}
