// Small NHWC data-movement kernels for the concat-free detector plans, bf16 or
// fp32 activations (dtype kBF16 / kF32):
//  * max-pool k x k, stride 1, pad k/2 (YOLOv5 SPPF) or strided (ResNet stem), slice in -> slice out
//  * nearest 2x upsample (YOLOv5 PANet), channel slice in -> slice out
// Both move 16 B per thread (8 bf16 or 4 fp32 channels); slices are ci_off/ldi, co_off/ldo.
#include "tca_common.h"

using namespace tca;

namespace {

template <typename T>
__device__ __forceinline__ void vec_max(uint4& acc, const uint4& v) {
  constexpr int E = 16 / sizeof(T);
  T* a = reinterpret_cast<T*>(&acc);
  const T* b = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int e = 0; e < E; ++e) a[e] = from_f32<T>(fmaxf(to_f32(a[e]), to_f32(b[e])));
}

// k x k max-pool, stride s, pad p (out-of-image taps ignored, as nn.MaxPool2d's -inf padding)
template <typename T>
__global__ void __launch_bounds__(256) maxpool_kernel(const T* __restrict__ in, int B, int H, int W, int C, int ldi,
                                                      int ci_off, int k, int s, int p, int Ho, int Wo,
                                                      T* __restrict__ out, int ldo, int co_off) {
  constexpr int E = 16 / sizeof(T);
  // 32-bit index math (host guarantees total < 2^31): 64-bit div/mod is ~150 VALU each
  const unsigned cv_n = C / E;
  const unsigned total = (unsigned)B * Ho * Wo * cv_n;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int cv = (int)(t % cv_n);
    const unsigned pix = t / cv_n;
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
        const uint4 v = *reinterpret_cast<const uint4*>(in + (((long)b * H + yy) * W + xx) * ldi + ci_off + cv * E);
        if (first) { acc = v; first = false; } else vec_max<T>(acc, v);
      }
    }
    *reinterpret_cast<uint4*>(out + (long)pix * ldo + co_off + cv * E) = acc;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) upsample2x_kernel(const T* __restrict__ in, int B, int H, int W, int C, int ldi,
                                                         int ci_off, T* __restrict__ out, int ldo, int co_off) {
  constexpr int E = 16 / sizeof(T);
  const unsigned cv_n = C / E;
  const int Ho = 2 * H, Wo = 2 * W;
  const unsigned total = (unsigned)B * Ho * Wo * cv_n;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int cv = (int)(t % cv_n);
    const unsigned pix = t / cv_n;
    const unsigned yx = pix % ((unsigned)Wo * Ho);
    const int x = (int)(yx % (unsigned)Wo), y = (int)(yx / (unsigned)Wo), b = (int)(pix / ((unsigned)Wo * Ho));
    const uint4 v = *reinterpret_cast<const uint4*>(in + (((long)b * H + y / 2) * W + x / 2) * ldi + ci_off + cv * E);
    *reinterpret_cast<uint4*>(out + (long)pix * ldo + co_off + cv * E) = v;
  }
}

// YOLOv5 SPPF's three chained k x k stride-1 max-pools in one launch: y1 = pool(y0), y2 = pool(y1),
// y3 = pool(y2) (the same clipped-window maxes as three maxpool_kernel launches, so the same bits).
// A workgroup owns one image and 4 16-B channel vectors; the plane lives in LDS and each pool is a
// row pass then a column pass (separable max), written out after each round.
template <typename T, int NV>
__global__ void __launch_bounds__(256) sppf_pool3_kernel(const T* __restrict__ in, int H, int W, int C, int ldi,
                                                         int ci_off, int k, T* __restrict__ out, int ldo, int o1,
                                                         int o2, int o3) {
  constexpr int E = 16 / sizeof(T);
  extern __shared__ uint4 lds[];  // [2][H * W][NV]
  const int HW = H * W, nvg = C / (E * NV);
  const int b = blockIdx.x / nvg, v0 = (blockIdx.x - (blockIdx.x / nvg) * nvg) * NV;
  uint4* A = lds;
  uint4* Tm = lds + HW * NV;
  const int r = k / 2;
  for (int i = threadIdx.x; i < HW * NV; i += blockDim.x) {
    const int p = i / NV, v = i - (i / NV) * NV;
    A[i] = *reinterpret_cast<const uint4*>(in + ((long)b * HW + p) * ldi + ci_off + (v0 + v) * E);
  }
  __syncthreads();
  const int offs[3] = {o1, o2, o3};
  for (int round = 0; round < 3; ++round) {
    for (int i = threadIdx.x; i < HW * NV; i += blockDim.x) {  // rows
      const int p = i / NV, v = i - (i / NV) * NV, y = p / W, x = p - (p / W) * W;
      const int x0 = x - r < 0 ? 0 : x - r, x1 = x + r >= W ? W - 1 : x + r;
      uint4 acc = A[(y * W + x0) * NV + v];
      for (int xx = x0 + 1; xx <= x1; ++xx) vec_max<T>(acc, A[(y * W + xx) * NV + v]);
      Tm[i] = acc;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HW * NV; i += blockDim.x) {  // columns
      const int p = i / NV, v = i - (i / NV) * NV, y = p / W, x = p - (p / W) * W;
      const int y0 = y - r < 0 ? 0 : y - r, y1 = y + r >= H ? H - 1 : y + r;
      uint4 acc = Tm[(y0 * W + x) * NV + v];
      for (int yy = y0 + 1; yy <= y1; ++yy) vec_max<T>(acc, Tm[(yy * W + x) * NV + v]);
      A[i] = acc;
      *reinterpret_cast<uint4*>(out + ((long)b * HW + p) * ldo + offs[round] + (v0 + v) * E) = acc;
    }
    __syncthreads();
  }
}

int grid_for(long work) { return (int)min((work + 255) / 256, (long)4096); }

bool slices_ok(int C, int ldi, int ci_off, int ldo, int co_off, int dtype) {
  if (dtype != kBF16 && dtype != kF32) return false;
  const int e = dtype == kF32 ? 3 : 7;  // channels per 16-B vector - 1
  return !((C & e) || (ldi & e) || (ci_off & e) || (ldo & e) || (co_off & e));
}

int launch_pool(const void* in, int B, int H, int W, int C, int ldi, int ci_off, int k, int s, int p, void* out,
                int Ho, int Wo, int ldo, int co_off, int dtype, hipStream_t stream) {
  const int E = dtype == kF32 ? 4 : 8;
  const int g = grid_for((long)B * Ho * Wo * (C / E));
  if (dtype == kF32)
    maxpool_kernel<float><<<g, 256, 0, stream>>>((const float*)in, B, H, W, C, ldi, ci_off, k, s, p, Ho, Wo,
                                                 (float*)out, ldo, co_off);
  else
    maxpool_kernel<__hip_bfloat16><<<g, 256, 0, stream>>>((const __hip_bfloat16*)in, B, H, W, C, ldi, ci_off, k, s,
                                                          p, Ho, Wo, (__hip_bfloat16*)out, ldo, co_off);
  TCA_LAUNCH_CHECK();
}

}  // namespace

TCA_API int tca_maxpool_nhwc(const void* in, int B, int H, int W, int C, int ldi, int ci_off, int k, void* out,
                             int ldo, int co_off, int dtype, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!slices_ok(C, ldi, ci_off, ldo, co_off, dtype)) return (int)hipErrorInvalidValue;
  if ((long)B * H * W * C >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit index math
  return launch_pool(in, B, H, W, C, ldi, ci_off, k, 1, k / 2, out, H, W, ldo, co_off, dtype, stream);
}

// strided max-pool (ResNet stem: k 3, s 2, p 1); output Ho x Wo given by the caller
TCA_API int tca_maxpool2d_nhwc(const void* in, int B, int H, int W, int C, int ldi, int ci_off, int k, int s, int p,
                               void* out, int Ho, int Wo, int ldo, int co_off, int dtype, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!slices_ok(C, ldi, ci_off, ldo, co_off, dtype) || s < 1 || k < 1) return (int)hipErrorInvalidValue;
  if ((long)B * Ho * Wo * C >= (1L << 31)) return (int)hipErrorInvalidValue;
  return launch_pool(in, B, H, W, C, ldi, ci_off, k, s, p, out, Ho, Wo, ldo, co_off, dtype, stream);
}

TCA_API int tca_upsample2x_nhwc(const void* in, int B, int H, int W, int C, int ldi, int ci_off, void* out, int ldo,
                                int co_off, int dtype, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!slices_ok(C, ldi, ci_off, ldo, co_off, dtype)) return (int)hipErrorInvalidValue;
  if ((long)B * 4 * H * W * C >= (1L << 31)) return (int)hipErrorInvalidValue;
  const int E = dtype == kF32 ? 4 : 8;
  const int g = grid_for((long)B * 4 * H * W * (C / E));
  if (dtype == kF32)
    upsample2x_kernel<float><<<g, 256, 0, stream>>>((const float*)in, B, H, W, C, ldi, ci_off, (float*)out, ldo,
                                                    co_off);
  else
    upsample2x_kernel<__hip_bfloat16><<<g, 256, 0, stream>>>((const __hip_bfloat16*)in, B, H, W, C, ldi, ci_off,
                                                             (__hip_bfloat16*)out, ldo, co_off);
  TCA_LAUNCH_CHECK();
}

// SPPF: the three chained k x k stride-1 max-pools of channels [ci_off, ci_off + C) of in into the
// slices at o1, o2, o3 of out (one launch; sppf_pool3_kernel).  Needs the image plane of 4 channel
// vectors twice in LDS (H * W * 128 B <= 64 KiB); returns hipErrorInvalidValue when it does not fit
// (ops/conv.py sppf_pools then runs three tca_maxpool_nhwc).
TCA_API int tca_sppf_pool3(const void* in, int B, int H, int W, int C, int ldi, int ci_off, int k, void* out, int ldo,
                           int o1, int o2, int o3, int dtype, hipStream_t stream) {
  if (B <= 0) return 0;
  constexpr int NV = 4;
  const int E = dtype == kF32 ? 4 : 8;
  if (!slices_ok(C, ldi, ci_off, ldo, o1, dtype) || (o2 % E) || (o3 % E) || (C % (E * NV)) || k < 1 || !(k & 1))
    return (int)hipErrorInvalidValue;
  const long lds = 2L * H * W * NV * 16;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;  // (the default dynamic-LDS limit of a launch)
  const int grid = B * (C / (E * NV));
  if (dtype == kF32)
    sppf_pool3_kernel<float, NV><<<grid, 256, lds, stream>>>((const float*)in, H, W, C, ldi, ci_off, k, (float*)out,
                                                            ldo, o1, o2, o3);
  else
    sppf_pool3_kernel<__hip_bfloat16, NV><<<grid, 256, lds, stream>>>((const __hip_bfloat16*)in, H, W, C, ldi, ci_off,
                                                                     k, (__hip_bfloat16*)out, ldo, o1, o2, o3);
  TCA_LAUNCH_CHECK();
}
