// Detectron2 one-stage detector device ops (RetinaNet / FCOS on ResNet-50-FPN),
// the models behind examples/RetinaNet_detectron/config.pbtxt (clients:
// clients/detectron_client.py, clients/postprocess/detectron_postprocess.py:26-38).
//
//   retina_decode  — one thread per (image, pixel, anchor) of one FPN level: 80
//                    class logits compared against logit(thresh) (no exp for the
//                    misses), anchor box decode (Box2BoxTransform, dw/dh clamped),
//                    clip to the image, multi-label candidates compacted per
//                    (image, level) segment with a (score, ~flat index) key.
//   fcos_decode    — one thread per (image, pixel): score = sqrt(sigmoid(cls) *
//                    sigmoid(ctrness)), ltrb = relu(deltas) * stride around the
//                    point centre.
//   segment_merge  — after per-segment top-k (nms.hip tca_topk_sort, pre_max =
//                    1000 = Detectron2's per-level topk_candidates), the L level
//                    segments of an image are concatenated into one per-image
//                    candidate list (deterministic level order) for the
//                    class-aware NMS + keep-100 pass.
//   group_norm     — NHWC bf16 GroupNorm(32) + affine + ReLU for the FCOS towers:
//                    a stats pass (one block per (image, group); with 8 channels
//                    per group each pixel's group is one 16-B load) and an apply
//                    pass (in place allowed).
#include "tca_common.h"

using namespace tca;

namespace {

constexpr int kMaxAnchors = 16;

struct RetinaLevel {
  int H, W, A, C, ld_cls, ld_box, stride;
  float logit_thresh, scale_clamp, img_h, img_w;
  float aw[kMaxAnchors], ah[kMaxAnchors];
};

template <typename T>
__device__ __forceinline__ void wave_append(bool pass_any, int n_mine, int* seg_count, int& base) {
  // reserve n_mine slots per lane with one atomic per wave
  const int lane = threadIdx.x & 63;
  int incl = n_mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const int total = __shfl(incl, 63, 64);
  int b0 = 0;
  if (lane == 63 && total) b0 = atomicAdd(seg_count, total);
  b0 = __shfl(b0, 63, 64);
  base = b0 + incl - n_mine;
}

template <typename T>
__global__ void __launch_bounds__(256) retina_decode_kernel(const T* __restrict__ cls, const T* __restrict__ box,
                                                            RetinaLevel L, int level, int nlevels,
                                                            float* __restrict__ cand_box, float* __restrict__ cand_score,
                                                            int* __restrict__ cand_cls, uint64_t* __restrict__ cand_key,
                                                            int* __restrict__ cand_count, int cap) {
  const int b = blockIdx.y;
  const int id = blockIdx.x * blockDim.x + threadIdx.x;  // (pixel, anchor)
  const int total = L.H * L.W * L.A;
  const int seg = b * nlevels + level;
  int n = 0;
  float bx[4] = {0.f, 0.f, 0.f, 0.f};
  const T* c = nullptr;
  if (id < total) {
    const int a = id % L.A, pix = id / L.A;
    c = cls + ((long)b * L.H * L.W + pix) * L.ld_cls + a * L.C;
    for (int k = 0; k < L.C; ++k) n += to_f32(c[k]) > L.logit_thresh;
    if (n) {
      const int y = pix / L.W, x = pix - y * L.W;
      const T* d = box + ((long)b * L.H * L.W + pix) * L.ld_box + a * 4;
      const float aw = L.aw[a], ah = L.ah[a];
      const float cx = (float)(x * L.stride), cy = (float)(y * L.stride);
      const float dw = fminf(to_f32(d[2]), L.scale_clamp), dh = fminf(to_f32(d[3]), L.scale_clamp);
      const float px = to_f32(d[0]) * aw + cx, py = to_f32(d[1]) * ah + cy;
      const float pw = __expf(dw) * aw, ph = __expf(dh) * ah;
      bx[0] = fminf(fmaxf(px - 0.5f * pw, 0.f), L.img_w);
      bx[1] = fminf(fmaxf(py - 0.5f * ph, 0.f), L.img_h);
      bx[2] = fminf(fmaxf(px + 0.5f * pw, 0.f), L.img_w);
      bx[3] = fminf(fmaxf(py + 0.5f * ph, 0.f), L.img_h);
    }
  }
  int base;
  wave_append<T>(n > 0, n, &cand_count[seg], base);
  if (n) {
    int o = base;
    for (int k = 0; k < L.C; ++k) {
      const float v = to_f32(c[k]);
      if (v > L.logit_thresh) {
        if (o < cap) {
          const long q = (long)seg * cap + o;
          cand_box[q * 4 + 0] = bx[0]; cand_box[q * 4 + 1] = bx[1];
          cand_box[q * 4 + 2] = bx[2]; cand_box[q * 4 + 3] = bx[3];
          const float s = sigmoidf_(v);
          cand_score[q] = s;
          cand_cls[q] = k;
          cand_key[q] = make_score_key(s, (uint32_t)(id * L.C + k));
        }
        ++o;
      }
    }
  }
}

struct FcosLevel {
  int H, W, C, ld_cls, ld_box, ld_ctr, stride;
  float thresh, img_h, img_w;
};

template <typename T>
__global__ void __launch_bounds__(256) fcos_decode_kernel(const T* __restrict__ cls, const T* __restrict__ box,
                                                          const T* __restrict__ ctr, FcosLevel L, int level, int nlevels,
                                                          float* __restrict__ cand_box, float* __restrict__ cand_score,
                                                          int* __restrict__ cand_cls, uint64_t* __restrict__ cand_key,
                                                          int* __restrict__ cand_count, int cap) {
  const int b = blockIdx.y;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = b * nlevels + level;
  int n = 0;
  float bx[4] = {0.f, 0.f, 0.f, 0.f}, cs = 0.f;
  const T* c = nullptr;
  if (pix < L.H * L.W) {
    const long pb = (long)b * L.H * L.W + pix;
    c = cls + pb * L.ld_cls;
    cs = sigmoidf_(to_f32(ctr[pb * L.ld_ctr]));
    // sqrt(sig(x) * cs) > t  <=>  sig(x) > t^2 / cs
    const float need = L.thresh * L.thresh / fmaxf(cs, 1e-12f);
    for (int k = 0; k < L.C; ++k) n += sigmoidf_(to_f32(c[k])) > need;
    if (n) {
      const int y = pix / L.W, x = pix - y * L.W;
      const T* d = box + pb * L.ld_box;
      const float s = (float)L.stride;
      const float cx = ((float)x + 0.5f) * s, cy = ((float)y + 0.5f) * s;
      bx[0] = fminf(fmaxf(cx - fmaxf(to_f32(d[0]), 0.f) * s, 0.f), L.img_w);
      bx[1] = fminf(fmaxf(cy - fmaxf(to_f32(d[1]), 0.f) * s, 0.f), L.img_h);
      bx[2] = fminf(fmaxf(cx + fmaxf(to_f32(d[2]), 0.f) * s, 0.f), L.img_w);
      bx[3] = fminf(fmaxf(cy + fmaxf(to_f32(d[3]), 0.f) * s, 0.f), L.img_h);
    }
  }
  int base;
  wave_append<T>(n > 0, n, &cand_count[seg], base);
  if (n) {
    int o = base;
    const float need = L.thresh * L.thresh / fmaxf(cs, 1e-12f);
    for (int k = 0; k < L.C; ++k) {
      const float p = sigmoidf_(to_f32(c[k]));
      if (p > need) {
        if (o < cap) {
          const long q = (long)seg * cap + o;
          cand_box[q * 4 + 0] = bx[0]; cand_box[q * 4 + 1] = bx[1];
          cand_box[q * 4 + 2] = bx[2]; cand_box[q * 4 + 3] = bx[3];
          const float sc = sqrtf(p * cs);
          cand_score[q] = sc;
          cand_cls[q] = k;
          cand_key[q] = make_score_key(sc, (uint32_t)(pix * L.C + k));
        }
        ++o;
      }
    }
  }
}

// one block per image: concatenate its L sorted level lists (top pre_max each)
__global__ void __launch_bounds__(256) segment_merge_kernel(
    const float* __restrict__ box, const float* __restrict__ score, const int* __restrict__ cls,
    const uint64_t* __restrict__ key, int D, int cap_in, const int* __restrict__ order, const int* __restrict__ sorted_n,
    int pre_max, int L, float* __restrict__ obox, float* __restrict__ oscore, int* __restrict__ ocls,
    uint64_t* __restrict__ okey, int* __restrict__ ocount, int cap_out) {
  const int b = blockIdx.x;
  int off = 0;
  for (int l = 0; l < L; ++l) {
    const int seg = b * L + l;
    const int n = sorted_n[seg];
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      const int o = off + j;
      if (o >= cap_out) break;
      const long src = (long)seg * cap_in + order[(long)seg * pre_max + j];
      const long dst = (long)b * cap_out + o;
      for (int k = 0; k < D; ++k) obox[dst * D + k] = box[src * D + k];
      oscore[dst] = score[src];
      ocls[dst] = cls[src];
      // keys stay globally unique per image: fold the level into the low bits' index
      okey[dst] = (key[src] & 0xffffffff00000000ull) | (uint64_t)(0xffffffffu - (uint32_t)o);
    }
    off += n;
  }
  if (threadIdx.x == 0) ocount[b] = min(off, cap_out);
}

// GroupNorm over NHWC slices of bf16 or fp32 activations (fp32 mode): 8 channels per
// 16-B (bf16) or 2 x 16-B (fp32) vector; statistics and the affine in fp32.
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&f)[8]) {
  if constexpr (sizeof(T) == 2) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const __hip_bfloat16* e = reinterpret_cast<const __hip_bfloat16*>(&v);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = __bfloat162float(e[k]);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), c = *reinterpret_cast<const float4*>(p + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = c.x; f[5] = c.y; f[6] = c.z; f[7] = c.w;
  }
}

template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&f)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint4 v;
    __hip_bfloat16* e = reinterpret_cast<__hip_bfloat16*>(&v);
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = __float2bfloat16(f[k]);
    *reinterpret_cast<uint4*>(p) = v;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
}

// GroupNorm stats: one block per (group, image).  C channels, G groups (C/G == 8).
template <typename T>
__global__ void __launch_bounds__(256) gn_stats_kernel(const T* __restrict__ x, int HW, int C, int ldc, int c_off,
                                                       int G, float eps, float* __restrict__ stats) {
  const int g = blockIdx.x, b = blockIdx.y;
  const int cg = C / G;
  float s = 0.f, ss = 0.f;
  const T* base = x + (long)b * HW * ldc + c_off + g * cg;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    const T* q = base + (long)p * ldc;
    if (cg == 8) {
      float f[8];
      load8(q, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s += f[k];
        ss += f[k] * f[k];
      }
    } else {
      for (int k = 0; k < cg; ++k) {
        const float f = to_f32(q[k]);
        s += f;
        ss += f * f;
      }
    }
  }
  __shared__ float rs[8], rss[8];
  s = wave_sumf(s);
  ss = wave_sumf(ss);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { rs[w] = s; rss[w] = ss; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = 0.f, SS = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { S += rs[i]; SS += rss[i]; }
    const float n = (float)HW * cg;
    const float mean = S / n;
    const float var = fmaxf(SS / n - mean * mean, 0.f);
    stats[(b * G + g) * 2] = mean;
    stats[(b * G + g) * 2 + 1] = rsqrtf(var + eps);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gn_apply_kernel(const T* __restrict__ x, int B, int HW, int C, int ldc,
                                                       int c_off, int G, const float* __restrict__ stats,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       int relu, T* __restrict__ y, int ldy, int y_off) {
  const unsigned c8 = C / 8;
  const unsigned total = (unsigned)B * HW * c8;  // < 2^31 (host-checked); 32-bit div/mod
  const int cg = C / G;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int cv = (int)(t % c8);
    const unsigned pix = t / c8;
    const int b = (int)(pix / (unsigned)HW);
    float f[8];
    load8(x + (long)pix * ldc + c_off + cv * 8, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = cv * 8 + k;
      const int g = ch / cg;
      const float mean = stats[(b * G + g) * 2], rstd = stats[(b * G + g) * 2 + 1];
      f[k] = (f[k] - mean) * rstd * gamma[ch] + beta[ch];
      if (relu) f[k] = fmaxf(f[k], 0.f);
    }
    store8(y + (long)pix * ldy + y_off + cv * 8, f);
  }
}

template <typename T>
int group_norm(const void* x, int B, int HW, int C, int ldc, int c_off, int G, float eps, const float* gamma,
               const float* beta, int relu, float* stats, void* y, int ldy, int y_off, hipStream_t stream) {
  gn_stats_kernel<T><<<dim3(G, B), 256, 0, stream>>>((const T*)x, HW, C, ldc, c_off, G, eps, stats);
  const long work = (long)B * HW * (C / 8);
  gn_apply_kernel<T><<<(int)min((work + 255) / 256, (long)8192), 256, 0, stream>>>(
      (const T*)x, B, HW, C, ldc, c_off, G, stats, gamma, beta, relu, (T*)y, ldy, y_off);
  return (int)hipGetLastError();
}

}  // namespace

// One FPN level of RetinaNet: cls/box are NHWC slices (ld_*), anchors [A][2] (w, h).
TCA_API int tca_retina_decode(const void* cls, const void* box, int dtype, int batch, int H, int W, int A, int C,
                              int ld_cls, int ld_box, int stride, const float* anchors_wh, float score_thresh,
                              float scale_clamp, float img_h, float img_w, int level, int nlevels, float* cand_box,
                              float* cand_score, int* cand_cls, void* cand_key, int* cand_count, int cap,
                              int zero_counts, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (A > kMaxAnchors) return (int)hipErrorInvalidValue;
  if (zero_counts) {
    const int rc = zero_i32_async(cand_count, batch * nlevels, stream);
    if (rc) return rc;
  }
  RetinaLevel L{};
  L.H = H; L.W = W; L.A = A; L.C = C; L.ld_cls = ld_cls; L.ld_box = ld_box; L.stride = stride;
  L.logit_thresh = logf(score_thresh / (1.f - score_thresh));
  L.scale_clamp = scale_clamp; L.img_h = img_h; L.img_w = img_w;
  for (int a = 0; a < A; ++a) { L.aw[a] = anchors_wh[2 * a]; L.ah[a] = anchors_wh[2 * a + 1]; }
  dim3 grid((H * W * A + 255) / 256, batch);
  uint64_t* key = (uint64_t*)cand_key;
  if (dtype == kBF16)
    retina_decode_kernel<__hip_bfloat16><<<grid, 256, 0, stream>>>((const __hip_bfloat16*)cls,
        (const __hip_bfloat16*)box, L, level, nlevels, cand_box, cand_score, cand_cls, key, cand_count, cap);
  else if (dtype == kF32)
    retina_decode_kernel<float><<<grid, 256, 0, stream>>>((const float*)cls, (const float*)box, L, level, nlevels,
                                                           cand_box, cand_score, cand_cls, key, cand_count, cap);
  else
    return (int)hipErrorInvalidValue;
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_fcos_decode(const void* cls, const void* box, const void* ctr, int dtype, int batch, int H, int W,
                            int C, int ld_cls, int ld_box, int ld_ctr, int stride, float score_thresh, float img_h,
                            float img_w, int level, int nlevels, float* cand_box, float* cand_score, int* cand_cls,
                            void* cand_key, int* cand_count, int cap, int zero_counts, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (zero_counts) {
    const int rc = zero_i32_async(cand_count, batch * nlevels, stream);
    if (rc) return rc;
  }
  FcosLevel L{H, W, C, ld_cls, ld_box, ld_ctr, stride, score_thresh, img_h, img_w};
  dim3 grid((H * W + 255) / 256, batch);
  uint64_t* key = (uint64_t*)cand_key;
  if (dtype == kBF16)
    fcos_decode_kernel<__hip_bfloat16><<<grid, 256, 0, stream>>>((const __hip_bfloat16*)cls,
        (const __hip_bfloat16*)box, (const __hip_bfloat16*)ctr, L, level, nlevels, cand_box, cand_score, cand_cls, key,
        cand_count, cap);
  else if (dtype == kF32)
    fcos_decode_kernel<float><<<grid, 256, 0, stream>>>((const float*)cls, (const float*)box, (const float*)ctr, L,
                                                         level, nlevels, cand_box, cand_score, cand_cls, key,
                                                         cand_count, cap);
  else
    return (int)hipErrorInvalidValue;
  TCA_LAUNCH_CHECK();
}

TCA_API int tca_segment_merge(const float* box, const float* score, const int* cls, const void* key, int D, int cap_in,
                              const int* order, const int* sorted_n, int pre_max, int batch, int L, float* obox,
                              float* oscore, int* ocls, void* okey, int* ocount, int cap_out, hipStream_t stream) {
  if (batch <= 0) return 0;
  segment_merge_kernel<<<batch, 256, 0, stream>>>(box, score, cls, (const uint64_t*)key, D, cap_in, order, sorted_n,
                                                  pre_max, L, obox, oscore, ocls, (uint64_t*)okey, ocount, cap_out);
  TCA_LAUNCH_CHECK();
}

// GroupNorm(G) + affine (+ ReLU) over NHWC [B, H*W, C] slices (dtype kBF16 or kF32); y may alias x.
TCA_API int tca_group_norm_nhwc_dt(const void* x, int B, int HW, int C, int ldc, int c_off, int G, float eps,
                                   const float* gamma, const float* beta, int relu, float* stats, void* y, int ldy,
                                   int y_off, int dtype, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((C % G) || (C & 7) || (ldc & 7) || (c_off & 7) || (ldy & 7) || (y_off & 7)) return (int)hipErrorInvalidValue;
  if ((long)B * HW * (C / 8) >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit index math
  if (dtype == kF32)
    return group_norm<float>(x, B, HW, C, ldc, c_off, G, eps, gamma, beta, relu, stats, y, ldy, y_off, stream);
  if (dtype == kBF16)
    return group_norm<__hip_bfloat16>(x, B, HW, C, ldc, c_off, G, eps, gamma, beta, relu, stats, y, ldy, y_off,
                                      stream);
  return (int)hipErrorInvalidValue;
}

TCA_API int tca_group_norm_nhwc(const void* x, int B, int HW, int C, int ldc, int c_off, int G, float eps,
                                const float* gamma, const float* beta, int relu, float* stats, void* y, int ldy,
                                int y_off, hipStream_t stream) {
  return tca_group_norm_nhwc_dt(x, B, HW, C, ldc, c_off, G, eps, gamma, beta, relu, stats, y, ldy, y_off, kBF16,
                                stream);
}
