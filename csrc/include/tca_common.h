// Common helpers for the triton_client_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions shared by every kernel in csrc/kernels:
//  * every launcher is `extern "C" int tca_<name>(..., hipStream_t stream)`
//    and returns the hipError_t of the launch (0 = success); it never
//    allocates, copies synchronously or synchronises, so every launcher is
//    hipGraph-capturable (cdna_hip_programming.md §6 Guideline 9);
//  * batch sizes / element counts that the *device* produces (number of
//    candidates, voxels, points) are read from device memory inside the
//    kernel; grids are sized for the capacity and idle work-groups exit
//    early, so a whole frame pipeline has static launch shapes;
//  * wave64: every block size is a multiple of 64, masks are 64-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define TCA_API extern "C" __attribute__((visibility("default")))

#define TCA_LAUNCH_CHECK() return (int)hipGetLastError()

namespace tca {

constexpr int kWave = 64;

enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2, kU8 = 3, kI32 = 4, kPair = 5 };

// fp32-mode "pair" activation storage: per 8 channels {hi bf16 x 8 | lo bf16 x 8}
// (32 B, the footprint of 8 fp32), x = hi + lo to 2^-17 relative; consumers feed
// the halves to MFMA as stored.  Tag type for kernels templated on storage.
struct PairTag {};

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__half x) { return __half2float(x); }
__device__ __forceinline__ float to_f32(__hip_bfloat16 x) { return __bfloat162float(x); }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ __half from_f32<__half>(float x) { return __float2half(x); }
template <> __device__ __forceinline__ __hip_bfloat16 from_f32<__hip_bfloat16>(float x) { return __float2bfloat16(x); }

// Load element i of a tensor whose dtype is only known at run time.
__device__ __forceinline__ float load_any(const void* p, long i, int dtype) {
  switch (dtype) {
    case kF16: return __half2float(((const __half*)p)[i]);
    case kBF16: return __bfloat162float(((const __hip_bfloat16*)p)[i]);
    case kU8: return (float)((const uint8_t*)p)[i];
    case kI32: return (float)((const int*)p)[i];
    default: return ((const float*)p)[i];
  }
}

// 16-B global -> LDS DMA (global_load_lds_dwordx4) issued from inline asm, so
// hipcc neither counts it nor inserts the conservative vmcnt(0) it places in
// front of any ds_read that might alias an in-flight LDS DMA: the caller waits
// with its own counted s_waitcnt vmcnt(N) and a barrier before reading the
// destination (cdna_hip_programming.md §5.7 item 1).  l: the wave's LDS
// destination base (wave-uniform); lane i writes l + 16 * i.
__device__ __forceinline__ void glds16_asm(const void* g, const void* l) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);  // flat -> LDS offset (low 32 bits)
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Order-preserving float <-> uint mapping (for atomicMax on floats and for
// radix keys): larger float -> larger uint, NaN excluded by callers.
__device__ __forceinline__ uint32_t float_to_ordered(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ordered_to_float(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Wave-level inclusive sum / max using DPP-friendly shuffles (64 lanes).
__device__ __forceinline__ int wave_incl_sum(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide exclusive scan of one int per thread (blockDim multiple of 64,
// <= 1024).  `lds` must hold blockDim/64 + 1 ints.  Returns the exclusive
// prefix; *total receives the block sum (all threads).
__device__ __forceinline__ int block_excl_scan(int v, int* lds, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int incl = wave_incl_sum(v);
  if (lane == 63) lds[wid] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < nw; ++w) { int t = lds[w]; lds[w] = acc; acc += t; }
    lds[nw] = acc;
  }
  __syncthreads();
  int r = lds[wid] + incl - v;
  *total = lds[nw];
  __syncthreads();
  return r;
}

// 64-bit sort key: score (ordered) in the high word, ~index in the low word,
// so a descending sort orders by score desc, then index asc (deterministic
// tie-break independent of the order atomics handed out slots).
__device__ __forceinline__ uint64_t make_score_key(float score, uint32_t idx) {
  return ((uint64_t)float_to_ordered(score) << 32) | (uint64_t)(0xffffffffu - idx);
}

// Zero n ints on `stream` with a kernel (graph-capture safe; see util.hip).
int zero_i32_async(int* p, int n, hipStream_t stream);

}  // namespace tca
