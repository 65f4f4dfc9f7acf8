// Fused NHWC bf16 convolution on MFMA (implicit GEMM) for the detector
// backbones (YOLOv5 CSP-Darknet/PANet, PointPillars BaseBEVBackbone/RPN,
// CenterPoint RPN + heads).
//
//   out[m, n] = act( sum_k A[m, k] * W[n, k] + bias[n] ) (+ residual[m, n])
//   m = (b, oy, ox) output pixel, n = output channel,
//   k = (ky, kx, ci) with A[m, k] = in[b, oy*s - p + ky, ox*s - p + kx, ci] (0 outside)
//
// Why a hand-written kernel: MIOpen runs every conv as igemm + a separate
// bias kernel + a separate activation kernel + separate concat copies
// (rocprof of the reference-shaped PyTorch path: ~50% of GPU time in those
// element-wise passes).  Here bias, ReLU/SiLU/LeakyReLU and the Bottleneck
// residual are applied in the epilogue, inputs/outputs are channel *slices*
// of wider NHWC buffers (ci_off/ldi, co_off/ldo) so C3/PAN/BEV concats cost
// nothing, and the k=s transpose convs of the BEV necks write through a
// pixel-shuffle epilogue (one per-pixel GEMM, no col2im).
//
// Structure (CDNA4): 256 threads = 4 waves; block tile BM x BN, BK = 32;
// mfma_f32_16x16x32_bf16; A and B tiles staged global -> registers -> LDS
// (register staging because out-of-image taps must be zero-filled) with the
// next K-step's global loads issued before the current step's MFMAs
// (T14 issue-early / write-late) and two LDS buffers; LDS rows are 64 B with
// an XOR swizzle of the 16-B chunk index so the ds_read_b128 fragment reads
// are bank-conflict free.  Epilogue stages the tile through LDS so global
// stores are 16-B vectors, coalesced along channels.
#include "tca_common.h"

using namespace tca;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int BK = 32;

struct ConvArgs {
  const __hip_bfloat16* in;  // [B, H, W, ldi] (use channels [ci_off, ci_off + Cin))
  const __hip_bfloat16* w;   // [N, Kp] K-contiguous, zero-padded to Kp (multiple of 32)
  const float* bias;         // [N] or null
  const __hip_bfloat16* res; // residual [B, Ho, Wo, ldr] (channels [r_off, r_off+N)) or null
  __hip_bfloat16* out;       // [B, Ho', Wo', ldo]
  int B, H, W, Cin, ldi, ci_off;
  int Ho, Wo, KH, KW, S, P;
  int N, K, Kp;
  int ldo, co_off, ldr, r_off;
  int act;          // 0 none, 1 relu, 2 silu, 3 leaky(0.1), 4 mish; | 16: act after the residual add
  int shuffle;      // >0: transpose-conv pixel shuffle factor s (N = s*s*Cout_real)
  int M;            // B*Ho*Wo
  // fp32 mode (tca_conv_nhwc_x3): activations are fp32 and `w` is the split
  // weight [N, Kp/8, {hi[8], lo[8]}] (row stride 2*Kp bf16); in/res/out above are unused
  const float* in_f;
  const float* res_f;
  float* out_f;
  // xb kernels with OCC: uint8 [B, H, W] input-pixel occupancy; a pixel marked 0 is
  // read as zeros through the descriptor range check (no memory traffic)
  const uint8_t* occ;
};

__device__ __forceinline__ float act_fn(float v, int act) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return v / (1.f + __expf(-v));
    case 3: return v > 0.f ? v : 0.1f * v;
    case 4: {  // mish: v * tanh(softplus(v)); tanh(log(1+e^v)) = (e^2v + 2e^v) / (e^2v + 2e^v + 2)
      if (v > 20.f) return v;
      const float e = __expf(v), n = e * (e + 2.f);
      return v * n / (n + 2.f);
    }
    default: return v;
  }
}

// byte offset of 16-B chunk c (0..3) of row r in a [rows][64 B] swizzled tile
__device__ __forceinline__ int swz(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); }

// ---- shared epilogue: acc[i][j] holds D = B^T-tile x A^T-tile: col (lane&15) -> m,
// rows (lane>>4)*4 + r -> n.  Bias/act, bf16 tile staged in LDS, 16-B coalesced
// stores (+ residual, + pixel-shuffle addressing).
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void epilogue(const ConvArgs& a, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                         unsigned char* smem, int m0, int n0) {
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int act = a.act & 15;
  const bool post_res = (a.act & 16) != 0 && a.res != nullptr;  // act(conv + residual) instead of act(conv) + residual
  constexpr int LD = BN + 8;  // +16 B per row: the 16 rows a lane group writes hit distinct banks
  __hip_bfloat16* st = reinterpret_cast<__hip_bfloat16*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = wm * TM + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nl = wn * TN + j * 16 + fq * 4;
      __hip_bfloat16 q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + nl + r;
        float v = acc[i][j][r];
        if (a.bias && n < a.N) v += a.bias[n];
        q[r] = __float2bfloat16(post_res ? v : act_fn(v, act));
      }
      *reinterpret_cast<uint2*>(st + ml * LD + nl) = *reinterpret_cast<uint2*>(q);
    }
  }
  __syncthreads();
  // coalesced 16-B stores: each thread writes 8 consecutive channels of a pixel
  constexpr int VEC_PER_ROW = BN / 8;
  for (int id = tid; id < BM * VEC_PER_ROW; id += WM * WN * 64) {
    const int ml = id / VEC_PER_ROW, c8 = (id % VEC_PER_ROW) * 8;
    const int m = m0 + ml, n = n0 + c8;
    if (m >= a.M || n >= a.N) continue;
    uint4 v = *reinterpret_cast<const uint4*>(st + ml * LD + c8);
    const int ox = m % a.Wo, oy = (m / a.Wo) % a.Ho, b = m / (a.Wo * a.Ho);
    long o;
    if (a.shuffle > 0) {  // n = (sy, sx, co) -> out[b, oy*s+sy, ox*s+sx, co]
      const int s = a.shuffle, coutr = a.N / (s * s);
      const int sy = n / (s * coutr), sx = (n / coutr) % s, co = n % coutr;
      o = (((long)b * a.Ho * s + oy * s + sy) * (a.Wo * s) + ox * s + sx) * a.ldo + a.co_off + co;
    } else {
      o = (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldo + a.co_off + n;
    }
    if (a.res) {
      const __hip_bfloat16* rp = a.res + (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldr + a.r_off + n;
      uint4 r = *reinterpret_cast<const uint4*>(rp);
      const __hip_bfloat16* x = reinterpret_cast<const __hip_bfloat16*>(&v);
      const __hip_bfloat16* y = reinterpret_cast<const __hip_bfloat16*>(&r);
      __hip_bfloat16 z[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sum = __bfloat162float(x[e]) + __bfloat162float(y[e]);
        z[e] = __float2bfloat16(post_res ? act_fn(sum, act) : sum);
      }
      v = *reinterpret_cast<uint4*>(z);
    }
    *reinterpret_cast<uint4*>(a.out + o) = v;
  }
}

template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(256) conv_nhwc_kernel(ConvArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM;  // rows per wave
  constexpr int TN = BN / WN;  // cols per wave
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_CHUNKS = BM * 4, B_CHUNKS = BN * 4;  // 16-B chunks per K-step
  constexpr int A_PER_T = (A_CHUNKS + 255) / 256, B_PER_T = (B_CHUNKS + 255) / 256;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int EPI = BM * (BN + 8) * 2;
  constexpr int LDS = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  // per-thread A chunk coordinates (fixed across the K loop)
  int a_row[A_PER_T], a_c[A_PER_T], a_b[A_PER_T], a_iy0[A_PER_T], a_ix0[A_PER_T];
  bool a_ok[A_PER_T];
#pragma unroll
  for (int t = 0; t < A_PER_T; ++t) {
    const int id = tid + t * 256;
    a_row[t] = id >> 2;
    a_c[t] = id & 3;
    const int m = m0 + a_row[t];
    a_ok[t] = id < A_CHUNKS && m < a.M;
    const int mm = a_ok[t] ? m : 0;
    const int ox = mm % a.Wo, oy = (mm / a.Wo) % a.Ho, b = mm / (a.Wo * a.Ho);
    a_b[t] = b;
    a_iy0[t] = oy * a.S - a.P;
    a_ix0[t] = ox * a.S - a.P;
  }

  uint4 ra[A_PER_T], rb[B_PER_T];
  auto load_tiles = [&](int kt) {
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t) {
      uint4 v = make_uint4(0, 0, 0, 0);
      const int k0 = kt * BK + a_c[t] * 8;
      if (a_ok[t] && k0 < a.K) {
        const int tap = k0 / a.Cin, ci = k0 - tap * a.Cin;
        const int ky = tap / a.KW, kx = tap - ky * a.KW;
        const int iy = a_iy0[t] + ky, ix = a_ix0[t] + kx;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
          const __hip_bfloat16* p = a.in + (((long)a_b[t] * a.H + iy) * a.W + ix) * a.ldi + a.ci_off + ci;
          v = *reinterpret_cast<const uint4*>(p);
        }
      }
      ra[t] = v;
    }
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int id = tid + t * 256;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (id < B_CHUNKS) {
        const int n = n0 + (id >> 2);
        if (n < a.N) v = *reinterpret_cast<const uint4*>(a.w + (long)n * a.Kp + kt * BK + (id & 3) * 8);
      }
      rb[t] = v;
    }
  };
  auto store_tiles = [&](int buf) {
    unsigned char* sa = smem + buf * STAGE;
    unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t)
      if (tid + t * 256 < A_CHUNKS) *reinterpret_cast<uint4*>(sa + swz(a_row[t], a_c[t])) = ra[t];
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int id = tid + t * 256;
      if (id < B_CHUNKS) *reinterpret_cast<uint4*>(sb + swz(id >> 2, id & 3)) = rb[t];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kp / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;  // fragment row / k-chunk
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);  // issue early: latency hides under the MFMAs
    const unsigned char* sa = smem + cur * STAGE;
    const unsigned char* sb = sa + A_BYTES;
    bf16x8 af[FM], bfg[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * TM + i * 16 + fr;
      af[i] = *reinterpret_cast<const bf16x8*>(sa + swz(r, fq));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int r = wn * TN + j * 16 + fr;
      bfg[j] = *reinterpret_cast<const bf16x8*>(sb + swz(r, fq));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) store_tiles(cur ^ 1);  // write late (other buffer; read next step)
    __syncthreads();
  }

  epilogue<BM, BN, WM, WN>(a, acc, smem, m0, n0);
}


// ============================================================================
// v2: BK = 64, both operands staged global -> LDS by global_load_lds_dwordx4
// (no VGPR round trip, no per-chunk branches).  Contract: Cin % 64 == 0, so a
// 64-deep K step never straddles a filter tap and the tap (ky, kx, ci0) is
// wave-uniform and advanced incrementally (no divisions in the loop).
// Out-of-image taps and M / N tails load from a zeroed device page.  LDS rows
// are 128 B; glds writes them lane-linearly, so the bank swizzle (16-B slot
// ^= (row >> 1) & 7: the 16 rows of a ds_read_b128 lane group land on 16
// distinct (bank-row half, slot) pairs) is applied to the per-lane SOURCE
// chunk and to the fragment read (cdna_hip_programming.md rule 21).  Two LDS
// stages; the next stage's loads stay in flight across the barrier (counted
// vmcnt + raw s_barrier, never vmcnt(0) in the loop).  Tiles are walked
// XCD-major so the N-tiles of one pixel panel share an L2.
// ============================================================================
__device__ uint4 g_conv_zero_page[64];  // 1 KiB of zeros (static device memory is zero-initialised)

typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* gbl_void_t;

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((gbl_void_t)g, (lds_void_t)l, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ int swz2(int row) { return (row >> 1) & 7; }

// ONEBAR = true: one barrier per K step.  Iteration kt waits for its own
// stage (counted vmcnt), passes ONE barrier (which also proves every wave has
// finished reading stage kt-1), then restages buffer (kt-1) % STAGES with
// K step kt+STAGES-1 and runs the MFMAs of stage kt; the DMAs of up to
// STAGES-1 future steps stay in flight under them (cdna_hip_programming.md
// T3/T4 "minimum 2-phase" form generalised to STAGES buffers).
template <int BM, int BN, int WM, int WN, int STAGES, bool ONEBAR = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_glds_kernel(ConvArgs a) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BK = 64, ROWB = 128;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split over the waves' 8-row DMAs");
  constexpr int A_INS = BM / (8 * NW), B_INS = BN / (8 * NW);  // glds per wave per K step
  constexpr int NL = A_INS + B_INS;
  constexpr int EPI = BM * (BN + 8) * 2;
  constexpr int LDS = (STAGES * STAGE > EPI) ? STAGES * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // XCD-aware bijective remap: consecutive logical tiles (the N-tiles of one
  // M panel, then neighbouring panels) run on the same XCD / L2.
  const int nmt = (a.M + BM - 1) / BM, nnt = (a.N + BN - 1) / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;

  // ---- per-lane load descriptors: row within the tile, logical chunk
  const int lrow = lane >> 3, lslot = lane & 7;
  long a_base[A_INS];
  int a_iy0[A_INS], a_ix0[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wid * A_INS + j) * 8 + lrow;
    const int m = m0 + row;
    const int c = lslot ^ swz2(row);
    if (m < a.M) {
      const int ox = m % a.Wo, t = m / a.Wo, oy = t % a.Ho, b = t / a.Ho;
      a_iy0[j] = oy * a.S - a.P;
      a_ix0[j] = ox * a.S - a.P;
      a_base[j] = (((long)b * a.H + a_iy0[j]) * a.W + a_ix0[j]) * a.ldi + a.ci_off + c * 8;
    } else {
      a_iy0[j] = -(1 << 28);  // never in bounds
      a_ix0[j] = 0;
      a_base[j] = 0;
    }
  }
  const __hip_bfloat16* b_ptr[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wid * B_INS + j) * 8 + lrow;
    const int n = n0 + row;
    b_ptr[j] = n < a.N ? a.w + (long)n * a.Kp + (lslot ^ swz2(row)) * 8 : nullptr;
  }
  const long tap_stride_x = a.ldi, tap_stride_y = (long)a.W * a.ldi;

  auto issue = [&](int kt, int buf, int ky, int kx, int ci0) {
    unsigned char* sa = smem + buf * STAGE;
    unsigned char* sb = sa + A_BYTES;
    const long toff = ky * tap_stride_y + kx * tap_stride_x + ci0;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int iy = a_iy0[j] + ky, ix = a_ix0[j] + kx;
      const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const void* g = ok ? (const void*)(a.in + a_base[j] + toff) : (const void*)g_conv_zero_page;
      glds16(g, sa + (wid * A_INS + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const void* g = b_ptr[j] ? (const void*)(b_ptr[j] + kt * BK) : (const void*)g_conv_zero_page;
      glds16(g, sb + (wid * B_INS + j) * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kp / BK;
  int ky = 0, kx = 0, ci0 = 0;  // tap of the next stage to issue (wave-uniform)
  auto advance = [&]() {
    ci0 += BK;
    if (ci0 == a.Cin) {
      ci0 = 0;
      if (++kx == a.KW) { kx = 0; ++ky; }
    }
  };
  // prologue: STAGES-1 stages in flight
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) {
      issue(s, s, ky, kx, ci0);
      advance();
    }
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (ONEBAR) {
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt % STAGES;
      // stages issued and not yet waited for, after kt: kt+1 .. min(kt+STAGES-2, nk-1)
      const int after = (nk - 1 - kt) < (STAGES - 2) ? (nk - 1 - kt) : (STAGES - 2);
      if (STAGES >= 4 && after >= 2) wait_vmcnt<(STAGES >= 4 ? 2 : 0) * NL>();
      else if (STAGES >= 3 && after >= 1) wait_vmcnt<(STAGES >= 3 ? 1 : 0) * NL>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int nx = kt + STAGES - 1;
      if (nx < nk) {
        issue(nx, nx % STAGES, ky, kx, ci0);
        advance();
      }
      const unsigned char* sa = smem + cur * STAGE;
      const unsigned char* sb = sa + A_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[FM], bfg[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int r = wm * TM + i * 16 + fr;
          af[i] = *reinterpret_cast<const bf16x8*>(sa + r * ROWB + (((ks * 4 + fq) ^ swz2(r)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wn * TN + j * 16 + fr;
          bfg[j] = *reinterpret_cast<const bf16x8*>(sb + r * ROWB + (((ks * 4 + fq) ^ swz2(r)) << 4));
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the epilogue reuses the staging LDS
    asm volatile("" ::: "memory");
    epilogue<BM, BN, WM, WN>(a, acc, smem, m0, n0);
    return;
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % STAGES;
    const int nx = kt + STAGES - 1;
    if (nx < nk) {
      issue(nx, nx % STAGES, ky, kx, ci0);
      advance();
    }
    // retire stage kt: the stages issued after it may stay in flight
    const int after = (nk - 1 - kt) < (STAGES - 1) ? (nk - 1 - kt) : (STAGES - 1);
    if (STAGES >= 3 && after >= 2) wait_vmcnt<2 * NL>();
    else if (after >= 1) wait_vmcnt<NL>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const unsigned char* sa = smem + cur * STAGE;
    const unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[FM], bfg[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * TM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(sa + r * ROWB + (((ks * 4 + fq) ^ swz2(r)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * TN + j * 16 + fr;
        bfg[j] = *reinterpret_cast<const bf16x8*>(sb + r * ROWB + (((ks * 4 + fq) ^ swz2(r)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading `cur` before it is restaged
    asm volatile("" ::: "memory");
  }
  epilogue<BM, BN, WM, WN>(a, acc, smem, m0, n0);
}

// ============================================================================
// v3 "halo": 3x3 / stride 1 / pad 1, Cin = N = 64 (PointPillars BEV block 1,
// CenterPoint RPN block 1: the layers v2 runs at ~0.5 PF/s).  There the
// implicit GEMM re-reads every input pixel once per tap (9x the tensor
// through L2 for a K of only 576), which is what bounds v2.  Here:
//   * persistent workgroups, one per CU; all 9 taps x 64 x 64 of the weights
//     (72 KiB) are staged into LDS once per workgroup;
//   * the output tile is a 16 x 16 pixel block; its 18 x 18 x 64 input halo
//     (41 KiB) is staged once and every tap's A fragments are read from it at
//     (row + ky, col + kx): the input crosses L2 ~1.3x instead of 9x;
//   * two halo buffers: tile i+1's halo DMAs run under tile i's MFMAs;
//   * wave w owns output rows 4w..4w+3 (16 pixels each) x all 64 channels
//     (64x64 per wave, 16 accumulators), so per 32-deep K sub-step a wave
//     issues 8 ds_read_b128 for 16 MFMAs;
//   * the epilogue stores bias+act straight from the accumulators (8 B per
//     lane, 4 channels); those stores drain under the next tile's MFMAs.
// LDS: 2 x 352 halo pixels x 128 B + 9 x 64 x 128 B = 163,840 B (all of it).
// Measured (pp.b1.conv, B 16, 248 x 216): MFMAs + halo loads alone 67 us
// (~940 TFLOP/s); with the epilogue 127-130 us, because one wave per SIMD
// cannot overlap its LDS-staged stores with MFMAs (deferring the stores into
// the next tile's K loop measured slower: in-order vmcnt then waits on them).
// Bias values are held in registers: a per-tile global bias load exposed a
// full memory round trip per tile (189 us).
// Swizzle: 16-B slot ^= row & 7 for both images (swz_h).
// ============================================================================
constexpr int HT = 16;                       // output tile edge
// 16-B slot swizzle of a 128-B row: slot ^= row & 7.  A ds_read_b128 lane group
// reads 16 consecutive rows starting at ANY row (the halo taps shift by kx,
// ky); row & 7 keeps all 16 on distinct (bank-row half, slot) pairs for every
// start, where (row >> 1) & 7 is 2-way for unaligned starts.
__device__ __forceinline__ int swz_h(int row) { return row & 7; }
constexpr int HH = HT + 2;                   // halo edge
constexpr int H_INS = 11;                    // halo glds per wave: 4 x 11 x 8 = 352 >= 18 x 18 pixels
constexpr int H_BYTES = 4 * H_INS * 1024;    // 45,056
constexpr int W_INS = 18;                    // weight glds per wave: 4 x 18 x 1 KiB = 72 KiB
constexpr int W_BYTES = 4 * W_INS * 1024;    // 73,728

__global__ void __launch_bounds__(256) conv_halo_kernel(ConvArgs a, int ntiles) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * H_BYTES + W_BYTES];
  unsigned char* const wl = smem + 2 * H_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, lslot = lane & 7;
  const int ntx = (a.Wo + HT - 1) / HT, nty = (a.Ho + HT - 1) / HT;

  // weights once: slot s -> (tap, n, chunk'), source chunk = chunk' ^ swz_h(n)
#pragma unroll
  for (int j = 0; j < W_INS; ++j) {
    const int r8 = wid * W_INS + j;          // 1-KiB piece = 8 rows (tap, n..n+7)
    const int t = r8 >> 3, n = (r8 & 7) * 8 + lrow;
    glds16(a.w + (long)n * a.Kp + t * 64 + (lslot ^ swz_h(n)) * 8, wl + r8 * 1024);
  }

  auto issue_halo = [&](int tile, unsigned char* hb) {
    const int b = tile / (nty * ntx), rem = tile - b * nty * ntx;
    const int iy0 = (rem / ntx) * HT - 1, ix0 = (rem % ntx) * HT - 1;
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      const int r8 = wid * H_INS + j;
      const int p = r8 * 8 + lrow;           // halo pixel of this lane
      const int hy = p / HH, hx = p - hy * HH;
      const int iy = iy0 + hy, ix = ix0 + hx;
      const bool ok = p < HH * HH && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const void* g = ok ? (const void*)(a.in + (((long)b * a.H + iy) * a.W + ix) * a.ldi + a.ci_off +
                                         (lslot ^ swz_h(p)) * 8)
                         : (const void*)g_conv_zero_page;
      glds16(g, hb + r8 * 1024);
    }
  };

  // workgroup w walks tiles [w*per, (w+1)*per): consecutive tiles are x-neighbours
  // whose halos overlap (L2 hits); measured ~3% faster than a grid stride
  const int per = (ntiles + gridDim.x - 1) / gridDim.x;
  const int t_begin = blockIdx.x * per, t_end = min(ntiles, t_begin + per);
  int tile = t_begin;
  if (tile < t_end) issue_halo(tile, smem);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int act = a.act & 15;
  // this lane's 16 bias values, loaded once: a global load in the per-tile
  // epilogue would expose a full memory round trip per tile (measured 2.6x)
  float bias_r[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias_r[j][r] = a.bias ? a.bias[j * 16 + fq * 4 + r] : 0.f;
  for (int it = 0; tile < t_end; ++it, ++tile) {
    unsigned char* hb = smem + (it & 1) * H_BYTES;
    const int nxt = tile + 1;
    if (nxt < t_end) issue_halo(nxt, smem + ((it + 1) & 1) * H_BYTES);

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - ky * 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + fq;
        bf16x8 af[4], bfg[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = (wid * 4 + i + ky) * HH + fr + kx;
          af[i] = *reinterpret_cast<const bf16x8*>(hb + p * 128 + ((c ^ swz_h(p)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = j * 16 + fr;
          bfg[j] = *reinterpret_cast<const bf16x8*>(wl + (t * 64 + n) * 128 + ((c ^ swz_h(n)) << 4));
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // the next tile's halo has landed (and every wave is done with this one)
    wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    // epilogue, staged through this tile's (now free) halo buffer so the global
    // stores are whole 128-B pixel lines (8 B per lane straight from the
    // accumulators would write 32-B pieces of each line).
    // lane (fr, fq) holds pixel fr of output row 4*wid + i, channels j*16 + fq*4 + 0..3
    constexpr int LDE = 72;  // staged pixel stride in bf16 (+16 B: conflict-free 8-B writes)
    __hip_bfloat16* st = reinterpret_cast<__hip_bfloat16*>(hb);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ml = (wid * 4 + i) * HT + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = j * 16 + fq * 4;
        __hip_bfloat16 q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          q[r] = __float2bfloat16(act_fn(acc[i][j][r] + bias_r[j][r], act));
        }
        *reinterpret_cast<uint2*>(st + ml * LDE + n) = *reinterpret_cast<uint2*>(q);
      }
    }
    // LDS-only barriers: __syncthreads() would also wait for vmcnt(0), i.e. for
    // the global stores still in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int b = tile / (nty * ntx), rem = tile - b * nty * ntx;
    const int ty0 = (rem / ntx) * HT, tx0 = (rem % ntx) * HT;
#pragma unroll
    for (int k = 0; k < HT * HT * 8 / 256; ++k) {
      const int id = tid + k * 256, ml = id >> 3, c8 = (id & 7) * 8;
      const int oy = ty0 + (ml >> 4), ox = tx0 + (ml & 15);
      if (oy < a.Ho && ox < a.Wo)
        *reinterpret_cast<uint4*>(a.out + (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldo + a.co_off + c8) =
            *reinterpret_cast<const uint4*>(st + ml * LDE + c8);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done: the buffer receives
    __builtin_amdgcn_s_barrier();                        // tile it+2's halo next
    asm volatile("" ::: "memory");
  }
}

// ============================================================================
// v4 "small halo": 3x3, pad 1, stride 1 or 2, Cin and N in {16, 32} (the
// YOLOv5n stem / stage-1 / C3-bottleneck 3x3s).  At these widths the v1 tile
// moves 32-64 B per pixel per tap through L2 in 16-B pieces, 9 taps over,
// and runs 5-7x off the HBM roofline.  Here one 16x16 output tile per
// workgroup: its input halo ((15*S+3)^2 pixels x Cin) is staged into LDS once
// by global_load_lds, the packed weights (N x Kp, rows padded by 16 B so the
// 16 rows of a ds_read_b128 lane group hit distinct banks) next to it, and
// every K step's A fragments are read from the halo at the tap's offset.
// K is packed across taps (Cin 16: one 32-deep MFMA step covers two taps).
// Small LDS (11-46 KiB) keeps several workgroups per CU, so one tile's
// stores overlap another's MFMAs.  Epilogue straight from the accumulators:
// 4 lanes write a pixel's 16 channels as 32 contiguous bytes, with bias, act
// and the Bottleneck residual as in v1/v2.
// ============================================================================
template <int CIN, int NOUT, int S>
__global__ void __launch_bounds__(256) conv_small_halo_kernel(ConvArgs a) {
  constexpr int TT = 16;
  constexpr int HW_ = (TT - 1) * S + 3;            // halo edge
  constexpr int NPX = HW_ * HW_;
  constexpr int PB = CIN * 2, CPP = CIN / 8;       // bytes / 16-B chunks per halo pixel
  constexpr int INS = (NPX * CPP + 255) / 256;     // halo glds per wave
  constexpr int H_BYTES = INS * 4 * 1024;
  constexpr int KP = (9 * CIN + 31) / 32 * 32, KS = KP / 32;
  constexpr int WRS = KP * 2 + 16;                 // padded weight row (bytes)
  constexpr int FN = NOUT / 16;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[H_BYTES + NOUT * WRS];
  unsigned char* const wl = smem + H_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  const int ntx = (a.Wo + TT - 1) / TT, nty = (a.Ho + TT - 1) / TT;
  const int tile = blockIdx.x;
  const int b = tile / (nty * ntx), rem = tile - b * nty * ntx;
  const int ty0 = (rem / ntx) * TT, tx0 = (rem % ntx) * TT;
  const int iy0 = ty0 * S - 1, ix0 = tx0 * S - 1;

  // halo: lane-linear 16-B chunks, chunk g = (pixel g / CPP, part g % CPP)
#pragma unroll
  for (int j = 0; j < INS; ++j) {
    const int g = (wid * INS + j) * 64 + lane;
    const int p = g / CPP, c = g - p * CPP;
    const int hy = p / HW_, hx = p - hy * HW_;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const bool ok = p < NPX && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    const void* src = ok ? (const void*)(a.in + (((long)b * a.H + iy) * a.W + ix) * a.ldi + a.ci_off + c * 8)
                         : (const void*)g_conv_zero_page;
    glds16(src, smem + (wid * INS + j) * 1024);
  }
  // weights: plain 16-B loads into the padded rows
  for (int g = tid; g < NOUT * KP / 8; g += 256) {
    const int n = g / (KP / 8), c = g - n * (KP / 8);
    *reinterpret_cast<uint4*>(wl + n * WRS + c * 16) = *reinterpret_cast<const uint4*>(a.w + (long)n * a.Kp + c * 8);
  }
  float bias_r[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias_r[j][r] = a.bias ? a.bias[j * 16 + fq * 4 + r] : 0.f;
  wait_vmcnt<0>();
  __syncthreads();

  f32x4 acc[4][FN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = s * 32 + fq * 8;                  // this lane's 8-deep K chunk
    const int tap = k0 / CIN, ci0 = k0 - tap * CIN;
    const int ky = tap / 3, kx = tap - ky * 3;
    bf16x8 af[4], bfg[FN];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = ((wid * 4 + i) * S + ky) * HW_ + fr * S + kx;
      af[i] = tap < 9 ? *reinterpret_cast<const bf16x8*>(smem + p * PB + ci0 * 2) : bf16x8{};
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) bfg[j] = *reinterpret_cast<const bf16x8*>(wl + (j * 16 + fr) * WRS + k0 * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
  }

  const int act = a.act & 15;
  const bool post_res = (a.act & 16) != 0 && a.res != nullptr;
  const int ox = tx0 + fr;
  if (ox >= a.Wo) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oy = ty0 + wid * 4 + i;
    if (oy >= a.Ho) break;
    const long pix = ((long)b * a.Ho + oy) * a.Wo + ox;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = j * 16 + fq * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias_r[j][r];
      if (a.res) {
        const uint2 rr = *reinterpret_cast<const uint2*>(a.res + pix * a.ldr + a.r_off + n);
        const __hip_bfloat16* rv = reinterpret_cast<const __hip_bfloat16*>(&rr);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] = post_res ? act_fn(v[r] + __bfloat162float(rv[r]), act)
                          : __bfloat162float(__float2bfloat16(act_fn(v[r], act))) + __bfloat162float(rv[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
      }
      __hip_bfloat16 q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) q[r] = __float2bfloat16(v[r]);
      *reinterpret_cast<uint2*>(a.out + pix * a.ldo + a.co_off + n) = *reinterpret_cast<uint2*>(q);
    }
  }
}

bool small_halo_ok(const ConvArgs& a) {
  const bool cin = a.Cin == 16 || a.Cin == 32, n = a.N == 16 || a.N == 32;
  return cin && n && a.KH == 3 && a.KW == 3 && a.P == 1 && (a.S == 1 || a.S == 2) && a.shuffle == 0 &&
         a.Kp == (9 * a.Cin + 31) / 32 * 32 && a.Ho == (a.H - 1) / a.S + 1 && a.Wo == (a.W - 1) / a.S + 1;
}

template <int CIN, int NOUT, int S>
int launch_small_halo_t(const ConvArgs& a, hipStream_t stream) {
  const int ntiles = a.B * ((a.Ho + 15) / 16) * ((a.Wo + 15) / 16);
  conv_small_halo_kernel<CIN, NOUT, S><<<ntiles, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

int launch_small_halo(const ConvArgs& a, hipStream_t stream) {
  if (!small_halo_ok(a)) return (int)hipErrorInvalidValue;
  const int key = (a.Cin == 32) * 4 + (a.N == 32) * 2 + (a.S == 2);
  switch (key) {
    case 0: return launch_small_halo_t<16, 16, 1>(a, stream);
    case 1: return launch_small_halo_t<16, 16, 2>(a, stream);
    case 2: return launch_small_halo_t<16, 32, 1>(a, stream);
    case 3: return launch_small_halo_t<16, 32, 2>(a, stream);
    case 4: return launch_small_halo_t<32, 16, 1>(a, stream);
    case 5: return launch_small_halo_t<32, 16, 2>(a, stream);
    case 6: return launch_small_halo_t<32, 32, 1>(a, stream);
    default: return launch_small_halo_t<32, 32, 2>(a, stream);
  }
}

int g_num_cus = 0;

bool halo_ok(const ConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.S == 1 && a.P == 1 && a.Cin == 64 && a.N == 64 && a.Kp == 576 && !a.res &&
         a.shuffle == 0 && a.Ho == a.H && a.Wo == a.W;
}

int launch_halo(const ConvArgs& a, hipStream_t stream) {
  if (!halo_ok(a)) return (int)hipErrorInvalidValue;
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_num_cus <= 0)
      g_num_cus = 256;
  }
  const int ntiles = a.B * ((a.Ho + HT - 1) / HT) * ((a.Wo + HT - 1) / HT);
  const int grid = ntiles < g_num_cus ? ntiles : g_num_cus;
  conv_halo_kernel<<<grid, 256, 0, stream>>>(a, ntiles);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int STAGES = 2, bool ONEBAR = false>
int launch_glds(const ConvArgs& a, hipStream_t stream) {
  static_assert(!ONEBAR || (STAGES >= 2 && STAGES <= 4), "one-barrier pipeline: 2..4 stages");
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  conv_glds_kernel<BM, BN, WM, WN, STAGES, ONEBAR><<<nwg, WM * WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
int launch(const ConvArgs& a, hipStream_t stream) {
  dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN);
  conv_nhwc_kernel<BM, BN, WM, WN><<<grid, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// ============================================================================
// fp32 mode ("x3"): fp32 activations, fp32-accurate products on the bf16 MFMA.
//
// The reference serves fp32 models (examples/YOLOv5/config.pbtxt:7,16,
// examples/pointpillar_kitti/config.pbtxt:33,54).  gfx950 has no xf32 and its
// f32-input MFMA runs at 1/16 of the bf16 rate, so every product is split:
//   x = xh + xl,  xh = bf16_rne(x),  xl = bf16_rne(x - xh)   (|x - xh - xl| <= 2^-17 |x|)
//   x * w ~= xh*wh + xh*wl + xl*wh                        (dropped xl*wl <= 2^-16 |x w|)
// three mfma_f32_16x16x32_bf16 per fragment pair with fp32 accumulation:
// ~16 significant bits per product, 3x the bf16 MFMA work (vs 16x for f32 MFMA).
// Weights are split once on the host into [N][Kp/8][hi 8 | lo 8] (one 32-B
// row chunk per 8 channels); activations stay fp32 in HBM and are split in
// registers — at LDS staging (v1, small halo) or at the fragment read (v2,
// whose operands go global -> LDS by DMA).  Epilogues compute in fp32 and
// store fp32, residuals are fp32.
// ============================================================================
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split8(const float4& x0, const float4& x1, bf16x8& hi, bf16x8& lo) {
  const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    hi[e] = h;
    lo[e] = (__bf16)(v[e] - (float)h);
  }
}

__device__ __forceinline__ void split4(const float4& x, uint2& hi, uint2& lo) {
  const float v[4] = {x.x, x.y, x.z, x.w};
  __bf16 h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (__bf16)v[e];
    l[e] = (__bf16)(v[e] - (float)h[e]);
  }
  hi = *reinterpret_cast<const uint2*>(h);
  lo = *reinterpret_cast<const uint2*>(l);
}

__device__ __forceinline__ void mfma3(f32x4& acc, const bf16x8& bh, const bf16x8& bl, const bf16x8& ah,
                                      const bf16x8& al) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc, 0, 0, 0);
}

// fp32 epilogue: bias/act into an fp32 LDS tile, then 16-B (4-channel) coalesced
// stores with residual and pixel-shuffle addressing as in the bf16 epilogue.
// "pair" activations (fp32 mode's storage for BEV chains): 8 channels as
// {hi bf16 x 8 | lo bf16 x 8} = 32 B, the same bytes and element offsets as 8
// fp32 values.  x == float(hi) + float(lo) to 2^-17 relative, and a consumer's
// MFMA fragments are the two 16-B halves as stored: no VALU split on the read.
__device__ __forceinline__ void pair_split8(const float* v, uint4& hi, uint4& lo) {
  __bf16 h[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = (__bf16)v[e];
    l[e] = (__bf16)(v[e] - (float)h[e]);
  }
  hi = *reinterpret_cast<const uint4*>(h);
  lo = *reinterpret_cast<const uint4*>(l);
}

__device__ __forceinline__ void pair_join8(const float* p, float* v) {
  const uint4 hq = *reinterpret_cast<const uint4*>(p);
  const uint4 lq = *reinterpret_cast<const uint4*>(p + 4);
  const __bf16* h = reinterpret_cast<const __bf16*>(&hq);
  const __bf16* l = reinterpret_cast<const __bf16*>(&lq);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)h[e] + (float)l[e];
}

template <int BM, int BN, int WM, int WN, bool PAIR_OUT = false>
__device__ __forceinline__ void epilogue_f32(const ConvArgs& a, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                             unsigned char* smem, int m0, int n0) {
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int NT = WM * WN * 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int act = a.act & 15;
  const bool post_res = (a.act & 16) != 0 && a.res_f != nullptr;
  constexpr int LD = BN + 4;
  float* st = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = wm * TM + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nl = wn * TN + j * 16 + fq * 4;
      float4 q;
      float* qv = reinterpret_cast<float*>(&q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + nl + r;
        float v = acc[i][j][r];
        if (a.bias && n < a.N) v += a.bias[n];
        qv[r] = post_res ? v : act_fn(v, act);
      }
      *reinterpret_cast<float4*>(st + ml * LD + nl) = q;
    }
  }
  __syncthreads();
  if constexpr (PAIR_OUT) {
    // pair storage: 8 channels per store (residual read as pairs too)
    constexpr int V8 = BN / 8;
    for (int id = tid; id < BM * V8; id += NT) {
      const int ml = id / V8, c8 = (id % V8) * 8;
      const int m = m0 + ml, n = n0 + c8;
      if (m >= a.M || n >= a.N) continue;
      float v[8];
      const float4 v0 = *reinterpret_cast<const float4*>(st + ml * LD + c8);
      const float4 v1 = *reinterpret_cast<const float4*>(st + ml * LD + c8 + 4);
      v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
      const int ox = m % a.Wo, oy = (m / a.Wo) % a.Ho, b = m / (a.Wo * a.Ho);
      long o;
      if (a.shuffle > 0) {
        const int s = a.shuffle, coutr = a.N / (s * s);
        const int sy = n / (s * coutr), sx = (n / coutr) % s, co = n % coutr;
        o = (((long)b * a.Ho * s + oy * s + sy) * (a.Wo * s) + ox * s + sx) * a.ldo + a.co_off + co;
      } else {
        o = (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldo + a.co_off + n;
      }
      if (a.res_f) {
        float r[8];
        pair_join8(a.res_f + (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldr + a.r_off + n, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = post_res ? act_fn(v[e] + r[e], act) : v[e] + r[e];
      }
      uint4 hi, lo;
      pair_split8(v, hi, lo);
      *reinterpret_cast<uint4*>(a.out_f + o) = hi;
      *reinterpret_cast<uint4*>(a.out_f + o + 4) = lo;
    }
    return;
  }
  constexpr int VEC_PER_ROW = BN / 4;
  for (int id = tid; id < BM * VEC_PER_ROW; id += NT) {
    const int ml = id / VEC_PER_ROW, c4 = (id % VEC_PER_ROW) * 4;
    const int m = m0 + ml, n = n0 + c4;
    if (m >= a.M || n >= a.N) continue;
    float4 v = *reinterpret_cast<const float4*>(st + ml * LD + c4);
    const int ox = m % a.Wo, oy = (m / a.Wo) % a.Ho, b = m / (a.Wo * a.Ho);
    long o;
    if (a.shuffle > 0) {
      const int s = a.shuffle, coutr = a.N / (s * s);
      const int sy = n / (s * coutr), sx = (n / coutr) % s, co = n % coutr;
      o = (((long)b * a.Ho * s + oy * s + sy) * (a.Wo * s) + ox * s + sx) * a.ldo + a.co_off + co;
    } else {
      o = (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldo + a.co_off + n;
    }
    if (a.res_f) {
      const float4 r = *reinterpret_cast<const float4*>(a.res_f + (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldr +
                                                        a.r_off + n);
      if (post_res) {
        v.x = act_fn(v.x + r.x, act); v.y = act_fn(v.y + r.y, act);
        v.z = act_fn(v.z + r.z, act); v.w = act_fn(v.w + r.w, act);
      } else {
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
    }
    *reinterpret_cast<float4*>(a.out_f + o) = v;
  }
}

// ---- x3 v1: register staging (any Cin % 8 == 0).  A chunk = 8 channels of one
// pixel (two 16-B fp32 loads, split into hi / lo bf16x8); LDS holds hi and lo
// images of A and B in the bf16 kernel's [rows][64 B] swizzled layout.
template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(256) conv_nhwc_x3_kernel(ConvArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_CHUNKS = BM * 4, B_CHUNKS = BN * 4;
  constexpr int A_PER_T = (A_CHUNKS + 255) / 256, B_PER_T = (B_CHUNKS + 255) / 256;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64;
  constexpr int STAGE = 2 * (A_BYTES + B_BYTES);  // A hi, A lo, B hi, B lo
  constexpr int EPI = BM * (BN + 4) * 4;
  constexpr int LDS = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  int a_row[A_PER_T], a_c[A_PER_T], a_b[A_PER_T], a_iy0[A_PER_T], a_ix0[A_PER_T];
  bool a_ok[A_PER_T];
#pragma unroll
  for (int t = 0; t < A_PER_T; ++t) {
    const int id = tid + t * 256;
    a_row[t] = id >> 2;
    a_c[t] = id & 3;
    const int m = m0 + a_row[t];
    a_ok[t] = id < A_CHUNKS && m < a.M;
    const int mm = a_ok[t] ? m : 0;
    const int ox = mm % a.Wo, oy = (mm / a.Wo) % a.Ho, b = mm / (a.Wo * a.Ho);
    a_b[t] = b;
    a_iy0[t] = oy * a.S - a.P;
    a_ix0[t] = ox * a.S - a.P;
  }
  const long ldw = 2L * a.Kp;

  uint4 rah[A_PER_T], ral[A_PER_T], rbh[B_PER_T], rbl[B_PER_T];
  auto load_tiles = [&](int kt) {
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t) {
      float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
      const int k0 = kt * BK + a_c[t] * 8;
      if (a_ok[t] && k0 < a.K) {
        const int tap = k0 / a.Cin, ci = k0 - tap * a.Cin;
        const int ky = tap / a.KW, kx = tap - ky * a.KW;
        const int iy = a_iy0[t] + ky, ix = a_ix0[t] + kx;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
          const float* p = a.in_f + (((long)a_b[t] * a.H + iy) * a.W + ix) * a.ldi + a.ci_off + ci;
          x0 = *reinterpret_cast<const float4*>(p);
          x1 = *reinterpret_cast<const float4*>(p + 4);
        }
      }
      bf16x8 h, l;
      split8(x0, x1, h, l);
      rah[t] = *reinterpret_cast<uint4*>(&h);
      ral[t] = *reinterpret_cast<uint4*>(&l);
    }
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int id = tid + t * 256;
      uint4 h = make_uint4(0, 0, 0, 0), l = h;
      if (id < B_CHUNKS) {
        const int n = n0 + (id >> 2);
        if (n < a.N) {
          const __hip_bfloat16* p = a.w + (long)n * ldw + (kt * BK + (id & 3) * 8) * 2;
          h = *reinterpret_cast<const uint4*>(p);
          l = *reinterpret_cast<const uint4*>(p + 8);
        }
      }
      rbh[t] = h;
      rbl[t] = l;
    }
  };
  auto store_tiles = [&](int buf) {
    unsigned char* sah = smem + buf * STAGE;
    unsigned char* sal = sah + A_BYTES;
    unsigned char* sbh = sal + A_BYTES;
    unsigned char* sbl = sbh + B_BYTES;
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t)
      if (tid + t * 256 < A_CHUNKS) {
        *reinterpret_cast<uint4*>(sah + swz(a_row[t], a_c[t])) = rah[t];
        *reinterpret_cast<uint4*>(sal + swz(a_row[t], a_c[t])) = ral[t];
      }
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int id = tid + t * 256;
      if (id < B_CHUNKS) {
        *reinterpret_cast<uint4*>(sbh + swz(id >> 2, id & 3)) = rbh[t];
        *reinterpret_cast<uint4*>(sbl + swz(id >> 2, id & 3)) = rbl[t];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kp / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const unsigned char* sah = smem + cur * STAGE;
    const unsigned char* sal = sah + A_BYTES;
    const unsigned char* sbh = sal + A_BYTES;
    const unsigned char* sbl = sbh + B_BYTES;
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * TM + i * 16 + fr;
      ah[i] = *reinterpret_cast<const bf16x8*>(sah + swz(r, fq));
      al[i] = *reinterpret_cast<const bf16x8*>(sal + swz(r, fq));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int r = wn * TN + j * 16 + fr;
      bh[j] = *reinterpret_cast<const bf16x8*>(sbh + swz(r, fq));
      bl[j] = *reinterpret_cast<const bf16x8*>(sbl + swz(r, fq));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mfma3(acc[i][j], bh[j], bl[j], ah[i], al[i]);
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }
  epilogue_f32<BM, BN, WM, WN>(a, acc, smem, m0, n0);
}

// ---- x3 v2: global_load_lds staging, Cin % 32 == 0 (a 32-channel K step never
// straddles a tap).  LDS rows are 128 B for both operands: A = 32 fp32
// channels (slot s = channels 4s..4s+3), B = 4 x {hi 8, lo 8}.  A lane group
// fq reads slots 2fq and 2fq+1 of its 16 rows; the slot swizzle
// s ^ ((r ^ (r >> 3)) & 7) keeps every ds_read_b128 lane group on 16 distinct
// (bank-row half, slot) pairs for that pattern (exhaustive check over the four
// gfx950 b128 lane groups, rows at any 16-row fragment base).
__device__ __forceinline__ int swz3(int row) { return (row ^ (row >> 3)) & 7; }

template <int N>
__device__ __forceinline__ void wait_vmcnt_upto(int k) {  // vmcnt(k * N), k in [0, 3]
  if (k >= 3) wait_vmcnt<3 * N>();
  else if (k == 2) wait_vmcnt<2 * N>();
  else if (k == 1) wait_vmcnt<N>();
  else wait_vmcnt<0>();
}

// STAGES-deep LDS ring, one barrier per K step (the bf16 kernel's ONEBAR form):
// iteration kt waits for its own stage with a counted vmcnt that leaves the
// STAGES-2 younger stages in flight, passes one barrier (which also proves
// every wave is done with stage kt-1), refills that buffer with K step
// kt+STAGES-1 and runs stage kt's MFMAs.  With 3 MFMAs per fragment pair a
// 32-deep K step is ~770 cycles of matrix work per SIMD, shorter than an HBM
// round trip, so 2 stages (one step in flight) leave the MFMAs waiting on the
// DMA; 3-4 stages hide it.
template <int BM, int BN, int WM, int WN, int STAGES, bool PAIR_IN = false, bool PAIR_OUT = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_glds_x3_kernel(ConvArgs a) {
  static_assert(STAGES >= 2 && STAGES <= 5, "stages");
  constexpr int NW = WM * WN;
  constexpr int BKC = 32, ROWB = 128;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split over the waves' 8-row DMAs");
  constexpr int A_INS = BM / (8 * NW), B_INS = BN / (8 * NW);
  constexpr int NL = A_INS + B_INS;
  constexpr int EPI = BM * (BN + 4) * 4;
  constexpr int LDS = (STAGES * STAGE > EPI) ? STAGES * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nmt = (a.M + BM - 1) / BM, nnt = (a.N + BN - 1) / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;

  const int lrow = lane >> 3, lslot = lane & 7;
  long a_base[A_INS];
  int a_iy0[A_INS], a_ix0[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wid * A_INS + j) * 8 + lrow;
    const int m = m0 + row;
    const int c = lslot ^ swz3(row);
    if (m < a.M) {
      const int ox = m % a.Wo, t = m / a.Wo, oy = t % a.Ho, b = t / a.Ho;
      a_iy0[j] = oy * a.S - a.P;
      a_ix0[j] = ox * a.S - a.P;
      a_base[j] = (((long)b * a.H + a_iy0[j]) * a.W + a_ix0[j]) * a.ldi + a.ci_off + c * 4;
    } else {
      a_iy0[j] = -(1 << 28);
      a_ix0[j] = 0;
      a_base[j] = 0;
    }
  }
  const __hip_bfloat16* b_ptr[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wid * B_INS + j) * 8 + lrow;
    const int n = n0 + row;
    b_ptr[j] = n < a.N ? a.w + (long)n * 2 * a.Kp + (lslot ^ swz3(row)) * 8 : nullptr;
  }
  const long tap_stride_x = a.ldi, tap_stride_y = (long)a.W * a.ldi;

  auto issue = [&](int kt, int buf, int ky, int kx, int ci0) {
    unsigned char* sa = smem + buf * STAGE;
    unsigned char* sb = sa + A_BYTES;
    const long toff = ky * tap_stride_y + kx * tap_stride_x + ci0;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int iy = a_iy0[j] + ky, ix = a_ix0[j] + kx;
      const bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const void* g = ok ? (const void*)(a.in_f + a_base[j] + toff) : (const void*)g_conv_zero_page;
      glds16_asm(g, sa + (wid * A_INS + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const void* g = b_ptr[j] ? (const void*)(b_ptr[j] + kt * BKC * 2) : (const void*)g_conv_zero_page;
      glds16_asm(g, sb + (wid * B_INS + j) * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kp / BKC;
  int ky = 0, kx = 0, ci0 = 0;
  auto advance = [&]() {
    ci0 += BKC;
    if (ci0 == a.Cin) {
      ci0 = 0;
      if (++kx == a.KW) { kx = 0; ++ky; }
    }
  };
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < nk) {
      issue(st, st, ky, kx, ci0);
      advance();
    }
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % STAGES;
    const int after = (nk - 1 - kt) < (STAGES - 2) ? (nk - 1 - kt) : (STAGES - 2);
    wait_vmcnt_upto<NL>(after);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nx = kt + STAGES - 1;
    if (nx < nk) {
      issue(nx, nx % STAGES, ky, kx, ci0);
      advance();
    }
    const unsigned char* sa = smem + cur * STAGE;
    const unsigned char* sb = sa + A_BYTES;
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int r = wn * TN + j * 16 + fr;
      bh[j] = *reinterpret_cast<const bf16x8*>(sb + r * ROWB + (((2 * fq) ^ swz3(r)) << 4));
      bl[j] = *reinterpret_cast<const bf16x8*>(sb + r * ROWB + (((2 * fq + 1) ^ swz3(r)) << 4));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * TM + i * 16 + fr;
      if constexpr (PAIR_IN) {  // slots 2fq / 2fq+1 already hold hi / lo of channels 8fq..8fq+7
        ah[i] = *reinterpret_cast<const bf16x8*>(sa + r * ROWB + (((2 * fq) ^ swz3(r)) << 4));
        al[i] = *reinterpret_cast<const bf16x8*>(sa + r * ROWB + (((2 * fq + 1) ^ swz3(r)) << 4));
      } else {
        const float4 x0 = *reinterpret_cast<const float4*>(sa + r * ROWB + (((2 * fq) ^ swz3(r)) << 4));
        const float4 x1 = *reinterpret_cast<const float4*>(sa + r * ROWB + (((2 * fq + 1) ^ swz3(r)) << 4));
        split8(x0, x1, ah[i], al[i]);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mfma3(acc[i][j], bh[j], bl[j], ah[i], al[i]);
    __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the epilogue reuses the staging LDS
  asm volatile("" ::: "memory");
  epilogue_f32<BM, BN, WM, WN, PAIR_OUT>(a, acc, smem, m0, n0);
}

// ---- x3 pair, buffer-resource LDS DMA ("xb"): the pair-input glds kernel with
// the K loop's VALU taken out (PMC of the glds form: 3.3 VALU per MFMA, the SIMD's
// vector-issue port oversubscribed at 4 waves per SIMD):
//  * operands go global -> LDS by `buffer_load_dwordx4 ... offen lds` through a
//    buffer descriptor per tensor: each lane's 32-bit row offset is formed once
//    per tap (A) or once per tile (B), the K step's advance is the scalar soffset,
//    and a padding tap or a row past M / N reads zeros by the descriptor's range
//    check (offset 0x80000000 >= num_records) instead of a select per load;
//  * the slot swizzle is 16-row periodic (swz3 of the row within its fragment;
//    conflict-free for the b128 fragment reads at any 16-row base), so fragment
//    i / j of a wave is a constant offset from one per-lane base per operand half
//    and the reads fold it into the ds_read immediate.
// Same K order, fragments and MFMA sequence as conv_glds_x3_kernel<..., PAIR_IN, .>:
// outputs are bit-identical to it (PAIR_IN = false: fp32 input split at the fragment
// read, the camera chain's form).
__device__ __forceinline__ int swzp(int row) { return swz3(row & 15); }

__device__ __forceinline__ void bdma16(unsigned voff, __amdgpu_buffer_rsrc_t rsrc, const void* l, unsigned soff) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
               : "memory");
}

constexpr unsigned kOutOfRange = 0x80000000u;  // >= any num_records the launcher accepts (< 2^31)

template <int BM, int BN, int WM, int WN, int STAGES, bool PAIR_OUT, bool PAIR_IN = true, bool OCC = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_xb_kernel(ConvArgs a) {
  static_assert(STAGES >= 2 && STAGES <= 4, "stages");
  constexpr int NW = WM * WN;
  constexpr int BKC = 32, ROWB = 128;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split over the waves' 8-row DMAs");
  constexpr int A_INS = BM / (8 * NW), B_INS = BN / (8 * NW);
  constexpr int NL = A_INS + B_INS;
  constexpr int EPI = BM * (BN + 4) * 4;
  constexpr int LDS = (STAGES * STAGE > EPI) ? STAGES * STAGE : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nmt = (a.M + BM - 1) / BM, nnt = (a.N + BN - 1) / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int m0 = mt * BM, n0 = nt * BN;

  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.in_f, (short)0, a.B * a.H * a.W * a.ldi * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.N * a.Kp * 4, 0x00020000);

  const int lrow = lane >> 3, lslot = lane & 7;
  int a_base[A_INS], a_iy0[A_INS], a_ix0[A_INS];  // element offset of the row's tap-(0,0) pixel + slot
  unsigned a_occ[A_INS];                          // OCC: bit ky*KW+kx set when that tap's pixel is occupied
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wid * A_INS + j) * 8 + lrow;
    const int m = m0 + row;
    a_occ[j] = ~0u;
    if (m < a.M) {
      const int ox = m % a.Wo, t = m / a.Wo, oy = t % a.Ho, b = t / a.Ho;
      a_iy0[j] = oy * a.S - a.P;
      a_ix0[j] = ox * a.S - a.P;
      a_base[j] = ((b * a.H + a_iy0[j]) * a.W + a_ix0[j]) * a.ldi + a.ci_off + (lslot ^ swzp(row)) * 4;
      if constexpr (OCC) {  // once per tile, before any DMA is in flight
        unsigned msk = 0;
        for (int ky = 0; ky < a.KH; ++ky)
          for (int kx = 0; kx < a.KW; ++kx) {
            const int iy = a_iy0[j] + ky, ix = a_ix0[j] + kx;
            if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W &&
                a.occ[((long)b * a.H + iy) * a.W + ix])
              msk |= 1u << (ky * a.KW + kx);
          }
        a_occ[j] = msk;
      }
    } else {
      a_iy0[j] = -(1 << 28);
      a_ix0[j] = 0;
      a_base[j] = 0;
    }
  }
  unsigned b_off[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wid * B_INS + j) * 8 + lrow;
    const int n = n0 + row;
    b_off[j] = n < a.N ? (unsigned)(n * 2 * a.Kp + (lslot ^ swzp(row)) * 8) * 2u : kOutOfRange;
  }
  unsigned a_off[A_INS];
  auto tap_offsets = [&](int ky, int kx) {
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int iy = a_iy0[j] + ky, ix = a_ix0[j] + kx;
      bool ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      if constexpr (OCC) ok = ok && ((a_occ[j] >> (ky * a.KW + kx)) & 1u);
      a_off[j] = ok ? (unsigned)(a_base[j] + (ky * a.W + kx) * a.ldi) * 4u : kOutOfRange;
    }
  };

  unsigned char* const sbase = smem + __builtin_amdgcn_readfirstlane(wid) * (A_INS * 1024);
  auto issue = [&](int kt, int buf, int ci0) {
    unsigned char* sa = sbase + buf * STAGE;
    unsigned char* sb = smem + buf * STAGE + A_BYTES + __builtin_amdgcn_readfirstlane(wid) * (B_INS * 1024);
#pragma unroll
    for (int j = 0; j < A_INS; ++j) bdma16(a_off[j], rin, sa + j * 1024, (unsigned)ci0 * 4u);
#pragma unroll
    for (int j = 0; j < B_INS; ++j) bdma16(b_off[j], rw, sb + j * 1024, (unsigned)kt * (BKC * 4));
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kp / BKC;
  int ky = 0, kx = 0, ci0 = 0;
  tap_offsets(0, 0);
  auto advance = [&]() {
    ci0 += BKC;
    if (ci0 == a.Cin) {
      ci0 = 0;
      if (++kx == a.KW) { kx = 0; ++ky; }
      if (ky < a.KH) tap_offsets(ky, kx);
    }
  };
#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st)
    if (st < nk) {
      issue(st, st, ci0);
      advance();
    }
  const int fr = lane & 15, fq = lane >> 4;
  // per-lane fragment bases (fragment i / j: + i * 16 rows, a constant)
  const int sw = swzp(fr);
  const int a_hi = (wm * TM + fr) * ROWB + (((2 * fq) ^ sw) << 4), a_lo = (wm * TM + fr) * ROWB + (((2 * fq + 1) ^ sw) << 4);
  const int b_hi = A_BYTES + (wn * TN + fr) * ROWB + (((2 * fq) ^ sw) << 4);
  const int b_lo = A_BYTES + (wn * TN + fr) * ROWB + (((2 * fq + 1) ^ sw) << 4);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % STAGES;
    const int after = (nk - 1 - kt) < (STAGES - 2) ? (nk - 1 - kt) : (STAGES - 2);
    wait_vmcnt_upto<NL>(after);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int nx = kt + STAGES - 1;
    if (nx < nk) {
      issue(nx, nx % STAGES, ci0);
      advance();
    }
    const unsigned char* st = smem + cur * STAGE;
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(st + b_hi + j * 16 * ROWB);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + b_lo + j * 16 * ROWB);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if constexpr (PAIR_IN) {  // slots hold hi / lo of 8 channels as stored
        ah[i] = *reinterpret_cast<const bf16x8*>(st + a_hi + i * 16 * ROWB);
        al[i] = *reinterpret_cast<const bf16x8*>(st + a_lo + i * 16 * ROWB);
      } else {  // slots hold fp32 channels 8fq..8fq+3 / +4..+7: split here
        const float4 x0 = *reinterpret_cast<const float4*>(st + a_hi + i * 16 * ROWB);
        const float4 x1 = *reinterpret_cast<const float4*>(st + a_lo + i * 16 * ROWB);
        split8(x0, x1, ah[i], al[i]);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mfma3(acc[i][j], bh[j], bl[j], ah[i], al[i]);
    __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the epilogue reuses the staging LDS
  asm volatile("" ::: "memory");
  epilogue_f32<BM, BN, WM, WN, PAIR_OUT>(a, acc, smem, m0, n0);
}

// ---- x3 pair, halo-tiled 3x3 stride 1 ("hx"): the xb kernel re-reads every
// input pixel once per tap (9x the activation bytes through L2 -> LDS, a fresh
// A tile per K step).  Here a workgroup owns a 2D output tile of TH rows x 16
// columns; per 32-channel chunk it stages the (TH + 2) x 18 halo ONCE (buffer-
// descriptor LDS DMA, zero padding by the range check) and runs the chunk's 9
// tap steps from it, only the weight tile (BN x 32 channel pairs) streaming per
// step through a 2-deep ring.  A fragment is one output row of 16 pixels, i.e. 16
// consecutive halo rows at base ky * 18 + kx + row offset
// (the xb 16-row periodic swizzle is conflict-free only at 16-aligned bases; a
// fragment here starts at column kx = 0..2, so the slot swizzle is a function of
// the halo column found by exhaustive search to be conflict-free for every ds_read_b128
// lane group at all three shifts: hswz below).  K order is
// (chunk, tap) instead of xb's (tap, chunk): same products, different fp32
// summation order (not bit-identical to xb; same accuracy vs fp64).
// slot swizzle of halo column hx (0..17): 3 bits per column pair
__device__ __forceinline__ int hswz(int hx) { return (0xb29108 >> (3 * (hx >> 1))) & 7; }

// CM (column-major): the fragment axis is y instead of x: tiles of 16 rows x TH
// columns, halo stored column by column (18 rows per column), so narrow images
// (pp.b3: 54 wide) tile without the 16-column waste.
// PAIR = false: plain fp32 activations (split at the fragment read, xb's fp32-input
// form) and plain fp32 output.
template <int TH, int BN, int WM, int WN, bool CM = false, bool PAIR = true>
__global__ void __launch_bounds__(WM * WN * 64) conv_hx_kernel(ConvArgs a) {
  constexpr int TW = 16, BM = TH * TW, NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  static_assert(TM % 16 == 0 && TN % 16 == 0, "fragments");
  constexpr int HWD = TW + 2, HROWS = (TH + 2) * HWD;
  constexpr int HINS = (HROWS + 7) / 8;  // 8-row (1 KiB) DMA instructions per chunk
  constexpr int HPW = (HINS + NW - 1) / NW;
  constexpr int HBYTES = HINS * 1024, BBYTES = BN * 128;
  static_assert(BN % (8 * NW) == 0, "weight rows split over the waves' 8-row DMAs");
  constexpr int B_INS = BN / (8 * NW);
  constexpr int EPI = BM * (BN + 4) * 4;
  constexpr int RING = 2 * HBYTES + 2 * BBYTES;
  constexpr int LDS = RING > EPI ? RING : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];
  unsigned char* const halo = smem;
  unsigned char* const bring = smem + 2 * HBYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // tile extent along x / y (the fragment axis spans 16)
  constexpr int EX = CM ? TH : TW, EY = CM ? TW : TH;
  const int tx_n = (a.Wo + EX - 1) / EX, ty_n = (a.Ho + EY - 1) / EY;
  const int nmt = a.B * ty_n * tx_n, nnt = (a.N + BN - 1) / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int b = mt / (ty_n * tx_n), rem = mt - b * (ty_n * tx_n);
  const int oy0 = (rem / tx_n) * EY, ox0 = (rem - (rem / tx_n) * tx_n) * EX;
  const int n0 = nt * BN;

  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.in_f, (short)0, a.B * a.H * a.W * a.ldi * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.N * a.Kp * 4, 0x00020000);

  const int lrow = lane >> 3, lslot = lane & 7;
  unsigned h_off[HPW];  // byte offset of this lane's 16-B piece of halo row p (chunk 0)
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int p = (wid + j * NW) * 8 + lrow;
    const int u = p / HWD, v = p - (p / HWD) * HWD;  // (line, position along the fragment axis)
    const int hy = CM ? v : u, hx = CM ? u : v;
    const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
    const bool ok = p < HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    h_off[j] = ok ? (unsigned)((((b * a.H + iy) * a.W + ix) * a.ldi + a.ci_off + (lslot ^ hswz(v)) * 4) * 4)
                  : kOutOfRange;
  }
  unsigned b_off[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wid * B_INS + j) * 8 + lrow;
    const int n = n0 + row;
    b_off[j] = n < a.N ? (unsigned)(n * 2 * a.Kp + (lslot ^ swzp(row)) * 8) * 2u : kOutOfRange;
  }
  auto issue_halo = [&](int buf, int c) {
    unsigned char* dst = halo + buf * HBYTES;
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int ins = wid + j * NW;  // wave-uniform
      if (ins < HINS) bdma16(h_off[j], rin, dst + ins * 1024, (unsigned)c * 128u);
    }
  };
  auto issue_b = [&](int buf, int kt) {
    unsigned char* dst = bring + buf * BBYTES + __builtin_amdgcn_readfirstlane(wid) * (B_INS * 1024);
#pragma unroll
    for (int j = 0; j < B_INS; ++j) bdma16(b_off[j], rw, dst + j * 1024, (unsigned)kt * 128u);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nc = a.Cin / 32, S = 9 * nc;
  issue_halo(0, 0);
  issue_b(0, 0);  // step 0 = (chunk 0, tap 0): weight K step tap * nc + chunk = 0
  const int fr = lane & 15, fq = lane >> 4;
  const int sb_ = swzp(fr);
  const int b_hi = (wn * TN + fr) * 128 + (((2 * fq) ^ sb_) << 4);
  const int b_lo = (wn * TN + fr) * 128 + (((2 * fq + 1) ^ sb_) << 4);
  int c = 0, t = 0;
  for (int s = 0; s < S; ++s) {
    // everything in flight is this step's weights (and at t == 0 the chunk's halo)
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int c1 = t == 8 ? c + 1 : c, t1 = t == 8 ? 0 : t + 1;
    if (s + 1 < S) {
      // the next halo buffer was last read in chunk c - 1: every wave is past it (barrier)
      if (t1 == 0) issue_halo(c1 & 1, c1);
      issue_b((s + 1) & 1, t1 * nc + c1);
    }
    const unsigned char* hb = halo + (c & 1) * HBYTES;
    const unsigned char* bb = bring + (s & 1) * BBYTES;
    const int ky = t / 3, kx = t - (t / 3) * 3;
    const int kl = CM ? kx : ky, kf = CM ? ky : kx;  // tap offset across lines / along the fragment axis
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(bb + b_hi + j * 16 * 128);
      bl[j] = *reinterpret_cast<const bf16x8*>(bb + b_lo + j * 16 * 128);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int hp = (wm * FM + i + kl) * HWD + kf + fr;
      const int sw = hswz(kf + fr);
      if constexpr (PAIR) {
        ah[i] = *reinterpret_cast<const bf16x8*>(hb + hp * 128 + (((2 * fq) ^ sw) << 4));
        al[i] = *reinterpret_cast<const bf16x8*>(hb + hp * 128 + (((2 * fq + 1) ^ sw) << 4));
      } else {
        const float4 x0 = *reinterpret_cast<const float4*>(hb + hp * 128 + (((2 * fq) ^ sw) << 4));
        const float4 x1 = *reinterpret_cast<const float4*>(hb + hp * 128 + (((2 * fq + 1) ^ sw) << 4));
        split8(x0, x1, ah[i], al[i]);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mfma3(acc[i][j], bh[j], bl[j], ah[i], al[i]);
    __builtin_amdgcn_s_setprio(0);
    c = c1;
    t = t1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the epilogue reuses the ring LDS
  asm volatile("" ::: "memory");

  // epilogue: tile row ml = (output row within the tile) * 16 + column
  constexpr int LD = BN + 4;
  float* st = reinterpret_cast<float*>(smem);
  const int act = a.act & 15;
  const bool post_res = (a.act & 16) != 0 && a.res_f != nullptr;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = wm * TM + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nl = wn * TN + j * 16 + fq * 4;
      float4 q;
      float* qv = reinterpret_cast<float*>(&q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + nl + r;
        float v = acc[i][j][r];
        if (a.bias && n < a.N) v += a.bias[n];
        qv[r] = post_res ? v : act_fn(v, act);
      }
      *reinterpret_cast<float4*>(st + ml * LD + nl) = q;
    }
  }
  __syncthreads();
  constexpr int V8 = BN / 8;
  for (int id = tid; id < BM * V8; id += NW * 64) {
    const int ml = id / V8, c8 = (id - (id / V8) * V8) * 8;
    const int oy = oy0 + (CM ? (ml & 15) : ml / 16), ox = ox0 + (CM ? ml / 16 : (ml & 15)), n = n0 + c8;
    if (oy >= a.Ho || ox >= a.Wo || n >= a.N) continue;
    float v[8];
    const float4 v0 = *reinterpret_cast<const float4*>(st + ml * LD + c8);
    const float4 v1 = *reinterpret_cast<const float4*>(st + ml * LD + c8 + 4);
    v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    const long pix = ((long)b * a.Ho + oy) * a.Wo + ox;
    if (a.res_f) {
      float r[8];
      const float* rp = a.res_f + pix * a.ldr + a.r_off + n;
      if constexpr (PAIR) {
        pair_join8(rp, r);
      } else {
        const float4 r0 = *reinterpret_cast<const float4*>(rp), r1 = *reinterpret_cast<const float4*>(rp + 4);
        r[0] = r0.x; r[1] = r0.y; r[2] = r0.z; r[3] = r0.w; r[4] = r1.x; r[5] = r1.y; r[6] = r1.z; r[7] = r1.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = post_res ? act_fn(v[e] + r[e], act) : v[e] + r[e];
    }
    const long o = pix * a.ldo + a.co_off + n;
    if constexpr (PAIR) {
      uint4 hi, lo;
      pair_split8(v, hi, lo);
      *reinterpret_cast<uint4*>(a.out_f + o) = hi;
      *reinterpret_cast<uint4*>(a.out_f + o + 4) = lo;
    } else {
      *reinterpret_cast<float4*>(a.out_f + o) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(a.out_f + o + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// hx contract: pair in and out, 3x3, stride 1, pad 1, no pixel shuffle, Cin % 32 == 0, Kp == 9 * Cin
bool hx_ok(const ConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.S == 1 && a.P == 1 && a.shuffle == 0 && a.Cin % 32 == 0 &&
         a.Kp == 9 * a.Cin && a.Ho == a.H && a.Wo == a.W;
}

template <int TH, int BN, int WM, int WN, bool CM = false, bool PAIR = true>
int launch_hx(const ConvArgs& a, hipStream_t stream) {
  const int ex = CM ? TH : 16, ey = CM ? 16 : TH;
  const int nwg = a.B * ((a.Ho + ey - 1) / ey) * ((a.Wo + ex - 1) / ex) * ((a.N + BN - 1) / BN);
  conv_hx_kernel<TH, BN, WM, WN, CM, PAIR><<<nwg, WM * WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// auto hx choice for a 3x3 stride-1 layer: 8 x 16 (N >= 128) or 12 x 16 (N = 64) tiles, row- or
// column-major by the smaller padding, when that padding is <= 10% of the pixels.  Returns the
// tile pair {column-major tile, row-major tile} entry to use, or 0.
int hx_pick(const ConvArgs& a, int cm_tile_wide, int rm_tile_wide, int cm_tile_64, int rm_tile_64) {
  if (!hx_ok(a) || !(a.N >= 128 || a.N == 64)) return 0;
  const int th = a.N == 64 ? 12 : 8;
  const long px = (long)a.Ho * a.Wo;
  const long rm = (long)((a.Wo + 15) / 16 * 16) * ((a.Ho + th - 1) / th * th);
  const long cm = (long)((a.Ho + 15) / 16 * 16) * ((a.Wo + th - 1) / th * th);
  if ((cm <= rm ? cm : rm) * 10 > px * 11) return 0;
  return a.N == 64 ? (cm <= rm ? cm_tile_64 : rm_tile_64) : (cm <= rm ? cm_tile_wide : rm_tile_wide);
}

// ---- x3 small halo: 3x3, pad 1, stride 1/2, Cin and N in {16, 32}.  The fp32
// halo is split once while staging (register path: every halo pixel is read by
// 9 taps, so splitting at the fragment read would cost 9x the VALU); hi and lo
// halo images and hi / lo weight rows sit side by side in LDS.
template <int CIN, int NOUT, int S>
struct SmallHaloX3 {
  static constexpr int TT = 16, HW_ = (TT - 1) * S + 3, NPX = HW_ * HW_;
  static constexpr int PB = CIN * 2;                      // bytes per pixel per image
  static constexpr int H_BYTES = (NPX * PB + 15) / 16 * 16;
  static constexpr int KP = (9 * CIN + 31) / 32 * 32, KS = KP / 32;
  static constexpr int WRS = KP * 2 + 16;
  static constexpr int LDS = 2 * H_BYTES + 2 * NOUT * WRS;
};

template <int CIN, int NOUT, int S>
__global__ void __launch_bounds__(256) conv_small_halo_x3_kernel(ConvArgs a) {
  using G = SmallHaloX3<CIN, NOUT, S>;
  constexpr int TT = G::TT, HW_ = G::HW_, NPX = G::NPX, PB = G::PB, KP = G::KP, KS = G::KS, WRS = G::WRS;
  constexpr int FN = NOUT / 16, CPP = CIN / 4;  // 16-B fp32 chunks per pixel
  static_assert(G::LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];
  unsigned char* const himg = smem;
  unsigned char* const limg = smem + G::H_BYTES;
  unsigned char* const wlh = smem + 2 * G::H_BYTES;
  unsigned char* const wll = wlh + NOUT * WRS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  const int ntx = (a.Wo + TT - 1) / TT, nty = (a.Ho + TT - 1) / TT;
  const int tile = blockIdx.x;
  const int b = tile / (nty * ntx), rem = tile - b * nty * ntx;
  const int ty0 = (rem / ntx) * TT, tx0 = (rem % ntx) * TT;
  const int iy0 = ty0 * S - 1, ix0 = tx0 * S - 1;

  for (int g = tid; g < NPX * CPP; g += 256) {
    const int p = g / CPP, c = g - p * CPP;
    const int hy = p / HW_, hx = p - hy * HW_;
    const int iy = iy0 + hy, ix = ix0 + hx;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
      v = *reinterpret_cast<const float4*>(a.in_f + (((long)b * a.H + iy) * a.W + ix) * a.ldi + a.ci_off + c * 4);
    uint2 h, l;
    split4(v, h, l);
    *reinterpret_cast<uint2*>(himg + p * PB + c * 8) = h;
    *reinterpret_cast<uint2*>(limg + p * PB + c * 8) = l;
  }
  for (int g = tid; g < NOUT * KP / 8; g += 256) {
    const int n = g / (KP / 8), c = g - n * (KP / 8);
    const __hip_bfloat16* src = a.w + (long)n * 2 * a.Kp + c * 16;
    *reinterpret_cast<uint4*>(wlh + n * WRS + c * 16) = *reinterpret_cast<const uint4*>(src);
    *reinterpret_cast<uint4*>(wll + n * WRS + c * 16) = *reinterpret_cast<const uint4*>(src + 8);
  }
  float bias_r[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias_r[j][r] = a.bias ? a.bias[j * 16 + fq * 4 + r] : 0.f;
  __syncthreads();

  f32x4 acc[4][FN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k0 = s * 32 + fq * 8;
    const int tap = k0 / CIN, ci0 = k0 - tap * CIN;
    const int ky = tap / 3, kx = tap - ky * 3;
    bf16x8 ah[4], al[4], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = ((wid * 4 + i) * S + ky) * HW_ + fr * S + kx;
      ah[i] = tap < 9 ? *reinterpret_cast<const bf16x8*>(himg + p * PB + ci0 * 2) : bf16x8{};
      al[i] = tap < 9 ? *reinterpret_cast<const bf16x8*>(limg + p * PB + ci0 * 2) : bf16x8{};
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(wlh + (j * 16 + fr) * WRS + k0 * 2);
      bl[j] = *reinterpret_cast<const bf16x8*>(wll + (j * 16 + fr) * WRS + k0 * 2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mfma3(acc[i][j], bh[j], bl[j], ah[i], al[i]);
  }

  const int act = a.act & 15;
  const bool post_res = (a.act & 16) != 0 && a.res_f != nullptr;
  const int ox = tx0 + fr;
  if (ox >= a.Wo) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oy = ty0 + wid * 4 + i;
    if (oy >= a.Ho) break;
    const long pix = ((long)b * a.Ho + oy) * a.Wo + ox;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = j * 16 + fq * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias_r[j][r];
      if (a.res_f) {
        const float4 rr = *reinterpret_cast<const float4*>(a.res_f + pix * a.ldr + a.r_off + n);
        const float rv[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = post_res ? act_fn(v[r] + rv[r], act) : act_fn(v[r], act) + rv[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fn(v[r], act);
      }
      *reinterpret_cast<float4*>(a.out_f + pix * a.ldo + a.co_off + n) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

template <int CIN, int NOUT, int S>
int launch_small_halo_x3_t(const ConvArgs& a, hipStream_t stream) {
  const int ntiles = a.B * ((a.Ho + 15) / 16) * ((a.Wo + 15) / 16);
  conv_small_halo_x3_kernel<CIN, NOUT, S><<<ntiles, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// (Cin 32, stride 2) needs a 33 x 33 x 32 halo (2 x 70 KiB): not instantiated, v1 takes it
bool small_halo_x3_ok(const ConvArgs& a) { return small_halo_ok(a) && !(a.Cin == 32 && a.S == 2); }

int launch_small_halo_x3(const ConvArgs& a, hipStream_t stream) {
  if (!small_halo_x3_ok(a)) return (int)hipErrorInvalidValue;
  const int key = (a.Cin == 32) * 4 + (a.N == 32) * 2 + (a.S == 2);
  switch (key) {
    case 0: return launch_small_halo_x3_t<16, 16, 1>(a, stream);
    case 1: return launch_small_halo_x3_t<16, 16, 2>(a, stream);
    case 2: return launch_small_halo_x3_t<16, 32, 1>(a, stream);
    case 3: return launch_small_halo_x3_t<16, 32, 2>(a, stream);
    case 4: return launch_small_halo_x3_t<32, 16, 1>(a, stream);
    case 6: return launch_small_halo_x3_t<32, 32, 1>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

template <int BM, int BN, int WM, int WN, int STAGES = 2, bool PAIR_IN = false, bool PAIR_OUT = false>
int launch_glds_x3(const ConvArgs& a, hipStream_t stream) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  conv_glds_x3_kernel<BM, BN, WM, WN, STAGES, PAIR_IN, PAIR_OUT><<<nwg, WM * WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int STAGES, bool PAIR_OUT, bool PAIR_IN = true>
int launch_xb(const ConvArgs& a, hipStream_t stream) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if constexpr (PAIR_IN) {
    if (a.occ) {
      conv_xb_kernel<BM, BN, WM, WN, STAGES, PAIR_OUT, true, true><<<nwg, WM * WN * 64, 0, stream>>>(a);
      return (int)hipGetLastError();
    }
  }
  conv_xb_kernel<BM, BN, WM, WN, STAGES, PAIR_OUT, PAIR_IN><<<nwg, WM * WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// the xb kernels address through 32-bit buffer offsets: tensors below 2 GiB
bool xb_ok(const ConvArgs& a) {
  return (long)a.B * a.H * a.W * a.ldi * 4 < (1L << 31) && (long)a.N * a.Kp * 4 < (1L << 31);
}

template <bool PAIR_OUT>
int launch_glds_x3p(const ConvArgs& a, int tile, hipStream_t stream) {
  if (tile >= 68 && !xb_ok(a)) return (int)hipErrorInvalidValue;
  switch (tile) {
    case 70: return launch_xb<128, 128, 2, 4, 2, PAIR_OUT>(a, stream);
    case 71: return launch_xb<256, 64, 4, 2, 2, PAIR_OUT>(a, stream);
    case 72: return launch_xb<128, 64, 4, 2, 3, PAIR_OUT>(a, stream);
    case 73: return launch_xb<128, 128, 4, 2, 2, PAIR_OUT>(a, stream);
    case 74: return launch_xb<128, 128, 2, 4, 3, PAIR_OUT>(a, stream);
    case 75: return launch_xb<256, 64, 4, 2, 3, PAIR_OUT>(a, stream);
    case 76: return launch_xb<256, 128, 4, 2, 2, PAIR_OUT>(a, stream);
    case 77: return launch_xb<128, 64, 4, 2, 2, PAIR_OUT>(a, stream);
    // 4 waves of 64x64: half the LDS fragment reads per MFMA of the 8-wave tiles
    case 78: return launch_xb<128, 128, 2, 2, 2, PAIR_OUT>(a, stream);
    case 79: return launch_xb<256, 64, 4, 1, 2, PAIR_OUT>(a, stream);
    // one wave column: every wave reads the whole B tile, A fragments split over 8 waves
    // halo-tiled 3x3 stride-1 (pair in and out only): TH x 16 output tiles
    case 90: return PAIR_OUT && hx_ok(a) ? launch_hx<8, 128, 2, 4>(a, stream) : (int)hipErrorInvalidValue;
    case 91: return PAIR_OUT && hx_ok(a) ? launch_hx<16, 64, 4, 2>(a, stream) : (int)hipErrorInvalidValue;
    case 92: return PAIR_OUT && hx_ok(a) ? launch_hx<8, 64, 2, 4>(a, stream) : (int)hipErrorInvalidValue;
    case 93: return PAIR_OUT && hx_ok(a) ? launch_hx<16, 128, 4, 2>(a, stream) : (int)hipErrorInvalidValue;
    // column-major twins: 16 rows x TH columns
    case 94: return PAIR_OUT && hx_ok(a) ? launch_hx<8, 128, 2, 4, true>(a, stream) : (int)hipErrorInvalidValue;
    case 95: return PAIR_OUT && hx_ok(a) ? launch_hx<8, 64, 2, 4, true>(a, stream) : (int)hipErrorInvalidValue;
    // N = 64 layers: 16 x 12 tiles (192 rows, 3 fragments per wave row), 80 KiB LDS -> 2 workgroups per CU
    case 96: return PAIR_OUT && hx_ok(a) ? launch_hx<12, 64, 4, 2, true>(a, stream) : (int)hipErrorInvalidValue;
    case 97: return PAIR_OUT && hx_ok(a) ? launch_hx<12, 64, 4, 2, false>(a, stream) : (int)hipErrorInvalidValue;
    // 4x2 waves (2 A / 4 B fragments per wave) instead of 2x4
    case 102: return PAIR_OUT && hx_ok(a) ? launch_hx<8, 128, 4, 2, true>(a, stream) : (int)hipErrorInvalidValue;
    case 68: return launch_xb<256, 64, 8, 1, 2, PAIR_OUT>(a, stream);
    case 69: return launch_xb<128, 64, 8, 1, 2, PAIR_OUT>(a, stream);
    case 20: return launch_glds_x3<128, 128, 4, 2, 2, true, PAIR_OUT>(a, stream);
    case 22: return launch_glds_x3<128, 64, 4, 2, 2, true, PAIR_OUT>(a, stream);
    case 24: return launch_glds_x3<64, 128, 2, 4, 2, true, PAIR_OUT>(a, stream);
    case 25: return launch_glds_x3<128, 128, 2, 4, 2, true, PAIR_OUT>(a, stream);
    case 26: return launch_glds_x3<256, 64, 4, 2, 2, true, PAIR_OUT>(a, stream);
    case 32: return launch_glds_x3<128, 64, 4, 2, 3, true, PAIR_OUT>(a, stream);
    case 37: return launch_glds_x3<256, 128, 4, 2, 2, true, PAIR_OUT>(a, stream);
    case 41: return launch_glds_x3<128, 64, 8, 1, 2, true, PAIR_OUT>(a, stream);
    case 42: return launch_glds_x3<256, 64, 8, 1, 2, true, PAIR_OUT>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

template <int BM, int BN, int WM, int WN>
int launch_x3(const ConvArgs& a, hipStream_t stream) {
  dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN);
  conv_nhwc_x3_kernel<BM, BN, WM, WN><<<grid, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

}  // namespace

// Returns hipErrorInvalidValue when the shape is outside the kernel's
// contract (Cin, ldi, ci_off multiples of 8; N, ldo, co_off multiples of 8).
TCA_API int tca_conv_nhwc(const void* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* w,
                          const float* bias, int N, int KH, int KW, int S, int P, int Kp, void* out, int Ho, int Wo,
                          int ldo, int co_off, int act, const void* res, int ldr, int r_off, int shuffle, int tile,
                          hipStream_t stream) {
  if (B <= 0) return 0;
  if ((Cin & 7) || (ldi & 7) || (ci_off & 7) || (N & 7) || (ldo & 7) || (co_off & 7) || (Kp & 31)) return (int)hipErrorInvalidValue;
  if (res && ((ldr & 7) || (r_off & 7))) return (int)hipErrorInvalidValue;
  ConvArgs a;
  a.in = (const __hip_bfloat16*)in; a.w = (const __hip_bfloat16*)w; a.bias = bias;
  a.res = (const __hip_bfloat16*)res; a.out = (__hip_bfloat16*)out;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off;
  a.Ho = Ho; a.Wo = Wo; a.KH = KH; a.KW = KW; a.S = S; a.P = P;
  a.N = N; a.K = KH * KW * Cin; a.Kp = Kp; a.ldo = ldo; a.co_off = co_off; a.ldr = ldr; a.r_off = r_off;
  a.act = act; a.shuffle = shuffle; a.M = B * Ho * Wo;
  a.in_f = nullptr; a.res_f = nullptr; a.out_f = nullptr; a.occ = nullptr;
  if (a.K > Kp) return (int)hipErrorInvalidValue;
  // tile: 0 = auto
  // measured on MI355X (tools/bench_conv.py): 128x32 for N<=32, 128x64 for N<=64, 64x128 above
  const bool v2ok = (Cin % 64) == 0 && (Kp % 64) == 0 && Kp == a.K;
  // auto tile (measured on MI355X, tools/bench_conv.py -> profiles/conv_tiles_r1.md):
  // v2 (glds, 8 waves): 128x64 for N <= 64; 128x128 (4x2 waves) for wide-M layers,
  // 64x128 (2x4 waves) when M is small; v1 (register staging) when Cin % 64 != 0
  // v4 small-halo for 3x3 Cin, N in {16, 32} (tools/bench_conv.py: YOLOv5n stem 90 -> 35 us,
  // C3 3x3 30 -> 13 us, stage-1 downsample 39 -> 33 us)
  if (tile == 0 && small_halo_ok(a)) tile = 60;
  if (tile == 0) tile = N <= 16 ? 6 : N <= 32 ? 1 : v2ok ? (N <= 64 ? 22 : (a.M >= 40000 ? 20 : 24)) : (N <= 64 ? 2 : 5);
  // the persistent halo kernel (tile 50) is opt-in: 130 vs 137 us alone on
  // pp.b1.conv, but it holds all of a CU's LDS, and inside the camera || LiDAR
  // step it measured no gain (profiles/conv_tiles_r1.md)
  if (tile >= 10 && tile < 60 && !v2ok) return (int)hipErrorInvalidValue;
  switch (tile) {
    case 50: return launch_halo(a, stream);  // 3x3 s1 Cin = N = 64, persistent + LDS halo
    case 60: return launch_small_halo(a, stream);  // 3x3 s1/s2, Cin, N in {16, 32}, LDS halo
    case 11: return launch_glds<128, 64, 4, 1>(a, stream);
    case 12: return launch_glds<128, 128, 2, 2>(a, stream);
    case 13: return launch_glds<256, 64, 4, 1>(a, stream);
    case 14: return launch_glds<128, 256, 2, 2>(a, stream);
    case 15: return launch_glds<64, 128, 1, 4>(a, stream);
    case 16: return launch_glds<128, 64, 4, 1, 3>(a, stream);
    case 17: return launch_glds<128, 128, 2, 2, 3>(a, stream);
    case 18: return launch_glds<64, 128, 1, 4, 3>(a, stream);
    case 19: return launch_glds<256, 128, 4, 2>(a, stream);      // 8 waves
    case 20: return launch_glds<128, 128, 4, 2>(a, stream);      // 8 waves
    case 21: return launch_glds<256, 64, 8, 1>(a, stream);       // 8 waves
    case 22: return launch_glds<128, 64, 4, 2>(a, stream);       // 8 waves, 32x32 per wave
    case 23: return launch_glds<128, 64, 8, 1>(a, stream);       // 8 waves, 16x64 per wave
    case 24: return launch_glds<64, 128, 2, 4>(a, stream);       // 8 waves, 32x32 per wave
    case 25: return launch_glds<128, 128, 2, 4>(a, stream);      // 8 waves, 64x32 per wave
    case 26: return launch_glds<256, 64, 4, 2>(a, stream);       // 8 waves, 64x32 per wave
    case 27: return launch_glds<128, 256, 2, 4>(a, stream);      // 8 waves, 64x64 per wave
    // one barrier per K step, STAGES-deep glds pipeline
    case 31: return launch_glds<128, 128, 4, 2, 2, true>(a, stream);
    case 32: return launch_glds<128, 128, 4, 2, 3, true>(a, stream);
    case 33: return launch_glds<128, 64, 4, 2, 3, true>(a, stream);
    case 34: return launch_glds<128, 64, 4, 2, 4, true>(a, stream);
    case 35: return launch_glds<256, 128, 4, 2, 2, true>(a, stream);
    case 36: return launch_glds<256, 128, 4, 2, 3, true>(a, stream);
    case 37: return launch_glds<64, 128, 2, 4, 3, true>(a, stream);
    case 38: return launch_glds<256, 64, 4, 2, 3, true>(a, stream);
    case 39: return launch_glds<128, 256, 2, 4, 3, true>(a, stream);
    case 40: return launch_glds<256, 256, 2, 4, 2, true>(a, stream);
    case 41: return launch_glds<128, 64, 4, 2, 2, true>(a, stream);
    case 42: return launch_glds<64, 128, 2, 4, 2, true>(a, stream);
    case 43: return launch_glds<128, 128, 2, 2, 3, true>(a, stream);   // 4 waves
    case 44: return launch_glds<128, 64, 2, 2, 3, true>(a, stream);    // 4 waves
    case 1: return launch<128, 32, 4, 1>(a, stream);
    case 6: return launch<128, 16, 4, 1>(a, stream);  // N <= 16 (YOLOv5n stem / C3 inner convs)
    case 7: return launch<256, 16, 4, 1>(a, stream);
    case 2: return launch<128, 64, 4, 1>(a, stream);
    case 3: return launch<128, 128, 2, 2>(a, stream);
    case 4: return launch<256, 64, 4, 1>(a, stream);
    case 5: return launch<64, 128, 1, 4>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

// fp32 mode: fp32 NHWC activations (in / res / out), split weights w
// [N, Kp/8, {hi 8, lo 8}] bf16 (2*Kp per row), fp32 bias.  Same slice / residual /
// pixel-shuffle contract as tca_conv_nhwc.  tile: 0 auto, 1 v1 128x16 ... (see switch).
TCA_API int tca_conv_nhwc_x3(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* w,
                             const float* bias, int N, int KH, int KW, int S, int P, int Kp, float* out, int Ho,
                             int Wo, int ldo, int co_off, int act, const float* res, int ldr, int r_off, int shuffle,
                             int tile, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((Cin & 7) || (ldi & 7) || (ci_off & 7) || (N & 7) || (ldo & 7) || (co_off & 7) || (Kp & 31)) return (int)hipErrorInvalidValue;
  if (res && ((ldr & 7) || (r_off & 7))) return (int)hipErrorInvalidValue;
  ConvArgs a;
  a.in = nullptr; a.res = nullptr; a.out = nullptr;
  a.in_f = in; a.res_f = res; a.out_f = out; a.occ = nullptr;
  a.w = (const __hip_bfloat16*)w; a.bias = bias;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off;
  a.Ho = Ho; a.Wo = Wo; a.KH = KH; a.KW = KW; a.S = S; a.P = P;
  a.N = N; a.K = KH * KW * Cin; a.Kp = Kp; a.ldo = ldo; a.co_off = co_off; a.ldr = ldr; a.r_off = r_off;
  a.act = act; a.shuffle = shuffle; a.M = B * Ho * Wo;
  if (a.K > Kp) return (int)hipErrorInvalidValue;
  const bool v2ok = (Cin % 32) == 0 && Kp == a.K;
  // auto tile, measured on MI355X at batch 32 (tools/bench_conv_x3.py -> profiles/r2/conv_x3_tiles.jsonl):
  // small halo only at stride 1 (stride 2: v1 128x32 is 1.9x faster); N <= 32: v1 (a 1x1 64->32 runs 26 us
  // vs 38 on glds); glds 128x64 with one wave column for N <= 64, 128x128 4x2 above
  if (tile == 0 && small_halo_x3_ok(a) && a.S == 1) tile = 60;
  // glds-class layers go to the xb twins (same bits; profiles/r2/xbf_tiles.jsonl at batch 32: 128x64 8x1 for
  // N <= 64 and for small M (YOLOv5n b7 39 vs 54 us on the old glds 128x128), 128x128 4x2 above)
  // plain-fp32 hx twins (tiles 98-101) stay opt-in: auto-selected they measured +1.7% on CenterPoint,
  // +0% on SECOND-IoU and -2.5% on RetinaNet / FCOS (profiles/r2/fam_hx_fp32/)
  if (tile == 0 && N > 32 && v2ok && xb_ok(a)) tile = (N <= 64 || a.M < 40000) ? 81 : 80;
  if (tile == 0) tile = N <= 16 ? 6 : N <= 32 ? 1 : v2ok ? (N <= 64 ? 41 : 20) : (N <= 64 ? 2 : 5);
  if (((tile >= 10 && tile < 60) || tile >= 70) && !v2ok) return (int)hipErrorInvalidValue;
  if (tile >= 80 && !xb_ok(a)) return (int)hipErrorInvalidValue;
  switch (tile) {
    case 60: return launch_small_halo_x3(a, stream);
    case 98: return hx_ok(a) ? launch_hx<8, 128, 2, 4, true, false>(a, stream) : (int)hipErrorInvalidValue;
    case 99: return hx_ok(a) ? launch_hx<8, 128, 2, 4, false, false>(a, stream) : (int)hipErrorInvalidValue;
    case 100: return hx_ok(a) ? launch_hx<12, 64, 4, 2, true, false>(a, stream) : (int)hipErrorInvalidValue;
    case 101: return hx_ok(a) ? launch_hx<12, 64, 4, 2, false, false>(a, stream) : (int)hipErrorInvalidValue;
    // xb twins (buffer-descriptor DMA, split at the fragment read; same bits as the glds tile named)
    case 80: return launch_xb<128, 128, 4, 2, 2, false, false>(a, stream);  // 20
    case 81: return launch_xb<128, 64, 8, 1, 2, false, false>(a, stream);   // 41
    case 82: return launch_xb<128, 128, 2, 4, 2, false, false>(a, stream);  // 25
    case 83: return launch_xb<256, 64, 4, 2, 2, false, false>(a, stream);   // 26
    case 84: return launch_xb<128, 64, 4, 2, 2, false, false>(a, stream);   // 22
    case 85: return launch_xb<64, 128, 2, 4, 2, false, false>(a, stream);   // 24
    case 86: return launch_xb<256, 64, 8, 1, 2, false, false>(a, stream);   // 42
    case 87: return launch_xb<64, 64, 4, 1, 2, false, false>(a, stream);    // 47
    case 20: return launch_glds_x3<128, 128, 4, 2>(a, stream);
    case 22: return launch_glds_x3<128, 64, 4, 2>(a, stream);
    case 24: return launch_glds_x3<64, 128, 2, 4>(a, stream);
    case 25: return launch_glds_x3<128, 128, 2, 4>(a, stream);
    case 26: return launch_glds_x3<256, 64, 4, 2>(a, stream);
    case 27: return launch_glds_x3<128, 256, 2, 4>(a, stream);
    // one wave column (WN = 1): every A fragment is split once per K step per tile
    // (round 5: the 3 / 4-stage rings and the remaining untested shapes were removed: no auto rule or
    // test selected them)
    case 41: return launch_glds_x3<128, 64, 8, 1>(a, stream);
    case 42: return launch_glds_x3<256, 64, 8, 1>(a, stream);
    case 47: return launch_glds_x3<64, 64, 4, 1>(a, stream);
    case 1: return launch_x3<128, 32, 4, 1>(a, stream);
    case 2: return launch_x3<128, 64, 4, 1>(a, stream);
    case 5: return launch_x3<64, 128, 1, 4>(a, stream);
    case 6: return launch_x3<128, 16, 4, 1>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

// fp32 mode, pair activations: `in` (and `res`) hold pairs (see pair_split8),
// `out` pairs when out_pair, else fp32.  Same slice / residual / pixel-shuffle
// contract as tca_conv_nhwc_x3; the global_load_lds kernels only (Cin % 32 == 0,
// Kp == K).  tile: 0 auto, else one of 20, 22, 24, 25, 26, 32, 37, 41, 42 (glds), 68-79 (xb) or 90-97, 102 (hx).
namespace {
int conv_x3p(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* w,
                              const float* bias, int N, int KH, int KW, int S, int P, int Kp, float* out, int Ho,
                              int Wo, int ldo, int co_off, int act, const float* res, int ldr, int r_off, int shuffle,
                              int tile, int out_pair, const uint8_t* occ, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((Cin & 7) || (ldi & 7) || (ci_off & 7) || (N & 7) || (ldo & 7) || (co_off & 7) || (Kp & 31)) return (int)hipErrorInvalidValue;
  if (res && ((ldr & 7) || (r_off & 7) || !out_pair)) return (int)hipErrorInvalidValue;
  if (shuffle > 0 && ((N / (shuffle * shuffle)) & 7)) return (int)hipErrorInvalidValue;
  ConvArgs a;
  a.in = nullptr; a.res = nullptr; a.out = nullptr;
  a.in_f = in; a.res_f = res; a.out_f = out; a.occ = KH * KW <= 32 ? occ : nullptr;
  a.w = (const __hip_bfloat16*)w; a.bias = bias;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off;
  a.Ho = Ho; a.Wo = Wo; a.KH = KH; a.KW = KW; a.S = S; a.P = P;
  a.N = N; a.K = KH * KW * Cin; a.Kp = Kp; a.ldo = ldo; a.co_off = co_off; a.ldr = ldr; a.r_off = r_off;
  a.act = act; a.shuffle = shuffle; a.M = B * Ho * Wo;
  if (a.K > Kp || (Cin % 32) != 0 || Kp != a.K) return (int)hipErrorInvalidValue;
  // auto tile, measured on MI355X at batch 32 (tools/bench_conv_x3.py --pair ->
  // profiles/r2/conv_x3p_tiles.jsonl): N <= 64: 256x64 (4x2 waves), 3-stage 128x64 for
  // stride 2; wider: 128x128 2x4
  // (4-wave 64x64-per-wave tiles measured slower on every layer)
  // xb (buffer-descriptor DMA) twins, same bits, 8-10% faster on every PointPillars layer
  // (profiles/r2/xb_tiles.jsonl): 256x64 / 128x64 for N <= 64 (stride 1 / 2), 128x128 2x4 / 4x2
  // halo-tiled hx for 3x3 stride-1 layers with N >= 128: row-major 8x16 tiles (90) or column-major
  // 16x8 (94), whichever pads the image less, when that padding is <= 10% of the pixels
  // (pp.b2.conv 335 vs 353 us, pp.b3.conv 297 vs 312: profiles/r2/hx_tiles_v3.jsonl)
  // N = 64: 16 x 12 tiles (96 column-major / 97 row-major; pp.b1.conv 439 / 436 vs 455 us)
  if (tile == 0 && out_pair && !a.occ && xb_ok(a)) tile = hx_pick(a, 94, 90, 96, 97);
  if (tile == 0 && xb_ok(a)) tile = N <= 64 ? (S == 1 ? 71 : 77) : (S == 1 ? 70 : 73);
  if (tile == 0) tile = N <= 64 ? (S == 1 ? 26 : 32) : 25;
  return out_pair ? launch_glds_x3p<true>(a, tile, stream) : launch_glds_x3p<false>(a, tile, stream);
}
}  // namespace

TCA_API int tca_conv_nhwc_x3p(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* w,
                              const float* bias, int N, int KH, int KW, int S, int P, int Kp, float* out, int Ho,
                              int Wo, int ldo, int co_off, int act, const float* res, int ldr, int r_off, int shuffle,
                              int tile, int out_pair, hipStream_t stream) {
  return conv_x3p(in, B, H, W, Cin, ldi, ci_off, w, bias, N, KH, KW, S, P, Kp, out, Ho, Wo, ldo, co_off, act, res, ldr,
                  r_off, shuffle, tile, out_pair, nullptr, stream);
}

// Same with an input-pixel occupancy map occ (uint8 [B, H, W]; the pillar scatter's,
// tca_pillar_vfe_*_occ): the xb kernels read a pixel marked 0 as zeros without touching
// memory (the descriptor range check), which for a sparse BEV canvas (a few % of cells
// occupied) removes most of the first conv's input traffic.  Bit-identical to the plain
// call whenever the unmarked pixels hold zeros; the glds tiles ignore occ.
TCA_API int tca_conv_nhwc_x3p_occ(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off,
                                  const void* w, const float* bias, int N, int KH, int KW, int S, int P, int Kp,
                                  float* out, int Ho, int Wo, int ldo, int co_off, int act, const float* res, int ldr,
                                  int r_off, int shuffle, int tile, int out_pair, const uint8_t* occ,
                                  hipStream_t stream) {
  return conv_x3p(in, B, H, W, Cin, ldi, ci_off, w, bias, N, KH, KW, S, P, Kp, out, Ho, Wo, ldo, co_off, act, res, ldr,
                  r_off, shuffle, tile, out_pair, occ, stream);
}
