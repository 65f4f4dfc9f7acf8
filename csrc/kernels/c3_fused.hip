// YOLOv5 C3 blocks fused into LDS-resident kernels, fp32 mode (split-product MFMA), for the
// blocks with c_ = 32 / 64 / 128 hidden channels (YOLOv5n: b4, b6, b8 and the four head C3s;
// the c_ = 16 block b2 is image.hip yolo_c3s_fused).  Reference block: C3 = cv3(cat(m(cv1(x)),
// cv2(x))) with m = n x Bottleneck(1x1, 3x3, + shortcut) (the YOLOv5 model the reference serves,
// examples/YOLOv5/config.pbtxt).
//
// Unfused (models/fast.py _C3Plan) a C3 is 4 + 2n launches; at batch 32 each is a 12-60 us
// kernel bound by its own latency and by moving the block's intermediates through HBM (an
// 80 x 80 block moves ~470 MB).  Here a workgroup owns a 16 x TH pixel tile of the block's
// output: it reads x (or, between bottlenecks, a) once, keeps a / u / b in LDS, and writes y.
//
// Modes (n bottlenecks, each needing a one-pixel halo):
//   FULL  (n = 1)  x -> a (halo), b (tile) -> u = m.cv1(a) (halo) -> a' = m.cv2(u) (+ a) -> y = cv3([a'|b])
//   FIRST (n > 1)  x -> a, b -> u -> a'  ; writes a' and b to global (the block's a / cat buffers)
//   MID            a (global, halo) -> u -> a'  ; writes a'
//   LAST           a (global, halo), b (global) -> u -> a' -> y = cv3([a'|b])
//
// LDS images are chunk-major: [C / 4][HPP][4] fp32 for a, [C / 8][HPP][8] bf16 (hi and lo
// planes) for u and b, HPP = the halo pixel count padded to 16.  An MFMA A fragment is 16
// consecutive pixels (one output row of the tile, or 16 consecutive halo pixels) x 8
// channels; the lane quads fq = 0..3 read channel chunks 2 fq, 2 fq + 1 (fp32) or fq (bf16),
// whose planes lie HPP * 16 B = 0 mod 256 B apart, so every 16-lane ds_read_b128 group covers
// the 64 banks once (conflict-free for the halo rows and for every 3x3 tap shift).
//
// Numerics: every MFMA operand is the bf16 hi / lo split of the fp32 value the unfused chain
// stores between its kernels (x, a, u, a', b), the three split products are issued in the
// x3 kernels' order and the K steps in the same order, so y matches the unfused chain to
// fp32 rounding (tests/test_c3_fused_gpu.py).
#include "tca_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum : int { kFull = 0, kFirst = 1, kMid = 2, kLast = 3 };

struct C3fArgs {
  const float* x;     // [B, H, W, ldx], channels [x_off, x_off + cin)          (FULL / FIRST)
  const float* a_in;  // [B, H, W, lda], channels [a_off, a_off + C)            (MID / LAST)
  const float* b_in;  // [B, H, W, ldb], channels [b_off, b_off + C)            (LAST)
  float* y;           // [B, H, W, ldy], channels [y_off, y_off + cout)         (FULL / LAST)
  float* a_out;       // [B, H, W, ldao], channels [ao_off, ao_off + C)         (FIRST / MID)
  float* b_out;       // [B, H, W, ldbo], channels [bo_off, bo_off + C)         (FIRST)
  const __bf16 *w12, *wm1, *wm2, *w3;  // fragment-order split weights (ops/conv.py frag_weights)
  const float *b12, *bm1, *bm2, *b3;
  int act12, actm1, actm2, act3, add;
  int B, H, W, cin, cout;
  int ldx, x_off, lda, a_off, ldb, b_off, ldy, y_off, ldao, ao_off, ldbo, bo_off;
};

__device__ __forceinline__ float actf(float v, int act) {  // conv_mfma.hip act_fn (same expressions)
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return v / (1.f + __expf(-v));
    case 3: return v > 0.f ? v : 0.1f * v;
    default: return v;
  }
}

__device__ __forceinline__ void mfma3(f32x4& acc, const bf16x8& wh, const bf16x8& wl, const bf16x8& xh,
                                      const bf16x8& xl) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh, acc, 0, 0, 0);
}

__device__ __forceinline__ void split8(const float4& u, const float4& v, bf16x8& h, bf16x8& l) {
  const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = (__bf16)f[e];
    l[e] = (__bf16)(f[e] - (float)h[e]);
  }
}

// fragment-order weight image [K / 32][N / 16][hi | lo][64 lanes][8]: fragment (ks, g) of this lane
__device__ __forceinline__ void wfrag(const __bf16* w, int ng, int ks, int g, int lane, bf16x8& h, bf16x8& l) {
  const __bf16* p = w + ((long)(ks * ng + g) * 2) * 512 + lane * 8;
  h = *reinterpret_cast<const bf16x8*>(p);
  l = *reinterpret_cast<const bf16x8*>(p + 512);
}

template <int C, int MODE, int TH>
__global__ void __launch_bounds__(256, C == 128 ? 1 : 2) c3_fused_kernel(C3fArgs a) {
  constexpr int TW = 16, HW_ = TW + 2, HP = (TH + 2) * HW_, HPP = (HP + 15) / 16 * 16;
  constexpr int MTH = HPP / 16, MTI = TH;  // halo M tiles; interior M tiles (one tile row each)
  constexpr int NW = 4;
  constexpr bool HAS_B = MODE == kFull;
  constexpr int A_BYTES = C * HPP * 4, U_BYTES = C * HPP * 2, B_BYTES = HAS_B ? C * TH * TW * 2 : 0;
  __shared__ __attribute__((aligned(16))) unsigned char smem[A_BYTES + 2 * U_BYTES + 2 * B_BYTES];
  float* const af = reinterpret_cast<float*>(smem);                   // [C/4][HPP][4]
  __bf16* const uh = reinterpret_cast<__bf16*>(smem + A_BYTES);        // [C/8][HPP][8]
  __bf16* const ul = reinterpret_cast<__bf16*>(smem + A_BYTES + U_BYTES);
  __bf16* const bh = reinterpret_cast<__bf16*>(smem + A_BYTES + 2 * U_BYTES);  // [C/8][TH*TW][8]
  __bf16* const bl = reinterpret_cast<__bf16*>(smem + A_BYTES + 2 * U_BYTES + B_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int ntx = (a.W + TW - 1) / TW, nty = (a.H + TH - 1) / TH;
  const int bid = blockIdx.x;
  const int b = bid / (nty * ntx), rem = bid - b * (nty * ntx);
  const int y0 = (rem / ntx) * TH, x0 = (rem - (rem / ntx) * ntx) * TW;

  auto halo_in = [&](int p, int& iy, int& ix) {  // halo pixel p -> image pixel, inside?
    const int hy = p / HW_, hx = p - (p / HW_) * HW_;
    iy = y0 - 1 + hy;
    ix = x0 - 1 + hx;
    return p < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
  };
  auto gpix = [&](int iy, int ix) { return ((long)b * a.H + iy) * a.W + ix; };
  // A fragment from an fp32 NHWC global tensor (zero when the pixel is outside)
  auto gfrag = [&](const float* base, int ld, int off, bool in, long pix, int k0, bf16x8& h, bf16x8& l) {
    float4 u = make_float4(0.f, 0.f, 0.f, 0.f), v = u;
    if (in) {
      const float* q = base + pix * ld + off + k0;
      u = *reinterpret_cast<const float4*>(q);
      v = *reinterpret_cast<const float4*>(q + 4);
    }
    split8(u, v, h, l);
  };
  // A fragment from the fp32 a image (halo pixel p, channels k0 .. k0 + 7)
  auto afrag = [&](int p, int k0, bf16x8& h, bf16x8& l) {
    const float4 u = *reinterpret_cast<const float4*>(af + ((k0 >> 2) * HPP + p) * 4);
    const float4 v = *reinterpret_cast<const float4*>(af + (((k0 >> 2) + 1) * HPP + p) * 4);
    split8(u, v, h, l);
  };

  // ---- P1: a = act(cv1 x) on the halo; b = act(cv2 x) on the tile (FULL, FIRST)
  //      or a loaded from a_in on the halo (MID, LAST)
  if constexpr (MODE == kFull || MODE == kFirst) {
    const int ks_n = a.cin / 32, ng12 = 2 * C / 16;
    constexpr int FN = C / 16 >= 4 ? 4 : C / 16;  // 16-channel fragments per work item
    constexpr int NGB = C / 16 / FN;
    // a on the halo tiles, then b on the interior tiles
    for (int item = wid; item < (MTH + MTI) * NGB; item += NW) {
      const bool is_a = item < MTH * NGB;
      const int it = is_a ? item : item - MTH * NGB;
      const int mt = it / NGB, g0 = (it - (it / NGB) * NGB) * FN + (is_a ? 0 : C / 16);
      int p, iy, ix;
      bool in;
      if (is_a) {
        p = mt * 16 + fr;
        in = halo_in(p, iy, ix);
      } else {
        p = (mt + 1) * HW_ + fr + 1;
        iy = y0 + mt;
        ix = x0 + fr;
        in = iy < a.H && ix < a.W;
      }
      const long pix = in ? gpix(iy, ix) : 0;
      f32x4 acc[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int ks = 0; ks < ks_n; ++ks) {
        bf16x8 xh, xl;
        gfrag(a.x, a.ldx, a.x_off, in, pix, ks * 32 + fq * 8, xh, xl);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          bf16x8 wh, wl;
          wfrag(a.w12, ng12, ks, g0 + j, lane, wh, wl);
          mfma3(acc[j], wh, wl, xh, xl);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = (g0 + j) * 16 + fq * 4;  // merged cv1 | cv2 channel
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = actf(acc[j][r] + (a.b12 ? a.b12[n + r] : 0.f), a.act12);
        if (is_a) {
          if (p < HPP)
            *reinterpret_cast<float4*>(af + ((n >> 2) * HPP + p) * 4) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          const int c = n - C;  // b channel
          if constexpr (MODE == kFull) {
            const int q = mt * TW + fr;
            __bf16 h[4], l[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              h[r] = (__bf16)v[r];
              l[r] = (__bf16)(v[r] - (float)h[r]);
            }
            const int o = ((c >> 3) * (TH * TW) + q) * 8 + (c & 7);
            *reinterpret_cast<uint2*>(bh + o) = *reinterpret_cast<const uint2*>(h);
            *reinterpret_cast<uint2*>(bl + o) = *reinterpret_cast<const uint2*>(l);
          } else if (in) {
            *reinterpret_cast<float4*>(a.b_out + pix * a.ldbo + a.bo_off + c) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    }
  } else {
    // a from a_in on the halo (zeros outside the image: they only reach masked u)
    for (int g = tid; g < HPP * (C / 4); g += NW * 64) {
      const int p = g % HPP, c4 = g / HPP;
      int iy, ix;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (halo_in(p, iy, ix)) v = *reinterpret_cast<const float4*>(a.a_in + gpix(iy, ix) * a.lda + a.a_off + c4 * 4);
      *reinterpret_cast<float4*>(af + (c4 * HPP + p) * 4) = v;
    }
  }
  __syncthreads();

  // ---- P2: u = act(m.cv1 a) on the halo, zero outside the image (the 3x3's padding)
  {
    constexpr int FN = C / 16 >= 4 ? 4 : C / 16;
    constexpr int NGB = C / 16 / FN, KS = C / 32, NG = C / 16;
    for (int item = wid; item < MTH * NGB; item += NW) {
      const int mt = item / NGB, g0 = (item - (item / NGB) * NGB) * FN;
      const int p = mt * 16 + fr;
      int iy, ix;
      const bool in = halo_in(p, iy, ix);
      f32x4 acc[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 xh, xl;
        afrag(p, ks * 32 + fq * 8, xh, xl);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          bf16x8 wh, wl;
          wfrag(a.wm1, NG, ks, g0 + j, lane, wh, wl);
          mfma3(acc[j], wh, wl, xh, xl);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = (g0 + j) * 16 + fq * 4;
        __bf16 h[4], l[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = in ? actf(acc[j][r] + (a.bm1 ? a.bm1[n + r] : 0.f), a.actm1) : 0.f;
          h[r] = (__bf16)v;
          l[r] = (__bf16)(v - (float)h[r]);
        }
        const int o = ((n >> 3) * HPP + p) * 8 + (n & 7);
        *reinterpret_cast<uint2*>(uh + o) = *reinterpret_cast<const uint2*>(h);
        *reinterpret_cast<uint2*>(ul + o) = *reinterpret_cast<const uint2*>(l);
      }
    }
  }
  __syncthreads();

  // ---- P3: a' = act(m.cv2 u) (+ a) on the tile: 3x3 over the u halo, K = 9 C in tap-major order
  {
    constexpr int FN = C / 16 >= 2 ? 2 : 1;
    constexpr int NGB = C / 16 / FN, KS = 9 * C / 32, NG = C / 16;
    for (int item = wid; item < MTI * NGB; item += NW) {
      const int mt = item / NGB, g0 = (item - (item / NGB) * NGB) * FN;
      f32x4 acc[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
      for (int ks = 0; ks < KS; ++ks) {
        const int k0 = ks * 32, tap = k0 / C, ci = k0 - tap * C + fq * 8;
        const int ky = tap / 3, kx = tap - (tap / 3) * 3;
        const int p = (mt + ky) * HW_ + fr + kx;
        const int o = ((ci >> 3) * HPP + p) * 8;
        const bf16x8 xh = *reinterpret_cast<const bf16x8*>(uh + o);
        const bf16x8 xl = *reinterpret_cast<const bf16x8*>(ul + o);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          bf16x8 wh, wl;
          wfrag(a.wm2, NG, ks, g0 + j, lane, wh, wl);
          mfma3(acc[j], wh, wl, xh, xl);
        }
      }
      const int p = (mt + 1) * HW_ + fr + 1;  // halo index of this lane's tile pixel
      const int iy = y0 + mt, ix = x0 + fr;
      const bool in = iy < a.H && ix < a.W;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = (g0 + j) * 16 + fq * 4;
        float* ap = af + ((n >> 2) * HPP + p) * 4;
        const float4 r0 = *reinterpret_cast<const float4*>(ap);
        const float rv[4] = {r0.x, r0.y, r0.z, r0.w};
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = actf(acc[j][r] + (a.bm2 ? a.bm2[n + r] : 0.f), a.actm2);
          if (a.add) v[r] += rv[r];
        }
        if constexpr (MODE == kFull || MODE == kLast) {
          *reinterpret_cast<float4*>(ap) = make_float4(v[0], v[1], v[2], v[3]);  // a' over a (same lane)
        } else if (in) {
          *reinterpret_cast<float4*>(a.a_out + gpix(iy, ix) * a.ldao + a.ao_off + n) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  }

  // ---- P4: y = act(cv3 [a' | b]) on the tile
  if constexpr (MODE == kFull || MODE == kLast) {
    __syncthreads();
    const int ng3 = a.cout / 16;
    constexpr int FN = 4;
    const int ngb = ng3 / FN;  // cout % 64 == 0
    constexpr int KA = C / 32, KS = 2 * C / 32;
    for (int item = wid; item < MTI * ngb; item += NW) {
      const int mt = item / ngb, g0 = (item - (item / ngb) * ngb) * FN;
      const int p = (mt + 1) * HW_ + fr + 1;
      const int iy = y0 + mt, ix = x0 + fr;
      const bool in = iy < a.H && ix < a.W;
      const long pix = in ? gpix(iy, ix) : 0;
      f32x4 acc[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 xh, xl;
        if (ks < KA) {
          afrag(p, ks * 32 + fq * 8, xh, xl);
        } else if constexpr (MODE == kFull) {
          const int c = (ks - KA) * 32 + fq * 8, q = mt * TW + fr;
          const int o = ((c >> 3) * (TH * TW) + q) * 8;
          xh = *reinterpret_cast<const bf16x8*>(bh + o);
          xl = *reinterpret_cast<const bf16x8*>(bl + o);
        } else {
          gfrag(a.b_in, a.ldb, a.b_off, in, pix, (ks - KA) * 32 + fq * 8, xh, xl);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          bf16x8 wh, wl;
          wfrag(a.w3, ng3, ks, g0 + j, lane, wh, wl);
          mfma3(acc[j], wh, wl, xh, xl);
        }
      }
      if (!in) continue;
      float* o = a.y + pix * a.ldy + a.y_off;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = (g0 + j) * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = actf(acc[j][r] + (a.b3 ? a.b3[n + r] : 0.f), a.act3);
        *reinterpret_cast<float4*>(o + n) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

template <int C, int MODE>
int launch_c3f(const C3fArgs& a, hipStream_t stream) {
  constexpr int TH = 4;
  const long tiles = (long)a.B * ((a.H + TH - 1) / TH) * ((a.W + 15) / 16);
  if (tiles >= (1L << 31)) return (int)hipErrorInvalidValue;
  c3_fused_kernel<C, MODE, TH><<<(unsigned)tiles, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

template <int C>
int dispatch_mode(int mode, const C3fArgs& a, hipStream_t stream) {
  switch (mode) {
    case kFull: return launch_c3f<C, kFull>(a, stream);
    case kFirst: return launch_c3f<C, kFirst>(a, stream);
    case kMid: return launch_c3f<C, kMid>(a, stream);
    case kLast: return launch_c3f<C, kLast>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// One fused C3 pass (c3_fused_kernel).  ptrs: x, a_in, b_in, y, a_out, b_out, w12, b12, wm1, bm1,
// wm2, bm2, w3, b3 (unused ones null).  ints: mode, C, cin, cout, add, B, H, W, ldx, x_off, lda,
// a_off, ldb, b_off, ldy, y_off, ldao, ao_off, ldbo, bo_off, act12, actm1, actm2, act3.
// Weights: fragment-order split images of the FusedConvs' fp32 GEMM weights: cv1|cv2 merged
// [2C, cin], m.cv1 [C, C], m.cv2 [C, 9C] (tap-major K), cv3 [cout, 2C].
TCA_API int tca_c3_fused(const void* const* ptrs, const int* v, hipStream_t stream) {
  C3fArgs a;
  a.x = (const float*)ptrs[0]; a.a_in = (const float*)ptrs[1]; a.b_in = (const float*)ptrs[2];
  a.y = (float*)ptrs[3]; a.a_out = (float*)ptrs[4]; a.b_out = (float*)ptrs[5];
  a.w12 = (const __bf16*)ptrs[6]; a.b12 = (const float*)ptrs[7];
  a.wm1 = (const __bf16*)ptrs[8]; a.bm1 = (const float*)ptrs[9];
  a.wm2 = (const __bf16*)ptrs[10]; a.bm2 = (const float*)ptrs[11];
  a.w3 = (const __bf16*)ptrs[12]; a.b3 = (const float*)ptrs[13];
  const int mode = v[0], C = v[1];
  a.cin = v[2]; a.cout = v[3]; a.add = v[4]; a.B = v[5]; a.H = v[6]; a.W = v[7];
  a.ldx = v[8]; a.x_off = v[9]; a.lda = v[10]; a.a_off = v[11]; a.ldb = v[12]; a.b_off = v[13];
  a.ldy = v[14]; a.y_off = v[15]; a.ldao = v[16]; a.ao_off = v[17]; a.ldbo = v[18]; a.bo_off = v[19];
  a.act12 = v[20]; a.actm1 = v[21]; a.actm2 = v[22]; a.act3 = v[23];
  if (a.B <= 0) return 0;
  // the contract every mode relies on: 16-B aligned channel slices, K multiples of 32, cout of 64
  const bool full_or_first = mode == kFull || mode == kFirst, uses_y = mode == kFull || mode == kLast;
  if ((full_or_first && (!a.x || (a.cin & 31) || (a.ldx & 3) || (a.x_off & 3) || a.ldx < a.x_off + a.cin)) ||
      (!full_or_first && (!a.a_in || (a.lda & 3) || (a.a_off & 3) || a.lda < a.a_off + C)) ||
      (mode == kLast && (!a.b_in || (a.ldb & 3) || (a.b_off & 3) || a.ldb < a.b_off + C)) ||
      (uses_y && (!a.y || !a.w3 || (a.cout & 63) || (a.ldy & 3) || (a.y_off & 3) || a.ldy < a.y_off + a.cout)) ||
      (!uses_y && (!a.a_out || (a.ldao & 3) || (a.ao_off & 3) || a.ldao < a.ao_off + C)) ||
      (mode == kFirst && (!a.b_out || (a.ldbo & 3) || (a.bo_off & 3) || a.ldbo < a.bo_off + C)) ||
      (full_or_first && !a.w12) || !a.wm1 || !a.wm2)
    return (int)hipErrorInvalidValue;
  switch (C) {
    case 32: return dispatch_mode<32>(mode, a, stream);
    case 64: return dispatch_mode<64>(mode, a, stream);
    case 128: return dispatch_mode<128>(mode, a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
