// YOLOv5 C3 blocks fused into LDS-resident kernels, fp32 mode (split-product MFMA), for the
// blocks with c_ = 16 / 32 / 64 hidden channels (YOLOv5n: b2, b4, b6, h13, h17, h20; the 20 x 20
// c_ = 128 blocks measured faster unfused: one workgroup of ~150 KiB LDS per CU over 320 tiles).  Reference block: C3 = cv3(cat(m(cv1(x)),
// cv2(x))) with m = n x Bottleneck(1x1, 3x3, + shortcut) (the YOLOv5 model the reference serves,
// examples/YOLOv5/config.pbtxt).
//
// Unfused (models/fast.py _C3Plan) a C3 is 4 + 2n launches; at batch 32 each is a 12-60 us
// kernel bound by its own latency and by moving the block's intermediates through HBM (an
// 80 x 80 block moves ~470 MB).  Here a workgroup owns a 16 x 4 pixel tile of the block's
// output: it reads x (or, between bottlenecks, a) once, keeps a / u / b in LDS, and writes y.
//
// Modes (n bottlenecks, each needing a one-pixel halo):
//   FULL  (n = 1)  x -> a (halo), b (tile) -> u = m.cv1(a) (halo) -> a' = m.cv2(u) (+ a) -> y = cv3([a'|b])
//   FIRST (n > 1)  x -> a, b -> u -> a'  ; writes a' and b to global (the block's a / cat buffers)
//   MID            a (global, halo) -> u -> a'  ; writes a'
//   LAST           a (global, halo), b (global) -> u -> a' -> y = cv3([a'|b])
//
// Every phase is a small GEMM blocked per wave as FM pixel tiles x FN 16-channel groups, so a
// weight fragment (streamed from L2 in MFMA fragment order, prefetched one K step ahead) feeds
// FM tiles and an activation fragment FN groups; the K loops are compile-time (cin = 2 c_ or
// 4 c_, cout = 2 c_: every C3 of the model), fully unrolled where short.
//
// LDS images are chunk-major pair planes, [C / 8][HPP][8] bf16 hi and lo, for a and u on the
// halo and b on the tile (HPP = the halo pixel count padded to 16), so every MFMA operand is
// read as stored (no split on the read path); the residual a of the tile pixels also stays in
// fp32.  An A fragment is 16 consecutive pixels (one output row of the tile, or 16
// consecutive halo pixels) x 8 channels; the lane quads fq = 0..3 read channel chunk fq,
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
  float* y;           // [B, H, W, ldy], channels [y_off, y_off + 2C)           (FULL / LAST)
  float* a_out;       // [B, H, W, ldao], channels [ao_off, ao_off + C)         (FIRST / MID)
  float* b_out;       // [B, H, W, ldbo], channels [bo_off, bo_off + C)         (FIRST)
  const __bf16 *w12, *wm1, *wm2, *w3;  // fragment-order split weights (ops/conv.py frag_weights)
  const float *b12, *bm1, *bm2, *b3;
  int act12, actm1, actm2, act3, add;
  int B, H, W;
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

__device__ __forceinline__ void split4(const float* v, uint2& h2, uint2& l2) {
  __bf16 h[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    h[r] = (__bf16)v[r];
    l[r] = (__bf16)(v[r] - (float)h[r]);
  }
  h2 = *reinterpret_cast<const uint2*>(h);
  l2 = *reinterpret_cast<const uint2*>(l);
}

// Weight fragments (ks, g0 .. g0 + FN - 1) of this lane from a fragment-order image
// [K / 32][NG][hi | lo][64 lanes][8] (one contiguous 1 KiB per fragment and half).
template <int FN>
__device__ __forceinline__ void wload(const __bf16* w, int ng, int ks, int g0, int lane, bf16x8 (&h)[FN],
                                      bf16x8 (&l)[FN]) {
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const __bf16* p = w + ((long)(ks * ng + g0 + j) * 2) * 512 + lane * 8;
    h[j] = *reinterpret_cast<const bf16x8*>(p);
    l[j] = *reinterpret_cast<const bf16x8*>(p + 512);
  }
}

// acc[i][j] += A(ks, i) . W(ks, g0 + j) over the K steps, the weights prefetched two steps ahead
// through a 3-deep register ring (unrolled by three: no dynamically indexed register arrays;
// an L2 hit outlives one step of FM x FN x 3 MFMAs).  mv: valid tiles.
template <int FM, int FN, int KS, class AF>
__device__ __forceinline__ void gemm(f32x4 (&acc)[FM][FN], const __bf16* w, int ng, int g0, int lane, int mv,
                                     AF&& afrag) {
  bf16x8 h0[FN], l0[FN], h1[FN], l1[FN], h2[FN], l2[FN];
  auto step = [&](int ks, const bf16x8 (&wh)[FN], const bf16x8 (&wl)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (i >= mv) break;
      bf16x8 xh, xl;
      afrag(ks, i, xh, xl);
#pragma unroll
      for (int j = 0; j < FN; ++j) mfma3(acc[i][j], wh[j], wl[j], xh, xl);
    }
  };
  auto clamp = [](int k) { return k < KS ? k : KS - 1; };
  wload<FN>(w, ng, 0, g0, lane, h0, l0);
  wload<FN>(w, ng, clamp(1), g0, lane, h1, l1);
  constexpr int UN = KS <= 9 ? 3 : 1;
#pragma unroll UN
  for (int ks = 0; ks < KS; ks += 3) {
    wload<FN>(w, ng, clamp(ks + 2), g0, lane, h2, l2);
    step(ks, h0, l0);
    if (ks + 1 < KS) {
      wload<FN>(w, ng, clamp(ks + 3), g0, lane, h0, l0);
      step(ks + 1, h1, l1);
    }
    if (ks + 2 < KS) {
      wload<FN>(w, ng, clamp(ks + 4), g0, lane, h1, l1);
      step(ks + 2, h2, l2);
    }
  }
}

template <int V> struct IC { static constexpr int value = V; };

template <int FM, int FN>
__device__ __forceinline__ void zero(f32x4 (&acc)[FM][FN]) {
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int C, int CINM, int MODE, bool RES>
__global__ void __launch_bounds__(256, 2) c3_fused_kernel(C3fArgs a) {
  constexpr int TH = 4, TW = 16, HW_ = TW + 2, HP = (TH + 2) * HW_, HPP = (HP + 15) / 16 * 16;
  constexpr int MTH = HPP / 16, MTI = TH;  // halo M tiles (7); tile M tiles (4: one tile row each)
  constexpr int CIN = CINM * C, COUT = 2 * C, NG = C / 16;
  constexpr bool HAS_B = MODE == kFull;
  constexpr int NI = TH * TW;
  // a on the halo as hi / lo planes (MFMA operands as stored), its tile pixels also in fp32 (the
  // residual); u on the halo; b on the tile (FULL).  a' (FULL / LAST) overwrites a's tile pixels.
  constexpr int P_BYTES = C * HPP * 2, R_BYTES = RES ? C * NI * 4 : 0, B_BYTES = HAS_B ? C * NI * 2 : 0;
  // x staging (P1) overlays the u planes, which come last: one 32-channel chunk needs 128 B per halo
  // pixel, the u planes hold 4 C (c_ = 16: extended)
  constexpr int U_REGION = 4 * C * HPP >= 128 * HPP ? 2 * P_BYTES : 128 * HPP;
  constexpr int U_OFF = 2 * P_BYTES + R_BYTES + 2 * B_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[U_OFF + U_REGION];
  __bf16* const ah = reinterpret_cast<__bf16*>(smem);                  // [C/8][HPP][8]
  __bf16* const al = reinterpret_cast<__bf16*>(smem + P_BYTES);
  float* const ar = reinterpret_cast<float*>(smem + 2 * P_BYTES);      // [C/4][NI][4]
  __bf16* const bh = reinterpret_cast<__bf16*>(smem + 2 * P_BYTES + R_BYTES);  // [C/8][NI][8]
  __bf16* const bl = reinterpret_cast<__bf16*>(smem + 2 * P_BYTES + R_BYTES + B_BYTES);
  __bf16* const uh = reinterpret_cast<__bf16*>(smem + U_OFF);          // [C/8][HPP][8]
  __bf16* const ul = reinterpret_cast<__bf16*>(smem + U_OFF + P_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int ntx = (a.W + TW - 1) / TW, nty = (a.H + TH - 1) / TH;
  const int bid = blockIdx.x;
  const int b = bid / (nty * ntx), rem = bid - b * (nty * ntx);
  const int y0 = (rem / ntx) * TH, x0 = (rem - (rem / ntx) * ntx) * TW;

  auto halo_in = [&](int p, long& pix) {  // halo pixel p inside the image? (and its pixel index)
    const int hy = p / HW_, hx = p - (p / HW_) * HW_;
    const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
    const bool in = p < HP && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    pix = in ? ((long)b * a.H + iy) * a.W + ix : 0;
    return in;
  };
  auto tile_in = [&](int mt, long& pix) {  // this lane's pixel of tile row mt
    const int iy = y0 + mt, ix = x0 + fr;
    const bool in = iy < a.H && ix < a.W;
    pix = in ? ((long)b * a.H + iy) * a.W + ix : 0;
    return in;
  };
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
  // A fragment from a pair image [C/8][npix][8] (pixel p, channels k0 .. k0 + 7)
  auto pfrag = [&](const __bf16* ph, const __bf16* pl, int npix, int p, int k0, bf16x8& h, bf16x8& l) {
    const int o = ((k0 >> 3) * npix + p) * 8;
    h = *reinterpret_cast<const bf16x8*>(ph + o);
    l = *reinterpret_cast<const bf16x8*>(pl + o);
  };
  // 4 channels n .. n + 3 of a at halo pixel p: the pair planes, and the fp32 residual on the tile
  auto put_a = [&](int p, int n, const float* v, bool residual) {
    uint2 h2, l2;
    split4(v, h2, l2);
    const int o = ((n >> 3) * HPP + p) * 8 + (n & 7);
    *reinterpret_cast<uint2*>(ah + o) = h2;
    *reinterpret_cast<uint2*>(al + o) = l2;
    if (RES && residual) {
      const int hy = p / HW_, hx = p - (p / HW_) * HW_;
      if (hy >= 1 && hy <= TH && hx >= 1 && hx <= TW)
        *reinterpret_cast<float4*>(ar + ((n >> 2) * NI + (hy - 1) * TW + hx - 1) * 4) = make_float4(v[0], v[1], v[2], v[3]);
    }
  };

  // ---- P1: a = act(cv1 x) on the halo, b = act(cv2 x) on the tile (FULL, FIRST);
  //      or a loaded from a_in on the halo (MID, LAST)
  if constexpr (MODE == kFull || MODE == kFirst) {
    // x streams through LDS one 32-channel chunk at a time, split into hi / lo planes once
    // ([4][HPP][8] bf16 each, in the u planes' space, free until P2), the next chunk's loads in
    // flight while this chunk's MFMAs run; every wave then reads its A fragments as stored.
    constexpr int KS = CIN / 32, XB = C >= 64 ? 2 : 1;  // staging buffers (one is 128 B per halo pixel)
    constexpr int XP = HPP * 8, XPL = (XP + 255) / 256;  // 16-B pieces per chunk, per thread
    __bf16* const xs = uh;  // buffer k: hi planes at xs + k * 2 * 4 * HPP * 8, lo planes after them
    float4 xr[XPL];
    int xo[XPL];
    long xg[XPL];
    // 16-B piece q -> (pixel p, float4 f4): 16 consecutive lanes take 8 pixels x both 8-B halves of
    // one hi / lo plane chunk, so each 16-lane ds_write_b64 group writes 128 contiguous bytes (the
    // pixel-major order wrote the four planes at one bank offset: 4-way); a wave still reads 8
    // whole 128-B pixel chunks from global
#pragma unroll
    for (int k = 0; k < XPL; ++k) {
      const int q = tid + k * 256;
      const int p = (q >> 6) * 8 + ((q >> 1) & 7), f4 = ((q >> 4) & 3) * 2 + (q & 1);
      long pix;
      const bool in = q < XP && halo_in(p, pix);
      xg[k] = in ? pix * a.ldx + a.x_off + f4 * 4 : -1;
      xo[k] = q < XP ? ((f4 >> 1) * HPP + p) * 8 + (f4 & 1) * 4 : -1;
    }
    auto xload = [&](int c) {
#pragma unroll
      for (int k = 0; k < XPL; ++k)
        xr[k] = xg[k] >= 0 ? *reinterpret_cast<const float4*>(a.x + xg[k] + c * 32) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto xstore = [&](int buf) {
      __bf16* hb = xs + buf * 2 * 4 * HPP * 8;
#pragma unroll
      for (int k = 0; k < XPL; ++k) {
        if (xo[k] < 0) continue;
        const float v[4] = {xr[k].x, xr[k].y, xr[k].z, xr[k].w};
        uint2 h2, l2;
        split4(v, h2, l2);
        *reinterpret_cast<uint2*>(hb + xo[k]) = h2;
        *reinterpret_cast<uint2*>(hb + 4 * HPP * 8 + xo[k]) = l2;
      }
    };
    // this wave's share: cv1 on FM halo tiles from m0 (a), or cv2 on the 4 tile rows (b), FN groups from g0
    auto run = [&](auto FMc, auto FNc, bool is_a, int m0, int g0) {
      constexpr int FM = decltype(FMc)::value, FN = decltype(FNc)::value;
      const int gw = (is_a ? 0 : NG) + g0;
      f32x4 acc[FM][FN];
      zero(acc);
      xload(0);
#pragma unroll
      for (int c = 0; c < KS; ++c) {
        const int buf = XB == 2 ? (c & 1) : 0;
        if (XB == 1 && c > 0) __syncthreads();  // every wave done with the previous chunk
        xstore(buf);
        if (c + 1 < KS) xload(c + 1);
        bf16x8 wh[FN], wl[FN];
        wload<FN>(a.w12, 2 * NG, c, gw, lane, wh, wl);
        __syncthreads();
        const __bf16* hb = xs + buf * 2 * 4 * HPP * 8;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int p = is_a ? (m0 + i) * 16 + fr : (m0 + i + 1) * HW_ + fr + 1;
          bf16x8 xh, xl;
          pfrag(hb, hb + 4 * HPP * 8, HPP, p, fq * 8, xh, xl);
#pragma unroll
          for (int j = 0; j < FN; ++j) mfma3(acc[i][j], wh[j], wl[j], xh, xl);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = (g0 + j) * 16 + fq * 4;  // a or b channel
        const float4 bv = a.b12 ? *reinterpret_cast<const float4*>(a.b12 + (is_a ? 0 : C) + c)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const float v[4] = {actf(acc[i][j][0] + bv.x, a.act12), actf(acc[i][j][1] + bv.y, a.act12),
                              actf(acc[i][j][2] + bv.z, a.act12), actf(acc[i][j][3] + bv.w, a.act12)};
          if (is_a) {
            const int p = (m0 + i) * 16 + fr;
            if (p < HPP) put_a(p, c, v, true);
          } else if constexpr (MODE == kFull) {
            uint2 h2, l2;
            split4(v, h2, l2);
            const int o = ((c >> 3) * NI + (m0 + i) * TW + fr) * 8 + (c & 7);
            *reinterpret_cast<uint2*>(bh + o) = h2;
            *reinterpret_cast<uint2*>(bl + o) = l2;
          } else {
            long pix;
            if (tile_in(m0 + i, pix))
              *reinterpret_cast<float4*>(a.b_out + pix * a.ldbo + a.bo_off + c) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    };
    if constexpr (NG == 1) {
      // c_ 16: 7 (a) + 4 (b) tiles: a tiles 0-3 / 4-6 on waves 0 / 1, b rows 0-1 / 2-3 on waves 2 / 3
      if (wid == 0) run(IC<4>{}, IC<1>{}, true, 0, 0);
      else if (wid == 1) run(IC<3>{}, IC<1>{}, true, 4, 0);
      else run(IC<2>{}, IC<1>{}, false, (wid - 2) * 2, 0);
    } else if constexpr (NG == 2) {
      // c_ 32: 7 x 2 (a) + 4 x 2 (b) tile-groups: a tiles 0-3 per group on waves 0, 1, a tiles 4-6 on
      // wave 3, b on wave 2
      if (wid < 2) run(IC<4>{}, IC<1>{}, true, 0, wid);
      else if (wid == 3) run(IC<3>{}, IC<2>{}, true, 4, 0);
      else run(IC<4>{}, IC<2>{}, false, 0, 0);
    } else {
      // waves 0, 1: a on all halo tiles, half the groups each; waves 2, 3: b, half each
      if (wid < 2) run(IC<MTH>{}, IC<NG / 2>{}, true, 0, (wid & 1) * (NG / 2));
      else run(IC<MTI>{}, IC<NG / 2>{}, false, 0, (wid & 1) * (NG / 2));
    }
  } else {
    // a from a_in on the halo (zeros outside the image: they only reach masked u); every load of
    // this thread issued before the first store
    constexpr int AP = HPP * (C / 4), APL = (AP + 255) / 256;
    // piece g -> (pixel p, 4-channel group c4): lane pairs take the two halves of one pixel's
    // 8-channel group, so 16 lanes write 128 contiguous LDS bytes (pixel-major: 2-way) and each
    // pair reads 32 contiguous global bytes
    auto piece = [&](int g, int& p, int& c4) {
      const int h = g >> 1;
      p = h % HPP;
      c4 = (h / HPP) * 2 + (g & 1);
    };
    float4 v[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      const int g = tid + k * 256;
      int p, c4;
      piece(g, p, c4);
      long pix;
      v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (g < AP && halo_in(p, pix)) v[k] = *reinterpret_cast<const float4*>(a.a_in + pix * a.lda + a.a_off + c4 * 4);
    }
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      const int g = tid + k * 256;
      int p, c4;
      piece(g, p, c4);
      const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      if (g < AP) put_a(p, c4 * 4, vv, true);
    }
  }
  __syncthreads();

  // ---- P2: u = act(m.cv1 a) on the halo, zero outside the image (the 3x3's padding)
  {
    // c_ 16: 4 tile blocks (2 + 2 + 2 + 1); 32: 2 blocks (4 + 3) x 2 groups; 64: 7 tiles x 1 group per wave
    constexpr int MB = NG >= 4 ? 1 : 4 / NG, WPB = 4 / MB, FM = (MTH + MB - 1) / MB, FN = NG >= 4 ? NG / 4 : 1;
    const int mb = wid / WPB, g0 = (wid % WPB) * FN;
    const int m0 = mb * FM, mv = MTH - m0 < FM ? MTH - m0 : FM;
    f32x4 acc[FM][FN];
    zero(acc);
    gemm<FM, FN, (C + 31) / 32>(acc, a.wm1, NG, g0, lane, mv, [&](int ks, int i, bf16x8& h, bf16x8& l) {
      const int k0 = ks * 32 + fq * 8;
      if (k0 < C) {
        pfrag(ah, al, HPP, (m0 + i) * 16 + fr, k0, h, l);
      } else {  // K padding (c_ 16): zero weights, zero operands
        h = bf16x8{};
        l = bf16x8{};
      }
    });
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = (g0 + j) * 16 + fq * 4;
      const float4 bv = a.bm1 ? *reinterpret_cast<const float4*>(a.bm1 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if (i >= mv) break;
        const int p = (m0 + i) * 16 + fr;
        long pix;
        const bool in = halo_in(p, pix);
        float v[4] = {actf(acc[i][j][0] + bv.x, a.actm1), actf(acc[i][j][1] + bv.y, a.actm1),
                      actf(acc[i][j][2] + bv.z, a.actm1), actf(acc[i][j][3] + bv.w, a.actm1)};
        if (!in) v[0] = v[1] = v[2] = v[3] = 0.f;
        uint2 h2, l2;
        split4(v, h2, l2);
        const int o = ((n >> 3) * HPP + p) * 8 + (n & 7);
        *reinterpret_cast<uint2*>(uh + o) = h2;
        *reinterpret_cast<uint2*>(ul + o) = l2;
      }
    }
  }
  __syncthreads();

  // LAST: this lane's b fragments of P4 (4 tile rows x C / 32 K steps x 8 channels), loaded now so
  // the global latency hides behind P3
  constexpr int KB = MODE == kLast ? (C + 31) / 32 : 1;
  float4 breg[MTI][KB][2];
  if constexpr (MODE == kLast) {
#pragma unroll
    for (int i = 0; i < MTI; ++i) {
      long pix;
      const bool in = tile_in(i, pix);
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const float* q = a.b_in + pix * a.ldb + a.b_off + k * 32 + fq * 8;
        breg[i][k][0] = in ? *reinterpret_cast<const float4*>(q) : make_float4(0.f, 0.f, 0.f, 0.f);
        breg[i][k][1] = in ? *reinterpret_cast<const float4*>(q + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }

  // ---- P3: a' = act(m.cv2 u) (+ a) on the tile: 3x3 over the u halo, K = 9 C in tap-major order
  {
    // c_ 16: one row per wave; 32: 2 row blocks x 2 groups; 64: 4 rows x 1 group per wave
    constexpr int MB = NG >= 4 ? 1 : 4 / NG, WPB = 4 / MB, FM = MTI / MB, FN = NG >= 4 ? NG / 4 : 1;
    const int mb = wid / WPB, g0 = (wid % WPB) * FN;
    const int m0 = mb * FM;
    f32x4 acc[FM][FN];
    zero(acc);
    gemm<FM, FN, (9 * C + 31) / 32>(acc, a.wm2, NG, g0, lane, FM, [&](int ks, int i, bf16x8& h, bf16x8& l) {
      const int k = ks * 32 + fq * 8, tap = k / C, ci = k - tap * C;  // tap-major K (c_ 16: two taps per step)
      if (tap < 9) {
        const int ky = tap / 3, kx = tap - (tap / 3) * 3;
        const int o = ((ci >> 3) * HPP + (m0 + i + ky) * HW_ + fr + kx) * 8;
        h = *reinterpret_cast<const bf16x8*>(uh + o);
        l = *reinterpret_cast<const bf16x8*>(ul + o);
      } else {  // K padding
        h = bf16x8{};
        l = bf16x8{};
      }
    });
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = (g0 + j) * 16 + fq * 4;
      const float4 bv = a.bm2 ? *reinterpret_cast<const float4*>(a.bm2 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int mt = m0 + i, p = (mt + 1) * HW_ + fr + 1;  // halo index of this lane's tile pixel
        float v[4] = {actf(acc[i][j][0] + bv.x, a.actm2), actf(acc[i][j][1] + bv.y, a.actm2),
                      actf(acc[i][j][2] + bv.z, a.actm2), actf(acc[i][j][3] + bv.w, a.actm2)};
        if constexpr (RES) {  // the shortcut (RES == add)
          const float4 r0 = *reinterpret_cast<const float4*>(ar + ((n >> 2) * NI + mt * TW + fr) * 4);
          v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
        }
        if constexpr (MODE == kFull || MODE == kLast) {
          put_a(p, n, v, false);  // a' over a's tile pixels (P2 is done with them)
        } else {
          long pix;
          if (tile_in(mt, pix))
            *reinterpret_cast<float4*>(a.a_out + pix * a.ldao + a.ao_off + n) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  }

  // ---- P4: y = act(cv3 [a' | b]) on the tile: 4 rows x cout / 4 channels per wave (c_ 16: one row x
  //      all 32 channels per wave)
  if constexpr (MODE == kFull || MODE == kLast) {
    __syncthreads();
    constexpr bool ROWS = COUT / 16 >= 4;
    constexpr int FN = ROWS ? COUT / 16 / 4 : COUT / 16, FM = ROWS ? MTI : 1;
    const int g0 = ROWS ? wid * FN : 0, m0 = ROWS ? 0 : wid;
    long pix[FM];
    bool in[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) in[i] = tile_in(m0 + i, pix[i]);
    f32x4 acc[FM][FN];
    zero(acc);
    gemm<FM, FN, 2 * C / 32>(acc, a.w3, COUT / 16, g0, lane, FM, [&](int ks, int i, bf16x8& h, bf16x8& l) {
      const int k = ks * 32 + fq * 8;  // [a' | b] channel (per lane: c_ 16 splits one step)
      if (k < C) {
        pfrag(ah, al, HPP, (m0 + i + 1) * HW_ + fr + 1, k, h, l);
      } else if constexpr (MODE == kFull) {
        pfrag(bh, bl, NI, (m0 + i) * TW + fr, k - C, h, l);
      } else {
        split8(breg[i][(k - C) >> 5][0], breg[i][(k - C) >> 5][1], h, l);
      }
    });
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = (g0 + j) * 16 + fq * 4;
      const float4 bv = a.b3 ? *reinterpret_cast<const float4*>(a.b3 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if (!in[i]) continue;
        *reinterpret_cast<float4*>(a.y + pix[i] * a.ldy + a.y_off + n) =
            make_float4(actf(acc[i][j][0] + bv.x, a.act3), actf(acc[i][j][1] + bv.y, a.act3),
                        actf(acc[i][j][2] + bv.z, a.act3), actf(acc[i][j][3] + bv.w, a.act3));
      }
    }
  }
}

template <int C, int CINM, int MODE, bool RES>
int launch_c3f(const C3fArgs& a, hipStream_t stream) {
  const long tiles = (long)a.B * ((a.H + 3) / 4) * ((a.W + 15) / 16);
  if (tiles >= (1L << 31)) return (int)hipErrorInvalidValue;
  c3_fused_kernel<C, CINM, MODE, RES><<<(unsigned)tiles, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

template <int C, int CINM>
int dispatch_mode(int mode, const C3fArgs& a, hipStream_t stream) {
  switch (mode) {  // a multi-bottleneck block's bottlenecks all have the shortcut (YOLOv5 backbone C3s)
    case kFull: return a.add ? launch_c3f<C, CINM, kFull, true>(a, stream) : launch_c3f<C, CINM, kFull, false>(a, stream);
    case kFirst: return a.add ? launch_c3f<C, CINM, kFirst, true>(a, stream) : (int)hipErrorInvalidValue;
    case kMid: return a.add ? launch_c3f<C, 2, kMid, true>(a, stream) : (int)hipErrorInvalidValue;  // (no x)
    case kLast: return a.add ? launch_c3f<C, 2, kLast, true>(a, stream) : (int)hipErrorInvalidValue;
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// One fused C3 pass (c3_fused_kernel).  ptrs: x, a_in, b_in, y, a_out, b_out, w12, b12, wm1, bm1,
// wm2, bm2, w3, b3 (unused ones null).  ints: mode, C, cin, cout, add, B, H, W, ldx, x_off, lda,
// a_off, ldb, b_off, ldy, y_off, ldao, ao_off, ldbo, bo_off, act12, actm1, actm2, act3.
// C in {16, 32, 64} (16: cin 2C), cin in {2C, 4C}, cout = 2C; FIRST / MID / LAST need the shortcut (add).  Weights: fragment-order split images of the
// FusedConvs' fp32 GEMM weights: cv1|cv2 merged [2C, cin], m.cv1 [C, C], m.cv2 [C, 9C] (tap-major
// K), cv3 [2C, 2C].  Biases fp32 (16-B aligned).
TCA_API int tca_c3_fused(const void* const* ptrs, const int* v, hipStream_t stream) {
  C3fArgs a;
  a.x = (const float*)ptrs[0]; a.a_in = (const float*)ptrs[1]; a.b_in = (const float*)ptrs[2];
  a.y = (float*)ptrs[3]; a.a_out = (float*)ptrs[4]; a.b_out = (float*)ptrs[5];
  a.w12 = (const __bf16*)ptrs[6]; a.b12 = (const float*)ptrs[7];
  a.wm1 = (const __bf16*)ptrs[8]; a.bm1 = (const float*)ptrs[9];
  a.wm2 = (const __bf16*)ptrs[10]; a.bm2 = (const float*)ptrs[11];
  a.w3 = (const __bf16*)ptrs[12]; a.b3 = (const float*)ptrs[13];
  const int mode = v[0], C = v[1], cin = v[2], cout = v[3];
  a.add = v[4]; a.B = v[5]; a.H = v[6]; a.W = v[7];
  a.ldx = v[8]; a.x_off = v[9]; a.lda = v[10]; a.a_off = v[11]; a.ldb = v[12]; a.b_off = v[13];
  a.ldy = v[14]; a.y_off = v[15]; a.ldao = v[16]; a.ao_off = v[17]; a.ldbo = v[18]; a.bo_off = v[19];
  a.act12 = v[20]; a.actm1 = v[21]; a.actm2 = v[22]; a.act3 = v[23];
  if (a.B <= 0) return 0;
  // the contract every mode relies on: 16-B aligned channel slices and biases
  const bool full_or_first = mode == kFull || mode == kFirst, uses_y = mode == kFull || mode == kLast;
  auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
  if ((full_or_first && (!a.x || (a.ldx & 3) || (a.x_off & 3) || a.ldx < a.x_off + cin)) ||
      (!full_or_first && (!a.a_in || (a.lda & 3) || (a.a_off & 3) || a.lda < a.a_off + C)) ||
      (mode == kLast && (!a.b_in || (a.ldb & 3) || (a.b_off & 3) || a.ldb < a.b_off + C)) ||
      (uses_y && (!a.y || !a.w3 || cout != 2 * C || (a.ldy & 3) || (a.y_off & 3) || a.ldy < a.y_off + cout)) ||
      (!uses_y && (!a.a_out || (a.ldao & 3) || (a.ao_off & 3) || a.ldao < a.ao_off + C)) ||
      (mode == kFirst && (!a.b_out || (a.ldbo & 3) || (a.bo_off & 3) || a.ldbo < a.bo_off + C)) ||
      (full_or_first && (!a.w12 || (cin != 2 * C && cin != 4 * C))) || !a.wm1 || !a.wm2 ||
      !al(a.b12) || !al(a.bm1) || !al(a.bm2) || !al(a.b3) || mode < 0 || mode > 3)
    return (int)hipErrorInvalidValue;
  const bool c4 = cin == 4 * C;
  switch (C) {
    case 16:  // (YOLOv5's c_ = 16 block has one bottleneck)
      if (c4 || mode != kFull) return (int)hipErrorInvalidValue;
      return a.add ? launch_c3f<16, 2, kFull, true>(a, stream) : launch_c3f<16, 2, kFull, false>(a, stream);
    case 32: return c4 ? dispatch_mode<32, 4>(mode, a, stream) : dispatch_mode<32, 2>(mode, a, stream);
    case 64: return c4 ? dispatch_mode<64, 4>(mode, a, stream) : dispatch_mode<64, 2>(mode, a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
