// fp32-mode halo-tiled 3x3 stride-1 convolution with register-streamed weights
// ("hx3") for the PointPillars / CenterPoint BEV backbones
// (data/pointpillar.yaml:64-70 BaseBEVBackbone, run by
// examples/pointpillar_kitti/1/model.py:163): pair activations in and out,
// split-product MFMA (bf16 x3, fp32 accumulation; see conv_mfma.hip "fp32 mode").
#include "tca_common.h"

#include <cstdlib>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Hx3Args {
  const float* in_f;   // pair storage [B, H, W, ldi], channels [ci_off, ci_off + Cin)
  const float* res_f;  // pair residual [B, H, W, ldr] (channels [r_off, r_off + N)) or null
  float* out_f;        // pair output [B, H, W, ldo], channels [co_off, co_off + N)
  const void* w;       // fragment-order split weights (tca_conv_hx3p)
  const float* bias;   // [N] or null
  int B, H, W, Cin, ldi, ci_off, Ho, Wo;
  int N, ldo, co_off, ldr, r_off;
  int act;  // 0 none, 1 relu, 2 silu, 3 leaky(0.1); | 16: act after the residual add
  const unsigned char* occ;  // stride 2 only: uint8 [B, H, W] input occupancy (0: read as zeros) or null
  // stride 1 only, optional: uint8 [B, Ho, Wo] uniform depth (tca_bev_uniform_depth) and the pair
  // storage [N] of this layer's output on a uniform pixel.  A tile whose in-image pixels all have
  // depth >= uni_min is written from uni_val without running the K loop.
  const unsigned char* uni;
  const float* uni_val;
  int uni_min;
};

constexpr unsigned kOutOfRange = 0x80000000u;  // buffer offset past any num_records (< 2^31): reads zeros

__device__ __forceinline__ float act_fn(float v, int act) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return v / (1.f + __expf(-v));
    case 3: return v > 0.f ? v : 0.1f * v;
    default: return v;
  }
}

// slot swizzle of halo position hx (0..17), as conv_mfma.hip hx: conflict-free b128
// fragment reads at the three tap shifts
__device__ __forceinline__ int hswz(int hx) { return (0xb29108 >> (3 * (hx >> 1))) & 7; }

// x * w ~= xh*wh + xh*wl + xl*wh on the bf16 MFMA (fp32 accumulate), same order as conv_mfma.hip.
// (The kernels below issue these three products product-major over their accumulators.)
[[maybe_unused]] __device__ __forceinline__ void mfma3(f32x4& acc, const bf16x8& bh, const bf16x8& bl, const bf16x8& ah,
                                      const bf16x8& al) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc, 0, 0, 0);
}

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

// epilogue: bias + act from the accumulators into an fp32 LDS tile (tile row ml = line * 16 +
// position along the fragment axis), then 16-B pair stores (+ residual).  The tile rows are
// BN floats with the 16-B quads XOR-swizzled by the row (quad q of row ml at q ^ (ml & 15)):
// the accumulator writes (ds_write_b128, 8-lane groups = 8 rows, one quad column) and the
// row-major reads (ds_read_b128 of two quads per lane, 16-lane groups over two to four rows)
// are both bank-conflict free (checked for BN = 64 and 128 with the MI355X_MICROARCH.md
// lane groups).  (The former BN + 4 padding was conflict-free for the writes only: the reads went
// 2- to 4-way, ~1.7M extra LDS cycles per BEV conv dispatch, profiles/r3/pmc_lidar_r3.)
template <int TH, int BN, int WM, int WN, bool CM>
__device__ __forceinline__ void hx3_epilogue(const Hx3Args& a, unsigned char* smem,
                                             const f32x4 (&acc)[TH / WM][BN / WN / 16], int b, int oy0, int ox0,
                                             int n0) {
  constexpr int BM = TH * 16, NT = WM * WN * 64, FM = TH / WM, FN = BN / WN / 16, LD = BN;
  static_assert(BN % 64 == 0, "the quad swizzle needs >= 16 quads per row");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN, fr = lane & 15, fq = lane >> 4;
  float* st = reinterpret_cast<float*>(smem);
  auto quad = [](int ml, int q) { return ml * LD + ((q ^ (ml & 15)) << 2); };
  const int act = a.act & 15;
  const bool post_res = (a.act & 16) != 0 && a.res_f != nullptr;
  const int eact = post_res ? 0 : act;  // wave-uniform: one branch per fragment, not per element
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = (wn * FN + j) * 16 + fq * 4;
    const float4 bv = a.bias ? *reinterpret_cast<const float4*>(a.bias + n0 + nl) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = (wm * FM + i) * 16 + fr;
      float4 q = make_float4(acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w);
      if (eact == 1) {
        q.x = fmaxf(q.x, 0.f); q.y = fmaxf(q.y, 0.f); q.z = fmaxf(q.z, 0.f); q.w = fmaxf(q.w, 0.f);
      } else if (eact != 0) {
        q.x = act_fn(q.x, eact); q.y = act_fn(q.y, eact); q.z = act_fn(q.z, eact); q.w = act_fn(q.w, eact);
      }
      *reinterpret_cast<float4*>(st + quad(ml, nl >> 2)) = q;
    }
  }
  __syncthreads();
  constexpr int V8 = BN / 8;  // 8 channels (two quads) per lane and pass
  for (int id = tid; id < BM * V8; id += NT) {
    const int ml = id / V8, c8 = (id - (id / V8) * V8) * 8;
    const int oy = oy0 + (CM ? (ml & 15) : ml / 16), ox = ox0 + (CM ? ml / 16 : (ml & 15)), n = n0 + c8;
    if (oy >= a.Ho || ox >= a.Wo) continue;
    float v[8];
    const float4 v0 = *reinterpret_cast<const float4*>(st + quad(ml, c8 >> 2));
    const float4 v1 = *reinterpret_cast<const float4*>(st + quad(ml, (c8 >> 2) + 1));
    v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    const long pix = ((long)b * a.Ho + oy) * a.Wo + ox;
    if (a.res_f) {
      float r[8];
      pair_join8(a.res_f + pix * a.ldr + a.r_off + n, r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = post_res ? act_fn(v[e] + r[e], act) : v[e] + r[e];
    }
    const long o = pix * a.ldo + a.co_off + n;
    if (a.act & 32) {  // fp32 storage out (the input of an F(2,3) layer, conv_wino.hip)
      *reinterpret_cast<float4*>(a.out_f + o) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(a.out_f + o + 4) = make_float4(v[4], v[5], v[6], v[7]);
      continue;
    }
    uint4 hi, lo;
    pair_split8(v, hi, lo);
    *reinterpret_cast<uint4*>(a.out_f + o) = hi;
    *reinterpret_cast<uint4*>(a.out_f + o + 4) = lo;
  }
}

// Uniform-tile skipping (Hx3Args::uni): every output pixel of the BM-pixel tile (16-pixel
// fragment lines, CM as the kernels) has uniform depth >= uni_min, i.e. every input the dense K
// loop would read is the previous layer's constant (or, for the stride-2 conv on the sparse
// canvas, its window is empty): store uni_val (this layer's own output on such a pixel, in its
// output storage) and skip the K loop.  Workgroup-uniform result.
template <int BM, int BN, bool CM, int NT>
__device__ __forceinline__ bool uni_tile_store(const Hx3Args& a, int b, int oy0, int ox0, int n0) {
  const int tid = threadIdx.x;
  bool bad = false;
  for (int ml = tid; ml < BM; ml += NT) {
    const int oy = oy0 + (CM ? (ml & 15) : ml / 16), ox = ox0 + (CM ? ml / 16 : (ml & 15));
    if (oy < a.Ho && ox < a.Wo) bad |= a.uni[((long)b * a.Ho + oy) * a.Wo + ox] < a.uni_min;
  }
  if (__syncthreads_or(bad)) return false;
  constexpr int Q = BN / 4;  // 16-B pieces per pixel
  for (int id = tid; id < BM * Q; id += NT) {
    const int ml = id / Q, q = id - (id / Q) * Q;
    const int oy = oy0 + (CM ? (ml & 15) : ml / 16), ox = ox0 + (CM ? ml / 16 : (ml & 15));
    if (oy >= a.Ho || ox >= a.Wo) continue;
    const long o = (((long)b * a.Ho + oy) * a.Wo + ox) * a.ldo + a.co_off + n0 + q * 4;
    *reinterpret_cast<uint4*>(a.out_f + o) = *reinterpret_cast<const uint4*>(a.uni_val + n0 + q * 4);
  }
  return true;
}

// ---- x3 pair, halo-tiled 3x3 stride 1, v3 ("hx3"): weights streamed to registers.
//
// PMC of hx (profiles/r2/pmc_lidar_end/summary.md): waves 34% parked at the per-step
// `vmcnt(0)` + barrier that the shared LDS weight ring needs (a 2-deep ring: the
// weights of step s+1 must land inside step s), 24 MFMAs per wave between barriers.
// Here the LDS holds only the input halo; each wave owns its own output channels
// (WM = 1: no two waves of a workgroup need the same weight fragment) and loads
// its B fragments straight from HBM/L2 into a 3-deep register ring, two steps
// ahead, from a host-permuted weight image in MFMA fragment order
// ([K step][16-channel group][hi | lo][lane][8 bf16]: every fragment load is one
// contiguous 1 KiB).  No barrier inside a 32-channel chunk: the 9 tap steps of a
// chunk run barrier-free (one or two barriers per chunk, at the halo swap).  The
// next chunk's halo is fetched into registers at the start of a chunk by
// buffer loads (zero padding by the descriptor range check; every load counted
// by the compiler, no mixed DMA / register-load queues) and written to LDS at
// its end.  Per wave 128 pixels x 32 channels: 16 ds_read_b128 per 48 MFMAs.
// Same products and fp32 summation order per output as hx (chunk-major, tap
// inner), so the results are bit-identical to hx.
template <int V> struct IC { static constexpr int value = V; };

// PAIRS: two chunks per loop iteration (even chunk counts), the tap groups alternating
// between two static weight register sets: no register copy between groups
template <int TH, int BN, int WM, int WN, bool CM, int HB, int MINW = 2, bool PAIRS = false>
__global__ void __launch_bounds__(WM * WN * 64, MINW) conv_hx3_kernel(Hx3Args a) {
  constexpr int TW = 16, BM = TH * TW, NW = WM * WN, NT = NW * 64;
  constexpr int FM = TH / WM, FN = BN / WN / 16;
  static_assert(TH % WM == 0 && BN % (WN * 16) == 0 && FN >= 1, "tiles");
  static_assert(HB == 1 || HB == 2, "halo buffers");
  constexpr int HWD = TW + 2, HP = (TH + 2) * HWD;  // halo pixels (lines x positions)
  constexpr int HPIECES = HP * 8;                    // 16-B pieces of one 32-channel pair chunk
  constexpr int HPL = (HPIECES + NT - 1) / NT;       // halo loads per lane per chunk
  constexpr int HBYTES = HP * 128;
  constexpr int EPI = BM * (BN + 4) * 4;
  constexpr int LDS = (HB * HBYTES > EPI) ? HB * HBYTES : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  constexpr int EX = CM ? TH : TW, EY = CM ? TW : TH;
  const int tx_n = (a.Wo + EX - 1) / EX, ty_n = (a.Ho + EY - 1) / EY;
  const int nmt = a.B * ty_n * tx_n, nnt = a.N / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int b = mt / (ty_n * tx_n), rem = mt - b * (ty_n * tx_n);
  const int oy0 = (rem / tx_n) * EY, ox0 = (rem - (rem / tx_n) * tx_n) * EX;
  const int n0 = nt * BN;

  if (a.uni && uni_tile_store<TH * TW, BN, CM, NT>(a, b, oy0, ox0, n0)) return;

  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.in_f, (short)0, a.B * a.H * a.W * a.ldi * 4, 0x00020000);
  // halo pieces of this lane: global byte offset (chunk 0) and LDS byte offset (-1: none)
  unsigned h_off[HPL];
  int h_lds[HPL];
#pragma unroll
  for (int k = 0; k < HPL; ++k) {
    const int q = tid + k * NT, p = q >> 3, piece = q & 7;
    h_off[k] = kOutOfRange;
    h_lds[k] = -1;
    if (q < HPIECES) {
      const int u = p / HWD, v = p - (p / HWD) * HWD;
      const int hy = CM ? v : u, hx = CM ? u : v;
      const int iy = oy0 - 1 + hy, ix = ox0 - 1 + hx;
      if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
        h_off[k] = (unsigned)((((b * a.H + iy) * a.W + ix) * a.ldi + a.ci_off) * 4 + piece * 16);
      h_lds[k] = p * 128 + ((piece ^ hswz(v)) << 4);
    }
  }
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 hreg[HPL];
  auto halo_load = [&](int c) {
#pragma unroll
    for (int k = 0; k < HPL; ++k) hreg[k] = __builtin_amdgcn_raw_buffer_load_b128(rin, h_off[k], c * 128, 0);
  };
  auto halo_write = [&](int buf) {
    unsigned char* dst = smem + buf * HBYTES;
#pragma unroll
    for (int k = 0; k < HPL; ++k)
      if (k + 1 < HPL || h_lds[k] >= 0) *reinterpret_cast<u32x4*>(dst + h_lds[k]) = hreg[k];
  };

  // weights, fragment image: block (ks, g, h) = 64 lanes x 8 bf16
  const int NG = a.N / 16, g0 = (n0 + wn * FN * 16) / 16;
  const __bf16* wf = reinterpret_cast<const __bf16*>(a.w) + (long)g0 * 1024 + lane * 8;
  const int nc = a.Cin / 32;
  auto wload = [&](int ks, bf16x8 (&dst)[FN][2]) {  // ks: K step in the [tap][ci] weight K order
    const __bf16* p = wf + (long)ks * NG * 1024;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      dst[j][0] = *reinterpret_cast<const bf16x8*>(p + j * 1024);
      dst[j][1] = *reinterpret_cast<const bf16x8*>(p + j * 1024 + 512);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A tap group = the 3 taps that share one shift kf along the fragment axis: their
  // A fragments are the same halo lines offset by kl = 0..2, so the group reads
  // FM + 2 line fragments (not 3 * FM) and feeds each to up to 3 taps at once.
  // Its 3 taps' weights are live for the whole group; the next group's are
  // prefetched into the second register set when the group starts.
  const int G = 3 * nc;
  auto gload = [&](int gs, bf16x8 (&dst)[3][FN][2]) {  // group gs = chunk gs / 3, shift gs % 3
    const int c = gs / 3, kf = gs - (gs / 3) * 3;
#pragma unroll
    for (int kl = 0; kl < 3; ++kl) {
      const int t = CM ? 3 * kf + kl : 3 * kl + kf;  // tap index ky * 3 + kx
      wload(t * nc + c, dst[kl]);
    }
  };
  bf16x8 wc[3][FN][2], wx[3][FN][2];
  halo_load(0);
  gload(0, wc);
  halo_write(0);
  halo_load(nc > 1 ? 1 : 0);  // next chunk's halo rides in registers through chunk 0
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int fr = lane & 15, fq = lane >> 4;
  // one tap group: prefetch the weights of group gs_next into wl, then 3 * FM * FN fragment
  // pairs from the FM + 2 halo lines at shift kf with the weights in wu
  auto group = [&](auto KF, const unsigned char* hb, bf16x8 (&wu)[3][FN][2], bf16x8 (&wl)[3][FN][2], int gs_next) {
    constexpr int kf = decltype(KF)::value;
    gload(gs_next < G ? gs_next : G - 1, wl);  // unconditional (clamped): no branch around the loads
    // keep the prefetch at the top of the group: hipcc's scheduler otherwise sinks the
    // loads to their first use and waits for them there
    __builtin_amdgcn_sched_barrier(0);
    const int sw = hswz(kf + fr);
    const unsigned char* colp = hb + (wm * FM) * HWD * 128 + (kf + fr) * 128;
    const int o_hi = ((2 * fq) ^ sw) << 4, o_lo = ((2 * fq + 1) ^ sw) << 4;
#pragma unroll
    for (int L = 0; L < FM + 2; ++L) {
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(colp + L * HWD * 128 + o_hi);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(colp + L * HWD * 128 + o_lo);
      // the three split products, product-major: the MFMAs of one product over every
      // (tap, channel group) accumulator of this line are independent, so a dependent
      // accumulator chain never issues back to back; each accumulator still sums its
      // products in mfma3's order (bit-identical results)
#pragma unroll
      for (int pr = 0; pr < 3; ++pr) {
#pragma unroll
        for (int kl = 0; kl < 3; ++kl) {
          const int i = L - kl;
          if (i < 0 || i >= FM) continue;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const bf16x8& b = pr == 0 ? wu[kl][j][1] : wu[kl][j][0];
            const bf16x8& x = pr == 1 ? al : ah;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, x, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
  };
  auto chunk_end = [&](int c) {
    if (c + 1 < nc) {
      if constexpr (HB == 1) {  // every wave done with this chunk's halo before it is overwritten
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      halo_write(HB == 2 ? (c + 1) & 1 : 0);
      halo_load(c + 2 < nc ? c + 2 : nc - 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };
  if constexpr (PAIRS) {
    const unsigned char* hb1 = smem + (HB == 2 ? HBYTES : 0);
    for (int c = 0; c < nc; c += 2) {
      group(IC<0>{}, smem, wc, wx, 3 * c + 1);
      group(IC<1>{}, smem, wx, wc, 3 * c + 2);
      group(IC<2>{}, smem, wc, wx, 3 * c + 3);
      chunk_end(c);
      group(IC<0>{}, hb1, wx, wc, 3 * c + 4);
      group(IC<1>{}, hb1, wc, wx, 3 * c + 5);
      group(IC<2>{}, hb1, wx, wc, 3 * c + 6);
      chunk_end(c + 1);
    }
  } else {
    for (int c = 0; c < nc; ++c) {
      const unsigned char* hb = smem + (HB == 2 ? (c & 1) * HBYTES : 0);
      auto copyw = [&]() {  // the prefetched set becomes the current one
#pragma unroll
        for (int kl = 0; kl < 3; ++kl)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            wc[kl][j][0] = wx[kl][j][0];
            wc[kl][j][1] = wx[kl][j][1];
          }
      };
      group(IC<0>{}, hb, wc, wx, 3 * c + 1);
      copyw();
      group(IC<1>{}, hb, wc, wx, 3 * c + 2);
      copyw();
      group(IC<2>{}, hb, wc, wx, 3 * c + 3);
      copyw();
      chunk_end(c);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the epilogue reuses the halo LDS
  asm volatile("" ::: "memory");

  hx3_epilogue<TH, BN, WM, WN, CM>(a, smem, acc, b, oy0, ox0, n0);
}

// ---- stride 2 ("hx3s2"): the 3x3 stride-2 pad-1 conv as four phase sub-convolutions.
//
// Output pixel o reads input 2o - 1 + k along each axis: k = 0 -> 2(o - 1) + 1, k = 1 -> 2o,
// k = 2 -> 2o + 1.  On the space-to-depth view of the input (S2D pixel P, phase p: input
// 2P + p), phase 0 carries tap 1 at P = o and phase 1 carries taps 0 (P = o - 1) and 2
// (P = o).  So each of the four (line, fragment-axis) phases is a stride-1 conv with one or
// two taps per axis over a (TH + 1) x 17 halo of S2D pixels, staged exactly like hx3's
// (stride-2 gathers from global, stride-1 fragment reads from LDS, the same hswz swizzle):
// 9 taps per 32-channel chunk in 6 groups (taps sharing the fragment-axis shift), 4 halo
// swaps per chunk.  Per chunk a wave reads 6 FM + 3 line fragments for 9 FM x FN fragment
// pairs (hx3: 3 FM + 6); the weight stream per MFMA is hx3's.  OCC: the halo loader reads an
// input pixel whose occupancy byte is 0 as zeros without fetching it (the sparse pillar canvas).
// Group g of a chunk: line parity PL = g >= 3, fragment parity PF and fragment tap FI.
template <int G> struct S2Group {
  static constexpr int PL = G >= 3 ? 1 : 0;
  static constexpr int PF = (G == 0 || G == 3) ? 0 : 1;
  static constexpr int FI = (G == 2 || G == 5) ? 1 : 0;
  static constexpr int KF = PF == 0 ? 1 : 2 * FI;     // fragment-axis tap (original index)
  static constexpr int FOFF = PF == 0 ? 1 : FI;        // its halo shift
  static constexpr int NL = PL == 0 ? 1 : 2;           // line taps
  static constexpr int PH = PL * 2 + PF;               // phase (halo buffer) of the group
  static constexpr bool LAST_OF_PHASE = G == 0 || G == 2 || G == 3 || G == 5;
  __device__ static constexpr int kl(int li) { return PL == 0 ? 1 : 2 * li; }   // line tap (original index)
  __device__ static constexpr int loff(int li) { return PL == 0 ? 1 : li; }     // its halo line shift
};

template <int TH, int BN, int WN, bool CM, int MINW, bool OCC>
__global__ void __launch_bounds__(WN * 64, MINW) conv_hx3s2_kernel(Hx3Args a) {
  constexpr int TW = 16, NT = WN * 64;
  constexpr int FM = TH, FN = BN / WN / 16;
  static_assert(BN % (WN * 16) == 0 && FN >= 1, "tiles");
  constexpr int HWD = TW + 1, HP = (TH + 1) * HWD;  // S2D halo pixels of one phase
  constexpr int HPIECES = HP * 8;
  constexpr int HPL = (HPIECES + NT - 1) / NT;
  constexpr int HBYTES = HP * 128;
  constexpr int EPI = TH * TW * (BN + 4) * 4;
  constexpr int LDS = (2 * HBYTES > EPI) ? 2 * HBYTES : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wn = tid >> 6;
  constexpr int EX = CM ? TH : TW, EY = CM ? TW : TH;
  const int tx_n = (a.Wo + EX - 1) / EX, ty_n = (a.Ho + EY - 1) / EY;
  const int nmt = a.B * ty_n * tx_n, nnt = a.N / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int b = mt / (ty_n * tx_n), rem = mt - b * (ty_n * tx_n);
  const int oy0 = (rem / tx_n) * EY, ox0 = (rem - (rem / tx_n) * tx_n) * EX;
  const int n0 = nt * BN;
  if (a.uni && uni_tile_store<TH * TW, BN, CM, NT>(a, b, oy0, ox0, n0)) return;

  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.in_f, (short)0, a.B * a.H * a.W * a.ldi * 4, 0x00020000);
  // phase byte offsets: line parity, fragment-axis parity
  const int pix_b = a.ldi * 4, row_b = a.W * a.ldi * 4;
  const int dl = CM ? pix_b : row_b, df = CM ? row_b : pix_b;
  // halo pieces of this lane: byte offset of the phase-(0, 0) input pixel, LDS offset, and the
  // phases (bit PL * 2 + PF) whose pixel is inside the image (and occupied)
  unsigned h_off[HPL];
  int h_lds[HPL];
  unsigned h_ph[HPL];
#pragma unroll
  for (int k = 0; k < HPL; ++k) {
    const int q = tid + k * NT, p = q >> 3, piece = q & 7;
    h_off[k] = kOutOfRange;
    h_lds[k] = -1;
    h_ph[k] = 0;
    if (q < HPIECES) {
      const int u = p / HWD, v = p - (p / HWD) * HWD;
      const int hy = CM ? v : u, hx = CM ? u : v;
      const int Y = oy0 - 1 + hy, X = ox0 - 1 + hx;
      if (Y >= 0 && X >= 0 && 2 * Y < a.H && 2 * X < a.W) {
        h_off[k] = (unsigned)((((b * a.H + 2 * Y) * a.W + 2 * X) * a.ldi + a.ci_off) * 4 + piece * 16);
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
          const int pl = ph >> 1, pf = ph & 1;
          const int iy = 2 * Y + (CM ? pf : pl), ix = 2 * X + (CM ? pl : pf);
          bool ok = iy < a.H && ix < a.W;
          if constexpr (OCC) ok = ok && a.occ[((long)b * a.H + iy) * a.W + ix] != 0;
          h_ph[k] |= ok ? (1u << ph) : 0u;
        }
      }
      h_lds[k] = p * 128 + ((piece ^ hswz(v)) << 4);
    }
  }
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  // two register sets: phase-chunk q's halo lives in hreg[q & 1] (= its phase's parity, a compile-time
  // index below), loaded three phases ahead so each load has two phases of MFMAs to land in
  u32x4 hreg[2][HPL];
  auto halo_load = [&](int ph, int c, auto SL) {  // ph: runtime-uniform phase
    constexpr int sl = decltype(SL)::value;
    const int so = c * 128 + (ph >> 1) * dl + (ph & 1) * df;
#pragma unroll
    for (int k = 0; k < HPL; ++k)
      hreg[sl][k] = __builtin_amdgcn_raw_buffer_load_b128(rin, ((h_ph[k] >> ph) & 1u) ? h_off[k] : kOutOfRange, so, 0);
  };
  auto halo_write = [&](int buf, auto SL) {
    constexpr int sl = decltype(SL)::value;
    unsigned char* dst = smem + buf * HBYTES;
#pragma unroll
    for (int k = 0; k < HPL; ++k)
      if (k + 1 < HPL || h_lds[k] >= 0) *reinterpret_cast<u32x4*>(dst + h_lds[k]) = hreg[sl][k];
  };

  const int NG = a.N / 16, g0 = (n0 + wn * FN * 16) / 16;
  const __bf16* wf = reinterpret_cast<const __bf16*>(a.w) + (long)g0 * 1024 + lane * 8;
  const int nc = a.Cin / 32;
  auto wload = [&](int ks, bf16x8 (&dst)[FN][2]) {
    const __bf16* p = wf + (long)ks * NG * 1024;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      dst[j][0] = *reinterpret_cast<const bf16x8*>(p + j * 1024);
      dst[j][1] = *reinterpret_cast<const bf16x8*>(p + j * 1024 + 512);
    }
  };
  // weights of group G of chunk c (c clamped by the caller)
  auto gload = [&](auto GC, int c, bf16x8 (&dst)[2][FN][2]) {
    using S = S2Group<decltype(GC)::value>;
#pragma unroll
    for (int li = 0; li < S::NL; ++li) {
      const int t = CM ? 3 * S::KF + S::kl(li) : 3 * S::kl(li) + S::KF;
      wload(t * nc + c, dst[li]);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (OCC) {
    // a tile whose whole input halo is unoccupied (the sparse pillar canvas far from the sensor)
    // reads only zeros: its accumulators are exactly 0, so skip the K loop (bias / act / residual
    // epilogue only) -- bit-identical to running it
    unsigned mine = 0;
#pragma unroll
    for (int k = 0; k < HPL; ++k) mine |= h_ph[k];
    if (!__syncthreads_or(mine != 0u)) {
      hx3_epilogue<TH, BN, 1, WN, CM>(a, smem, acc, b, oy0, ox0, n0);
      return;
    }
  }
  bf16x8 w0[2][FN][2], w1[2][FN][2];
  halo_load(0, 0, IC<0>{});
  gload(IC<0>{}, 0, w0);
  halo_write(0, IC<0>{});
  halo_load(1, 0, IC<1>{});                                    // q = 1
  halo_load(4 * nc > 2 ? 2 : 4 * nc - 1, 0, IC<0>{});          // q = 2 (nc >= 1: 4 phases per chunk)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int fr = lane & 15, fq = lane >> 4;
  // phase-chunk q = 4 c + ph lives in halo buffer q & 1 = ph & 1 and, before that, in register set ph & 1
  auto phase_end = [&](auto PH, int c) {
    constexpr int ph = decltype(PH)::value;
    const int q = 4 * c + ph;
    if (q + 1 < 4 * nc) {
      halo_write((ph + 1) & 1, IC<(ph + 1) & 1>{});
      const int q3 = q + 3 < 4 * nc ? q + 3 : 4 * nc - 1;
      halo_load(q3 & 3, q3 >> 2, IC<(ph + 1) & 1>{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };
  auto group = [&](auto GC, int c, bf16x8 (&wu)[2][FN][2], bf16x8 (&wl)[2][FN][2]) {
    constexpr int G = decltype(GC)::value;
    using S = S2Group<G>;
    // prefetch the next group's weights (group 0 of chunk c + 1 after group 5, clamped)
    if constexpr (G < 5) gload(IC<G + 1>{}, c, wl);
    else gload(IC<0>{}, c + 1 < nc ? c + 1 : nc - 1, wl);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned char* hb = smem + (S::PH & 1) * HBYTES;
    const int sw = hswz(S::FOFF + fr);
    const unsigned char* colp = hb + (S::FOFF + fr) * 128;
    const int o_hi = ((2 * fq) ^ sw) << 4, o_lo = ((2 * fq + 1) ^ sw) << 4;
#pragma unroll
    for (int L = (S::NL == 1 ? 1 : 0); L < FM + 1; ++L) {
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(colp + L * HWD * 128 + o_hi);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(colp + L * HWD * 128 + o_lo);
#pragma unroll
      for (int pr = 0; pr < 3; ++pr) {  // product-major, as the stride-1 kernel (same per-accumulator order)
#pragma unroll
        for (int li = 0; li < S::NL; ++li) {
          const int i = L - S::loff(li);
          if (i < 0 || i >= FM) continue;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const bf16x8& b = pr == 0 ? wu[li][j][1] : wu[li][j][0];
            const bf16x8& x = pr == 1 ? al : ah;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, x, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    if constexpr (S::LAST_OF_PHASE) phase_end(IC<S::PH>{}, c);
  };
  for (int c = 0; c < nc; ++c) {
    group(IC<0>{}, c, w0, w1);
    group(IC<1>{}, c, w1, w0);
    group(IC<2>{}, c, w0, w1);
    group(IC<3>{}, c, w1, w0);
    group(IC<4>{}, c, w0, w1);
    group(IC<5>{}, c, w1, w0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the epilogue reuses the halo LDS
  asm volatile("" ::: "memory");
  hx3_epilogue<TH, BN, 1, WN, CM>(a, smem, acc, b, oy0, ox0, n0);
}


template <int TH, int BN, int WM, int WN, bool CM, int HB, int MINW = 2>
int launch_hx3(const Hx3Args& a, hipStream_t stream) {
  if (a.N % BN) return (int)hipErrorInvalidValue;
  const int ex = CM ? TH : 16, ey = CM ? 16 : TH;
  const int nwg = a.B * ((a.Ho + ey - 1) / ey) * ((a.Wo + ex - 1) / ex) * (a.N / BN);
  if ((a.Cin / 32) % 2 == 0)
    conv_hx3_kernel<TH, BN, WM, WN, CM, HB, MINW, true><<<nwg, WM * WN * 64, 0, stream>>>(a);
  else
    conv_hx3_kernel<TH, BN, WM, WN, CM, HB, MINW, false><<<nwg, WM * WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// hx3 tiles.  0 = auto: N % 128 == 0 -> 8 x 16 tiles, 4 waves of 128 pixels x 32 channels
// (row- or column-major by the smaller padding); N == 64 -> 8 x 16 tiles, 4 waves of 128
// pixels x 16 channels (3 workgroups per CU).  Every variant: 2 waves per SIMD (<= 256 VGPRs, no spill), two
// workgroups per CU (<= 80 KiB LDS).  (16-line N = 64 tiles measured on par: 361-371 vs 365 us for
// pp.b1.conv at batch 32, profiles/r4/hx3_16line_tiles_removed.jsonl.)
int hx3_launch(const Hx3Args& a, int tile, hipStream_t stream) {
  if (tile == 0) {
    const long rm8 = (long)((a.Wo + 15) / 16 * 16) * ((a.Ho + 7) / 8 * 8);
    const long cm8 = (long)((a.Ho + 15) / 16 * 16) * ((a.Wo + 7) / 8 * 8);
    // measured at batch 32 (profiles/r3/hx3_tiles2.jsonl): pp.b1.conv (N 64) 362 us on tile 6 vs 427 on
    // tile 4 (2 x 2 waves load every weight fragment twice per workgroup); pp.b2 / b3 283 / 257 us on tile 1 / 2
    if (a.N % 128 == 0) tile = cm8 < rm8 ? 2 : 1;
    else if (a.N % 64 == 0) tile = cm8 < rm8 ? 6 : 5;
    else return (int)hipErrorInvalidValue;
  }
  switch (tile) {
    case 1: return launch_hx3<8, 128, 1, 4, false, 2>(a, stream);
    case 2: return launch_hx3<8, 128, 1, 4, true, 2>(a, stream);
    case 3: return launch_hx3<8, 64, 2, 2, false, 2>(a, stream);
    case 4: return launch_hx3<8, 64, 2, 2, true, 2>(a, stream);
    // one wave row, 16 channels per wave: no weight fragment loaded twice per workgroup,
    // <= 168 VGPRs -> 3 workgroups (12 waves) per CU
    case 5: return launch_hx3<8, 64, 1, 4, false, 2, 3>(a, stream);
    case 6: return launch_hx3<8, 64, 1, 4, true, 2, 3>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}


template <int TH, int BN, int WN, bool CM, int MINW>
int launch_hx3s2(const Hx3Args& a, hipStream_t stream) {
  if (a.N % BN) return (int)hipErrorInvalidValue;
  const int ex = CM ? TH : 16, ey = CM ? 16 : TH;
  const int nwg = a.B * ((a.Ho + ey - 1) / ey) * ((a.Wo + ex - 1) / ex) * (a.N / BN);
  if (a.occ) conv_hx3s2_kernel<TH, BN, WN, CM, MINW, true><<<nwg, WN * 64, 0, stream>>>(a);
  else conv_hx3s2_kernel<TH, BN, WN, CM, MINW, false><<<nwg, WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// stride-2 tiles.  0 = auto: 8 x 16 output tiles (row- or column-major by the smaller padding),
// 4 waves of 128 pixels x 32 (N % 128 == 0) or 16 (N == 64) channels
int hx3s2_launch(const Hx3Args& a, int tile, hipStream_t stream) {
  if (tile == 0) {
    const long rm8 = (long)((a.Wo + 15) / 16 * 16) * ((a.Ho + 7) / 8 * 8);
    const long cm8 = (long)((a.Ho + 15) / 16 * 16) * ((a.Wo + 7) / 8 * 8);
    if (a.N % 128 == 0) tile = cm8 < rm8 ? 2 : 1;
    else if (a.N % 64 == 0) tile = cm8 < rm8 ? 4 : 3;
    else return (int)hipErrorInvalidValue;
  }
  switch (tile) {
    case 1: return launch_hx3s2<8, 128, 4, false, 2>(a, stream);
    case 2: return launch_hx3s2<8, 128, 4, true, 2>(a, stream);
    case 3: return launch_hx3s2<8, 64, 4, false, 3>(a, stream);
    case 4: return launch_hx3s2<8, 64, 4, true, 3>(a, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// fp32 mode, pair activations in and out, 3x3 stride 1 pad 1 (conv_hx3_kernel).
// wfrag: the split weights permuted to MFMA fragment order (ops/conv.py frag_weights):
// [9 * Cin / 32][N / 16][hi | lo][64 lanes][8 bf16]; N % 64 == 0, Cin % 32 == 0.
// Residual (pairs) and act as tca_conv_nhwc_x3p.  tile: 0 auto, 1-4 (hx3_launch).
TCA_API int tca_conv_hx3p(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* wfrag,
                          const float* bias, int N, float* out, int ldo, int co_off, int act, const float* res,
                          int ldr, int r_off, int tile, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((Cin & 31) || (ldi & 7) || (ci_off & 7) || (N & 63) || (ldo & 7) || (co_off & 7)) return (int)hipErrorInvalidValue;
  if (res && ((ldr & 7) || (r_off & 7))) return (int)hipErrorInvalidValue;
  Hx3Args a;
  a.in_f = in; a.res_f = res; a.out_f = out; a.w = wfrag; a.bias = bias; a.occ = nullptr;
  a.uni = nullptr; a.uni_val = nullptr; a.uni_min = 0;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off; a.Ho = H; a.Wo = W;
  a.N = N; a.ldo = ldo; a.co_off = co_off; a.ldr = ldr; a.r_off = r_off; a.act = act;
  if ((long)B * H * W * ldi * 4 >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit buffer offsets
  return hx3_launch(a, tile, stream);
}

// fp32 mode, pair activations in and out, 3x3 stride 2 pad 1 (conv_hx3s2_kernel), same weight
// image as tca_conv_hx3p.  act | 32: fp32 storage out instead of pairs (no residual).  Output [B, Ho, Wo, ldo] with Ho = (H + 1) / 2, Wo = (W + 1) / 2.
// occ: optional uint8 [B, H, W] input occupancy (a pixel marked 0 is read as zeros).
// uni / uni_min / uni_val: optional uniform-tile skipping on the output grid (tca_conv_hx3p_uni;
// uni_min 1 = the stride-2 window holds no occupied cell, tca_bev_uniform_depth).
// tile: 0 auto, 1-4 (hx3s2_launch).
TCA_API int tca_conv_hx3s2p(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* wfrag,
                            const float* bias, int N, float* out, int ldo, int co_off, int act, const float* res,
                            int ldr, int r_off, const unsigned char* occ, const unsigned char* uni, int uni_min,
                            const float* uni_val, int tile, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((act & 32) && res) return (int)hipErrorInvalidValue;
  if ((Cin & 31) || (ldi & 7) || (ci_off & 7) || (N & 63) || (ldo & 7) || (co_off & 7)) return (int)hipErrorInvalidValue;
  if (res && ((ldr & 7) || (r_off & 7))) return (int)hipErrorInvalidValue;
  Hx3Args a;
  if (uni && (!uni_val || uni_min < 1 || res)) return (int)hipErrorInvalidValue;
  a.in_f = in; a.res_f = res; a.out_f = out; a.w = wfrag; a.bias = bias; a.occ = occ;
  a.uni = uni; a.uni_val = uni_val; a.uni_min = uni ? uni_min : 0;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off; a.Ho = (H + 1) / 2; a.Wo = (W + 1) / 2;
  a.N = N; a.ldo = ldo; a.co_off = co_off; a.ldr = ldr; a.r_off = r_off; a.act = act;
  if ((long)B * H * W * ldi * 4 >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit buffer offsets
  return hx3s2_launch(a, tile, stream);
}

// tca_conv_hx3p with uniform-tile skipping (Hx3Args::uni): uni uint8 [B, H, W] uniform depth
// (tca_bev_uniform_depth), uni_min the depth this layer's output needs to be the constant
// uni_val (pair storage [N], the dense kernel's own output on such a pixel).  No residual.
TCA_API int tca_conv_hx3p_uni(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* wfrag,
                              const float* bias, int N, float* out, int ldo, int co_off, int act,
                              const unsigned char* uni, int uni_min, const float* uni_val, int tile,
                              hipStream_t stream) {
  if (B <= 0) return 0;
  if ((Cin & 31) || (ldi & 7) || (ci_off & 7) || (N & 63) || (ldo & 7) || (co_off & 7)) return (int)hipErrorInvalidValue;
  if (!uni || !uni_val || uni_min < 1) return (int)hipErrorInvalidValue;
  Hx3Args a;
  a.in_f = in; a.res_f = nullptr; a.out_f = out; a.w = wfrag; a.bias = bias; a.occ = nullptr;
  a.uni = uni; a.uni_val = uni_val; a.uni_min = uni_min;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off; a.Ho = H; a.Wo = W;
  a.N = N; a.ldo = ldo; a.co_off = co_off; a.ldr = 0; a.r_off = 0; a.act = act;
  if ((long)B * H * W * ldi * 4 >= (1L << 31)) return (int)hipErrorInvalidValue;
  return hx3_launch(a, tile, stream);
}

// ---- uniform depth of a sparse BEV canvas behind a 3x3 stride-2 pad-1 conv.
//
// u(p) (output pixel p of that first conv, [Ho, Wo] = [(H + 1) / 2, (W + 1) / 2]): its 3 x 3
// stride-2 input window holds no occupied canvas cell, so its accumulators are exactly 0 and it
// holds act(bias), the same vector everywhere.  A following 3x3 stride-1 pad-1 conv maps a pixel
// whose 9 neighbours are all inside the image and uniform to one constant again, and so on: the
// j-th conv of the chain (the stride-2 one is j = 1) outputs its constant at p iff every pixel
// within Chebyshev radius j - 1 of p is inside the image and has u.  depth(p) = the largest such
// j, capped at maxd (0: p itself is not uniform).  One workgroup per 16 x 64 output tile: u of
// the tile plus a (maxd - 1) halo into LDS, then a ring scan per pixel.
namespace {

constexpr int UD_TY = 16, UD_TX = 64, UD_MAXR = 7;
static_assert(UD_TX + 2 * UD_MAXR < 128, "u rows are walked 128 columns at a time");

__global__ void __launch_bounds__(256) bev_uniform_depth_kernel(const unsigned char* __restrict__ occ, int H, int W,
                                                                 int Ho, int Wo, int maxd,
                                                                 unsigned char* __restrict__ depth) {
  constexpr int LY = UD_TY + 2 * UD_MAXR, LX = UD_TX + 2 * UD_MAXR;
  constexpr int OY = 2 * LY + 1, OX = 2 * LX + 1;  // the canvas window behind the u region
  __shared__ unsigned char u[LY * LX];
  __shared__ unsigned char os[OY * OX];
  const int b = blockIdx.z, ty0 = blockIdx.y * UD_TY, tx0 = blockIdx.x * UD_TX;
  const int R = maxd - 1;
  const int ry = UD_TY + 2 * R, rx = UD_TX + 2 * R;
  const unsigned char* oc = occ + (long)b * H * W;
  // the occupancy window once into LDS (coalesced byte rows; each canvas byte feeds up to 4 u
  // cells' 3 x 3 stride-2 windows), outside the canvas as occupied-free
  const int iy0 = 2 * (ty0 - R) - 1, ix0 = 2 * (tx0 - R) - 1, oy = 2 * ry + 1, ox = 2 * rx + 1;
  // rows by wave, columns by lane: no per-element integer division (a runtime divisor costs ~40
  // VALU instructions per element)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = wv; r < oy; r += nw) {
    const int iy = iy0 + r;
    const bool row_in = (unsigned)iy < (unsigned)H;
    for (int c = lane; c < ox; c += 64) {
      const int ix = ix0 + c;
      os[r * OX + c] = (row_in && (unsigned)ix < (unsigned)W) ? oc[(long)iy * W + ix] : 0;
    }
  }
  __syncthreads();
  for (int id = threadIdx.x; id < ry * 128; id += blockDim.x) {  // rx <= UD_TX + 2 * UD_MAXR < 128
    const int ly = id >> 7, lx = id & 127;
    if (lx >= rx) continue;
    const int Y = ty0 - R + ly, X = tx0 - R + lx;
    unsigned char good = 0;
    if (Y >= 0 && X >= 0 && Y < Ho && X < Wo) {
      const unsigned char* w = os + (2 * ly) * OX + 2 * lx;  // window rows 2 ly .. 2 ly + 2
      const unsigned any = w[0] | w[1] | w[2] | w[OX] | w[OX + 1] | w[OX + 2] | w[2 * OX] | w[2 * OX + 1] |
                           w[2 * OX + 2];
      good = any ? 0 : 1;
    }
    u[ly * LX + lx] = good;
  }
  __syncthreads();
  for (int id = threadIdx.x; id < UD_TY * UD_TX; id += blockDim.x) {
    const int py = id / UD_TX, px = id - (id / UD_TX) * UD_TX;
    const int Y = ty0 + py, X = tx0 + px;
    if (Y >= Ho || X >= Wo) continue;
    const int cy = py + R, cx = px + R;
    int d = 0;
    if (u[cy * LX + cx]) {
      d = 1;
      for (int k = 1; k <= R; ++k) {  // ring of radius k
        bool ok = true;
        for (int t = -k; t <= k && ok; ++t)
          ok = u[(cy - k) * LX + cx + t] && u[(cy + k) * LX + cx + t] && u[(cy + t) * LX + cx - k] &&
               u[(cy + t) * LX + cx + k];
        if (!ok) break;
        d = k + 1;
      }
    }
    depth[((long)b * Ho + Y) * Wo + X] = (unsigned char)d;
  }
}

}  // namespace

// occ: uint8 [B, H, W] canvas occupancy; depth: uint8 [B, (H + 1) / 2, (W + 1) / 2]; 1 <= maxd <= 8.
TCA_API int tca_bev_uniform_depth(const unsigned char* occ, int B, int H, int W, int maxd, unsigned char* depth,
                                  hipStream_t stream) {
  if (B <= 0) return 0;
  if (maxd < 1 || maxd > UD_MAXR + 1) return (int)hipErrorInvalidValue;
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  dim3 grid((unsigned)((Wo + UD_TX - 1) / UD_TX), (unsigned)((Ho + UD_TY - 1) / UD_TY), (unsigned)B);
  bev_uniform_depth_kernel<<<grid, 256, 0, stream>>>(occ, H, W, Ho, Wo, maxd, depth);
  TCA_LAUNCH_CHECK();
}
