// Sparse-gather 3x3 stride-2 pad-1 conv for the first PointPillars BEV conv
// (data/pointpillar.yaml:64-70 BaseBEVBackbone block 1, LAYER_STRIDES[0] = 2, run by
// examples/pointpillar_kitti/1/model.py:163), fp32 mode: pair activations in, pair (or fp32)
// activations out, split-product MFMA (bf16 x3, fp32 accumulation), BN folded + act.
//
// The input is the scattered pillar canvas: ~3% of its cells are occupied, the rest are zero.
// The dense kernel (conv_hx3.hip hx3s2) runs all 9 taps x Cin of every output pixel and masks
// the loads of empty cells; here only the (output pixel, tap) pairs whose input cell is occupied
// are computed:
//   1. per TH x 32 output tile, the threads test the 9 input cells' occupancy bytes of every
//      output pixel; per tap, a ballot + cross-wave prefix builds the list of
//      (input cell, pixel) entries in LDS (deterministic order);
//   2. wave w owns output channels [16 w, 16 w + 16): for tap 0..8 in order it takes the tap's
//      list 16 entries at a time -- the activation fragment of entry fr is the input cell's
//      8-channel pair group (one 32-B load: 8 hi + 8 lo bf16, no split), the weight fragments
//      are conv_hx3's (ops/conv.py frag_weights) -- and adds the 16 x 16 result into the tile's
//      fp32 accumulators in LDS.  A pixel appears at most once per tap and the taps run in order,
//      so the accumulation order is fixed (bit-reproducible run to run) without atomics;
//   3. epilogue: bias + act, pair split (or fp32), 16-B stores of the whole dense tile (a pixel
//      without an occupied input gets act(bias): the dense kernel's value there, bit for bit).
// The MFMA work is ~2.25 x (occupied cells) 16-row fragments instead of 9 x (output pixels);
// the kernel is bound by its dense output stores.
#include "tca_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct S2spArgs {
  const float* in;           // pair storage [B, H, W, ldi], channels [ci_off, ci_off + Cin)
  const unsigned char* occ;  // uint8 [B, H, W]: 0 = the cell is zero in every channel
  const uint4* w;            // fragment-order split weights [9 * Cin / 32][N / 16][hi | lo][64 lanes] (16 B)
  const float* bias;         // [N] or null
  float* out;                // [B, Ho, Wo, ldo], channels [co_off, co_off + N)
  int B, H, W, ldi, ci_off, Ho, Wo, ldo, co_off;
  int act;                   // 0 none, 1 relu, 2 silu, 3 leaky(0.1); | 32: fp32 storage out
  int tiles_x, tiles;        // output tiles per row / per image
};

constexpr int TW = 32, N = 64, LDA = N + 4;

__device__ __forceinline__ float act_fn(float v, int act) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return v / (1.f + __expf(-v));
    case 3: return v > 0.f ? v : 0.1f * v;
    default: return v;
  }
}

// TH = 8: 256 pixels, one per thread (78 KiB LDS, two workgroups per CU); TH = 4: 128 pixels
// (40 KiB, four per CU); TH = 2: 64 pixels (20 KiB, eight per CU)
template <int KC, int TH>
__global__ void __launch_bounds__(256) conv_s2sp_kernel(S2spArgs a) {
  constexpr int NPIX = TH * TW;
  __shared__ float acc_s[NPIX * LDA];   // the tile's fp32 accumulators, pixel-major
  __shared__ int list_s[9][NPIX];       // per tap: (input cell << 8) | pixel
  __shared__ int cnt_s[9][4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // blockIdx.x walks the tiles of one image: consecutive workgroups (round-robined over the
  // XCDs) share input rows in L2 only through the 2-row halo, so no remapping is needed
  const int b = blockIdx.y, tile = blockIdx.x;
  const int oy0 = (tile / a.tiles_x) * TH, ox0 = (tile % a.tiles_x) * TW;

  for (int i = tid; i < NPIX * LDA / 4; i += 256) reinterpret_cast<float4*>(acc_s)[i] = make_float4(0.f, 0.f, 0.f, 0.f);

  // 1. per-tap lists of occupied (input cell, pixel) entries
  const int p = tid % NPIX, oy = oy0 + p / TW, ox = ox0 + p % TW;
  const bool in_out = oy < a.Ho && ox < a.Wo;
  // 256 / NPIX thread groups share the taps: group g tests taps t with t % G == g
  constexpr int G = 256 / NPIX;
  const int tg = tid / NPIX;
  auto mine = [&](int t) { return G == 1 || t % G == tg; };
  const unsigned char* occ_b = a.occ + (long)b * a.H * a.W;
  unsigned okm = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = 2 * oy - 1 + t / 3, ix = 2 * ox - 1 + t % 3;
    const bool ok = mine(t) && in_out && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W && occ_b[iy * a.W + ix] != 0;
    okm |= (unsigned)ok << t;
    const unsigned long long m = __ballot(ok);
    if (lane == 0) cnt_s[t][wid] = __popcll(m);
  }
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const bool ok = (okm >> t) & 1u;
    const unsigned long long m = __ballot(ok);
    int off = 0;
    for (int w = 0; w < wid; ++w) off += cnt_s[t][w];
    if (ok) {
      const int iy = 2 * oy - 1 + t / 3, ix = 2 * ox - 1 + t % 3;
      list_s[t][off + __popcll(m & lt)] = ((iy * a.W + ix) << 8) | p;
    }
  }
  __syncthreads();

  // 2. wave wid: output channels [16 wid, 16 wid + 16); the (tap, 16-entry chunk) items in tap
  // order, the next item's activation and weight fragments loaded while this one computes
  const int fr = lane & 15, fq = lane >> 4;
  const float* in_b = a.in + (long)b * a.H * a.W * a.ldi + a.ci_off + 8 * fq;
  int cnt[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) cnt[t] = cnt_s[t][0] + cnt_s[t][1] + cnt_s[t][2] + cnt_s[t][3];
  struct Item {
    uint4 xh[KC], xl[KC], wh[KC], wl[KC];
    int e;
    bool valid;
  };
  auto load = [&](int t, int c0, Item& it) {
    it.valid = c0 + fr < cnt[t];
    it.e = list_s[t][it.valid ? c0 + fr : c0];
    const float* src = in_b + (long)(it.e >> 8) * a.ldi;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      it.xh[kc] = *reinterpret_cast<const uint4*>(src + kc * 32);
      it.xl[kc] = *reinterpret_cast<const uint4*>(src + kc * 32 + 4);
      const uint4* wf = a.w + ((long)((t * KC + kc) * (N / 16) + wid) * 2) * 64 + lane;
      it.wh[kc] = wf[0];
      it.wl[kc] = wf[64];
    }
  };
  // next item after (t, c0): the following chunk of tap t, else the first chunk of the next
  // tap with entries; t == 9: none
  auto advance = [&](int& t, int& c0) {
    c0 += 16;
    if (t >= 0 && t < 9 && c0 < cnt[t]) return;
    c0 = 0;
    for (++t; t < 9 && cnt[t] == 0; ++t) {
    }
  };
  int t = -1, c0 = 0;
  advance(t, c0);
  Item cur, nxt;
  if (t < 9) load(t, c0, cur);
  while (t < 9) {
    int tn = t, cn = c0;
    advance(tn, cn);
    if (tn < 9) load(tn, cn, nxt);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {  // products in conv_hx3.hip mfma3's order
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(&cur.xh[kc]);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(&cur.xl[kc]);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&cur.wh[kc]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&cur.wl[kc]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc, 0, 0, 0);
    }
    if (cur.valid) {  // lane: channels 16 wid + 4 fq .. + 4 of entry fr's pixel
      float4* dst = reinterpret_cast<float4*>(acc_s + (cur.e & 255) * LDA + 16 * wid + 4 * fq);
      float4 v = *dst;
      v.x += acc[0]; v.y += acc[1]; v.z += acc[2]; v.w += acc[3];
      *dst = v;
    }
    cur = nxt;
    t = tn;
    c0 = cn;
  }
  __syncthreads();

  // 3. epilogue: 8 channels (one pair group) per thread and pass
  const int act = a.act & 15;
  for (int id = tid; id < NPIX * (N / 8); id += 256) {
    const int q = id / (N / 8), c8 = (id % (N / 8)) * 8;
    const int y = oy0 + q / TW, x = ox0 + q % TW;
    if (y >= a.Ho || x >= a.Wo) continue;
    const float4 v0 = *reinterpret_cast<const float4*>(acc_s + q * LDA + c8);
    const float4 v1 = *reinterpret_cast<const float4*>(acc_s + q * LDA + c8 + 4);
    float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    if (a.bias) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += a.bias[c8 + k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_fn(v[k], act);
    float* o = a.out + (((long)b * a.Ho + y) * a.Wo + x) * a.ldo + a.co_off + c8;
    if (a.act & 32) {
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
      continue;
    }
    __bf16 h[8], l[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      h[k] = (__bf16)v[k];
      l[k] = (__bf16)(v[k] - (float)h[k]);
    }
    *reinterpret_cast<uint4*>(o) = *reinterpret_cast<const uint4*>(h);
    *reinterpret_cast<uint4*>(o + 4) = *reinterpret_cast<const uint4*>(l);
  }
}

}  // namespace

// fp32 mode, pair activations in, 3x3 stride 2 pad 1, N == 64, Cin 32 or 64, no residual:
// the same arguments and weights as tca_conv_hx3s2p (conv_hx3.hip), occ required.
// act | 32: fp32 storage out.  tile: 0 auto (4 x 32 output tiles), 1 (8 x 32), 2 (2 x 32).
TCA_API int tca_conv_s2sp(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, const void* wfrag,
                          const float* bias, int n, float* out, int ldo, int co_off, int act,
                          const unsigned char* occ, int tile, hipStream_t stream) {
  if (B <= 0) return 0;
  if (!occ || n != N || (Cin != 32 && Cin != 64) || (ldi & 7) || (ci_off & 7) || (ldo & 7) || (co_off & 7))
    return (int)hipErrorInvalidValue;
  if ((long)H * W >= (1L << 23)) return (int)hipErrorInvalidValue;  // cell index << 8 fits an int
  S2spArgs a;
  a.in = in; a.occ = occ; a.w = reinterpret_cast<const uint4*>(wfrag); a.bias = bias; a.out = out;
  a.B = B; a.H = H; a.W = W; a.ldi = ldi; a.ci_off = ci_off; a.Ho = (H + 1) / 2; a.Wo = (W + 1) / 2;
  a.ldo = ldo; a.co_off = co_off; a.act = act;
  const int TH = tile == 1 ? 8 : tile == 2 ? 2 : 4;  // 0 = auto (4 x 32), 1 = 8 x 32, 2 = 2 x 32
  a.tiles_x = (a.Wo + TW - 1) / TW;
  a.tiles = a.tiles_x * ((a.Ho + TH - 1) / TH);
  const dim3 grid(a.tiles, B);
  if (TH == 4) {
    if (Cin == 64) conv_s2sp_kernel<2, 4><<<grid, 256, 0, stream>>>(a);
    else conv_s2sp_kernel<1, 4><<<grid, 256, 0, stream>>>(a);
  } else if (TH == 2) {
    if (Cin == 64) conv_s2sp_kernel<2, 2><<<grid, 256, 0, stream>>>(a);
    else conv_s2sp_kernel<1, 2><<<grid, 256, 0, stream>>>(a);
  } else {
    if (Cin == 64) conv_s2sp_kernel<2, 8><<<grid, 256, 0, stream>>>(a);
    else conv_s2sp_kernel<1, 8><<<grid, 256, 0, stream>>>(a);
  }
  TCA_LAUNCH_CHECK();
}
