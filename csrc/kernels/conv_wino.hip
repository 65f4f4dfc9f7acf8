// fp32-mode 3x3 stride-1 pad-1 convolution by 1-D Winograd F(2,3) along the fragment axis
// ("wino") for the PointPillars / CenterPoint BEV backbones (data/pointpillar.yaml:64-70
// BaseBEVBackbone, run by examples/pointpillar_kitti/1/model.py:163).
//
// Why: conv_hx3.hip runs these layers at 46-58 % of the bf16 MFMA peak with 9 taps x 3 split
// products per output.  F(2,3) along one axis computes two outputs from four transformed inputs
// per tap row: 4 x 3 = 12 (position, line-tap) products per output pair instead of 18, 1.5x fewer
// MFMAs for the same fp32 result (split-product accuracy, tests/test_wino_gpu.py: rel-L2 within
// the fp32-mode budget of tests/test_fp32_mode_gpu.py).
//
// Axes (as hx3): the fragment axis F carries 16 Winograd tiles = 32 output pixels per workgroup
// (the N dimension of mfma_f32_16x16x32_bf16), the line axis L carries TH output lines.  CM:
// F = y (image rows), L = x; else F = x, L = y.  Per 32-channel chunk:
//   1. the workgroup's lanes transform the input: item (U line u, 8-channel group cq, tile t)
//      loads the 4 input pixels 2t-1 .. 2t+2 along F (buffer loads, zeros outside the image by
//      the descriptor range check), joins pair storage to fp32 (or reads fp32), forms
//      U0 = d0 - d2, U1 = d1 + d2, U2 = d2 - d1, U3 = d1 - d3 and writes their bf16 hi / lo
//      split to an LDS image [u][position][cq][hi|lo][t][16 B] (the B-operand fragment of lane
//      (t, cq) is 16 contiguous bytes; reads and writes bank-conflict free);
//   2. every wave runs its output channels against the whole image: position group p reads the
//      TH + 2 U lines once and feeds each to the three line taps kl (output line u - kl), with
//      the transformed weights V_p[kl] streamed from L2 into registers one group ahead (hx3's
//      fragment-order image; ops/conv.py wino_weights).
// The raw halo of chunk c + 1 lands by LDS DMA during chunk c's MFMAs; its transform runs between
// chunks (one image, two workgroups per CU, so one's transform overlaps the other's MFMAs).  Epilogue: y0 = m0 + m1 + m2, y1 = m1 - m2 - m3 per lane (the lane
// holds all four positions of its tile), bias + act, an LDS staging tile, 16-B stores.
#include "tca_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr unsigned kOutOfRange = 0x80000000u;  // buffer offset past any num_records (< 2^31): reads zeros

struct WinoArgs {
  const float* in_f;  // [B, H, W, ldi] pair or fp32 storage, channels [ci_off, ci_off + Cin)
  float* out_f;       // [B, H, W, ldo] pair or fp32 storage, channels [co_off, co_off + N)
  const void* w;      // fragment-order split transformed weights (ops/conv.py wino_weights)
  const float* bias;  // [N] or null
  int B, H, W, Cin, ldi, ci_off;
  int N, ldo, co_off, act;  // act: 0 none, 1 relu
  // optional, as conv_hx3.hip Hx3Args: uint8 [B, H, W] uniform depth and the output storage [N]
  // of this layer on a uniform pixel; a tile whose pixels all reach uni_min stores it directly
  const unsigned char* uni;
  const float* uni_val;
  int uni_min;
};

__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// plain (unpacked) f32 add / sub: the SLP vectoriser would pair them into v_pk_add_f32, which
// costs more issue cycles beside the partner wave's MFMAs (MI355X_MICROARCH constants table)
__device__ __forceinline__ float fadd1(float x, float y) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ float fsub1(float x, float y) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

__device__ __forceinline__ void split8(const float* v, u32x4& hi, u32x4& lo) {
  __bf16 h[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = (__bf16)v[e];
    l[e] = (__bf16)fsub1(v[e], (float)h[e]);
  }
  hi = *reinterpret_cast<const u32x4*>(h);
  lo = *reinterpret_cast<const u32x4*>(l);
}

// 8 channels of one input pixel as fp32: pair storage (8 hi bf16 | 8 lo bf16) or fp32 (two quads)
template <bool PIN>
__device__ __forceinline__ void join8(const u32x4& p0, const u32x4& p1, float* d) {
  if constexpr (PIN) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[2 * q] = bf_lo(p0[q]) + bf_lo(p1[q]);
      d[2 * q + 1] = bf_hi(p0[q]) + bf_hi(p1[q]);
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[q] = __uint_as_float(p0[q]);
      d[4 + q] = __uint_as_float(p1[q]);
    }
  }
}

template <int P> struct PosC { static constexpr int value = P; };

// one 16-B-per-lane LDS DMA through a buffer resource: voffset per lane, soffset scalar; the wave's
// 64 pieces land contiguously at the wave-uniform LDS address l (lane i at l + 16 i)
__device__ __forceinline__ void bdma16(unsigned voff, __amdgpu_buffer_rsrc_t rsrc, const void* l, unsigned soff) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
               : "memory");
}

__device__ __forceinline__ void wait_vmcnt0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
template <int N>
__device__ __forceinline__ void wait_vm() {  // at most this wave's N youngest vector-memory ops in flight
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Raw-halo layout of (pixel fi along F, 16-B piece slot = cq * 2 + hl).  A transform read (fixed
// j and hl) has lane (cq, t) at pixel 2t + j; a ds_read_b128 lane group holds tiles t of two cq
// ({0-3, 12-15} of one, {4-11} of the other).  With 128 B per pixel all 16 lanes of a group fall
// in one 128-B half of the 64 banks (2-way at best), so pixel pairs swap places by bit 1 of fi
// (raw_pos: the half alternates with t), and the slot XOR (raw_slot) takes (fi >> 2) & 3 plus
// bit 3 of fi / 2 + 4, which separates the two cq's tile sets: conflict-free for j = 0, 1, a few
// 2-way lanes for j = 2, 3 (was 2-way throughout).
__device__ __forceinline__ int raw_pos(int fi) { return fi ^ ((fi >> 1) & 1); }
__device__ __forceinline__ int raw_slot(int fi, int slot) {
  return slot ^ (((fi >> 2) & 3) | (((((fi >> 1) + 4) >> 3) & 1) << 2));
}

template <int TH, int WN, int FN, bool CM, bool PIN, bool POUT>
__global__ void __launch_bounds__(WN * 64, 2) conv_wino_kernel(WinoArgs a) {
  constexpr int NT = WN * 64, BN = WN * FN * 16, TF = 32, NU = TH + 2;
  constexpr int NITEM = NU * 64, IPT = (NITEM + NT - 1) / NT;
  constexpr int UB = NU * 8192;  // one U image: NU lines x 4 positions x 4 groups x 2 x 16 tiles x 16 B
  // raw halo of one chunk: NU lines x 34 pixels x 8 pieces of 16 B, staged by LDS DMA (whole
  // wave-instructions of 64 pieces; the pieces past the halo read zeros into padding)
  constexpr int NPIECE = NU * 34 * 8, NINS = (NPIECE + 63) / 64, DPW = (NINS + WN - 1) / WN;
  constexpr int RAWB = NINS * 1024;  // instruction k * WN + wn of wave wn; waves past NINS idle
  constexpr int EPI = TH * TF * BN * 4;
  constexpr int LDS = (UB + RAWB) > EPI ? UB + RAWB : EPI;
  static_assert(2 * LDS <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];
  unsigned char* const raw = smem + UB;

  const int tid = threadIdx.x, lane = tid & 63, wn = tid >> 6;
  const int FH = CM ? a.H : a.W, LW = CM ? a.W : a.H;
  const int nF = (FH + TF - 1) / TF, nL = (LW + TH - 1) / TH;
  const int nmt = a.B * nF * nL, nnt = a.N / BN, nwg = nmt * nnt;
  int bid = blockIdx.x;
  {  // XCD-aware: consecutive tiles (sharing halo lines and weights in L2) on one XCD
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int mt = bid / nnt, nt = bid - mt * nnt;
  const int b = mt / (nF * nL), rem = mt - b * (nF * nL);
  const int f0 = (rem / nL) * TF, l0 = (rem - (rem / nL) * nL) * TH;
  const int n0 = nt * BN;
  auto pix_yx = [&](int f, int l, int& y, int& x) {
    y = CM ? f : l;
    x = CM ? l : f;
  };

  if (a.uni) {
    bool bad = false;
    for (int ml = tid; ml < TH * TF; ml += NT) {
      int y, x;
      pix_yx(f0 + (ml & 31), l0 + (ml >> 5), y, x);
      if (y < a.H && x < a.W) bad |= a.uni[((long)b * a.H + y) * a.W + x] < a.uni_min;
    }
    if (!__syncthreads_or(bad)) {
      constexpr int Q = BN / 4;
      for (int id = tid; id < TH * TF * Q; id += NT) {
        const int ml = id / Q, q = id - (id / Q) * Q;
        int y, x;
        pix_yx(f0 + (ml & 31), l0 + (ml >> 5), y, x);
        if (y >= a.H || x >= a.W) continue;
        const long o = (((long)b * a.H + y) * a.W + x) * a.ldo + a.co_off + n0 + q * 4;
        *reinterpret_cast<u32x4*>(a.out_f + o) = *reinterpret_cast<const u32x4*>(a.uni_val + n0 + q * 4);
      }
      return;
    }
  }

  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.in_f, (short)0, a.B * a.H * a.W * a.ldi * 4, 0x00020000);
  // DMA pieces of this lane: piece q = (instruction k * WN + wn) * 64 + lane = (u * 34 + fi) * 8 + phys
  unsigned dvo[DPW];
#pragma unroll
  for (int k = 0; k < DPW; ++k) {
    const int q = (k * WN + wn) * 64 + lane;
    const int u = q / 272, fi = raw_pos((q / 8) % 34), slot = raw_slot(fi, q & 7);
    int y, x;
    pix_yx(f0 - 1 + fi, l0 - 1 + u, y, x);
    dvo[k] = (q < NPIECE && (unsigned)y < (unsigned)a.H && (unsigned)x < (unsigned)a.W)
                 ? (unsigned)(((((long)b * a.H + y) * a.W + x) * a.ldi + a.ci_off + (slot >> 1) * 8) * 4 + (slot & 1) * 16)
                 : kOutOfRange;
  }
  auto raw_dma = [&](int c) {
#pragma unroll
    for (int k = 0; k < DPW; ++k)
      if (NINS % WN == 0 || k * WN + wn < NINS) bdma16(dvo[k], rin, raw + (k * WN + wn) * 1024, (unsigned)(c * 128));
  };
  // transform: item id = (u * 4 + cq) * 16 + t -> the 4 positions' hi / lo slots of (u, cq, t)
  // always inlined: with pair input the inliner kept it a function (a call per chunk, its
  // captures passed through scratch memory)
  auto transform = [&]() __attribute__((always_inline)) {
    unsigned char* ub = smem;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int id = tid + k * NT;
      if (NITEM % NT != 0 && id >= NITEM) continue;
      const int u = id >> 6, cq = (id >> 4) & 3, t = id & 15;
      float d[4][8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int fi = 2 * t + j;
        const unsigned char* rp = raw + (u * 34 + raw_pos(fi)) * 128;
        const u32x4 p0 = *reinterpret_cast<const u32x4*>(rp + raw_slot(fi, cq * 2) * 16);
        const u32x4 p1 = *reinterpret_cast<const u32x4*>(rp + raw_slot(fi, cq * 2 + 1) * 16);
        join8<PIN>(p0, p1, d[j]);
      }
      // image slot: ((((u * 4 + p) * 4 + cq) * 2 + hl) * 16 + t) * 16
      unsigned char* wp = ub + ((u * 16 + cq) * 32 + t) * 16;
      float uv[8];
      u32x4 hi, lo;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          uv[e] = p == 0 ? fsub1(d[0][e], d[2][e]) : p == 1 ? fadd1(d[1][e], d[2][e])
                  : p == 2 ? fsub1(d[2][e], d[1][e]) : fsub1(d[1][e], d[3][e]);
        split8(uv, hi, lo);
        *reinterpret_cast<u32x4*>(wp + p * 2048) = hi;
        *reinterpret_cast<u32x4*>(wp + p * 2048 + 256) = lo;
      }
    }
  };

  // weights: block (ks, g, hl) = 64 lanes x 8 bf16, ks = (kl * 4 + p) * nc + c.  Streamed per
  // step (c, p, kl) through a 3-deep register ring (set = kl), two steps ahead.
  // Buffer loads: the lane part of the address is fixed, the step part is scalar (no VALU per load).
  const int NG = a.N / 16, g0 = n0 / 16 + wn * FN;
  const int nc = a.Cin / 32, NS = 12 * nc;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, NS * NG * 2048, 0x00020000);
  const unsigned wvo = (unsigned)(g0 * 2048 + lane * 16);
  auto wload = [&](int s, bf16x8 (&dst)[FN][2]) {  // step s = (c * 4 + p) * 3 + kl
    s = s < NS ? s : NS - 1;
    const int kl = s % 3, p = (s / 3) & 3, c = s / 12;
    const unsigned so = (unsigned)(((kl * 4 + p) * nc + c) * NG * 2048);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      dst[j][0] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wvo + j * 2048, so, 0));
      dst[j][1] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wvo + j * 2048 + 1024, so, 0));
    }
  };

  // position 1 enters both outputs (y0 = m0 + m1 + m2, y1 = m1 - m2 - m3): its accumulators start
  // at the bias, so the epilogue adds none
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[TH][4][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const f32x4 bv = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + n0 + (wn * FN + j) * 16 + fq * 4)
                            : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int p = 0; p < 4; ++p) acc[i][p][j] = p == 1 ? bv : f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int rd = (fq * 2 * 16 + fr) * 16;  // this lane's B-fragment slot (hi) inside a (line, position) block
  bf16x8 w[3][FN][2];
  // one step: line tap kl of position p over the TH output lines (U lines i + kl), two lines at a
  // time, its weights streamed two steps ahead.  (Reading the position's NU lines into registers
  // once for its three taps measured ~10 % slower: profiles/r5/wino_ab.md.)
  auto step = [&](auto PC, auto KC, const unsigned char* ub, int s_next) {
    constexpr int p = decltype(PC)::value, kl = decltype(KC)::value;
    wload(s_next, w[(kl + 2) % 3]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i0 = 0; i0 < TH; i0 += 2) {
      bf16x8 ah[2], al[2];
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const unsigned char* sp = ub + ((i0 + ii + kl) * 4 + p) * 2048 + rd;
        ah[ii] = *reinterpret_cast<const bf16x8*>(sp);
        al[ii] = *reinterpret_cast<const bf16x8*>(sp + 256);
      }
#pragma unroll
      for (int pr = 0; pr < 3; ++pr)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const bf16x8& wv = pr == 0 ? w[kl][j][1] : w[kl][j][0];
            const bf16x8& x = pr == 1 ? al[ii] : ah[ii];
            acc[i0 + ii][p][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, x, acc[i0 + ii][p][j], 0, 0, 0);
          }
    }
  };
  auto position = [&](auto PC, const unsigned char* ub, int s0) {
    step(PC, PosC<0>{}, ub, s0 + 2);
    step(PC, PosC<1>{}, ub, s0 + 3);
    step(PC, PosC<2>{}, ub, s0 + 4);
  };

  // one U image and one raw halo: two workgroups per CU overlap one's transform with the
  // other's MFMAs.  Chunk c: MFMAs on U(c) while the DMA of raw(c + 1) lands; then
  // transform raw(c + 1) -> U(c + 1) between two barriers and start the DMA of raw(c + 2).
  raw_dma(0);
  wload(0, w[0]);
  wload(1, w[1]);
  wait_vmcnt0();
  lds_barrier();
  transform();
  lds_barrier();  // the image is visible and every wave is done with the raw halo
  if (nc > 1) raw_dma(1);
  const unsigned char* ub = smem;
  for (int c = 0; c < nc; ++c) {
    const int s0 = c * 12;
    position(PosC<0>{}, ub, s0);
    position(PosC<1>{}, ub, s0 + 3);
    position(PosC<2>{}, ub, s0 + 6);
    position(PosC<3>{}, ub, s0 + 9);
    if (c + 1 < nc) {
      wait_vm<4 * FN>();  // all but the next chunk's two prefetched weight steps: raw(c + 1) landed
      lds_barrier();      // ... for every wave; every wave is done reading U(c)
      transform();
      lds_barrier();
      if (c + 2 < nc) raw_dma(c + 2);
    }
  }
  wait_vmcnt0();  // the clamped tail prefetches
  lds_barrier();  // the epilogue reuses the image

  // ---- epilogue: output transform + bias + act -> fp32 staging tile [TH * 32 rows][BN] (16-B
  // quads XOR-swizzled by the row) -> 16-B stores.  A lane writes rows 2 fr and 2 fr + 1 (a tile's
  // two outputs), so hx3's row swizzle (ml & 15) gave the 8 lanes of a ds_write_b128 group only 4
  // distinct quads mod 8 (2-way conflicts); bit 3 of the row folded into bit 0 makes them 8, and
  // rows 2k / 2k + 1 still differ in bit 0 (the ds_read_b128 groups span two rows: conflict-free).
  float* st = reinterpret_cast<float*>(smem);
  auto quad = [](int ml, int q) { return ml * BN + ((q ^ ((ml & 15) ^ ((ml >> 3) & 1))) << 2); };
  const float lo = a.act == 1 ? 0.f : -__builtin_inff();  // ReLU as one max
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = (wn * FN + j) * 16 + fq * 4;
#pragma unroll
    for (int i = 0; i < TH; ++i) {
      float y0[4], y1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float m0 = acc[i][0][j][r], m1 = acc[i][1][j][r], m2 = acc[i][2][j][r], m3 = acc[i][3][j][r];
        y0[r] = fmaxf((m0 + m1) + m2, lo);
        y1[r] = fmaxf((m1 - m2) - m3, lo);
      }
      const int ml = i * TF + 2 * fr;
      *reinterpret_cast<float4*>(st + quad(ml, nl >> 2)) = make_float4(y0[0], y0[1], y0[2], y0[3]);
      *reinterpret_cast<float4*>(st + quad(ml + 1, nl >> 2)) = make_float4(y1[0], y1[1], y1[2], y1[3]);
    }
  }
  __syncthreads();
  constexpr int V8 = BN / 8;
  for (int id = tid; id < TH * TF * V8; id += NT) {
    const int ml = id / V8, c8 = (id - (id / V8) * V8) * 8;
    int y, x;
    pix_yx(f0 + (ml & 31), l0 + (ml >> 5), y, x);
    if (y >= a.H || x >= a.W) continue;
    const float4 v0 = *reinterpret_cast<const float4*>(st + quad(ml, c8 >> 2));
    const float4 v1 = *reinterpret_cast<const float4*>(st + quad(ml, (c8 >> 2) + 1));
    float* o = a.out_f + (((long)b * a.H + y) * a.W + x) * a.ldo + a.co_off + n0 + c8;
    if constexpr (POUT) {
      const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      u32x4 hi, lo;
      split8(v, hi, lo);
      *reinterpret_cast<u32x4*>(o) = hi;
      *reinterpret_cast<u32x4*>(o + 4) = lo;
    } else {
      *reinterpret_cast<float4*>(o) = v0;
      *reinterpret_cast<float4*>(o + 4) = v1;
    }
  }
}

template <int TH, int WN, int FN, bool CM>
int launch_wino(const WinoArgs& a, bool pin, bool pout, hipStream_t stream) {
  constexpr int BN = WN * FN * 16;
  if (a.N % BN) return (int)hipErrorInvalidValue;
  const int FH = CM ? a.H : a.W, LW = CM ? a.W : a.H;
  const long nwg = (long)a.B * ((FH + 31) / 32) * ((LW + TH - 1) / TH) * (a.N / BN);
  if (nwg <= 0 || nwg >= (1L << 31)) return (int)hipErrorInvalidValue;
  if (pin && pout) conv_wino_kernel<TH, WN, FN, CM, true, true><<<(unsigned)nwg, WN * 64, 0, stream>>>(a);
  else if (pin) conv_wino_kernel<TH, WN, FN, CM, true, false><<<(unsigned)nwg, WN * 64, 0, stream>>>(a);
  else if (pout) conv_wino_kernel<TH, WN, FN, CM, false, true><<<(unsigned)nwg, WN * 64, 0, stream>>>(a);
  else conv_wino_kernel<TH, WN, FN, CM, false, false><<<(unsigned)nwg, WN * 64, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// tiles.  0 = auto: N % 128 == 0 -> 4 waves x 32 channels, else 4 waves x 16 channels; F along
// the axis with the smaller padding to 32.
int wino_launch(const WinoArgs& a, int tile, bool pin, bool pout, hipStream_t stream) {
  if (tile == 0) {
    const long pad_y = (long)((a.H + 31) / 32 * 32) * a.W, pad_x = (long)((a.W + 31) / 32 * 32) * a.H;
    const bool cm = pad_y <= pad_x;
    if (a.N % 128 == 0) tile = cm ? 2 : 1;
    else if (a.N % 64 == 0) tile = cm ? 4 : 3;
    else return (int)hipErrorInvalidValue;
  }
  switch (tile) {
    case 1: return launch_wino<4, 4, 2, false>(a, pin, pout, stream);
    case 2: return launch_wino<4, 4, 2, true>(a, pin, pout, stream);
    case 3: return launch_wino<4, 4, 1, false>(a, pin, pout, stream);
    case 4: return launch_wino<4, 4, 1, true>(a, pin, pout, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// fp32 mode, 3x3 stride 1 pad 1 by F(2,3) (conv_wino_kernel).  in / out: pair storage
// (pair_in / pair_out = 1) or fp32 NHWC; wfrag: ops/conv.py wino_weights, [12 * Cin / 32][N / 16]
// [hi | lo][64 lanes][8 bf16] over the transformed taps (kl * 4 + position); act 0 / 1 (ReLU).
// uni / uni_min / uni_val: optional uniform-tile skipping (conv_hx3.hip tca_conv_hx3p_uni).
// tile: 0 auto, 1-4 (wino_launch).
TCA_API int tca_conv_wino(const float* in, int B, int H, int W, int Cin, int ldi, int ci_off, int pair_in,
                          const void* wfrag, const float* bias, int N, float* out, int ldo, int co_off, int pair_out,
                          int act, const unsigned char* uni, int uni_min, const float* uni_val, int tile,
                          hipStream_t stream) {
  if (B <= 0) return 0;
  if ((Cin & 31) || (ldi & 7) || (ci_off & 7) || (N & 63) || (ldo & 7) || (co_off & 7)) return (int)hipErrorInvalidValue;
  if (act != 0 && act != 1) return (int)hipErrorInvalidValue;
  if (uni && (!uni_val || uni_min < 1)) return (int)hipErrorInvalidValue;
  if ((long)B * H * W * ldi * 4 >= (1L << 31)) return (int)hipErrorInvalidValue;  // 32-bit buffer offsets
  WinoArgs a;
  a.in_f = in; a.out_f = out; a.w = wfrag; a.bias = bias;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.ldi = ldi; a.ci_off = ci_off;
  a.N = N; a.ldo = ldo; a.co_off = co_off; a.act = act;
  a.uni = uni; a.uni_val = uni_val; a.uni_min = uni ? uni_min : 0;
  return wino_launch(a, tile, pair_in != 0, pair_out != 0, stream);
}
