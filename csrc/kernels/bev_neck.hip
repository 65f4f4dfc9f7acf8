// K15 — fused BEV neck + anchor head (PointPillars / SECOND BaseBEVBackbone
// deblocks + AnchorHeadSingle's three 1x1 convs; reference config
// data/pointpillar.yaml:48-72 — UPSAMPLE_STRIDES [1, 2, 4], NUM_UPSAMPLE_FILTERS
// [128, 128, 128]; head conv_cls / conv_box / conv_dir on the 384-channel concat).
//
// Unfused, the three transpose convs write a [B, H, W, 384] bf16 concat
// (658 MB at batch 16 on the KITTI canvas) and the head reads it back: ~1.3 GB
// of HBM traffic and four launches.  Here one workgroup owns 128 output pixels
// that share a sub-pixel class (y mod S, x mod S), S = the largest upsample
// stride.  Every branch's transpose conv is then ONE GEMM with a single weight
// block (rows (y mod s_i, x mod s_i) of the k = s_i, stride s_i kernel) over
// the branch input pixel (y / s_i, x / s_i); its ReLU'd accumulators are fed
// straight back into the head GEMM as MFMA operands, never leaving registers:
//
//   acc1[i][j] (mfma 16x16x32 D layout) holds, in lane l, pixel (l & 15) and
//   branch channels 16j + 4(l >> 4) + r.  A 32-deep operand fragment needs
//   8 k values per lane group g = l >> 4; taking (acc1[2t][0..3], acc1[2t+1][0..3])
//   gives channels {32t + 4g + r, 32t + 16 + 4g + r}.  The head weights are
//   stored with each 32-channel chunk permuted the same way on the host
//   (perm(8g + e) = e < 4 ? 4g + e : 16 + 4g + e - 4), so the contraction
//   pairs matching channels.
//
// Persistent: one 512-thread workgroup per CU walks a contiguous range of
// 256-pixel tiles (ranges split per XCD so the 16 class tiles of one pixel
// panel share an L2); each of the 8 waves owns 32 pixels x all 128 channels of
// a branch and its own 32 x 80 head tile (no cross-wave reduction).  Operands
// are staged by global_load_lds in 64-channel K steps through two LDS stages;
// the pipeline runs straight across tile boundaries (step g+1 of the flat
// (tile, step) sequence is in flight while step g computes, one barrier per
// step).  Each stage also carries the step's 128 deconv biases (so the K loop
// issues no ordinary global load, which would make hipcc drain the DMA queue);
// head weights and bias are loaded once per workgroup and stay in LDS.
#include "tca_common.h"

using namespace tca;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int MAXBR = 3;
constexpr int CB = 128;   // output channels per branch
constexpr int BM = 256;   // pixels per tile
constexpr int NH = 80;    // head rows (72 padded to a multiple of 16)
constexpr int NW = 8, NT = NW * 64;
constexpr int ROWB = 128;  // 64 bf16 channels per staged row
constexpr int A_BYTES = BM * ROWB, B_BYTES = CB * ROWB, BIAS_BYTES = CB * 4;
constexpr int STAGE = A_BYTES + B_BYTES + BIAS_BYTES;
constexpr int A_INS = BM / (8 * NW), B_INS = CB / (8 * NW);
constexpr int NL = A_INS + B_INS + 1;  // glds per wave per step (+1: a 64-B piece of the biases)
constexpr int WH_OFF = 2 * STAGE;
constexpr int WH_BYTES = NH * ROWB * 2 * MAXBR;  // up to 6 64-channel blocks
constexpr int BH_OFF = WH_OFF + WH_BYTES;
constexpr int LDS_BYTES = BH_OFF + NH * 4;

struct NeckArgs {
  const __hip_bfloat16* x[MAXBR];  // branch inputs [B, H/s, W/s, ldx] (channels [offx, offx + cin))
  int ldx[MAXBR], offx[MAXBR], cin[MAXBR], s[MAXBR];
  const __hip_bfloat16* w[MAXBR];  // [s*s*CB, cin]: row (sy*s + sx)*CB + co
  const float* bias[MAXBR];        // [s*s*CB]
  const __hip_bfloat16* wh;        // [NH, nbr*CB], 32-chunk K-permuted
  const float* bh;                 // [NH]
  __hip_bfloat16* out;             // [B, H, W, ldo] (channels [0, nh))
  int ldo, nh;
  int B, H, W, S, nbr, nsteps, ntiles;
};

__device__ uint4 g_neck_zero_page[64];

typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* gbl_void_t;

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((gbl_void_t)g, (lds_void_t)l, 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ int swz2(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ bf16x8 pack8(const f32x4& lo, const f32x4& hi) {
  bf16x8 v;
  v[0] = (__bf16)lo[0]; v[1] = (__bf16)lo[1]; v[2] = (__bf16)lo[2]; v[3] = (__bf16)lo[3];
  v[4] = (__bf16)hi[0]; v[5] = (__bf16)hi[1]; v[6] = (__bf16)hi[2]; v[7] = (__bf16)hi[3];
  return v;
}

struct Tile {
  int b, cy, cx, q0;
};

__device__ __forceinline__ Tile tile_of(int S, int t, int nqt, int bm = BM) {
  const int ncls = S * S;
  const int cls = t % ncls, rest = t / ncls;
  Tile r;
  r.b = rest / nqt;
  r.q0 = (rest - r.b * nqt) * bm;
  r.cy = cls / S;
  r.cx = cls - r.cy * S;
  return r;
}

__global__ void __launch_bounds__(NT) bev_neck_head_kernel(NeckArgs a) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, lslot = lane & 7;

  const int S = a.S;
  const int Wq = a.W / S, nq = (a.H / S) * Wq;
  const int nqt = (nq + BM - 1) / BM;

  // this workgroup's tiles: XCD x gets the contiguous range [T*x/8, T*(x+1)/8),
  // walked by the XCD's G/8 workgroups with stride G/8
  const int G = gridDim.x, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = G >> 3;
  const int t_lo = (int)((long)a.ntiles * xcd / 8), t_hi = (int)((long)a.ntiles * (xcd + 1) / 8);
  const int my_tiles = t_lo + slot < t_hi ? (t_hi - t_lo - slot + nslot - 1) / nslot : 0;
  const int total = my_tiles * a.nsteps;

  // resident head weights (64-channel blocks [NH rows][128 B], swizzled) + head bias
  {
    const int nins = a.nbr * 2 * (NH / 8);
    const int ldw = a.nbr * CB;
    for (int ins = wid; ins < nins; ins += NW) {
      const int kb = ins / (NH / 8), r8 = ins - kb * (NH / 8);
      const int row = r8 * 8 + lrow;
      glds16(a.wh + (long)row * ldw + kb * 64 + (lslot ^ swz2(row)) * 8, smem + WH_OFF + kb * NH * ROWB + r8 * 1024);
    }
    if (wid == 0 && lane < NH / 4) glds16(a.bh + lane * 4, smem + BH_OFF);
  }

  // flat step g -> (tile, branch, chunk); the issue side walks it incrementally
  int i_k = 0, i_br = 0, i_kc = 0;
  Tile it = tile_of(a.S, t_lo + slot, nqt);
  auto issue = [&](int buf) {
    unsigned char* sa = smem + buf * STAGE;
    unsigned char* sb = sa + A_BYTES;
    unsigned char* sbias = sb + B_BYTES;
    const int s = a.s[i_br], f = S / s;
    const int Hi = a.H / s, Wi = a.W / s;
    const int sy = it.cy / s, sx = it.cx / s;
    const int ci0 = i_kc * 64;
    const __hip_bfloat16* xb = a.x[i_br] + a.offx[i_br] + ci0;
    const int ldx = a.ldx[i_br];
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int row = (wid * A_INS + j) * 8 + lrow;
      const int q = it.q0 + row;
      const void* g = g_neck_zero_page;
      if (q < nq) {
        const int Y = q / Wq, X = q - Y * Wq;
        g = xb + (((long)it.b * Hi + Y * f + sy) * Wi + X * f + sx) * ldx + (lslot ^ swz2(row)) * 8;
      }
      glds16(g, sa + (wid * A_INS + j) * 1024);
    }
    const int sub = (it.cy % s) * s + (it.cx % s);
    const __hip_bfloat16* wb = a.w[i_br] + (long)sub * CB * a.cin[i_br] + ci0;
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int row = (wid * B_INS + j) * 8 + lrow;
      glds16(wb + (long)row * a.cin[i_br] + (lslot ^ swz2(row)) * 8, sb + (wid * B_INS + j) * 1024);
    }
    // biases: wave w stages floats [16w, 16w + 16) with lanes 0..3
    if (lane < 4) glds16(a.bias[i_br] + sub * CB + wid * 16 + lane * 4, sbias + wid * 64);
    if (++i_kc * 64 == a.cin[i_br]) {
      i_kc = 0;
      if (++i_br == a.nbr) {
        i_br = 0;
        ++i_k;
        it = tile_of(a.S, t_lo + slot + i_k * nslot, nqt);
      }
    }
  };

  f32x4 acc1[2][8], acc2[2][NH / 16];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NH / 16; ++u) acc2[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  if (total > 0) issue(0);
  int c_k = 0, c_br = 0, c_kc = 0;  // compute side
  Tile ct = tile_of(a.S, t_lo + slot, nqt);
  for (int g = 0; g < total; ++g) {
    const int cur = g & 1;
    wait_vmcnt0();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage g landed for every wave; every wave is done with g-1's buffer
    asm volatile("" ::: "memory");
    if (g + 1 < total) issue(cur ^ 1);

    const unsigned char* sa = smem + cur * STAGE;
    const unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[2], bfg[8];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wid * 32 + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(sa + r * ROWB + (((ks * 4 + fq) ^ swz2(r)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = j * 16 + fr;
        bfg[j] = *reinterpret_cast<const bf16x8*>(sb + r * ROWB + (((ks * 4 + fq) ^ swz2(r)) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc1[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }

    if (++c_kc * 64 != a.cin[c_br]) continue;
    // ---- branch done: bias + ReLU, repack as operand fragments, head GEMM
    c_kc = 0;
    {
      const float* bias = reinterpret_cast<const float*>(sb + B_BYTES);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 bv = *reinterpret_cast<const float4*>(bias + j * 16 + fq * 4);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc1[i][j][0] = fmaxf(acc1[i][j][0] + bv.x, 0.f);
          acc1[i][j][1] = fmaxf(acc1[i][j][1] + bv.y, 0.f);
          acc1[i][j][2] = fmaxf(acc1[i][j][2] + bv.z, 0.f);
          acc1[i][j][3] = fmaxf(acc1[i][j][3] + bv.w, 0.f);
        }
      }
      const unsigned char* wh = smem + WH_OFF + c_br * 2 * NH * ROWB;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bf16x8 xf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) xf[i] = pack8(acc1[i][2 * t], acc1[i][2 * t + 1]);
        const unsigned char* whb = wh + (t >> 1) * NH * ROWB;
#pragma unroll
        for (int u = 0; u < NH / 16; ++u) {
          const int h = u * 16 + fr;
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(whb + h * ROWB + ((((t & 1) * 4 + fq) ^ swz2(h)) << 4));
#pragma unroll
          for (int i = 0; i < 2; ++i) acc2[i][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf[i], acc2[i][u], 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (++c_br != a.nbr) continue;
    // ---- tile done: head bias, bf16, store (lane: pixel fr, channels 16u + 4fq .. +3)
    c_br = 0;
    {
      const float* bh = reinterpret_cast<const float*>(smem + BH_OFF);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = ct.q0 + wid * 32 + i * 16 + fr;
        if (q < nq) {
          const int Y = q / Wq, X = q - Y * Wq;
          __hip_bfloat16* op = a.out + (((long)ct.b * a.H + Y * S + ct.cy) * a.W + X * S + ct.cx) * a.ldo;
#pragma unroll
          for (int u = 0; u < NH / 16; ++u) {
            const int h = u * 16 + fq * 4;
            if (h < a.nh) {
              const float4 bv = *reinterpret_cast<const float4*>(bh + h);
              __hip_bfloat16 o[4] = {__float2bfloat16(acc2[i][u][0] + bv.x), __float2bfloat16(acc2[i][u][1] + bv.y),
                                     __float2bfloat16(acc2[i][u][2] + bv.z), __float2bfloat16(acc2[i][u][3] + bv.w)};
              *reinterpret_cast<uint2*>(op + h) = *reinterpret_cast<uint2*>(o);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < NH / 16; ++u) acc2[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    ++c_k;
    ct = tile_of(a.S, t_lo + slot + c_k * nslot, nqt);
  }
  wait_vmcnt0();  // no LDS DMA may outlive the workgroup (a tile-less workgroup still loaded the head)
}

// ============================================================================
// fp32 mode ("x3", see conv_mfma.hip): fp32 branch inputs and output, split
// weights (deconv [s*s*CB, cin/8, {hi 8, lo 8}], head [NH, nbr*CB/8, {hi, lo}]
// with the same 32-chunk permutation), three MFMAs per fragment pair.  The
// split head weights (2 x 60 KiB) do not fit in LDS next to the fp32
// staging, so they are streamed through the ring instead: each branch's
// flat step sequence is its cin/32 deconv K steps followed by 2 head steps
// whose A slot carries the 80 x 64 split head weights of 64 of that branch's
// channels; the head GEMM consumes the branch's ReLU'd accumulators chunk by
// chunk (split to hi/lo in registers).
// LDS rows are 128 B; slot swizzle s ^ ((r ^ (r >> 3)) & 7) (conv_mfma.hip swz3).
// ============================================================================
// v2 tiling: 256 pixels per tile (32 per wave, two 16-pixel fragments), so
// every B fragment read from LDS feeds two fragment pairs; a 3-stage ring (two
// steps in flight, counted vmcnt, one barrier per step; LDS DMA from inline asm
// so hipcc inserts no vmcnt(0) in front of the fragment reads); tiles run over
// the flat (frame, pixel) index of a sub-pixel class, so no tile is cut short at
// a frame edge; each head step carries 64 of the branch's channels (two 32-channel
// chunks of split head weights in the stage's A slot).
constexpr int X_ROWB = 128;                       // 32 fp32 channels / 4 x {hi 8, lo 8}
// Tiling traits: NWV waves per workgroup (32 pixels each), STAGES-deep ring.
// <8, 3>: one 512-thread workgroup per CU; <4, 2>: two independent 256-thread
// workgroups per CU (66.5 KiB each), whose barriers do not line up, so one
// workgroup's MFMAs fill the other's barrier / LDS-latency bubbles.
template <int NWV, int STAGES, int FM_ = 2>
struct NeckX3 {
  static constexpr int NWAVES = NWV, NTH = NWV * 64;
  static constexpr int FM = FM_;                           // 16-pixel fragments per wave
  static constexpr int BM = 16 * FM * NWV;                 // pixels per tile
  static constexpr int A_BYTES = BM * X_ROWB;              // head steps: 2 x [80 rows][128 B]
  static constexpr int B_BYTES = CB * X_ROWB;              // 16 KiB
  static constexpr int STAGE = A_BYTES + B_BYTES + BIAS_BYTES;
  static constexpr int BH_OFF = STAGES * STAGE;
  static constexpr int LDS_BYTES = BH_OFF + NH * 4;
  static constexpr int A_INS = BM / (8 * NWV), B_INS = CB / (8 * NWV);
  static constexpr int BIAS_LANES = CB / 4 / NWV;          // 16-B bias pieces per wave
  static constexpr int DC_LOADS = A_INS + B_INS + 1;       // DMA instructions per wave per deconv step
  static constexpr int HEAD_PIECES = 2 * (NH / 8);         // 1-KiB DMA pieces per head step
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  static_assert(2 * NH * X_ROWB <= A_BYTES + B_BYTES, "a head step's weights fit the stage's A + B slots");
  static_assert(STAGES == 2 || STAGES == 3, "ring depth");
  __device__ static int head_loads(int wid) { return (HEAD_PIECES - wid + NWV - 1) / NWV; }
};
constexpr int Y_HEAD_STEPS = CB / 64;  // head steps per branch (64 channels each)

template <int V> struct IC { static constexpr int value = V; };

// 16-row periodic slot swizzle: conv_mfma.hip's swz3 on the row's position in
// its 16-row fragment (conflict-free for the b128 fragment reads at any 16-row
// base), so the fragment-read address is a per-lane base plus a constant per
// fragment (folded into the ds_read offset instead of one VGPR per fragment)
__device__ __forceinline__ int swz3(int row) { return ((row & 15) ^ ((row & 15) >> 3)) & 7; }

__device__ __forceinline__ void split8(const float4& x0, const float4& x1, bf16x8& hi, bf16x8& lo) {
  const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    hi[e] = h;
    lo[e] = (__bf16)(v[e] - (float)h);
  }
}

// max(x, 0) as ONE v_max_i32 on the bits (a negative float is a negative int; -0 -> +0): fmaxf in
// IEEE mode costs a canonicalizing v_max_f32 per input on top of the max
__device__ __forceinline__ float relu_bits(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

__device__ __forceinline__ void mfma3(f32x4& acc, const bf16x8& bh, const bf16x8& bl, const bf16x8& ah,
                                      const bf16x8& al) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc, 0, 0, 0);
}

constexpr unsigned kOutOfRange = 0x80000000u;  // >= any num_records the launcher accepts (< 2^31): reads zeros

// one 16-B-per-lane LDS DMA through a buffer resource: voffset per lane, soffset scalar
__device__ __forceinline__ void bdma16(unsigned voff, __amdgpu_buffer_rsrc_t rsrc, const void* l, unsigned soff) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}
// all but this wave's n youngest vector-memory ops done (n = the DMA pieces of
// the one step allowed to stay in flight; an unlisted n waits for everything)
template <typename T>
__device__ __forceinline__ void wait_vm_rt(int n) {
  constexpr int H_HI = (T::HEAD_PIECES + T::NWAVES - 1) / T::NWAVES, H_LO = T::HEAD_PIECES / T::NWAVES;
  if (n == T::DC_LOADS) wait_vm<T::DC_LOADS>();
  else if (n == H_HI) wait_vm<H_HI>();
  else if (n == H_LO) wait_vm<H_LO>();
  else wait_vm<0>();
}

struct NeckArgsX3 {
  const float* x[MAXBR];
  int ldx[MAXBR], offx[MAXBR], cin[MAXBR], s[MAXBR];
  const __hip_bfloat16* w[MAXBR];  // split [s*s*CB, 2*cin]
  const float* bias[MAXBR];
  const __hip_bfloat16* wh;        // split [NH, 2*nbr*CB], 32-chunk permuted
  const float* bh;
  float* out;
  int ldo, nh;
  int B, H, W, S, nbr, nsteps, ntiles;
};

// PAIR: branch inputs in pair storage ({hi 8 | lo 8} per 8 channels, see
// conv_mfma.hip pair_split8): the A fragments are read as stored, no split.
template <bool PAIR, int NWV, int STAGES, int FM_ = 2>
__global__ void __launch_bounds__(NWV * 64, NWV == 4 ? 2 : 1) bev_neck_head_x3_kernel(NeckArgsX3 a) {
  using T = NeckX3<NWV, STAGES, FM_>;
  constexpr int Y_BM = T::BM, Y_FM = T::FM, Y_STAGES = STAGES, Y_STAGE = T::STAGE, Y_A_BYTES = T::A_BYTES;
  constexpr int Y_B_BYTES = T::B_BYTES, Y_BH_OFF = T::BH_OFF, Y_A_INS = T::A_INS, Y_B_INS = T::B_INS;
  constexpr int Y_DC_LOADS = T::DC_LOADS, Y_HEAD_PIECES = T::HEAD_PIECES, NW = NWV;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[T::LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int lrow = lane >> 3, lslot = lane & 7;

  const int S = a.S, ncls = S * S;
  const int Wq = a.W / S, nq = (a.H / S) * Wq;
  const int np = a.B * nq;  // pixels of one sub-pixel class over the batch
  const int G = gridDim.x, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = G >> 3;
  const int t_lo = (int)((long)a.ntiles * xcd / 8), t_hi = (int)((long)a.ntiles * (xcd + 1) / 8);
  const int my_tiles = t_lo + slot < t_hi ? (t_hi - t_lo - slot + nslot - 1) / nslot : 0;
  const int total = my_tiles * a.nsteps;
  const int ldwh = 2 * a.nbr * CB;  // bf16 per split head-weight row

  if (wid == 0 && lane < NH / 4) glds16_asm(a.bh + lane * 4, smem + Y_BH_OFF);

  // ---- issue side: (tile, branch, chunk); chunk < cin/32 a deconv step, else a head step
  int i_k = 0, i_br = 0, i_kc = 0, i_cy = 0, i_cx = 0;
  // this lane's A rows of the issue-side tile: (global q-row Yg = b * H/S + Y) << 16 | X, or -1.
  // A branch of stride s reads input pixel (Yg * S/s + sy, X * S/s + sx) of its [B * H/s, W/s] map.
  int r_yx[Y_A_INS];
  auto tile_rows = [&](int t) {
    const int cls = t % ncls, pt = t / ncls;
    i_cy = cls / S;
    i_cx = cls - i_cy * S;
#pragma unroll
    for (int j = 0; j < Y_A_INS; ++j) {
      const int p = pt * Y_BM + (wid * Y_A_INS + j) * 8 + lrow;
      r_yx[j] = -1;
      if (p < np) {
        const int yg = p / Wq;
        r_yx[j] = (yg << 16) | (p - yg * Wq);
      }
    }
  };
  // LDS DMA through buffer resources (conv_mfma.hip "xb"): every lane's 32-bit byte offset
  // of a DMA is formed once per (tile, branch) -- A rows, B rows, bias -- or once per kernel
  // (head weight pieces); a K step only advances the scalar soffset, so the K loop's DMA
  // issue needs no VALU.  A row outside the image is offset kOutOfRange: the descriptor's
  // range check reads zeros.
  unsigned a_vo[Y_A_INS], b_vo[Y_B_INS], bias_vo = 0;
  __amdgpu_buffer_rsrc_t rs_a = __builtin_amdgcn_make_buffer_rsrc((void*)a.x[0], (short)0, 0, 0x00020000);
  __amdgpu_buffer_rsrc_t rs_w = rs_a, rs_bias = rs_a;
  auto row_sources = [&]() {  // once per (tile, branch): the K steps only add their channel offset
    const int s = a.s[i_br], f = S / s;
    const int Hi = a.H / s, Wi = a.W / s;
    const int sy = i_cy / s, sx = i_cx / s;
    const int ldx = a.ldx[i_br], cin = a.cin[i_br];
    rs_a = __builtin_amdgcn_make_buffer_rsrc((void*)a.x[i_br], (short)0, a.B * Hi * Wi * ldx * 4, 0x00020000);
    rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)a.w[i_br], (short)0, s * s * CB * cin * 4, 0x00020000);
    rs_bias = __builtin_amdgcn_make_buffer_rsrc((void*)a.bias[i_br], (short)0, s * s * CB * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < Y_A_INS; ++j) {
      const int row = (wid * Y_A_INS + j) * 8 + lrow;
      const int yg = r_yx[j] >> 16, x = r_yx[j] & 0xFFFF;
      a_vo[j] = r_yx[j] < 0 ? kOutOfRange
                            : (unsigned)((((yg * f + sy) * Wi + x * f + sx) * ldx + a.offx[i_br] +
                                          (lslot ^ swz3(row)) * 4) * 4);
    }
    const int sub = (i_cy % s) * s + (i_cx % s);
#pragma unroll
    for (int j = 0; j < Y_B_INS; ++j) {
      const int row = (wid * Y_B_INS + j) * 8 + lrow;
      b_vo[j] = (unsigned)(((sub * CB + row) * 2 * cin + (lslot ^ swz3(row)) * 8) * 2);
    }
    bias_vo = (unsigned)((sub * CB + wid * (4 * T::BIAS_LANES) + lane * 4) * 4);
  };
  // head weight pieces of this wave (p = wid + k * NW): per-lane byte offsets, fixed for the kernel
  constexpr int HP_MAX = (Y_HEAD_PIECES + NW - 1) / NW;
  unsigned h_vo[HP_MAX];
  int h_lds[HP_MAX];
#pragma unroll
  for (int k = 0; k < HP_MAX; ++k) {
    const int p = wid + k * NW;
    const int c = p / (NH / 8), r8 = p - c * (NH / 8), h = r8 * 8 + lrow;
    h_vo[k] = (unsigned)((h * ldwh + c * 64 + (lslot ^ swz3(h)) * 8) * 2);
    h_lds[k] = p < Y_HEAD_PIECES ? c * NH * X_ROWB + r8 * 1024 : -1;
  }
  const __amdgpu_buffer_rsrc_t rs_wh = __builtin_amdgcn_make_buffer_rsrc((void*)a.wh, (short)0, NH * ldwh * 2, 0x00020000);
  auto issue = [&](int buf) -> int {
    unsigned char* sa = smem + buf * Y_STAGE;
    unsigned char* sb = sa + Y_A_BYTES;
    unsigned char* sbias = sb + Y_B_BYTES;
    const int nkc = a.cin[i_br] / 32;
    int n = 0;
    if (i_kc < nkc) {
      if (i_kc == 0) row_sources();
      const unsigned so = (unsigned)(i_kc * 32 * 4);  // fp32 inputs and split weights: 4 B per channel
#pragma unroll
      for (int j = 0; j < Y_A_INS; ++j) bdma16(a_vo[j], rs_a, sa + (wid * Y_A_INS + j) * 1024, so);
#pragma unroll
      for (int j = 0; j < Y_B_INS; ++j) bdma16(b_vo[j], rs_w, sb + (wid * Y_B_INS + j) * 1024, so);
      if (lane < T::BIAS_LANES) bdma16(bias_vo, rs_bias, sbias + wid * (16 * T::BIAS_LANES), 0u);
      n = Y_DC_LOADS;
    } else {
      // head step t: rows h < 80 of the split head weights, channels [br*CB + 64t, +64)
      // as two 32-channel blocks [80][128 B] in the A slot
      const int t = i_kc - nkc;
      const unsigned so = (unsigned)((i_br * CB + 64 * t) * 2 * 2);
#pragma unroll
      for (int k = 0; k < HP_MAX; ++k)
        if (h_lds[k] >= 0) {  // wave-uniform
          bdma16(h_vo[k], rs_wh, sa + h_lds[k], so);
          ++n;
        }
    }
    if (++i_kc == nkc + Y_HEAD_STEPS) {
      i_kc = 0;
      if (++i_br == a.nbr) {
        i_br = 0;
        if (++i_k < my_tiles) tile_rows(t_lo + slot + i_k * nslot);
      }
    }
    return n;
  };

  f32x4 acc1[Y_FM][8], acc2[Y_FM][NH / 16];
#pragma unroll
  for (int i = 0; i < Y_FM; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NH / 16; ++u) acc2[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  int nxt = 0;  // 3 stages: DMA pieces of the step after the current one (0: not issued)
  if (total > 0) {
    tile_rows(t_lo + slot);
    issue(0);
    if (Y_STAGES == 3 && total > 1) nxt = issue(1);
  }
  // compute side: nested loops (tile -> branch -> deconv K steps, head steps), each with
  // one latch, so the accumulators stay in fixed registers (a flat step state machine
  // made hipcc copy every accumulator back at each of its loop latches); the DMA side
  // walks the same flat sequence one step ahead through begin_step()
  int g = 0;
  auto begin_step = [&]() -> const unsigned char* {
    const int cur = g % Y_STAGES;
    if constexpr (Y_STAGES == 3) wait_vm_rt<T>(nxt);
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // step g landed for every wave; every wave is done with step g-1's buffer
    asm volatile("" ::: "memory");
    if (g + Y_STAGES - 1 < total) {
      const int n = issue((g + Y_STAGES - 1) % Y_STAGES);
      if constexpr (Y_STAGES == 3) nxt = n;
    } else {
      nxt = 0;
    }
    ++g;
    return smem + cur * Y_STAGE;
  };
  auto head_chunk = [&](auto QC, const unsigned char* whb) {
    constexpr int q = decltype(QC)::value;  // static register indices (a runtime index would spill acc1)
    bf16x8 xh[Y_FM], xl[Y_FM];
#pragma unroll
    for (int i = 0; i < Y_FM; ++i) {
      const f32x4 p0 = acc1[i][2 * q], p1 = acc1[i][2 * q + 1];  // ReLU'd here, chunk by chunk
      split8(make_float4(relu_bits(p0[0]), relu_bits(p0[1]), relu_bits(p0[2]), relu_bits(p0[3])),
             make_float4(relu_bits(p1[0]), relu_bits(p1[1]), relu_bits(p1[2]), relu_bits(p1[3])), xh[i], xl[i]);
    }
#pragma unroll
    for (int u = 0; u < NH / 16; ++u) {
      const int h = u * 16 + fr;
      const bf16x8 wh_ = *reinterpret_cast<const bf16x8*>(whb + h * X_ROWB + (((2 * fq) ^ swz3(h)) << 4));
      const bf16x8 wl_ = *reinterpret_cast<const bf16x8*>(whb + h * X_ROWB + (((2 * fq + 1) ^ swz3(h)) << 4));
#pragma unroll
      for (int i = 0; i < Y_FM; ++i) mfma3(acc2[i][u], wh_, wl_, xh[i], xl[i]);
    }
  };
  for (int c_k = 0; c_k < my_tiles; ++c_k) {
    for (int c_br = 0; c_br < a.nbr; ++c_br) {
      const int nkc = a.cin[c_br] / 32;
      for (int c_kc = 0; c_kc < nkc; ++c_kc) {
        // ---- deconv K step: 2 x 8 fragment pairs, three MFMAs each
        const unsigned char* sa = begin_step();
        const unsigned char* sb = sa + Y_A_BYTES;
        if (c_kc == 0) {  // the branch's accumulators start at its deconv bias (staged with every K step)
          const float* bias = reinterpret_cast<const float*>(sb + Y_B_BYTES);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float4 bv = *reinterpret_cast<const float4*>(bias + j * 16 + fq * 4);
#pragma unroll
            for (int i = 0; i < Y_FM; ++i) acc1[i][j] = f32x4{bv.x, bv.y, bv.z, bv.w};
          }
        }
        bf16x8 ah[Y_FM], al[Y_FM];
#pragma unroll
        for (int i = 0; i < Y_FM; ++i) {
          const int r = wid * 16 * Y_FM + i * 16 + fr;
          if constexpr (PAIR) {
            ah[i] = *reinterpret_cast<const bf16x8*>(sa + r * X_ROWB + (((2 * fq) ^ swz3(r)) << 4));
            al[i] = *reinterpret_cast<const bf16x8*>(sa + r * X_ROWB + (((2 * fq + 1) ^ swz3(r)) << 4));
          } else {
            const float4 x0 = *reinterpret_cast<const float4*>(sa + r * X_ROWB + (((2 * fq) ^ swz3(r)) << 4));
            const float4 x1 = *reinterpret_cast<const float4*>(sa + r * X_ROWB + (((2 * fq + 1) ^ swz3(r)) << 4));
            split8(x0, x1, ah[i], al[i]);
          }
        }
        __builtin_amdgcn_s_setprio(1);
        // B fragments in groups of JB: keeps the hoisted LDS reads (and so the VGPRs) to part of the tile
        constexpr int JB = Y_FM >= 4 ? 2 : 4;
#pragma unroll
        for (int jh = 0; jh < 8 / JB; ++jh) {
          bf16x8 wh_[JB], wl_[JB];
#pragma unroll
          for (int jj = 0; jj < JB; ++jj) {
            const int r = (jh * JB + jj) * 16 + fr;
            wh_[jj] = *reinterpret_cast<const bf16x8*>(sb + r * X_ROWB + (((2 * fq) ^ swz3(r)) << 4));
            wl_[jj] = *reinterpret_cast<const bf16x8*>(sb + r * X_ROWB + (((2 * fq + 1) ^ swz3(r)) << 4));
          }
#pragma unroll
          for (int jj = 0; jj < JB; ++jj)
#pragma unroll
            for (int i = 0; i < Y_FM; ++i) mfma3(acc1[i][jh * JB + jj], wh_[jj], wl_[jj], ah[i], al[i]);
          __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
      // branch GEMM done (its bias was the accumulators' start); the head chunks apply the ReLU
      // ---- head steps: branch channels 64t..64t+63 (acc1[.][4t .. 4t+3]) x 80 head rows
      static_assert(Y_HEAD_STEPS == 2, "head steps unrolled below");
      {
        const unsigned char* sa = begin_step();
        __builtin_amdgcn_s_setprio(1);
        head_chunk(IC<0>{}, sa);
        __builtin_amdgcn_sched_barrier(0);
        head_chunk(IC<1>{}, sa + NH * X_ROWB);
        __builtin_amdgcn_s_setprio(0);
      }
      {
        const unsigned char* sa = begin_step();
        __builtin_amdgcn_s_setprio(1);
        head_chunk(IC<2>{}, sa);
        __builtin_amdgcn_sched_barrier(0);
        head_chunk(IC<3>{}, sa + NH * X_ROWB);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    {  // ---- tile done: head bias, fp32 store (lane: pixel fr, head rows 16u + 4fq .. +3)
      const int ct = t_lo + slot + c_k * nslot;
      const int cls = ct % ncls, pt = ct / ncls, cy = cls / S, cx = cls - cy * S;
      // lane's head-bias LDS offset, formed here (the opaque copy keeps hipcc from
      // hoisting the five per-u addresses out of the step loop, where they spill)
      int bofs = Y_BH_OFF + fq * 16;
      asm volatile("" : "+v"(bofs));
      const unsigned char* bh = smem + bofs;
#pragma unroll
      for (int i = 0; i < Y_FM; ++i) {
        const int p = pt * Y_BM + wid * 16 * Y_FM + i * 16 + fr;
        if (p < np) {
          const int b = p / nq, q = p - b * nq, Y = q / Wq, X = q - Y * Wq;
          float* op = a.out + (((long)b * a.H + Y * S + cy) * a.W + X * S + cx) * a.ldo;
#pragma unroll
          for (int u = 0; u < NH / 16; ++u) {
            const int h = u * 16 + fq * 4;
            if (h < a.nh) {
              const float4 bv = *reinterpret_cast<const float4*>(bh + u * 64);
              *reinterpret_cast<float4*>(op + h) = make_float4(acc2[i][u][0] + bv.x, acc2[i][u][1] + bv.y,
                                                               acc2[i][u][2] + bv.z, acc2[i][u][3] + bv.w);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < NH / 16; ++u) acc2[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  wait_vm<0>();  // no LDS DMA may outlive the workgroup (a tile-less workgroup still loaded the head bias)
}

}  // namespace

// Branch i: input x[i] [B, H/s_i, W/s_i, ldx[i]] channels [offx[i], offx[i]+cin[i]),
// weights w[i] [s_i*s_i*128, cin[i]] (FusedConv's transpose-conv GEMM layout),
// bias[i] [s_i*s_i*128].  wh: [80, nbr*128] head weights, 32-chunk permuted
// (see the header comment); bh [80].  out: [B, H, W, ldo], channels [0, nh).
// grid: workgroups to launch (a multiple of 8; one per CU is the design point).
TCA_API int tca_bev_neck_head(int nbr, const void* const* x, const int* ldx, const int* offx, const int* cin,
                              const int* s, const void* const* w, const float* const* bias, const void* wh,
                              const float* bh, int nh, void* out, int ldo, int B, int H, int W, int grid,
                              hipStream_t stream) {
  if (B <= 0) return 0;
  if (nbr < 1 || nbr > MAXBR || nh <= 0 || nh > NH || (nh & 3) || (ldo & 3) || grid < 8 || (grid & 7))
    return (int)hipErrorInvalidValue;
  NeckArgs a;
  int S = 1, nsteps = 0;
  for (int i = 0; i < nbr; ++i) {
    if (s[i] < 1 || (cin[i] & 63) || (ldx[i] & 7) || (offx[i] & 7)) return (int)hipErrorInvalidValue;
    S = s[i] > S ? s[i] : S;
  }
  for (int i = 0; i < nbr; ++i) {
    if (S % s[i]) return (int)hipErrorInvalidValue;
    a.x[i] = (const __hip_bfloat16*)x[i]; a.ldx[i] = ldx[i]; a.offx[i] = offx[i]; a.cin[i] = cin[i]; a.s[i] = s[i];
    a.w[i] = (const __hip_bfloat16*)w[i]; a.bias[i] = bias[i];
    nsteps += cin[i] / 64;
  }
  for (int i = nbr; i < MAXBR; ++i) {
    a.x[i] = nullptr; a.ldx[i] = a.offx[i] = a.cin[i] = 0; a.s[i] = 1; a.w[i] = nullptr; a.bias[i] = nullptr;
  }
  if ((H % S) || (W % S)) return (int)hipErrorInvalidValue;
  a.wh = (const __hip_bfloat16*)wh; a.bh = bh; a.out = (__hip_bfloat16*)out; a.ldo = ldo; a.nh = nh;
  a.B = B; a.H = H; a.W = W; a.S = S; a.nbr = nbr; a.nsteps = nsteps;
  const int nq = (H / S) * (W / S);
  a.ntiles = B * ((nq + BM - 1) / BM) * S * S;
  bev_neck_head_kernel<<<grid, NT, 0, stream>>>(a);
  TCA_LAUNCH_CHECK();
}

// fp32 mode: x[i] fp32, w[i] split [s_i*s_i*128, 2*cin[i]] bf16, wh split [80, 2*nbr*128]
// (32-chunk permuted, then split), out fp32 [B, H, W, ldo].  Other arguments as tca_bev_neck_head.
namespace {
// tiling: <8 waves, 2 stages>, one workgroup per CU.  Measured at batch 32 on MI355X against <8, 3>,
// <4, 2> (two per CU) and the 64-pixel-wave <4, 3, FM 4> / <4, 2, FM 4>: 1008 us vs 1192-1483
// (profiles/r4/neck_variants.jsonl, profiles/r2/neck_variants.json); the others were removed.
template <int NWV, int STAGES, int FM = 2>
void launch_neck_x3(NeckArgsX3& a, long np, int grid, bool pair, hipStream_t stream) {
  using T = NeckX3<NWV, STAGES, FM>;
  a.ntiles = (int)((np + T::BM - 1) / T::BM) * a.S * a.S;
  if (pair) bev_neck_head_x3_kernel<true, NWV, STAGES, FM><<<grid, T::NTH, 0, stream>>>(a);
  else bev_neck_head_x3_kernel<false, NWV, STAGES, FM><<<grid, T::NTH, 0, stream>>>(a);
}

int neck_x3(int nbr, const void* const* x, const int* ldx, const int* offx, const int* cin, const int* s,
            const void* const* w, const float* const* bias, const void* wh, const float* bh, int nh, void* out,
            int ldo, int B, int H, int W, int grid, bool pair, int variant, hipStream_t stream) {
  if (B <= 0) return 0;
  if (nbr < 1 || nbr > MAXBR || nh <= 0 || nh > NH || (nh & 3) || (ldo & 3) || grid < 8 || (grid & 7))
    return (int)hipErrorInvalidValue;
  // 0: <8 waves, 2 stages>; 1: <8, 3> (two K steps in flight); 2: <4, 2>, 128-pixel tiles, two
  // workgroups per CU (66 KiB LDS and <= 256 VGPRs each; the grid doubles)
  if (variant < 0 || variant > 2) return (int)hipErrorInvalidValue;
  NeckArgsX3 a;
  int S = 1, nsteps = 0;
  for (int i = 0; i < nbr; ++i) {
    if (s[i] < 1 || (cin[i] & 31) || (ldx[i] & 3) || (offx[i] & 3)) return (int)hipErrorInvalidValue;
    S = s[i] > S ? s[i] : S;
  }
  for (int i = 0; i < nbr; ++i) {
    if (S % s[i]) return (int)hipErrorInvalidValue;
    a.x[i] = (const float*)x[i]; a.ldx[i] = ldx[i]; a.offx[i] = offx[i]; a.cin[i] = cin[i]; a.s[i] = s[i];
    a.w[i] = (const __hip_bfloat16*)w[i]; a.bias[i] = bias[i];
    nsteps += cin[i] / 32 + Y_HEAD_STEPS;
  }
  for (int i = nbr; i < MAXBR; ++i) {
    a.x[i] = nullptr; a.ldx[i] = a.offx[i] = a.cin[i] = 0; a.s[i] = 1; a.w[i] = nullptr; a.bias[i] = nullptr;
  }
  if ((H % S) || (W % S)) return (int)hipErrorInvalidValue;
  // the kernel packs q-grid rows as (Yg << 16 | X) and reads branch inputs / weights through buffer
  // resources with 32-bit byte offsets (< kOutOfRange): batches whose inputs exceed that run in chunks
  if (W / S >= 65536 || (long)NH * 2 * nbr * CB * 2 >= (1L << 31)) return (int)hipErrorInvalidValue;
  long per_frame_max = 0;
  for (int i = 0; i < nbr; ++i) {
    const long fb = (long)(H / s[i]) * (W / s[i]) * ldx[i] * 4;
    per_frame_max = fb > per_frame_max ? fb : per_frame_max;
    if ((long)s[i] * s[i] * CB * cin[i] * 4 >= (1L << 31)) return (int)hipErrorInvalidValue;
  }
  int chunk = (int)(((1L << 31) - 1) / per_frame_max);
  if ((long)(H / S) * chunk >= 32768) chunk = 32767 / (H / S);
  if (chunk < 1) return (int)hipErrorInvalidValue;
  a.wh = (const __hip_bfloat16*)wh; a.bh = bh; a.ldo = ldo; a.nh = nh;
  a.H = H; a.W = W; a.S = S; a.nbr = nbr; a.nsteps = nsteps;
  const int nq = (H / S) * (W / S);
  if (pair)
    for (int i = 0; i < nbr; ++i)
      if ((ldx[i] & 7) || (offx[i] & 7)) return (int)hipErrorInvalidValue;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nb = B - b0 < chunk ? B - b0 : chunk;
    for (int i = 0; i < nbr; ++i) a.x[i] = (const float*)x[i] + (long)b0 * (H / s[i]) * (W / s[i]) * ldx[i];
    a.out = (float*)out + (long)b0 * H * W * ldo;
    a.B = nb;
    // grid: workgroup slots of the persistent kernel, one per CU
    if (variant == 1) launch_neck_x3<8, 3>(a, (long)nb * nq, grid, pair, stream);
    else if (variant == 2) launch_neck_x3<4, 2>(a, (long)nb * nq, 2 * grid, pair, stream);
    else launch_neck_x3<8, 2>(a, (long)nb * nq, grid, pair, stream);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
}  // namespace

TCA_API int tca_bev_neck_head_x3(int nbr, const void* const* x, const int* ldx, const int* offx, const int* cin,
                                 const int* s, const void* const* w, const float* const* bias, const void* wh,
                                 const float* bh, int nh, void* out, int ldo, int B, int H, int W, int grid,
                                 hipStream_t stream) {
  return neck_x3(nbr, x, ldx, offx, cin, s, w, bias, wh, bh, nh, out, ldo, B, H, W, grid, false, 0, stream);
}

// Same, branch inputs x[i] in pair storage.
TCA_API int tca_bev_neck_head_x3p(int nbr, const void* const* x, const int* ldx, const int* offx, const int* cin,
                                  const int* s, const void* const* w, const float* const* bias, const void* wh,
                                  const float* bh, int nh, void* out, int ldo, int B, int H, int W, int grid,
                                  hipStream_t stream) {
  return neck_x3(nbr, x, ldx, offx, cin, s, w, bias, wh, bh, nh, out, ldo, B, H, W, grid, true, 0, stream);
}

// Same with the input storage as an argument (pair != 0: pair storage); variant: 0 (the one tiling,
// also accepted as 3, its former number).
TCA_API int tca_bev_neck_head_x3v(int nbr, const void* const* x, const int* ldx, const int* offx, const int* cin,
                                  const int* s, const void* const* w, const float* const* bias, const void* wh,
                                  const float* bh, int nh, void* out, int ldo, int B, int H, int W, int grid,
                                  int pair, int variant, hipStream_t stream) {
  return neck_x3(nbr, x, ldx, offx, cin, s, w, bias, wh, bh, nh, out, ldo, B, H, W, grid, pair != 0, variant,
                 stream);
}
