// K3' — YOLOv5 Detect head (the three 1x1 convs, fp32 mode) fused with the decode + candidate
// filter of yolo.hip (reference: clients/postprocess/yolov5_postprocess.py:36-92, the Detect
// layer of the exported ONNX model; see yolo.hip K3 for the filter semantics).
//
// Unfused, the head convs write [B, H, W, 256] fp32 maps (262 MB at batch 32 for the three
// levels, ~80% of it the 80 x 80 level) and the filter reads them back.  Here one workgroup owns
// 64 pixels of one image and level: the input pixels are split once into bf16 hi / lo planes in
// LDS, the 4 waves each compute 64 of the 256 head channels with the split-product MFMA
// (bf16 x3, fp32 accumulation) in the K order, fragment layout and product order of conv_mfma.hip
// conv_xb_kernel (so the logits are bit-identical to the unfused conv's output), the logits
// (+ bias) go to LDS, and one thread per (pixel, anchor) runs yolo.hip's filter on them.  Only
// the candidates leave the kernel.
#include "tca_common.h"

using namespace tca;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TP = 64;         // pixels per workgroup
constexpr int NCH = 256;       // head channels (na * (5 + nc) <= 256)
constexpr int MAXC = 256;      // input channels
constexpr int LDL = NCH + 4;   // logit row stride (floats)
constexpr int PLANE = (MAXC / 8) * TP * 16;  // one split plane: [C/8][64 px][8 bf16]
constexpr int LDS_BYTES = (2 * PLANE > TP * LDL * 4) ? 2 * PLANE : TP * LDL * 4;

struct DetLevel {
  const float* x;       // fp32 NHWC [B, H, W, ldx], channels [x_off, x_off + cin)
  const __bf16* w;      // split_pairs image [256, 2 * cin] (conv_mfma.hip weight layout)
  const float* bias;    // [256]
  int ldx, x_off, cin, H, W, stride, tiles;  // tiles per image
  float anchor[4][2];
};

struct DetArgs {
  DetLevel lv[3];
  int B, na, nc, cap;
  float conf_thres;
  const uint32_t* class_mask;
  float* cand_box;
  float* cand_score;
  int* cand_cls;
  uint64_t* cand_key;
  int* cand_count;
};

// byte offset of (channel group c8, pixel px) in a split plane: pixel XOR-swizzled by c8 within its
// 16-pixel group, so the staging writes (8 lanes = 8 groups of one pixel) and the fragment reads
// (16 lanes = 16 pixels of one group) are both bank-conflict free
__device__ __forceinline__ int slot(int c8, int px) { return (c8 * TP + (px ^ (c8 & 15))) * 16; }

// stage the 64 input pixels (split planes) and run the head GEMM: CIN known at compile time, so
// every staging load of a lane is in flight at once and the weight fragments of K step kt + 1 are
// loaded while step kt's MFMAs run
template <int CIN>
__device__ __forceinline__ void det_gemm(const DetLevel& L, int b, int p0, int HW, unsigned char* smem,
                                         f32x4 (&acc)[4][4]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  unsigned char* const hp = smem;
  unsigned char* const lp = smem + PLANE;
  // ---- stage: 64 pixels x CIN fp32 -> hi / lo planes [CIN / 8][64][8] bf16 (zeros past HW);
  // 8 lanes per pixel at CIN 64: coalesced 256-B row reads
  constexpr int N8 = CIN / 8, IT = TP * N8 / 256;
  float4 xv[IT][2];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int id = tid + u * 256, px = id / N8, c8 = id % N8;
    xv[u][0] = xv[u][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p0 + px < HW) {
      const float* src = L.x + ((long)b * HW + p0 + px) * L.ldx + L.x_off + c8 * 8;
      xv[u][0] = *reinterpret_cast<const float4*>(src);
      xv[u][1] = *reinterpret_cast<const float4*>(src + 4);
    }
  }
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int id = tid + u * 256, px = id / N8, c8 = id % N8;
    const float v[8] = {xv[u][0].x, xv[u][0].y, xv[u][0].z, xv[u][0].w,
                        xv[u][1].x, xv[u][1].y, xv[u][1].z, xv[u][1].w};
    bf16x8 h, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // conv_mfma.hip split8
      const __bf16 hb = (__bf16)v[e];
      h[e] = hb;
      lo[e] = (__bf16)(v[e] - (float)hb);
    }
    *reinterpret_cast<bf16x8*>(hp + slot(c8, px)) = h;
    *reinterpret_cast<bf16x8*>(lp + slot(c8, px)) = lo;
  }
  // weights of K step 0 while the staging lands
  const __bf16* wrow = L.w + (long)(wid * 64 + fr) * 2 * CIN + fq * 16;
  bf16x8 wb[2][4][2];
  auto wload = [&](int kt, bf16x8 (&dst)[4][2]) {  // row n = 64 wid + 16 j + fr, K group 4 kt + fq
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const __bf16* p = wrow + (long)j * 16 * 2 * CIN + kt * 64;
      dst[j][0] = *reinterpret_cast<const bf16x8*>(p);
      dst[j][1] = *reinterpret_cast<const bf16x8*>(p + 8);
    }
  };
  wload(0, wb[0]);
  __syncthreads();

  // ---- GEMM: wave wid owns channels [64 wid, 64 wid + 64): 4 x 4 fragments of 16 x 16
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int NK = CIN / 32;
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) {
    bf16x8 (&w)[4][2] = wb[kt & 1];
    if (kt + 1 < NK) wload(kt + 1, wb[(kt + 1) & 1]);
    const int c8 = kt * 4 + fq;
    bf16x8 ah[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(hp + slot(c8, i * 16 + fr));
      al[i] = *reinterpret_cast<const bf16x8*>(lp + slot(c8, i * 16 + fr));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // conv_mfma.hip mfma3 order
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][1], ah[i], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][0], al[i], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][0], ah[i], acc[i][j], 0, 0, 0);
      }
  }
}

__global__ void __launch_bounds__(256, 2) yolo_detect_filter_kernel(DetArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __shared__ int s_cnt, s_base;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  // heaviest level (largest cin, the 20 x 20 one) first: blocks 0.. walk levels 2, 1, 0
  int t = blockIdx.x, l = 2;
  while (l > 0 && t >= a.B * a.lv[l].tiles) { t -= a.B * a.lv[l].tiles; --l; }
  const DetLevel& L = a.lv[l];
  const int b = t / L.tiles, p0 = (t - b * L.tiles) * TP;
  const int HW = L.H * L.W;
  if (tid == 0) s_cnt = 0;

  f32x4 acc[4][4];
  switch (L.cin) {  // block-uniform; the host admits only these
    case 64: det_gemm<64>(L, b, p0, HW, smem, acc); break;
    case 128: det_gemm<128>(L, b, p0, HW, smem, acc); break;
    default: det_gemm<256>(L, b, p0, HW, smem, acc); break;
  }
  __syncthreads();  // every wave done with the planes: the logits overlay them

  // ---- logits (+ bias, as conv_mfma.hip epilogue_f32) -> LDS [64 px][LDL]
  float* lg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = wid * 64 + j * 16 + fq * 4;
    const float4 bv = *reinterpret_cast<const float4*>(L.bias + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int px = i * 16 + fr;
      *reinterpret_cast<float4*>(lg + px * LDL + n) =
          make_float4(acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w);
    }
  }
  __syncthreads();

  // ---- filter (yolo.hip yolo_filter_kernel, single-label): thread = (anchor, pixel)
  const int no = a.nc + 5;
  const int px = tid & (TP - 1), an = tid / TP;
  const int yx = p0 + px;
  bool pass = false;
  float box[4] = {0.f, 0.f, 0.f, 0.f}, best = -1.f;
  int best_c = 0, aidx = 0;
  if (an < a.na && yx < HW) {
    int off = 0;
    for (int q = 0; q < l; ++q) off += a.na * a.lv[q].H * a.lv[q].W;
    aidx = off + an * HW + yx;
    const float* row = lg + px * LDL + an * no;
    const float obj = sigmoidf_(row[4]);
    if (obj > a.conf_thres) {
      const int y = yx / L.W, x = yx - (yx / L.W) * L.W;
      const float sx = sigmoidf_(row[0]), sy = sigmoidf_(row[1]);
      const float sw = sigmoidf_(row[2]), sh = sigmoidf_(row[3]);
      const float st = (float)L.stride;
      const float cx = (sx * 2.f - 0.5f + (float)x) * st;
      const float cy = (sy * 2.f - 0.5f + (float)y) * st;
      const float bw = (sw * 2.f) * (sw * 2.f) * L.anchor[an][0];
      const float bh = (sh * 2.f) * (sh * 2.f) * L.anchor[an][1];
      box[0] = cx - bw * 0.5f; box[1] = cy - bh * 0.5f; box[2] = cx + bw * 0.5f; box[3] = cy + bh * 0.5f;
      float m = -INFINITY;
      int mc = 0;
      for (int c = 0; c < a.nc; ++c) {  // best over all classes, then the class filter (reference order)
        const float v = row[5 + c];
        if (v > m) { m = v; mc = c; }
      }
      if (m > -INFINITY) {
        best = sigmoidf_(m) * obj;
        best_c = mc;
        pass = best > a.conf_thres && !(a.class_mask && !((a.class_mask[mc >> 5] >> (mc & 31)) & 1u));
      }
    }
  }
  int my = -1;
  if (pass) my = atomicAdd(&s_cnt, 1);
  __syncthreads();
  if (tid == 0) s_base = s_cnt ? atomicAdd(&a.cand_count[b], s_cnt) : 0;
  __syncthreads();
  if (pass) {
    const int slot = s_base + my;
    if (slot < a.cap) {
      const long o = (long)b * a.cap + slot;
      a.cand_box[o * 4 + 0] = box[0]; a.cand_box[o * 4 + 1] = box[1];
      a.cand_box[o * 4 + 2] = box[2]; a.cand_box[o * 4 + 3] = box[3];
      a.cand_score[o] = best; a.cand_cls[o] = best_c; a.cand_key[o] = make_score_key(best, (uint32_t)aidx);
    }
  }
}

}  // namespace

// x[l]: fp32 NHWC head inputs (channels [x_off[l], x_off[l] + cin[l]) of rows ldx[l]), hw[6] their
// grids, w[l]: split_pairs weight images [256, 2 * cin[l]] (bf16), bias[l] [256] (channels past
// na * (5 + nc) unused), strides[3], anchors [3][na][2] (host, pixels).  Candidates as
// tca_yolo_decode_filter (single-label; cand_count zeroed here).  cin[l] in {64, 128, 256};
// na * (nc + 5) <= 256; na <= 4.
TCA_API int tca_yolo_detect_filter(const float* const* x, const int* ldx, const int* x_off, const int* cin,
                                   const int* hw, const void* const* w, const float* const* bias, const int* strides,
                                   const float* anchors, int B, int na, int nc, float conf_thres,
                                   const uint32_t* class_mask, float* cand_box, float* cand_score, int* cand_cls,
                                   uint64_t* cand_key, int* cand_count, int cap, hipStream_t stream) {
  if (B <= 0) return 0;
  if (na <= 0 || na > 4 || na * (nc + 5) > NCH || na > 256 / TP) return (int)hipErrorInvalidValue;
  DetArgs a;
  long blocks = 0;
  for (int l = 0; l < 3; ++l) {
    DetLevel& L = a.lv[l];
    if ((cin[l] != 64 && cin[l] != 128 && cin[l] != 256) || (ldx[l] & 3) || (x_off[l] & 3) || ldx[l] < x_off[l] + cin[l])
      return (int)hipErrorInvalidValue;
    L.x = x[l]; L.w = (const __bf16*)w[l]; L.bias = bias[l];
    L.ldx = ldx[l]; L.x_off = x_off[l]; L.cin = cin[l]; L.H = hw[2 * l]; L.W = hw[2 * l + 1]; L.stride = strides[l];
    L.tiles = (L.H * L.W + TP - 1) / TP;
    for (int k = 0; k < 4; ++k) {
      L.anchor[k][0] = k < na ? anchors[(l * na + k) * 2] : 0.f;
      L.anchor[k][1] = k < na ? anchors[(l * na + k) * 2 + 1] : 0.f;
    }
    blocks += (long)B * L.tiles;
  }
  a.B = B; a.na = na; a.nc = nc; a.cap = cap; a.conf_thres = conf_thres; a.class_mask = class_mask;
  a.cand_box = cand_box; a.cand_score = cand_score; a.cand_cls = cand_cls; a.cand_key = cand_key;
  a.cand_count = cand_count;
  if (blocks >= (1L << 31)) return (int)hipErrorInvalidValue;
  int e = zero_i32_async(cand_count, B, stream);
  if (e) return e;
  yolo_detect_filter_kernel<<<(unsigned)blocks, 256, 0, stream>>>(a);
  TCA_LAUNCH_CHECK();
}
