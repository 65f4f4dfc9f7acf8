// K15 — annotation of the published camera frames, on the device.
//
// Reference: ros_inference.py:149-169 draws each kept detection onto the
// frame (cv2.rectangle + cv2.putText of "<class> <conf>") before publishing
// the rgb8 Image.  Here the frames are already resident on
// the GPU (the camera pipeline's uint8 NHWC input buffer) and the detections
// are the NMS result buffers, so boxes AND label text are drawn in place
// before the one D2H copy the publisher needs anyway — the host never touches
// a pixel.
//
// One workgroup per frame.  Pass 1 draws every box's rectangle, pass 2 every
// box's label, each in result order with a barrier between boxes, so where
// two overlap the later one wins — pixel-identical to the host painter
// (utils/draw.py draw_detections: round-half-even corners clipped to the
// frame, `thickness`-pixel bands inside the box, colour = class_color(cls);
// labels in the 6x11 cell font of tca_font6x11.h at (x1 + 2, max(y1 - 11, 0)),
// text "<name> <conf:.2f>" with conf rounded half-even from its exact value).
// Consecutive threads write consecutive pixels of a row, so stores coalesce.
#include "tca_common.h"
#include "tca_font6x11.h"

namespace {

constexpr int kNameMax = 32;  // names table row: <= 31 printable chars + NUL
constexpr int kLabelMax = 64;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

struct Corner {
  int x1, y1, x2, y2;
};

__device__ __forceinline__ Corner corners(const float* bx, int H, int W) {
  return {clampi((int)rintf(bx[0]), 0, W - 1), clampi((int)rintf(bx[1]), 0, H - 1),
          clampi((int)rintf(bx[2]), 0, W - 1), clampi((int)rintf(bx[3]), 0, H - 1)};
}

__device__ __forceinline__ void class_rgb(int c, unsigned char& c0, unsigned char& c1, unsigned char& c2) {
  const unsigned h = ((unsigned)c * 2654435761u) & 0xFFFFFFu;
  c0 = (h >> 16) & 255;
  c1 = (h >> 8) & 255;
  c2 = h & 255;
}

// "<name> <int>.<2 digits>" into lbl; returns the length.  Names outside the
// table print as the decimal class id (the host painter's str(c)).
__device__ int format_label(char* lbl, int c, float conf, const unsigned char* names, int n_names) {
  int L = 0;
  if (names != nullptr && c >= 0 && c < n_names) {
    const unsigned char* s = names + (long)c * kNameMax;
    for (int i = 0; i < kNameMax - 1 && s[i]; ++i) lbl[L++] = (char)s[i];
  } else {
    long v = c;
    if (v < 0) {
      lbl[L++] = '-';
      v = -v;
    }
    char d[12];
    int nd = 0;
    do {
      d[nd++] = (char)('0' + v % 10);
      v /= 10;
    } while (v && nd < 12);
    while (nd) lbl[L++] = d[--nd];
  }
  lbl[L++] = ' ';
  // conf * 100 is exact in fp64 (24-bit mantissa x 7 bits), so rint rounds the
  // exact value half-even like Python's '{:.2f}'
  double p = rint((double)conf * 100.0);
  long v = p > 0.0 ? (p < 1e9 ? (long)p : 999999999L) : 0L;
  long ip = v / 100;
  char d[12];
  int nd = 0;
  do {
    d[nd++] = (char)('0' + ip % 10);
    ip /= 10;
  } while (ip && nd < 12);
  while (nd) lbl[L++] = d[--nd];
  lbl[L++] = '.';
  lbl[L++] = (char)('0' + (v % 100) / 10);
  lbl[L++] = (char)('0' + v % 10);
  return L;
}

__global__ void __launch_bounds__(1024) draw_kernel(unsigned char* __restrict__ img, long frame_stride, int H, int W,
                                                    int row_stride, const float* __restrict__ box, int box_ld,
                                                    int box_dim, const float* __restrict__ score,
                                                    const int* __restrict__ cls, const int* __restrict__ count,
                                                    int max_boxes, int thickness, const unsigned char* names,
                                                    int n_names) {
  __shared__ char lbl[kLabelMax];
  __shared__ int lbl_len;
  const int b = blockIdx.x;
  unsigned char* f = img + (long)b * frame_stride;
  const int n = min(count[b], max_boxes);
  const int t = max(1, thickness);
  for (int k = 0; k < n; ++k) {
    const Corner q = corners(box + ((long)b * box_ld + k) * box_dim, H, W);
    if (q.x2 >= q.x1 && q.y2 >= q.y1) {
      unsigned char c0, c1, c2;
      class_rgb(cls[(long)b * box_ld + k], c0, c1, c2);
      // bands: top, bottom (full width), left, right (full height)
      int ya[4] = {q.y1, max(q.y2 - t + 1, q.y1), q.y1, q.y1};
      int yb[4] = {min(q.y1 + t, q.y2 + 1), q.y2 + 1, q.y2 + 1, q.y2 + 1};
      int xa[4] = {q.x1, q.x1, q.x1, max(q.x2 - t + 1, q.x1)};
      int xb[4] = {q.x2 + 1, q.x2 + 1, min(q.x1 + t, q.x2 + 1), q.x2 + 1};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int bw = xb[s] - xa[s], total = (yb[s] - ya[s]) * bw;
        for (int i = threadIdx.x; i < total; i += blockDim.x) {
          const int y = ya[s] + i / bw, x = xa[s] + i % bw;
          unsigned char* p = f + (long)y * row_stride + x * 3;
          p[0] = c0;
          p[1] = c1;
          p[2] = c2;
        }
      }
    }
    __syncthreads();  // the next box overwrites this one where they overlap
  }
  if (score == nullptr) return;
  for (int k = 0; k < n; ++k) {
    const long r = (long)b * box_ld + k;
    const Corner q = corners(box + r * box_dim, H, W);
    const bool valid = q.x2 >= q.x1 && q.y2 >= q.y1;
    if (threadIdx.x == 0) lbl_len = valid ? format_label(lbl, cls[r], score[r], names, n_names) : 0;
    __syncthreads();
    const int L = lbl_len;
    if (L > 0) {
      unsigned char c0, c1, c2;
      class_rgb(cls[r], c0, c1, c2);
      const int x0 = q.x1 + 2, y0 = max(q.y1 - TCA_FONT_H, 0);
      const int cols = L * TCA_FONT_W, total = cols * TCA_FONT_H;
      for (int i = threadIdx.x; i < total; i += blockDim.x) {
        const int row = i / cols, col = i % cols;
        const int y = y0 + row, x = x0 + col;
        if (y >= H || x >= W) continue;
        int ch = (unsigned char)lbl[col / TCA_FONT_W];
        ch = (ch < TCA_FONT_FIRST || ch > TCA_FONT_LAST) ? '?' : ch;
        if ((tca_font6x11[ch - TCA_FONT_FIRST][row] >> (col % TCA_FONT_W)) & 1) {
          unsigned char* p = f + (long)y * row_stride + x * 3;
          p[0] = c0;
          p[1] = c1;
          p[2] = c2;
        }
      }
    }
    __syncthreads();  // lbl is rewritten for the next box; later labels win
  }
}

int check_args(int H, int W, int row_stride, int box_dim, int box_ld, long frame_stride) {
  if (H <= 0 || W <= 0 || row_stride < 3 * W || box_dim < 4 || box_ld <= 0 || frame_stride < (long)H * row_stride)
    return (int)hipErrorInvalidValue;
  return 0;
}

}  // namespace

// img: B uint8 HxWx3 frames (frame_stride bytes apart, row_stride bytes per
// row); box [B, box_ld, box_dim] fp32 x1,y1,x2,y2,… in frame pixels;
// cls [B, box_ld] int32; count [B] int32 (device).  Draws boxes 0..count-1.
TCA_API int tca_draw_boxes(void* img, long frame_stride, int B, int H, int W, int row_stride, const float* box,
                           int box_ld, int box_dim, const int* cls, const int* count, int thickness,
                           hipStream_t stream) {
  if (B <= 0) return 0;
  if (int e = check_args(H, W, row_stride, box_dim, box_ld, frame_stride)) return e;
  draw_kernel<<<B, 1024, 0, stream>>>((unsigned char*)img, frame_stride, H, W, row_stride, box, box_ld, box_dim,
                                      nullptr, cls, count, box_ld, thickness, nullptr, 0);
  return (int)hipGetLastError();
}

// Boxes and labels: as tca_draw_boxes, then the "<name> <conf>" label of each
// box (score [B, box_ld] fp32).  names: n_names rows of 32 bytes (printable
// ASCII, NUL-terminated; device memory), or null for numeric class ids.
TCA_API int tca_draw_annotations(void* img, long frame_stride, int B, int H, int W, int row_stride, const float* box,
                                 int box_ld, int box_dim, const float* score, const int* cls, const int* count,
                                 int thickness, const void* names, int n_names, hipStream_t stream) {
  if (B <= 0) return 0;
  if (int e = check_args(H, W, row_stride, box_dim, box_ld, frame_stride)) return e;
  if (score == nullptr || n_names < 0) return (int)hipErrorInvalidValue;
  draw_kernel<<<B, 1024, 0, stream>>>((unsigned char*)img, frame_stride, H, W, row_stride, box, box_ld, box_dim,
                                      score, cls, count, box_ld, thickness, (const unsigned char*)names,
                                      names ? n_names : 0);
  return (int)hipGetLastError();
}
