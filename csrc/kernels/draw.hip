// K15 — box annotation of the published camera frames, on the device.
//
// Reference: ros_inference.py:149-169 draws each kept detection onto the
// frame with cv2.rectangle before publishing the rgb8 Image (SURVEY §2.3
// K15).  Here the frames are already resident on the GPU (the camera
// pipeline's uint8 NHWC input buffer) and the detections are the NMS
// result buffers, so the rectangles are drawn in place before the one D2H
// copy the publisher needs anyway.
//
// One workgroup per frame; boxes are drawn in result order with a barrier
// between boxes, so where boxes overlap the later one wins — pixel-identical
// to the host painter (utils/draw.py draw_rect: round-half-even corners,
// clipped to the frame, `thickness`-pixel bands inside the box, colour
// = class_color(cls)).  Each band is a set of row segments: consecutive
// threads write consecutive pixels, so the stores coalesce along x.
#include "tca_common.h"

namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__global__ void __launch_bounds__(1024) draw_boxes_kernel(unsigned char* __restrict__ img, long frame_stride,
                                                          int H, int W, int row_stride,
                                                          const float* __restrict__ box, int box_ld, int box_dim,
                                                          const int* __restrict__ cls, const int* __restrict__ count,
                                                          int max_boxes, int thickness) {
  const int b = blockIdx.x;
  unsigned char* f = img + (long)b * frame_stride;
  const int n = min(count[b], max_boxes);
  const int t = max(1, thickness);
  for (int k = 0; k < n; ++k) {
    const float* bx = box + ((long)b * box_ld + k) * box_dim;
    const int x1 = clampi((int)rintf(bx[0]), 0, W - 1), y1 = clampi((int)rintf(bx[1]), 0, H - 1);
    const int x2 = clampi((int)rintf(bx[2]), 0, W - 1), y2 = clampi((int)rintf(bx[3]), 0, H - 1);
    if (x2 >= x1 && y2 >= y1) {
      const unsigned h = ((unsigned)cls[(long)b * box_ld + k] * 2654435761u) & 0xFFFFFFu;
      const unsigned char c0 = (h >> 16) & 255, c1 = (h >> 8) & 255, c2 = h & 255;
      // bands: top, bottom (full width), left, right (full height)
      int ya[4] = {y1, max(y2 - t + 1, y1), y1, y1};
      int yb[4] = {min(y1 + t, y2 + 1), y2 + 1, y2 + 1, y2 + 1};
      int xa[4] = {x1, x1, x1, max(x2 - t + 1, x1)};
      int xb[4] = {x2 + 1, x2 + 1, min(x1 + t, x2 + 1), x2 + 1};
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
}

}  // namespace

// img: B uint8 HxWx3 frames (frame_stride bytes apart, row_stride bytes per
// row); box [B, box_ld, box_dim] fp32 x1,y1,x2,y2,… in frame pixels;
// cls [B, box_ld] int32; count [B] int32 (device).  Draws boxes 0..count-1.
TCA_API int tca_draw_boxes(void* img, long frame_stride, int B, int H, int W, int row_stride, const float* box,
                           int box_ld, int box_dim, const int* cls, const int* count, int thickness,
                           hipStream_t stream) {
  if (B <= 0) return 0;
  if (H <= 0 || W <= 0 || row_stride < 3 * W || box_dim < 4 || box_ld <= 0 || frame_stride < (long)H * row_stride)
    return (int)hipErrorInvalidValue;
  draw_boxes_kernel<<<B, 1024, 0, stream>>>((unsigned char*)img, frame_stride, H, W, row_stride, box, box_ld,
                                            box_dim, cls, count, box_ld, thickness);
  return (int)hipGetLastError();
}
