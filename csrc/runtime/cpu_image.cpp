// Host-side image preprocess for GPU-less hosts (BASELINE config 1: client and
// server on a CPU-only machine).  Same contract as the HIP kernel
// tca_image_preprocess (csrc/kernels/image.hip) and the NumPy golden
// (ops/golden.py preprocess_image): bilinear resize of a uint8 HWC frame into
// a (letterboxed) region of the destination, optional uint8 quantisation of
// the resized value (what cv2.resize to uint8 does, reference
// clients/preprocess/yolov5_preprocess.py), padding elsewhere, then
// x * scale + bias per channel, written as NCHW or NHWC fp32.
//
// Rows are split over std::threads; the per-pixel arithmetic is fp32 in the
// golden's order, so results are bit-identical to it.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

struct Axis {
  std::vector<int> s0, s1;
  std::vector<float> a;
};

// pixel-centre mapping, clamped at both ends (ops/golden.py _axis_coords)
Axis axis_coords(int n_dst, int n_src) {
  Axis ax;
  ax.s0.resize(n_dst);
  ax.s1.resize(n_dst);
  ax.a.resize(n_dst);
  const float scale = float(n_src) / float(n_dst);
  for (int i = 0; i < n_dst; ++i) {
    const float f = (float(i) + 0.5f) * scale - 0.5f;
    int s = int(std::floor(f));
    float a = f - float(s);
    if (s < 0) {
      s = 0;
      a = 0.0f;
    }
    if (s >= n_src - 1) {
      s = n_src - 1;
      a = 0.0f;
    }
    ax.s0[i] = s;
    ax.s1[i] = std::min(s + 1, n_src - 1);
    ax.a[i] = a;
  }
  return ax;
}

// round half to even for 0 <= v < 2^22 (np.rint); adding and removing 1.5*2^23
// rounds in the FPU's default mode without nearbyint's fenv save / restore
inline float round_even(float v) {
  volatile float big = 12582912.0f;
  return (v + big) - big;
}

template <bool NCHW, bool QUANT>
void preprocess_rows(const uint8_t* src, int w0, int c0, int swap_rb, float* out, int H, int W, int top, int left,
                     int nh, int nw, float pad, const float* scale, const float* bias, const Axis& ay, const Axis& ax,
                     int y_begin, int y_end) {
  const int64_t plane = int64_t(H) * W;
  // output channel k takes source channel src_c[k] (swap_rb reverses the canvas)
  const int src_c[3] = {swap_rb ? 2 : 0, 1, swap_rb ? 0 : 2};
  float padv[3];
  for (int k = 0; k < 3; ++k) padv[k] = pad * scale[k] + bias[k];
  for (int y = y_begin; y < y_end; ++y) {
    float* o[3];
    for (int k = 0; k < 3; ++k) o[k] = NCHW ? out + k * plane + int64_t(y) * W : out + int64_t(y) * W * 3 + k;
    const int step = NCHW ? 1 : 3;
    const int ry = y - top;
    if (ry < 0 || ry >= nh) {
      for (int x = 0; x < W; ++x)
        for (int k = 0; k < 3; ++k) o[k][x * step] = padv[k];
      continue;
    }
    const uint8_t* r0 = src + int64_t(ay.s0[ry]) * w0 * c0;
    const uint8_t* r1 = src + int64_t(ay.s1[ry]) * w0 * c0;
    const float fy = ay.a[ry];
    const int x_end = left + nw;
    for (int x = 0; x < W; ++x) {
      if (x < left || x >= x_end) {
        for (int k = 0; k < 3; ++k) o[k][x * step] = padv[k];
        continue;
      }
      const int rx = x - left;
      const int x0 = ax.s0[rx] * c0, x1 = ax.s1[rx] * c0;
      const float fx = ax.a[rx];
      for (int k = 0; k < 3; ++k) {
        const int c = src_c[k];
        const float p00 = r0[x0 + c], p01 = r0[x1 + c], p10 = r1[x0 + c], p11 = r1[x1 + c];
        const float t = p00 + fx * (p01 - p00);
        const float b = p10 + fx * (p11 - p10);
        float v = t + fy * (b - t);
        if (QUANT) v = std::min(255.0f, std::max(0.0f, round_even(v)));
        o[k][x * step] = v * scale[k] + bias[k];
      }
    }
  }
}

}  // namespace

extern "C" {

// src: [h0][w0][c0] uint8 (c0 >= 3; channels beyond 3 ignored); out: fp32
// [3][H][W] (layout 0) or [H][W][3] (layout 1).  Region (top, left, nh, nw)
// receives the resized frame, the rest `pad`.  Returns 0.
int tca_cpu_preprocess(const uint8_t* src, int h0, int w0, int c0, int swap_rb, float* out, int layout, int H, int W,
                       int top, int left, int nh, int nw, float pad, int quantize, const float* scale,
                       const float* bias, int nthreads) {
  const Axis ay = axis_coords(nh, h0), ax = axis_coords(nw, w0);
  auto rows = [&](int b, int e) {
    auto fn = layout == 0 ? (quantize ? preprocess_rows<true, true> : preprocess_rows<true, false>)
                          : (quantize ? preprocess_rows<false, true> : preprocess_rows<false, false>);
    fn(src, w0, c0, swap_rb, out, H, W, top, left, nh, nw, pad, scale, bias, ay, ax, b, e);
  };
  nthreads = std::max(1, std::min(nthreads, H));
  std::vector<std::thread> pool;
  const int chunk = (H + nthreads - 1) / nthreads;
  for (int t = 1; t < nthreads; ++t) {
    const int b = t * chunk, e = std::min(H, b + chunk);
    if (b < e) pool.emplace_back(rows, b, e);
  }
  rows(0, std::min(H, chunk));
  for (auto& th : pool) th.join();
  return 0;
}

}  // extern "C"
