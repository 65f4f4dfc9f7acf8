// Small utility kernels shared by the launchers.
//
// Counters that kernels accumulate into are cleared with a kernel rather
// than hipMemsetAsync: a kernel node behaves identically eager and under
// hipGraph capture/replay, and costs the same ~1-2 us as a memset node.
#include "tca_common.h"

namespace {
__global__ void zero_i32_kernel(int* __restrict__ p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0;
}
}  // namespace

namespace tca {
int zero_i32_async(int* p, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  const int bs = 256;
  const int grid = min((n + bs - 1) / bs, 1024);
  zero_i32_kernel<<<grid, bs, 0, stream>>>(p, n);
  return (int)hipGetLastError();
}
}  // namespace tca

TCA_API int tca_zero_i32(int* p, int n, hipStream_t stream) { return tca::zero_i32_async(p, n, stream); }
