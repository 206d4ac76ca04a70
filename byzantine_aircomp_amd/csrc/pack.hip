// Row f2: the caller-side packing.  The reference stacks the K
// flattened client vectors row-major (flatten_list, MNIST_Air_weight.py:206-209);
// the streaming pass reads them fastest in the panel layout [ceil(d/W)][K][W]
// (DESIGN.md §1).  One kernel converts: thread e moves one float4 (or one float),
// consecutive threads walk the W/4 groups of one row segment, then the next row,
// then the next panel, so a wave reads 8 row segments of 128 B (W = 32) and
// writes 1 KiB contiguously.  Padding columns (>= d) of the last panel are left
// as they are (ClientPanels allocates them zeroed).
#include "gmagg_internal.h"

namespace gmk {

template <bool VEC4>
__global__ void __launch_bounds__(256) rows_to_panels(const float* __restrict__ X, int64_t K,
                                                      int64_t d, int64_t ldx,
                                                      float* __restrict__ P, int64_t W,
                                                      int64_t pstride) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int E = VEC4 ? 4 : 1;                 // floats per thread-item
  const int64_t per_row = W / E;                  // items per (panel, row)
  const int64_t npan = (d + W - 1) / W;
  const int64_t n = npan * K * per_row;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = e % per_row, rk = e / per_row;
    const int64_t k = rk % K, p = rk / K;
    const int64_t col = p * W + q * E;
    if (col >= d) continue;
    float* dst = P + p * pstride + k * W + q * E;
    const float* src = X + k * ldx + col;
    if constexpr (VEC4) {
      if (col + 4 <= d) {
        __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const f4*>(src)),
                                    reinterpret_cast<f4*>(dst));
      } else {
        for (int u = 0; col + u < d; ++u) dst[u] = src[u];
      }
    } else {
      *dst = *src;
    }
  }
}

hipError_t launch_rows_to_panels(const float* X, int64_t K, int64_t d, int64_t ldx, float* P,
                                 int64_t W, int64_t pstride, hipStream_t s) {
  const bool vec4 = reinterpret_cast<uintptr_t>(X) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(P) % 16 == 0 && ldx % 4 == 0 && W % 4 == 0 &&
                    pstride % 4 == 0;
  const int64_t items = ((d + W - 1) / W) * K * (vec4 ? W / 4 : W);
  int64_t grid = (items + 255) / 256;
  if (grid > 16384) grid = 16384;
  if (grid < 1) grid = 1;
  if (vec4)
    hipLaunchKernelGGL(rows_to_panels<true>, dim3((unsigned)grid), dim3(256), 0, s, X, K, d, ldx,
                       P, W, pstride);
  else
    hipLaunchKernelGGL(rows_to_panels<false>, dim3((unsigned)grid), dim3(256), 0, s, X, K, d, ldx,
                       P, W, pstride);
  return hipGetLastError();
}

}  // namespace gmk
