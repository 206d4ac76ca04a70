// The reference's other aggregators, MNIST_Air_weight.py:186-204:
//   mean          M:186-187   column mean
//   trimmed_mean  M:189-192   mean of each column without its b smallest and b largest
//   median        M:194-195   lower median of each column (torch.median)
//   Krum          M:197-204   the row with the smallest sum of squared distances to
//                              its honestSize-1 nearest rows (itself included, M:200-201)
// Column statistics stage a 64-column x K tile in LDS; selections rank each
// element against its column with a stable tie-break (x_j < x_i, or x_j == x_i
// and j < i), which gives torch's order statistics exactly for the median and
// the trimmed set; sums are fp64, rounded once.
#include "device_util.h"
#include "gmagg_internal.h"

namespace gmk {

constexpr int kColBlock = 64;     // columns per block (one per thread of wave 0.. )

// mean: one thread per column, fp64 accumulation.
__global__ void __launch_bounds__(256) col_mean(const float* __restrict__ X, int64_t K, int64_t d,
                                                int64_t ldx, float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d;
       j += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int64_t k = 0; k < K; ++k) s += (double)X[k * ldx + j];
    out[j] = (float)(s / (double)K);
  }
}

// Order statistics over a 64-column tile in LDS.  mode 0: lower median;
// mode 1: trimmed mean dropping b values at each end.
template <int KMAX>
__global__ void __launch_bounds__(256) col_select(const float* __restrict__ X, int64_t K,
                                                  int64_t d, int64_t ldx, int mode, int64_t b,
                                                  float* __restrict__ out) {
  __shared__ float tile[KMAX][kColBlock + 1];
  const int64_t j0 = (int64_t)blockIdx.x * kColBlock;
  const int tc = threadIdx.x % kColBlock, tr = threadIdx.x / kColBlock;   // 4 row lanes
  for (int64_t k = tr; k < K; k += blockDim.x / kColBlock)
    tile[k][tc] = j0 + tc < d ? X[k * ldx + j0 + tc] : 0.f;
  __syncthreads();
  // 4 threads per column split the candidates i; combine through LDS.
  __shared__ double acc[4][kColBlock];
  __shared__ float med[4][kColBlock];
  __shared__ int found[4][kColBlock];
  const int64_t m = (K - 1) / 2;
  double s = 0.0;
  float mv = 0.f;
  int fnd = 0;
  for (int64_t i = tr; i < K; i += 4) {
    const float xi = tile[i][tc];
    int64_t rank = 0;
    for (int64_t jj = 0; jj < K; ++jj) {
      const float xj = tile[jj][tc];
      rank += (xj < xi) || (xj == xi && jj < i);
    }
    if (mode == 0) {
      if (rank == m) { mv = xi; fnd = 1; }
    } else if (rank >= b && rank < K - b) {
      s += (double)xi;
    }
  }
  acc[tr][tc] = s;
  med[tr][tc] = mv;
  found[tr][tc] = fnd;
  __syncthreads();
  if (tr == 0 && j0 + tc < d) {
    if (mode == 0) {
      float v = 0.f;
      for (int r = 0; r < 4; ++r)
        if (found[r][tc]) v = med[r][tc];
      out[j0 + tc] = v;
    } else {
      double t = 0.0;
      for (int r = 0; r < 4; ++r) t += acc[r][tc];
      out[j0 + tc] = (float)(t / (double)(K - 2 * b));
    }
  }
}

// Krum, step 1: squared distance of every row pair (i <= j), one block per pair,
// fp32 squared differences accumulated in fp64 (M:199 sums over d in fp32).
__global__ void __launch_bounds__(256) pair_dist(const float* __restrict__ X, int64_t K, int64_t d,
                                                 int64_t ldx, double* __restrict__ D) {
  __shared__ double scratch[16];
  const int64_t p = blockIdx.x;
  // decode p -> (i, j), i <= j, row-major over the upper triangle
  int64_t i = 0, rem = p;
  while (rem >= K - i) { rem -= K - i; ++i; }
  const int64_t j = i + rem;
  double s = 0.0;
  const float* a = X + i * ldx;
  const float* bb = X + j * ldx;
  for (int64_t c = threadIdx.x; c < d; c += blockDim.x) {
    const float t = a[c] - bb[c];
    s += (double)(t * t);
  }
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) {
    D[i * K + j] = s;
    D[j * K + i] = s;
  }
}

// Krum, step 2 (one block): score_i = sum of the kk smallest D[i][*] (self included),
// index = first argmin (torch.argmin), out = that row.
__global__ void __launch_bounds__(256) krum_select(const double* __restrict__ D, int64_t K,
                                                   int64_t kk, const float* __restrict__ X,
                                                   int64_t d, int64_t ldx, float* __restrict__ out,
                                                   int64_t* index) {
  __shared__ double score[1024];
  __shared__ int64_t s_best;
  for (int64_t i = threadIdx.x; i < K; i += blockDim.x) {
    const double* row = D + i * K;
    double sc = 0.0;
    for (int64_t jj = 0; jj < K; ++jj) {          // stable rank of D[i][jj] in its row
      int64_t rank = 0;
      for (int64_t t = 0; t < K; ++t) rank += (row[t] < row[jj]) || (row[t] == row[jj] && t < jj);
      if (rank < kk) sc += row[jj];
    }
    score[i] = sc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t best = 0;
    for (int64_t i = 1; i < K; ++i)
      if (score[i] < score[best]) best = i;
    s_best = best;
    if (index) *index = best;
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < d; c += blockDim.x) out[c] = X[s_best * ldx + c];
}

static int grid_cols(int64_t d) {
  const int64_t g = (d + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

hipError_t launch_col_mean(const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                           hipStream_t s) {
  hipLaunchKernelGGL(col_mean, dim3(grid_cols(d)), dim3(256), 0, s, X, K, d, ldx, out);
  return hipGetLastError();
}

hipError_t launch_col_select(const float* X, int64_t K, int64_t d, int64_t ldx, int mode,
                             int64_t b, float* out, hipStream_t s) {
  const dim3 grid((unsigned)((d + kColBlock - 1) / kColBlock));
  if (K <= 64)
    hipLaunchKernelGGL(col_select<64>, grid, dim3(256), 0, s, X, K, d, ldx, mode, b, out);
  else if (K <= 256)
    hipLaunchKernelGGL(col_select<256>, grid, dim3(256), 0, s, X, K, d, ldx, mode, b, out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_krum(const float* X, int64_t K, int64_t d, int64_t ldx, int64_t kk, double* D,
                       float* out, int64_t* index, hipStream_t s) {
  if (K > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pair_dist, dim3((unsigned)(K * (K + 1) / 2)), dim3(256), 0, s, X, K, d, ldx,
                     D);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(krum_select, dim3(1), dim3(256), 0, s, D, K, kk, X, d, ldx, out, index);
  return hipGetLastError();
}

}  // namespace gmk
