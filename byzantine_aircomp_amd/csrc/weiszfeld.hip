// Weiszfeld geometric-median: slab reduction, the K-space step, and the
// two-pass streaming path for any K.  (The fused streaming pass is in
// stream_pass.hip.)
//
// Reference semantics (goldenBill/Byzantine_AirComp, MNIST_Air_weight.py):
//   gm2  M:162-184  d_k = max(1e-4, ||x_k - g||); g' = sum_k x_k/d_k / sum_k 1/d_k;
//                   stop when ||g - g'|| <= tol, returning g'.
//   gm   M:131-160  the same step with the weighted sums formed "over the air"
//                   by OMA2 (M:396-414): channel-inverted gains + AWGN.
// All per-iteration decisions (weights, tol test) are taken on the device by
// kspace_step, so the host only polls a `done` word.
#include "device_util.h"
#include "gmagg_internal.h"
#include "philox.h"

namespace gmk {

// Sum the per-block slab rows, column by column, in a fixed order.
__global__ void __launch_bounds__(1024) slab_reduce(const double* __restrict__ slab, int nb,
                                                    int64_t S, double* __restrict__ sums,
                                                    const KState* st, int64_t sums_ps) {
  const int64_t pb = blockIdx.y;             // batched problems
  st += pb;
  slab += pb * nb * S;
  sums += pb * sums_ps;
  if (st->done) return;
  __shared__ double red[32][33];
  const int cx = threadIdx.x & 31, by = threadIdx.x >> 5;
  const int64_t j = (int64_t)blockIdx.x * 32 + cx;
  // rows by, by + 32, ... summed in that order; their loads issued 16 at a time (a
  // dependent load per add made this latency-bound: round 6, 6.9 us at nb = 512)
  double acc = 0.0;
  if (j < S) {
    constexpr int U = 16;
    for (int b0 = by; b0 < nb; b0 += 32 * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int b = b0 + 32 * u;
        v[u] = b < nb ? slab[(int64_t)b * S + j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b0 + 32 * u < nb) acc += v[u];
    }
  }
  red[by][cx] = acc;
  __syncthreads();
  if (by == 0 && j < S) {
    double s = 0.0;
#pragma unroll
    for (int y = 0; y < 32; ++y) s += red[y][cx];
    sums[j] = s;
  }
}

// The K-space step: the tol test of the pass that just finished, then the
// next pass's coefficients.  One block.
__device__ void kspace_body(KspaceArgs& a);

// With a.mirror set, thread 0 copies the final KState into host-mapped memory as the
// kernel's last act (plain vector stores; visible to the host once an event recorded
// after this kernel has completed): the lagged convergence poll reads it there instead of
// queueing a device-to-host copy behind every iteration (round 6: one blit kernel and
// ~10 us of launch gap per iteration, 1.2 % of a C3 pass at d_local = 1.375M).
// (every KState field kspace_step writes is written by thread 0, so thread 0's copy after
// its own last write needs no barrier)
__global__ void __launch_bounds__(1024) kspace_step(KspaceArgs a) {
  kspace_body(a);
  if (a.mirror && threadIdx.x == 0 && gridDim.x == 1) *a.mirror = *a.st;
}

__device__ void kspace_body(KspaceArgs& a) {
  if (gridDim.x > 1) {                       // batched problems: block = problem
    const int64_t pb = blockIdx.x;
    a.sums += pb * a.sums_ps;
    a.r += pb * a.K;
    a.coef += pb * a.K;
    a.st += pb;
    a.seed += (uint64_t)pb * kSeedStride;
  }
  KState* st = a.st;
  if (st->done) return;
  __shared__ double scratch[16];
  __shared__ int s_stop;
  const int tid = threadIdx.x;
  const int64_t K = a.K;
  const bool init = a.t < 0;
  const double* D2 = a.sums;
  const double gn2 = init ? a.sums[2 * K + 1] : a.sums[K + 1];

  if (tid == 0) {
    s_stop = 0;
    if (a.do_check && !init) {
      const float mv = (float)sqrt(a.sums[K]);   // (guess - guess_next).norm() (M:180)
      st->last_movement = (double)mv;
      st->iters = a.t + 1;
      if (mv <= a.tol) {                         // M:182 (NaN never passes)
        st->done = 1;
        st->converged = 1;
        s_stop = 1;
        if (a.n_done) atomicAdd(a.n_done, 1);
      }
    }
  }
  if (init && a.mode == 1)
    for (int64_t k = tid; k < K; k += blockDim.x) a.r[k] = a.sums[K + k];
  __syncthreads();
  if (s_stop || !a.do_coef) return;

  if (a.mode == 0) {
    // gm2: g' = sum_k x_k/d_k / sum_k 1/d_k  (M:179), weights normalised here.
    double wsum = 0.0;
    for (int64_t k = tid; k < K; k += blockDim.x) wsum += 1.0 / (double)clamp_dist(D2[k], a.eps);
    const double W = block_sum(wsum, scratch);
    for (int64_t k = tid; k < K; k += blockDim.x)
      a.coef[k] = (float)((1.0 / (double)clamp_dist(D2[k], a.eps)) / W);
    return;
  }

  // gm: the OMA2 weighted sum folded into K-space (SURVEY §3C restatement).
  const int64_t it = a.t + 1;                               // iteration the coefs are for
  const float s = sqrtf((float)(gn2 / (double)a.d_total));  // sqrt(mean(guess^2)) (M:146)
  const float thr = (s * s) * 500.0f;                       // threshold (M:152)
  const double s2 = (double)s * (double)s;
  double csum = 0.0;
  for (int64_t k = tid; k < K; k += blockDim.x) {
    float hr, hi;
    if (a.noise_src == 0) {
      float n[4];
      normal4(a.seed, kStreamChannel, (uint64_t)it, (uint64_t)k, n);
      hr = n[0] * 0.70710678118654752f;
      hi = n[1] * 0.70710678118654752f;
    } else {
      hr = a.h_re[k];
      hi = a.h_im[k];
    }
    const float h2 = hr * hr + hi * hi;                     // M:403
    const float dist = clamp_dist(D2[k], a.eps);
    const double dd = (double)dist;
    // mean_j (msg_kj^2 / h2_k) over the d+1 entries of [x_k/dist_k, s/dist_k]   (M:404-405)
    const double p = (a.r[k] + s2) / (dd * dd * (double)(a.d_total + 1)) / (double)h2;
    const double pup = p != p ? p : fmax(p, (double)thr);
    const double gain = sqrt(a.P_max / pup);                // M:407
    const double ck = gain / dd;
    a.coef[k] = (float)ck;                                  // rescaled below
    csum += ck;
  }
  const double Sc = block_sum(csum, scratch);
  double nd = 0.0;
  if (a.has_noise)
    nd = a.noise_src == 0
             ? a.noise_sd * (double)normal1(a.seed, kStreamNoise, (uint64_t)it, (uint64_t)a.d_total)
             : (double)a.n_last[0];
  const double yd = (double)s * Sc + nd;                    // y[d]: the denominator (M:154)
  const double scale = (double)s / yd;                      // g' = y[:d] / y[d] * s (M:155)
  __syncthreads();
  for (int64_t k = tid; k < K; k += blockDim.x) a.coef[k] = (float)((double)a.coef[k] * scale);
  if (tid == 0) {
    st->s = s;
    st->a_noise = a.has_noise ? (float)(scale * (a.noise_src == 0 ? a.noise_sd : 1.0)) : 0.f;
  }
}

// ---------------------------------------------------------------------------
// Two-pass path (any K): a column pass for g' (and the movement), a row pass
// for the distances.  Two reads of X per iteration; used where the fused tile
// does not fit (K > 2048) or on request.

__global__ void __launch_bounds__(256) twopass_sum(const float* __restrict__ X, int64_t K,
                                                   int64_t d, int64_t ldx,
                                                   const float* __restrict__ g_old,
                                                   float* __restrict__ g_new,
                                                   const float* __restrict__ coef,
                                                   const KState* st, int noise,
                                                   const float* __restrict__ hnoise,
                                                   uint64_t seed, int64_t iter, int64_t col_off,
                                                   double* slab) {
  if (st->done) return;
  __shared__ double scratch[16];
  double mv = 0.0, gn = 0.0;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d;
       j += (int64_t)gridDim.x * blockDim.x) {
    if (g_new == nullptr) {              // INIT: only ||g0||^2
      const float g = g_old[j];
      gn += (double)(g * g);
      continue;
    }
    float acc = 0.f;
    int64_t k = 0;
    for (; k + 8 <= K; k += 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(X + (k + u) * ldx + j);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fmaf(coef[k + u], x[u], acc);
    }
    for (; k < K; ++k) acc = fmaf(coef[k], X[k * ldx + j], acc);
    if (noise == 1) acc = fmaf(st->a_noise, normal1(seed, kStreamNoise, iter, col_off + j), acc);
    else if (noise == 2) acc = fmaf(st->a_noise, hnoise[j], acc);
    g_new[j] = acc;
    const float diff = g_old[j] - acc;
    mv += (double)(diff * diff);
    gn += (double)(acc * acc);
  }
  const double m = block_sum(mv, scratch);
  const double g = block_sum(gn, scratch);
  if (threadIdx.x == 0) {
    slab[(int64_t)blockIdx.x * 2] = m;
    slab[(int64_t)blockIdx.x * 2 + 1] = g;
  }
}

// One block per row: squared distance to g (and ||x||^2 at init).
__global__ void __launch_bounds__(256) twopass_dist(const float* __restrict__ X, int64_t K,
                                                    int64_t d, int64_t ldx,
                                                    const float* __restrict__ g, bool init,
                                                    const KState* st, double* sums) {
  if (st->done) return;
  __shared__ double scratch[16];
  const int64_t k = blockIdx.x;
  const float* row = X + k * ldx;
  double acc = 0.0, acc2 = 0.0;
  for (int64_t j = threadIdx.x; j < d; j += blockDim.x) {
    const float x = __builtin_nontemporal_load(row + j);
    const float t = x - g[j];
    acc += (double)(t * t);
    acc2 += (double)(x * x);
  }
  const double s1 = block_sum(acc, scratch);
  const double s2 = init ? block_sum(acc2, scratch) : 0.0;
  if (threadIdx.x == 0) {
    sums[k] = s1;
    if (init) sums[K + k] = s2;
  }
}

// Batched problems: out_p = the buffer holding problem p's last iterate.
__global__ void __launch_bounds__(256) batched_finalize(const float* __restrict__ g0,
                                                        const float* __restrict__ g1, int64_t d,
                                                        const KState* st, float* out,
                                                        int64_t ldo) {
  const int64_t pb = blockIdx.y;
  const int64_t it = st[pb].iters;
  const float* src = ((it - 1) & 1) ? g1 : g0;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d;
       j += (int64_t)gridDim.x * blockDim.x)
    out[pb * ldo + j] = src[pb * d + j];
}

hipError_t launch_batched_finalize(const float* g0, const float* g1, int64_t d, int problems,
                                   const KState* st, float* out, int64_t ldo, hipStream_t s) {
  const int64_t bx = (d + 255) / 256;
  hipLaunchKernelGGL(batched_finalize, dim3((unsigned)(bx < 64 ? bx : 64), problems), dim3(256), 0,
                     s, g0, g1, d, st, out, ldo);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Launch plumbing.

hipError_t launch_slab_reduce(const double* slab, int nb, int64_t S, double* sums,
                              const KState* st, hipStream_t s, int problems, int64_t sums_ps) {
  const int grid = (int)((S + 31) / 32);
  hipLaunchKernelGGL(slab_reduce, dim3(grid, problems), dim3(1024), 0, s, slab, nb, S, sums, st,
                     sums_ps);
  return hipGetLastError();
}

hipError_t launch_kspace(const KspaceArgs& a, hipStream_t s, int problems) {
  const int threads = a.K >= 1024 ? 1024 : (int)((a.K + 63) / 64 * 64);
  hipLaunchKernelGGL(kspace_step, dim3(problems), dim3(threads), 0, s, a);
  return hipGetLastError();
}

int twopass_blocks(int64_t K, int64_t d, int num_cu) {
  (void)K;
  const int64_t want = (d + 255) / 256;
  const int64_t cap = (int64_t)num_cu * 8;
  return (int)(want < cap ? (want > 0 ? want : 1) : cap);
}

// Writes the (K+2) / (2K+2) sums vector.
hipError_t launch_twopass(bool init, const float* X, int64_t K, int64_t d, int64_t ldx,
                          const float* g_old, float* g_new, const float* coef, const KState* st,
                          int noise, const float* hnoise, uint64_t seed, int64_t iter,
                          int64_t col_off, double* slab, int nb, double* sums, hipStream_t s) {
  const int64_t base = init ? 2 * K : K;
  hipLaunchKernelGGL(twopass_sum, dim3(nb), dim3(256), 0, s, X, K, d, ldx, g_old,
                     init ? nullptr : g_new, coef, st, noise, hnoise, seed, iter, col_off, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(twopass_dist, dim3((unsigned)K), dim3(256), 0, s, X, K, d, ldx,
                     init ? g_old : g_new, init, st, sums);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_slab_reduce(slab, nb, 2, sums + base, st, s);
}

}  // namespace gmk
