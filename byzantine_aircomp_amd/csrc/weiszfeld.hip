// Weiszfeld geometric-median kernels for gfx950 (MI355X).
//
// Reference semantics (goldenBill/Byzantine_AirComp, MNIST_Air_weight.py):
//   gm2  M:162-184  d_k = max(1e-4, ||x_k - g||); g' = sum_k x_k/d_k / sum_k 1/d_k;
//                   stop when ||g - g'|| <= tol, returning g'.
//   gm   M:131-160  the same step with the weighted sums formed "over the air"
//                   by OMA2 (M:396-414): channel-inverted gains + AWGN.
//
// Design: ONE HBM read of X per Weiszfeld iteration.  A block
// owns a chunk of J columns x all K rows at a time, held in VGPRs:
//   phase A  g'_j = sum_k c_k x_kj            (c_k from the K-space step)
//   phase B  D_k += sum_{j in chunk} (x_kj - g'_j)^2   for the NEXT iteration
// plus ||g - g'||^2 and ||g'||^2 for the tol test and the AirComp scaler.
// Per-block partials land in a slab [blocks][K+2] (fp64) that slab_reduce sums
// in a fixed order (deterministic, no atomics); kspace_step turns the sums into
// the next iteration's coefficients on the device, so the host only polls.
#include "gmagg_internal.h"
#include "philox.h"

namespace gmk {

template <int V> struct vec;
template <> struct vec<1> { typedef float t; };
template <> struct vec<2> { typedef float t __attribute__((ext_vector_type(2))); };
template <> struct vec<4> { typedef float t __attribute__((ext_vector_type(4))); };

template <int V>
__device__ __forceinline__ void load_cols(const float* __restrict__ p, float (&o)[V]) {
  if constexpr (V == 1) {
    o[0] = __builtin_nontemporal_load(p);
  } else {
    typedef typename vec<V>::t T;
    T v = __builtin_nontemporal_load(reinterpret_cast<const T*>(p));
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = v[i];
  }
}

template <int V>
__device__ __forceinline__ void load_cols_cached(const float* __restrict__ p, float (&o)[V]) {
  if constexpr (V == 1) {
    o[0] = *p;
  } else {
    typedef typename vec<V>::t T;
    T v = *reinterpret_cast<const T*>(p);
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = v[i];
  }
}

template <int A, int B> struct cmin { static constexpr int v = A < B ? A : B; };
template <int N> struct ilog2 { static constexpr int v = 1 + ilog2<N / 2>::v; };
template <> struct ilog2<1> { static constexpr int v = 0; };

// Reduce R per-row values across the LPR lanes of a row segment so that each
// lane ends up holding complete row sums ("transpose-reduce"): halving
// butterfly steps (each lane keeps the half of its registers selected by its
// lane bit, and adds the partner's other half), then plain butterflies over
// any lane bits left.  Afterwards lane c holds RPL = max(1, R/LPR) row sums in
// e[0..RPL); slot m is row row_of_lane<LPR,R>(c) + m.
template <int LPR, int R>
__device__ __forceinline__ void transpose_reduce(float (&e)[R], int c) {
  constexpr int STEPS = cmin<ilog2<R>::v, ilog2<LPR>::v>::v;
#pragma unroll
  for (int step = 0; step < STEPS; ++step) {
    const int half = R >> (step + 1);
    const int o = LPR >> (step + 1);
    const bool up = (c & o) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      float keep = up ? e[i + half] : e[i];
      float send = up ? e[i] : e[i + half];
      e[i] = keep + __shfl_xor(send, o, 64);
    }
  }
  if constexpr (R < LPR) {
#pragma unroll
    for (int o = LPR / (2 * R); o >= 1; o >>= 1) e[0] += __shfl_xor(e[0], o, 64);
  }
}

template <int LPR, int R>
__device__ __forceinline__ int row_of_lane(int c) {
  constexpr int STEPS = cmin<ilog2<R>::v, ilog2<LPR>::v>::v;
  int i = 0;
#pragma unroll
  for (int step = 0; step < STEPS; ++step)
    if (c & (LPR >> (step + 1))) i += R >> (step + 1);
  return i;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One streaming pass.  INIT: distances to the initial guess, ||x_k||^2 and
// ||g0||^2.  STEP: g' = sum c_k x_k (+ noise), distances to g', movement, ||g'||^2.
template <int V, int LPR, int R, bool INIT>
__global__ void __launch_bounds__(kTPB) weiszfeld_pass(PassArgs a) {
  constexpr int QW = 64 / LPR;          // row groups per wave
  constexpr int NRG = kWaves * QW;      // row groups per block
  constexpr int J = LPR * V;            // columns per chunk
  constexpr int RPL = R > LPR ? R / LPR : 1;   // row sums held per lane after the reduce

  __shared__ float s_red[kWaves][J];
  __shared__ float s_g[J];
  __shared__ double s_fin[2][kWaves];

  if (a.st->done) return;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int c = lane % LPR, q = lane / LPR;
  const int rg = w * QW + q;
  const int64_t K = a.K, d = a.d;

  float wt[R];
  if constexpr (!INIT) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t k = rg + (int64_t)NRG * i;
      wt[i] = k < K ? a.coef[k] : 0.f;
    }
  }

  double row_acc[RPL], row_acc2[RPL];
#pragma unroll
  for (int m = 0; m < RPL; ++m) row_acc[m] = row_acc2[m] = 0.0;
  double mv_acc = 0.0, gn_acc = 0.0;
  const int64_t nch = (d + J - 1) / J;
  for (int64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int64_t col = ch * J + (int64_t)c * V;
    const bool cval = col < d;          // V divides d: a lane's group is all-in or all-out
    float x[R][V];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t k = rg + (int64_t)NRG * i;
      if (cval && k < K) {
        load_cols<V>(a.X + k * a.ldx + col, x[i]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) x[i][v] = 0.f;
      }
    }

    float gv[V];
    if constexpr (INIT) {
      if (cval) {
#pragma unroll
        for (int v = 0; v < V; ++v) gv[v] = a.g_old[col + v];
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) gv[v] = 0.f;
      }
      if (w == 0 && q == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) gn_acc += (double)(gv[v] * gv[v]);
      }
    } else {
      // phase A: weighted column sums over this thread's rows ...
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = fmaf(wt[i], x[i][v], acc[v]);
      // ... across the wave's row groups ...
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += __shfl_xor(acc[v], o, 64);
      if (q == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) s_red[w][c * V + v] = acc[v];
      }
      __syncthreads();
      // ... and across waves; one finisher thread per column.
      if (tid < J) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < kWaves; ++ww) sum += s_red[ww][tid];
        const int64_t gj = ch * J + tid;
        float gnew = 0.f;
        if (gj < d) {
          gnew = sum;
          if (a.noise == 1) {
            gnew = fmaf(a.st->a_noise, normal1(a.seed, kStreamNoise, a.iter, a.col_off + gj), gnew);
          } else if (a.noise == 2) {
            gnew = fmaf(a.st->a_noise, a.hnoise[gj], gnew);
          }
          a.g_new[gj] = gnew;
          const float diff = a.g_old[gj] - gnew;
          mv_acc += (double)(diff * diff);
          gn_acc += (double)(gnew * gnew);
        }
        s_g[tid] = gnew;
      }
      __syncthreads();
#pragma unroll
      for (int v = 0; v < V; ++v) gv[v] = s_g[c * V + v];
    }

    // phase B: squared distances of this thread's rows to the (new) iterate.
    float e[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float t = x[i][v] - gv[v];
        s = fmaf(t, t, s);
      }
      e[i] = s;
    }
    transpose_reduce<LPR, R>(e, c);
#pragma unroll
    for (int m = 0; m < RPL; ++m) row_acc[m] += (double)e[m];
    if constexpr (INIT) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < V; ++v) s = fmaf(x[i][v], x[i][v], s);
        e[i] = s;
      }
      transpose_reduce<LPR, R>(e, c);
#pragma unroll
      for (int m = 0; m < RPL; ++m) row_acc2[m] += (double)e[m];
    }
  }

  // Per-block partials -> slab row.  Layout: [D2 (K)] [r (K), INIT only] [mv2] [gn2]
  double* out = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  const int i_c = row_of_lane<LPR, R>(c);
  constexpr int SPAN = R < LPR ? LPR / R : 1;   // lanes holding copies of one row sum
  if ((c % SPAN) == 0) {
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      const int64_t k = rg + (int64_t)NRG * (i_c + m);
      if (k < K) {
        out[k] = row_acc[m];
        if constexpr (INIT) out[K + k] = row_acc2[m];
      }
    }
  }
  const double mv = wave_sum(mv_acc), gn = wave_sum(gn_acc);
  if (lane == 0) {
    s_fin[0][w] = mv;
    s_fin[1][w] = gn;
  }
  __syncthreads();
  if (tid == 0) {
    double m = 0.0, g = 0.0;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {
      m += s_fin[0][ww];
      g += s_fin[1][ww];
    }
    const int64_t base = INIT ? 2 * K : K;
    out[base] = m;
    out[base + 1] = g;
  }
}

// Sum the per-block slab rows, column by column, in a fixed order.
__global__ void __launch_bounds__(1024) slab_reduce(const double* __restrict__ slab, int nb,
                                                    int64_t S, double* __restrict__ sums,
                                                    const KState* st) {
  if (st->done) return;
  __shared__ double red[32][33];
  const int cx = threadIdx.x & 31, by = threadIdx.x >> 5;
  const int64_t j = (int64_t)blockIdx.x * 32 + cx;
  double acc = 0.0;
  if (j < S)
    for (int b = by; b < nb; b += 32) acc += slab[(int64_t)b * S + j];
  red[by][cx] = acc;
  __syncthreads();
  if (by == 0 && j < S) {
    double s = 0.0;
#pragma unroll
    for (int y = 0; y < 32; ++y) s += red[y][cx];
    sums[j] = s;
  }
}

__device__ double block_sum(double v, double* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += scratch[i];
  return s;
}

__device__ __forceinline__ float clamp_dist(double d2, float eps) {
  // dist = max(1e-4, ||x_k - g||) in fp32 with torch.max's NaN propagation (M:178)
  const float dist = (float)sqrt(d2);
  return dist != dist ? dist : fmaxf(dist, eps);
}

// The K-space step: the tol test of the pass that just finished, then the
// next pass's coefficients.  One block.
__global__ void __launch_bounds__(1024) kspace_step(KspaceArgs a) {
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
  if (a.has_noise) nd = a.noise_src == 0 ? a.noise_sd * (double)normal1(a.seed, kStreamNoise, (uint64_t)it, (uint64_t)a.d_total)
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
// Two-pass path (any K): column pass for g', row pass for the distances.

__global__ void __launch_bounds__(256) twopass_sum(const float* __restrict__ X, int64_t K,
                                                   int64_t d, int64_t ldx,
                                                   const float* __restrict__ g_old,
                                                   float* __restrict__ g_new,
                                                   const float* __restrict__ coef,
                                                   const KState* st, int noise,
                                                   const float* __restrict__ hnoise,
                                                   uint64_t seed, int64_t iter, int64_t col_off,
                                                   double* slab, int64_t S, int64_t base) {
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
    slab[(int64_t)blockIdx.x * S + base] = m;
    slab[(int64_t)blockIdx.x * S + base + 1] = g;
  }
}

// One block per (row, column slice): partial squared distance (and ||x||^2 at init).
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

// ---------------------------------------------------------------------------
// Launch plumbing.

template <int V, int LPR, int R>
static hipError_t launch_cfg(bool init, int grid, const PassArgs& a, hipStream_t s) {
  if (init)
    hipLaunchKernelGGL((weiszfeld_pass<V, LPR, R, true>), dim3(grid), dim3(kTPB), 0, s, a);
  else
    hipLaunchKernelGGL((weiszfeld_pass<V, LPR, R, false>), dim3(grid), dim3(kTPB), 0, s, a);
  return hipGetLastError();
}

template <int V, int LPR, int R>
static int occ_cfg(bool init) {
  int n = 0;
  hipError_t e = init ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                            &n, weiszfeld_pass<V, LPR, R, true>, kTPB, 0)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                            &n, weiszfeld_pass<V, LPR, R, false>, kTPB, 0);
  return (e == hipSuccess && n > 0) ? n : 1;
}

#define GMK_FOR_EACH_LR(X_, V_)                                                              \
  X_(V_, 64, 1) X_(V_, 64, 2) X_(V_, 64, 4) X_(V_, 32, 4) X_(V_, 16, 4) X_(V_, 8, 4)          \
  X_(V_, 8, 8) X_(V_, 8, 16)

hipError_t launch_pass(const PassCfg& cfg, bool init, int grid, const PassArgs& a, hipStream_t s) {
#define GMK_CASE(V_, L_, R_) \
  if (cfg.V == V_ && cfg.LPR == L_ && cfg.R == R_) return launch_cfg<V_, L_, R_>(init, grid, a, s);
  GMK_FOR_EACH_LR(GMK_CASE, 4)
  GMK_FOR_EACH_LR(GMK_CASE, 2)
  GMK_FOR_EACH_LR(GMK_CASE, 1)
#undef GMK_CASE
  return hipErrorInvalidValue;
}

int pass_blocks_per_cu(const PassCfg& cfg, bool init) {
#define GMK_CASE(V_, L_, R_) \
  if (cfg.V == V_ && cfg.LPR == L_ && cfg.R == R_) return occ_cfg<V_, L_, R_>(init);
  GMK_FOR_EACH_LR(GMK_CASE, 4)
  GMK_FOR_EACH_LR(GMK_CASE, 2)
  GMK_FOR_EACH_LR(GMK_CASE, 1)
#undef GMK_CASE
  return 1;
}

hipError_t launch_slab_reduce(const double* slab, int nb, int64_t S, double* sums,
                              const KState* st, hipStream_t s) {
  const int grid = (int)((S + 31) / 32);
  hipLaunchKernelGGL(slab_reduce, dim3(grid), dim3(1024), 0, s, slab, nb, S, sums, st);
  return hipGetLastError();
}

hipError_t launch_kspace(const KspaceArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(kspace_step, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

int twopass_blocks(int64_t K, int64_t d, int num_cu) {
  const int64_t want = (d + 255) / 256;
  const int64_t cap = (int64_t)num_cu * 8;
  return (int)(want < cap ? (want > 0 ? want : 1) : cap);
}

// Two-pass driver used by api.hip: writes the (K+2) / (2K+2) sums vector.
hipError_t launch_twopass(bool init, const float* X, int64_t K, int64_t d, int64_t ldx,
                          const float* g_old, float* g_new, const float* coef, const KState* st,
                          int noise, const float* hnoise, uint64_t seed, int64_t iter,
                          int64_t col_off, double* slab, int nb, double* sums, hipStream_t s) {
  const int64_t base = init ? 2 * K : K;
  hipLaunchKernelGGL(twopass_sum, dim3(nb), dim3(256), 0, s, X, K, d, ldx, g_old,
                     init ? nullptr : g_new, coef, st, noise, hnoise, seed, iter, col_off, slab,
                     (int64_t)2, (int64_t)0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(twopass_dist, dim3((unsigned)K), dim3(256), 0, s, X, K, d, ldx,
                     init ? g_old : g_new, init, st, sums);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_slab_reduce(slab, nb, 2, sums + base, st, s);
}
}  // namespace gmk
