// Register-resident persistent Weiszfeld for small problems (BASELINE C1/C2:
// the reference's own K = 50 x d = 7850 MNIST aggregation, 1000 AirComp
// iterations per training step, 96 % of the reference's step time).
//
// At that size a launch-per-phase loop is launch-bound (3 kernels + polls per
// iteration).  Here ONE cooperative launch runs every iteration: each block
// owns one J-column chunk of X, loaded into VGPRs once; per iteration it
//   1. reads every block's partials of the previous pass from a double-buffered
//      slab and reduces them in a fixed order (every block computes the
//      identical K-space step redundantly: no second barrier, no broadcast),
//   2. takes the tol test (M:182) and forms the next coefficients (M:178-179,
//      or the OMA2 fold for gm, M:146-155 / M:401-412, Philox draws),
//   3. runs phases A/B of the streaming pass on its register tile,
//   4. publishes its partials and meets the others at ONE grid barrier.
// The iterate never leaves the chip until the final write.  Draw keys are the
// same as the launch-per-phase path's, so both give the same gm results.
#include "device_util.h"
#include "gmagg_internal.h"
#include "philox.h"

#ifndef GMK_RES_SLEEP
#define GMK_RES_SLEEP 1   // spin back-off of the grid barrier (A/B knob)
#endif

// -DGMK_RES_PROF: block 0 / thread 0 accumulates s_memrealtime (100 MHz) deltas per
// phase of the iteration and prints them at the end (timing probe builds only).
#ifdef GMK_RES_PROF
#define RES_T(i)                                                        \
  if (blockIdx.x == 0 && threadIdx.x == 0) {                            \
    const uint64_t now_ = __builtin_amdgcn_s_memrealtime();             \
    prof_[i] += now_ - prev_;                                           \
    prev_ = now_;                                                       \
  }
#else
#define RES_T(i)
#endif

namespace gmk {

// (ResArgs: gmagg_internal.h)

constexpr uint64_t kBarrierTicks = 200000000ull;   // 2 s at the 100 MHz real-time clock

// Grid barrier: arrival counter + generation word, agent-scope release before
// arriving and acquire after leaving (cdna_hip_programming.md §6 G16).  The spin
// is bounded in WALL time (s_memrealtime, 100 MHz: kBarrierTicks = 2 s, so a
// time-sliced GPU does not trip it by spinning slowly): on timeout a flag is
// raised, every block gives up, and the host reruns the problem on the
// streaming path (api.hip run_resident).
__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned nblocks, unsigned& gen,
                                          int* s_ok) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ok = 1;
    const unsigned g = gen;
    if (__hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        nblocks - 1) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&bar[1], g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
#if GMK_RES_SLEEP > 0
        __builtin_amdgcn_s_sleep(GMK_RES_SLEEP);
#endif
        if (((++spins & 1023u) == 0 &&
             __builtin_amdgcn_s_memrealtime() - t0 > kBarrierTicks) ||
            __hip_atomic_load(&bar[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          __hip_atomic_store(&bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    gen = g + 1;
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

template <int V, int NW, int LPR, int R>
__global__ void __launch_bounds__(NW * 64) weiszfeld_resident(ResArgs a) {
  constexpr int QW = 64 / LPR;
  constexpr int NRG = NW * QW;
  constexpr int J = LPR * V;
  constexpr int RPL = R > LPR ? R / LPR : 1;
  constexpr int SPAN = R < LPR ? LPR / R : 1;
  constexpr int KMAX = NRG * R;

  __shared__ float s_red[NW][J];
  __shared__ float s_g[J];
  __shared__ float s_coef[KMAX];
  __shared__ double s_d2[KMAX];
  __shared__ double s_r[KMAX];
  __shared__ double s_fin[2][NW];
  __shared__ double s_tot[2];
  __shared__ double s_part[NW * 64];
  __shared__ double scratch[16];
  __shared__ float s_anoise;
  __shared__ int s_ok;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane % LPR, q = lane / LPR;
  const int rg = w * QW + q;
  const int64_t K = a.K, d = a.d;
  const unsigned nb = gridDim.x;
  const int64_t S = 2 * K + 2;
  const int64_t ch = blockIdx.x;
  const int64_t col = ch * J + (int64_t)c * V;
  const bool cval = col < d;
  const int64_t gj = ch * J + tid;
  const bool fin = tid < J && gj < d;
  unsigned gen = 0;

  // ---- the block's tile: loaded once, resident for the whole call
  float x[R][V];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int64_t k = rg + (int64_t)NRG * i;
#pragma unroll
    for (int v = 0; v < V; ++v) x[i][v] = (cval && k < K) ? a.X[k * a.ldx + col + v] : 0.f;
  }
  float gcur = fin ? a.guess0[gj] : 0.f;       // finisher thread: the iterate at column gj

  const int i_c = row_of_lane<LPR, R>(c);
  auto publish = [&](int buf, const double* racc, const double* racc2, double mv, double gn) {
    double* out = a.slab + ((int64_t)buf * nb + blockIdx.x) * S;
    if ((c % SPAN) == 0) {
#pragma unroll
      for (int m = 0; m < RPL; ++m) {
        const int64_t k = rg + (int64_t)NRG * (i_c + m);
        if (k < K) {
          out[k] = racc[m];
          if (racc2) out[K + k] = racc2[m];
        }
      }
    }
    mv = wave_sum(mv);
    gn = wave_sum(gn);
    if (lane == 0) {
      s_fin[0][w] = mv;
      s_fin[1][w] = gn;
    }
    __syncthreads();
    if (tid == 0) {
      double m = 0.0, g = 0.0;
      for (int ww = 0; ww < NW; ++ww) {
        m += s_fin[0][ww];
        g += s_fin[1][ww];
      }
      out[2 * K] = m;
      out[2 * K + 1] = g;
    }
  };

  // ---- INIT: distances to g_0, ||x_k||^2 and ||g_0||^2 -> slab buffer 0
  {
    float gv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) gv[v] = cval ? a.guess0[col + v] : 0.f;
    float e[R], e2[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float t = x[i][v] - gv[v];
        s1 = fmaf(t, t, s1);
        s2 = fmaf(x[i][v], x[i][v], s2);
      }
      e[i] = s1;
      e2[i] = s2;
    }
    transpose_reduce<LPR, R>(e, c);
    transpose_reduce<LPR, R>(e2, c);
    double racc[RPL], racc2[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) {
      racc[m] = e[m];
      racc2[m] = e2[m];
    }
    publish(0, racc, racc2, 0.0, fin ? (double)(gcur * gcur) : 0.0);
  }
  if (!grid_sync(a.bar, nb, gen, &s_ok)) return;

  int64_t it = 0;
  double last_mv = NAN;
  int conv = 0;
#ifdef GMK_RES_PROF
  uint64_t prof_[6] = {0, 0, 0, 0, 0, 0};
  uint64_t prev_ = __builtin_amdgcn_s_memrealtime();
#endif
  for (;; ++it) {
    // (1) reduce the previous pass's partials, same order in every block: the
    // slab columns needed (D2, at it = 0 also r, then mv2 / gn2) are spread over
    // G thread groups that each sum every G-th block row; the G partials are
    // then combined in LDS in group order (deterministic, and G loads in flight
    // per column instead of nb dependent ones).
    {
      const double* sl = a.slab + (int64_t)(it & 1) * nb * S;
      const int64_t ncol = (it == 0 ? 2 * K : K) + 2;      // [D2 | (r) | mv2 gn2]
      const int64_t span = ncol <= 64 ? 64 : ncol <= 128 ? 128 : ncol <= 256 ? 256
                          : ncol <= 512 ? 512 : 1024;
      const int G = (int)(blockDim.x / span) > 0 ? (int)(blockDim.x / span) : 1;
      for (int64_t col0 = 0; col0 < ncol; col0 += span) {
        const int g = tid / (int)span;
        const int64_t cc = col0 + tid % span;
        const int64_t src = cc < ncol - 2 ? cc : 2 * K + (cc - (ncol - 2));
        double s = 0.0;
        if (g < G && cc < ncol)
          for (unsigned b = g; b < nb; b += G) s += sl[(int64_t)b * S + src];
        __syncthreads();
        if (g < G) s_part[g * span + tid % span] = s;
        __syncthreads();
        if (tid < span && col0 + tid < ncol) {
          double t = 0.0;
          for (int gg = 0; gg < G; ++gg) t += s_part[gg * span + tid];
          const int64_t c2 = col0 + tid;
          if (c2 < K) s_d2[c2] = t;
          else if (c2 < ncol - 2) s_r[c2 - K] = t;
          else s_tot[c2 - (ncol - 2)] = t;
        }
      }
    }
    __syncthreads();
    RES_T(0)
    // (2) tol test of the pass that produced g_it (M:180-183)
    if (it >= 1) {
      const float mv = (float)sqrt(s_tot[0]);
      last_mv = (double)mv;
      if (mv <= a.tol) { conv = 1; break; }
    }
    if (it == a.maxiter) break;

    // (3) coefficients for pass `it`
    if (a.mode == 0) {
      double wsum = 0.0;
      for (int64_t k = tid; k < K; k += blockDim.x) wsum += 1.0 / (double)clamp_dist(s_d2[k], a.eps);
      const double W = block_sum(wsum, scratch);
      for (int64_t k = tid; k < K; k += blockDim.x)
        s_coef[k] = (float)((1.0 / (double)clamp_dist(s_d2[k], a.eps)) / W);
      if (tid == 0) s_anoise = 0.f;
    } else {
      const float s = sqrtf((float)(s_tot[1] / (double)d));      // M:146
      const float thr = (s * s) * 500.0f;                         // M:152
      const double s2 = (double)s * (double)s;
      double csum = 0.0;
      for (int64_t k = tid; k < K; k += blockDim.x) {
        float n4[4];
        normal4(a.seed, kStreamChannel, (uint64_t)it, (uint64_t)k, n4);
        const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
        const float h2 = hr * hr + hi * hi;                       // M:403
        const float dist = clamp_dist(s_d2[k], a.eps);
        const double dd = (double)dist;
        const double p = (s_r[k] + s2) / (dd * dd * (double)(d + 1)) / (double)h2;   // M:404
        const double pup = p != p ? p : fmax(p, (double)thr);     // M:405
        const double ck = sqrt(a.P_max / pup) / dd;               // M:407
        s_coef[k] = (float)ck;
        csum += ck;
      }
      const double Sc = block_sum(csum, scratch);
      const double nd = a.has_noise ? a.noise_sd * (double)normal1(a.seed, kStreamNoise,
                                                                   (uint64_t)it, (uint64_t)d)
                                    : 0.0;
      const double scale = (double)s / ((double)s * Sc + nd);     // M:153-155
      __syncthreads();
      for (int64_t k = tid; k < K; k += blockDim.x) s_coef[k] = (float)((double)s_coef[k] * scale);
      if (tid == 0) s_anoise = a.has_noise ? (float)(scale * a.noise_sd) : 0.f;
    }
    __syncthreads();
    RES_T(1)

    // (4) phase A on the resident tile
    float wt[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t k = rg + (int64_t)NRG * i;
      wt[i] = k < K ? s_coef[k] : 0.f;
    }
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = fmaf(wt[i], x[i][v], acc[v]);
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] += __shfl_xor(acc[v], o, 64);
    if (q == 0) {
#pragma unroll
      for (int v = 0; v < V; ++v) s_red[w][c * V + v] = acc[v];
    }
    __syncthreads();
    double mvp = 0.0, gnp = 0.0;
    if (tid < J) {
      float gnew = 0.f;
      if (fin) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sum += s_red[ww][tid];
        gnew = sum;
        if (a.has_noise && a.mode == 1)
          gnew = fmaf(s_anoise, normal1(a.seed, kStreamNoise, (uint64_t)it, (uint64_t)gj), gnew);
        const float diff = gcur - gnew;
        mvp = (double)(diff * diff);
        gnp = (double)(gnew * gnew);
        gcur = gnew;
      }
      s_g[tid] = gnew;
    }
    __syncthreads();
    RES_T(2)
    // (5) phase B: distances to the new iterate
    float gv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) gv[v] = s_g[c * V + v];
    float e[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float s1 = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float t = x[i][v] - gv[v];
        s1 = fmaf(t, t, s1);
      }
      e[i] = s1;
    }
    transpose_reduce<LPR, R>(e, c);
    double racc[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) racc[m] = e[m];
    RES_T(3)
    publish((int)((it + 1) & 1), racc, nullptr, mvp, gnp);
    RES_T(4)
    if (!grid_sync(a.bar, nb, gen, &s_ok)) return;
    RES_T(5)
  }
#ifdef GMK_RES_PROF
  if (blockIdx.x == 0 && threadIdx.x == 0)
    printf("GMK_RES_PROF nb=%u iters=%ld ns/iter: reduce %.0f coef %.0f phaseA %.0f phaseB %.0f "
           "publish %.0f barrier %.0f\n", nb, (long)it, 10.0 * prof_[0] / it, 10.0 * prof_[1] / it,
           10.0 * prof_[2] / it, 10.0 * prof_[3] / it, 10.0 * prof_[4] / it, 10.0 * prof_[5] / it);
#endif

  if (fin) a.out[gj] = gcur;
  if (blockIdx.x == 0 && tid == 0) {
    a.st->iters = it;
    a.st->last_movement = last_mv;
    a.st->converged = conv;
    a.st->done = 1;
  }
}

// ---------------------------------------------------------------------------

template <int V, int NW, int LPR, int R>
static const void* res_fn() {
  return reinterpret_cast<const void*>(&weiszfeld_resident<V, NW, LPR, R>);
}

static const void* resident_kernel(const PassCfg& cfg) {
#define GMK_RES(V_, W_, L_, R_) \
  if (cfg.V == V_ && cfg.NW == W_ && cfg.LPR == L_ && cfg.R == R_) return res_fn<V_, W_, L_, R_>();
#define GMK_RES_V(V_)                                                                         \
  GMK_RES(V_, 16, 64, 1) GMK_RES(V_, 16, 64, 2) GMK_RES(V_, 16, 64, 4) GMK_RES(V_, 16, 64, 8)   \
  GMK_RES(V_, 16, 32, 8) GMK_RES(V_, 16, 16, 8) GMK_RES(V_, 16, 8, 8) GMK_RES(V_, 16, 4, 8)
  GMK_RES_V(4)
  GMK_RES_V(2)
  GMK_RES_V(1)
#undef GMK_RES_V
#undef GMK_RES
  return nullptr;
}

int resident_max_blocks(const PassCfg& cfg, int num_cu) {
  const void* fn = resident_kernel(cfg);
  int n = 0;
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, cfg.NW * 64, 0) != hipSuccess)
    return 0;
  return n * num_cu;
}

hipError_t launch_resident(const PassCfg& cfg, int grid, const ResArgs& a, hipStream_t s) {
  const void* fn = resident_kernel(cfg);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<ResArgs*>(&a)};
  return hipLaunchCooperativeKernel(fn, dim3(grid), dim3(cfg.NW * 64), args, 0, s);
}

}  // namespace gmk
