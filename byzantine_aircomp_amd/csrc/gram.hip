// Gram-space Weiszfeld (north_star's second design; BASELINE config C4).
//
// With p = the initial guess and x'_k = x_k - p, every Weiszfeld iterate of gm2
// (M:162-184) lies in p + span{x'_k}: g_t = p + X'^T a_t with sum(a_t) = 1 for t >= 1
// (a_0 = 0).  Given G = X' X'^T (K x K) the whole loop runs in K-space:
//   D_k   = ||x_k - g||^2   = G_kk - 2 (G a)_k + a^T G a            (M:174)
//   a'    = (1/max(1e-4, sqrt D)) normalised                        (M:178-179)
//   ||g - g'||^2 = (a - a')^T G (a - a')                             (M:180)
// and one final pass writes g = p + X'^T a = sum_k a_k x_k.  X is read twice
// per aggregation (Gram + final), instead of (n+1) times by the streaming pass.
//
// gram_partial: G = X' X'^T on v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains),
// centering fused into the LDS staging.  K padded to KP = 32*KT; only the upper
// triangle of the KT x KT tile grid is computed.  Wave w owns tile rows w and
// KT-1-w (KT+1 tiles: balanced), so for KT = 8 each of the 4 waves issues 9
// MFMAs per 2 columns.  Blocks own disjoint column ranges; fp32 partials per
// block go to a slab that gram_reduce sums in fp64 (fixed order).
#include "device_util.h"
#include "gmagg_internal.h"

namespace gmk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGramJC = 64;   // columns per LDS stage

template <int KT>
struct GramShape {
  static constexpr int KP = 32 * KT;
  static constexpr int TILES = KT * (KT + 1) / 2;           // upper-triangle 32x32 tiles
  static constexpr int PER_WAVE = KT == 1 ? 1 : KT + 1;     // tiles per active wave
  static constexpr int ACTIVE = KT == 1 ? 1 : KT / 2;       // waves holding tiles
  static constexpr int S = KP + 1;                          // LDS column stride (floats)
  static constexpr int ROWS_PER_THREAD = KP / 16;           // 16 lanes per row x 16 B
};

// Tile t of wave w: (row tile a, column tile b), a <= b.
template <int KT>
__device__ __forceinline__ void wave_tile(int w, int t, int& a, int& b) {
  if (KT == 1) { a = 0; b = 0; return; }
  const int first = KT - w;            // tiles of row w: (w, w..KT-1)
  if (t < first) { a = w; b = w + t; }
  else { a = KT - 1 - w; b = a + (t - first); }
}

// Canonical index of upper-triangle tile (a, b), a <= b.
__host__ __device__ __forceinline__ int tri_index(int a, int b, int KT) {
  return a * KT - a * (a - 1) / 2 + (b - a);
}

template <int KT>
__global__ void __launch_bounds__(256) gram_partial(const float* __restrict__ X, int64_t K,
                                                    int64_t d, int64_t ldx,
                                                    const float* __restrict__ p,
                                                    int64_t cols_per_block,
                                                    float* __restrict__ slab) {
  using Sh = GramShape<KT>;
  constexpr int S = Sh::S, RPT = Sh::ROWS_PER_THREAD, NT = Sh::PER_WAVE;
  __shared__ float lds[2][kGramJC * S];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = tid & 15;          // float4 column group within the 64-column stage
  const int r0 = tid >> 4;          // first row; rows r0 + 16*i
  const int64_t c_begin = (int64_t)blockIdx.x * cols_per_block;
  const int64_t c_end = c_begin + cols_per_block < d ? c_begin + cols_per_block : d;
  const int nstage = c_begin < c_end ? (int)((c_end - c_begin + kGramJC - 1) / kGramJC) : 0;

  // Two-level fp32 accumulation: a 64-column stage accumulates in `acc` (MFMA
  // chains of 32 steps), then is added to `tot`: the long sum over a block's
  // columns sees ~cols/64 roundings instead of cols/2.
  f32x16 acc[NT], tot[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = tot[t][e] = 0.f;

  f32x4 stage[RPT];
  f32x4 pc;
  auto fetch = [&](int s) {
    const int64_t col = c_begin + (int64_t)s * kGramJC + cg * 4;
    const bool cval = col < c_end;                     // d % 4 == 0: groups all-in/out
    pc = cval ? *reinterpret_cast<const f32x4*>(p + col) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int64_t r = r0 + 16 * i;
      stage[i] = (cval && r < K)
                     ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(X + r * ldx + col))
                     : pc;                             // padded rows centre to exactly 0
    }
  };
  auto commit = [&](int buf) {                         // centre + transpose into [col][row]
    float* L = lds[buf];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + 16 * i;
#pragma unroll
      for (int v = 0; v < 4; ++v) L[(cg * 4 + v) * S + r] = stage[i][v] - pc[v];
    }
  };

  if (nstage > 0) {
    fetch(0);
    commit(0);
  }
  __syncthreads();
  const int half = lane >> 5, li = lane & 31;
  for (int s = 0; s < nstage; ++s) {
    const int buf = s & 1;
    if (s + 1 < nstage) fetch(s + 1);                  // in flight under the MFMAs
    if (w < Sh::ACTIVE) {
      const float* L = lds[buf];
#pragma unroll 4
      for (int ks = 0; ks < kGramJC; ks += 2) {
        const float* colp = L + (ks + half) * S + li;  // A[i][k] / B[k][j]: row li, col ks+half
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          int a, b;
          wave_tile<KT>(w, t, a, b);
          const float fa = colp[a * 32];
          const float fb = colp[b * 32];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, fb, acc[t], 0, 0, 0);
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        tot[t] += acc[t];
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
      }
    }
    __syncthreads();
    if (s + 1 < nstage) commit(buf ^ 1);
    __syncthreads();
  }

  if (w < Sh::ACTIVE) {
    float* out = slab + (int64_t)blockIdx.x * Sh::TILES * 1024;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      int a, b;
      wave_tile<KT>(w, t, a, b);
      float* o = out + tri_index(a, b, KT) * 1024;
#pragma unroll
      for (int e = 0; e < 16; ++e) o[e * 64 + lane] = tot[t][e];
    }
  }
}

// Sum the fp32 block partials in fp64 (fixed order) and unpack the upper
// triangle into a full symmetric G[KP][KP].  Element e of a tile: register
// reg = e / 64, lane = e % 64 -> row (reg&3) + 8*(reg>>2) + 4*(lane>>5), col lane&31.
__global__ void __launch_bounds__(256) gram_reduce(const float* __restrict__ slab, int nb,
                                                   int KT, double* __restrict__ G) {
  const int tiles = KT * (KT + 1) / 2;
  const int64_t n = (int64_t)tiles * 1024;
  const int KP = 32 * KT;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += (double)slab[(int64_t)b * n + e];
    const int tix = (int)(e >> 10), el = (int)(e & 1023);
    int a = 0;
    while (tri_index(a, KT - 1, KT) < tix) ++a;        // row tile of this triangle index
    const int bt = a + (tix - tri_index(a, a, KT));
    const int reg = el >> 6, ln = el & 63;
    const int row = a * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (ln >> 5);
    const int col = bt * 32 + (ln & 31);
    G[(int64_t)row * KP + col] = s;
    G[(int64_t)col * KP + row] = s;
  }
}

// The Weiszfeld loop in K-space, fp64, all iterations in one launch.  Writes
// the final normalised weights (fp32) for the closing pass and the KState.
__global__ void __launch_bounds__(1024) gram_solve(const double* __restrict__ G, int KP, int64_t K,
                                                   int64_t maxiter, float tol, float eps,
                                                   double* __restrict__ alpha,
                                                   double* __restrict__ u, float* coef,
                                                   KState* st) {
  __shared__ double scratch[16];
  __shared__ int s_stop;
  const int tid = threadIdx.x;
  // a_0 = 0 (g_0 = p): u = G a = 0, a^T u = 0
  for (int64_t k = tid; k < K; k += blockDim.x) { alpha[k] = 0.0; u[k] = 0.0; }
  double aTu = 0.0;
  __syncthreads();
  int64_t it = 0;
  double last_mv = NAN;
  int conv = 0;
  for (; it < maxiter; ++it) {
    // next weights from D_k = G_kk - 2 u_k + a^T u   (clamped at 0 against cancellation)
    double wsum = 0.0;
    for (int64_t k = tid; k < K; k += blockDim.x) {
      const double D = G[k * KP + k] - 2.0 * u[k] + aTu;
      wsum += 1.0 / (double)clamp_dist(D > 0.0 ? D : (D != D ? D : 0.0), eps);
    }
    const double W = block_sum(wsum, scratch);
    // a' into coef (fp32 copy) and the delta; u' = G a' by 4 lanes per row
    for (int64_t k = tid; k < K; k += blockDim.x) {
      const double D = G[k * KP + k] - 2.0 * u[k] + aTu;
      const double an = (1.0 / (double)clamp_dist(D > 0.0 ? D : (D != D ? D : 0.0), eps)) / W;
      coef[k] = (float)an;
    }
    __syncthreads();
    double part_mv = 0.0, part_atu = 0.0;
    for (int64_t k0 = tid >> 2; k0 < K; k0 += blockDim.x >> 2) {
      double s = 0.0;
      for (int64_t j = tid & 3; j < K; j += 4) s += G[k0 * KP + j] * (double)coef[j];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if ((tid & 3) == 0) {
        const double an = (double)coef[k0];
        const double dlt = alpha[k0] - an;
        part_mv += dlt * (u[k0] - s);       // (a - a')^T (G a - G a')
        part_atu += an * s;
        alpha[k0] = an;
        u[k0] = s;
      }
    }
    const double mv2 = block_sum(part_mv, scratch);
    aTu = block_sum(part_atu, scratch);
    const float mv = (float)sqrt(mv2 > 0.0 ? mv2 : (mv2 != mv2 ? mv2 : 0.0));
    last_mv = (double)mv;
    if (tid == 0) s_stop = mv <= tol ? 1 : 0;
    __syncthreads();
    if (s_stop) { conv = 1; ++it; break; }
  }
  if (tid == 0) {
    st->iters = it;
    st->last_movement = last_mv;
    st->converged = conv;
    st->done = 0;   // let the closing pass run
  }
}

template <int KT>
static hipError_t launch_gram_kt(const float* X, int64_t K, int64_t d, int64_t ldx,
                                 const float* p, int nb, int64_t cpb, float* slab, hipStream_t s) {
  hipLaunchKernelGGL(gram_partial<KT>, dim3(nb), dim3(256), 0, s, X, K, d, ldx, p, cpb, slab);
  return hipGetLastError();
}

int gram_kt(int64_t K) { return K <= 32 ? 1 : K <= 64 ? 2 : K <= 128 ? 4 : K <= 256 ? 8 : 0; }

size_t gram_slab_floats(int KT, int nb) { return (size_t)nb * (KT * (KT + 1) / 2) * 1024; }

hipError_t launch_gram(const float* X, int64_t K, int64_t d, int64_t ldx, const float* p, int nb,
                       float* slab, double* G, hipStream_t s) {
  const int KT = gram_kt(K);
  const int64_t cpb = ((d + nb - 1) / nb + kGramJC - 1) / kGramJC * kGramJC;
  hipError_t e;
  switch (KT) {
    case 1: e = launch_gram_kt<1>(X, K, d, ldx, p, nb, cpb, slab, s); break;
    case 2: e = launch_gram_kt<2>(X, K, d, ldx, p, nb, cpb, slab, s); break;
    case 4: e = launch_gram_kt<4>(X, K, d, ldx, p, nb, cpb, slab, s); break;
    case 8: e = launch_gram_kt<8>(X, K, d, ldx, p, nb, cpb, slab, s); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  const int64_t n = (int64_t)(KT * (KT + 1) / 2) * 1024;
  hipLaunchKernelGGL(gram_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slab, nb, KT,
                     G);
  return hipGetLastError();
}

hipError_t launch_gram_solve(const double* G, int KP, int64_t K, int64_t maxiter, float tol,
                             float eps, double* alpha, double* u, float* coef, KState* st,
                             hipStream_t s) {
  hipLaunchKernelGGL(gram_solve, dim3(1), dim3(1024), 0, s, G, KP, K, maxiter, tol, eps, alpha, u,
                     coef, st);
  return hipGetLastError();
}

}  // namespace gmk
