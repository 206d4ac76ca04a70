// OMA per-client pre-noise (MNIST_Air_weight.py:385-394) and the seeded
// synthetic client-update generator used by the benchmark.
//
// OMA:  X[k, j] += (h_re[k] * n_re[k, j] + h_im[k] * n_im[k, j]) / (h_re[k]^2 + h_im[k]^2)
// One read + one write of X (8 B per element); the draws either come from the
// caller (the reference's own CPU-generator values, bit-exact) or from Philox.
#include <algorithm>

#include "gmagg_internal.h"
#include "philox.h"

namespace gmk {

// Host-injected draws.  fp contraction is off so the fp32 op order is the
// reference's: mul, mul, add, mul, mul, add, div, add (M:393-394).
__global__ void __launch_bounds__(256) oma_apply(float* __restrict__ X, int64_t K, int64_t d,
                                                 int64_t ldx, const float* __restrict__ hr,
                                                 const float* __restrict__ hi,
                                                 const float* __restrict__ nr,
                                                 const float* __restrict__ ni) {
#pragma clang fp contract(off)
  const int64_t n = K * d;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = e / d, j = e - k * d;
    const float a = hr[k], b = hi[k];
    const float num = a * nr[e] + b * ni[e];
    const float den = a * a + b * b;
    float* p = X + k * ldx + j;
    *p = *p + num / den;
  }
}

// Philox draws (the production path: at C3 size one OMA call adds 1.1e10 noise
// values).  The reference adds (h_re n_re + h_im n_im) / |h|^2 with n_re, n_im ~
// N(0, var) independent (M:389-394): a sum of independent zero-mean normals, i.e.
// exactly N(0, var |h|^2) / |h|^2 = N(0, var / |h|^2).  So one standard normal z per
// element suffices: X += (sd / |h_k|) z, the same distribution as the reference's
// two draws at half the random numbers.  Client k's channel h_k ~ CN(0, 1) is the
// Philox block keyed (row k); element (k, global column c) takes normal c & 3 of
// the block keyed (row k, c >> 2): one Philox block and two Box-Muller pairs per 4
// elements, and a d-shard regenerates its own columns from its offset.
// blockIdx.y walks rows (the row scale once per thread and row); a thread owns
// groups of 4 columns (one float4 read + write when aligned).
// wshift > 0: X is in the panel layout [ceil(d/W)][K][W], W = 1 << wshift, ldx = the
// panel stride (elements); the draws are keyed the same way, so panels and rows agree.
// ALIGNED: col_off % 4 == 0 (every unsharded call and the 256-aligned shards), so
// a group of 4 columns is exactly one Philox block; otherwise (the shift is the same
// for every group of the launch) a group spans two blocks.
// Batched (BASELINE C5, the reference's `--agg gm2 --var v` pre-noise on P
// independent problems): rows r = p * Kp + k of P problems [P][Kp] at X + p * pstride;
// problem p is keyed with seed + p * kSeedStride (row k, as a single call would).
template <bool ALIGNED, bool VEC4>
__global__ void __launch_bounds__(256) oma_philox(float* __restrict__ X, int64_t K, int64_t d,
                                                  int64_t ldx, int64_t col_off, float sd,
                                                  uint64_t seed0, int wshift, int64_t Kp,
                                                  int64_t pstride) {
  // x + scale*z rounds the same (no FMA) on the float4 and the scalar path, in
  // every instantiation: a shard or a layout must reproduce the others bit for bit
#pragma clang fp contract(off)
  typedef float f4 __attribute__((ext_vector_type(4)));
#ifndef GMK_OMA_U
#define GMK_OMA_U 4
#endif
  constexpr int U = GMK_OMA_U;                // groups per thread per step: U=4 17.4 ms vs U=2 17.7 at C3 size
  const int64_t G = (d + 3) / 4;
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r = blockIdx.y; r < K; r += gridDim.y) {
    const int64_t pi = r / Kp, k = r - pi * Kp;
    const uint64_t seed = seed0 + (uint64_t)pi * kSeedStride;
    const float scale = oma_row_scale(seed, (uint64_t)k, sd);
    float* row = (wshift ? X + (k << wshift) : X + k * ldx) + pi * pstride;
    // Step s covers groups g0 + q*T (q < U).  Step s+1's loads are issued before
    // step s's Philox math and stores, so each thread keeps U loads in flight
    // across its whole loop (the draws do not depend on the data).
    auto load = [&](int64_t g0, f4* v, float** rp, bool* full) {
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int64_t j0 = 4 * (g0 + q * T);
        // element j of this row: row[j] (rows), or panel j >> wshift, slot j & (W-1)
        // (panels; W % 4 == 0, so a group of 4 never straddles panels)
        rp[q] = wshift ? row + (j0 >> wshift) * ldx + (j0 & ((1 << wshift) - 1)) - j0 : row;
        full[q] = VEC4 && j0 + 4 <= d;
        // branch-free: a partial group loads the (aligned, valid) row start instead
        // and takes the scalar path below.  A conditional load would merge into
        // v[q] through a copy that waits for the load (vmcnt(0)), serialising them.
        if constexpr (VEC4)
          v[q] = __builtin_nontemporal_load(reinterpret_cast<f4*>(full[q] ? rp[q] + j0 : row));
      }
    };
    f4 v[U];
    float* rp[U];
    bool full[U];
    int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g0 < G) load(g0, v, rp, full);
    for (; g0 < G; g0 += U * T) {
      f4 nv[U];
      float* nrp[U];
      bool nfull[U] = {};
      if (g0 + U * T < G) load(g0 + U * T, nv, nrp, nfull);
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int64_t j0 = 4 * (g0 + q * T);
        if (j0 >= d) break;
        const uint64_t c0 = (uint64_t)(col_off + j0);
        float z[8];
        normal4_hw(seed, kStreamOmaNoise, (uint64_t)k, c0 >> 2, z);
        float zz[4];
        if constexpr (ALIGNED) {
#pragma unroll
          for (int u = 0; u < 4; ++u) zz[u] = z[u];
        } else {
          const int sh = (int)(c0 & 3);
          normal4_hw(seed, kStreamOmaNoise, (uint64_t)k, (c0 >> 2) + 1, z + 4);
#pragma unroll
          for (int u = 0; u < 4; ++u) zz[u] = z[u + sh];
        }
        if (full[q]) {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[q][u] = oma_noisy(v[q][u], scale, zz[u]);
          __builtin_nontemporal_store(v[q], reinterpret_cast<f4*>(rp[q] + j0));
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < d) rp[q][j0 + u] = oma_noisy(rp[q][j0 + u], scale, zz[u]);
        }
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        v[q] = nv[q];
        rp[q] = nrp[q];
        full[q] = nfull[q];
      }
    }
  }
}

// Synthetic client updates: honest rows ~ N(mu_h, sd_h^2), the
// last B rows ~ N(mu_b, sd_b^2).  Element (k, global column c) uses normal
// (c & 3) of Philox block (k, c >> 2), so any shard reproduces its columns.
__global__ void __launch_bounds__(256) fill_clients(float* __restrict__ X, int64_t K, int64_t d,
                                                    int64_t ldx, int64_t B, float mu_h,
                                                    float sd_h, float mu_b, float sd_b,
                                                    int64_t col_off, uint64_t seed) {
  const int64_t groups = (d + 3) / 4;
  const int64_t n = K * groups;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = e / groups, g = e - k * groups;
    const bool byz = k >= K - B;
    const float mu = byz ? mu_b : mu_h, sd = byz ? sd_b : sd_h;
    float* row = X + k * ldx;
    float z[4];
    int64_t cached = -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = g * 4 + u;
      if (j >= d) break;
      const int64_t c = col_off + j;
      if ((c >> 2) != cached) {
        cached = c >> 2;
        normal4(seed, kStreamFill, (uint64_t)k, (uint64_t)cached, z);
      }
      row[j] = mu + sd * z[c & 3];
    }
  }
}

__global__ void __launch_bounds__(256) fill_normal(float* __restrict__ v, int64_t n, float mu,
                                                   float sd, int64_t off, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = off + i;
    float z[4];
    normal4(seed, kStreamFill, 0xFFFFFFFFull, (uint64_t)(c >> 2), z);
    v[i] = mu + sd * z[c & 3];
  }
}

static int grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (int)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

hipError_t launch_oma_apply(float* X, int64_t K, int64_t d, int64_t ldx, const float* hr,
                            const float* hi, const float* nr, const float* ni, hipStream_t s) {
  hipLaunchKernelGGL(oma_apply, dim3(grid_for(K * d)), dim3(256), 0, s, X, K, d, ldx, hr, hi, nr,
                     ni);
  return hipGetLastError();
}

hipError_t launch_oma_philox(float* X, int64_t K, int64_t d, int64_t ldx, int64_t d_total,
                             int64_t col_off, float sd, uint64_t seed, hipStream_t s,
                             int wshift, int64_t problems, int64_t pstride) {
  (void)d_total;   // draws are keyed by (row, global column quad): no d_total needed
  const int64_t Kp = K;
  K *= problems;   // rows of all problems
  const int64_t G = (d + 3) / 4;
  const int gy = (int)(K < 65535 ? K : 65535);
  int64_t gx = (G + 255) / 256;
  const int64_t cap = std::max<int64_t>(1, (8192 + gy - 1) / gy);   // ~8K blocks in flight
  if (gx > cap) gx = cap;
  const int vec4 = (reinterpret_cast<uintptr_t>(X) % 16 == 0) && ldx % 4 == 0 &&
                   (problems == 1 || pstride % 4 == 0);
  const dim3 grid((unsigned)gx, gy);
  if (col_off % 4 == 0 && vec4)
    hipLaunchKernelGGL((oma_philox<true, true>), grid, dim3(256), 0, s, X, K, d, ldx, col_off, sd,
                       seed, wshift, Kp, pstride);
  else if (col_off % 4 == 0)
    hipLaunchKernelGGL((oma_philox<true, false>), grid, dim3(256), 0, s, X, K, d, ldx, col_off, sd,
                       seed, wshift, Kp, pstride);
  else if (vec4)
    hipLaunchKernelGGL((oma_philox<false, true>), grid, dim3(256), 0, s, X, K, d, ldx, col_off, sd,
                       seed, wshift, Kp, pstride);
  else
    hipLaunchKernelGGL((oma_philox<false, false>), grid, dim3(256), 0, s, X, K, d, ldx, col_off, sd,
                       seed, wshift, Kp, pstride);
  return hipGetLastError();
}

hipError_t launch_fill_clients(float* X, int64_t K, int64_t d, int64_t ldx, int64_t B,
                               float mu_h, float sd_h, float mu_b, float sd_b, int64_t d_total,
                               int64_t col_off, uint64_t seed, hipStream_t s) {
  (void)d_total;
  hipLaunchKernelGGL(fill_clients, dim3(grid_for(K * ((d + 3) / 4))), dim3(256), 0, s, X, K, d,
                     ldx, B, mu_h, sd_h, mu_b, sd_b, col_off, seed);
  return hipGetLastError();
}

hipError_t launch_fill_normal(float* v, int64_t n, float mu, float sd, int64_t off, uint64_t seed,
                              hipStream_t s) {
  hipLaunchKernelGGL(fill_normal, dim3(grid_for(n)), dim3(256), 0, s, v, n, mu, sd, off, seed);
  return hipGetLastError();
}

}  // namespace gmk
