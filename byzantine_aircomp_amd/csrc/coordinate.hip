// The reference's other aggregators, MNIST_Air_weight.py:186-204:
//   mean          M:186-187   column mean
//   trimmed_mean  M:189-192   mean of each column without its b smallest and b largest
//   median        M:194-195   lower median of each column (torch.median)
//   Krum          M:197-204   the row with the smallest sum of squared distances to
//                              its honestSize-1 nearest rows (itself included, M:200-201)
// median / trimmed_mean select order statistics bit by bit (col_select below);
// sums are fp64, rounded once.
#include <algorithm>

#include "device_util.h"
#include "gmagg_internal.h"

namespace gmk {

// Element (row k, column j) of a client matrix: row-major [K][ldx] (ws = 0), or the
// panel layout [ceil(d/W)][K][W] with W = 2^ws and ldx = the panel stride.  A group of
// 4 columns starting at a multiple of 4 never straddles a panel (W % 4 == 0), so the
// float4 paths below read it as one vector either way.
__device__ __forceinline__ const float* elem(const float* X, int64_t ldx, int ws, int64_t k,
                                             int64_t j) {
  return ws ? X + (j >> ws) * ldx + (k << ws) + (j & ((1 << ws) - 1)) : X + k * ldx + j;
}

// mean: W consecutive columns per thread (W = 4: one float4 per row, 1 KiB per wave
// instruction), 8 rows' loads in flight, each column summed in fp64 in row order
// and rounded once (the same sums for every W).
template <int W>
__global__ void __launch_bounds__(256) col_mean(const float* __restrict__ X, int64_t K, int64_t d,
                                                int64_t ldx, int ws, float* __restrict__ out) {
  typedef float fv __attribute__((ext_vector_type(W)));
  constexpr int U = 8;
  const int64_t G = d / W;            // W > 1: d % W == 0 (checked by the launcher)
  const int64_t rs = ws ? ((int64_t)1 << ws) : ldx;   // row stride
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G;
       g += (int64_t)gridDim.x * blockDim.x) {
    const float* col = elem(X, ldx, ws, 0, g * W);
    double s[W];
#pragma unroll
    for (int v = 0; v < W; ++v) s[v] = 0.0;
    int64_t k = 0;
    for (; k + U <= K; k += U) {
      fv x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[u] = __builtin_nontemporal_load(reinterpret_cast<const fv*>(col + (k + u) * rs));
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < W; ++v) s[v] += (double)x[u][v];
    }
    for (; k < K; ++k) {
      const fv x = *reinterpret_cast<const fv*>(col + k * rs);
#pragma unroll
      for (int v = 0; v < W; ++v) s[v] += (double)x[v];
    }
#pragma unroll
    for (int v = 0; v < W; ++v) out[g * W + v] = (float)(s[v] / (double)K);
  }
}

// getVarience (M:127-129): mean over the H honest rows of ||h_k - mean_k h||^2
// = (1/H) sum_j sum_k (h_kj - m_j)^2, in ONE streaming pass: per column the sums
// of (h_kj - h_0j) and of its square in fp64 (shifted by the column's first row:
// no cancellation for data far from 0), var_j = b - a^2/H; block partials in fp64,
// summed in a fixed order by honest_var_final.  W columns per thread as in
// col_mean (W = 4: float4 rows).  wshift > 0: X in the panel layout
// [ceil(d/2^wshift)][K][2^wshift], ldx = the panel stride (a float4 group never
// straddles a panel).
template <int W>
__global__ void __launch_bounds__(256) honest_var_part(const float* __restrict__ X, int64_t H,
                                                       int64_t d, int64_t ldx, int wshift,
                                                       double* __restrict__ part) {
  typedef float fv __attribute__((ext_vector_type(W)));
  __shared__ double scratch[16];
  constexpr int U = 8;
  const int64_t G = d / W;
  double acc = 0.0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j0 = g * W;
    const float* col = wshift ? X + (j0 >> wshift) * ldx + (j0 & ((1 << wshift) - 1)) : X + j0;
    const int64_t rs = wshift ? ((int64_t)1 << wshift) : ldx;        // row stride
    const fv c = *reinterpret_cast<const fv*>(col);
    double a[W], b[W];
#pragma unroll
    for (int v = 0; v < W; ++v) a[v] = b[v] = 0.0;
    int64_t k = 0;
    for (; k + U <= H; k += U) {
      fv x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[u] = __builtin_nontemporal_load(reinterpret_cast<const fv*>(col + (k + u) * rs));
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < W; ++v) {
          const double t = (double)x[u][v] - (double)c[v];
          a[v] += t;
          b[v] = fma(t, t, b[v]);
        }
    }
    for (; k < H; ++k) {
      const fv x = *reinterpret_cast<const fv*>(col + k * rs);
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const double t = (double)x[v] - (double)c[v];
        a[v] += t;
        b[v] = fma(t, t, b[v]);
      }
    }
#pragma unroll
    for (int v = 0; v < W; ++v) acc += b[v] - a[v] * a[v] / (double)H;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) honest_var_final(const double* __restrict__ part, int nb,
                                                        int64_t H, float* __restrict__ out) {
  __shared__ double scratch[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) out[0] = (float)(s / (double)H);
}

int honest_var_blocks(int64_t d, int num_cu) {
  const int64_t g = (d / 4 + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 4 * (int64_t)num_cu));
}

hipError_t launch_honest_var(const float* X, int64_t H, int64_t d, int64_t ldx, int wshift,
                             int nb, double* part, float* out, hipStream_t s) {
  const bool v4 = d % 4 == 0 && (wshift ? true : ldx % 4 == 0) &&
                  reinterpret_cast<uintptr_t>(X) % 16 == 0;
  if (v4)
    hipLaunchKernelGGL(honest_var_part<4>, dim3(nb), dim3(256), 0, s, X, H, d, ldx, wshift, part);
  else
    hipLaunchKernelGGL(honest_var_part<1>, dim3(nb), dim3(256), 0, s, X, H, d, ldx, wshift, part);
  hipLaunchKernelGGL(honest_var_final, dim3(1), dim3(256), 0, s, part, nb, H, out);
  return hipGetLastError();
}

// Order statistics by bit-wise selection on order-preserving keys.
//
// A column's K values live across one wave: lane l holds rows l, l+64, ...
// (R = ceil(K/64) per lane).  Each float maps to a 32-bit key whose unsigned
// order is the float order (negatives bit-inverted, positives with the sign bit
// set; -0 folded onto +0; every NaN -> 0xFFFFFFFF, the largest key, as torch's
// topk ranks NaN).  The r-th smallest key is built MSB-first: 32 steps, each
// one v_cmp per held value and a scalar popcount of the ballot (the count is
// wave-uniform, no cross-lane reduction).  That is 32·K/64 vector compares per
// column instead of K^2 for pairwise ranking.  The value at a rank does not depend
// on how ties are broken, so these are torch's order statistics exactly:
//   median        r = (K-1)/2 (torch's lower median); any NaN in the column -> NaN
//                 (torch.median propagates NaN);
//   trimmed_mean  the sum of ranks b..K-b-1 = the values strictly between the two
//                 selected keys + the ties at each end counted from the ballots,
//                 summed in fp64 and rounded once.
// Staging: a block loads a K x C tile (C columns, 4C-byte row segments) into LDS
// with coalesced loads, then its 4 waves select C/4 columns each, reading the
// column down the tile (row stride C+1 words: conflict-free).
__device__ __forceinline__ uint32_t order_key(float x) {
  uint32_t u = __float_as_uint(x);
  if (x != x) return 0xFFFFFFFFu;
  if (x == 0.f) u = 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// The key of a held slot (round 5: 4-6 VALU, no branch; the LDS read before it is
// unconditional — padding rows hold finite garbage or zeros — so a wave's reads issue back
// to back): ok = false (a row past K, a column past d) -> 0xFFFFFFFF; -0 as +0 (x + 0);
// NaN -> 0xFFFFFFFF (above +inf: torch's order for topk) when NANTOP, else whatever key
// its bits give (the median returns NaN for a column holding one, select_pair).
template <bool NANTOP>
__device__ __forceinline__ uint32_t slot_key(float x, bool ok) {
  const uint32_t u = __float_as_uint(x + 0.0f);
  uint32_t k = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
  if constexpr (NANTOP) k = x != x ? 0xFFFFFFFFu : k;
  return ok ? k : 0xFFFFFFFFu;
}
__device__ __forceinline__ float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// NC columns x NR ranks selected together: independent chains interleaved, so the
// compare -> count -> decide latency of one chain hides behind the others.
// count(t, cnt): cnt[c][q] = #(keys of chain (c, q) < t[c][q]), wave-uniform.
// EXIT: stop as soon as every chain's interval holds a single key (returns the bit
// just decided: that key is the answer); -1 when the steps ran to `lo`.
template <int NC, int NR, bool EXIT = false, typename Count>
__device__ __forceinline__ int select_steps(int hi, int lo, uint32_t (&ans)[NC][NR],
                                            int (&clo)[NC][NR], int (&chi)[NC][NR],
                                            const int (&rr)[NR], Count count) {
  for (int bit = hi; bit >= lo; --bit) {
    uint32_t t[NC][NR];
    int cnt[NC][NR];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int q = 0; q < NR; ++q) t[c][q] = ans[c][q] | (1u << bit);
    count(t, cnt);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        if (cnt[c][q] <= rr[q]) {
          ans[c][q] |= 1u << bit;
          clo[c][q] = cnt[c][q];
        } else {
          chi[c][q] = cnt[c][q];
        }
      }
    if constexpr (EXIT) {
      bool one = true;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) one = one && chi[c][q] - clo[c][q] == 1;
      if (one) return bit;
    }
  }
  return -1;
}

// Sum over the wave of a per-lane int (DPP row shifts + row broadcasts, gfx9
// family), returned wave-uniform.
__device__ __forceinline__ int wave_sum_i32(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}

// Inclusive prefix sum over the wave of a per-lane int (the DPP sequence of wave_sum_i32
// without its final read of lane 63).
__device__ __forceinline__ int wave_scan_i32(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return v;
}

// The trimmed mean's two ranks (round 4): the top byte of each chain's answer from ONE
// histogram of the keys' top bytes (256 bins in LDS, one atomic add per held key, a wave
// prefix scan), shared by the column's two ranks, instead of 8 counting steps per rank over
// every key; then, when the top byte left more candidates than the compaction takes, the
// next byte from a histogram of the keys inside each rank's top-byte bin.  K=1000 x 2M:
// 7.26 -> 6.30 ms; the median (one rank) measured slower with it, 3.81 -> 4.23 ms (the
// adds to the few bins a column's top bytes fill serialize), so it keeps the counting
// steps (profiles/r4s1_select_hist_ab.jsonl).  GMK_SELECT_HIST: 0 never, 1 the top byte
// only, 2 both bytes; applied where the chain selects >= GMK_SELECT_HIST_NR ranks.
#ifndef GMK_SELECT_HIST
#define GMK_SELECT_HIST 2
#endif
#ifndef GMK_SELECT_NBALLOT
#define GMK_SELECT_NBALLOT 0
#endif
#ifndef GMK_SELECT_HIST_NR
#define GMK_SELECT_HIST_NR 2
#endif

// Candidate compaction (round 2).  Before step `bit` a chain's answer lies in
// [L, L + 2^(bit+1)); the step's count n = #(key < L + 2^bit) is also the count
// below one end of the new interval, so the number of keys still in it (chi - clo)
// is known for free.  At two fixed points of the schedule (after bits 31..24, and
// after 23..16) the chains check it: if every chain has <= 64*R2 keys left, each
// writes those keys (a ballot + mbcnt per held value) to LDS, reads back R2 per lane,
// and the remaining steps count only them: n = c0 + #(candidate < t), c0 = the
// count below L at compaction (every dropped key is below that L or at/above the
// interval's end).  Spread data (the C3 recipe, N(0,1)) compacts after the first 8
// steps (simulated: <= 128 of 1000 keys left after ~7); clustered data after 16 or
// never, and then the loop counts every key as before.  The schedule is fixed and
// branch-free inside each run of steps: a per-step compaction check cost more than
// it saved.  buf(c, q): LDS slots of chain (c, q), STR words apart, >= 64*R2 of them.
template <int R, int NC, int NR, int R2, int STR, typename Buf>
__device__ __forceinline__ void select_ranks(const uint32_t (&key)[NC][R], const int64_t (&r)[NR],
                                             uint32_t (&ans)[NC][NR], int (&clo)[NC][NR],
                                             int (&chi)[NC][NR], Buf buf) {
  constexpr bool COMPACT = R2 > 0 && R > R2;
  int rr[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) rr[q] = (int)r[q];   // counts fit 32 bits (K <= 2048)
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      ans[c][q] = 0;
      clo[c][q] = 0;
      chi[c][q] = 64 * R;      // padding keys (0xFFFFFFFF) count as keys: never below t
    }
  // Counting every held key.  A ballot costs three instructions per key (v_cmp, a
  // scalar popcount, a scalar add) and the loop is issue-bound (one instruction per
  // wave per cycle slot), so at R >= 8 each lane counts its own keys instead (v_cmp +
  // v_addc: two) and two chains share one DPP wave sum (16-bit halves: <= 2048 each).
  // GMK_SELECT_NBALLOT (A/B knob): the first NB keys of each lane counted by ballot
  // (1 VALU + 2 SALU per key) and the rest per lane (2 VALU), to balance the two issue ports
  auto full = [&](const uint32_t (&t)[NC][NR], int (&cnt)[NC][NR]) {
    if constexpr (R >= 8) {
      constexpr int NB = GMK_SELECT_NBALLOT < R ? GMK_SELECT_NBALLOT : R - 1;
      int lc[NC * NR], sc[NC * NR];
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          int v = 0, sb = 0;
#pragma unroll
          for (int i = 0; i < NB; ++i) sb += __popcll(__ballot(key[c][i] < t[c][q]));
#pragma unroll
          for (int i = NB; i < R; ++i) v += (int)(key[c][i] < t[c][q]);
          lc[c * NR + q] = v;
          sc[c * NR + q] = sb;
        }
#pragma unroll
      for (int p = 0; p < NC * NR; p += 2) {
        if (p + 1 < NC * NR) {
          const int s2 = wave_sum_i32(lc[p] + (lc[p + 1] << 16));
          cnt[p / NR][p % NR] = (s2 & 0xFFFF) + sc[p];
          cnt[(p + 1) / NR][(p + 1) % NR] = (s2 >> 16) + sc[p + 1];
        } else {
          cnt[p / NR][p % NR] = wave_sum_i32(lc[p]) + sc[p];   // (an odd chain count: NC = NR = 1)
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          int n = 0;
#pragma unroll
          for (int i = 0; i < R; ++i) n += __popcll(__ballot(key[c][i] < t[c][q]));
          cnt[c][q] = n;
        }
    }
  };
  if constexpr (!COMPACT) {
    select_steps<NC, NR>(31, 0, ans, clo, chi, rr, full);
  } else {
    const int lane = threadIdx.x & 63;
    auto small = [&]() {
      bool ok = true;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) ok = ok && chi[c][q] - clo[c][q] <= 64 * R2;
      return ok;
    };
    // keys in [ans, ans + 2^bit) of every chain -> LDS (lane order) -> R2 per lane,
    // then steps bit-1 .. 0 on them
    auto finish_compacted = [&](int bit) {
      uint32_t ck[NC][NR][R2];
      int cbase[NC][NR];
      const uint32_t span = 1u << bit;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          uint32_t* b = buf(c, q);
          const uint32_t lo = ans[c][q];
          int base = 0;
#pragma unroll
          for (int i = 0; i < R; ++i) {
            const bool in = key[c][i] - lo < span;
            const uint64_t m = __ballot(in);
            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                                       (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (in) b[pos * STR] = key[c][i];
            base += __popcll(m);
          }
          cbase[c][q] = clo[c][q];
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          const uint32_t* b = buf(c, q);
          const int nc = chi[c][q] - clo[c][q];
#pragma unroll
          for (int i = 0; i < R2; ++i) {
            const int s = lane + 64 * i;
            ck[c][q][i] = s < nc ? b[s * STR] : 0xFFFFFFFFu;
          }
        }
      // a chain whose interval holds one candidate has found its key (simulated: one
      // key left after 13-18 of the 32 steps on spread data), so the steps stop
      // when every chain is there and each takes that key
      const int stop = select_steps<NC, NR, true>(bit - 1, 0, ans, clo, chi, rr,
                           [&](const uint32_t (&t)[NC][NR], int (&cnt)[NC][NR]) {
#pragma unroll
                             for (int c = 0; c < NC; ++c)
#pragma unroll
                               for (int q = 0; q < NR; ++q) {
                                 int n = cbase[c][q];
#pragma unroll
                                 for (int i = 0; i < R2; ++i)
                                   n += __popcll(__ballot(ck[c][q][i] < t[c][q]));
                                 cnt[c][q] = n;
                               }
                           });
      if (stop > 0) {
        const uint32_t sp = 1u << stop;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int q = 0; q < NR; ++q) {
            // the first slot in range: the candidates fill slots [0, nc), the 0xFFFFFFFF
            // padding after them falls in range when the interval ends at 2^32
            uint32_t v = ans[c][q];
            bool got = false;
#pragma unroll
            for (int i = 0; i < R2; ++i) {
              const uint64_t m = __ballot(ck[c][q][i] - ans[c][q] < sp);
              if (m && !got) {
                v = __builtin_amdgcn_readlane(ck[c][q][i], __builtin_ctzll(m));
                got = true;
              }
            }
            ans[c][q] = v;
          }
      }
    };
    if constexpr (GMK_SELECT_HIST >= 1 && NR >= GMK_SELECT_HIST_NR) {
      // bins of column c: buf(c, 0)[b * STR], b < 256 (the wave's own dead tile column)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        uint32_t* h = buf(c, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) h[(4 * lane + j) * STR] = 0u;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        uint32_t* h = buf(c, 0);
#pragma unroll
        for (int i = 0; i < R; ++i)
          __hip_atomic_fetch_add(&h[(key[c][i] >> 24) * STR], 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WAVEFRONT);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t* h = buf(c, 0);
        int hb[4], sl = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hb[j] = (int)h[(4 * lane + j) * STR];
          sl += hb[j];
        }
        const int incl = wave_scan_i32(sl), excl = incl - sl;
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          // the lane whose 4 bins hold rank rr[q] (the bins count all 64 R keys, padding
          // included, and rr < K <= 64 R: exactly one lane)
          const uint64_t m = __ballot(excl <= rr[q] && rr[q] < incl);
          const int L = __builtin_amdgcn_readfirstlane(__builtin_ctzll(m));
          int lo = __builtin_amdgcn_readlane(excl, L);
          int bsel = 4 * L + 3, blo = lo, bhi = 64 * R;
          bool found = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int hj = __builtin_amdgcn_readlane(hb[j], L);
            if (!found && lo + hj > rr[q]) {
              found = true;
              bsel = 4 * L + j;
              blo = lo;
              bhi = lo + hj;
            }
            lo += hj;
          }
          ans[c][q] = (uint32_t)bsel << 24;     // keys < ans: blo; keys < ans + 2^24: bhi
          clo[c][q] = blo;
          chi[c][q] = bhi;
        }
      }
      // (the compaction below reuses the same LDS slots: the bins are consumed)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      select_steps<NC, NR>(31, 24, ans, clo, chi, rr, full);
    }
    if (small()) {
      finish_compacted(24);
      return;
    }
    if constexpr (GMK_SELECT_HIST >= 2 && NR >= GMK_SELECT_HIST_NR && R >= 8) {
      // bits 23..16 from a second histogram per chain: the keys inside the chain's top-byte
      // bin, binned by their next byte (slots 256 q + b of column c's dead tile column)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        uint32_t* h = buf(c, 0);
#pragma unroll
        for (int q = 0; q < NR; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) h[(256 * q + 4 * lane + j) * STR] = 0u;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        uint32_t* h = buf(c, 0);
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          const uint32_t top = ans[c][q] >> 24;
#pragma unroll
          for (int i = 0; i < R; ++i)
            if ((key[c][i] >> 24) == top)
              __hip_atomic_fetch_add(&h[(256 * q + ((key[c][i] >> 16) & 255u)) * STR], 1u,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t* h = buf(c, 0);
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          int hb[4], sl = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hb[j] = (int)h[(256 * q + 4 * lane + j) * STR];
            sl += hb[j];
          }
          const int incl = wave_scan_i32(sl) + clo[c][q], excl = incl - sl;
          const uint64_t m = __ballot(excl <= rr[q] && rr[q] < incl);
          const int L = __builtin_amdgcn_readfirstlane(__builtin_ctzll(m));
          int lo = __builtin_amdgcn_readlane(excl, L);
          int bsel = 4 * L + 3, blo = lo, bhi = chi[c][q];
          bool found = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int hj = __builtin_amdgcn_readlane(hb[j], L);
            if (!found && lo + hj > rr[q]) {
              found = true;
              bsel = 4 * L + j;
              blo = lo;
              bhi = lo + hj;
            }
            lo += hj;
          }
          ans[c][q] |= (uint32_t)bsel << 16;
          clo[c][q] = blo;
          chi[c][q] = bhi;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      select_steps<NC, NR>(23, 16, ans, clo, chi, rr, full);
    }
    if (small()) {
      finish_compacted(16);
      return;
    }
    select_steps<NC, NR>(15, 0, ans, clo, chi, rr, full);
  }
}

// Wave min / max (DPP row shifts + row broadcasts, as wave_sum_i32), wave-uniform.
template <bool MAX>
__device__ __forceinline__ float wave_minmax_f32(float v) {
  const int id = __float_as_int(MAX ? -__builtin_inff() : __builtin_inff());
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(v), 0x111, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(v), 0x112, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(v), 0x114, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(v), 0x118, 0xf, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(v), 0x142, 0xa, 0xf, false)));
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(v), 0x143, 0xc, 0xf, false)));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
template <bool MAX>
__device__ __forceinline__ uint32_t wave_minmax_u32(uint32_t v) {
  const int id = MAX ? 0 : -1;
  auto op = [](uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xf, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x142, 0xa, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x143, 0xc, 0xf, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// The median of a column pair from a VALUE-linear histogram (round 4 session 2): 256 bins
// over [min, max] of the column, bin(x) = min(255, trunc((x - min) * 256 / (max - min))) —
// monotone in x (each step is a correctly rounded monotone operation), so the bins are
// consecutive intervals of the key order and the counts below a bin are counts below its
// keys.  Spread data fills many bins (few LDS atomic conflicts, unlike the keys' top byte,
// whose few exponent bins serialized the adds: the histogram variant above measured slower
// for the median); the rank's bin holds a few keys, compacted to LDS and finished by the
// bitwise steps from their common prefix.  Returns false — the caller runs the bitwise
// selection — on an infinite or subnormal range, or when the rank's bin holds more keys
// than the compaction takes (e.g. a column dominated by a few huge outliers).  NaN columns
// never come here.  `rr`: the rank; buf(h, 0): column h's LDS slots (the wave's dead tile
// column), STR words apart.  MEASURED SLOWER, so off (A/B knob): K=1000 x 2M 4.75 vs
// 3.85 ms for the counting steps with their compaction (profiles/r4s2_select_vhist_ab.jsonl;
// the f3 GPU tests green on it) — the min / max reductions, the atomic adds and a second
// pass over the keys for the compaction cost more than the 8 counting steps they replace.
#ifndef GMK_SELECT_VHIST
#define GMK_SELECT_VHIST 0
#endif
template <int R, int R2, int STR, typename Buf>
__device__ __forceinline__ bool median_vhist(const uint32_t (&key)[2][R], int rr, Buf buf,
                                             uint32_t (&ans)[2]) {
  const int lane = threadIdx.x & 63;
  float mn[2], sc[2];
  bool flat[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float lo = __builtin_inff(), hi = -__builtin_inff();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const bool v = key[h][i] != 0xFFFFFFFFu;      // (padding rows)
      const float x = key_value(key[h][i]);
      lo = v ? fminf(lo, x) : lo;
      hi = v ? fmaxf(hi, x) : hi;
    }
    mn[h] = wave_minmax_f32<false>(lo);
    const float mx = wave_minmax_f32<true>(hi);
    flat[h] = !(mx > mn[h]);
    sc[h] = 256.0f / (mx - mn[h]);
    if (!flat[h] && !(mx - mn[h] <= 3.0e38f && sc[h] <= 3.0e38f)) return false;
  }
  auto bin = [&](int h, uint32_t k) {
    const int b = (int)((key_value(k) - mn[h]) * sc[h]);
    return b < 255 ? b : 255;
  };
  // histogram: 4 bins per lane, zeroed, one atomic add per held key
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t* hb = buf(h, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) hb[(4 * lane + j) * STR] = 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (flat[h]) continue;
    uint32_t* hb = buf(h, 0);
#pragma unroll
    for (int i = 0; i < R; ++i)
      if (key[h][i] != 0xFFFFFFFFu)
        __hip_atomic_fetch_add(&hb[bin(h, key[h][i]) * STR], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int tb[2], blo[2], bhi[2];
  bool fits = true;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t* hb = buf(h, 0);
    int c4[4], sl = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c4[j] = (int)hb[(4 * lane + j) * STR];
      sl += c4[j];
    }
    const int incl = wave_scan_i32(sl), excl = incl - sl;
    const uint64_t m = __ballot(excl <= rr && rr < incl);
    const int L = __builtin_amdgcn_readfirstlane(m ? __builtin_ctzll(m) : 0);
    int lo = __builtin_amdgcn_readlane(excl, L);
    tb[h] = 4 * L + 3; blo[h] = lo; bhi[h] = lo;
    bool found = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int hj = __builtin_amdgcn_readlane(c4[j], L);
      if (!found && lo + hj > rr) {
        found = true;
        tb[h] = 4 * L + j;
        blo[h] = lo;
        bhi[h] = lo + hj;
      }
      lo += hj;
    }
    fits = fits && (flat[h] || (m != 0 && bhi[h] - blo[h] <= 64 * R2));
  }
  if (!fits) return false;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the rank's bin -> LDS (lane order) -> R2 candidates per lane
  uint32_t ck[2][1][R2];
  int cbase[2][1], clo[2][1], chi[2][1];
  uint32_t a2[2][1];
  const int rq[1] = {rr};
  int hi_bit = -1;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t* b = buf(h, 0);
    int base = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const bool in = !flat[h] && key[h][i] != 0xFFFFFFFFu && bin(h, key[h][i]) == tb[h];
      const uint64_t m = __ballot(in);
      const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (in) b[pos * STR] = key[h][i];
      base += __popcll(m);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t* b = buf(h, 0);
    const int nc = flat[h] ? 0 : bhi[h] - blo[h];
    uint32_t cmn = 0xFFFFFFFFu, cmx = 0u;
#pragma unroll
    for (int i = 0; i < R2; ++i) {
      const int s = lane + 64 * i;
      ck[h][0][i] = s < nc ? b[s * STR] : 0xFFFFFFFFu;
      if (s < nc) {
        cmn = ck[h][0][i] < cmn ? ck[h][0][i] : cmn;
        cmx = ck[h][0][i] > cmx ? ck[h][0][i] : cmx;
      }
    }
    cmn = wave_minmax_u32<false>(cmn);
    cmx = wave_minmax_u32<true>(cmx);
    if (flat[h]) {
      // every held key is the same value (min == max): the answer, -0 folded onto +0
      a2[h][0] = order_key(mn[h]);
      cmn = cmx = a2[h][0];
    }
    // the steps start below the candidates' common prefix: keys < that prefix are the
    // blo below the bin, keys < prefix + 2^(p+1) all the bin's
    const uint32_t x = cmn ^ cmx;
    const int p = x ? 31 - __builtin_clz(x) : -1;
    if (p >= 0) a2[h][0] = cmn & ~((2u << p) - 1u);
    else a2[h][0] = cmn;
    hi_bit = p > hi_bit ? p : hi_bit;
    cbase[h][0] = blo[h];
    clo[h][0] = blo[h];
    chi[h][0] = flat[h] ? blo[h] + 1 : bhi[h];
  }
  if (hi_bit >= 0) {
    // both chains step from the higher of their two prefixes (a chain whose prefix is
    // lower just takes 0 bits until its own; its answer bits above stay its prefix's)
    const int stop = select_steps<2, 1, true>(hi_bit, 0, a2, clo, chi, rq,
                         [&](const uint32_t (&t)[2][1], int (&cnt)[2][1]) {
#pragma unroll
                           for (int h = 0; h < 2; ++h) {
                             int n = cbase[h][0];
#pragma unroll
                             for (int i = 0; i < R2; ++i) n += __popcll(__ballot(ck[h][0][i] < t[h][0]));
                             cnt[h][0] = n;
                           }
                         });
    if (stop > 0) {
      const uint32_t sp = 1u << stop;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint32_t v = a2[h][0];
        bool got = false;   // (the first slot in range: padding follows the candidates)
#pragma unroll
        for (int i = 0; i < R2; ++i) {
          const uint64_t m = __ballot(ck[h][0][i] - a2[h][0] < sp);
          if (m && !got) {
            v = __builtin_amdgcn_readlane(ck[h][0][i], __builtin_ctzll(m));
            got = true;
          }
        }
        a2[h][0] = v;
      }
    }
  }
  // (a flat chain's steps ran on no candidates: its answer is its value)
  ans[0] = flat[0] ? order_key(mn[0]) : a2[0][0];
  ans[1] = flat[1] ? order_key(mn[1]) : a2[1][0];
  // (the slots are the caller's again)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return true;
}

// The order statistics of one column pair whose keys the wave holds (lane l: rows
// l + 64 i): res[h] = the median (mode 0) or the trimmed mean (mode 1) of column h.
// buf(h, q): LDS slots for chain (h, q)'s compaction, STR words apart.
// NCOL = 1: one column per wave (col_select1).
template <int MODE, int R, int R2, int STR, int NCOL = 2, typename Buf>
__device__ __forceinline__ void select_pair(const uint32_t (&key)[NCOL][R], const bool (&nan)[NCOL],
                                            int64_t K, int64_t b, Buf buf, float (&res)[NCOL]) {
  if constexpr (MODE == 0) {
    const int64_t rk[1] = {(K - 1) / 2};
    uint32_t ans[NCOL][1];
    bool done = false;
    if constexpr (NCOL == 2 && GMK_SELECT_VHIST && R >= 8 && R2 > 0) {
      if (!__ballot(nan[0]) && !__ballot(nan[1])) {   // a NaN column's median is NaN
        uint32_t a2[2];
        done = median_vhist<R, R2, STR>(key, (int)rk[0], buf, a2);
        if (done) {
          ans[0][0] = a2[0];
          ans[1][0] = a2[1];
        }
      }
    }
    if (!done) {
      int clo[NCOL][1], chi[NCOL][1];
      select_ranks<R, NCOL, 1, R2, STR>(key, rk, ans, clo, chi, buf);
    }
#pragma unroll
    for (int h = 0; h < NCOL; ++h)
      res[h] = __ballot(nan[h]) ? __uint_as_float(0x7FC00000u) : key_value(ans[h][0]);
  } else {
    const int64_t rk[2] = {b, K - b - 1};
    uint32_t ans[NCOL][2];
    int clo[NCOL][2], chi[NCOL][2];
    select_ranks<R, NCOL, 2, R2, STR>(key, rk, ans, clo, chi, buf);
    const int64_t n = K - 2 * b;
#pragma unroll
    for (int h = 0; h < NCOL; ++h) {
      const uint32_t lo = ans[h][0], hi = ans[h][1];
      const float vlo = key_value(lo), vhi = key_value(hi);
      double sum;
      if (lo == hi) {
        sum = (double)n * (double)vlo;
      } else {
        // the selection's final intervals hold the boundary counts (round 5): rank b's
        // interval is [lo, lo + 1) or a one-key interval, so #(keys <= lo) = chi, and
        // #(keys < hi) = rank K-b-1's clo (padding keys count on both sides alike)
        double sv0 = 0.0, sv1 = 0.0;
        const int64_t le_lo = chi[h][0], lt_hi = clo[h][1];
#pragma unroll
        for (int i = 0; i < R; i += 2) {
          if (key[h][i] > lo && key[h][i] < hi) sv0 += (double)key_value(key[h][i]);
          if (i + 1 < R && key[h][i + 1] > lo && key[h][i + 1] < hi)
            sv1 += (double)key_value(key[h][i + 1]);
        }
        double sv = sv0 + sv1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sv += __shfl_xor(sv, o);
        sum = sv + (double)(le_lo - b) * (double)vlo + (double)((K - b) - lt_hi) * (double)vhi;
      }
      res[h] = (float)(sum / (double)n);
    }
  }
}

// The selection of one staged K x C tile (columns j0 .. j0 + C - 1).
template <int MODE, int R, int C, int NWV>
__device__ __forceinline__ void select_tile(float (&tile)[64 * R][C + 1], int64_t K, int64_t d,
                                            int64_t j0, int64_t b,
                                            float* __restrict__ out) {
  // wave w selects columns in pairs (w + 2m NWV, w + 2m NWV + NWV): C % (2 NWV) == 0
  static_assert(C % (2 * NWV) == 0, "column pairs");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c0 = w; c0 < C; c0 += 2 * NWV) {
    if (j0 + c0 >= d) break;
    uint32_t key[2][R];      // values are recovered from keys (key_value) when summed
    bool nan[2] = {false, false};
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = lane + 64 * i;
        const bool ok = row < (int)K && j0 + c0 + NWV * h < d;
        const float x = tile[row][c0 + NWV * h];
        key[h][i] = slot_key<MODE == 1>(x, ok);
        nan[h] |= ok && x != x;
      }
    float res[2];
    // compaction slots of chain (h, q): column c0 + NWV h of the tile (this wave's own
    // column, dead once its keys are in registers), rows from q * 64 * R2
    constexpr int R2 = R >= 4 ? 2 : 0;
    auto buf = [&](int h, int q) {
      return reinterpret_cast<uint32_t*>(&tile[q * 64 * (R2 > 0 ? R2 : 1)][c0 + NWV * h]);
    };
    select_pair<MODE, R, R2, C + 1>(key, nan, K, b, buf, res);
    if (lane == 0) {
      out[j0 + c0] = res[0];
      if (j0 + c0 + NWV < d) out[j0 + c0 + NWV] = res[1];
    }
  }
}

#ifndef GMK_SELECT_DBG
#define GMK_SELECT_DBG 0
#endif

// PERSIST: one grid of co-resident blocks walks the tiles (grid stride), each block
// loading tile t + grid into registers while its waves select tile t's columns, so the
// loads of a CU are in flight during its selection instead of only between tiles (the
// plain form: one tile per block, loads then selection).
template <int MODE, int R, int C, int NWV, bool PERSIST>
__global__ void __launch_bounds__(NWV * 64) col_select(const float* __restrict__ X, int64_t K,
                                                  int64_t d, int64_t ldx, int ws, int64_t b,
                                                  int vec4, float* __restrict__ out) {
  __shared__ float tile[64 * R][C + 1];
  const int64_t ntiles = (d + C - 1) / C;
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int LPR = C / 4, RPI = NWV * 64 / LPR;
  static_assert(16 * RPI >= 64 * R, "one round of 16 loads per thread covers the tile");
  const int tq = threadIdx.x % LPR, tr = threadIdx.x / LPR;
  // XCD-aware: blocks bid and bid+8 run on the same XCD; give them adjacent tiles
  // so the two halves of a 128-B line (C = 16) are fetched into one L2.
  auto tile_of = [&](int64_t v) {
    return (C < 32 && v < ntiles / 16 * 16) ? v / 16 * 16 + (v % 8) * 2 + (v / 8) % 2 : v;
  };
  // float4 per lane (LPR lanes per row segment), 16 loads in flight per thread
  f4 buf[16];
  auto load = [&](int64_t t) {
    const int64_t col = t * C + 4 * tq;
    const bool vec = vec4 && col + 4 <= d;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int64_t k = tr + (int64_t)u * RPI;
      buf[u] = f4{0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        const float* src = elem(X, ldx, ws, k, col);
        if (vec) {
          buf[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) buf[u][e] = col + e < d ? src[e] : 0.f;
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int64_t k = tr + (int64_t)u * RPI;
      if (k < K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[k][4 * tq + e] = buf[u][e];
      }
    }
  };
  int64_t v = blockIdx.x;
  if (v >= ntiles) return;
  // GMK_SELECT_DBG (probe builds; 0 in the product): 1 = load + stage the tile only (no
  // selection), 2 = every block loads one of 64 tiles (L2 / Infinity-Cache resident) and
  // selects it: the two phases priced apart
  auto src_tile = [&](int64_t u) { return GMK_SELECT_DBG == 2 ? tile_of(u % 64) : tile_of(u); };
  load(src_tile(v));
  for (; v < ntiles; v += PERSIST ? (int64_t)gridDim.x : ntiles) {
    const int64_t j0 = tile_of(v) * C;
    if (PERSIST) __syncthreads();          // the previous tile's columns are in registers
    store();
    __syncthreads();
    if (PERSIST && v + gridDim.x < ntiles) load(src_tile(v + gridDim.x));
    if constexpr (GMK_SELECT_DBG == 1) {
      if (threadIdx.x < C && j0 + threadIdx.x < d) out[j0 + threadIdx.x] = tile[threadIdx.x][threadIdx.x];
    } else {
      select_tile<MODE, R, C, NWV>(tile, K, d, j0, b, out);
    }
  }
}
// One column per wave (round 4 session 2; the trimmed mean's kernel, launch_col_select): K <= 1024, a block of
// C = 16 waves stages a 1024 x 16 tile (69.6 KB, two blocks per CU) and wave w selects
// column w alone, so that a wave holds 16 keys instead of 32 and the kernel fits 64 VGPRs:
// 8 waves per SIMD instead of 4, to hide the per-step compare -> count -> decide latency
// that bounds the pair kernel.  Loads: 4 float4 per thread in flight.
template <int MODE, int R, int C>
__global__ void __launch_bounds__(C * 64, 2) col_select1(const float* __restrict__ X, int64_t K,
                                                      int64_t d, int64_t ldx, int ws, int64_t b, int vec4,
                                                      float* __restrict__ out) {
  __shared__ float tile[64 * R][C + 1];
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int LPR = C / 4, RPI = C * 64 / LPR;
  constexpr int NLD = (64 * R + RPI - 1) / RPI;
  const int tq = threadIdx.x % LPR, tr = threadIdx.x / LPR;
  const int64_t ntiles = (d + C - 1) / C;
  const int64_t v = blockIdx.x;
  if (v >= ntiles) return;
  // blocks bid and bid + 8 share an XCD: adjacent tiles, one 128-B line's two halves
  const int64_t t = (v < ntiles / 16 * 16) ? v / 16 * 16 + (v % 8) * 2 + (v / 8) % 2 : v;
  const int64_t j0 = t * C;
  {
    const int64_t col = j0 + 4 * tq;
    const bool vec = vec4 && col + 4 <= d;
    f4 buf[NLD];
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int64_t k = tr + (int64_t)u * RPI;
      buf[u] = f4{0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        const float* src = elem(X, ldx, ws, k, col);
        if (vec) {
          buf[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) buf[u][e] = col + e < d ? src[e] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int64_t k = tr + (int64_t)u * RPI;
      if (k < 64 * R) {
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[k][4 * tq + e] = buf[u][e];
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (j0 + w >= d) return;
  uint32_t key[1][R];
  bool nan[1] = {false};
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = lane + 64 * i;
    const bool ok = row < (int)K;
    const float x = tile[row][w];
    key[0][i] = slot_key<MODE == 1>(x, ok);
    nan[0] |= ok && x != x;
  }
  constexpr int R2 = R >= 4 ? 2 : 0;
  auto bufc = [&](int, int q) {
    return reinterpret_cast<uint32_t*>(&tile[q * 64 * (R2 > 0 ? R2 : 1)][w]);
  };
  float res[1];
  select_pair<MODE, R, R2, C + 1, 1>(key, nan, K, b, bufc, res);
  if (lane == 0) out[j0 + w] = res[0];
}

// Staged-transpose selection (round 5): the column tile never sits in LDS whole.  A block
// of NWV waves owns C = NWV x NC columns (C = 16: 64-byte row segments, adjacent tiles on
// one XCD as col_select1); 256-row rounds go HBM -> registers -> a 17-KB LDS stage -> each
// wave's NC columns as keys in registers, so LDS no longer caps the columns in flight per
// CU (col_select: two 69.6-KB tiles = 32 columns) and the VGPRs do: NC chains per wave.
// The compaction slots are per chain (scr), contiguous.
#ifndef GMK_SELECT_ST_PREFETCH
#define GMK_SELECT_ST_PREFETCH 0   // A/B: the next staging round's loads in flight
#endif
#ifndef GMK_SELECT_ST_WPE
#define GMK_SELECT_ST_WPE 0   // A/B: minimum waves per SIMD the compiler must fit (0: its choice)
#endif
#if GMK_SELECT_ST_WPE
#define GMK_ST_ATTR __attribute__((amdgpu_waves_per_eu(GMK_SELECT_ST_WPE, 8)))
#else
#define GMK_ST_ATTR
#endif
template <int MODE, int R, int NC, int NWV>
__global__ void __launch_bounds__(NWV * 64) GMK_ST_ATTR col_select_st(const float* __restrict__ X, int64_t K,
                                                         int64_t d, int64_t ldx, int ws, int64_t b,
                                                         int vec4, float* __restrict__ out) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int C = NWV * NC;
  static_assert(C == 16, "64-byte row segments");
  constexpr int SR = 256;                          // rows per staging round
  constexpr int NRD = (64 * R + SR - 1) / SR;      // rounds
  constexpr int R2 = R >= 4 ? 2 : 0;
  constexpr int SLOTS = MODE == 0 ? 64 * (R2 > 0 ? R2 : 1) : 512;
  constexpr int LPR = C / 4, RPI = NWV * 64 / LPR, NLD = SR / RPI;
  static_assert(SR % RPI == 0 && SR % 64 == 0 && (64 * R) % SR == 0, "round shape");
  __shared__ float stage[SR][C + 1];
  __shared__ uint32_t scr[NWV][NC][SLOTS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tq = threadIdx.x % LPR, tr = threadIdx.x / LPR;
  const int64_t ntiles = (d + C - 1) / C;
  const int64_t v = blockIdx.x;
  if (v >= ntiles) return;
  // blocks bid and bid + 8 share an XCD: adjacent tiles, one 128-B line's two halves
  const int64_t t = (v < ntiles / 16 * 16) ? v / 16 * 16 + (v % 8) * 2 + (v / 8) % 2 : v;
  const int64_t j0 = t * C;
  const int64_t col = j0 + 4 * tq;
  const bool vec = vec4 && col + 4 <= d;
  uint32_t key[NC][R];
  bool nan[NC];
#pragma unroll
  for (int h = 0; h < NC; ++h) nan[h] = false;
  // round rd + 1's loads are issued before round rd's staging (GMK_SELECT_ST_PREFETCH)
  f4 buf[GMK_SELECT_ST_PREFETCH == 1 ? 2 : 1][NLD];
  // a whole in-range, aligned tile (wave-uniform): every load issued unconditionally from a
  // clamped row, rows past K zeroed after, so the loads go out back to back (a per-load
  // branch made the compiler wait for each); the edge tile takes the guarded path
  const bool vec_tile = vec4 && j0 + C <= d;
  auto load = [&](int rd, f4 (&dst)[NLD]) {
    if (vec_tile) {
#pragma unroll
      for (int u = 0; u < NLD; ++u) {
        const int k = rd * SR + tr + u * RPI;
        const f4 x = __builtin_nontemporal_load(
            reinterpret_cast<const f4*>(elem(X, ldx, ws, k < (int)K ? k : (int)K - 1, col)));
        dst[u] = k < (int)K ? x : f4{0.f, 0.f, 0.f, 0.f};
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int64_t k = rd * SR + tr + (int64_t)u * RPI;
      dst[u] = f4{0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        const float* src = elem(X, ldx, ws, k, col);
        if (vec) {
          dst[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) dst[u][e] = col + e < d ? src[e] : 0.f;
        }
      }
    }
  };
  // GMK_SELECT_ST_PREFETCH = 2: every round's loads issued up front (NRD x NLD float4)
  f4 all[GMK_SELECT_ST_PREFETCH == 2 ? NRD : 1][NLD];
  if constexpr (GMK_SELECT_ST_PREFETCH == 2) {
#pragma unroll
    for (int rd = 0; rd < NRD; ++rd) load(rd, all[rd]);
  } else if constexpr (GMK_SELECT_ST_PREFETCH == 1) {
    load(0, buf[0]);
  }
#pragma unroll
  for (int rd = 0; rd < NRD; ++rd) {
    constexpr int P = GMK_SELECT_ST_PREFETCH == 1 ? 1 : 0;
    f4 (&cur)[NLD] = GMK_SELECT_ST_PREFETCH == 2 ? all[GMK_SELECT_ST_PREFETCH == 2 ? rd : 0]
                                                  : buf[P ? (rd & 1) : 0];
    if constexpr (GMK_SELECT_ST_PREFETCH == 1) {
      if (rd + 1 < NRD) load(rd + 1, buf[(rd + 1) & 1]);
    } else if constexpr (GMK_SELECT_ST_PREFETCH == 0) {
      load(rd, cur);
    }
    if (rd > 0) __syncthreads();                   // the previous round's reads are done
#pragma unroll
    for (int u = 0; u < NLD; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) stage[tr + u * RPI][4 * tq + e] = cur[u][e];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < NC; ++h) {
      const bool cok = j0 + w * NC + h < d;       // wave-uniform
#pragma unroll
      for (int i = 0; i < SR / 64; ++i) {
        const int row = rd * SR + lane + 64 * i;
        const bool ok = cok && row < (int)K;
        const float x = stage[lane + 64 * i][w * NC + h];
        key[h][rd * (SR / 64) + i] = slot_key<MODE == 1>(x, ok);
        nan[h] |= ok && x != x;
      }
    }
  }
  auto bufc = [&](int h, int q) { return &scr[w][h][q * 64 * (R2 > 0 ? R2 : 1)]; };
  float res[NC];
  select_pair<MODE, R, R2, 1, NC>(key, nan, K, b, bufc, res);
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < NC; ++h)
      if (j0 + w * NC + h < d) out[j0 + w * NC + h] = res[h];
  }
}

// Krum, step 1: squared distances of every row pair, register-tiled.
// A block owns a 128 x 128 tile of pairs (row tiles bi <= bj: D is symmetric)
// over one slice of the columns; each of 512 threads an 8 x 4 sub-tile (8 x 8 with
// 256 threads needed 326 VGPRs: one wave per SIMD, the LDS reads exposed).  Per
// 32-column stage both row tiles go to LDS column-major (sA[c][r]), so a thread
// reads its 8 + 4 values of one column as three ds_read_b128 and does 32 (sub, fma)
// pairs (packed two at a time by the compiler): the
// exact differences of M:199 in fp32, squares summed in fp32 over the stage and
// in fp64 across stages.  Slices write fp64 partials [S][K][K]; pair_reduce sums
// them in a fixed order (deterministic, no atomics).
constexpr int kPT = 128;   // pair-tile edge (rows)
constexpr int kPC = 32;    // columns per LDS stage
constexpr int kPDT = 512;  // pair_dist threads per block

template <bool VEC>
__global__ void __launch_bounds__(kPDT) pair_dist(const float* __restrict__ X, int64_t K,
                                                 int64_t d, int64_t ldx, int ws, int64_t chunk,
                                                 double* __restrict__ part) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float sA[kPC][kPT + 4];
  __shared__ __attribute__((aligned(16))) float sB[kPC][kPT + 4];
  const int64_t nT = (K + kPT - 1) / kPT;
  int64_t p = blockIdx.x, bi = 0;
  while (p >= nT - bi) { p -= nT - bi; ++bi; }
  const int64_t bj = bi + p;
  const int64_t cb = (int64_t)blockIdx.y * chunk, ce = cb + chunk < d ? cb + chunk : d;
  const int ti = threadIdx.x >> 5, tj = threadIdx.x & 31;
  double accd[8][4];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) accd[u][v] = 0.0;
  // stage loads: thread owns (row r, columns cg..cg+3) of both row tiles for q = 0..1;
  // the next stage's loads are issued before this stage's arithmetic (register prefetch)
  f4 pre[2][2];
  auto load_stage = [&](int64_t c0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = threadIdx.x + kPDT * q, r = idx >> 3, cg = (idx & 7) * 4;
      const int64_t col = c0 + cg;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int64_t row = (t ? bj : bi) * kPT + r;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (row < K && col < ce) {
          const float* src = elem(X, ldx, ws, row, col);
          if (VEC && col + 4 <= ce) {
            v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = col + u < ce ? src[u] : 0.f;
          }
        }
        pre[q][t] = v;
      }
    }
  };
  if (cb < ce) load_stage(cb);
  for (int64_t c0 = cb; c0 < ce; c0 += kPC) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = threadIdx.x + kPDT * q, r = idx >> 3, cg = (idx & 7) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sA[cg + u][r] = pre[q][0][u];
        sB[cg + u][r] = pre[q][1][u];
      }
    }
    __syncthreads();
    if (c0 + kPC < ce) load_stage(c0 + kPC);
    float acc[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[u][v] = 0.f;
#pragma unroll 4
    for (int c = 0; c < kPC; ++c) {
      const f4 a0 = *reinterpret_cast<const f4*>(&sA[c][ti * 8]);
      const f4 a1 = *reinterpret_cast<const f4*>(&sA[c][ti * 8 + 4]);
      const f4 b0 = *reinterpret_cast<const f4*>(&sB[c][tj * 4]);
      const float a[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const float b[4] = {b0[0], b0[1], b0[2], b0[3]};
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float t = a[u] - b[v];
          acc[u][v] = fmaf(t, t, acc[u][v]);
        }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) accd[u][v] += (double)acc[u][v];
  }
  double* P = part + (int64_t)blockIdx.y * K * K;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int64_t i = bi * kPT + ti * 8 + u;
    if (i >= K) break;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t j = bj * kPT + tj * 4 + v;
      if (j < K) P[i * K + j] = accd[u][v];
    }
  }
}

// D[i][j] (i <= j: the tile of (i, j) has bi <= bj, so it was computed) = the sum
// over slices in slice order; one wave per 64 consecutive elements, 4 waves split
// the slices and combine in a fixed order (deterministic, no atomics).
__global__ void __launch_bounds__(256) pair_reduce(const double* __restrict__ part, int64_t S,
                                                   int64_t K, double* __restrict__ D) {
  __shared__ double red[4][64];
  const int64_t n = K * K;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const int64_t i = e / K, j = e - i * K;
  const bool on = e < n && i <= j;
  const int64_t s0 = S * w / 4, s1 = S * (w + 1) / 4;
  double s = 0.0;
  if (on) {
#pragma unroll 8
    for (int64_t t = s0; t < s1; ++t) s += part[t * n + e];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && on) D[e] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// The sum of the kk smallest entries of a row staged in LDS (stable rank), summed per
// thread in j order and over the block by block_sum: every Krum score — the exact path's
// and the Gram path's refined candidates' — goes through this one function, so equal rows
// give equal bits.
__device__ __forceinline__ double krum_row_score(const double* srow, int64_t K, int64_t kk,
                                                 double* scratch) {
  double sc = 0.0;
  for (int64_t j = threadIdx.x; j < K; j += blockDim.x) {
    const double x = srow[j];
    int64_t rank = 0;
    for (int64_t t = 0; t < K; ++t) rank += (srow[t] < x) || (srow[t] == x && t < j);
    if (rank < kk) sc += x;
  }
  return block_sum(sc, scratch);
}

// Krum, step 2 (one block per row): score_i = sum of the kk smallest D[i][*] (self
// included, M:200-201), by stable rank over the row staged in LDS.
__global__ void __launch_bounds__(256) krum_score(const double* __restrict__ D, int64_t K,
                                                  int64_t kk, double* __restrict__ score) {
  extern __shared__ double srow[];
  __shared__ double scratch[8];
  const int64_t i = blockIdx.x;
  for (int64_t j = threadIdx.x; j < K; j += blockDim.x) srow[j] = D[i <= j ? i * K + j : j * K + i];
  __syncthreads();
  const double sc = krum_row_score(srow, K, kk, scratch);
  if (threadIdx.x == 0) score[i] = sc;
}

// Krum, step 3: index = first argmin of the scores (torch.argmin), one wave.
__global__ void __launch_bounds__(64) krum_argmin(const double* __restrict__ score, int64_t K,
                                                  int64_t* __restrict__ index) {
  int64_t best = -1;
  double bv = 0.0;
  for (int64_t i = threadIdx.x; i < K; i += 64)
    if (best < 0 || score[i] < bv) { bv = score[i]; best = i; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o);
    const int64_t oi = __shfl_xor(best, o);
    if (oi >= 0 && (best < 0 || ov < bv || (ov == bv && oi < best))) { bv = ov; best = oi; }
  }
  if (threadIdx.x == 0) *index = best;
}

// Krum, step 4: out = row *index, grid-wide copy.
__global__ void __launch_bounds__(256) copy_row(const float* __restrict__ X, int64_t d,
                                                int64_t ldx, int ws,
                                                const int64_t* __restrict__ index,
                                                float* __restrict__ out) {
  const int64_t k = *index;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < d;
       c += (int64_t)gridDim.x * blockDim.x)
    out[c] = *elem(X, ldx, ws, k, c);
}

// ---------------------------------------------------------------------------
// Krum through the Gram MFMA kernel (round 5; SURVEY §8 f3: D = diag(G) 1^T + 1 diag(G)^T
// - 2G).  G~ = (X - p)(X - p)^T from gram.hip's scaled-f16 split (p = row 0), then
//   D~_ij = G~_ii + G~_jj - 2 G~_ij,
//   |D_ij - D~_ij| <= e_ij = epsg (n_i + n_j)^2 + 4 A (n_i + n_j) + 4 A^2 + 1e-5 |D~_ij|
// (n_i = ||x_i - p||.  epsg bounds the RELATIVE errors |G~ - G| / (n_i n_j): the split's
// 2^-22 terms, the fp32 accumulation chains between flushes, the centring — api.hip
// krum_gram_eps.  A bounds the ABSOLUTE part, the f16 subnormal floor: the Gram kernel
// scales every element of a column block by ONE power of two 2^e_b, chosen from the block's
// largest |x - p| over all rows (gram.hip h16_producer), so an element's split loses up to
// 2^-25 2^-e_b whatever its own row's size — one large (Byzantine) row raises it for every
// honest row of the block.  With E = max_b 2^-e_b, ||delta_i|| <= A = 2^-25 E sqrt(d), and
// |G~_ij - G_ij| <= A (n_i + n_j) + A^2, so D~ is off by <= 4 A (n_i + n_j) + 4 A^2.  The
// 1e-5 |D~| covers the exact path's own fp32 rounding.)  A row's score is the sum of its kk
// smallest distances (self = 0), monotone in each distance, so
//   LB_i = score(max(0, D~ - e)) <= score_i <= UB_i = score(D~ + e).
// Every row with LB_i <= min_j UB_j is a candidate — the exact argmin always is — and the
// candidates' distance rows are recomputed with the exact path's arithmetic (same slices,
// 32-column fp32 stages, fp64 across stages, pair_reduce's order, krum_row_score): their
// scores carry the exact path's bits, so the index equals the exact path's.

// One block per row i: LB_i, UB_i.  A bound that cannot hold (D~ + e < 0, a non-finite G)
// gives NaN, which sends the call to the exact path.
__global__ void __launch_bounds__(256) krum_gram_bounds(const double* __restrict__ G, int KP,
                                                        int64_t K, int64_t kk, double epsg,
                                                        const int* __restrict__ bexp, int nb,
                                                        int64_t d, double* __restrict__ lb,
                                                        double* __restrict__ ub) {
  extern __shared__ double sb[];
  double* sl = sb;
  double* su = sb + K;
  __shared__ double scratch[8];
  __shared__ int s_emin;
  const int64_t i = blockIdx.x;
  // A = 2^-25 max_b 2^-e_b sqrt(d): the smallest block exponent (the largest block scale)
  int em = 1 << 20;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) em = min(em, bexp[b]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) em = min(em, __shfl_xor(em, o, 64));
  if (threadIdx.x == 0) s_emin = 1 << 20;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) atomicMin(&s_emin, em);
  __syncthreads();
  const double A = s_emin >= (1 << 20) ? 0.0 : ldexp(sqrt((double)d), -25 - s_emin);
  // n_i from G~_ii: G~_ii >= (1 - 2 epsg) n_i^2 - 2 A n_i - A^2, so n_i <= this + 3 A
  const double gii = G[i * KP + i];
  const double ni = sqrt(fmax(gii, 0.0) * (1.0 + 2.0 * epsg)) + 3.0 * A;
  for (int64_t j = threadIdx.x; j < K; j += blockDim.x) {
    const double gjj = G[j * KP + j];
    const double nj = sqrt(fmax(gjj, 0.0) * (1.0 + 2.0 * epsg)) + 3.0 * A;
    const double dt = (gii + gjj) - 2.0 * G[i * KP + j];
    const double e = epsg * (ni + nj) * (ni + nj) + 4.0 * A * (ni + nj) + 4.0 * A * A +
                     1e-5 * fabs(dt);
    const double hi = dt + e;
    sl[j] = j == i ? 0.0 : fmax(dt - e, 0.0);
    su[j] = j == i ? 0.0 : (hi >= 0.0 ? hi : __builtin_nan(""));
  }
  __syncthreads();
  const double l = krum_row_score(sl, K, kk, scratch);
  const double u = krum_row_score(su, K, kk, scratch);
  if (threadIdx.x == 0) {
    lb[i] = l;
    ub[i] = u;
  }
}

// One wave: the candidates {i : LB_i <= min UB} in index order -> cand[1..], their count
// -> cand[0]; -1 when a bound is NaN (the exact path runs), -2 when the count exceeds maxc;
// cand[maxc + 1] = the row of the smallest UB (the next centre when the count is too large).
__global__ void __launch_bounds__(64) krum_candidates(const double* __restrict__ lb,
                                                      const double* __restrict__ ub, int64_t K,
                                                      int64_t maxc, int64_t* __restrict__ cand) {
  const int lane = threadIdx.x;
  double m = __builtin_inf();
  int64_t mi = K;
  bool bad = false;
  for (int64_t i = lane; i < K; i += 64) {
    const double u = ub[i], l = lb[i];
    bad |= u != u || l != l;
    if (u < m) { m = u; mi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double om = __shfl_xor(m, o);
    const int64_t oi = __shfl_xor(mi, o);
    if (om < m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
  bad = __ballot(bad) != 0;
  int64_t n = 0;
  for (int64_t i0 = 0; i0 < K; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool in = i < K && lb[i] <= m;
    const uint64_t b = __ballot(in);
    const int64_t pos = n + (int64_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (in && pos < maxc) cand[1 + pos] = i;
    n += __popcll(b);
  }
  if (lane == 0) {
    cand[0] = (bad || n < 1) ? -1 : n > maxc ? -2 : n;
    cand[maxc + 1] = mi < K ? mi : 0;
  }
}

// The candidates' distance rows with pair_dist's arithmetic: slice blockIdx.y of the
// columns (the exact path's krum_slices / chunk), 32-column stages, t = x_c - x_j (the
// square of -t is the same bits), fp32 fma chain per stage, fp64 across stages.  A block
// = 64 rows x up to kRefC candidates; per stage the rows go to LDS (coalesced: 8 lanes per
// 128-byte row segment) and the candidates to LDS as interleaved PAIRS (c, c+1 of one
// column adjacent), so one broadcast ds_read_b128 gives two columns of a candidate pair
// and v_pk_add_f32 / v_pk_fma_f32 run the pair's two chains (per lane IEEE: the scalar
// chain's bits).  Thread = (row jl, candidate-pair group grp): pairs grp, grp + 4, ...;
// the next stage's loads in registers during this stage's arithmetic.  (Two rows per
// thread — half the broadcast reads per FMA, half the blocks — measured slower: 2.40 vs
// 1.77 ms without the prefetch.)
// Measured against three register-heavy forms (each lane's rows straight from HBM, the
// candidates by scalar loads, one wave per SIMD): 2.8 vs 4.4-5.8 ms at K = 256 x 4M.
constexpr int kRefC = 32;
template <bool VEC, int NPP>   // NPP: candidate pairs per thread (ceil(pairs / 4): no idle chains)
__global__ void __launch_bounds__(256) krum_cand_dist(const float* __restrict__ X, int64_t K,
                                                      int64_t d, int64_t ldx, int ws, int64_t chunk,
                                                      const int64_t* __restrict__ cidx, int m,
                                                      double* __restrict__ part) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) float sC[kRefC / 2][kPC * 2];   // [pair][col][2]
  // rows as column PAIRS: sR2[c / 2][row] = (x[row][c], x[row][c + 1]), one ds_read_b64 per
  // two columns (consecutive lanes, consecutive 8 B); row stride 65 pairs spreads the
  // staging writes over the banks
  __shared__ __attribute__((aligned(16))) float sR2[kPC / 2][65][2];
  const int tid = threadIdx.x, jl = tid & 63, grp = tid >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + jl;
  const int64_t cb = (int64_t)blockIdx.y * chunk, ce = cb + chunk < d ? cb + chunk : d;
  static_assert(NPP >= 1 && NPP <= kRefC / 8, "candidate pairs per thread");
  double accd[NPP][2];
#pragma unroll
  for (int u = 0; u < NPP; ++u) accd[u][0] = accd[u][1] = 0.0;
  auto ld4 = [&](int64_t row, int64_t col) {
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (col < ce) {
      const float* src = elem(X, ldx, ws, row, col);
      if (VEC && col + 4 <= ce) {
        v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = col + u < ce ? src[u] : 0.f;
      }
    }
    return v;
  };
  // stage loads in registers, the next stage's issued before this stage's arithmetic:
  // rows (64 x 8 float4: two per thread), candidates (8 NPP x 8 float4: one per thread of
  // the first 64 NPP; candidates >= m load zeros and are never stored)
  const int cr = tid >> 3, ccg = (tid & 7) * 4;
  const int64_t crow = tid < 64 * NPP && cr < m ? cidx[cr] : -1;
  f4 pr[2], pc;
  auto load_stage = [&](int64_t c0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q, r = idx >> 3, cg = (idx & 7) * 4;
      const int64_t row = (int64_t)blockIdx.x * 64 + r;
      pr[q] = row < K ? ld4(row, c0 + cg) : f4{0.f, 0.f, 0.f, 0.f};
    }
    pc = crow >= 0 ? ld4(crow, c0 + ccg) : f4{0.f, 0.f, 0.f, 0.f};
  };
  if (cb < ce) load_stage(cb);
  for (int64_t c0 = cb; c0 < ce; c0 += kPC) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q, r = idx >> 3, cg = (idx & 7) * 4;
      *reinterpret_cast<f2*>(&sR2[cg / 2][r][0]) = f2{pr[q][0], pr[q][1]};
      *reinterpret_cast<f2*>(&sR2[cg / 2 + 1][r][0]) = f2{pr[q][2], pr[q][3]};
    }
    if (tid < 64 * NPP) {
#pragma unroll
      for (int u = 0; u < 4; ++u) sC[cr >> 1][2 * (ccg + u) + (cr & 1)] = pc[u];
    }
    __syncthreads();
    if (c0 + kPC < ce) load_stage(c0 + kPC);
    f2 acc[NPP];
#pragma unroll
    for (int u = 0; u < NPP; ++u) acc[u] = f2{0.f, 0.f};
#pragma unroll 4
    for (int c = 0; c < kPC; c += 2) {
      const f2 xx = *reinterpret_cast<const f2*>(&sR2[c / 2][jl][0]);
      const float x0 = xx[0], x1 = xx[1];
#pragma unroll
      for (int u = 0; u < NPP; ++u) {
        const f4 cc = *reinterpret_cast<const f4*>(&sC[grp + 4 * u][2 * c]);
        const f2 t0 = f2{cc[0], cc[1]} - f2{x0, x0};
        acc[u] = __builtin_elementwise_fma(t0, t0, acc[u]);
        const f2 t1 = f2{cc[2], cc[3]} - f2{x1, x1};
        acc[u] = __builtin_elementwise_fma(t1, t1, acc[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < NPP; ++u) {
      accd[u][0] += (double)acc[u][0];
      accd[u][1] += (double)acc[u][1];
    }
  }
  if (j < K) {
#pragma unroll
    for (int u = 0; u < NPP; ++u)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int cc = 2 * (grp + 4 * u) + e;
        if (cc < m) part[((int64_t)blockIdx.y * m + cc) * K + j] = accd[u][e];
      }
  }
}

// Dc[c][j] = the sum over slices in pair_reduce's order (4 waves split the slices,
// ((w0 + w1) + w2) + w3).
__global__ void __launch_bounds__(256) krum_cand_reduce(const double* __restrict__ part, int64_t S,
                                                        int64_t n, double* __restrict__ Dc) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const bool on = e < n;
  const int64_t s0 = S * w / 4, s1 = S * (w + 1) / 4;
  double s = 0.0;
  if (on) {
#pragma unroll 8
    for (int64_t t = s0; t < s1; ++t) s += part[t * n + e];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && on) Dc[e] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// Candidate c's score from its distance row (krum_score's arithmetic).
__global__ void __launch_bounds__(256) krum_cand_score(const double* __restrict__ Dc, int64_t K,
                                                       int64_t kk, double* __restrict__ score) {
  extern __shared__ double srow[];
  __shared__ double scratch[8];
  const int64_t c = blockIdx.x;
  for (int64_t j = threadIdx.x; j < K; j += blockDim.x) srow[j] = Dc[c * K + j];
  __syncthreads();
  const double sc = krum_row_score(srow, K, kk, scratch);
  if (threadIdx.x == 0) score[c] = sc;
}

// The first minimum over the candidates (ascending indices: krum_argmin's tie rule).
__global__ void __launch_bounds__(64) krum_cand_argmin(const double* __restrict__ score,
                                                       const int64_t* __restrict__ cidx, int64_t m,
                                                       int64_t* __restrict__ index) {
  int64_t best = -1;
  double bv = 0.0;
  for (int64_t q = threadIdx.x; q < m; q += 64)
    if (best < 0 || score[q] < bv) { bv = score[q]; best = cidx[q]; }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o);
    const int64_t oi = __shfl_xor(best, o);
    if (oi >= 0 && (best < 0 || ov < bv || (ov == bv && oi < best))) { bv = ov; best = oi; }
  }
  if (threadIdx.x == 0) *index = best;
}

// out = row k (k on the host)
__global__ void __launch_bounds__(256) copy_row_k(const float* __restrict__ X, int64_t d,
                                                  int64_t ldx, int ws, int64_t k,
                                                  float* __restrict__ out) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < d;
       c += (int64_t)gridDim.x * blockDim.x)
    out[c] = *elem(X, ldx, ws, k, c);
}

static int grid_cols(int64_t d) {
  const int64_t g = (d + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

hipError_t launch_col_mean(const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                           hipStream_t s, int ws) {
  const bool vec4 = reinterpret_cast<uintptr_t>(X) % 16 == 0 && ldx % 4 == 0 && d % 4 == 0;
  if (vec4)
    hipLaunchKernelGGL(col_mean<4>, dim3(grid_cols(d / 4)), dim3(256), 0, s, X, K, d, ldx, ws, out);
  else
    hipLaunchKernelGGL(col_mean<1>, dim3(grid_cols(d)), dim3(256), 0, s, X, K, d, ldx, ws, out);
  return hipGetLastError();
}

hipError_t launch_col_select(const float* X, int64_t K, int64_t d, int64_t ldx, int mode,
                             int64_t b, float* out, hipStream_t s, int ws) {
  const int vec4 = reinterpret_cast<uintptr_t>(X) % 16 == 0 && ldx % 4 == 0;
  // GMAGG_SELECT_PERSIST=1: the persistent form (grid-stride tiles, the next tile's loads
  // in registers during the selection).  Measured slower on every shape, so off by default:
  // K=1000 x 2M median 6.14 vs 3.80 ms, trimmed mean 10.5 vs 7.05; K=256 2.07 vs 1.32 and
  // 4.04 vs 2.52 (two interleaved rounds, profiles/history/r3s2_select_persist_ab.txt)
  static const int persist = [] {
    const char* e = getenv("GMAGG_SELECT_PERSIST");
    return e ? atoi(e) : 0;
  }();
  // persistent: as many blocks as are co-resident (at most one per tile)
  auto resident = [&](const void* fn, int threads) -> unsigned {
    int dev = 0, cus = 256, occ = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, 0) != hipSuccess || occ < 1)
      occ = 1;
    return (unsigned)(cus * occ);
  };
  // the two modes are separate kernels (round 5): as one kernel with a runtime mode, the
  // trimmed mean's tail set the median's registers and schedule (K=256 median 1.20 -> 1.55 ms
  // when the trimmed mean's tail changed, profiles/r5s2_select_tm_ab.jsonl)
#define GMK_SEL_M(M, R, C, NWV)                                                                 \
  do {                                                                                          \
    const int64_t nt_ = (d + C - 1) / C;                                                        \
    if (persist) {                                                                              \
      const unsigned g_ = resident(reinterpret_cast<const void*>(&col_select<M, R, C, NWV, true>), \
                                   NWV * 64);                                                   \
      hipLaunchKernelGGL((col_select<M, R, C, NWV, true>),                                      \
                         dim3((unsigned)std::min<int64_t>(nt_, g_)), dim3(NWV * 64), 0, s, X, K, \
                         d, ldx, ws, b, vec4, out);                                             \
    } else {                                                                                    \
      hipLaunchKernelGGL((col_select<M, R, C, NWV, false>), dim3((unsigned)nt_), dim3(NWV * 64), \
                         0, s, X, K, d, ldx, ws, b, vec4, out);                                 \
    }                                                                                           \
  } while (0)
#define GMK_SEL(R, C, NWV)                                                                      \
  do {                                                                                          \
    if (mode == 0) GMK_SEL_M(0, R, C, NWV);                                                     \
    else GMK_SEL_M(1, R, C, NWV);                                                               \
  } while (0)
#define GMK_SEL1(R, C)                                                                          \
  do {                                                                                          \
    if (mode == 0)                                                                              \
      hipLaunchKernelGGL((col_select1<0, R, C>), dim3((unsigned)((d + C - 1) / C)), dim3(C * 64), \
                         0, s, X, K, d, ldx, ws, b, vec4, out);                                 \
    else                                                                                        \
      hipLaunchKernelGGL((col_select1<1, R, C>), dim3((unsigned)((d + C - 1) / C)), dim3(C * 64), \
                         0, s, X, K, d, ldx, ws, b, vec4, out);                                 \
  } while (0)
  // (round 4: gathering each wave's column pair straight from HBM, no LDS tile, so that
  // VGPRs rather than two 69.6-KB tiles limit the CU: K=1000 x 2M median 21.0 vs 3.83 ms —
  // 64 scattered 4-byte loads per wave instruction; profiles/r4s1_select_direct_ab.jsonl)
  // K <= 1024: 8 waves per 69.6-KB tile (one column pair each) so that the CU holds
  // 4 waves per SIMD (the LDS allows 2 tiles) instead of 2
  // one column per wave (col_select1) for the trimmed mean at 512 < K <= 1024: 6.29 ->
  // 5.90 ms at K=1000 x 2M; the median measured slower on it (3.87 -> 4.23 ms: its single
  // chain loses the paired wave sums and half the independent steps per wave), so the median
  // keeps the column-pair kernel (profiles/r4s2_select_1col_ab.jsonl).  GMAGG_SELECT_1COL:
  // 1 both, 0 neither (A/B); at K <= 256 see below
  static const int one_col_env = [] {
    const char* e = getenv("GMAGG_SELECT_1COL");
    return e ? atoi(e) : -1;
  }();
  const bool one_col = one_col_env < 0 ? mode == 1 : one_col_env != 0;
  // The median at 128 < K <= 1024 on the staged-transpose kernel (col_select_st: two
  // columns per wave, 8 waves, the tile never whole in LDS): x 2M columns, K = 200 / 256 /
  // 400 / 1000: 1.15 / 1.20 / 1.81 / 3.78 -> 1.01 / 1.05 / 1.42 / 3.19 ms; at K = 2000
  // (R = 32: 166 VGPRs) slower, 12.85 vs 12.17 (profiles/r5s2_select_st_ab.jsonl).  The
  // trimmed mean gains on it at K <= 512 (K = 256 / 400: 2.09 / 3.15 -> 1.95 / 2.99 ms) and
  // loses at K = 1000 (4.52 vs 4.22 on col_select1; profiles/r5s3_select_st_tm_ab.jsonl);
  // four columns per wave slower for both, forced 7 / 8 waves per SIMD (spills) slower too.
  // GMAGG_SELECT_ST: 0 never, 1 (default) the median to K = 1024 and the trimmed mean to
  // K = 512, 2 both to K = 1024 (A/B).
  static const int st_env = [] {
    const char* e = getenv("GMAGG_SELECT_ST");
    return e ? atoi(e) : 1;
  }();
  if (K > 128 && (st_env == 2 ? K <= 1024 : st_env == 1 && K <= (mode == 0 ? 1024 : 512))) {
    const dim3 g((unsigned)((d + 15) / 16));
#define GMK_ST(R_)                                                                              \
  do {                                                                                          \
    if (mode == 0)                                                                              \
      hipLaunchKernelGGL((col_select_st<0, R_, 2, 8>), g, dim3(512), 0, s, X, K, d, ldx, ws, b,   \
                         vec4, out);                                                            \
    else                                                                                        \
      hipLaunchKernelGGL((col_select_st<1, R_, 2, 8>), g, dim3(512), 0, s, X, K, d, ldx, ws, b,   \
                         vec4, out);                                                            \
  } while (0)
    if (K <= 256) GMK_ST(4);
    else if (K <= 512) GMK_ST(8);
    else GMK_ST(16);
#undef GMK_ST
    return hipGetLastError();
  }
  if (K <= 64) GMK_SEL(1, 32, 4);
  else if (K <= 128) GMK_SEL(2, 32, 4);
  // at 128 < K <= 256 the other way round: the median gains on one column per wave (1.34 ->
  // 1.26 ms at K=256 x 2M), the trimmed mean loses (2.24 -> 2.36); GMAGG_SELECT_1COL=2
  // puts both there (profiles/r4s2_select_1col_k256_ab.jsonl)
  else if (K <= 256 && (one_col_env < 0 ? mode == 0 : one_col_env == 2)) {
    GMK_SEL1(4, 16);
  }
  else if (K <= 256) GMK_SEL(4, 32, 4);
  else if (K <= 512) GMK_SEL(8, 16, 4);
  else if (K <= 1024 && one_col) {
    GMK_SEL1(16, 16);
  }
  else if (K <= 1024) GMK_SEL(16, 16, 8);
  else if (K <= 2048) GMK_SEL(32, 8, 4);
  else return hipErrorInvalidValue;
#undef GMK_SEL
#undef GMK_SEL_M
#undef GMK_SEL1
  return hipGetLastError();
}

// Column slices for pair_dist: the block count pairs * S is chosen so the grid fills
// whole rounds of co-resident blocks (time ~ rounds / S), partials <= 512 MiB.
int64_t krum_slices(int64_t K, int64_t d) {
  static int per_round = 0;                          // co-resident pair_dist blocks
  if (!per_round) {
    int dev = 0, cus = 256, occ = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, pair_dist<true>, kPDT, 0) != hipSuccess ||
        occ < 1)
      occ = 1;
    per_round = cus * occ;
  }
  const int64_t nT = (K + kPT - 1) / kPT, pairs = nT * (nT + 1) / 2;
  int64_t smax = (int64_t)(512ull << 20) / (8 * K * K);
  const int64_t stages = (d + kPC - 1) / kPC;
  if (smax > stages) smax = stages;
  if (smax > 4 * (int64_t)per_round) smax = 4 * (int64_t)per_round;
  if (smax < 1) return 1;
  int64_t best = 1;
  double best_cost = 1e300;
  for (int64_t S = 1; S <= smax; ++S) {
    const double cost = (double)((pairs * S + per_round - 1) / per_round) / (double)S;
    if (cost < best_cost * (1 - 1e-9)) { best_cost = cost; best = S; }
  }
  return best;
}

hipError_t launch_copy_row_k(const float* X, int64_t d, int64_t ldx, int ws, int64_t k, float* out,
                             hipStream_t s) {
  if (d > 0)
    hipLaunchKernelGGL(copy_row_k, dim3((unsigned)std::min<int64_t>((d + 255) / 256, 2048)),
                       dim3(256), 0, s, X, d, ldx, ws, k, out);
  return hipGetLastError();
}

hipError_t launch_krum_gram_select(const double* G, int KP, int64_t K, int64_t kk, double epsg,
                                   const int* bexp, int nb, int64_t d, double* lb, double* ub,
                                   int64_t maxc, int64_t* cand, hipStream_t s) {
  hipLaunchKernelGGL(krum_gram_bounds, dim3((unsigned)K), dim3(256), 2 * sizeof(double) * K, s, G,
                     KP, K, kk, epsg, bexp, nb, d, lb, ub);
  hipLaunchKernelGGL(krum_candidates, dim3(1), dim3(64), 0, s, lb, ub, K, maxc, cand);
  return hipGetLastError();
}

int krum_refine_max() { return kRefC; }

hipError_t launch_krum_refine(const float* X, int64_t K, int64_t d, int64_t ldx, int ws,
                              const int64_t* cidx, int m, int64_t kk, double* part, double* Dc,
                              double* score, hipStream_t s) {
  if (m < 1 || m > kRefC) return hipErrorInvalidValue;
  const int64_t S = krum_slices(K, d);
  const int64_t chunk = ((d + S - 1) / S + kPC - 1) / kPC * kPC;   // launch_krum's slices
  const bool vec = reinterpret_cast<uintptr_t>(X) % 16 == 0 && ldx % 4 == 0;
  const dim3 grid((unsigned)((K + 63) / 64), (unsigned)S);
  const int npp = ((m + 1) / 2 + 3) / 4;                         // pairs per thread
#define GMK_CAND(V_, N_)                                                                        \
  hipLaunchKernelGGL((krum_cand_dist<V_, N_>), grid, dim3(256), 0, s, X, K, d, ldx, ws, chunk, cidx, \
                     m, part)
  if (vec) {
    if (npp == 1) GMK_CAND(true, 1);
    else if (npp == 2) GMK_CAND(true, 2);
    else GMK_CAND(true, 4);
  } else {
    if (npp == 1) GMK_CAND(false, 1);
    else if (npp == 2) GMK_CAND(false, 2);
    else GMK_CAND(false, 4);
  }
#undef GMK_CAND
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t n = (int64_t)m * K;
  hipLaunchKernelGGL(krum_cand_reduce, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, part, S, n,
                     Dc);
  hipLaunchKernelGGL(krum_cand_score, dim3((unsigned)m), dim3(256), sizeof(double) * K, s, Dc, K, kk,
                     score);
  return hipGetLastError();
}

hipError_t launch_krum_pick(const double* score, const int64_t* cidx, int64_t m, const float* X,
                            int64_t d, int64_t ldx, int ws, int64_t* index, float* out,
                            hipStream_t s) {
  hipLaunchKernelGGL(krum_cand_argmin, dim3(1), dim3(64), 0, s, score, cidx, m, index);
  if (d > 0)
    hipLaunchKernelGGL(copy_row, dim3((unsigned)std::min<int64_t>((d + 255) / 256, 2048)),
                       dim3(256), 0, s, X, d, ldx, ws, index, out);
  return hipGetLastError();
}

hipError_t launch_krum(const float* X, int64_t K, int64_t d, int64_t ldx, int64_t kk, double* D,
                       double* part, double* score, float* out, int64_t* index, hipStream_t s,
                       int ws) {
  const int64_t nT = (K + kPT - 1) / kPT, pairs = nT * (nT + 1) / 2;
  const int64_t S = krum_slices(K, d);
  const int64_t chunk = ((d + S - 1) / S + kPC - 1) / kPC * kPC;
  const bool vec = reinterpret_cast<uintptr_t>(X) % 16 == 0 && ldx % 4 == 0;
  if (vec)
    hipLaunchKernelGGL(pair_dist<true>, dim3((unsigned)pairs, (unsigned)S), dim3(kPDT), 0, s, X, K,
                       d, ldx, ws, chunk, part);
  else
    hipLaunchKernelGGL(pair_dist<false>, dim3((unsigned)pairs, (unsigned)S), dim3(kPDT), 0, s, X,
                       K, d, ldx, ws, chunk, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pair_reduce, dim3((unsigned)((K * K + 63) / 64)), dim3(256), 0, s, part, S, K,
                     D);
  hipLaunchKernelGGL(krum_score, dim3((unsigned)K), dim3(256), sizeof(double) * K, s, D, K, kk,
                     score);
  hipLaunchKernelGGL(krum_argmin, dim3(1), dim3(64), 0, s, score, K, index);
  if (d > 0)
    hipLaunchKernelGGL(copy_row, dim3((unsigned)std::min<int64_t>((d + 255) / 256, 2048)),
                       dim3(256), 0, s, X, d, ldx, ws, index, out);
  return hipGetLastError();
}

}  // namespace gmk
