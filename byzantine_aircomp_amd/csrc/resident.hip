// Register-resident persistent Weiszfeld for small problems (BASELINE C1/C2:
// the reference's own K = 50 x d = 7850 MNIST aggregation, 1000 AirComp
// iterations per training step, 96 % of the reference's step time).
//
// At that size a launch-per-phase loop is launch-bound (3 kernels + polls per
// iteration).  Here ONE launch (every block co-resident) runs every iteration: each block
// owns CPB consecutive J-column chunks of X, loaded into VGPRs once; per
// iteration it
//   1. gathers every block's partials of the previous pass and reduces them in
//      a fixed order (every block computes the identical K-space step
//      redundantly: no broadcast),
//   2. takes the tol test (M:182) and forms the next coefficients (M:178-179,
//      or the OMA2 fold for gm, M:146-155 / M:401-412, Philox draws) — one
//      wave, lane = client, when K <= 64,
//   3. runs phases A/B of the streaming pass on its register tiles,
//   4. publishes its partials.
// The exchange is the data itself: every per-block partial (D2_k, ||x_k||^2, the
// movement and ||g||^2) is the block's fp64 sum rounded once to fp32 and carried by
// ONE 8-byte {tag, fp32 value} granule written by one relaxed store — agent scope
// (write-through), or, when the check-in finds every block on one XCD (C2's grid, round 4
// session 2), workgroup scope, which keeps the line in that XCD's L2; readers poll the
// granules with agent-scope relaxed loads (L2-served) until every tag equals the pass
// (cdna_hip_programming.md Guideline 16, R2), and sum the blocks' values in fp64 in a
// fixed order.  No
// grid barrier, no release/acquire fences: the r1 version (62 one-chunk blocks,
// counter barrier + fenced slab) spent 5.05 us of a 12.4 us iteration in the
// barrier and 2.15 us in the slab reduction.  Passes alternate
// between two granule buffers: a block writes pass p+2 into p's buffer only after
// it has read every block's pass p+1, which each block published after reading
// pass p, so no pass is overwritten before every block has read it.
// The iterate never leaves the chip until the final write.  Draw keys are the
// same as the launch-per-phase path's, so both give the same gm results to rounding:
// the two differ by the per-block fp32 rounding of the partials above and, at K <= 64,
// by the AirComp coefficients formed in fp32 here (fp64 there).
#include "device_util.h"
#include "gmagg_internal.h"
#include "philox.h"

#ifndef GMK_RES_SLEEP
#define GMK_RES_SLEEP 1   // spin back-off of the granule polls (A/B knob)
#endif
#ifndef GMK_RES_L2SLEEP
#define GMK_RES_L2SLEEP GMK_RES_SLEEP   // back-off of the hierarchical gather's level-2 polls (A/B)
#endif
#ifndef GMK_RES_POLL1
#define GMK_RES_POLL1 0   // poll one granule per chunk before reading the chunk (A/B knob; 0 was faster)
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

constexpr uint64_t kPollTicks = 200000000ull;   // 2 s at the 100 MHz real-time clock

// GMK_RES_DBG (probe builds only; 0 in the product): phases skipped to price the
// iteration's exchange alone (tools/gpu.sh probe steps, DESIGN.md §4 latency rooflines):
// 1 phase B's row sums, 2 the K-space step, 4 phase A's weighted sum.  7 leaves the
// gather, the barriers and the publish: the exchange floor of the protocol.
#ifndef GMK_RES_DBG
#define GMK_RES_DBG 0
#endif

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// One partial = ONE 8-byte granule {tag, fp32 value}: a block's partial is an fp64
// sum rounded once to fp32 (relative 6e-8; the reference's own norms are fp32
// sums, M:174/M:180), the sum over blocks is fp64.  Half the granules of an fp64
// {hi, lo} pair: the poll traffic on those lines is what the exchange costs.
// `local` (every block of the grid on ONE XCD, checked at check-in from XCC_ID): the
// store keeps the line in that XCD's L2 (workgroup scope: `sc0`), where the readers'
// `sc1` polls are served; an agent-scope (`sc1`) store drops it from the L2, so a
// same-XCD reader fetches it at the cross-XCD rate (MI355X_MICROARCH.md, store flavours).
// A granule is one 8-byte store either way (tag and value never torn apart).
// Hardware contract of the local form (gfx950 only — the library is built for nothing else):
// the HIP scoped model does not promise that a workgroup-scope store becomes visible to an
// agent-scope load of another workgroup; here it does because (1) gfx950's vector L1 is
// write-through, so the `sc0` store reaches the XCD's L2, and (2) the readers' `sc1` polls
// miss the L1 and read that same L2 — every block of a local grid sits on the one XCD
// (XCC_ID at the check-in).  tests/test_abi.py test_resident_granule_store_flavours pins the
// store / poll flavours in the ISA; a break would surface as the 2 s poll timeout, after
// which the call reruns on the streaming path (single problem) or fails loudly (batched
// pre-noise begun).
__device__ __forceinline__ void put_value(gu64* g, unsigned tag, float v, bool local = false) {
  const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
  if (local) __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over blocks b = g, g + G, g + 2G, ... (< nb, in that order) of one value of
// pass `tag`: the granule pairs are loaded at once (kNbChunk blocks per round
// trip) and re-read until every tag matches.  The poll is bounded in WALL time
// (s_memrealtime): on timeout (a time-sliced GPU, blocks not co-resident) the
// flag tmo is raised and every block gives up; the host then reruns the problem
// on the streaming path.
// The AirComp coefficients (K <= 64) on v_rcp / v_rsq (1 ulp) and fp32 square roots
// instead of IEEE divisions and fp64 square roots on the iteration's dependent chain: C2
// 228.4 -> 234.5 aggregations/s (profiles/r4s2_c2_coef_gather_ab.jsonl); 0 = the exact
// sequence (A/B knob)
#ifndef GMK_RES_FASTCOEF
#define GMK_RES_FASTCOEF 1
#endif
// Granules per poll round trip.  32 (>= C2's 31 blocks: one round trip, one stage, G = 1)
// spilled 336 bytes and measured 4x slower (55.9 aggregations/s, same A/B)
#ifndef GMK_RES_FUSE_COEF
#define GMK_RES_FUSE_COEF 0   // A/B knob: see the gather (one block barrier fewer per iteration)
#endif
#ifndef GMK_RES_NBCHUNK
#define GMK_RES_NBCHUNK 4
#endif
constexpr int kNbChunk = GMK_RES_NBCHUNK;

__device__ __forceinline__ bool gather_value(const gu64* g, int64_t bstride, unsigned b_first,
                                             unsigned b_step, unsigned nb, unsigned tag,
                                             gu32* tmo, double& sum) {
  sum = 0.0;
  for (unsigned b0 = b_first; b0 < nb; b0 += kNbChunk * b_step) {
    unsigned long long hi[kNbChunk];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; ++spins) {
      // wait on ONE granule of the chunk first: every thread of every block polls,
      // and re-reading the whole chunk per round multiplied the uncached poll
      // traffic on the few lines that hold the granules
#if GMK_RES_POLL1
      for (unsigned s1 = 0;; ++s1) {
        const unsigned long long h0 = __hip_atomic_load(g + (int64_t)b0 * bstride, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(h0 >> 32) == tag) break;
        __builtin_amdgcn_s_sleep(GMK_RES_SLEEP > 0 ? GMK_RES_SLEEP : 1);
        if ((s1 & 255u) == 255u && (__builtin_amdgcn_s_memrealtime() - t0 > kPollTicks ||
                                    __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return false;
        }
      }
#endif
      bool ok = true;
#pragma unroll
      for (int j = 0; j < kNbChunk; ++j) {
        const unsigned b = b0 + j * b_step;
        if (b < nb) {
          const gu64* q = g + (int64_t)b * bstride;
          hi[j] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(hi[j] >> 32) == tag;
        }
      }
      if (ok) break;
#if GMK_RES_SLEEP > 0
      __builtin_amdgcn_s_sleep(GMK_RES_SLEEP);
#endif
      if (((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t0 > kPollTicks) ||
          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
#pragma unroll
    for (int j = 0; j < kNbChunk; ++j)
      if (b0 + j * b_step < nb)
        sum += (double)__uint_as_float((unsigned)(hi[j] & 0xffffffffull));
  }
  return true;
}

// The split-scope exchange (a.split): gather_value over blocks whose granules sit in one of
// two copies — blocks b % 8 == mine (the reader's own XCD) from the L2-kept copy gL, every
// other block from the agent-scope copy g.  The same values in the same order: the same sum.
__device__ __forceinline__ bool gather_value_split(const gu64* g, const gu64* gL, int64_t bstride,
                                                   unsigned b_first, unsigned b_step, unsigned nb,
                                                   unsigned mine, unsigned tag, gu32* tmo,
                                                   double& sum) {
  sum = 0.0;
  for (unsigned b0 = b_first; b0 < nb; b0 += kNbChunk * b_step) {
    unsigned long long hi[kNbChunk];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < kNbChunk; ++j) {
        const unsigned b = b0 + j * b_step;
        if (b < nb) {
          const gu64* q = ((b & 7u) == mine ? gL : g) + (int64_t)b * bstride;
          hi[j] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(hi[j] >> 32) == tag;
        }
      }
      if (ok) break;
#if GMK_RES_SLEEP > 0
      __builtin_amdgcn_s_sleep(GMK_RES_SLEEP);
#endif
      if (((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t0 > kPollTicks) ||
          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
#pragma unroll
    for (int j = 0; j < kNbChunk; ++j)
      if (b0 + j * b_step < nb)
        sum += (double)__uint_as_float((unsigned)(hi[j] & 0xffffffffull));
  }
  return true;
}

// The XCD-hierarchical gather's second level: value v of the ng group sums, each an fp32
// {hi, lo} granule pair (hi + lo = the leader's fp64 sum to ~2^-48), polled in one round
// trip and summed in group order.
__device__ __forceinline__ bool gather_pairs(const gu64* g, int64_t gstride, unsigned ng,
                                             unsigned tag, gu32* tmo, double& sum) {
  unsigned long long hv[8], lv[8];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if ((unsigned)j < ng) {
        hv[j] = __hip_atomic_load(g + (int64_t)j * gstride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lv[j] = __hip_atomic_load(g + (int64_t)j * gstride + 1, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        ok &= (unsigned)(hv[j] >> 32) == tag && (unsigned)(lv[j] >> 32) == tag;
      }
    }
    if (ok) break;
#if GMK_RES_L2SLEEP > 0
    __builtin_amdgcn_s_sleep(GMK_RES_L2SLEEP);
#endif
    if (((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t0 > kPollTicks) ||
        __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  sum = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if ((unsigned)j < ng)
      sum += (double)__uint_as_float((unsigned)(hv[j] & 0xffffffffull)) +
             (double)__uint_as_float((unsigned)(lv[j] & 0xffffffffull));
  return true;
}

// Granule slots of one block and pass: value v at slot v;
//   v < K: D2_k; K <= v < 2K: ||x_k||^2 (INIT); 2K, 2K + 1: the block's movement
//   and ||g||^2 partials (summed over its waves in wave order).
template <int NW>
__host__ __device__ constexpr int64_t res_values(int64_t K) { return 2 * K + 2; }

// EXCH (the exchange, a template parameter so that each variant carries only its own code:
// C2's one-XCD kernel is the round-4 instruction stream): 0 flat (agent-scope, or L2-kept on
// one XCD), 1 the XCD-hierarchical gather, 2 the split-scope exchange (api.hip chooses)
template <int V, int NW, int LPR, int R, int CPB, int EXCH = 0>
__global__ void __launch_bounds__(NW * 64) weiszfeld_resident(ResArgs a) {
  constexpr int QW = 64 / LPR;
  constexpr int NRG = NW * QW;
  constexpr int J = LPR * V;
  constexpr int RPL = R > LPR ? R / LPR : 1;
  constexpr int SPAN = R < LPR ? LPR / R : 1;
  constexpr int KMAX = NRG * R;
  constexpr int JB = J * CPB;                       // columns per block
  static_assert(JB <= NW * 64, "one finisher column per thread");

  __shared__ float s_red[NW][JB];
  __shared__ float s_g[JB];
  __shared__ float s_coef[KMAX];
  __shared__ double s_d2[KMAX];
  __shared__ double s_r[KMAX];
  __shared__ double s_wp[2];
  __shared__ float s_h2[KMAX];
  __shared__ float s_nd;
  __shared__ double s_fin[2][NW];
  __shared__ double s_part[NW * 64];
  __shared__ double scratch[16];
  __shared__ float s_anoise;
  __shared__ int s_ok, s_same;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane % LPR, q = lane / LPR;
  const int rg = w * QW + q;
  const int64_t K = a.K, d = a.d;
  if (blockIdx.x % a.stride) return;                // (stride 8: a placeholder block)
  const unsigned bid = blockIdx.x / a.stride;       // logical block
  const unsigned nb = gridDim.x / a.stride;
  // XCD-hierarchical gather (a.hier, stride 1): group x = the blocks b % 8 == x, which
  // round-robin dispatch places on XCD x; the check-in numbers its slots group by group, so
  // each group's slots are contiguous and its `same` test covers exactly its members
  constexpr bool hier = EXCH == 1;
  // split scope (a.split, stride 1, not hier): one hop as the flat gather, each granule
  // published agent-scope AND L2-kept; a reader polls the L2-kept copies of its own group
  // (XCD) once the check-in confirms the group on one XCD
  constexpr bool split = EXCH == 2;
  const bool xg = hier || split;
  const unsigned XG = hier ? min(8u, nb) : 1u;
  const unsigned grp = xg ? bid % 8u : 0u;
  const unsigned nmem = hier ? (nb - grp + 7u) / 8u : nb;     // blocks this block gathers
  const unsigned ngrp = xg ? (nb - grp + 7u) / 8u : nb;       // blocks of this group
  const unsigned slot0 = xg ? grp * (nb / 8u) + min(grp, nb % 8u) : 0u;
  const unsigned slot = xg ? slot0 + bid / 8u : bid;
  const bool leader = hier && bid < 8u;                      // member 0 of its group
  const int64_t NV = res_values<NW>(K);            // values per block and pass
  const int64_t ch0 = (int64_t)bid * CPB;          // first chunk of this block
  const int64_t gj = ch0 * J + tid;                // finisher column (tid < JB)
  const bool fin = tid < JB && gj < d;
  gu64* gran = (gu64*)a.gran;                      // [2][nb][2 NV]
  gu32* tmo = (gu32*)a.bar + 2;
  // every block of the grid co-resident before anything is read (device_util.h)
  if (!grid_checkin(a.checkin, slot, a.need, a.bar + 2, a.bar + 3, kCheckinTicks, &s_ok, &s_same,
                    slot0, slot0 + ngrp))
    return;
  // identical in every block of the group (the same slots); hier: the group's member ->
  // leader granules only (the group sums always go agent-scope)
  const bool local = a.local && s_same && !split;
  const unsigned mine = (split && s_same) ? grp : 8u;        // split: the group read from gL
  gu64* granL = (gu64*)a.granL;                              // split: [2][nb][NV] L2-kept copies
  if (bid == 0 && tid == 0)                        // reported to the host (bar[0]: 1 + local)
    __hip_atomic_store((gu32*)a.bar, 1u + (unsigned)(local || mine < 8u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);

  // ---- the block's tiles: loaded once, resident for the whole call
  float x[CPB][R][V];
#pragma unroll
  for (int h = 0; h < CPB; ++h) {
    const int64_t col = (ch0 + h) * J + (int64_t)c * V;
    const bool cval = col < d;
    if (a.pstride == 0) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int64_t k = rg + (int64_t)NRG * i;
#pragma unroll
        for (int v = 0; v < V; ++v) x[h][i][v] = (cval && k < K) ? a.X[k * a.ldx + col + v] : 0.f;
      }
    } else {
      // panels: the V columns of a lane lie in one panel (V divides its width); the last
      // panel's padding past d is never read
      const int64_t W = (int64_t)1 << a.wshift;
      const float* pc = a.X + (col >> a.wshift) * a.pstride + (col & (W - 1));
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int64_t k = rg + (int64_t)NRG * i;
#pragma unroll
        for (int v = 0; v < V; ++v) x[h][i][v] = (cval && col + v < d && k < K) ? pc[k * W + v] : 0.f;
      }
    }
  }
  float gcur = fin ? a.guess0[gj] : 0.f;       // finisher thread: the iterate at column gj

  const int i_c = row_of_lane<LPR, R>(c);
  // row sums over the LPR lanes of a row segment: at LPR = 64 (the C2 tile) on gfx950's
  // permlane / DPP moves (device_util.h xlane_transpose64, the same lane -> row map)
  auto row_reduce = [&](float (&e)[R]) {
    if constexpr (LPR == 64) xlane_transpose64<R>(e, c);
    else transpose_reduce<LPR, R>(e, c);
  };
  // publish this block's partials of pass p (granules, tag p + 1, buffer p & 1)
  auto publish = [&](int64_t p, const double* racc, const double* racc2, double mv, double gn) {
    gu64* out = gran + ((p & 1) * nb + bid) * NV;
    gu64* outL = granL + ((p & 1) * nb + bid) * NV;
    const unsigned tag = (unsigned)(p + 1);
    auto put = [&](int64_t slot, float v) {
      put_value(out + slot, tag, v, local);
      if (split) put_value(outL + slot, tag, v, true);
    };
    if ((c % SPAN) == 0) {
#pragma unroll
      for (int m = 0; m < RPL; ++m) {
        const int64_t k = rg + (int64_t)NRG * (i_c + m);
        if (k < K) {
          put(k, (float)racc[m]);
          if (racc2) put(K + k, (float)racc2[m]);
        }
      }
    }
    if (tid == 0) {                 // s_fin: the waves' partials, published before a barrier
      double m = 0.0, g = 0.0;
      for (int ww = 0; ww < NW; ++ww) {
        m += s_fin[0][ww];
        g += s_fin[1][ww];
      }
      put(2 * K, (float)m);
      put(2 * K + 1, (float)g);
    }
  };
  // wave partials of the movement and ||g||^2 -> s_fin (read by publish after a
  // barrier): fp32 sums over the finisher lanes (as the reference's fp32 norms),
  // only in the waves that hold finisher columns
  auto wave_partials = [&](float mv, float gn) {
    if (w * 64 < JB) {   // (permlane / DPP moves, no LDS round trips: device_util.h)
      mv = xlane_wave_sum_f32(mv);
      gn = xlane_wave_sum_f32(gn);
    }
    if (lane == 0) {
      s_fin[0][w] = w * 64 < JB ? (double)mv : 0.0;
      s_fin[1][w] = w * 64 < JB ? (double)gn : 0.0;
    }
  };

  // ---- INIT: distances to g_0, ||x_k||^2 and ||g_0||^2 (pass 0)
  {
    double racc[RPL], racc2[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) racc[m] = racc2[m] = 0.0;
#pragma unroll
    for (int h = 0; h < CPB; ++h) {
      const int64_t col = (ch0 + h) * J + (int64_t)c * V;
      const bool cval = col < d;
      float gv[V];
#pragma unroll
      for (int v = 0; v < V; ++v) gv[v] = cval ? a.guess0[col + v] : 0.f;
      float e[R], e2[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float t = x[h][i][v] - gv[v];
          s1 = fmaf(t, t, s1);
          s2 = fmaf(x[h][i][v], x[h][i][v], s2);
        }
        e[i] = s1;
        e2[i] = s2;
      }
      row_reduce(e);
      row_reduce(e2);
#pragma unroll
      for (int m = 0; m < RPL; ++m) {
        racc[m] += (double)e[m];
        racc2[m] += (double)e2[m];
      }
    }
    wave_partials(0.f, fin ? gcur * gcur : 0.f);
    __syncthreads();
    publish(0, racc, racc2, 0.0, 0.0);
  }

  int64_t it = 0;
  double last_mv = NAN;
  int conv = 0;
  // the finisher column's AirComp noise draw of the coming pass: data-independent, so it
  // is drawn right after the previous pass is published, while the other blocks'
  // partials are still on their way (off the iteration's critical path)
  const bool col_noise = a.has_noise && a.mode == 1 && fin;
  float nz = col_noise ? normal1(a.seed, kStreamNoise, 0, (uint64_t)gj) : 0.f;
#ifdef GMK_RES_PROF
  uint64_t prof_[6] = {0, 0, 0, 0, 0, 0};
  uint64_t prev_ = __builtin_amdgcn_s_memrealtime();
#endif
  bool pre_h2 = false;
  bool fused = false;
  for (;; ++it) {
    // (1) gather pass `it` (INIT at it = 0): D2 (+ r at it = 0) and the per-wave
    // movement / norm partials.  G thread groups each sum every G-th block (in
    // block order, one round trip of loads), then the G group sums are added in
    // group order: a fixed order whatever the timing.
    {
      const gu64* in = gran + (it & 1) * nb * NV;
      const unsigned tag = (unsigned)(it + 1);
      const int nk = (int)(it == 0 ? 2 * K : K);
      const int ncol = nk + 2;
      const int G = max(1, min((int)blockDim.x / ncol, (int)((nmem + kNbChunk - 1) / kNbChunk)));
      // the K-space step's channel draws do not depend on the data: an idle wave
      // draws them while the others gather
      pre_h2 = a.mode == 1 && K <= 64 && G * ncol <= (NW - 1) * 64;
      if (pre_h2 && w == NW - 1) {
        if (lane < K) {
          float n4[4];
          normal4(a.seed, kStreamChannel, (uint64_t)it, (uint64_t)lane, n4);
          const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
          s_h2[lane] = hr * hr + hi * hi;                            // M:403
        }
        if (lane == 0)
          s_nd = a.has_noise ? normal1(a.seed, kStreamNoise, (uint64_t)it, (uint64_t)d) : 0.f;
      }
      // G > 1 only when G * ncol <= blockDim (= NW * 64 = the size of s_part): one
      // (group, value) per thread.  G == 1 (ncol > blockDim / 2, e.g. INIT's 2K + 2
      // values at K >= 512) sums every block in one thread and stores the value
      // directly: s_part is not used, so no value count can overrun it.
      auto store_value = [&](int cc, double sum) {
        if (cc < K) s_d2[cc] = sum;
        else if (cc < nk) s_r[cc - K] = sum;
        else s_wp[cc - nk] = sum;
      };
      bool ok = true;
      if (hier) {
        // level 1, the group's leader: its members' partials (the granules of blocks
        // grp + 8 m, m < nmem), G thread groups as below, summed in member order
        if (leader) {
          if (tid < G * ncol) {
            const int g = tid / ncol, cc = tid - g * ncol;
            const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
            double sum;
            if (gather_value(in + (int64_t)grp * NV + v, 8 * NV, (unsigned)g, (unsigned)G, nmem,
                             tag, tmo, sum))
              s_part[tid] = sum;
            else
              ok = false;
          }
          if (!ok) s_ok = 0;
          __syncthreads();
          if (s_ok == 0) return;
          gu64* l2o = (gu64*)a.lvl2 + ((int64_t)(it & 1) * 8 + grp) * 2 * NV;
          for (int cc = tid; cc < ncol; cc += blockDim.x) {
            double sum = 0.0;
            for (int g = 0; g < G; ++g) sum += s_part[g * ncol + cc];
            const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
            const float hi = (float)sum;
            put_value(l2o + 2 * v, tag, hi);
            put_value(l2o + 2 * v + 1, tag, (float)(sum - (double)hi));
          }
        }
        // level 2, every block: the XG group sums in group order (identical everywhere)
        const gu64* l2i = (const gu64*)a.lvl2 + (int64_t)(it & 1) * 8 * 2 * NV;
        for (int cc = tid; cc < ncol; cc += blockDim.x) {
          const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
          double sum;
          if (!gather_pairs(l2i + 2 * v, 2 * NV, XG, tag, tmo, sum)) {
            ok = false;
            break;
          }
          store_value(cc, sum);
        }
        if (!ok) s_ok = 0;
        __syncthreads();
        if (s_ok == 0) return;
      } else if (G == 1) {
        for (int cc = tid; cc < ncol; cc += blockDim.x) {
          const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
          double sum;
          const gu64* inL = granL + (it & 1) * nb * NV;
          if (!(split ? gather_value_split(in + v, inL + v, NV, 0u, 1u, nb, mine, tag, tmo, sum)
                      : gather_value(in + v, NV, 0u, 1u, nb, tag, tmo, sum))) {
            ok = false;
            break;
          }
          store_value(cc, sum);
        }
        if (!ok) s_ok = 0;
        __syncthreads();
        if (s_ok == 0) return;                     // timed out: every thread leaves
      } else {
        if (tid < G * ncol) {
          const int g = tid / ncol, cc = tid - g * ncol;
          const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
          double sum;
          const gu64* inL = granL + (it & 1) * nb * NV;
          if (split ? gather_value_split(in + v, inL + v, NV, (unsigned)g, (unsigned)G, nb, mine,
                                         tag, tmo, sum)
                    : gather_value(in + v, NV, (unsigned)g, (unsigned)G, nb, tag, tmo, sum))
            s_part[tid] = sum;
          else
            ok = false;
        }
        if (!ok) s_ok = 0;
        __syncthreads();
        if (s_ok == 0) return;                     // timed out: every thread leaves
        for (int cc = tid; cc < ncol; cc += blockDim.x) {
          double sum = 0.0;
          for (int g = 0; g < G; ++g) sum += s_part[g * ncol + cc];
          store_value(cc, sum);
        }
      }
      // GMK_RES_FUSE_COEF: when wave 0 alone summed the values (K <= 64, ncol <= 64) it also
      // forms the coefficients, so the block barrier between the two goes: a wave-scope
      // fence orders its lanes' LDS writes before their cross-lane reads, and the tol test
      // moves behind the coefficient step's barrier (the coefficients of a converged or
      // final pass are formed and not used)
      fused = GMK_RES_FUSE_COEF && K <= 64 && ncol <= 64 && G > 1 && it >= 1;
      if (fused) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
        __syncthreads();   // (s_wp is read in place: its next write follows this iteration's barriers)
      }
    }
    RES_T(0)
    // (2) tol test of the pass that produced g_it (M:180-183)
    auto tol_test = [&]() {
      if (it >= 1) {
        const float mv = (float)sqrt(s_wp[0]);
        last_mv = (double)mv;
        if (mv <= a.tol) {
          conv = 1;
          return true;
        }
      }
      return it == a.maxiter;
    };
    if (!fused && tol_test()) break;

    // (3) coefficients for pass `it`: one wave, lane = client, when K <= 64
    if constexpr ((GMK_RES_DBG & 2) != 0) {
      if (tid == 0) s_anoise = 0.f;
    } else if (K <= 64) {
      if (w == 0) {
        const int k = lane;
        const bool kv = k < K;
        if (a.mode == 0) {
          const double wk = kv ? 1.0 / (double)clamp_dist(s_d2[k], a.eps) : 0.0;
          const double W = xlane_wave_sum(wk);
          if (kv) s_coef[k] = (float)(wk / W);
          if (lane == 0) s_anoise = 0.f;
        } else if (GMK_RES_FASTCOEF) {
          // the same steps with the hardware reciprocal / reciprocal square root (1 ulp)
          // and fp32 square roots, off the iteration's dependent chain's slow sequences
          const float s = sqrtf((float)(s_wp[1] * (1.0 / (double)d)));      // M:146
          const float thr = (s * s) * 500.0f;                                  // M:152
          float ck = 0.f;
          if (kv) {
            float h2;
            if (pre_h2) {
              h2 = s_h2[k];
            } else {
              float n4[4];
              normal4(a.seed, kStreamChannel, (uint64_t)it, (uint64_t)k, n4);
              const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
              h2 = hr * hr + hi * hi;                                          // M:403
            }
            const float d0 = sqrtf((float)s_d2[k]);
            const float dist = d0 != d0 ? d0 : fmaxf(d0, a.eps);
            const float rd = __builtin_amdgcn_rcpf(dist);
            const float pk = ((float)s_r[k] + s * s) *
                             __builtin_amdgcn_rcpf(dist * dist * (float)(d + 1) * h2);  // M:404
            const float pup = pk != pk ? pk : fmaxf(pk, thr);                   // M:405
            ck = sqrtf((float)a.P_max) * __builtin_amdgcn_rsqf(pup) * rd;       // M:407
          }
          const float Sc = xlane_wave_sum_f32(ck);                             // fp32, as M:153
          const float nd = !a.has_noise ? 0.f
                           : (float)a.noise_sd * (pre_h2 ? s_nd
                                                         : normal1(a.seed, kStreamNoise,
                                                                   (uint64_t)it, (uint64_t)d));
          const float scale = s * __builtin_amdgcn_rcpf(s * Sc + nd);          // M:153-155
          if (kv) s_coef[k] = ck * scale;
          if (lane == 0) s_anoise = a.has_noise ? scale * (float)a.noise_sd : 0.f;
        } else {
          const float s = sqrtf((float)(s_wp[1] / (double)d));      // M:146
          const float thr = (s * s) * 500.0f;                         // M:152
          double ck = 0.0;
          if (kv) {
            float h2;
            if (pre_h2) {
              h2 = s_h2[k];
            } else {
              float n4[4];
              normal4(a.seed, kStreamChannel, (uint64_t)it, (uint64_t)k, n4);
              const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
              h2 = hr * hr + hi * hi;                                 // M:403
            }
            // fp32, the reference's own precision (M:403-407): the wave's fp64 divisions
            // and square roots sat on the iteration's critical path; C2 6.38 -> 6.24-6.35 ms
            // per aggregation (profiles/history/r2_c2_kspace_fp32.txt)
            const float dist = clamp_dist(s_d2[k], a.eps);
            const float pk = ((float)s_r[k] + s * s) / (dist * dist * (float)(d + 1)) / h2;   // M:404
            const float pup = pk != pk ? pk : fmaxf(pk, thr);          // M:405
            ck = (double)(sqrtf((float)a.P_max / pup) / dist);         // M:407
          }
          const double Sc = xlane_wave_sum(ck);
          const double nd = !a.has_noise ? 0.0
                            : a.noise_sd * (double)(pre_h2 ? s_nd
                                                           : normal1(a.seed, kStreamNoise,
                                                                     (uint64_t)it, (uint64_t)d));
          const double scale = (double)s / ((double)s * Sc + nd);     // M:153-155
          if (kv) s_coef[k] = (float)(ck * scale);
          if (lane == 0) s_anoise = a.has_noise ? (float)(scale * a.noise_sd) : 0.f;
        }
      }
    } else if (a.mode == 0) {
      double wsum = 0.0;
      for (int64_t k = tid; k < K; k += blockDim.x) wsum += 1.0 / (double)clamp_dist(s_d2[k], a.eps);
      const double W = block_sum(wsum, scratch);
      for (int64_t k = tid; k < K; k += blockDim.x)
        s_coef[k] = (float)((1.0 / (double)clamp_dist(s_d2[k], a.eps)) / W);
      if (tid == 0) s_anoise = 0.f;
    } else {
      const float s = sqrtf((float)(s_wp[1] / (double)d));      // M:146
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
        const double pk = (s_r[k] + s2) / (dd * dd * (double)(d + 1)) / (double)h2;   // M:404
        const double pup = pk != pk ? pk : fmax(pk, (double)thr);  // M:405
        const double ck = sqrt(a.P_max / pup) / dd;                // M:407
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
    if (fused && tol_test()) break;
    RES_T(1)

    // (4) phase A on the resident tiles
    float wt[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t k = rg + (int64_t)NRG * i;
      wt[i] = k < K ? s_coef[k] : 0.f;
    }
#pragma unroll
    for (int h = 0; h < CPB; ++h) {
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
      if constexpr ((GMK_RES_DBG & 4) == 0) {
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = fmaf(wt[i], x[h][i][v], acc[v]);
      }
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += __shfl_xor(acc[v], o, 64);
      if (q == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) s_red[w][h * J + c * V + v] = acc[v];
      }
    }
    __syncthreads();
    float mvp = 0.f, gnp = 0.f;
    if (tid < JB) {
      float gnew = 0.f;
      if (fin) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sum += s_red[ww][tid];
        gnew = sum;
        if (col_noise) gnew = fmaf(s_anoise, nz, gnew);
        const float diff = gcur - gnew;
        mvp = diff * diff;
        gnp = gnew * gnew;
        gcur = gnew;
      }
      s_g[tid] = gnew;
    }
    wave_partials(mvp, gnp);
    __syncthreads();
    RES_T(2)
    // (5) phase B: distances to the new iterate, every chunk, fp64 across chunks
    double racc[RPL];
#pragma unroll
    for (int m = 0; m < RPL; ++m) racc[m] = 0.0;
#pragma unroll
    for (int h = 0; h < CPB && (GMK_RES_DBG & 1) == 0; ++h) {
      float gv[V];
#pragma unroll
      for (int v = 0; v < V; ++v) gv[v] = s_g[h * J + c * V + v];
      float e[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        float s1 = 0.f;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float t = x[h][i][v] - gv[v];
          s1 = fmaf(t, t, s1);
        }
        e[i] = s1;
      }
      row_reduce(e);
#pragma unroll
      for (int m = 0; m < RPL; ++m) racc[m] += (double)e[m];
    }
    RES_T(3)
    publish(it + 1, racc, nullptr, mvp, gnp);
    if (col_noise) nz = normal1(a.seed, kStreamNoise, (uint64_t)(it + 1), (uint64_t)gj);
    RES_T(4)
  }
#ifdef GMK_RES_PROF
  if (bid == 0 && threadIdx.x == 0)
    printf("GMK_RES_PROF nb=%u CPB=%d iters=%ld ns/iter: gather %.0f coef %.0f phaseA %.0f "
           "phaseB %.0f publish %.0f\n", nb, CPB, (long)it, 10.0 * prof_[0] / it,
           10.0 * prof_[1] / it, 10.0 * prof_[2] / it, 10.0 * prof_[3] / it, 10.0 * prof_[4] / it);
#endif

  if (fin) a.out[gj] = gcur;
  if (bid == 0 && tid == 0) {
    a.st->iters = it;
    a.st->last_movement = last_mv;
    a.st->converged = conv;
    a.st->done = 1;
  }
}

// ---------------------------------------------------------------------------

// Chunks per block: CPB * J columns must map one finisher column per thread, and
// the tile x[CPB][R][V] must stay within 16 VGPRs (1024-thread blocks have 128
// VGPRs; 32-register tiles spilled).
#ifndef GMK_RES_TILE_REGS
#define GMK_RES_TILE_REGS 16   // A/B knob: 32 allows 16 blocks at C2 (with spills)
#endif
constexpr bool res_cpb_ok(int V, int NW, int LPR, int R, int CPB) {
  // (512-thread blocks have 256 VGPRs per lane: a 64-register tile fits)
  return CPB == 1 || (CPB * LPR * V <= NW * 64 &&
                      CPB * R * V <= (NW >= 16 ? GMK_RES_TILE_REGS : 64));
}

template <int V, int NW, int LPR, int R, int CPB>
static const void* res_fn(int xg) {
  // the hierarchical / split-scope variants exist for the 8-wave tile (32 < K <= 64, where
  // they measured faster); every other tile gathers flat beyond one XCD
  if constexpr (res_cpb_ok(V, NW, LPR, R, CPB)) {
    if (xg == 0) return reinterpret_cast<const void*>(&weiszfeld_resident<V, NW, LPR, R, CPB>);
    if constexpr (NW == 8 && LPR == 64 && R == 8) {
      if (xg == 1) return reinterpret_cast<const void*>(&weiszfeld_resident<V, NW, LPR, R, CPB, 1>);
      if (xg == 2) return reinterpret_cast<const void*>(&weiszfeld_resident<V, NW, LPR, R, CPB, 2>);
    }
  }
  return nullptr;
}

static const void* resident_kernel(const PassCfg& cfg, int cpb, int xg = 0) {
#define GMK_RES(V_, W_, L_, R_)                                              \
  if (cfg.V == V_ && cfg.NW == W_ && cfg.LPR == L_ && cfg.R == R_) {         \
    switch (cpb) {                                                           \
      case 1: return res_fn<V_, W_, L_, R_, 1>(xg);                          \
      case 2: return res_fn<V_, W_, L_, R_, 2>(xg);                          \
      case 3: return res_fn<V_, W_, L_, R_, 3>(xg);                          \
      case 4: return res_fn<V_, W_, L_, R_, 4>(xg);                          \
      case 8: return res_fn<V_, W_, L_, R_, 8>(xg);                          \
      default: return nullptr;                                               \
    }                                                                        \
  }
#define GMK_RES_V(V_)                                                                         \
  GMK_RES(V_, 16, 64, 1) GMK_RES(V_, 16, 64, 2) GMK_RES(V_, 16, 64, 4) GMK_RES(V_, 16, 64, 8)   \
  GMK_RES(V_, 16, 32, 8) GMK_RES(V_, 16, 16, 8) GMK_RES(V_, 16, 8, 8) GMK_RES(V_, 16, 4, 8)    \
  GMK_RES(V_, 8, 64, 8) GMK_RES(V_, 4, 64, 16)
  GMK_RES_V(4)
  GMK_RES_V(2)
  GMK_RES_V(1)
#undef GMK_RES_V
#undef GMK_RES
  return nullptr;
}

// Blocks of CPB chunks each: the smallest CPB (up to 8) that brings the grid to at most
// kResTargetBlocks blocks, or the largest valid one; GMAGG_RES_CPB=n forces
// n (A/B).  Returns false when the grid cannot be co-resident.
constexpr int kResTargetBlocks = 32;   // one XCD's CUs (the L2-kept exchange, api.hip)

bool resident_plan(const PassCfg& cfg, int64_t nch, int num_cu, int* cpb_out, int* nb_out) {
  int cpb = 0;
  if (const char* e = getenv("GMAGG_RES_CPB")) {
    cpb = atoi(e);
    if (!resident_kernel(cfg, cpb)) return false;
  } else {
    for (int c = 1; c <= 8; c *= 2) {
      if (!resident_kernel(cfg, c)) break;
      cpb = c;
      if ((nch + c - 1) / c <= kResTargetBlocks) break;
    }
    // beyond one XCD in the hierarchical gather's range (>= 90 blocks of the largest
    // tile): half the columns per block, twice the blocks (up to 192), measured faster —
    // 50 x 48,670 (V = 2) 96 -> 191 blocks 7.6 -> 7.0 us per iteration, 40 / 64 x 48,670
    // likewise, 50 x 48,671 (V = 1) 7.8 -> 7.3; at 40-80 blocks the larger blocks stay
    // ahead (50 x 20,001: 6.7 vs 7.2; profiles/r5s3_resident_cpb_*ab.jsonl).  The 8-wave
    // tile only (32 < K <= 64, the one with the hierarchical gather): the flat gather of
    // the K <= 32 tiles ran slower on smaller blocks (20 / 30 x 48,670: 6.4 / 6.6 -> 7.3 /
    // 7.6; profiles/r5s3_resident_halve_ab.jsonl)
    static const bool halve = [] {           // GMAGG_RES_HALVE=0: the largest tile (A/B)
      const char* e = getenv("GMAGG_RES_HALVE");
      return !e || atoi(e) != 0;
    }();
    const int64_t nb0 = cpb ? (nch + cpb - 1) / cpb : 0;
    const bool hier_tile = cfg.NW == 8 && cfg.LPR == 64 && cfg.R == 8;   // 32 < K <= 64
    if (halve && hier_tile && cpb >= 2 && nb0 > kResTargetBlocks && nb0 >= 90 &&
        (nch + cpb / 2 - 1) / (cpb / 2) <= 192 && resident_kernel(cfg, cpb / 2))
      cpb /= 2;
  }
  if (cpb == 0) return false;
  const void* fn = resident_kernel(cfg, cpb);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, cfg.NW * 64, 0) != hipSuccess) return false;
  const int64_t nb = (nch + cpb - 1) / cpb;
  if (nb > (int64_t)n * num_cu) return false;
  *cpb_out = cpb;
  *nb_out = (int)nb;
  return true;
}

size_t resident_gran_words(int64_t K, const PassCfg& cfg, int nb) {
  (void)cfg;
  // [2][nb][2K + 2] granules, then nb + 1 co-residency check-in slots, then the
  // hierarchical gather's group sums [2][8][2 (2K + 2)], then the split-scope exchange's
  // L2-kept copies [2][nb][2K + 2]
  return (size_t)4 * nb * (size_t)(2 * K + 2) + (size_t)nb + 1 + (size_t)32 * (2 * K + 2);
}

bool res_coop_launch() {
  static const bool coop = [] {
    const char* e = getenv("GMAGG_RES_COOP");
    return e && atoi(e) != 0;
  }();
  return coop;
}

bool resident_has_exchange(const PassCfg& cfg, int cpb, int xg) {
  return resident_kernel(cfg, cpb, xg) != nullptr;
}

hipError_t launch_resident(const PassCfg& cfg, int cpb, int grid, const ResArgs& a, hipStream_t s) {
  const void* fn = resident_kernel(cfg, cpb, a.hier ? 1 : a.split ? 2 : 0);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<ResArgs*>(&a)};
  // A plain launch by default: co-residency is established by resident_plan's occupancy
  // test (and policed by the wall-clock-bounded polls), not by a cooperative launch.  A
  // process that made a cooperative launch segfaults inside the ROCm runtime's exit
  // handlers under rocprofv3 --kernel-trace — a 40-line program with none of this library
  // does too (tools/coop_exit_probe.hip, profiles/history/r3s2_c2_exit_crash.txt) — and the plain
  // launch costs nothing (C2 158.4 vs 159.7 aggregations/s, interleaved A/B).
  // GMAGG_RES_COOP=1: the cooperative launch (A/B).
  const bool coop = res_coop_launch();
  if (!coop) return hipLaunchKernel(fn, dim3(grid), dim3(cfg.NW * 64), args, 0, s);
  return hipLaunchCooperativeKernel(fn, dim3(grid), dim3(cfg.NW * 64), args, 0, s);
}

}  // namespace gmk
