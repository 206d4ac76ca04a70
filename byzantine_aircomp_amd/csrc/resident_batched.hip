// Register-resident batched Weiszfeld: many independent small problems (BASELINE C5,
// the draw.ipynb-style sweep: K = 50 x d = 100k per problem) with every problem's X
// read from HBM ONCE.
//
// The streaming batched path (stream_pass.hip, blockIdx.y = problem) reads X once
// per pass: INIT + ~4.7 iterations = ~5.7 reads of 20 MB per problem.  A K = 50 x
// 100k problem is 20 MB; the chip's VGPR file is 128 MiB, so ~5 problems fit in
// registers at once.  Here the grid is NG groups of NB co-resident blocks; group g
// runs problems g, g + NG, ... one after the other, each with its K x (NB * 2048)
// tile held in VGPRs for all of its iterations:
//   load the tile (+ the reference's OMA pre-noise, M:385-394, applied in registers
//   and written back: gm2 --var, M:351-352), INIT partials, then per iteration the
//   gather of every block's partials, the tol test (M:180-183), the coefficients
//   (M:178-179, or OMA2's for gm, M:146-155 / M:401-412), phase A (g' = sum c_k x_k,
//   no cross-thread reduction: a thread owns whole columns) and phase B (the next
//   distances), then the publish.
// The exchange is resident.hip's (tagged fp32 granules, agent-scope relaxed stores and
// polls, no barrier, no fences, a wall-clock-bounded poll); the group's pass counter
// runs on across its problems, so tags never repeat within a launch.
//
// Thread map (512 threads = 8 waves, 2 per SIMD, <= 256 VGPRs): thread (wave w, lane l)
// owns the 4 columns bi * 2048 + w * 256 + 4 l + {0..3} of block bi, ALL K rows of them
// (x[KR][4], KR = K rounded up); a wave's float4 load of one row reads 1 KiB of
// contiguous columns (rows layout) or two 512-B panel rows (panels, W = 128).
// Row sums (the distances D_k) are transpose-reduced over the wave 16 rows at a time
// (device_util.h), summed over the 8 waves in fp64 and published rounded to fp32, as in
// resident.hip; the sum over blocks is fp64 in a fixed order.
#include <algorithm>
#include <type_traits>
#include "device_util.h"
#include "gmagg_internal.h"
#include "philox.h"

namespace gmk {

namespace {

constexpr int kRbCols = 2048;                    // columns per block
constexpr uint64_t kRbPollTicks = 200000000ull;  // 2 s at the 100 MHz real-time clock
constexpr int kRbChunk = 8;                      // granules in flight per poll round

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void rb_put(gu64* g, unsigned tag, float v) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over blocks b = first, first + step, ... < nb of the value at g + b * bstride of
// pass `tag` (kRbChunk granules per round trip, re-read until every tag matches; the
// poll is bounded in wall time and raises *tmo on expiry).
__device__ __forceinline__ bool rb_gather(const gu64* g, int64_t bstride, int first, int step,
                                          int nb, unsigned tag, gu32* tmo, double& sum) {
  sum = 0.0;
  for (int b0 = first; b0 < nb; b0 += kRbChunk * step) {
    unsigned long long v[kRbChunk];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < kRbChunk; ++j) {
        const int b = b0 + j * step;
        if (b < nb) {
          v[j] = __hip_atomic_load(g + (int64_t)b * bstride, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(v[j] >> 32) == tag;
        }
      }
      if (ok) break;
      __builtin_amdgcn_s_sleep(1);
      if (((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t0 > kRbPollTicks) ||
          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
#pragma unroll
    for (int j = 0; j < kRbChunk; ++j)
      if (b0 + j * step < nb) sum += (double)__uint_as_float((unsigned)(v[j] & 0xffffffffull));
  }
  return true;
}

// transpose_reduce<64, R> (device_util.h) with the lane-dependent keep / send choice
// made on the bits (x ^ ((x ^ y) & m)): written as selects, the compiler turned them
// into selects of ARRAY INDICES hoisted out of the row blocks, and every use of e[]
// into a compare / v_cndmask chain over the whole array (1,350 of each per kernel and
// 180 VGPRs of index tables).  Same results: the bits of one operand are taken whole.
template <int R>
__device__ __forceinline__ void rb_transpose(float (&e)[R], int c) {
  constexpr int STEPS = ilog2<R>::v;
#pragma unroll
  for (int step = 0; step < STEPS; ++step) {
    const int half = R >> (step + 1);
    const int o = 32 >> step;
    const unsigned m = (c & o) ? 0xffffffffu : 0u;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const unsigned lo = __float_as_uint(e[i]), hi = __float_as_uint(e[i + half]);
      const unsigned x = (lo ^ hi) & m;
      const float keep = __uint_as_float(lo ^ x), send = __uint_as_float(hi ^ x);
      e[i] = keep + __shfl_xor(send, o, 64);
    }
  }
#pragma unroll
  for (int o = 64 / (2 * R); o >= 1; o >>= 1) e[0] += __shfl_xor(e[0], o, 64);
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N).  Every row index
// of the tile is a constant expression, so the tile is always split into registers (with
// plain `#pragma unroll` loops the 52-row kernel's tile was left in scratch).
template <int I0, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>{});
    sfor<I0 + 1, N>(f);
  }
}

// Rows [K0, K0 + R) of a per-thread row quantity (f(k) over the thread's 4 columns),
// transpose-reduced over the wave: lane c ends with row K0 + row_of_lane<64, R>(c);
// the lanes c % (64 / R) == 0 hold distinct rows and store them to srow.
template <int R, int K0, int KR, class F>
__device__ __forceinline__ void rb_rows(F f, float* srow, int lane) {
  float e[R];
  sfor<0, R>([&](auto i) { e[i] = f(std::integral_constant<int, K0 + i>{}); });
  rb_transpose<R>(e, lane);
  if ((lane % (64 / R)) == 0) srow[K0 + row_of_lane<64, R>(lane)] = e[0];
  // one row block at a time: interleaving the blocks (the scheduler's choice) holds every
  // block's e[] at once, KR more live registers beside the tile
  __builtin_amdgcn_sched_barrier(0);
}

// All KR rows: blocks of 16, then a tail of 8 and / or 4 (KR % 4 == 0).
template <int KR, int K0 = 0, class F>
__device__ __forceinline__ void rb_all_rows(F f, float* srow, int lane) {
  if constexpr (KR - K0 >= 16) {
    rb_rows<16, K0, KR>(f, srow, lane);
    rb_all_rows<KR, K0 + 16>(f, srow, lane);
  } else if constexpr (KR - K0 >= 8) {
    rb_rows<8, K0, KR>(f, srow, lane);
    rb_all_rows<KR, K0 + 8>(f, srow, lane);
  } else if constexpr (KR - K0 >= 4) {
    rb_rows<4, K0, KR>(f, srow, lane);
  }
}

}  // namespace

template <int KR, int KV, int MODE>
__global__ void __launch_bounds__(512) weiszfeld_resident_batched(ResBArgs a) {
  // KR rows per column (K rounded up to 4): rows [0, KV) live in the thread's VGPRs, rows
  // [KV, KR) in LDS (s_x, the thread's own 16 bytes per row).  MODE: gm_mode, a template
  // parameter so that the gm2 kernel carries none of the AirComp code's registers.
  static_assert(KR % 4 == 0 && KV % 4 == 0 && KV <= KR && KR <= 64, "rows per thread");
  constexpr int NT = 512;
  constexpr int NW = NT / 64;
  constexpr int KL = KR - KV;                      // rows held in LDS
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  __shared__ f4 s_x[KL > 0 ? KL : 1][NT];
  __shared__ float s_coef[KR];
  __shared__ float s_osc[KR];
  __shared__ float s_rows[NW][KR];
  __shared__ float s_rows2[NW][KR];
  __shared__ double s_d2[KR];
  __shared__ double s_r[KR];
  __shared__ double s_wp[2];
  __shared__ float s_fin[2][NW];
  __shared__ double s_part[NT];
  __shared__ float s_anoise;
  __shared__ int s_ok;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NB = a.nb;
  const int grp = (int)blockIdx.x / NB, bi = (int)blockIdx.x - grp * NB;
  const int NG = (int)gridDim.x / NB;
  const int64_t K = a.K, d = a.d;
  const int64_t NV = 2 * K + 2;                    // granule slots per block and pass
  gu64* gran = (gu64*)a.gran + (int64_t)grp * 2 * NB * NV;
  gu32* tmo = (gu32*)a.flag;
  const int64_t W = a.pstride ? ((int64_t)1 << a.wshift) : 0;
  const int64_t rstride = a.pstride ? W : a.ldx;   // between rows k and k + 1
  // this thread's 4 columns: 256 w + 4 lane of the block's 2048 (one wave instruction
  // reads 256 contiguous columns of a row)
  const int64_t col0 = (int64_t)bi * kRbCols + w * 256 + lane * 4;
  const bool full = col0 + 3 < d, any = col0 < d;
  // element (k, col0) of a problem: rows [k][ldx], panels [(j/W)][K][W]
  const int64_t e0 = a.pstride ? (col0 >> a.wshift) * a.pstride + (col0 & (W - 1)) : col0;
  const uint32_t voff = any ? (uint32_t)(e0 * 4) : 0x80000000u;
  if (tid == 0) s_ok = 1;
  if (tid < KR) s_coef[tid] = 0.f;

  f4 x[KV > 0 ? KV : 1];   // the tile's register rows: row k of the thread's 4 columns
  float g[4];              // the iterate at those columns
  unsigned pc = 0;   // passes this group has published (pass pc: tag pc + 1, buffer pc & 1)
  // row k of the tile (k a constant expression): registers or LDS
  auto row = [&](auto k) -> f4 {
    if constexpr (k < KV) return x[k];
    else return s_x[k - KV][tid];
  };
  auto set_row = [&](auto k, f4 v) {
    if constexpr (k < KV) x[k] = v;
    else s_x[k - KV][tid] = v;
  };

  // publish this block's partials of pass pc: D_k (threads k < K), r_k (threads 64 + k,
  // INIT of gm), the movement / ||g||^2 (thread 128), from s_rows / s_rows2 / s_fin
  auto publish = [&](bool with_r) {
    gu64* out = gran + ((int64_t)(pc & 1) * NB + bi) * NV;
    const unsigned tag = pc + 1;
    if (tid < K) {
      double sm = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sm += (double)s_rows[ww][tid];
      rb_put(out + tid, tag, (float)sm);
    }
    if (with_r && tid >= 64 && tid < 64 + K) {
      const int k = tid - 64;
      double sm = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sm += (double)s_rows2[ww][k];
      rb_put(out + K + k, tag, (float)sm);
    }
    if (tid == 128) {
      double m = 0.0, gg = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        m += (double)s_fin[0][ww];
        gg += (double)s_fin[1][ww];
      }
      rb_put(out + 2 * K, tag, (float)m);
      rb_put(out + 2 * K + 1, tag, (float)gg);
    }
  };
  auto wave_fin = [&](float mv, float gn) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mv += __shfl_xor(mv, o, 64);
      gn += __shfl_xor(gn, o, 64);
    }
    if (lane == 0) {
      s_fin[0][w] = mv;
      s_fin[1][w] = gn;
    }
  };
  // the per-row squared distance over the thread's columns, in column order
  auto dist_row = [&](auto k) {
    const f4 r = row(k);
    float sm = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float t = r[v] - g[v];
      sm = fmaf(t, t, sm);
    }
    return sm;
  };

  for (int64_t p = grp; p < a.P; p += NG) {
    const float* Xp = a.X + p * a.x_ps;
    const uint64_t seed_p = a.seed + (uint64_t)p * kSeedStride;

    // ---- the problem's tile: loaded once (streamed: X is read once).  One buffer
    // resource per problem and row (SGPRs; the base made wave-uniform explicitly: a
    // resource the compiler cannot prove uniform is used through a readfirstlane
    // waterfall loop per load, each ending in vmcnt(0)), the thread's column offset in one
    // VGPR, the row offset scalar.  Rows past K load through a zero-record resource (the
    // range check returns 0) and threads past d use an out-of-range offset, so every load
    // writes its tile registers directly: no branch per row (each load its own basic
    // block, ended by vmcnt(0)) and no masking pass (twice the live registers).
    const uint64_t xb = reinterpret_cast<uint64_t>(Xp);
    // (readfirstlane returns int: each half goes through unsigned, or a low half >= 2^31
    // sign-extends over the high half)
    float* const Xu = reinterpret_cast<float*>(
        ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(xb >> 32)) << 32) |
        (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)xb));
    const int nrec = __builtin_amdgcn_readfirstlane(a.prob_bytes);
    auto rsrc = [&](auto k) {
      return __builtin_amdgcn_make_buffer_rsrc(Xu, 0, k < K ? nrec : 0, 0x00020000);
    };
    auto roff = [&](auto k) { return __builtin_amdgcn_readfirstlane((int)(k * rstride * 4)); };
    if constexpr (KL > 0) __syncthreads();   // s_x of the previous problem fully read
    sfor<0, KR>([&](auto k) {
      f4 v = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(k), voff, roff(k), 2));
      if (!full) {                 // the partial last group: columns >= d are 0
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (col0 + u >= d) v[u] = 0.f;
      }
      set_row(k, v);
    });
    // ---- OMA pre-noise (M:385-394), the draws of gm_oma_philox_f32 / the fused pass:
    // element (k, j) takes normal j & 3 of the Philox block (row k, j >> 2), scaled by the
    // row's sd / |h_k|; written back in place (the reference's OMA mutates wList).  Rows
    // past K: scale 0 (they stay 0) and a zero-record resource (their stores are dropped).
    if (a.pre_oma) {
      const uint64_t oseed = a.oma_seed + (uint64_t)p * kSeedStride;
      __syncthreads();   // s_osc of the previous problem fully read
      if (tid < KR) s_osc[tid] = tid < K ? oma_row_scale(oseed, (uint64_t)tid, a.oma_sd) : 0.f;
      __syncthreads();
      sfor<0, KR>([&](auto k) {
        const float sc = s_osc[k];
        float z[4];
        normal4_hw(oseed, kStreamOmaNoise, (uint64_t)k, (uint64_t)col0 >> 2, z);
        f4 v = row(k);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (col0 + u < d) v[u] = oma_noisy(v[u], sc, z[u]);
        set_row(k, v);
        if (full) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), rsrc(k), voff,
                                                 roff(k), 0);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[u]), rsrc(k),
                                                  col0 + u < d ? voff + 4 * u : 0x80000000u,
                                                  roff(k), 0);
        }
        __builtin_amdgcn_sched_barrier(0);   // one row's draws at a time
      });
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) g[v] = col0 + v < d ? a.guess0[p * a.ldg + col0 + v] : 0.f;

    // ---- INIT (pass pc): D_k to g_0, ||x_k||^2 (gm), ||g_0||^2
    constexpr bool want_r = MODE == 1;
    __syncthreads();   // s_rows / s_fin of the previous problem's last publish consumed
    rb_all_rows<KR>(dist_row, &s_rows[w][0], lane);
    if constexpr (want_r) {
      rb_all_rows<KR>([&](auto k) {
        const f4 r = row(k);
        float sm = 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) sm = fmaf(r[v], r[v], sm);
        return sm;
      }, &s_rows2[w][0], lane);
    }
    {
      float gn = 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) gn = fmaf(g[v], g[v], gn);
      wave_fin(0.f, gn);
    }
    __syncthreads();
    publish(want_r);

    int64_t it = 0;
    double last_mv = NAN;
    int conv = 0;
    for (;; ++it) {
      // (1) gather pass pc: D (+ r at INIT of gm), movement, ||g||^2; G thread groups
      // each sum every G-th block, then the group sums are added in group order
      {
        const gu64* in = gran + (int64_t)(pc & 1) * NB * NV;
        const unsigned tag = pc + 1;
        const int nk = (int)((it == 0 && want_r) ? 2 * K : K);
        const int ncol = nk + 2;
        const int G = max(1, min(NT / ncol, NB));
        bool ok = true;
        if (tid < G * ncol) {
          const int gi = tid / ncol, cc = tid - gi * ncol;
          const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
          double sum;
          if (rb_gather(in + v, NV, gi, G, NB, tag, tmo, sum)) s_part[tid] = sum;
          else ok = false;
        }
        if (!ok) s_ok = 0;
        __syncthreads();
        if (s_ok == 0) return;                       // timed out: every thread leaves
        for (int cc = tid; cc < ncol; cc += NT) {
          double sum = 0.0;
          for (int gi = 0; gi < G; ++gi) sum += s_part[gi * ncol + cc];
          if (cc < K) s_d2[cc] = sum;
          else if (cc < nk) s_r[cc - K] = sum;
          else s_wp[cc - nk] = sum;
        }
        ++pc;
        __syncthreads();
      }
      // (2) tol test of the pass that produced g_it (M:180-183)
      if (it >= 1) {
        const float mv = (float)sqrt(s_wp[0]);
        last_mv = (double)mv;
        if (mv <= a.tol) { conv = 1; break; }
      }
      if (it == a.maxiter) break;
      // (3) coefficients of pass `it`: one wave, lane = client (K <= 64)
      if (w == 0) {
        const int k = lane;
        const bool kv = k < K;
        const int kk = kv ? k : 0;                   // (s_d2 / s_r hold KR <= 64 entries)
        if constexpr (MODE == 0) {
          const double wk = kv ? 1.0 / (double)clamp_dist(s_d2[kk], a.eps) : 0.0;   // M:178
          const double Wsum = wave_sum(wk);
          if (kv) s_coef[k] = (float)(wk / Wsum);                                   // M:179
          if (lane == 0) s_anoise = 0.f;
        } else {
          const float s = sqrtf((float)(s_wp[1] / (double)d));      // M:146
          const float thr = (s * s) * 500.0f;                         // M:152
          double ck = 0.0;
          if (kv) {
            float n4[4];
            normal4(seed_p, kStreamChannel, (uint64_t)it, (uint64_t)k, n4);
            const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
            const float h2 = hr * hr + hi * hi;                       // M:403
            const float dist = clamp_dist(s_d2[kk], a.eps);
            const float pk = ((float)s_r[kk] + s * s) / (dist * dist * (float)(d + 1)) / h2;   // M:404
            const float pup = pk != pk ? pk : fmaxf(pk, thr);          // M:405
            ck = (double)(sqrtf((float)a.P_max / pup) / dist);         // M:407
          }
          const double Sc = wave_sum(ck);
          const double nd = !a.has_noise ? 0.0
                            : a.noise_sd * (double)normal1(seed_p, kStreamNoise, (uint64_t)it,
                                                           (uint64_t)d);
          const double scale = (double)s / ((double)s * Sc + nd);     // M:153-155
          if (kv) s_coef[k] = (float)(ck * scale);
          if (lane == 0) s_anoise = a.has_noise ? (float)(scale * a.noise_sd) : 0.f;
        }
      }
      __syncthreads();
      // (4) phase A: the thread's columns of g' = sum_k c_k x_k (+ the column noise).
      // Packed FMAs on the tile's own register pairs (x.xy, x.zw): left to itself the
      // compiler paired the FMAs across the wrong elements and copied the whole tile into
      // new pairs first (2 x KR more live registers).  v_pk_fma_f32 is one fused FMA per
      // element: the same bits as fmaf.
      f2 ga = {0.f, 0.f}, gb = {0.f, 0.f};
      sfor<0, KR / 4>([&](auto qq) {
        constexpr int k4 = 4 * qq;
        const f4 cw = *reinterpret_cast<const f4*>(&s_coef[k4]);
        sfor<0, 4>([&](auto u) {
          const f4 r = row(std::integral_constant<int, k4 + u>{});
          constexpr int uu = u;
          const f2 c2 = {cw[uu], cw[uu]};
          ga = __builtin_elementwise_fma(c2, f2{r[0], r[1]}, ga);
          gb = __builtin_elementwise_fma(c2, f2{r[2], r[3]}, gb);
        });
        // (the scheduler would issue every coefficient read first: KR more live registers)
        if constexpr ((k4 & 15) == 12) __builtin_amdgcn_sched_barrier(0);
      });
      float mvp = 0.f, gnp = 0.f;
      const float an = s_anoise;
      const float gnew4[4] = {ga[0], ga[1], gb[0], gb[1]};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float gv = gnew4[v];
        if (col0 + v < d) {
          if (MODE == 1 && a.has_noise)
            gv = fmaf(an, normal1(seed_p, kStreamNoise, (uint64_t)it, (uint64_t)(col0 + v)), gv);
          const float diff = g[v] - gv;
          mvp = fmaf(diff, diff, mvp);
          gnp = fmaf(gv, gv, gnp);
        } else {
          gv = 0.f;
        }
        g[v] = gv;
      }
      // (5) phase B: the distances to the new iterate
      __syncthreads();   // every wave's reads of s_rows / s_fin (publish of the last pass) done
      rb_all_rows<KR>(dist_row, &s_rows[w][0], lane);
      wave_fin(mvp, gnp);
      __syncthreads();
      publish(false);
    }

    // ---- the problem's aggregate and state
#pragma unroll
    for (int v = 0; v < 4; ++v)
      if (col0 + v < d) a.out[p * a.ldo + col0 + v] = g[v];
    if (bi == 0 && tid == 0) {
      a.st[p].iters = it;
      a.st[p].last_movement = last_mv;
      a.st[p].converged = conv;
      a.st[p].done = 1;
    }
  }
}

// ---------------------------------------------------------------------------

// (rows, rows in VGPRs): K <= 32 wholly in registers; K <= 52 with rows 36..51 in LDS
// (a 52-row register tile does not fit 256 VGPRs beside the kernel's own ~90)
static const void* rb_kernel(int kr, int mode) {
#define GMK_RB(KR_, KV_)                                                                       \
  if (kr == KR_)                                                                               \
    return mode == 0 ? reinterpret_cast<const void*>(&weiszfeld_resident_batched<KR_, KV_, 0>) \
                     : reinterpret_cast<const void*>(&weiszfeld_resident_batched<KR_, KV_, 1>);
  GMK_RB(16, 16) GMK_RB(32, 32) GMK_RB(52, 36)
#undef GMK_RB
  return nullptr;
}

int rb_rows_for(int64_t K) { return K <= 16 ? 16 : K <= 32 ? 32 : K <= 52 ? 52 : 0; }

bool rb_plan(int64_t K, int64_t d, int64_t P, int mode, int num_cu, RbPlan* plan) {
  const int kr = rb_rows_for(K);
  // the AirComp kernel (column draws in phase A, Philox channel draws in the K-space wave)
  // spills beyond 16 rows: K > 16 AirComp problems stream
  if (mode != 0 && kr > 16) return false;
  const void* fn = kr ? rb_kernel(kr, mode) : nullptr;
  if (!fn || d < 1 || P < 1) return false;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 512, 0) != hipSuccess || n < 1)
    return false;
  const int64_t cap = (int64_t)n * num_cu;
  const int64_t nb = (d + kRbCols - 1) / kRbCols;
  if (nb > cap) return false;
  plan->kr = kr;
  plan->mode = mode;
  plan->nb = (int)nb;
  plan->ng = (int)std::min<int64_t>(P, cap / nb);
  return true;
}

size_t rb_gran_words(int64_t K, const RbPlan& plan) {
  return (size_t)plan.ng * 2 * plan.nb * (size_t)(2 * K + 2);
}

hipError_t launch_resident_batched(const RbPlan& plan, const ResBArgs& a, bool coop, hipStream_t s) {
  const void* fn = rb_kernel(plan.kr, plan.mode);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<ResBArgs*>(&a)};
  const dim3 grid(plan.ng * plan.nb);
  if (coop) return hipLaunchCooperativeKernel(fn, grid, dim3(512), args, 0, s);
  return hipLaunchKernel(fn, grid, dim3(512), args, 0, s);
}

}  // namespace gmk
