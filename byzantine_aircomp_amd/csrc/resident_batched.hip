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
// GMK_RB_COEF_WAVE0=1: wave 0 alone forms the coefficients (one more block barrier)
// instead of every wave redundantly (A/B)
#ifndef GMK_RB_COEF_WAVE0
#define GMK_RB_COEF_WAVE0 0
#endif
// GMK_RB_PREFETCH_ROWS = n > 0: during iteration it of problem p, the rows
// [n·it, n·it + n) of the group's NEXT problem are read into a junk LDS line (LDS-DMA, no
// registers), so that the next tile load finds them in the Infinity Cache (A/B)
#ifndef GMK_RB_PREFETCH_ROWS
#define GMK_RB_PREFETCH_ROWS 0
#endif
#ifndef GMK_RB_FASTCOEF
#define GMK_RB_FASTCOEF 0   // A/B knob: the AirComp coefficients as resident.hip's (needs EARLY_H2)
#endif
// GMK_RB_EARLY_H2=1: the AirComp channel gains |h_k|^2 drawn in draw_pass, after the
// previous publish, instead of inside the coefficient step on the iteration's dependent
// chain: with the four-column noise blocks (philox.h normal1) C5 AirComp 803.6 -> 816.7
// problems/s (profiles/r4s2_c5air_draws_ab.jsonl); 0 = in the coefficient step (A/B)
#ifndef GMK_RB_EARLY_H2
#define GMK_RB_EARLY_H2 1
#endif
#ifndef GMK_RB_OMA_ROWS
#define GMK_RB_OMA_ROWS 2
#endif

constexpr uint64_t kRbPollTicks = 200000000ull;  // 2 s at the 100 MHz real-time clock
// the poll's back-off between rounds, in units of 64 cycles (A/B knob)
#ifndef GMK_RB_SLEEP
#define GMK_RB_SLEEP 1
#endif
constexpr int kRbChunk = 8;                      // granules in flight per poll round

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// `local`: every block of the group on one XCD (checked at check-in): the granule stays in
// that XCD's L2 (workgroup-scope store, `sc0`) for the group's `sc1` polls (resident.hip
// put_value)
__device__ __forceinline__ void rb_put(gu64* g, unsigned tag, float v, bool local) {
  const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
  if (local) __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
#ifndef GMK_RB_NOSLEEP
      __builtin_amdgcn_s_sleep(GMK_RB_SLEEP);
#endif
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

// The hierarchical gather's second level (a.hier): value v of the ns sub-group sums, each
// an fp32 {hi, lo} granule pair, polled 4 pairs per round trip (the 8 granules of rb_gather's
// round trip: no more registers beside the tile) and summed in sub-group order.
__device__ __forceinline__ bool rb_gather_pairs(const gu64* g, int64_t gstride, int ns,
                                                unsigned tag, gu32* tmo, double& sum) {
  sum = 0.0;
  for (int j0 = 0; j0 < ns; j0 += 4) {
    unsigned long long v[8];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j0 + j < ns) {
          const gu64* q = g + (int64_t)(j0 + j) * gstride;
          v[2 * j] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[2 * j + 1] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(v[2 * j] >> 32) == tag && (unsigned)(v[2 * j + 1] >> 32) == tag;
        }
      }
      if (ok) break;
#ifndef GMK_RB_NOSLEEP
      __builtin_amdgcn_s_sleep(GMK_RB_SLEEP);
#endif
      if (((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t0 > kRbPollTicks) ||
          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j0 + j < ns)
        sum += (double)__uint_as_float((unsigned)(v[2 * j] & 0xffffffffull)) +
               (double)__uint_as_float((unsigned)(v[2 * j + 1] & 0xffffffffull));
  }
  return true;
}

// Rows [K0, K0 + R) of a per-thread row quantity (f(k) over the thread's 4 columns),
// transpose-reduced over the wave: lane c ends with row K0 + row_of_lane<64, R>(c);
// the lanes c % (64 / R) == 0 hold distinct rows and store them to srow.
template <int R, int K0, int KR, int KV, class F>
__device__ __forceinline__ void rb_rows(F f, float* srow, int lane) {
  float e[R];
  sfor<0, R>([&](auto i) {
    e[i] = f(std::integral_constant<int, K0 + i>{});
    // rows held in LDS (k >= KV) are read four at a time: the scheduler would issue every
    // row's ds_read_b128 first, four live registers per row beside the tile
    if constexpr (K0 + i >= KV && (i & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  });
  xlane_transpose64<R>(e, lane);
  if ((lane % (64 / R)) == 0) srow[K0 + row_of_lane<64, R>(lane)] = e[0];
  // one row block at a time: interleaving the blocks (the scheduler's choice) holds every
  // block's e[] at once, KR more live registers beside the tile
  __builtin_amdgcn_sched_barrier(0);
}

// All KR rows: blocks of 16, then a tail of 8, 4 and / or 2 (KR even).
template <int KR, int KV, int K0 = 0, class F>
__device__ __forceinline__ void rb_all_rows(F f, float* srow, int lane) {
  if constexpr (KR - K0 >= 16) {
    rb_rows<16, K0, KR, KV>(f, srow, lane);
    rb_all_rows<KR, KV, K0 + 16>(f, srow, lane);
  } else if constexpr (KR - K0 >= 8) {
    rb_rows<8, K0, KR, KV>(f, srow, lane);
    rb_all_rows<KR, KV, K0 + 8>(f, srow, lane);
  } else if constexpr (KR - K0 >= 4) {
    rb_rows<4, K0, KR, KV>(f, srow, lane);
    rb_all_rows<KR, KV, K0 + 4>(f, srow, lane);
  } else if constexpr (KR - K0 >= 2) {
    rb_rows<2, K0, KR, KV>(f, srow, lane);
  }
}

}  // namespace

// DBG (probe builds, -DGMK_RB_DBG_VARIANTS; 0 in the product): phases skipped to price
// them (tools/rb_probe.py --dbg; 7 = the exchange alone, the latency roofline's floor):
// 1 phase B rows, 2 the K-space step, 4 phase A, 8 the
// gather's wait for the tags, 16 the publish, 32 the tile load, 64 the INIT rows, 128 the
// LDS rows' loads, 256 the register rows' loads
template <int KR, int KV, int MODE, int DBG = 0, int XG = 0>
__global__ void __launch_bounds__(512) weiszfeld_resident_batched(ResBArgs a) {
  // KR rows per column (K rounded up to 4): rows [0, KV) live in the thread's VGPRs, rows
  // [KV, KR) in LDS (s_x, the thread's own 16 bytes per row).  MODE: gm_mode, a template
  // parameter so that the gm2 kernel carries none of the AirComp code's registers.
  static_assert(KR % 2 == 0 && KV % 4 == 0 && KV <= KR && KR <= 64, "rows per thread");
  constexpr int NT = 512;
  constexpr int NW = NT / 64;
  constexpr int KL = KR - KV;                      // rows held in LDS
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  __shared__ f4 s_x[KL > 0 ? KL : 1][NT];
  __shared__ f4 s_junk[GMK_RB_PREFETCH_ROWS > 0 ? 64 : 1];   // prefetch landing line
  // each wave's own copy of the coefficients, rows padded to 16 bytes (phase A reads them
  // as float4)
  constexpr int KC = (KR + 2 + 3) / 4 * 4;
  __shared__ __attribute__((aligned(16))) float s_coef[NW][KC];
  __shared__ float s_osc[KR];
  // row partials and the waves' movement / norm partials, by the parity of the pass they
  // belong to: a publish reads buffer p & 1 while the next pass's phase B fills the other
  __shared__ float s_rows[2][NW][KR];
  __shared__ float s_rows2[NW][KR];
  __shared__ float s_fin[2][2][NW];
  __shared__ double s_part[NT];
  __shared__ float s_rk[MODE == 1 ? NW : 1][64];   // gm: lane k's ||x_k||^2, each wave's copy
  __shared__ float s_an;
  __shared__ int s_ok, s_same;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NB = a.nb;
  int lb = (int)blockIdx.x;                        // logical block
  if (a.xcd_major) {
    // XCD x = b % 8 holds blocks x, x + 8, ...: number them XCD by XCD
    const int n = (int)gridDim.x, x = lb & 7;
    int before = 0;
    for (int y = 0; y < x; ++y) before += (n - y + 7) >> 3;
    lb = before + (lb >> 3);
  }
  const int grp = lb / NB, bi = lb - grp * NB;
  const int NG = (int)gridDim.x / NB;
  // XCD-hierarchical gather (a.hier, XCD-major numbering): a group's blocks split into
  // sub-groups by XCD (the group's logical range cut at the XCD ranges: logical blocks
  // [xlo(x), xlo(x) + n(x)) sit on XCD x); each sub-group's first block (its leader) sums
  // its members, publishes the sum as an fp32 {hi, lo} pair, and every block sums the
  // sub-group sums in XCD order.  Without it: one sub-group, the whole group.
  // XG (a template parameter: the flat kernels carry none of its registers): 0 flat, 1 the
  // sub-group leaders above.  (A split-scope variant — every granule published agent-scope
  // and L2-kept, each reader polling its own XCD's blocks from the L2-kept copy: one hop —
  // measured slower still, C5 AirComp 815 -> 736 problems/s; profiles/r5s1_c5_rb_split_ab.jsonl)
  const bool hier = XG == 1 && a.xcd_major;
  auto xcd_lo = [&](int x) {             // first logical block of XCD x (x in 0..8)
    int b = 0;
    for (int y = 0; y < x; ++y) b += ((int)gridDim.x - y + 7) >> 3;
    return b;
  };
  int sub_lo = grp * NB, sub_hi = grp * NB + NB, x_first = 0, n_sub = 1, s_idx = 0;
  if (hier) {
    const int x = (int)(blockIdx.x & 7);
    while (x_first < 7 && xcd_lo(x_first + 1) <= grp * NB) ++x_first;
    int x_last = x_first;
    while (x_last < 7 && xcd_lo(x_last + 1) < grp * NB + NB) ++x_last;
    n_sub = x_last - x_first + 1;
    s_idx = x - x_first;
    sub_lo = max(grp * NB, xcd_lo(x));
    sub_hi = min(grp * NB + NB, xcd_lo(x + 1));
  }
  const bool leader = hier && lb == sub_lo;
  const int64_t K = a.K, d = a.d;
  const int64_t NV = 2 * K + 2;                    // granule slots per block and pass
  gu64* gran = (gu64*)a.gran + (int64_t)grp * 2 * NB * NV;
  gu64* lvl2 = (gu64*)a.lvl2 + (int64_t)grp * 2 * 8 * 2 * NV;   // [2][8 sub-groups][2 NV]
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
  if (tid < NW * KC) (&s_coef[0][0])[tid] = 0.f;
  // every block of the grid co-resident before any problem's X is read or (pre-noise)
  // written: a grid that is not fails here with X untouched (device_util.h)
  // (slot = logical block: a group's slots are contiguous, so the check-in also tells
  // whether the whole group shares one XCD)
  if (!grid_checkin(a.checkin, (unsigned)lb, a.need, a.flag, a.flag + 2, kCheckinTicks, &s_ok,
                    &s_same, (unsigned)sub_lo, (unsigned)sub_hi))
    return;
  // identical in the (sub-)group's blocks; hier: the member -> leader granules only
  const bool local = a.local && s_same;
  if (local && lb == sub_lo && tid == 0)           // (sub-)groups on one XCD, for the host
    __hip_atomic_fetch_add((gu32*)a.flag + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

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
    auto put = [&](int64_t slot, float v) { rb_put(out + slot, tag, v, local); };
    const int pb = pc & 1;
    if (tid < K) {
      double sm = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sm += (double)s_rows[pb][ww][tid];
      put(tid, (float)sm);
    }
    if (with_r && tid >= 64 && tid < 64 + K) {
      const int k = tid - 64;
      double sm = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sm += (double)s_rows2[ww][k];
      put(K + k, (float)sm);
    }
    if (tid == 128) {
      double m = 0.0, gg = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        m += (double)s_fin[pb][0][ww];
        gg += (double)s_fin[pb][1][ww];
      }
      put(2 * K, (float)m);
      put(2 * K + 1, (float)gg);
    }
  };
  auto wave_fin = [&](float mv, float gn) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mv += __shfl_xor(mv, o, 64);
      gn += __shfl_xor(gn, o, 64);
    }
    if (lane == 0) {
      s_fin[pc & 1][0][w] = mv;
      s_fin[pc & 1][1][w] = gn;
    }
  };
  // the per-row squared distance over the thread's columns, on packed pairs (columns
  // 0/1 and 2/3: v_pk_add + v_pk_mul + v_pk_fma, then one add: 5 instructions per row
  // instead of 8); the order (t0^2 + t2^2) + (t1^2 + t3^2)
  auto dist_row = [&](auto k) {
    const f4 r = row(k);
    const f2 t01 = f2{r[0], r[1]} - f2{g[0], g[1]};
    const f2 t23 = f2{r[2], r[3]} - f2{g[2], g[3]};
    const f2 s2 = __builtin_elementwise_fma(t23, t23, t01 * t01);
    return s2[0] + s2[1];
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
    // Every load issued before any is waited for: the LDS rows straight into LDS
    // (buffer_load ... lds: LDS-DMA, no registers), the register rows into the tile, then
    // ONE wait.  Columns >= d of a partial last group are zeroed afterwards (selects on the
    // register rows; the partial thread rewrites its LDS slots).  A branch per row splits
    // the loads into basic blocks, each ended by vmcnt(0) — the 50 loads of a problem then
    // run one HBM round trip at a time; staging the LDS rows through registers spills.
    if constexpr ((DBG & 32) == 0) {
    if constexpr ((DBG & 128) == 0) sfor<KV, KR>([&](auto k) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc(k), (__attribute__((address_space(3))) void*)&s_x[k - KV][w * 64], 16, voff,
          roff(k), 0, 2);
    });
    if constexpr ((DBG & 256) == 0) sfor<0, KV>([&](auto k) {
      x[k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(k), voff, roff(k), 2));
    });
    } else if (p == grp) {
      sfor<0, KV>([&](auto k) { x[k] = f4{0.f, 0.f, 0.f, 0.f}; });
    }
    // the guess at the thread's columns, in flight with the tile (one buffer resource:
    // columns past d read 0)
    {
      const uint64_t gb = reinterpret_cast<uint64_t>(a.guess0 + p * a.ldg);
      float* const Gu = reinterpret_cast<float*>(
          ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(gb >> 32)) << 32) |
          (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)gb));
      const __amdgpu_buffer_rsrc_t rg =
          __builtin_amdgcn_make_buffer_rsrc(Gu, 0, (int)(d * 4), 0x00020000);
#pragma unroll
      for (int v = 0; v < 4; ++v)
        g[v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rg, any ? (uint32_t)((col0 + v) * 4) : 0x80000000u,
                                             0, 0));
    }
    __builtin_amdgcn_s_waitcnt(0);                   // every load of the tile landed
    {
      bool cok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) cok[u] = col0 + u < d;
      sfor<0, KV>([&](auto k) {
#pragma unroll
        for (int u = 0; u < 4; ++u) x[k][u] = cok[u] ? x[k][u] : 0.f;
      });
      if (!full) {
        sfor<KV, KR>([&](auto k) {
          f4 v = s_x[k - KV][tid];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = cok[u] ? v[u] : 0.f;
          s_x[k - KV][tid] = v;
        });
      }
    }
    // ---- OMA pre-noise (M:385-394), the draws of gm_oma_philox_f32 / the fused pass:
    // element (k, j) takes normal j & 3 of the Philox block (row k, j >> 2), scaled by the
    // row's sd / |h_k|; written back in place (the reference's OMA mutates wList).  Rows
    // past K: scale 0 (they stay 0) and a zero-record resource (their stores are dropped).
    // (gm2 only: the AirComp kernel carries no OMA code)
    if (MODE == 0 && a.pre_oma) {
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
        // GMK_RB_OMA_ROWS rows' draws at a time: one Philox chain per row is latency-bound,
        // every chain at once spills (hoisting the partial-group test out of the row loop
        // duplicates the loop and spilled 55-90 VGPRs)
        if constexpr ((k + 1) % GMK_RB_OMA_ROWS == 0) __builtin_amdgcn_sched_barrier(0);
      });
    }

    // ---- INIT (pass pc): D_k to g_0, ||x_k||^2 (gm), ||g_0||^2
    constexpr bool want_r = MODE == 1;
    __syncthreads();   // s_rows2 / s_osc of the previous problem consumed
    if constexpr ((DBG & 64) == 0) rb_all_rows<KR, KV>(dist_row, &s_rows[pc & 1][w][0], lane);
    if constexpr (want_r) {
      // (a memory clobber: without it the LDS rows' reads of the pass above are kept live
      // for this one — 18 float4 beside the tile)
      asm volatile("" ::: "memory");
      rb_all_rows<KR, KV>([&](auto k) {
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

    // AirComp: pass `it`'s draws depend on (problem, it, column / client) only, so each
    // pass's are drawn right after the previous publish, while the other blocks' partials
    // are in flight (off the gather -> phase A -> phase B chain): the column noise (M:411,
    // the thread's four columns: one Philox block), lane k's channel gain |h_k|^2 (M:403)
    // and the scalar noise of M:153-155
    float nz[4] = {0.f, 0.f, 0.f, 0.f};
    float h2k = 1.f, ndr = 0.f;
    auto draw_pass = [&](int64_t i) {
      if constexpr (MODE == 1) {
        if (GMK_RB_EARLY_H2 && lane < K) {
          float n4[4];
          normal4(seed_p, kStreamChannel, (uint64_t)i, (uint64_t)lane, n4);
          const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
          h2k = hr * hr + hi * hi;
        }
        if (a.has_noise) {
          // the thread's 4 columns (col0 % 4 == 0) are one Philox block (philox.h normal1)
          ndr = normal1(seed_p, kStreamNoise, (uint64_t)i, (uint64_t)d);
          normal4_hw(seed_p, kStreamNoise, (uint64_t)i, (uint64_t)col0 >> 2, nz);
        }
      }
    };
    draw_pass(0);

    int64_t it = 0;
    float last_mv = NAN;
    int conv = 0;
    for (;; ++it) {
      // (1) gather pass pc: D (+ r at INIT of gm), movement, ||g||^2; G thread groups
      // each sum every G-th block (one round trip), then every wave adds the G group sums
      // in group order for the values it needs (no second pass through LDS, no barrier)
      const int nk = (int)((it == 0 && want_r) ? 2 * K : K);
      const int ncol = nk + 2;
      const int nmem = sub_hi - sub_lo;                // blocks this (sub-)group gathers
      int G = max(1, min(NT / ncol, nmem));
      if (hier) {
        // level 1 (the sub-group's leader) and level 2 (every block): the values land in
        // s_part[0, ncol) as one "group" for the waves' sums below
        const gu64* in = gran + (int64_t)(pc & 1) * NB * NV + (int64_t)(sub_lo - grp * NB) * NV;
        const unsigned tag = pc + 1;
        bool ok = true;
        if (leader) {
          if (tid < G * ncol) {
            const int gi = tid / ncol, cc = tid - gi * ncol;
            const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
            double sum;
            if (rb_gather(in + v, NV, gi, G, nmem, tag, tmo, sum)) s_part[tid] = sum;
            else ok = false;
          }
          if (!ok) s_ok = 0;
          __syncthreads();
          if (s_ok == 0) return;
          gu64* l2o = lvl2 + ((int64_t)(pc & 1) * 8 + s_idx) * 2 * NV;
          double sum = 0.0;
          int64_t v = 0;
          if (tid < ncol) {
            for (int gi = 0; gi < G; ++gi) sum += s_part[gi * ncol + tid];
            v = tid < nk ? tid : 2 * K + (tid - nk);
          }
          __syncthreads();                             // (s_part is refilled below)
          if (tid < ncol) {
            const float hi = (float)sum;
            rb_put(l2o + 2 * v, tag, hi, false);
            rb_put(l2o + 2 * v + 1, tag, (float)(sum - (double)hi), false);
          }
        }
        if (tid < ncol) {
          const int64_t v = tid < nk ? tid : 2 * K + (tid - nk);
          double sum;
          if (rb_gather_pairs(lvl2 + (int64_t)(pc & 1) * 8 * 2 * NV + 2 * v, 2 * NV, n_sub, tag,
                              tmo, sum))
            s_part[tid] = sum;
          else
            ok = false;
        }
        if (!ok) s_ok = 0;
        __syncthreads();
        if (s_ok == 0) return;
        G = 1;
        ++pc;
      } else {
        const gu64* in = gran + (int64_t)(pc & 1) * NB * NV;
        const unsigned tag = pc + 1;
        bool ok = true;
        if (tid < G * ncol) {
          const int gi = tid / ncol, cc = tid - gi * ncol;
          const int64_t v = cc < nk ? cc : 2 * K + (cc - nk);
          double sum;
          if constexpr ((DBG & 8) != 0) {
            sum = 0.0;
            for (int bb = gi; bb < NB; bb += G)
              sum += (double)__uint_as_float((unsigned)(__hip_atomic_load(
                  in + v + (int64_t)bb * NV, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                  0xffffffffull));
            s_part[tid] = sum;
          } else if (rb_gather(in + v, NV, gi, G, NB, tag, tmo, sum)) {
            s_part[tid] = sum;
          } else {
            ok = false;
          }
        }
        if (!ok) s_ok = 0;
        __syncthreads();
        if (s_ok == 0) return;                       // timed out: every thread leaves
        ++pc;
      }
      if constexpr (GMK_RB_PREFETCH_ROWS > 0) {
        // the next problem's rows n·it .. n·it + n - 1 into the Infinity Cache (their LDS-DMA
        // lands in a junk line; the phases below cover the loads' latency before the next
        // barrier drains them)
        const int64_t pn = p + NG;
        if (pn < a.P && it * GMK_RB_PREFETCH_ROWS < K) {
          const uint64_t nb64 = reinterpret_cast<uint64_t>(a.X + pn * a.x_ps);
          float* const Xn = reinterpret_cast<float*>(
              ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(nb64 >> 32)) << 32) |
              (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)nb64));
          const int nrec = __builtin_amdgcn_readfirstlane(a.prob_bytes);
          const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(Xn, 0, nrec, 0x00020000);
          sfor<0, GMK_RB_PREFETCH_ROWS>([&](auto j) {
            const int64_t kk = it * GMK_RB_PREFETCH_ROWS + j;
            if (kk < K)
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  rn, (__attribute__((address_space(3))) void*)&s_junk[0], 16, voff,
                  __builtin_amdgcn_readfirstlane((int)(kk * rstride * 4)), 0, 0);
          });
        }
      }
      // every wave: the movement / ||g||^2 sums (uniform) and, lane = client, D_k (and r_k
      // at INIT of gm), each a fixed-order sum of the G group sums
      const int k = lane;
      const bool kv = k < K;
      double mv2 = 0.0, gn2 = 0.0, d2k = 0.0;
      for (int gi = 0; gi < G; ++gi) {
        mv2 += s_part[gi * ncol + nk];
        gn2 += s_part[gi * ncol + nk + 1];
        if (kv) d2k += s_part[gi * ncol + k];
      }
      if (want_r && it == 0 && kv) {
        // (kept in the wave's LDS copy, not a register: the AirComp tile is at the VGPR limit)
        double r_k = 0.0;
        for (int gi = 0; gi < G; ++gi) r_k += s_part[gi * ncol + K + k];
        s_rk[w][k] = (float)r_k;
      }
      // (2) tol test of the pass that produced g_it (M:180-183)
      if (it >= 1) {
        const float mv = (float)sqrt(mv2);
        last_mv = mv;
        if (mv <= a.tol) { conv = 1; break; }
      }
      if (it == a.maxiter) break;
      // (3) coefficients of pass `it`, in every wave (lane = client, K <= 64) into the
      // wave's own LDS copy: the waves need no barrier before phase A
      float an = 0.f;
      constexpr int CW = GMK_RB_COEF_WAVE0 ? 0 : -1;   // the coefficient copy phase A reads
      if ((DBG & 2) == 0 && (!GMK_RB_COEF_WAVE0 || w == 0)) {
        if constexpr (MODE == 0) {
          const double wk = kv ? 1.0 / (double)clamp_dist(d2k, a.eps) : 0.0;   // M:178
          const double Wsum = xlane_wave_sum(wk);
          if (k < KR) s_coef[w][k] = kv ? (float)(wk / Wsum) : 0.f;           // M:179
        } else if (GMK_RB_FASTCOEF) {
          // (resident.hip's fast coefficients: v_rcp / v_rsq, fp32 square roots and sums)
          const float s = sqrtf((float)(gn2 * (1.0 / (double)d)));  // M:146
          const float thr = (s * s) * 500.0f;                         // M:152
          float ck = 0.f;
          if (kv) {
            const float d0 = sqrtf((float)d2k);
            const float dist = d0 != d0 ? d0 : fmaxf(d0, a.eps);
            const float pk = (s_rk[w][k] + s * s) *
                             __builtin_amdgcn_rcpf(dist * dist * (float)(d + 1) * h2k);   // M:404
            const float pup = pk != pk ? pk : fmaxf(pk, thr);          // M:405
            ck = sqrtf((float)a.P_max) * __builtin_amdgcn_rsqf(pup) *
                 __builtin_amdgcn_rcpf(dist);                          // M:407
          }
          const float Sc = xlane_wave_sum_f32(ck);
          const float nd = !a.has_noise ? 0.f : (float)a.noise_sd * ndr;
          const float scale = s * __builtin_amdgcn_rcpf(s * Sc + nd);   // M:153-155
          if (k < KR) s_coef[w][k] = kv ? ck * scale : 0.f;
          an = a.has_noise ? scale * (float)a.noise_sd : 0.f;
        } else {
          const float s = sqrtf((float)(gn2 / (double)d));          // M:146
          const float thr = (s * s) * 500.0f;                         // M:152
          double ck = 0.0;
          if (kv) {
            float h2 = h2k;                                           // M:403 (draw_pass)
            if constexpr (!GMK_RB_EARLY_H2) {
              float n4[4];
              normal4(seed_p, kStreamChannel, (uint64_t)it, (uint64_t)k, n4);
              const float hr = n4[0] * 0.70710678118654752f, hi = n4[1] * 0.70710678118654752f;
              h2 = hr * hr + hi * hi;
            }
            const float dist = clamp_dist(d2k, a.eps);
            const float pk = (s_rk[w][k] + s * s) / (dist * dist * (float)(d + 1)) / h2;   // M:404
            const float pup = pk != pk ? pk : fmaxf(pk, thr);          // M:405
            ck = (double)(sqrtf((float)a.P_max / pup) / dist);         // M:407
          }
          const double Sc = xlane_wave_sum(ck);
          const double nd = !a.has_noise ? 0.0 : a.noise_sd * (double)ndr;
          const double scale = (double)s / ((double)s * Sc + nd);     // M:153-155
          if (k < KR) s_coef[w][k] = kv ? (float)(ck * scale) : 0.f;
          an = a.has_noise ? (float)(scale * a.noise_sd) : 0.f;
        }
        if (GMK_RB_COEF_WAVE0 && lane == 0) s_an = an;
      }
      if constexpr (GMK_RB_COEF_WAVE0) {
        __syncthreads();
        an = s_an;
      }
      const int cw_row = CW < 0 ? w : CW;
      // (4) phase A: the thread's columns of g' = sum_k c_k x_k (+ the column noise).
      // Packed FMAs on the tile's own register pairs (x.xy, x.zw): left to itself the
      // compiler paired the FMAs across the wrong elements and copied the whole tile into
      // new pairs first (2 x KR more live registers).  v_pk_fma_f32 is one fused FMA per
      // element: the same bits as fmaf.
      f2 ga = {0.f, 0.f}, gb = {0.f, 0.f};
      if constexpr ((DBG & 4) == 0) {
        sfor<0, KR / 4>([&](auto qq) {
          constexpr int k4 = 4 * qq;
          const f4 cw = *reinterpret_cast<const f4*>(&s_coef[cw_row][k4]);
          sfor<0, 4>([&](auto u) {
            const f4 r = row(std::integral_constant<int, k4 + u>{});
            constexpr int uu = u;
            const f2 c2 = {cw[uu], cw[uu]};
            ga = __builtin_elementwise_fma(c2, f2{r[0], r[1]}, ga);
            gb = __builtin_elementwise_fma(c2, f2{r[2], r[3]}, gb);
          });
          // (the scheduler would issue every coefficient / LDS-row read first: KR more live
          // registers; the LDS rows a quad at a time)
          if constexpr ((k4 & 15) == 12 || k4 + 4 > KV) __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (KR % 4 == 2) {       // the last two rows (KR = 50)
          constexpr int k2 = KR - 2;
          const f2 cw = *reinterpret_cast<const f2*>(&s_coef[cw_row][k2]);
          sfor<0, 2>([&](auto u) {
            const f4 r = row(std::integral_constant<int, k2 + u>{});
            constexpr int uu = u;
            const f2 c2 = {cw[uu], cw[uu]};
            ga = __builtin_elementwise_fma(c2, f2{r[0], r[1]}, ga);
            gb = __builtin_elementwise_fma(c2, f2{r[2], r[3]}, gb);
          });
        }
      }
      float mvp = 0.f, gnp = 0.f;
      const float gnew4[4] = {ga[0], ga[1], gb[0], gb[1]};
      // (AirComp: the column noise nz of pass `it` was drawn after the last publish)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float gv = gnew4[v];
        if (col0 + v < d) {
          if (MODE == 1 && a.has_noise) gv = fmaf(an, nz[v], gv);
          const float diff = g[v] - gv;
          mvp = fmaf(diff, diff, mvp);
          gnp = fmaf(gv, gv, gnp);
        } else {
          gv = 0.f;
        }
        g[v] = gv;
      }
      // (5) phase B: the distances to the new iterate, into the buffer of pass pc (the
      // publish of pass pc - 1 reads the other one)
      if constexpr ((DBG & 1) == 0) rb_all_rows<KR, KV>(dist_row, &s_rows[pc & 1][w][0], lane);
      wave_fin(mvp, gnp);
      __syncthreads();
      if constexpr ((DBG & 16) == 0) publish(false);
      if (it < a.maxiter) draw_pass(it + 1);
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
static const void* rb_kernel(int kr, int mode, int xg = 0) {
#ifdef GMK_RB_DBG_VARIANTS
  static const int dbg = getenv("GMAGG_RB_DBG") ? atoi(getenv("GMAGG_RB_DBG")) : 0;
  if (kr == 50 && mode == 0) {
    switch (dbg) {
      case 1: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 1>);
      case 2: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 2>);
      case 4: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 4>);
      case 7: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 7>);
      case 8: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 8>);
      case 16: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 16>);
      case 31: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 31>);
      case 32: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 32>);
      case 64: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 64>);
      case 128: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 128>);
      case 256: return reinterpret_cast<const void*>(&weiszfeld_resident_batched<50, 32, 0, 256>);
      default: break;
    }
  }
#endif
#define GMK_RB_XG(KR_, KV_, M_)                                                                \
  (xg == 1 ? reinterpret_cast<const void*>(&weiszfeld_resident_batched<KR_, KV_, M_, 0, 1>)    \
           : reinterpret_cast<const void*>(&weiszfeld_resident_batched<KR_, KV_, M_>))
#define GMK_RB(KR_, KV_, AIRCOMP_)                                                             \
  if (kr == KR_) {                                                                             \
    if (mode == 0) return GMK_RB_XG(KR_, KV_, 0);                                              \
    if constexpr (AIRCOMP_) return GMK_RB_XG(KR_, KV_, 1);                                     \
    return nullptr;                                                                            \
  }
  // (K <= 50 keeps 32 rows in VGPRs and 18 in LDS (144 KB); K = 51, 52 36 + 16, with a few
  // VGPRs spilled.  The AirComp kernel: K <= 50; at 33..50 rows it spills ~90 VGPRs of
  // loop invariants, ~44 scratch reloads per iteration)
  GMK_RB(16, 16, true) GMK_RB(32, 32, true) GMK_RB(50, 32, true) GMK_RB(52, 36, false)
#undef GMK_RB
#undef GMK_RB_XG
  return nullptr;
}

int rb_rows_for(int64_t K) { return K <= 16 ? 16 : K <= 32 ? 32 : K <= 50 ? 50 : K <= 52 ? 52 : 0; }

bool rb_plan(int64_t K, int64_t d, int64_t P, int mode, int num_cu, RbPlan* plan, bool xcd_whole) {
  int kr = rb_rows_for(K);
  // GMAGG_RB_ROWS=52: the 36 + 16-row tile for K <= 50 too (A/B of the row split)
  static const int force = getenv("GMAGG_RB_ROWS") ? atoi(getenv("GMAGG_RB_ROWS")) : 0;
  if (force == 52 && kr == 50) kr = 52;
  // the AirComp kernel (column draws in phase A, Philox channel draws in the coefficient
  // step) is built for K <= 50 (the 52-row tile spills): K = 51, 52 AirComp problems stream
  if (mode != 0 && kr > 50) return false;
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
  if (xcd_whole && cap / 8 / nb >= 1) plan->ng = (int)std::min<int64_t>(P, 8 * (cap / 8 / nb));
  return true;
}

size_t rb_gran_words(int64_t K, const RbPlan& plan) {
  // [NG][2][NB][2K + 2] granules, then the hierarchical gather's sub-group sums
  // [NG][2][8][2 (2K + 2)]
  return (size_t)plan.ng * 2 * plan.nb * (size_t)(2 * K + 2) +
         (size_t)plan.ng * 32 * (size_t)(2 * K + 2);
}

hipError_t launch_resident_batched(const RbPlan& plan, const ResBArgs& a, bool coop, hipStream_t s) {
  const void* fn = rb_kernel(plan.kr, plan.mode, a.hier);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<ResBArgs*>(&a)};
  const dim3 grid(plan.ng * plan.nb);
  if (coop) return hipLaunchCooperativeKernel(fn, grid, dim3(512), args, 0, s);
  return hipLaunchKernel(fn, grid, dim3(512), args, 0, s);
}

}  // namespace gmk
