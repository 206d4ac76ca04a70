// The fused streaming Weiszfeld pass for gfx950: ONE HBM read of X per
// iteration.
//
// Reference (MNIST_Air_weight.py): gm2's loop body M:174-181 computes
//   dist = max(1e-4, ||x_k - g||)          (a K x d read)
//   g'   = sum_k x_k/dist_k / sum 1/dist_k (another K x d read)
//   movement = ||g - g'||
// and the next body starts by re-reading X for the distances to g'.  Here a
// block owns a chunk of J columns x ALL K rows (in VGPRs) at a time:
//   phase A  g'_j = sum_k c_k x_kj          (c_k from the K-space step: 1/dist_k
//                                            normalised, or the AirComp gains)
//   phase B  D_k += sum_{j in chunk} (x_kj - g'_j)^2  -- the NEXT iteration's
//            distances, while the tile is still in registers
// plus ||g - g'||^2 and ||g'||^2.  INIT passes compute D_k to the initial
// guess (and ||x_k||^2 for the AirComp power control).
//
// Thread map (1024 threads = 16 waves): lane c of a row segment covers columns
// [c*V, c*V+V) of the chunk, QW = 64/LPR row groups per wave, NRG = 16*QW row
// groups per block, row group rg owns rows rg + NRG*i (i < R).  Every wave
// instruction reads LPR*V*4 contiguous bytes of QW rows: 1 KiB per
// instruction for V = 4.  Per-block partials go to a slab (fp64), summed by
// slab_reduce in a fixed order: deterministic, no atomics.
#include "device_util.h"
#include "gmagg_internal.h"
#include "philox.h"

namespace gmk {

template <int V, int R>
struct Tile {
  float x[R][V];
  float gold;    // finisher thread: g_t at its column (INIT: the guess)
  float hn;      // STEP finisher thread, host noise: its column's draw
};

// MODE: 0 step, 1 init, 2 init + ||x_k||^2, 3 Gram closing sum, 4 init after the OMA
// pre-noise (the tile gets the reference's per-client AWGN, M:385-394, in registers and is
// written back: one read + one write of X instead of OMA's read + write and INIT's read).  SCHED 0: load a
// chunk, then reduce it; 1 (PIPE): chunk c+1's loads are in flight while chunk
// c is reduced (two tiles of registers); 2 (ROLL): row i of chunk c+1 is loaded
// into the registers phase B has just freed (one tile).
// OCC: blocks per CU the register budget is capped for (2 -> <= 64 VGPRs at
// 16 waves); with OCC > 1 the row weights are read from LDS instead of VGPRs.
// PANEL: X is the panel layout [nch][K][J] (a.panel_stride elements between
// panels, rows J apart): a chunk is one contiguous block, every row offset in
// it fits the 32-bit lane offset, and the HBM stream is sequential.
template <int V, int NW, int LPR, int R, int MODE, int SCHED, int OCC = 1, bool PANEL = false>
__global__ void __launch_bounds__(NW * 64, OCC * NW / 4) weiszfeld_pass(PassArgs a) {
  constexpr bool PIPE = SCHED == 1, ROLL = SCHED == 2 || SCHED == 3, ROLL2 = SCHED == 3;
  constexpr bool SUM_ONLY = MODE == 3;     // closing pass of the Gram variant: g = sum c_k x_k
  constexpr bool OMA_INIT = MODE == 4;
  constexpr bool INIT = MODE == 1 || MODE == 2 || OMA_INIT;
  constexpr bool WANT_R = MODE == 2;
  static_assert(!OMA_INIT || V == 4, "fused OMA: one Philox block per float4 group");
  constexpr int QW = 64 / LPR;
  constexpr int NRG = NW * QW;
  constexpr int J = LPR * V;
  constexpr int RPL = R > LPR ? R / LPR : 1;
  static_assert(J <= NW * 64, "one finisher thread per column");
  using T = Tile<V, R>;

  __shared__ float s_red[NW][J];
  __shared__ float s_g[INIT ? 2 : 1][J];   // INIT: by chunk parity (one barrier per chunk)
  __shared__ double s_fin[2][NW];
  __shared__ float s_w[OCC > 1 ? NW * QW * R : 1];

  if (gridDim.y > 1) {                       // batched independent problems
    const int64_t pb = blockIdx.y;
    a.X += pb * a.x_ps;
    a.g_old += pb * a.gold_ps;
    if (a.g_new) a.g_new += pb * a.gnew_ps;
    a.coef += pb * a.K;
    a.st += pb;
    a.slab += pb * (int64_t)gridDim.x * a.slab_stride;
    a.seed += (uint64_t)pb * kSeedStride;
    a.oma_seed += (uint64_t)pb * kSeedStride;
  }
  if (!SUM_ONLY && a.st->done) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane % LPR, q = lane / LPR;
  const int rg = w * QW + q;
  const int64_t K = a.K, d = a.d;
  const int64_t nch = (d + J - 1) / J;
  const int64_t grid = gridDim.x;

  // Row r of this thread = wave-uniform row-group base (SGPRs) + ONE 32-bit lane
  // offset shared by all R rows (measured 1.8 % faster than buffer_load with one
  // shared VGPR offset on the C3 pass: 6.90 vs 7.03 ms, same box;
  // profiles/history/r02_ab_loads.txt).
  bool rval[R];
#pragma unroll
  for (int i = 0; i < R; ++i) rval[i] = rg + (int64_t)NRG * i < K;
  const float* base[R];
#pragma unroll
  for (int i = 0; i < R; ++i) base[i] = a.X + (int64_t)(w * QW + NRG * i) * a.ldx;
  const uint32_t goff = (uint32_t)q * (uint32_t)a.ldx;
  const uint32_t poff = ((uint32_t)q * J + (uint32_t)(c * V)) * 4u;   // PANEL: bytes from the wave's rows

  // fused OMA: this thread's rows' equalisation scales sd / |h_k| (row k keyed as in
  // the standalone OMA kernel)
  float osc[OMA_INIT ? R : 1];
  if constexpr (OMA_INIT) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      osc[i] = rval[i] ? oma_row_scale(a.oma_seed, (uint64_t)(rg + NRG * i), a.oma_sd) : 0.f;
  }
  float wt[OCC > 1 ? 1 : R];
  float a_noise = 0.f;
  if constexpr (!INIT) {
    if constexpr (OCC > 1) {
      for (int k = tid; k < NRG * R; k += NW * 64) s_w[k] = k < K ? a.coef[k] : 0.f;
      __syncthreads();
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) wt[i] = rval[i] ? a.coef[rg + NRG * i] : 0.f;
    }
    a_noise = a.st->a_noise;
  }

  auto fetch_row = [&](int64_t ch, T& t, int i) {
    if constexpr (PANEL) {
      // One buffer resource per (chunk, row group i) in SGPRs, sized to the rows
      // that exist (rows >= K read 0 through the range check), + the one lane
      // offset (columns >= d: an out-of-range offset).  Branch-free.
      constexpr int64_t GB = (int64_t)NRG * J * 4;   // bytes per row group
      const int64_t wb = (int64_t)(w * QW) * J * 4 + i * GB;   // this wave's rows, bytes
      const int64_t nrec = (int64_t)K * J * 4 - wb;
      const uint32_t vo = (ch < nch && ch * J + c * V < d) ? poff : 0x80000000u;
      load_rows<V>(reinterpret_cast<const float*>(
                       reinterpret_cast<const char*>(a.X + ch * a.panel_stride) + wb),
                   vo, t.x[i], nrec <= 0 ? 0 : nrec > 0x7fffffff ? 0x7fffffff : (int)nrec);
      if ((ch + 1) * J > d) {   // last chunk (block-uniform): padding columns read as 0
#pragma unroll
        for (int v = 0; v < V; ++v)
          if (ch * J + c * V + v >= d) t.x[i][v] = 0.f;
      }
      return;
    }
    const int64_t col = ch * J + (int64_t)c * V;
    const bool cval = ch < nch && col < d;   // V | d: a lane's group is all-in or all-out
    if (cval && rval[i]) {
      load_cols<V>(base[i] + (goff + (uint32_t)col), t.x[i]);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) t.x[i][v] = 0.f;
    }
  };
  // The column-wise operands ride with the chunk on the J finisher threads (one
  // register each), not on every lane: INIT then costs the registers STEP does,
  // and both take the rolling prefetch without spilling.
  auto fetch_aux = [&](int64_t ch, T& t) {
    const int64_t gj = ch * J + tid;
    const bool fin = tid < J && ch < nch && gj < d;
    t.gold = fin ? a.g_old[gj] : 0.f;
    if constexpr (!INIT) t.hn = (fin && a.noise == 2) ? a.hnoise[gj] : 0.f;
  };
  auto fetch = [&](int64_t ch, T& t) {
#pragma unroll
    for (int i = 0; i < R; ++i) fetch_row(ch, t, i);
    fetch_aux(ch, t);
  };

  double row_acc[RPL], row_acc2[RPL];
#pragma unroll
  for (int m = 0; m < RPL; ++m) row_acc[m] = row_acc2[m] = 0.0;
  double mv_acc = 0.0, gn_acc = 0.0;

  // ROLL: row i of chunk `nxt` is loaded into t.x[i] as soon as phase B has
  // consumed row i of chunk ch, so the next chunk's loads are in flight during
  // phase B, the row reductions and the next chunk's barriers (no second tile).
  int par = 0;   // INIT: chunk parity -> s_g buffer
  // fused OMA: noise the tile's real elements (element (k, global column c) takes normal
  // c & 3 of the Philox block (row k, c >> 2): V = 4 columns = one block) and write them
  // back where they were read; padding columns and rows are left untouched
  auto oma_tile = [&](int64_t ch, T& t) {
    const int64_t col = ch * J + (int64_t)c * V;
    if (ch >= nch || col >= d) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (!rval[i]) continue;
      const int64_t k = rg + (int64_t)NRG * i;
      float z[4];
      normal4_hw(a.oma_seed, kStreamOmaNoise, (uint64_t)k, (uint64_t)(a.col_off + col) >> 2, z);
      // (the padding columns of a partial last group stay 0: they enter the distances)
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (col + v < d) t.x[i][v] = oma_noisy(t.x[i][v], osc[i], z[v]);
      float* dst;
      if constexpr (PANEL)
        dst = const_cast<float*>(a.X) + ch * a.panel_stride + k * J + c * V;
      else
        dst = const_cast<float*>(base[i]) + goff + col;
      if (col + V <= d) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<f4*>(dst) = f4{t.x[i][0], t.x[i][1], t.x[i][2], t.x[i][3]};
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v)
          if (col + v < d) dst[v] = t.x[i][v];
      }
    }
  };
  auto process = [&](int64_t ch, T& t, int64_t nxt) {
    float gv[V];
    if constexpr (OMA_INIT) oma_tile(ch, t);
    if constexpr (INIT) {
      // the guess at this chunk's columns -> LDS (buffer by parity: a thread still
      // reading the previous chunk's buffer has not passed this chunk's barrier)
      if (tid < J) {
        s_g[par][tid] = t.gold;
        gn_acc += (double)(t.gold * t.gold);
      }
      __syncthreads();
#pragma unroll
      for (int v = 0; v < V; ++v) gv[v] = s_g[par][c * V + v];
      par ^= 1;
    } else {
      // phase A: weighted column sums over this thread's rows ...
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        float wi;
        if constexpr (OCC > 1) wi = s_w[rg + NRG * i];
        else wi = wt[i];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = fmaf(wi, t.x[i][v], acc[v]);
      }
      // ... over the wave's row groups ...
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += __shfl_xor(acc[v], o, 64);
      if (q == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) s_red[w][c * V + v] = acc[v];
      }
      __syncthreads();
      // ... and over the waves: one finisher thread per column writes g'.
      if (tid < J) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sum += s_red[ww][tid];
        const int64_t gj = ch * J + tid;
        float gnew = 0.f;
        if (gj < d) {
          gnew = sum;
          if (a.noise == 1) {
            gnew = fmaf(a_noise, normal1(a.seed, kStreamNoise, a.iter, a.col_off + gj), gnew);
          } else if (a.noise == 2) {
            gnew = fmaf(a_noise, t.hn, gnew);
          }
          a.g_new[gj] = gnew;
          const float diff = t.gold - gnew;
          mv_acc += (double)(diff * diff);
          gn_acc += (double)(gnew * gnew);
        }
        s_g[0][tid] = gnew;
      }
      __syncthreads();
#pragma unroll
      for (int v = 0; v < V; ++v) gv[v] = s_g[0][c * V + v];
    }
    if constexpr (SUM_ONLY) {
      if constexpr (ROLL) fetch(nxt, t);
      return;
    }
    // phase B: squared distances of this thread's rows to the (new) iterate
    // (+ ||x_k||^2 for the AirComp INIT pass).
    float e[R], e2[WANT_R ? R : 1];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float tt = t.x[i][v] - gv[v];
        s = fmaf(tt, tt, s);
        if constexpr (WANT_R) s2 = fmaf(t.x[i][v], t.x[i][v], s2);
      }
      e[i] = s;
      if constexpr (WANT_R) e2[i] = s2;
      if constexpr (ROLL) {
        // keep row i's next load behind row i's use: without the fence the
        // compiler hoists all R loads above phase B (two live tiles, spills)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
        fetch_row(nxt, t, i);
      }
    }
    if constexpr (ROLL) fetch_aux(nxt, t);
    transpose_reduce<LPR, R>(e, c);
#pragma unroll
    for (int m = 0; m < RPL; ++m) row_acc[m] += (double)e[m];
    if constexpr (WANT_R) {
      transpose_reduce<LPR, R>(e2, c);
#pragma unroll
      for (int m = 0; m < RPL; ++m) row_acc2[m] += (double)e2[m];
    }
  };

  if constexpr (PIPE) {
    T ta, tb;
    int64_t ch = blockIdx.x;
    fetch(ch, ta);
    for (; ch < nch; ch += 2 * grid) {
      fetch(ch + grid, tb);
      process(ch, ta, -1);
      if (ch + grid >= nch) break;       // block-uniform
      fetch(ch + 2 * grid, ta);
      process(ch + grid, tb, -1);
    }
  } else if constexpr (ROLL2) {
    // two tiles, each rolled two grid strides ahead: chunks c+1 and c+2 in flight while
    // c is reduced (for passes whose blocks are latency-bound on too few bytes in flight:
    // small chunks, C5's K = 50 x 128 panels)
    T ta, tb;
    int64_t ch = blockIdx.x;
    fetch(ch, ta);
    fetch(ch + grid, tb);
    for (; ch < nch; ch += 2 * grid) {
      process(ch, ta, ch + 2 * grid);
      if (ch + grid >= nch) break;       // block-uniform
      process(ch + grid, tb, ch + 3 * grid);
    }
  } else if constexpr (ROLL) {
    T t;
    fetch(blockIdx.x, t);
    for (int64_t ch = blockIdx.x; ch < nch; ch += grid) process(ch, t, ch + grid);
  } else {
    for (int64_t ch = blockIdx.x; ch < nch; ch += grid) {
      T t;
      fetch(ch, t);
      process(ch, t, -1);
    }
  }

  // Per-block partials -> slab row.  [D2 (K)] [r (K), INIT only] [mv2] [gn2];
  // the Gram closing pass (SUM_ONLY) writes [||p - g||^2] [||g||^2] only.
  double* out = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  const int i_c = row_of_lane<LPR, R>(c);
  constexpr int SPAN = R < LPR ? LPR / R : 1;   // lanes holding copies of one row sum
  if (!SUM_ONLY && (c % SPAN) == 0) {
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
    for (int ww = 0; ww < NW; ++ww) {
      m += s_fin[0][ww];
      g += s_fin[1][ww];
    }
    const int64_t b = SUM_ONLY ? 0 : INIT ? 2 * K : K;
    out[b] = m;
    out[b + 1] = g;
  }
}

// ---------------------------------------------------------------------------
// Launch plumbing.  GMAGG_PASS_VARIANT: -1 auto (default), 0 plain, 1 pipelined
// (-DGMK_PIPE_VARIANT builds only), 2 rolling prefetch, 3 two tiles rolled two chunks
// ahead (panels).

static int pass_variant() {
  static const int v = [] {
    const char* e = getenv("GMAGG_PASS_VARIANT");
    return e ? atoi(e) : -1;
  }();
  return v;
}

template <int V, int NW, int LPR, int R, int MODE, int OCC>
static const void* pass_fn(bool panel) {
  // Measured on MI355X (profiles/history/r01_ab_pass.txt, r01_pipe_sweep.txt): the plain
  // pass is as fast or faster than the two-tile PIPE variant at every K, so that
  // one is only built with -DGMK_PIPE_VARIANT for A/B runs.
  // Panels: the rolling-prefetch STEP pass (6.44-6.56 vs 6.63 ms at C3), and since round 6
  // the INIT pass too (mode 1 / 2; the fused-OMA INIT, mode 4, stays plain): the plain INIT
  // ran 117-128 us above the STEP pass at C3 in three of four interleaved pairs (12 in the
  // first), the rolling one 32-48 us (profiles/r6s3_init_roll_ab.jsonl; round 2 had measured no
  // gain, profiles/history/r2_init_ab.txt).  The schedule moves loads, not arithmetic: the
  // results are the same bits.
  constexpr bool kRollDefault = MODE == 0;
  constexpr bool kRollPanel = kRollDefault || MODE == 1 || MODE == 2;
  if constexpr (V == 4) {
    if (panel) {
      const int pv = pass_variant();
      if (pv == 3)
        return reinterpret_cast<const void*>(&weiszfeld_pass<V, NW, LPR, R, MODE, 3, OCC, true>);
      if (pv == 2 || (pv < 0 && kRollPanel))
        return reinterpret_cast<const void*>(&weiszfeld_pass<V, NW, LPR, R, MODE, 2, OCC, true>);
      return reinterpret_cast<const void*>(&weiszfeld_pass<V, NW, LPR, R, MODE, 0, OCC, true>);
    }
  } else if (panel) {
    return nullptr;
  }
#ifdef GMK_PIPE_VARIANT
  if (pass_variant() == 1)
    return reinterpret_cast<const void*>(&weiszfeld_pass<V, NW, LPR, R, MODE, 1, OCC>);
#endif
  // Row-major STEP passes with float4 rows also take the rolling prefetch: C5's
  // batched K=50 tile streams 4.64 vs 4.43 TB/s (profiles/history/r04_c5_roll_ab.txt).
  if (pass_variant() == 2 || (pass_variant() < 0 && kRollDefault && V == 4))
    return reinterpret_cast<const void*>(&weiszfeld_pass<V, NW, LPR, R, MODE, 2, OCC>);
  return reinterpret_cast<const void*>(&weiszfeld_pass<V, NW, LPR, R, MODE, 0, OCC>);
}

template <int V, int NW, int LPR, int R, int OCC>
static const void* pass_fn_mode(int mode, bool panel) {
  switch (mode) {
    case 0: return pass_fn<V, NW, LPR, R, 0, OCC>(panel);
    case 1: return pass_fn<V, NW, LPR, R, 1, OCC>(panel);
    case 2: return pass_fn<V, NW, LPR, R, 2, OCC>(panel);
    case 4:
      if constexpr (V == 4) return pass_fn<V, NW, LPR, R, 4, OCC>(panel);
      else return nullptr;
    default: return pass_fn<V, NW, LPR, R, 3, OCC>(panel);
  }
}

// (waves per block, lanes per row segment, rows per thread, blocks per CU) tiles built.
#define GMK_FOR_EACH_CFG(X_, V_)                                                             \
  X_(V_, 16, 64, 1, 1) X_(V_, 16, 64, 2, 1) X_(V_, 16, 64, 4, 1) X_(V_, 16, 64, 8, 1)        \
  X_(V_, 16, 32, 8, 1) X_(V_, 16, 16, 8, 1) X_(V_, 16, 8, 8, 1) X_(V_, 16, 4, 8, 1)          \
  X_(V_, 16, 4, 4, 1) X_(V_, 16, 16, 4, 1) X_(V_, 8, 8, 16, 1) X_(V_, 8, 4, 8, 1)            \
  X_(V_, 8, 16, 8, 1) X_(V_, 8, 8, 8, 1) X_(V_, 4, 8, 8, 1) X_(V_, 4, 16, 4, 1)              \
  X_(V_, 8, 32, 4, 1) X_(V_, 16, 8, 8, 2) X_(V_, 16, 16, 16, 1) X_(V_, 8, 8, 16, 2)          \
  X_(V_, 8, 32, 4, 4)                                                                        \
  X_(V_, 16, 32, 8, 2) X_(V_, 16, 64, 4, 2) X_(V_, 16, 64, 16, 1) X_(V_, 8, 16, 8, 2)

static const void* pass_kernel(const PassCfg& cfg, int mode, bool panel = false) {
#define GMK_CASE(V_, W_, L_, R_, O_)                                                 \
  if (cfg.V == V_ && cfg.NW == W_ && cfg.LPR == L_ && cfg.R == R_ && cfg.OCC == O_) \
    return pass_fn_mode<V_, W_, L_, R_, O_>(mode, panel);
  GMK_FOR_EACH_CFG(GMK_CASE, 4)
  GMK_FOR_EACH_CFG(GMK_CASE, 2)
  GMK_FOR_EACH_CFG(GMK_CASE, 1)
#undef GMK_CASE
  return nullptr;
}

bool pass_cfg_supported(const PassCfg& cfg) { return pass_kernel(cfg, 0) != nullptr; }

hipError_t launch_pass(const PassCfg& cfg, int mode, int grid, const PassArgs& a, hipStream_t s,
                       int problems) {
  // the K <= 1024 row-major tile's gm2 passes: the 32-wave rows kernel (rows_pass.hip), the
  // same two blocks per CU, so the same grid and slab
  if (problems == 1 && cfg.V == 4 && cfg.NW == 8 && cfg.LPR == 8 && cfg.R == 16 && cfg.OCC == 2 &&
      rows_pass_eligible(a, mode))
    return launch_rows_pass(mode, grid, a, s);
  const void* fn = pass_kernel(cfg, mode, a.panel_stride > 0);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<PassArgs*>(&a)};
  return hipLaunchKernel(fn, dim3(grid, problems), dim3(cfg.NW * 64), args, 0, s);
}

int pass_blocks_per_cu(const PassCfg& cfg, int mode) {
  const void* fn = pass_kernel(cfg, mode);
  int n = 0;
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, cfg.NW * 64, 0) != hipSuccess ||
      n < 1)
    return 1;
  return n;
}

}  // namespace gmk
