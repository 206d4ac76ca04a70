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
#include <algorithm>

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

// ---------------------------------------------------------------------------
// Split-bf16 Gram (the default Gram path).  Each centred element is split as
// x' = h + m with h = bf16(x'), m = bf16(x' - h): h + m carries 16 significant
// bits and every bf16 x bf16 product is exact in fp32, so
//   G = (h+m)(h+m)^T = hh^T + hm^T + mh^T + mm^T
// costs four v_mfma_f32_32x32x16_bf16 per 32x32 tile and 16 columns: 1/4 of the
// issue cycles of the f32-input MFMA.  Dropping mm^T (three products) is NOT
// enough: for rows that nearly coincide the m parts are coherent and mm^T is a
// 2^-16-relative bias on D (measured: 2.5e-4 relative error on a tight
// cluster).  What is left — the bits of x' beyond h + m (<= 2^-17 |x'|) and fp32
// accumulation — is priced at run time by the AUTO guard (api.hip, run_gram).
//
// Block: 256 threads; stage = 64 columns x KP rows, loaded as float4 by all
// threads (16 B per row segment, 16 rows per wave instruction), centred, split
// and written as bf16 h/m images [KP][72] (144-B rows: conflict-free
// ds_read_b128 fragment reads).  Two stages of LDS: the global loads of stage
// s+1 are in flight under stage s's MFMAs; one barrier per stage.  Blocks own
// disjoint column ranges of ~8K columns; fp32 partials per block are summed in
// fp64 by gram_reduce (single-level accumulation over <= cpb/4 MFMA steps).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kSplitBK = 64;                // columns per stage
constexpr int kSplitLS = kSplitBK + 8;      // LDS row stride (bf16): 144 B

// Tile t of wave W at compile time (same map as wave_tile).
template <int KT, int W, int T>
struct SplitTile {
  static constexpr int first = KT - W;
  static constexpr int a = KT == 1 ? 0 : (T < first ? W : KT - 1 - W);
  static constexpr int b = KT == 1 ? 0 : (T < first ? W + T : KT - 1 - W + (T - first));
};

template <int KT, int W, int T>
__device__ __forceinline__ void split_tile_mfma(const bf16x8 (&fh)[KT], const bf16x8 (&fm)[KT],
                                                f32x16 (&acc)[GramShape<KT>::PER_WAVE]) {
  if constexpr (T < GramShape<KT>::PER_WAVE) {
    constexpr int a = SplitTile<KT, W, T>::a, b = SplitTile<KT, W, T>::b;
    acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh[a], fh[b], acc[T], 0, 0, 0);
    acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fh[a], fm[b], acc[T], 0, 0, 0);
    acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fm[a], fh[b], acc[T], 0, 0, 0);
    acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fm[a], fm[b], acc[T], 0, 0, 0);
    split_tile_mfma<KT, W, T + 1>(fh, fm, acc);
  }
}

// Split Gram block: 512 threads = 4 MFMA waves (consumers, one compile-time
// specialisation per wave) + 4 staging waves (producers).  A producer thread
// owns 16-byte row segments of a 64-column stage (rows r0 + 16 i, column group
// cg) and keeps TWO stages of loads in flight in two register sets (set = stage
// parity, static after unrolling the stage loop by 2): while the consumers run
// stage s from LDS buffer s&1, the producers centre/split/store stage s+1 into
// buffer (s+1)&1 and re-issue the freed set for stage s+3.  One barrier per
// stage.  ~128 KiB of loads in flight per CU instead of 64.
template <int KT>
struct SplitProducer {
  static constexpr int RPT = GramShape<KT>::ROWS_PER_THREAD;
  const float* X;
  const float* p;
  int64_t K, ldx, c_begin, c_end;
  int r0, cg;
  uint32_t lrow;
  f32x4 st[2][RPT];
  f32x4 pc[2];
  bool cval[2];

  // Every load is issued unconditionally (rows >= K read a real row, columns
  // past c_end read column 0 of the stage) and the padding is applied at commit
  // time — a select at load time lets the compiler turn the load into a branch.
  template <int SET>
  __device__ __forceinline__ void fetch(int s) {
    const int64_t c0 = c_begin + (int64_t)s * kSplitBK;
    cval[SET] = c0 + cg * 4 < c_end;
    const uint32_t lc = cval[SET] ? (uint32_t)(cg * 4) : 0u;
    pc[SET] = *reinterpret_cast<const f32x4*>(p + c0 + lc);
    const float* xs = X + c0;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int64_t rb = 16 * i < K ? 16 * i : 0;      // wave-uniform, always a real row
      const uint32_t off = (r0 + 16 * i < K ? lrow : 0u) + lc;
      st[SET][i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(xs + rb * ldx + off));
    }
  }
  template <int SET>
  __device__ __forceinline__ void commit(__bf16* Lh, __bf16* Lm) {   // centre, split, store
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + 16 * i;
      const f32x4 x = (cval[SET] && r < K) ? st[SET][i] - pc[SET] : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x2 x01 = {x[0], x[1]}, x23 = {x[2], x[3]};
      const bf16x2 h01 = __builtin_convertvector(x01, bf16x2);
      const bf16x2 h23 = __builtin_convertvector(x23, bf16x2);
      const f32x2 r01 = x01 - __builtin_convertvector(h01, f32x2);
      const f32x2 r23 = x23 - __builtin_convertvector(h23, f32x2);
      const bf16x2 m01 = __builtin_convertvector(r01, bf16x2);
      const bf16x2 m23 = __builtin_convertvector(r23, bf16x2);
      *reinterpret_cast<bf16x4*>(Lh + r * kSplitLS + cg * 4) = bf16x4{h01[0], h01[1], h23[0], h23[1]};
      *reinterpret_cast<bf16x4*>(Lm + r * kSplitLS + cg * 4) = bf16x4{m01[0], m01[1], m23[0], m23[1]};
    }
  }
};

template <int KT, int DBG>
__device__ __forceinline__ void split_producer(const float* __restrict__ X, int64_t K,
                                               int64_t ldx, const float* __restrict__ p,
                                               int64_t c_begin, int64_t c_end, int nstage,
                                               __bf16 (*lds)[2][GramShape<KT>::KP * kSplitLS]) {
  SplitProducer<KT> P;
  const int t = threadIdx.x - 256;
  if constexpr (DBG == 2) {          // timing probe: no global loads
    for (int s = 0; s <= nstage; ++s) __syncthreads();
    return;
  }
  P.X = X; P.p = p; P.K = K; P.ldx = ldx; P.c_begin = c_begin; P.c_end = c_end;
  P.r0 = t >> 4; P.cg = t & 15;
  P.lrow = (uint32_t)P.r0 * (uint32_t)ldx;
  // prologue: stage 0 -> buffer 0, stages 1 (set 1) and 2 (set 0) in flight
  if (nstage > 0) P.template fetch<0>(0);
  if (nstage > 1) P.template fetch<1>(1);
  if (nstage > 0) P.template commit<0>(lds[0][0], lds[0][1]);
  if (nstage > 2) P.template fetch<0>(2);
  __syncthreads();
  for (int s = 0; s < nstage; s += 2) {
    // stage s runs on the consumers; commit s+1 (set 1), re-issue set 1 for s+3
    if (s + 1 < nstage) P.template commit<1>(lds[1][0], lds[1][1]);
    if (s + 3 < nstage) P.template fetch<1>(s + 3);
    __syncthreads();
    if (s + 1 >= nstage) break;
    // stage s+1 runs; commit s+2 (set 0), re-issue set 0 for s+4
    if (s + 2 < nstage) P.template commit<0>(lds[0][0], lds[0][1]);
    if (s + 4 < nstage) P.template fetch<0>(s + 4);
    __syncthreads();
  }
}

// Consumer wave W (W < 0: idle slot for KT < 8): per 16-column step it reads the
// h/m fragments of row tiles W..KT-1 once (one ds_read_b128 each) and issues 4
// MFMAs per tile, all registers statically indexed.
template <int KT, int W, int DBG>
__device__ __forceinline__ void split_consumer(int nstage, float* __restrict__ slab,
                                               __bf16 (*lds)[2][GramShape<KT>::KP * kSplitLS]) {
  using Sh = GramShape<KT>;
  constexpr int NT = Sh::PER_WAVE;
  constexpr bool MMA = W >= 0 && DBG != 1;    // DBG 1: timing probe without MFMAs
  constexpr int LO = KT == 1 ? 0 : (W < 0 ? 0 : W);
  const int lane = threadIdx.x & 63;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  const int fo = (lane & 31) * kSplitLS + (lane >> 5) * 8;   // fragment offset in a tile
  __syncthreads();                                           // stage 0 is in buffer 0
  for (int s = 0; s < nstage; ++s) {
    if constexpr (MMA) {
      const __bf16* Lh = lds[s & 1][0];
      const __bf16* Lm = lds[s & 1][1];
#pragma unroll
      for (int ks = 0; ks < kSplitBK / 16; ++ks) {
        bf16x8 fh[KT], fm[KT];
#pragma unroll
        for (int t = LO; t < KT; ++t) {
          fh[t] = *reinterpret_cast<const bf16x8*>(Lh + t * 32 * kSplitLS + ks * 16 + fo);
          fm[t] = *reinterpret_cast<const bf16x8*>(Lm + t * 32 * kSplitLS + ks * 16 + fo);
        }
        split_tile_mfma<KT, (W < 0 ? 0 : W), 0>(fh, fm, acc);
      }
    }
    __syncthreads();
  }
  if constexpr (MMA) {
    float* out = slab + (int64_t)blockIdx.x * Sh::TILES * 1024;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      int a, b;
      wave_tile<KT>(W, t, a, b);
      float* o = out + tri_index(a, b, KT) * 1024;
#pragma unroll
      for (int e = 0; e < 16; ++e) o[e * 64 + lane] = acc[t][e];
    }
  }
}

template <int KT, int DBG = 0>
__global__ void __launch_bounds__(512, 1) gram_split_partial(const float* __restrict__ X,
                                                             int64_t K, int64_t d, int64_t ldx,
                                                             const float* __restrict__ p,
                                                             int64_t cols_per_block,
                                                             float* __restrict__ slab) {
  __shared__ __bf16 lds[2][2][GramShape<KT>::KP * kSplitLS];   // [buffer][h|m]
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t c_begin = (int64_t)blockIdx.x * cols_per_block;
  const int64_t c_end = c_begin + cols_per_block < d ? c_begin + cols_per_block : d;
  const int nstage = c_begin < c_end ? (int)((c_end - c_begin + kSplitBK - 1) / kSplitBK) : 0;
  if (w >= 4) {
    split_producer<KT, DBG>(X, K, ldx, p, c_begin, c_end, nstage, lds);
    return;
  }
  if constexpr (KT == 8) {
    switch (w) {
      case 0: split_consumer<KT, 0, DBG>(nstage, slab, lds); break;
      case 1: split_consumer<KT, 1, DBG>(nstage, slab, lds); break;
      case 2: split_consumer<KT, 2, DBG>(nstage, slab, lds); break;
      default: split_consumer<KT, 3, DBG>(nstage, slab, lds); break;
    }
  } else if constexpr (KT == 4) {
    switch (w) {
      case 0: split_consumer<KT, 0, DBG>(nstage, slab, lds); break;
      case 1: split_consumer<KT, 1, DBG>(nstage, slab, lds); break;
      default: split_consumer<KT, -1, DBG>(nstage, slab, lds); break;
    }
  } else {
    if (w == 0) split_consumer<KT, 0, DBG>(nstage, slab, lds);
    else split_consumer<KT, -1, DBG>(nstage, slab, lds);
  }
}

// ---------------------------------------------------------------------------
// Scaled fp16 split Gram (the default Gram path since round 2).
//
// Each centred element is scaled by a per-(row, block) power of two 2^e_k and
// split as y = x' 2^e_k = h + m, h = f16(y), m = f16(y - h): h + m carries 22
// significant bits (the remainder is <= 2^-22 |y|), and f16 x f16 products are
// exact in fp32.  Three v_mfma_f32_32x32x16_f16 per 32x32 tile and 16 columns
// (hh^T + hm^T + mh^T) then give the fp32 Gram of 22-bit inputs: the dropped
// mm^T is <= 2^-22 |y_k||y_l| per column, a quarter of an fp32 rounding, where
// the bf16 split (16 bits) needed all four products.  G_kl = 2^-(e_k+e_l) (the
// accumulated tile), applied exactly (ldexp) when a partial is written.
//
// f16 has 5 exponent bits, hence the scale: e_k puts the row's largest |x'| over
// the block's first two stages (128 columns, read before anything is
// converted) at [2^3, 2^4).  Elements up to 4095x that size stay finite; much
// smaller ones keep an absolute precision of 2^-24 (f16 subnormals, which the
// f16 MFMA and conversion keep), i.e. 2^-27 of the row's largest element.  An
// element beyond the headroom becomes inf, G non-finite: gram_check flags it
// (KState::gram_bad) and the host reruns the bf16 split (api.hip run_gram).
//
// Block = 4 waves, ONE per SIMD with the whole 512-entry register file, and no
// producer/consumer split: every wave streams a quarter of each 64-column stage
// (16 rows x float4 per lane), converts it into the LDS h/m images and runs its
// 9 tiles' MFMAs.  Three stages of loads are in flight in three register sets
// (192 KiB per CU): while the MFMAs of stage s read LDS buffer s&1, each wave
// commits stage s+1 (set (s+1)%3) into buffer (s+1)&1 four rows per 16-column
// MFMA step and re-issues each committed row's registers for stage s+4 at once
// (rolling).  One barrier per stage.  The bf16 kernel's two-role block held two
// sets at most and its producers streamed 5.0 TB/s on their own
// (profiles/history/r02_gram_split.txt).  Persistent: one block per CU over a contiguous
// ~d/num_cu column range; the fp32 accumulators are flushed to a partial every
// kH16Flush stages (8192 columns, the bf16 kernel's accumulation length).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

#ifndef GMK_H16_PROBE
#define GMK_H16_PROBE 0       // timing-probe builds only (3: no LDS stores, 4: no LDS reads)
#endif
#ifndef GMK_H16_DIAG
#define GMK_H16_DIAG 1        // diagonal tiles in 2 MFMA products (0: 3, A/B builds)
#endif
#ifndef GMK_H16_MIX
#define GMK_H16_MIX 1         // 0: the residual by convert-back + subtract (A/B builds)
#endif
// m = f16(y - h) for the two halves of h = f16(y0, y1): one v_fma_mix per element
// (y - h is exact in the mixed FMA, then ONE rounding to f16: the same bits as the
// f32 subtract + convert, at a third of the instructions; checked bit for bit by
// tools/mixcheck.hip).  The compiler selects no fma_mix for this pattern itself.
__device__ __forceinline__ f16x2 f16_residual(f16x2 h, float y0, float y1) {
  uint32_t m;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(m) : "v"(h), "v"(y0));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(m) : "v"(h), "v"(y1));
  return __builtin_bit_cast(f16x2, m);
}
constexpr int kH16BK = 64;            // columns per stage
constexpr int kH16LS = kH16BK + 8;    // LDS row stride (halves): 144 B
constexpr int kH16Flush = 128;        // stages per fp32 partial

template <int KT>
using H16Lds = _Float16[2][2][GramShape<KT>::KP * kH16LS];   // [buffer][h|m][row][col]

// WS = 0: X row-major; WS > 0: the panel layout [ceil(d/W)][K][W], W = 1 << WS.
template <int KT, int NS, int WS>
struct H16Stream {
  static constexpr bool PANEL = WS > 0;
  static constexpr int RPT = GramShape<KT>::ROWS_PER_THREAD;
  // Rows of a producer thread (r0 = 0..15).  Row-major: rows 16 i + r0 (one resource
  // per row group).  Panels: runs of RUN consecutive rows, r0 * RUN + j in run q at
  // q * RSTRIDE, so a row's byte offset in the stage is a constant that mostly fits
  // the load's immediate field, and the 16-lane halves of a ds_write hit disjoint
  // banks (rows 8 apart: 288 dwords, 32 banks off).
  static constexpr int RUN = RPT < 8 ? RPT : 8;
  static constexpr int RSTRIDE = GramShape<KT>::KP / (RPT / RUN);
  static __device__ __forceinline__ constexpr int prow(int i) {   // panels: row - r0 * RUN
    return (i / RUN) * RSTRIDE + i % RUN;
  }
  const float* X;
  const float* p;
  int64_t K, ldx, c_begin, c_end;
  int64_t pstride;   // panels: elements between panels (>= K * W)
  int r0, cg;
  uint32_t voff;   // byte offset of this lane's first row (row-major: within a row group)
  __device__ __forceinline__ int row(int i) const { return PANEL ? r0 * RUN + prow(i) : 16 * i + r0; }
  f32x4 st[NS][RPT];
  f32x4 pc[NS];
  float cm[NS];    // 1 for a stage's real columns, 0 past c_end
  float sb;        // the block's scale 2^e

  // Row-major: row group i (rows 16i + r0) is a raw buffer resource in SGPRs at row
  // 16i plus the lane's VGPR offset r0 * ldx * 4 (the same for every full group);
  // lanes past K read row 16i (or row 0 for a group wholly past K).  Panels: ONE
  // resource per stage, sized to the panel's K rows, and the row in the lane offset
  // + a constant (rows past K read 0 from the range check; 16 SGPR resources per
  // stage spilled).  Columns past c_end re-read the stage's first columns, zeroed by cm.
  __device__ __forceinline__ uint32_t stage_cols(int s, float& cmv) const {
    const int64_t c0 = c_begin + (int64_t)s * kH16BK;
    const bool cval = c0 + cg * 4 < c_end;
    cmv = cval ? 1.f : 0.f;
    return cval ? (uint32_t)(cg * 16) : 0u;
  }
  // lb: stage_cols' column offset; returns the lane offset load_row takes
  __device__ __forceinline__ uint32_t stage_off(uint32_t lb) const {
    return PANEL ? lb + voff : lb;
  }
  __device__ __forceinline__ f32x4 load_row(int s, int i, uint32_t lo) const {
    const int64_t c0 = c_begin + (int64_t)s * kH16BK;
    if constexpr (PANEL) {
      // a 64-column stage never straddles a panel (W a multiple of 64); its rows
      // are W floats apart: 256 B row segments 4W B apart, K * 4W bytes per stage
      const float* base = X + (c0 >> WS) * pstride + (c0 & ((1 << WS) - 1));
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(base), 0, (int)(K << (WS + 2)), 0x00020000);
      return __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lo + ((uint32_t)prow(i) << (WS + 2)), 0, 2));
    } else {
      const int64_t rem = K - 16 * i;                      // wave-uniform
      const int64_t rb = rem > 0 ? 16 * i : 0;
      // r0 <= 15: every lane of a full group (rem >= 16) is real; branch-free select
      const uint32_t off = lo + (voff & (0u - (uint32_t)((int64_t)r0 < rem)));
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(X + c0 + rb * ldx), 0, -1, 0x00020000);
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2));
    }
  }
  __device__ __forceinline__ f32x4 load_p(int s, float cmv) const {
    const int64_t c0 = c_begin + (int64_t)s * kH16BK;
    return *reinterpret_cast<const f32x4*>(p + c0 + (cmv != 0.f ? cg * 4 : 0));
  }
  template <int SET>
  __device__ __forceinline__ void fetch(int s) {
    const uint32_t lo = stage_off(stage_cols(s, cm[SET]));
    pc[SET] = load_p(s, cm[SET]);
#pragma unroll
    for (int i = 0; i < RPT; ++i) st[SET][i] = load_row(s, i, lo);
  }
  template <int SET>
  __device__ __forceinline__ float absmax(int i) const {
    const f32x4 x = (st[SET][i] - pc[SET]) * cm[SET];
    return fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3])));
  }
  // y = (x - p) * 2^e as ONE fma per element: f = 2^e (0 past c_end), q = -p f,
  // both per stage and lane.  Rows past K (lanes of a partial last row group) hold
  // a duplicate of a real row: finite values whose G rows / columns >= K no K-space
  // kernel reads.
  template <int SET>
  __device__ __forceinline__ void commit_row(int i, _Float16* Lh, _Float16* Lm, float f,
                                             const f32x4& q) {
    f32x4 x;
#pragma unroll
    for (int v = 0; v < 4; ++v) x[v] = fmaf(st[SET][i][v], f, q[v]);
    const f32x2 x01 = {x[0], x[1]}, x23 = {x[2], x[3]};
    const f16x2 h01 = __builtin_convertvector(x01, f16x2);
    const f16x2 h23 = __builtin_convertvector(x23, f16x2);
#if GMK_H16_MIX
    const f16x2 m01 = f16_residual(h01, x[0], x[1]);
    const f16x2 m23 = f16_residual(h23, x[2], x[3]);
#else
    const f16x2 m01 = __builtin_convertvector(x01 - __builtin_convertvector(h01, f32x2), f16x2);
    const f16x2 m23 = __builtin_convertvector(x23 - __builtin_convertvector(h23, f32x2), f16x2);
#endif
#if GMK_H16_PROBE == 3   // timing probe: the conversion without its LDS stores (wrong G)
    asm volatile("" ::"v"(h01), "v"(h23), "v"(m01), "v"(m23));
    (void)Lh; (void)Lm;
#else
    // Lh / Lm point at this lane's slot of its first row: row i is a constant offset
    // (fits the ds_write immediate: no per-row address arithmetic)
    const int rr = PANEL ? prow(i) : 16 * i;
    *reinterpret_cast<f16x4*>(Lh + rr * kH16LS) = f16x4{h01[0], h01[1], h23[0], h23[1]};
    *reinterpret_cast<f16x4*>(Lm + rr * kH16LS) = f16x4{m01[0], m01[1], m23[0], m23[1]};
#endif
  }
  // commit stage data of set SET into (Lh, Lm), re-issuing each row's registers
  // for stage sn right after its commit (rolling)
  template <int SET>
  __device__ __forceinline__ void commit_refetch(_Float16* Lh, _Float16* Lm, int sn) {
    float cmn;
    const uint32_t lon = stage_off(stage_cols(sn, cmn));
    const f32x4 pcn = load_p(sn, cmn);
    const float f = sb * cm[SET];
    const f32x4 q = -pc[SET] * f;
    _Float16* lh = Lh + (PANEL ? r0 * RUN : r0) * kH16LS + cg * 4;
    _Float16* lm = Lm + (PANEL ? r0 * RUN : r0) * kH16LS + cg * 4;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      commit_row<SET>(i, lh, lm, f, q);
      asm volatile("" ::: "memory");       // the re-issue stays behind this row's commit
      st[SET][i] = load_row(sn, i, lon);
    }
    pc[SET] = pcn;
    cm[SET] = cmn;
  }
};

// Wave W's tiles for one 16-column step, ordered by column tile b descending so
// a b fragment is read just before the MFMAs that use it and dies after them:
// b = KT-1 .. KT-1-W carry two tiles, (W, b) and (KT-1-W, b); b = KT-2-W .. W one,
// (W, b).  Live fragments: the two row tiles' h/m + the current b's (+ the next
// b's, prefetched by the scheduler), instead of every b of the step.
// acc slot of tile (a, b) = its position in wave_tile's order.
template <int KT, int W>
struct H16Order {
  static constexpr int first = KT - W;        // tiles (W, W..KT-1) come first in wave_tile
  static constexpr int slot_w(int b) { return b - W; }
  static constexpr int slot_o(int b) { return first + (b - (KT - 1 - W)); }
};

template <int KT, int W, int B>
__device__ __forceinline__ void h16_step_b(const _Float16* Lh, const _Float16* Lm, int off,
                                           const f16x8& haw, const f16x8& maw,
                                           const f16x8& hao, const f16x8& mao,
                                           f32x16 (&acc)[GramShape<KT>::PER_WAVE]) {
  if constexpr (B >= W) {
    using O = H16Order<KT, W>;
#if GMK_H16_PROBE == 4   // timing probe: MFMAs on register fragments, no LDS reads (wrong G)
    const f16x8 hb = haw * (_Float16)B, mb = maw * (_Float16)B;
#else
    const f16x8 hb = *reinterpret_cast<const f16x8*>(Lh + B * 32 * kH16LS + off);
    const f16x8 mb = *reinterpret_cast<const f16x8*>(Lm + B * 32 * kH16LS + off);
#endif
    constexpr int tw = O::slot_w(B);
    if constexpr (GMK_H16_DIAG && B == W) {
      // diagonal tile: h h^T + h (2m)^T = hh^T + 2 S, S = h m^T; its symmetric part
      // is hh^T + S + S^T, taken by gram_reduce_final (2m: exact in f16)
      acc[tw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(haw, hb, acc[tw], 0, 0, 0);
      acc[tw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(haw, mb + mb, acc[tw], 0, 0, 0);
    } else {
      acc[tw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(haw, hb, acc[tw], 0, 0, 0);
      acc[tw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(haw, mb, acc[tw], 0, 0, 0);
      acc[tw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(maw, hb, acc[tw], 0, 0, 0);
    }
    if constexpr (KT > 1 && B >= KT - 1 - W) {
      constexpr int to = O::slot_o(B);
      if constexpr (GMK_H16_DIAG && B == KT - 1 - W) {
        acc[to] = __builtin_amdgcn_mfma_f32_32x32x16_f16(hao, hb, acc[to], 0, 0, 0);
        acc[to] = __builtin_amdgcn_mfma_f32_32x32x16_f16(hao, mb + mb, acc[to], 0, 0, 0);
      } else {
        acc[to] = __builtin_amdgcn_mfma_f32_32x32x16_f16(hao, hb, acc[to], 0, 0, 0);
        acc[to] = __builtin_amdgcn_mfma_f32_32x32x16_f16(hao, mb, acc[to], 0, 0, 0);
        acc[to] = __builtin_amdgcn_mfma_f32_32x32x16_f16(mao, hb, acc[to], 0, 0, 0);
      }
    }
    h16_step_b<KT, W, B - 1>(Lh, Lm, off, haw, maw, hao, mao, acc);
  }
}

template <int KT, int W>
__device__ __forceinline__ void h16_step(const _Float16* Lh, const _Float16* Lm, int off,
                                         f32x16 (&acc)[GramShape<KT>::PER_WAVE]) {
#if GMK_H16_PROBE == 4
  const f16x8 haw = __builtin_bit_cast(f16x8, (int __attribute__((ext_vector_type(4)))){off, off + 1, off + 2, off + 3});
  const f16x8 maw = haw * (_Float16)0.5f, hao = haw * (_Float16)0.25f, mao = haw * (_Float16)0.125f;
#else
  constexpr int AO = KT == 1 ? 0 : KT - 1 - W;
  const f16x8 haw = *reinterpret_cast<const f16x8*>(Lh + W * 32 * kH16LS + off);
  const f16x8 maw = *reinterpret_cast<const f16x8*>(Lm + W * 32 * kH16LS + off);
  const f16x8 hao = *reinterpret_cast<const f16x8*>(Lh + AO * 32 * kH16LS + off);
  const f16x8 mao = *reinterpret_cast<const f16x8*>(Lm + AO * 32 * kH16LS + off);
#endif
  h16_step_b<KT, W, KT - 1>(Lh, Lm, off, haw, maw, hao, mao, acc);
}

// The same tiles on v_mfma_f32_16x16x32_f16 (GMK_H16_SHAPE == 16, the default since
// round 3; 32 = the 32x32x16 consumer above): each 32 x 32 tile as 2 x 2 sub-tiles of
// 16 x 16, one 32-column k-step per MFMA.  The same cycles per FLOP as 32x32x16; the chip
// holds a higher clock on the 16x16 shape under load (MI355X_MICROARCH.md 'DVFS
// give-back' item 7): C4 shard Gram partial 2,976 -> 2,916 us, aggregation 171.3 -> 174.5
// per s, three interleaved rounds on one box (profiles/history/r3_gram_shape_ab.jsonl).
// Fragment of rows R0..R0+15, k-step columns c..c+31: lane l holds row R0 + (l & 15),
// columns c + 8 (l >> 4) .. +7.
#ifndef GMK_H16_SHAPE
#define GMK_H16_SHAPE 16
#endif
#ifndef GMK_H16_REUSE
#define GMK_H16_REUSE 1       // own row tiles' fragments reused as column fragments (0: A/B)
#endif
typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int KT, int W, int B>
__device__ __forceinline__ void h16s_step_b(const _Float16* Lh, const _Float16* Lm, int off,
                                            const f16x8 (&ha)[2], const f16x8 (&ma)[2],
                                            const f16x8 (&ho)[2], const f16x8 (&mo)[2],
                                            f32x4v (&acc)[GramShape<KT>::PER_WAVE][4]) {
  if constexpr (B >= W) {
    using O = H16Order<KT, W>;
    // G = Y Y^T: a B (column) fragment is addressed like the A (row) fragment of the same
    // rows, so the wave's own row tiles (B == W, B == KT-1-W) reuse their registers: 8 of
    // the 40 LDS fragment reads of wave 0's k-step (KT = 8) are not issued
    f16x8 hb[2], mb[2];
    constexpr int AO = KT == 1 ? 0 : KT - 1 - W;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      if constexpr (GMK_H16_REUSE && B == W) {
        hb[sb] = ha[sb];
        mb[sb] = ma[sb];
      } else if constexpr (GMK_H16_REUSE && B == AO) {
        hb[sb] = ho[sb];
        mb[sb] = mo[sb];
      } else {
        hb[sb] = *reinterpret_cast<const f16x8*>(Lh + (B * 32 + 16 * sb) * kH16LS + off);
        mb[sb] = *reinterpret_cast<const f16x8*>(Lm + (B * 32 + 16 * sb) * kH16LS + off);
      }
    }
    constexpr int tw = O::slot_w(B);
#pragma unroll
    for (int sa = 0; sa < 2; ++sa)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        f32x4v& c = acc[tw][sa * 2 + sb];
        if constexpr (GMK_H16_DIAG && B == W) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha[sa], hb[sb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha[sa], mb[sb] + mb[sb], c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha[sa], hb[sb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha[sa], mb[sb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ma[sa], hb[sb], c, 0, 0, 0);
        }
      }
    if constexpr (KT > 1 && B >= KT - 1 - W) {
      constexpr int to = O::slot_o(B);
#pragma unroll
      for (int sa = 0; sa < 2; ++sa)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
          f32x4v& c = acc[to][sa * 2 + sb];
          if constexpr (GMK_H16_DIAG && B == KT - 1 - W) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ho[sa], hb[sb], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ho[sa], mb[sb] + mb[sb], c, 0, 0, 0);
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ho[sa], hb[sb], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ho[sa], mb[sb], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(mo[sa], hb[sb], c, 0, 0, 0);
          }
        }
    }
    h16s_step_b<KT, W, B - 1>(Lh, Lm, off, ha, ma, ho, mo, acc);
  }
}

template <int KT, int W>
__device__ __forceinline__ void h16s_step(const _Float16* Lh, const _Float16* Lm, int off,
                                          f32x4v (&acc)[GramShape<KT>::PER_WAVE][4]) {
  constexpr int AO = KT == 1 ? 0 : KT - 1 - W;
  f16x8 ha[2], ma[2], ho[2], mo[2];
#pragma unroll
  for (int sa = 0; sa < 2; ++sa) {
    ha[sa] = *reinterpret_cast<const f16x8*>(Lh + (W * 32 + 16 * sa) * kH16LS + off);
    ma[sa] = *reinterpret_cast<const f16x8*>(Lm + (W * 32 + 16 * sa) * kH16LS + off);
    ho[sa] = *reinterpret_cast<const f16x8*>(Lh + (AO * 32 + 16 * sa) * kH16LS + off);
    mo[sa] = *reinterpret_cast<const f16x8*>(Lm + (AO * 32 + 16 * sa) * kH16LS + off);
  }
  h16s_step_b<KT, W, KT - 1>(Lh, Lm, off, ha, ma, ho, mo, acc);
}

// Producer waves (4..7): stream every stage into the LDS images, two stages of
// loads in flight (rolling re-issue).  Three sets fit the 256 VGPRs of a
// two-waves-per-SIMD block only without the unroll by 6 that static set indices
// need (the compiler spilled 50-300 VGPRs at every unroll >= 3 tried).
constexpr int kH16Sets = 2;

template <int KT, int DBG, int WS>
__device__ __forceinline__ void h16_producer(const float* __restrict__ X, int64_t K, int64_t ldx,
                                             int64_t pstride,
                                             const float* __restrict__ p, int64_t c_begin,
                                             int64_t c_end, int nstage, H16Lds<KT>& lds,
                                             int* s_exp, float* s_bmax,
                                             int* __restrict__ bexp) {
  constexpr int RPT = GramShape<KT>::ROWS_PER_THREAD;
  using Str = H16Stream<KT, kH16Sets, WS>;
  Str P;
  const int t = threadIdx.x - 256;
  P.X = X; P.p = p; P.K = K; P.ldx = ldx; P.c_begin = c_begin; P.c_end = c_end;
  P.pstride = pstride;
  P.r0 = t >> 4; P.cg = t & 15;
  P.voff = WS ? (uint32_t)(P.r0 * Str::RUN) << (WS + 2) : (uint32_t)P.r0 * (uint32_t)ldx * 4u;
  if (nstage == 0 || DBG == 2) {                 // no columns: meet the consumers' barriers
    if (DBG == 2)
      for (int k = t; k < GramShape<KT>::KP; k += 256) s_exp[k] = 0;
    if (t == 0) bexp[blockIdx.x] = DBG == 2 ? 0 : 100;   // (no elements: no rounding)
    for (int s = 0; s <= (DBG == 2 ? nstage : 0) + 1; ++s) __syncthreads();   // DBG 2: no loads
    return;
  }
  // Every fetch and commit is unconditional: a stage index past the end is
  // clamped to the last stage (a re-read of <= 3 stages per block) and a commit
  // past the end fills the LDS buffer nobody reads.  A conditional re-issue would
  // keep the set's old value live on the skipped path (a fourth set: spills).
  const int last = nstage - 1;
  P.template fetch<0>(0);
  P.template fetch<1>(min(1, last));
  // the block's scale from the first two stages: max |x'| over its real rows and
  // columns -> wave max -> the 4 producer waves through LDS (one extra barrier,
  // matched by the consumers)
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < RPT; ++i)
    if (P.row(i) < K) mx = fmaxf(mx, fmaxf(P.template absmax<0>(i), P.template absmax<1>(i)));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((t & 63) == 0) s_bmax[t >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(s_bmax[0], s_bmax[1]), fmaxf(s_bmax[2], s_bmax[3]));
  {
    int ex = 0;
    (void)frexpf(mx, &ex);                       // mx = f 2^ex, f in [0.5, 1)
    int e = (mx > 0.f && mx <= 3.0e38f) ? 4 - ex : 0;
    e = e < -100 ? -100 : (e > 100 ? 100 : e);
    P.sb = ldexpf(1.f, e);
    for (int k = t; k < GramShape<KT>::KP; k += 256) s_exp[k] = e;
    // the block's exponent for the callers that bound the split's absolute error (Krum:
    // an element's f16 subnormal floor is 2^-25 of the SCALED value, 2^-25 2^-e unscaled,
    // whatever row it belongs to; coordinate.hip krum_gram_bounds)
    if (t == 0) bexp[blockIdx.x] = e;
  }
  P.template commit_refetch<0>(lds[0][0], lds[0][1], min(2, last));
  __syncthreads();                               // stage 0 in buffer 0, exponents published
  // while the consumers run stage s: commit s+1 (set and buffer (s+1)&1),
  // re-issuing its rows for s+3 one by one: stages s+2 and s+3 in flight.
  // Unrolled by 2 so set and buffer indices are compile-time.
#define GMK_H16_STEP(J)                                                                     \
  {                                                                                         \
    if (s + J >= nstage) break;                                                             \
    P.template commit_refetch<(J + 1) & 1>(lds[(J + 1) & 1][0], lds[(J + 1) & 1][1],        \
                                           min(s + J + 3, last));                           \
    __syncthreads();                                                                        \
  }
  for (int s = 0; s < nstage; s += 2) {
    GMK_H16_STEP(0) GMK_H16_STEP(1)
  }
#undef GMK_H16_STEP
}

// Consumer wave W (0..3; W < 0: no tiles for K <= 128): MFMAs of every stage,
// fp32 partial `seg` to slab[(blockIdx.x * nseg + seg)][tiles][1024], unscaled.
template <int KT, int W, int DBG>
__device__ __forceinline__ void h16_consumer(int nstage, int nseg, float* __restrict__ slab,
                                             H16Lds<KT>& lds, const int* s_exp) {
  using Sh = GramShape<KT>;
  constexpr int NT = Sh::PER_WAVE;
  constexpr bool MMA = W >= 0 && DBG != 1;     // DBG 1: timing probe without MFMAs
  constexpr int WW = W < 0 ? 0 : W;
  const int lane = threadIdx.x & 63;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  float* base = slab + (int64_t)blockIdx.x * nseg * Sh::TILES * 1024;
  auto flush = [&](int seg, bool zero) {
    float* out = base + (int64_t)seg * Sh::TILES * 1024;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      int a, b;
      wave_tile<KT>(WW, t, a, b);
      float* o = out + tri_index(a, b, KT) * 1024;
      const int ec = s_exp[b * 32 + (lane & 31)];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int er = s_exp[a * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)];
        o[e * 64 + lane] = zero ? 0.f : ldexpf(acc[t][e], -(er + ec));
        acc[t][e] = 0.f;
      }
    }
  };
  const int fo = (lane & 31) * kH16LS + (lane >> 5) * 8;   // fragment offset in a tile
  __syncthreads();                                           // the producers' scale exchange
  __syncthreads();                                           // stage 0 is in buffer 0
  int seg = 0;
  for (int s = 0; s < nstage; ++s) {
    if constexpr (MMA) {
      const _Float16* Lh = lds[s & 1][0];
      const _Float16* Lm = lds[s & 1][1];
#pragma unroll
      for (int ks = 0; ks < kH16BK / 16; ++ks) h16_step<KT, WW>(Lh, Lm, ks * 16 + fo, acc);
      if ((s + 1) % kH16Flush == 0 || s + 1 == nstage) flush(seg++, false);
    }
    __syncthreads();
  }
  if constexpr (MMA)
    for (; seg < nseg; ++seg) flush(seg, true);              // blocks with fewer stages
}

// h16_consumer on the 16x16x32 shape: the same slab format (every 32 x 32 tile written
// in the 32x32 accumulator's element order, so gram_reduce_* are unchanged).
template <int KT, int W, int DBG>
__device__ __forceinline__ void h16s_consumer(int nstage, int nseg, float* __restrict__ slab,
                                              H16Lds<KT>& lds, const int* s_exp) {
  using Sh = GramShape<KT>;
  constexpr int NT = Sh::PER_WAVE;
  constexpr bool MMA = W >= 0 && DBG != 1;
  constexpr int WW = W < 0 ? 0 : W;
  const int lane = threadIdx.x & 63;
  f32x4v acc[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[t][q] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float* base = slab + (int64_t)blockIdx.x * nseg * Sh::TILES * 1024;
  auto flush = [&](int seg, bool zero) {
    float* out = base + (int64_t)seg * Sh::TILES * 1024;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      int a, b;
      wave_tile<KT>(WW, t, a, b);
      float* o = out + tri_index(a, b, KT) * 1024;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int sa = q >> 1, sb = q & 1;
        const int C = 16 * sb + (lane & 15);                   // column in the 32x32 tile
        const int ec = s_exp[b * 32 + C];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * sa + 4 * (lane >> 4) + r;          // row in the 32x32 tile
          const int e = ((R & 3) + 4 * (R >> 3)) * 64 + C + 32 * ((R >> 2) & 1);
          o[e] = zero ? 0.f : ldexpf(acc[t][q][r], -(s_exp[a * 32 + R] + ec));
        }
        acc[t][q] = f32x4v{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  const int fo = (lane & 15) * kH16LS + (lane >> 4) * 8;   // fragment offset in a sub-tile
  __syncthreads();                                           // the producers' scale exchange
  __syncthreads();                                           // stage 0 is in buffer 0
  int seg = 0;
  for (int s = 0; s < nstage; ++s) {
    if constexpr (MMA) {
      const _Float16* Lh = lds[s & 1][0];
      const _Float16* Lm = lds[s & 1][1];
#pragma unroll
      for (int ks = 0; ks < kH16BK / 32; ++ks) h16s_step<KT, WW>(Lh, Lm, ks * 32 + fo, acc);
      if ((s + 1) % kH16Flush == 0 || s + 1 == nstage) flush(seg++, false);
    }
    __syncthreads();
  }
  if constexpr (MMA)
    for (; seg < nseg; ++seg) flush(seg, true);
}

template <int KT, int DBG, int WS>
__global__ void __launch_bounds__(512, 1) gram_h16_partial(const float* __restrict__ X, int64_t K,
                                                           int64_t d, int64_t ldx, int64_t pstride,
                                                           const float* __restrict__ p,
                                                           int64_t cols_per_block, int nseg,
                                                           float* __restrict__ slab,
                                                           int* __restrict__ bexp) {
  __shared__ H16Lds<KT> lds;
  __shared__ int s_exp[GramShape<KT>::KP];
  __shared__ float s_bmax[4];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t c_begin = (int64_t)blockIdx.x * cols_per_block;
  const int64_t c_end = c_begin + cols_per_block < d ? c_begin + cols_per_block : d;
  const int nstage = c_begin < c_end ? (int)((c_end - c_begin + kH16BK - 1) / kH16BK) : 0;
  if (w >= 4) {
    h16_producer<KT, DBG, WS>(X, K, ldx, pstride, p, c_begin, c_end, nstage, lds, s_exp, s_bmax,
                              bexp);
    return;
  }
#if GMK_H16_SHAPE == 16
#define GMK_H16_CONSUMER h16s_consumer
#else
#define GMK_H16_CONSUMER h16_consumer
#endif
  if constexpr (KT == 8) {
    switch (w) {
      case 0: GMK_H16_CONSUMER<KT, 0, DBG>(nstage, nseg, slab, lds, s_exp); break;
      case 1: GMK_H16_CONSUMER<KT, 1, DBG>(nstage, nseg, slab, lds, s_exp); break;
      case 2: GMK_H16_CONSUMER<KT, 2, DBG>(nstage, nseg, slab, lds, s_exp); break;
      default: GMK_H16_CONSUMER<KT, 3, DBG>(nstage, nseg, slab, lds, s_exp); break;
    }
  } else if constexpr (KT == 4) {
    switch (w) {
      case 0: GMK_H16_CONSUMER<KT, 0, DBG>(nstage, nseg, slab, lds, s_exp); break;
      case 1: GMK_H16_CONSUMER<KT, 1, DBG>(nstage, nseg, slab, lds, s_exp); break;
      default: GMK_H16_CONSUMER<KT, -1, DBG>(nstage, nseg, slab, lds, s_exp); break;
    }
  } else {
    if (w == 0) GMK_H16_CONSUMER<KT, 0, DBG>(nstage, nseg, slab, lds, s_exp);
    else GMK_H16_CONSUMER<KT, -1, DBG>(nstage, nseg, slab, lds, s_exp);
  }
#undef GMK_H16_CONSUMER
}

// Sum the fp32 block partials in fp64 in a fixed order, in two steps so that
// every element has many loads in flight: gram_reduce_part sums blocks
// y, y+NG, y+2NG, ... (four interleaved fp64 chains, combined in order) into
// tmp[y][e]; gram_reduce_final adds tmp[0..NG) and unpacks the upper triangle
// into a full symmetric G[KP][KP].  Element e of a tile: register reg = e / 64,
// lane = e % 64 -> row (reg&3) + 8*(reg>>2) + 4*(lane>>5), col lane&31.
constexpr int kReduceGroups = 32;

__global__ void __launch_bounds__(256) gram_reduce_part(const float* __restrict__ slab, int nb,
                                                        int64_t n, double* __restrict__ tmp) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y, NG = gridDim.y;
  if (e >= n) return;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  int b = y, i = 0;
  for (; b + 3 * NG < nb; b += 4 * NG) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += (double)slab[(int64_t)(b + u * NG) * n + e];
  }
  for (; b < nb; b += NG, ++i) acc[i & 3] += (double)slab[(int64_t)b * n + e];
  tmp[(int64_t)y * n + e] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// symdiag: the diagonal tiles hold hh^T + 2 h m^T (the f16 kernel): G takes their
// symmetric part, (s(r,c) + s(c,r)) / 2, the same value at both positions.
__global__ void __launch_bounds__(256) gram_reduce_final(const double* __restrict__ tmp, int NG,
                                                         int KT, double* __restrict__ G,
                                                         KState* st, int symdiag) {
  const int tiles = KT * (KT + 1) / 2;
  const int64_t n = (int64_t)tiles * 1024;
  const int KP = 32 * KT;
  bool bad = false;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int y = 0; y < NG; ++y) s += tmp[(int64_t)y * n + e];
    bad |= !isfinite(s);
    const int tix = (int)(e >> 10), el = (int)(e & 1023);
    int a = 0;
    while (tri_index(a, KT - 1, KT) < tix) ++a;        // row tile of this triangle index
    const int bt = a + (tix - tri_index(a, a, KT));
    const int reg = el >> 6, ln = el & 63;
    const int ri = (reg & 3) + 8 * (reg >> 2) + 4 * (ln >> 5), ci = ln & 31;
    const int row = a * 32 + ri;
    const int col = bt * 32 + ci;
    if (symdiag && a == bt && ri != ci) {
      // the element at (ci, ri) of the same tile: lane ri + 32 * ((ci >> 2) & 1),
      // register (ci & 3) + 4 * (ci >> 3)
      const int64_t eT = ((int64_t)tix << 10) + (((ci & 3) + 4 * (ci >> 3)) << 6) + ri + 32 * ((ci >> 2) & 1);
      double sT = 0.0;
      for (int y = 0; y < NG; ++y) sT += tmp[(int64_t)y * n + eT];
      bad |= !isfinite(sT);
      s = 0.5 * (s + sT);                      // the same value at both positions
    }
    G[(int64_t)row * KP + col] = s;
    G[(int64_t)col * KP + row] = s;
  }
  if (bad) st->gram_bad = 1;                           // plain vector store, same value
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
  double last_mv = NAN, prev_mv = NAN;
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
    prev_mv = last_mv;
    last_mv = (double)mv;
    if (tid == 0) s_stop = mv <= tol ? 1 : 0;
    __syncthreads();
    if (s_stop) { conv = 1; ++it; break; }
  }
  if (tid == 0) {
    st->iters = it;
    st->last_movement = last_mv;
    st->converged = conv;
    st->guard_r = last_mv / prev_mv;   // contraction estimate for the AUTO guard (NaN if 1 step)
    st->done = 0;   // let the closing pass run
  }
}

// A posteriori check of the Gram path (AUTO guard, api.hip run_gram).  The
// closing pass was a full streaming STEP pass at the returned weights a, so
// `Dx` holds the exact ||x_k - g||^2 (fp32 elements, fp64 sums, as the
// streaming path computes them).  Compare the next Weiszfeld weights from the
// exact distances with those the K-space loop would take (from G): the
// difference b is the one-step error of the K-space map at g, and its size in
// R^d is sqrt(b^T G b).  Writes it to st->guard_q.  One block.
__global__ void __launch_bounds__(1024) gram_verify(const double* __restrict__ G, int KP, int64_t K,
                                                    float eps, const double* __restrict__ u,
                                                    const double* __restrict__ alpha,
                                                    const double* __restrict__ Dx,
                                                    double* __restrict__ bvec, KState* st) {
  __shared__ double scratch[16];
  const int tid = threadIdx.x;
  double atu = 0.0;
  for (int64_t k = tid; k < K; k += blockDim.x) atu += alpha[k] * u[k];
  atu = block_sum(atu, scratch);
  double wg = 0.0, wx = 0.0;
  for (int64_t k = tid; k < K; k += blockDim.x) {
    const double Dg = G[k * KP + k] - 2.0 * u[k] + atu;
    wg += 1.0 / (double)clamp_dist(Dg > 0.0 ? Dg : (Dg != Dg ? Dg : 0.0), eps);
    wx += 1.0 / (double)clamp_dist(Dx[k], eps);
  }
  const double Wg = block_sum(wg, scratch), Wx = block_sum(wx, scratch);
  for (int64_t k = tid; k < K; k += blockDim.x) {
    const double Dg = G[k * KP + k] - 2.0 * u[k] + atu;
    bvec[k] = (1.0 / (double)clamp_dist(Dg > 0.0 ? Dg : (Dg != Dg ? Dg : 0.0), eps)) / Wg -
              (1.0 / (double)clamp_dist(Dx[k], eps)) / Wx;
  }
  __syncthreads();
  double q = 0.0;
  for (int64_t k0 = tid >> 2; k0 < K; k0 += blockDim.x >> 2) {
    double sacc = 0.0;
    for (int64_t j = tid & 3; j < K; j += 4) sacc += G[k0 * KP + j] * bvec[j];
    sacc += __shfl_xor(sacc, 1, 64);
    sacc += __shfl_xor(sacc, 2, 64);
    if ((tid & 3) == 0) q += bvec[k0] * sacc;
  }
  q = block_sum(q, scratch);
  if (tid == 0) st->guard_q = sqrt(q > 0.0 ? q : (q != q ? q : 0.0));
}

// Non-finite entries in the (all-reduced) Gram -> st->gram_bad.  One block.
__global__ void __launch_bounds__(1024) gram_check(const double* __restrict__ G, int KP, KState* st) {
  bool bad = false;
  for (int i = threadIdx.x; i < KP * KP; i += blockDim.x) bad |= !isfinite(G[i]);
  if (bad) st->gram_bad = 1;                           // plain vector store, same value
}

hipError_t launch_gram_check(const double* G, int KP, KState* st, hipStream_t s) {
  hipLaunchKernelGGL(gram_check, dim3(1), dim3(1024), 0, s, G, KP, st);
  return hipGetLastError();
}

hipError_t launch_gram_verify(const double* G, int KP, int64_t K, float eps, const double* u,
                              const double* alpha, const double* Dx, double* bvec, KState* st,
                              hipStream_t s) {
  hipLaunchKernelGGL(gram_verify, dim3(1), dim3(1024), 0, s, G, KP, K, eps, u, alpha, Dx, bvec, st);
  return hipGetLastError();
}

template <int KT>
static hipError_t launch_gram_kt(const float* X, int64_t K, int64_t d, int64_t ldx,
                                 const float* p, int nb, int64_t cpb, float* slab, hipStream_t s) {
  hipLaunchKernelGGL(gram_partial<KT>, dim3(nb), dim3(256), 0, s, X, K, d, ldx, p, cpb, slab);
  return hipGetLastError();
}

int gram_kt(int64_t K) { return K <= 32 ? 1 : K <= 64 ? 2 : K <= 128 ? 4 : K <= 256 ? 8 : 0; }

// partials [nb * nseg][tiles][1024] fp32, then the reduction's fp64 tmp[kReduceGroups][n],
// then the f16 kernel's per-block scale exponents [nb] (int)
size_t gram_slab_floats(int KT, const GramGrid& g) {
  return (size_t)(g.nb * g.nseg + 2 * kReduceGroups) * (KT * (KT + 1) / 2) * 1024 +
         (size_t)(g.nb + 1) / 2 * 2;
}

int* gram_block_exp(float* slab, int KT, const GramGrid& g) {
  return reinterpret_cast<int*>(slab + (size_t)(g.nb * g.nseg + 2 * kReduceGroups) *
                                           (KT * (KT + 1) / 2) * 1024);
}

template <int KT>
static hipError_t launch_split_kt(const float* X, int64_t K, int64_t d, int64_t ldx,
                                  const float* p, int nb, int64_t cpb, float* slab,
                                  hipStream_t s) {
  // GMAGG_GRAM_DEBUG = 1 / 2: timing probes without MFMAs / without loads (wrong G)
  static const int dbg = [] { const char* e = getenv("GMAGG_GRAM_DEBUG"); return e ? atoi(e) : 0; }();
  if (dbg == 1)
    hipLaunchKernelGGL((gram_split_partial<KT, 1>), dim3(nb), dim3(512), 0, s, X, K, d, ldx, p, cpb,
                       slab);
  else if (dbg == 2)
    hipLaunchKernelGGL((gram_split_partial<KT, 2>), dim3(nb), dim3(512), 0, s, X, K, d, ldx, p, cpb,
                       slab);
  else
    hipLaunchKernelGGL((gram_split_partial<KT, 0>), dim3(nb), dim3(512), 0, s, X, K, d, ldx, p, cpb,
                       slab);
  return hipGetLastError();
}

template <int KT, int DBG>
static hipError_t launch_h16_dbg(const float* X, int64_t K, int64_t d, int64_t ldx, int64_t pstride,
                                 int wshift, const float* p, int nb, int64_t cpb, int nseg,
                                 float* slab, int* bexp, hipStream_t s) {
  // panel widths of the Gram tiles (gm_panel_width at K <= 256): 64, 128, 256
#define GMK_H16_LAUNCH(WS_)                                                                  \
  hipLaunchKernelGGL((gram_h16_partial<KT, DBG, WS_>), dim3(nb), dim3(512), 0, s, X, K, d, ldx, \
                     pstride, p, cpb, nseg, slab, bexp)
  if (!pstride) GMK_H16_LAUNCH(0);
  else if (wshift == 7) GMK_H16_LAUNCH(7);
  else if (wshift == 6) GMK_H16_LAUNCH(6);
  else if (wshift == 8) GMK_H16_LAUNCH(8);
  else return hipErrorInvalidValue;
#undef GMK_H16_LAUNCH
  return hipSuccess;
}

template <int KT>
static hipError_t launch_h16_kt(const float* X, int64_t K, int64_t d, int64_t ldx, int64_t pstride,
                                int wshift, const float* p, int nb, int64_t cpb, int nseg,
                                float* slab, int* bexp, hipStream_t s) {
  // GMAGG_GRAM_DEBUG = 1 / 2: timing probes without MFMAs / without loads (wrong G)
  static const int dbg = [] { const char* e = getenv("GMAGG_GRAM_DEBUG"); return e ? atoi(e) : 0; }();
  hipError_t e;
  if (KT == 8 && dbg == 1)   // probes built for the 256-row tile only
    e = launch_h16_dbg<KT, KT == 8 ? 1 : 0>(X, K, d, ldx, pstride, wshift, p, nb, cpb, nseg, slab, bexp, s);
  else if (KT == 8 && dbg == 2)
    e = launch_h16_dbg<KT, KT == 8 ? 2 : 0>(X, K, d, ldx, pstride, wshift, p, nb, cpb, nseg, slab, bexp, s);
  else
    e = launch_h16_dbg<KT, 0>(X, K, d, ldx, pstride, wshift, p, nb, cpb, nseg, slab, bexp, s);
  return e != hipSuccess ? e : hipGetLastError();
}

// Grid of one Gram launch: blocks, columns per block, fp32 partials per block.
GramGrid gram_grid(int64_t d, GramKind kind, int num_cu) {
  GramGrid g{};
  if (kind == GramKind::H16) {          // persistent: one block per CU
    g.nb = (int)std::max<int64_t>(1, std::min<int64_t>(num_cu, (d + kH16BK - 1) / kH16BK));
    g.cpb = ((d + g.nb - 1) / g.nb + kH16BK - 1) / kH16BK * kH16BK;
    g.nb = (int)std::max<int64_t>(1, (d + g.cpb - 1) / g.cpb);
    const int64_t st = g.cpb / kH16BK;
    g.nseg = (int)((st + kH16Flush - 1) / kH16Flush);
    return g;
  }
  const bool split = kind == GramKind::BF16;
  if (split) {   // ~8K columns per block, whole rounds of one block per CU
    g.nb = (int)std::max<int64_t>(1, (d + 8191) / 8192);
    if (g.nb > num_cu) g.nb = (g.nb + num_cu - 1) / num_cu * num_cu;
  } else {
    g.nb = std::max(1, std::min(4 * num_cu, (int)((d + 4095) / 4096)));
  }
  const int64_t q = split ? kSplitBK : kGramJC;
  g.cpb = ((d + g.nb - 1) / g.nb + q - 1) / q * q;
  g.nb = (int)std::max<int64_t>(1, (d + g.cpb - 1) / g.cpb);
  g.nseg = 1;
  return g;
}

hipError_t launch_gram(const float* X, int64_t K, int64_t d, int64_t ldx, const float* p,
                       GramKind kind, const GramGrid& g, float* slab, double* G, KState* st,
                       hipStream_t s, int64_t pstride, int wshift) {
  if (pstride && kind != GramKind::H16) return hipErrorInvalidValue;   // panels: f16 kernel only
  const int KT = gram_kt(K);
  const int nb = g.nb;
  const int64_t cpb = g.cpb;
  hipError_t e;
  if (kind == GramKind::H16) {
    int* bexp = gram_block_exp(slab, KT, g);
    switch (KT) {
      case 1: e = launch_h16_kt<1>(X, K, d, ldx, pstride, wshift, p, nb, cpb, g.nseg, slab, bexp, s); break;
      case 2: e = launch_h16_kt<2>(X, K, d, ldx, pstride, wshift, p, nb, cpb, g.nseg, slab, bexp, s); break;
      case 4: e = launch_h16_kt<4>(X, K, d, ldx, pstride, wshift, p, nb, cpb, g.nseg, slab, bexp, s); break;
      case 8: e = launch_h16_kt<8>(X, K, d, ldx, pstride, wshift, p, nb, cpb, g.nseg, slab, bexp, s); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (KT * (kind == GramKind::BF16 ? -1 : 1)) {
      case 1: e = launch_gram_kt<1>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case 2: e = launch_gram_kt<2>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case 4: e = launch_gram_kt<4>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case 8: e = launch_gram_kt<8>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case -1: e = launch_split_kt<1>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case -2: e = launch_split_kt<2>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case -4: e = launch_split_kt<4>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      case -8: e = launch_split_kt<8>(X, K, d, ldx, p, nb, cpb, slab, s); break;
      default: return hipErrorInvalidValue;
    }
  }
  if (e != hipSuccess) return e;
  const int parts = nb * g.nseg;
  const int64_t n = (int64_t)(KT * (KT + 1) / 2) * 1024;
  const int ng = std::min(kReduceGroups, parts);
  double* tmp = reinterpret_cast<double*>(slab + (size_t)parts * n);
  hipLaunchKernelGGL(gram_reduce_part, dim3((unsigned)((n + 255) / 256), ng), dim3(256), 0, s,
                     slab, parts, n, tmp);
  hipLaunchKernelGGL(gram_reduce_final, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tmp,
                     ng, KT, G, st, (int)(kind == GramKind::H16 && GMK_H16_DIAG));
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
