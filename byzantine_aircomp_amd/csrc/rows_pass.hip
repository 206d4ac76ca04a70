// The fused Weiszfeld pass on the reference's own row-major [K, ldx] stack at 512 < K <= 1024
// (round 6): the drop-in layout's STEP pass for gm2 (M:174-181, stream_pass.hip's algorithm).
//
// Why a second kernel for the same arithmetic.  On row-major X every 128-byte row segment of
// a chunk lies in its own 2 MB page (rows are 4 * ldx bytes apart), so the per-CU address
// translation cache misses on about every second request: UTCL1 miss rate 47 % against
// 0.01 % on panels, at the same HBM bytes (profiles/r6s1_utcl1_c3_rows_vs_panels.json;
// the read-only probe profiles/r6s1_rows_probe.jsonl shows the step as the row gap crosses
// 2 MB).  Translation misses are a latency, so the cure is more of them in flight: 32 waves
// per CU instead of 16 — two 1024-thread blocks, each thread holding 8 rows x 4 columns (32
// floats instead of stream_pass's 64), which the generic template cannot fit in the 64
// VGPRs that occupancy allows (it spills 40-83).  This kernel is that tile with nothing
// else: gm2 only (no column noise, no OMA), rows through buffer resources whose range check
// zeroes rows >= K (no per-row masks), the row weights and the finisher threads' movement /
// norm partials in LDS, every cross-lane sum on DPP / permlane moves (no index registers):
// 1-6 VGPRs spilled.  Measured at C3 on rows (profiles/r6s1_rows_lean32w_dpp_ab.jsonl, four
// interleaved rounds): STEP 6,811 vs 6,949 us (0.807 vs 0.791 of HBM), 24.49 vs 24.01
// aggregations/s; the read-only probe of this tile shape reached 0.854
// (profiles/history/r03_panels_ab.txt, "1024thr J=32").
//
// Thread map: wave w, lane = 8 q + c: column group c (4 columns, 16 B), row group
// rg = 8 w + q; rows rg + 128 i, i < 8.  A wave instruction reads 8 rows x 128 B.
// Chunk order: grid-stride, except that the two blocks one CU holds (b, b + #CUs) take
// adjacent chunks when the grid is two blocks per CU (PassArgs.chunk_pair; STEP 6,844 ->
// 6,788 us at C3, profiles/r6s2_rows_chunk_pair_ab.jsonl).
#include "device_util.h"
#include "gmagg_internal.h"

namespace gmk {

namespace {
constexpr int kRW = 16;             // waves per block
constexpr int kRL = 8;              // lanes per row segment
constexpr int kRR = 8;              // rows per thread
constexpr int kRJ = 4 * kRL;        // chunk width (columns)
constexpr int kRQ = 64 / kRL;       // rows per wave instruction
constexpr int kRG = kRW * kRQ;      // row groups per block (128)
}  // namespace

template <bool INIT>
__global__ void __launch_bounds__(kRW * 64, 8) rows_pass(PassArgs a) {
  __shared__ float s_w[kRG * kRR];
  __shared__ float s_red[kRW][kRJ];
  __shared__ float s_g[2][kRJ];
  __shared__ double s_acc[2][kRJ];   // finisher thread j's movement / norm partials (LDS, not VGPRs)
  if (a.st->done) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane % kRL, q = lane / kRL;
  const int rg = w * kRQ + q;
  const int64_t K = a.K, d = a.d, ldx = a.ldx;
  const int64_t nch = (d + kRJ - 1) / kRJ;
  const int64_t grid = gridDim.x;
  if constexpr (!INIT) {
    for (int k = tid; k < kRG * kRR; k += kRW * 64) s_w[k] = k < K ? a.coef[k] : 0.f;
    __syncthreads();
  }
  typedef float f4 __attribute__((ext_vector_type(4)));
  // Row group i of this wave (rows w*8 + 128 i .. +7): ONE buffer resource per group, sized
  // to its rows < K (the range check zeroes the others), chunk-independent (SGPRs); the lane
  // offset q * ldx + the chunk's column (one VGPR per chunk, shared by the 8 groups).
  __amdgpu_buffer_rsrc_t rs[kRR];
#pragma unroll
  for (int i = 0; i < kRR; ++i) {
    const int64_t r0 = (int64_t)w * kRQ + (int64_t)kRG * i;
    const int64_t nv = K - r0 < kRQ ? (K - r0 > 0 ? K - r0 : 0) : kRQ;
    rs[i] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.X + r0 * ldx), 0,
                                              (int)(nv * ldx * 4), 0x00020000);
  }
  const uint32_t qoff = (uint32_t)q * (uint32_t)ldx * 4u;
  const uint32_t c4 = 4u * (uint32_t)c;
  auto lane_off = [&](int64_t ch) -> uint32_t {
    const int64_t col0 = ch * kRJ;                       // wave-uniform
    return (ch < nch && (uint64_t)col0 + c4 < (uint64_t)d) ? qoff + ((uint32_t)col0 + c4) * 4u
                                                           : 0x80000000u;
  };
  auto load = [&](uint32_t off, f4& x, int i) {
    x = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs[i], off, 0, 2));
  };

  f4 x[kRR];
  double row_acc = 0.0;
  if (tid < kRJ) {
    s_acc[0][tid] = 0.0;
    s_acc[1][tid] = 0.0;
  }
  float gold = 0.f;
  auto fetch_gold = [&](int64_t ch) {
    const int64_t gj = ch * kRJ + tid;
    gold = (tid < kRJ && ch < nch && gj < d) ? a.g_old[gj] : 0.f;
  };
  int par = 0;
  int64_t ch = first_chunk(a.chunk_pair, blockIdx.x, grid);   // chunks ch, ch + grid, ...
  {
    const uint32_t off = lane_off(ch);
#pragma unroll
    for (int i = 0; i < kRR; ++i) load(off, x[i], i);
  }
  fetch_gold(ch);
  for (; ch < nch; ch += grid) {
    const int64_t nxt = ch + grid;
    f4 gv;
    if constexpr (INIT) {
      if (tid < kRJ) {
        s_g[par][tid] = gold;
        s_acc[1][tid] += (double)(gold * gold);
      }
      __syncthreads();
      gv = f4{s_g[par][4 * c], s_g[par][4 * c + 1], s_g[par][4 * c + 2], s_g[par][4 * c + 3]};
      par ^= 1;
    } else {
      // phase A: g'_j = sum_k c_k x_kj over this thread's rows, the wave's row groups,
      // then the waves (one finisher thread per column)
      f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < kRR; ++i) acc += s_w[rg + kRG * i] * x[i];
      // the wave's 8 row groups (lane bits 3-5) on DPP / permlane moves: no LDS round trip
      // and no index registers (row_ror:8 inside a 16-lane row is lane ^ 8)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float t = acc[v];
        t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x128, 0xf, 0xf, false));
        const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(t), __float_as_uint(t), false, false);
        t = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
        const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
        acc[v] = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
      }
      if (q == 0) *reinterpret_cast<f4*>(&s_red[w][4 * c]) = acc;
      __syncthreads();
      if (tid < kRJ) {
        float sum = 0.f;
#pragma unroll
        for (int ww = 0; ww < kRW; ++ww) sum += s_red[ww][tid];
        const int64_t gj = ch * kRJ + tid;
        float gnew = 0.f;
        if (gj < d) {
          gnew = sum;
          a.g_new[gj] = gnew;
          const float diff = gold - gnew;
          s_acc[0][tid] += (double)(diff * diff);
          s_acc[1][tid] += (double)(gnew * gnew);
        }
        s_g[0][tid] = gnew;
      }
      __syncthreads();
      gv = f4{s_g[0][4 * c], s_g[0][4 * c + 1], s_g[0][4 * c + 2], s_g[0][4 * c + 3]};
    }
    // phase B: this thread's rows' squared distances to the new iterate; row i's next
    // chunk is loaded into its registers right after (rolling prefetch)
    float e[kRR];
    const uint32_t offn = lane_off(nxt);
#pragma unroll
    for (int i = 0; i < kRR; ++i) {
      const f4 t = x[i] - gv;
      e[i] = fmaf(t[3], t[3], fmaf(t[2], t[2], fmaf(t[1], t[1], t[0] * t[0])));
      // e[i] exists HERE (not sunk to its use in transpose_reduce), so row i's registers
      // are free before its next load: otherwise both tiles are live and spill
      asm volatile("" : "+v"(e[i])::"memory");
      __builtin_amdgcn_sched_barrier(0);
      load(offn, x[i], i);
    }
    fetch_gold(nxt);
    // the 8 lanes of a row segment (lane bits 0-2): halving steps on DPP partners, lane c
    // ends with row row_of_lane<8, 8>(c) (xlane_transpose64's scheme for the low bits)
    sfor<0, 3>([&](auto step) {
      constexpr int half = kRR >> (step + 1);
      constexpr int o = 4 >> step;
      const unsigned m = (c & o) ? 0xffffffffu : 0u;
      sfor<0, half>([&](auto i) {
        const unsigned lo = __float_as_uint(e[i]), hi = __float_as_uint(e[i + half]);
        const unsigned x = (lo ^ hi) & m;
        e[i] = __uint_as_float(lo ^ x) + xlane_partner<o>(__uint_as_float(hi ^ x));
      });
    });
    row_acc += (double)e[0];
  }

  // per-block partials -> slab row: [D2 (K)] [r (K), INIT: 0 here, gm2] [mv2] [gn2]
  double* out = a.slab + (int64_t)blockIdx.x * a.slab_stride;
  const int64_t k = rg + (int64_t)kRG * row_of_lane<kRL, kRR>(c);
  if (k < K) {
    out[k] = row_acc;
    if constexpr (INIT) out[K + k] = 0.0;
  }
  __syncthreads();
  if (tid == 0) {
    double m = 0.0, g = 0.0;
    for (int j = 0; j < kRJ; ++j) {
      m += s_acc[0][j];
      g += s_acc[1][j];
    }
    const int64_t b = INIT ? 2 * K : K;
    out[b] = m;
    out[b + 1] = g;
  }
}

// GMAGG_ROWS_LEAN (read per call): 1 (default) this kernel for the row-major gm2 STEP passes,
// 2 the INIT pass too, 0 the generic stream_pass tile (A/B, tests)
static bool rows_lean_on() {
  const char* e = getenv("GMAGG_ROWS_LEAN");
  return e ? atoi(e) != 0 : true;
}

bool rows_pass_eligible(const PassArgs& a, int mode) {
  // STEP only: the INIT pass stays on the generic tile so that gm2 with the fused OMA
  // pre-noise (INIT mode 4, generic) and OMA followed by gm2 (INIT mode 1) keep computing the
  // initial distances identically — the fused form equals the separate one bit for bit
  // (tests/test_gpu_weiszfeld.py); the INIT template stays built for A/B (GMAGG_ROWS_LEAN=2)
  const char* e = getenv("GMAGG_ROWS_LEAN");
  const bool init_too = e && atoi(e) == 2;
  return rows_lean_on() && a.panel_stride == 0 && a.noise == 0 &&
         (mode == 0 || (mode == 1 && init_too)) &&
         a.K > 512 && a.K <= kRG * kRR && a.d % 4 == 0 && a.ldx % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(a.X) & 15) == 0 &&
         // a group's 8 rows (the resource's size) below 2^31 bytes, so the out-of-range lane
         // offset 0x80000000 is past every resource and reads 0
         (uint64_t)a.ldx * kRQ * 4u < (1ull << 31);
}

hipError_t launch_rows_pass(int mode, int grid, const PassArgs& a, hipStream_t s) {
  void* args[] = {const_cast<PassArgs*>(&a)};
  const void* fn = mode == 1 ? reinterpret_cast<const void*>(&rows_pass<true>)
                             : reinterpret_cast<const void*>(&rows_pass<false>);
  return hipLaunchKernel(fn, dim3(grid), dim3(kRW * 64), args, 0, s);
}

}  // namespace gmk
