// Small device helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace gmk {

template <int V> struct vec;
template <> struct vec<1> { typedef float t; };
template <> struct vec<2> { typedef float t __attribute__((ext_vector_type(2))); };
template <> struct vec<4> { typedef float t __attribute__((ext_vector_type(4))); };

// V consecutive floats, streamed (non-temporal: X is read once per pass and
// must not evict the small re-read state from L2).
template <int V>
__device__ __forceinline__ void load_cols(const float* __restrict__ p, float (&o)[V]) {
  if constexpr (V == 1) {
    o[0] = __builtin_nontemporal_load(p);
  } else {
    typedef typename vec<V>::t T;
    T v = __builtin_nontemporal_load(reinterpret_cast<const T*>(p));
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = v[i];
  }
}

// V consecutive floats at byte offset `off` from the wave-uniform `base`, through
// a raw buffer resource (offsets >= nrec read 0),
// streamed (slc).  One VGPR of address per load instead of a 64-bit pointer.
// `nrec` = the resource's size in bytes (offsets >= nrec read 0).
template <int V>
__device__ __forceinline__ void load_rows(const float* base, uint32_t off, float (&o)[V],
                                          int nrec = 0x7fffffff) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, nrec, 0x00020000);
  if constexpr (V == 4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2));
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = v[i];
  } else if constexpr (V == 2) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 2));
    o[0] = v[0];
    o[1] = v[1];
  } else {
    o[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 2));
  }
}

template <int A, int B> struct cmin { static constexpr int v = A < B ? A : B; };
template <int N> struct ilog2 { static constexpr int v = 1 + ilog2<N / 2>::v; };
template <> struct ilog2<1> { static constexpr int v = 0; };

// Reduce R per-row values across the LPR lanes of a row segment so that each
// lane ends up holding complete row sums ("transpose-reduce"): halving
// butterfly steps (each lane keeps the half of its registers selected by its
// lane bit and adds the partner's other half), then plain butterflies over
// any lane bits left.  Afterwards lane c holds RPL = max(1, R/LPR) row sums in
// e[0..RPL); slot m is row row_of_lane<LPR,R>(c) + m.  ~R shuffles for R rows.
template <int LPR, int R>
__device__ __forceinline__ void transpose_reduce(float (&e)[R], int c) {
  constexpr int STEPS = cmin<ilog2<R>::v, ilog2<LPR>::v>::v;
#pragma unroll
  for (int step = 0; step < STEPS; ++step) {
    const int half = R >> (step + 1);
    const int o = LPR >> (step + 1);
    const bool up = (c & o) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      float keep = up ? e[i + half] : e[i];
      float send = up ? e[i] : e[i + half];
      e[i] = keep + __shfl_xor(send, o, 64);
    }
  }
  if constexpr (R < LPR) {
#pragma unroll
    for (int o = LPR / (2 * R); o >= 1; o >>= 1) e[0] += __shfl_xor(e[0], o, 64);
  }
}

template <int LPR, int R>
__device__ __forceinline__ int row_of_lane(int c) {
  constexpr int STEPS = cmin<ilog2<R>::v, ilog2<LPR>::v>::v;
  int i = 0;
#pragma unroll
  for (int step = 0; step < STEPS; ++step)
    if (c & (LPR >> (step + 1))) i += R >> (step + 1);
  return i;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the block (blockDim.x a multiple of 64, <= 1024); every thread gets it.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += scratch[i];
  return s;
}

// dist = max(1e-4, ||x_k - g||) in fp32 with torch.max's NaN propagation (M:178)
__device__ __forceinline__ float clamp_dist(double d2, float eps) {
  const float dist = (float)sqrt(d2);
  return dist != dist ? dist : fmaxf(dist, eps);
}


// ---------------------------------------------------------------------------
// gfx950 cross-lane moves without LDS (round 3, resident_batched.hip):
// v_permlane32_swap / v_permlane16_swap and DPP instead of ds_bpermute (__shfl_xor), an
// LDS round trip per shuffle.

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

// transpose_reduce<64, R> (device_util.h) on gfx950's cross-lane moves instead of
// ds_bpermute (an LDS round trip per shuffle, ~70 of them in a chain per 50 rows):
//   bit 5: v_permlane32_swap of the pair (e[i], e[i + R/2]) IS the halving step (the low
//          half of the lanes ends with both lanes' e[i], the high half with both lanes'
//          e[i + R/2]), then one add;
//   bit 4: v_permlane16_swap likewise (odd 16-lane rows of one register swapped with the
//          even rows of the other);
//   bits 3, 2: the keep / send choice on the bits (x ^ ((x ^ y) & m): written as selects,
//          the compiler turned them into selects of ARRAY INDICES and every use of e[]
//          into a compare / v_cndmask chain), and the partner's value through DPP
//          row_mirror (lane c ^ 15) / row_half_mirror (c ^ 7): the partner differs in the
//          keep bit and shares the bits above it, so each lane still sums disjoint lane
//          sets; bits 1, 0: DPP quad_perm (c ^ 2, c ^ 1).
// Lane c ends with row row_of_lane<64, R>(c) summed over the 64 lanes, as transpose_reduce.
template <int CTRL>
__device__ __forceinline__ float xlane_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int O>
__device__ __forceinline__ float xlane_partner(float v) {   // lane c's partner across bit O
  if constexpr (O == 8) return xlane_dpp<0x140>(v);         // row_mirror: c ^ 15
  else if constexpr (O == 4) return xlane_dpp<0x141>(v);    // row_half_mirror: c ^ 7
  else if constexpr (O == 2) return xlane_dpp<0x4E>(v);     // quad_perm [2,3,0,1]
  else return xlane_dpp<0xB1>(v);                           // quad_perm [1,0,3,2]
}
template <int R>
__device__ __forceinline__ void xlane_transpose64(float (&e)[R], int c) {
  constexpr int STEPS = ilog2<R>::v;
  sfor<0, STEPS>([&](auto step) {
    constexpr int half = R >> (step + 1);
    constexpr int o = 32 >> step;
    if constexpr (o >= 16) {
      sfor<0, half>([&](auto i) {
        const auto r = o == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(e[i]),
                                                                  __float_as_uint(e[i + half]),
                                                                  false, false)
                               : __builtin_amdgcn_permlane16_swap(__float_as_uint(e[i]),
                                                                  __float_as_uint(e[i + half]),
                                                                  false, false);
        e[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      });
    } else {
      const unsigned m = (c & o) ? 0xffffffffu : 0u;
      sfor<0, half>([&](auto i) {
        const unsigned lo = __float_as_uint(e[i]), hi = __float_as_uint(e[i + half]);
        const unsigned x = (lo ^ hi) & m;
        e[i] = __uint_as_float(lo ^ x) + xlane_partner<o>(__uint_as_float(hi ^ x));
      });
    }
  });
  // the lane bits below the halving steps: plain butterflies
  constexpr int O0 = 64 / (2 * R);
  if constexpr (O0 >= 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(e[0]), __float_as_uint(e[0]),
                                                    false, false);
    e[0] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if constexpr (O0 >= 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(e[0]), __float_as_uint(e[0]),
                                                    false, false);
    e[0] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if constexpr (O0 >= 8) e[0] += xlane_partner<8>(e[0]);
  if constexpr (O0 >= 4) e[0] += xlane_partner<4>(e[0]);
  if constexpr (O0 >= 2) e[0] += xlane_partner<2>(e[0]);
  if constexpr (O0 >= 1) e[0] += xlane_partner<1>(e[0]);
}

// fp64 sum over the wave, every lane the same bits (each butterfly level adds the same two
// values in both lanes): the cross-lane moves of xlane_transpose64 on both 32-bit halves
__device__ __forceinline__ double xlane_wave_sum(double v) {
  auto swap_add = [&](auto swap) {
    const uint64_t b = __double_as_longlong(v);
    const auto lo = swap((unsigned)b), hi = swap((unsigned)(b >> 32));
    const double a0 = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
    const double a1 = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
    v = a0 + a1;
  };
  swap_add([](unsigned x) { return __builtin_amdgcn_permlane32_swap(x, x, false, false); });
  swap_add([](unsigned x) { return __builtin_amdgcn_permlane16_swap(x, x, false, false); });
  auto part = [&](auto ctrl) {
    const uint64_t b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, ctrl(), 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), ctrl(), 0xf, 0xf, false);
    v += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  };
  part([] { return 0x140; });   // row_mirror
  part([] { return 0x141; });   // row_half_mirror
  part([] { return 0x4E; });    // quad_perm [2,3,0,1]
  part([] { return 0xB1; });    // quad_perm [1,0,3,2]
  return v;
}

// fp32 sum over the wave, every lane the same bits (the pairings of xlane_wave_sum)
__device__ __forceinline__ float xlane_wave_sum_f32(float v) {
  auto sw = [&](auto r) { v = __uint_as_float(r[0]) + __uint_as_float(r[1]); };
  sw(__builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false));
  sw(__builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false));
  v += xlane_partner<8>(v);
  v += xlane_partner<4>(v);
  v += xlane_partner<2>(v);
  v += xlane_partner<1>(v);
  return v;
}

// Co-residency check-in of a plain-launched persistent grid (resident.hip,
// resident_batched.hip), before a block reads or writes anything of the problem: block
// b stores the tag into ci[slot] (slot = its logical index); every block then waits,
// bounded by `ticks` of the 100 MHz
// real-time clock, until slots [0, need) all carry it (need = the grid's block count;
// GMAGG_RES_CHECKIN_FAIL makes it one more, a slot nobody writes, to test the fallback).
// A grid that is not co-resident (a shared GPU, CUs held by another stream's kernel)
// fails here within `ticks`, with X untouched, instead of in an iteration's 2 s poll:
// the first block to give up raises *tmo (the kernel's timeout word), and every block —
// including one that only starts after the others left and finds every slot written —
// then returns.  A block that passes raises *passed before touching X, so the host can
// tell the two cases apart.  `s_ok`: the block's shared pass / fail word.
constexpr unsigned kCheckinTag = 0xC0DEC0DEu;
constexpr uint64_t kCheckinTicks = 10000000ull;   // 100 ms

// The XCD this wave runs on (0-7): hardware register XCC_ID.
__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg(20 | (0 << 6) | ((4 - 1) << 11)) & 7u;   // hwreg(XCC_ID, 0, 4)
}

// s_same (optional): every slot in [same_lo, same_hi) carries this block's XCD (each block
// writes xcc_id() + 1 into its slot's low word), i.e. those blocks share one L2; read from
// the same slots by every block of the range, so the range's blocks agree on it.
__device__ __forceinline__ bool grid_checkin(unsigned long long* ci, unsigned slot, unsigned need,
                                             unsigned* tmo_word, unsigned* passed,
                                             uint64_t ticks, int* s_ok, int* s_same = nullptr,
                                             unsigned same_lo = 0, unsigned same_hi = 0) {
  typedef __attribute__((address_space(1))) unsigned long long gu64_t;
  typedef __attribute__((address_space(1))) unsigned gu32_t;
  gu64_t* c = (gu64_t*)ci;
  gu32_t* tmo = (gu32_t*)tmo_word;
  const unsigned tid = threadIdx.x;
  const unsigned mine = xcc_id() + 1u;
  if (tid == 0) {
    *s_ok = 1;
    if (s_same) *s_same = 1;
    __hip_atomic_store(c + slot, ((unsigned long long)kCheckinTag << 32) | mine, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  bool ok = true, same = true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned b = tid; ok && b < need; b += blockDim.x) {
    for (unsigned spins = 0;; ++spins) {
      const unsigned long long v = __hip_atomic_load(c + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(v >> 32) == kCheckinTag) {
        if (b >= same_lo && b < same_hi && (unsigned)v != mine) same = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      if (((spins & 63u) == 63u && __builtin_amdgcn_s_memrealtime() - t0 > ticks) ||
          __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
  }
  if (!ok) *s_ok = 0;
  if (!same && s_same) *s_same = 0;
  __syncthreads();
  if (tid == 0 && *s_ok && __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    *s_ok = 0;                       // every slot written, but the grid already gave up
  __syncthreads();
  const bool pass = *s_ok != 0;
  if (tid == 0 && pass)
    __hip_atomic_store((gu32_t*)passed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_s_waitcnt(0);     // the flag stores complete before the block leaves
  return pass;
}

}  // namespace gmk
