// Small device helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

}  // namespace gmk
