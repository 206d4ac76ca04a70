// Counter-based Philox4x32-10 + Box-Muller normals for the AirComp channel.
//
// Every draw is a pure function of (seed, stream, iteration, global index), so
// d-shards regenerate identical channel coefficients h_k and identical noise
// columns without communicating, and a launch can be replayed.  Streams keep
// the reference's draw families apart (OMA2 M:401-402 / M:411, OMA M:389-392).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gmk {

enum : uint32_t {
  kStreamChannel = 0x43484E4Cu,   // OMA2 h_re/h_im per client, per iteration
  kStreamNoise = 0x4E4F4953u,     // OMA2 additive noise per column, per iteration
  kStreamOmaChannel = 0x4F4D4143u,
  kStreamOmaNoise = 0x4F4D414Eu,
  kStreamFill = 0x46494C4Cu,      // synthetic client updates
};

struct u4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

// Philox4x32 with 10 rounds (Salmon et al., SC'11).
__host__ __device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c.x, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, &hi1);
#ifdef __HIP_DEVICE_COMPILE__
    // gfx950's three-input bitwise op (truth table 0x96 = a ^ b ^ c): one VALU
    // instruction per word instead of two v_xor_b32 (the compiler selects no bitop3
    // for a ^ b ^ c itself); the same bits
    c = u4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
           (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
#else
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
#endif
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// (0, 1] uniform from 32 random bits, never 0 so log() is finite.
__host__ __device__ __forceinline__ float u01(uint32_t v) {
  return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Two independent standard normals from two uniform words (Box-Muller).
__host__ __device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float* n0, float* n1) {
  float r = sqrtf(-2.0f * logf(u01(a)));
  float t = 6.283185307179586f * u01(b);
  float s, c;
#ifdef __HIP_DEVICE_COMPILE__
  __sincosf(t, &s, &c);
#else
  s = sinf(t); c = cosf(t);
#endif
  *n0 = r * c;
  *n1 = r * s;
}

// Four standard normals for counter (idx, iter) on `stream`.
__host__ __device__ __forceinline__ void normal4(uint64_t seed, uint32_t stream, uint64_t iter,
                                                 uint64_t idx, float out[4]) {
  u4 c{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)iter, stream ^ (uint32_t)(iter >> 32)};
  u4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller(r.x, r.y, &out[0], &out[1]);
  box_muller(r.z, r.w, &out[2], &out[3]);
}

// Box-Muller on the hardware transcendentals: v_log_f32 (log2), v_sqrt_f32 and
// v_sin/v_cos_f32, which take their argument in revolutions, so u01(b) goes in
// unscaled.  ~1 ulp each; contraction off so every DEVICE call site rounds alike
// (a normal must come out identical whichever kernel regenerates it).  Host code
// has no equivalent: the CPU restatement (oracle/philox.py) uses libm-precision
// Box-Muller and is compared with a tolerance, never bit for bit.
__device__ __forceinline__ void box_muller_hw(uint32_t a, uint32_t b, float* n0, float* n1) {
#pragma clang fp contract(off)
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(a)));
  const float t = u01(b);
  *n0 = r * __builtin_amdgcn_cosf(t);
  *n1 = r * __builtin_amdgcn_sinf(t);
}

// normal4 with the hardware Box-Muller (the OMA production path).
__device__ __forceinline__ void normal4_hw(uint64_t seed, uint32_t stream, uint64_t iter,
                                           uint64_t idx, float out[4]) {
  u4 c{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)iter, stream ^ (uint32_t)(iter >> 32)};
  u4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller_hw(r.x, r.y, &out[0], &out[1]);
  box_muller_hw(r.z, r.w, &out[2], &out[3]);
}

// OMA (M:385-394) with Philox draws: client k's equalisation scale sd / |h_k|, h_k ~ CN(0, 1)
// from the block keyed (row k), and the noisy element x + scale * z.  Contraction off:
// the standalone OMA kernel and the OMA fused into a streaming pass run these same two
// functions, so their results are identical bit for bit.
__device__ __forceinline__ float oma_row_scale(uint64_t seed, uint64_t k, float sd) {
#pragma clang fp contract(off)
  float h[4];
  normal4_hw(seed, kStreamOmaChannel, 0, k, h);
  const float a = h[0] * 0.70710678118654752f, b = h[1] * 0.70710678118654752f;
  return sd / sqrtf(a * a + b * b);
}
__device__ __forceinline__ float oma_noisy(float x, float scale, float z) {
#pragma clang fp contract(off)
  return x + scale * z;
}

// One standard normal for element `idx`: normal idx & 3 of the Philox block (iter, idx >> 2)
// on the hardware Box-Muller — four consecutive elements share a block, as in the fill and
// OMA draws (round 4 session 2; before, one block per element, normal 0: the batched
// resident kernel's four columns per thread then took four blocks per iteration; C5 AirComp
// 773.8 -> 803.6 problems/s, profiles/r4s2_c5air_draws_ab.jsonl).  The AirComp column noise
// and the denominator's draw (element d_total).  Device-only: every call site that
// regenerates a draw runs this same code, so a draw is identical wherever it is made.
__device__ __forceinline__ float normal1(uint64_t seed, uint32_t stream, uint64_t iter,
                                         uint64_t idx) {
  float z[4];
  normal4_hw(seed, stream, iter, idx >> 2, z);
  const unsigned e = (unsigned)(idx & 3u);
  return e == 0 ? z[0] : e == 1 ? z[1] : e == 2 ? z[2] : z[3];
}

}  // namespace gmk
