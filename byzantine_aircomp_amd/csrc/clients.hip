// The K simulated clients' local SGD steps of one federated step, as ONE kernel
// (with the aggregation on the GPU, the reference's sequential
// client loop — K tiny forward/backward passes driven from Python, M:291-343 — is
// what a training step costs).
//
// Reference semantics kept exactly (MNIST_Air_weight.py):
//   * the model is the linear softmax classifier MLP(784, C) (M:53-61) trained with
//     CrossEntropyLoss (mean over the batch, M:573) and plain SGD
//     p <- p - gamma * (grad + weight_decay * p)  (M:302-303 / M:339-340);
//   * the clients run IN SEQUENCE on one model: modelSnapshot returns the state_dict,
//     which aliases the parameters, so "modelRecovery" restores nothing and client k
//     starts from client k-1's updated weights (M:290, M:343) — a chain, so the K steps
//     cannot run as independent batched gradients;
//   * Byzantine clients (node >= honest) train on 1 - x (dataflip, M:326) or on the
//     relabelled C-1-y (classflip, M:320; EMNIST 61-y, E:321);
//   * client k's updated parameters become row k of the client matrix in
//     model.parameters() order (weight [C][F] row-major, then bias [C]: flatten_list,
//     M:206-209), written straight into the aggregator's input (rows or panels).
// After the call W / b hold the last client's parameters, which the reference's loop
// passes as the aggregator's guess (M:349).
//
// One workgroup of 512 threads (8 waves, up to 256 VGPRs each) walks the chain.  Per
// client:
//   A  logits z[s][c] = x_s . W_c + b_c: wave w owns samples s = w + 8 i (the batch
//      tile stays in its registers), its lanes the features f = lane + 64 j; per group
//      of 4 classes each lane accumulates the 8 x 4 partial dots over its features, one
//      transpose-reduce over the wave's 64 lanes completes them (one shuffle per value
//      instead of six);
//   B  softmax cross-entropy gradient per sample, one wave per sample, lane = class,
//      torch's order: log_softmax, then dz = gout - exp(logp) * sum(gout) with
//      gout = -1/B at the label (nll_loss mean backward);
//   C  thread = features f, f + 512: gW[c][f] = sum_s dz[s][c] x[s][f] (s ascending),
//      the SGD update of column f of W, and the client's row of the client matrix.
// The batch rows are gathered by index from the training set on the device (the
// samplers' index streams are drawn on the host in the reference's order).
#include "device_util.h"
#include "gmagg_internal.h"

namespace gmk {

// Phase A's tile loads at clamped addresses, masked after the load (A/B knob; 0: a branch
// per load, and a wait per row)
#ifndef GMK_CC_CLAMP
#define GMK_CC_CLAMP 1
#endif
// Phase A's class-group loop unrolled at C <= 10 (3 groups of 4; A/B knob).  (Tried: the
// next group's W columns loaded into registers before this group's transpose, or with the
// batch tile: 358 VGPRs spilled)
#ifndef GMK_CC_UNROLL_A
#define GMK_CC_UNROLL_A 1
#endif

constexpr int kCcThreads = 512;
constexpr int kCcWaves = kCcThreads / 64;
constexpr int kCcSpw = 8;        // samples per wave in phase A (B <= 64)
constexpr int kCcCg = 4;         // classes per phase-A group
constexpr int kCcFpt = 2;        // features per thread in phase C
constexpr int kCcNj = 13;        // features per lane in phase A: F <= 832
constexpr int kCcCgC = 16;       // classes per phase-C group (CGC: 10 when C <= 10)
constexpr int kCcMaxC = 64;
// dz row stride for phase C's class groups of CGC (C <= 10 with CGC = 10, else <= 64):
// every column a group reads, rounded up to 16 bytes
__host__ __device__ constexpr int cc_zs(int cgc) { return cgc == 10 ? 12 : 64; }
constexpr int kCcMaxB = kCcWaves * kCcSpw;

__device__ __forceinline__ void put_param(const ClientChainArgs& a, int64_t k, int64_t jj, float v) {
  if (a.pstride > 0)
    a.X[(jj >> a.wshift) * a.pstride + k * ((int64_t)1 << a.wshift) +
        (jj & (((int64_t)1 << a.wshift) - 1))] = v;
  else
    a.X[k * a.ldx + jj] = v;
}

// fp32 max / sum over the wave, every lane the result (gfx950 permlane swaps + DPP, no LDS
// round trips; device_util.h xlane_wave_sum_f32's pairings)
__device__ __forceinline__ float cc_wave_max(float v) {
  auto sw = [&](auto r) { v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])); };
  sw(__builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false));
  sw(__builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false));
  v = fmaxf(v, xlane_partner<8>(v));
  v = fmaxf(v, xlane_partner<4>(v));
  v = fmaxf(v, xlane_partner<2>(v));
  v = fmaxf(v, xlane_partner<1>(v));
  return v;
}

// NJ = features per lane in phase A (F <= 64 * NJ).  Dynamic LDS: the client's batch tile
// x[B][F] (phase A stages it, phase C reads it instead of re-reading the rows from L2 per
// sample), when B * F * 4 bytes fit (a.stage); else phase C reads global memory.
template <int NJ, int CGC>
__global__ void __launch_bounds__(kCcThreads, 1) client_chain(ClientChainArgs a) {
  __shared__ int s_row[kCcMaxB];                  // dataset rows of the client's batch
  __shared__ int s_lab[kCcMaxB];                  // (relabelled) targets
  __shared__ float s_b[kCcMaxC];                  // the bias, read by phase A's logits
  extern __shared__ float s_dyn[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = (int)a.F, C = (int)a.C, B = (int)a.B;
  const float invB = 1.0f / (float)B;
  // dynamic LDS: the logits, then the gradient dz, [B][ZS] (ZS: phase C's class groups
  // covered, rounded up to 16-byte rows: its dz reads are 128-bit), then the batch tile
  // [B][F] when a.stage
  constexpr int ZS = cc_zs(CGC);
  float* s_z = s_dyn;
  float* s_x = s_dyn + B * ZS;

#ifdef GMK_CC_PROF
  uint64_t prof_[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t prev_ = __builtin_amdgcn_s_memrealtime();
#define CC_T(i) if (tid == 0) { const uint64_t n_ = __builtin_amdgcn_s_memrealtime(); prof_[i] += n_ - prev_; prev_ = n_; }
#else
#define CC_T(i)
#endif
  // the wave's batch tile: samples w + 8 i, features lane + 64 j (rows by the sampler's
  // index, s_row; 0 outside the batch).  (The row indices from LDS: read from global memory,
  // which the kernel also writes, they are vector loads, and each one's wait drained every
  // earlier row's loads: 8 round trips in sequence.)
  float xr[kCcSpw][NJ];
  auto load_tile = [&]() {
    int rows[kCcSpw];
#pragma unroll
    for (int i = 0; i < kCcSpw; ++i) {
      const int s = w + kCcWaves * i;
      rows[i] = s < B ? s_row[s] : 0;
    }
#pragma unroll
    for (int i = 0; i < kCcSpw; ++i) {
      [[maybe_unused]] const int s = w + kCcWaves * i;
      const float* row = a.data + (int64_t)rows[i] * a.ldd;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int f = lane + 64 * j;
#if GMK_CC_CLAMP
        xr[i][j] = row[min(f, F - 1)];   // every load issued, no branch; masked below
#else
        xr[i][j] = (s < B && f < F) ? row[f] : 0.f;
#endif
      }
    }
#if GMK_CC_CLAMP
#pragma unroll
    for (int i = 0; i < kCcSpw; ++i) {
      const bool sv = w + kCcWaves * i < B;
#pragma unroll
      for (int j = 0; j < NJ; ++j) xr[i][j] = (sv && lane + 64 * j < F) ? xr[i][j] : 0.f;
    }
#endif
  };
  for (int64_t k = 0; k < a.K; ++k) {
    const bool byz = k >= a.honest;
    const bool flip_x = byz && a.attack == 2;
    if (tid < B) {
      const int r = a.idx[k * B + tid];
      s_row[tid] = r;
      const int y = (int)a.labels[r];
      s_lab[tid] = (byz && a.attack == 1) ? (C - 1 - y) : y;
    }
    if (tid < C) s_b[tid] = a.b[tid];
    __syncthreads();
    CC_T(0)

    // ---- A: logits on the batch tile
    load_tile();
    if (flip_x) {
#pragma unroll
      for (int i = 0; i < kCcSpw; ++i) {
        const int s = w + kCcWaves * i;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          if (s < B && lane + 64 * j < F) xr[i][j] = 1.0f - xr[i][j];   // M:326
      }
    }
    if (a.stage) {
#pragma unroll
      for (int i = 0; i < kCcSpw; ++i) {
        const int s = w + kCcWaves * i;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int f = lane + 64 * j;
          if (s < B && f < F) s_x[s * F + f] = xr[i][j];
        }
      }
    }
    CC_T(4)
    auto logits = [&](const int c0) {
      float e[kCcSpw * kCcCg];                            // value i * CG + cc
#pragma unroll
      for (int q = 0; q < kCcSpw * kCcCg; ++q) e[q] = 0.f;
#pragma unroll
      for (int cc = 0; cc < kCcCg; ++cc) {
        const int c = c0 + cc < C ? c0 + cc : C - 1;      // (a padding class repeats C-1)
        const float* wc = a.W + (int64_t)c * F;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int f = lane + 64 * j;
          const float wv = f < F ? wc[f] : 0.f;
#pragma unroll
          for (int i = 0; i < kCcSpw; ++i) e[i * kCcCg + cc] = fmaf(xr[i][j], wv, e[i * kCcCg + cc]);
        }
      }
      xlane_transpose64<kCcSpw * kCcCg>(e, lane);   // (transpose_reduce's lane -> value map)
      // lanes 2v and 2v + 1 hold value row_of_lane(lane) (32 values over 64 lanes)
      if ((lane & 1) == 0) {
        const int v = row_of_lane<64, kCcSpw * kCcCg>(lane);
        const int i = v / kCcCg, cc = v % kCcCg;
        const int s = w + kCcWaves * i, c = c0 + cc;
        if (s < B && c < C) s_z[s * ZS + c] = e[0] + s_b[c];
      }
    };
    if constexpr (GMK_CC_UNROLL_A && CGC == 10) {
#pragma unroll
      for (int g = 0; g < 3; ++g)
        if (g * kCcCg < C) logits(g * kCcCg);
    } else {
      for (int c0 = 0; c0 < C; c0 += kCcCg) logits(c0);
    }
    __syncthreads();
    CC_T(1)

    // ---- B: dz = d mean CE / dz, torch's log_softmax backward order.  C <= 16 (the
    // CGC = 10 kernel): four samples per wave, one 16-lane DPP row each (the 64-lane sums
    // below add exact zeros above lane C, so the bits are the same)
    if constexpr (CGC == 10) {
      const int q = lane >> 4, cl = lane & 15;
      for (int s0 = 4 * w; s0 < B; s0 += 4 * kCcWaves) {
        const int s = s0 + q;
        const bool cv = cl < C && s < B;
        const float z = cv ? s_z[s * ZS + cl] : -INFINITY;
        float m = z;
        m = fmaxf(m, xlane_partner<8>(m));
        m = fmaxf(m, xlane_partner<4>(m));
        m = fmaxf(m, xlane_partner<2>(m));
        m = fmaxf(m, xlane_partner<1>(m));
        float sum = cv ? expf(z - m) : 0.f;
        sum += xlane_partner<8>(sum);
        sum += xlane_partner<4>(sum);
        sum += xlane_partner<2>(sum);
        sum += xlane_partner<1>(sum);
        const float logp = (z - m) - logf(sum);
        const float gout = (cv && cl == s_lab[s]) ? -invB : 0.f;
        if (cv) s_z[s * ZS + cl] = gout - expf(logp) * (-invB);
      }
    } else
    for (int s = w; s < B; s += kCcWaves) {
      const bool cv = lane < C;
      const float z = cv ? s_z[s * ZS + lane] : -INFINITY;
      const float m = cc_wave_max(z);
      const float sum = xlane_wave_sum_f32(cv ? expf(z - m) : 0.f);
      const float logp = (z - m) - logf(sum);
      const float gout = (lane == s_lab[s]) ? -invB : 0.f;
      if (cv) s_z[s * ZS + lane] = gout - expf(logp) * (-invB);
    }
    __syncthreads();
    CC_T(2)

    // ---- C: gradient, SGD update (M:303) and the client's row; thread = 2 features,
    // classes in groups of 16 (the batch columns are re-read per group from L1 / L2)
    for (int c0 = 0; c0 < C; c0 += CGC) {
      // the columns of W this thread updates, loaded before the sample loop (their latency
      // hides behind it; loaded in the update loop they ran one round trip per element,
      // each load ordered after the previous element's store to W): clamped addresses, no
      // branches
      float wold[kCcFpt][CGC];
#pragma unroll
      for (int h = 0; h < kCcFpt; ++h)
#pragma unroll
        for (int cc = 0; cc < CGC; ++cc) {
          const int f = min(tid + kCcThreads * h, F - 1), c = min(c0 + cc, C - 1);
          wold[h][cc] = a.W[(int64_t)c * F + f];
        }
      float g[kCcFpt][CGC], gb[CGC];   // gb: the bias gradient (used by thread 0)
#pragma unroll
      for (int cc = 0; cc < CGC; ++cc) {
        gb[cc] = 0.f;
#pragma unroll
        for (int h = 0; h < kCcFpt; ++h) g[h][cc] = 0.f;
      }
#pragma unroll 2
      for (int s = 0; s < B; ++s) {
        float xv[kCcFpt];
        if (a.stage) {
#pragma unroll
          for (int h = 0; h < kCcFpt; ++h) {
            const int f = tid + kCcThreads * h;
            xv[h] = f < F ? s_x[s * F + f] : 0.f;             // (flipped when staged)
          }
        } else {
          const float* row = a.data + (int64_t)s_row[s] * a.ldd;
#pragma unroll
          for (int h = 0; h < kCcFpt; ++h) {
            const int f = tid + kCcThreads * h;
            xv[h] = f < F ? row[f] : 0.f;
            if (flip_x) xv[h] = 1.0f - xv[h];
          }
        }
#pragma unroll
        for (int cc = 0; cc < CGC; ++cc) {
          const float dz = s_z[s * ZS + c0 + cc];        // (columns >= C: never stored)
          gb[cc] += dz;
#pragma unroll
          for (int h = 0; h < kCcFpt; ++h) g[h][cc] = fmaf(dz, xv[h], g[h][cc]);
        }
      }
      CC_T(5)
#pragma unroll
      for (int h = 0; h < kCcFpt; ++h) {
        const int f = tid + kCcThreads * h;
        if (f < F) {
#pragma unroll
          for (int cc = 0; cc < CGC; ++cc) {
            const int c = c0 + cc;
            if (c < C) {
              const float p = wold[h][cc];
              const float np = fmaf(-a.gamma, g[h][cc] + a.wd * p, p);
              a.W[(int64_t)c * F + f] = np;
              put_param(a, k, (int64_t)c * F + f, np);
            }
          }
        }
      }
      if (tid == 0) {   // the bias: sum over s ascending, as the weights' gradients
#pragma unroll
        for (int cc = 0; cc < CGC; ++cc) {
          const int c = c0 + cc;
          if (c < C) {
            const float p = s_b[c];
            const float np = fmaf(-a.gamma, gb[cc] + a.wd * p, p);
            a.b[c] = np;
            put_param(a, k, (int64_t)C * F + c, np);
          }
        }
      }
      CC_T(6)
    }
    __syncthreads();   // W / b of this client before the next client's reads
    CC_T(3)
  }
#ifdef GMK_CC_PROF
  if (tid == 0)
    printf("GMK_CC_PROF K=%ld ns/client: setup %.0f A-load/stage %.0f A-logits %.0f B %.0f "
           "C-samples %.0f C-update %.0f C-end %.0f\n",
           (long)a.K, 10.0 * prof_[0] / a.K, 10.0 * prof_[4] / a.K, 10.0 * prof_[1] / a.K,
           10.0 * prof_[2] / a.K, 10.0 * prof_[5] / a.K, 10.0 * prof_[6] / a.K,
           10.0 * prof_[3] / a.K);
#endif
}

bool client_chain_supported(int64_t F, int64_t C, int64_t B) {
  return F >= 1 && F <= 64 * kCcNj && F <= kCcThreads * kCcFpt && C >= 1 && C <= kCcMaxC && B >= 1 &&
         B <= kCcMaxB;
}

hipError_t launch_client_chain(const ClientChainArgs& a, hipStream_t s) {
  // 13 features per lane: F <= 832 covers the reference's 28 x 28 inputs (MNIST and
  // EMNIST, F = 784) without idle iterations; 16 per lane spilled 164 VGPRs
  // phase C's class groups: exactly C = 10 for MNIST's classifier (no padding classes: 16
  // computed 6 never stored), 16 otherwise (EMNIST's 62: 4 groups).  Dynamic LDS: dz [B][ZS]
  // and, when it fits beside it in the CU's 160 KB, the batch tile [B][F] (the reference's
  // B = 50 at F = 784: 157 KB + 2.2 KB of dz at C = 10; EMNIST's C = 62 leaves no room)
  constexpr size_t kLdsMax =   // (s_row, s_lab, s_b static)
      (160u << 10) - 2 * kCcMaxB * sizeof(int) - kCcMaxC * sizeof(float);
  auto raise = [](const void* fn) {   // the kernel's dynamic-LDS limit, once per process
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsMax) ==
           hipSuccess;
  };
  static const bool ok10 = raise(reinterpret_cast<const void*>(&client_chain<kCcNj, 10>));
  static const bool ok16 = raise(reinterpret_cast<const void*>(&client_chain<kCcNj, kCcCgC>));
  const bool c10 = a.C <= 10;
  const int cgc = c10 ? 10 : kCcCgC;
  const size_t zs = (size_t)cc_zs(cgc);
  const size_t dz = (size_t)a.B * zs * sizeof(float);
  const size_t tile = (size_t)a.B * (size_t)a.F * sizeof(float);
  ClientChainArgs b = a;
  b.stage = (c10 ? ok10 : ok16) && dz + tile <= kLdsMax ? 1 : 0;
  const size_t lds = dz + (b.stage ? tile : 0);
  if (c10)
    hipLaunchKernelGGL((client_chain<kCcNj, 10>), dim3(1), dim3(kCcThreads), lds, s, b);
  else
    hipLaunchKernelGGL((client_chain<kCcNj, kCcCgC>), dim3(1), dim3(kCcThreads), lds, s, b);
  return hipGetLastError();
}

}  // namespace gmk
