// Layout / block-mapping probe for the C3 streaming pass (K=1000 x d=11M fp32).
// The pass's exact thread map (NW waves, LPR lanes x 16 B per row segment, R
// rows per thread, grid-strided chunks of J = 4*LPR columns x all K rows)
// reading, without arithmetic, from:
//   rm     row-major [K][ldx] (the drop-in layout), ldx = d or padded
//   xcd    row-major, chunks remapped so each XCD streams one contiguous
//          d/8 column range (blocks are dispatched round-robin over 8 XCDs)
//   panel  column panels [nch][K][J]: one chunk = one contiguous K*J*4 bytes
// Prints GB/s (algorithmic bytes K*d*4 / time).
//
//   hipcc -O3 --offload-arch=gfx950 tools/hbm_probe2.hip -o build/hbm_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// element (k, j) of chunk ch at X + ch*ps + k*rs + (j - ch*J)
template <int NW, int LPR, int R, int MAP>
__global__ void __launch_bounds__(NW * 64) tile_read(const float* __restrict__ X, int K, long d,
                                                     long rs, long ps, float* sink) {
  constexpr int QW = 64 / LPR, NRG = NW * QW, J = LPR * 4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane % LPR, q = lane / LPR, rg = w * QW + q;
  const long nch = (d + J - 1) / J;
  long ch0 = blockIdx.x, step = gridDim.x, lo = 0, hi = nch;
  if (MAP == 1) {   // XCD x = blockIdx % 8 owns chunks [x*nch/8, (x+1)*nch/8)
    const int x = blockIdx.x & 7;
    const long per = (nch + 7) / 8;
    lo = x * per;
    hi = lo + per < nch ? lo + per : nch;
    ch0 = lo + (blockIdx.x >> 3);
    step = gridDim.x >> 3;
  }
  float acc = 0.f;
  for (long ch = ch0; ch < hi; ch += step) {
    f4 v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int k = rg + NRG * i;
      v[i] = (k < K) ? __builtin_nontemporal_load(
                           reinterpret_cast<const f4*>(X + ch * ps + (long)k * rs + c * 4))
                     : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < R; ++i) acc += v[i].x + v[i].y + v[i].z + v[i].w;
  }
  (void)lo;
  if (acc == 1234.5f) *sink = acc;
}

template <int NW, int LPR, int R, int MAP>
static double run(const float* X, int K, long d, long rs, long ps, float* sink, int blocks) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL((tile_read<NW, LPR, R, MAP>), dim3(blocks), dim3(NW * 64), 0, 0, X, K, d, rs,
                     ps, sink);
  CHK(hipDeviceSynchronize());
  const int reps = 5;
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((tile_read<NW, LPR, R, MAP>), dim3(blocks), dim3(NW * 64), 0, 0, X, K, d,
                       rs, ps, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  return (double)K * d * 4.0 * reps / (ms * 1e-3) / 1e9;
}

int main() {
  const int K = 1000;
  const long d = 11000000;
  const long ldx_max = d + 4096;
  float* X;
  float* sink;
  CHK(hipMalloc(&X, (size_t)K * ldx_max * 4 + (1 << 20)));
  CHK(hipMalloc(&sink, 4));
  CHK(hipMemset(X, 0, (size_t)K * ldx_max * 4 + (1 << 20)));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    for (int bpc : {2, 3, 4}) {
      const int bl = cus * bpc;
      printf("bpc=%d 512thr J=32 (8,8,16): rm %.0f  rm+32 %.0f  rm+1024 %.0f  rm+4096 %.0f  xcd %.0f  panel %.0f GB/s\n",
             bpc, run<8, 8, 16, 0>(X, K, d, d, 32, sink, bl),
             run<8, 8, 16, 0>(X, K, d, d + 32, 32, sink, bl),
             run<8, 8, 16, 0>(X, K, d, d + 1024, 32, sink, bl),
             run<8, 8, 16, 0>(X, K, d, d + 4096, 32, sink, bl),
             run<8, 8, 16, 1>(X, K, d, d, 32, sink, bl),
             run<8, 8, 16, 0>(X, K, d, 32, (long)K * 32, sink, bl));
      printf("bpc=%d 512thr J=64 (8,16,32): rm %.0f  xcd %.0f  panel %.0f GB/s\n", bpc,
             run<8, 16, 32, 0>(X, K, d, d, 64, sink, bl),
             run<8, 16, 32, 1>(X, K, d, d, 64, sink, bl),
             run<8, 16, 32, 0>(X, K, d, 64, (long)K * 64, sink, bl));
    }
    for (int bpc : {1, 2}) {
      const int bl = cus * bpc;
      printf("bpc=%d 1024thr J=32 (16,8,8): rm %.0f  xcd %.0f  panel %.0f GB/s\n", bpc,
             run<16, 8, 8, 0>(X, K, d, d, 32, sink, bl),
             run<16, 8, 8, 1>(X, K, d, d, 32, sink, bl),
             run<16, 8, 8, 0>(X, K, d, 32, (long)K * 32, sink, bl));
    }
  }
  return 0;
}
