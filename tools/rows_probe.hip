// Where does the row-major C3 read lose against the panel layout?  
//
// The STEP pass's exact tile (8 waves, 8 lanes x 16 B per row segment, 16 rows per
// thread: a chunk of J = 32 columns x all K = 1000 rows, grid-strided, 2 blocks per CU)
// reading, without arithmetic, a K x d = 1000 x 11M fp32 matrix stored as column panels of
// width W: element (k, c) at X + (c / W) * K * W + k * W + (c % W).
//   W = 32      the ClientPanels layout (a chunk is one contiguous 128 KB block)
//   W = d       the reference's row-major [K, d] stack (rows 44 MB apart)
// and the widths between.  Every variant reads the same 44 GB in the same chunk order;
// only the distance between a chunk's rows changes (W * 4 bytes).  If the loss appears
// once rows sit in different 2 MB pages (W >= 512K), translation reach is the bound; if it
// grows with W from the start, DRAM page locality is.
//
//   hipcc -O3 --offload-arch=gfx950 tools/rows_probe.hip -o build/rows_probe
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

template <int NW, int LPR, int R>
__global__ void __launch_bounds__(NW * 64) panel_read(const float* __restrict__ X, int K, long d,
                                                      long W, float* sink) {
  constexpr int QW = 64 / LPR, NRG = NW * QW, J = LPR * 4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane % LPR, q = lane / LPR, rg = w * QW + q;
  const long nch = d / J;
  float acc = 0.f;
  for (long ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const long col = ch * J + c * 4;
    const float* base = X + (col / W) * (long)K * W + (col % W);
    f4 v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int k = rg + NRG * i;
      v[i] = (k < K) ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(base + (long)k * W))
                     : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < R; ++i) acc += v[i].x + v[i].y + v[i].z + v[i].w;
  }
  if (acc == 1234.5f) *sink = acc;
}

static double run(const float* X, int K, long d, long W, float* sink, int blocks) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL((panel_read<8, 8, 16>), dim3(blocks), dim3(512), 0, 0, X, K, d, W, sink);
  CHK(hipDeviceSynchronize());
  const int reps = 5;
  CHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((panel_read<8, 8, 16>), dim3(blocks), dim3(512), 0, 0, X, K, d, W, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  return (double)K * d * 4.0 * reps / (ms * 1e-3) / 1e9;
}

int main() {
  const int K = 1000;
  const long d = 21L << 19;                   // 11,010,048: C3's width, divisible by 2^19
  float* X;
  float* sink;
  CHK(hipMalloc(&X, (size_t)K * d * 4));
  CHK(hipMalloc(&sink, 4));
  CHK(hipMemset(X, 0, (size_t)K * d * 4));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const long widths[] = {32, 256, 2048, 16384, 131072, 524288, 7L << 19, d};
  for (int rep = 0; rep < 2; ++rep)
    for (long W : widths) {
      if (d % W) continue;
      printf("{\"probe\": \"rows_probe\", \"W\": %ld, \"row_gap_bytes\": %ld, \"GBps\": %.0f}\n", W,
             W * 4, run(X, K, d, W, sink, 2 * cus));
      fflush(stdout);
    }
  return 0;
}
