// Probe: does a process that made ONE cooperative launch crash at exit under
// rocprofv3 --kernel-trace, with none of this library loaded?  (C2's resident kernel
// is the only cooperative launch of the build; the C2 bench segfaulted inside the HIP
// runtime's exit handler -> ROCr teardown under rocprofv3, the C3 bench did not:
// profiles/history/r3s2_c2_exit_crash.txt.)
//
//   hipcc --offload-arch=gfx950 -O2 tools/coop_exit_probe.hip -o tools/coop_exit_probe
//   rocprofv3 --kernel-trace --stats -d gpurun_out/x -- ./tools/coop_exit_probe [coop|plain]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void probe_kernel(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = (int)blockIdx.x;
}

int main(int argc, char** argv) {
  const bool coop = argc < 2 || strcmp(argv[1], "plain") != 0;
  int* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
  void* args[] = {&d};
  const hipError_t e = coop ? hipLaunchCooperativeKernel((const void*)probe_kernel, dim3(32),
                                                          dim3(256), args, 0, nullptr)
                            : hipLaunchKernel((const void*)probe_kernel, dim3(32), dim3(256),
                                              args, 0, nullptr);
  if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "launch failed: %s\n", hipGetErrorString(e));
    return 3;
  }
  int h[32];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  hipFree(d);
  printf("%s launch ok (block 31 wrote %d); exiting\n", coop ? "cooperative" : "plain", h[31]);
  return 0;
}
