// Does a launch with 4.8 KB of kernel arguments run (a one-frame launch at N = 1024 would carry 4,096 bytes
// of samples after the 432-byte KernelArgs)? Prints the launch status and the argument word read back.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ubench/kernarg_size tools/ubench/kernarg_size.hip
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big {
  float f[1200];
  int n;
};
__global__ void k(Big b, float* out) {
  if (threadIdx.x == 0) out[0] = b.f[b.n];
}
int main() {
  Big b;
  for (int i = 0; i < 1200; ++i) b.f[i] = (float)i;
  b.n = 1100;
  float* d = nullptr;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, b, d);
  const hipError_t e = hipGetLastError();
  float h = -1;
  const hipError_t e2 = hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("{\"kernarg_bytes\": %zu, \"launch\": \"%s\", \"copy\": \"%s\", \"value\": %g}\n", sizeof(Big), hipGetErrorString(e),
         hipGetErrorString(e2), h);
  return e == hipSuccess && e2 == hipSuccess && h == 1100.0f ? 0 : 1;
}
