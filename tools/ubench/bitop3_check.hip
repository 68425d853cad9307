#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned s0 = 0xF0F0F0F0u, s1 = 0xCCCCCCCCu, s2 = 0xAAAAAAAAu, r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xAC" : "=v"(r) : "v"(s0), "v"(s1), "v"(s2));
  out[0] = r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xCA" : "=v"(r) : "v"(s0), "v"(s1), "v"(s2));
  out[1] = r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xE2" : "=v"(r) : "v"(s0), "v"(s1), "v"(s2));
  out[2] = r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xB8" : "=v"(r) : "v"(s0), "v"(s1), "v"(s2));
  out[3] = r;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xD8" : "=v"(r) : "v"(s0), "v"(s1), "v"(s2));
  out[4] = r;
}
int main() {
  unsigned* d; hipMalloc(&d, 64); hipLaunchKernelGGL(k, 1, 1, 0, 0, d); unsigned h[5]; hipMemcpy(h, d, 20, hipMemcpyDeviceToHost);
  // s0=F0 s1=CC s2=AA per byte: the truth-table index of bit i is what the result's byte equals for each table
  for (int i = 0; i < 5; ++i) printf("table %d -> %08x\n", i, h[i]);
  return 0;
}
