// Probe: does a kernel take an 8 KiB by-value argument on this stack?  (the codec job would
// grow to ~7.4 KB with 32 transform blocks).  Prints the sum read back from the device.
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big { unsigned v[2048]; };
__global__ void k(const Big b, unsigned* out) {
  unsigned s = 0;
  for (int i = threadIdx.x; i < 2048; i += 64) s += b.v[i];
  atomicAdd(out, s);
}
int main() {
  Big b;
  unsigned want = 0;
  for (int i = 0; i < 2048; ++i) { b.v[i] = i * 3 + 1; want += b.v[i]; }
  unsigned* d;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, b, d);
  hipError_t e = hipDeviceSynchronize();
  unsigned got = 0;
  hipMemcpy(&got, d, 4, hipMemcpyDeviceToHost);
  printf("kernarg 8 KiB: %s got %u want %u\n", hipGetErrorString(e), got, want);
  return got == want ? 0 : 2;
}
