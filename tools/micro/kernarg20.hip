// Probe: does a kernel take a ~20 KiB by-value argument (the codec job with 64 transform blocks
// is 18.7 KB)?  The output pointer comes first, so a truncated argument copy shows up as a wrong
// sum, never as a wild address.  Prints the sum read back from the device.
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big { unsigned v[5120]; };
__global__ void k(unsigned* out, const Big b) {
  unsigned s = 0;
  for (int i = threadIdx.x; i < 5120; i += 64) s += b.v[i];
  atomicAdd(out, s);
}
int main() {
  static Big b;
  unsigned want = 0;
  for (int i = 0; i < 5120; ++i) { b.v[i] = i * 3 + 1; want += b.v[i]; }
  unsigned* d;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, b);
  hipError_t e = hipDeviceSynchronize();
  unsigned got = 0;
  hipMemcpy(&got, d, 4, hipMemcpyDeviceToHost);
  printf("kernarg 20 KiB: %s got %u want %u\n", hipGetErrorString(e), got, want);
  return got == want ? 0 : 2;
}
