// Known-size read kernels for calibrating the TCC FETCH_SIZE counter on gfx950: each kernel
// reads exactly `bytes` bytes of a buffer once (no reuse) with one access form, and writes one
// dword per workgroup.  Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and compare the
// per-dispatch counter with the bytes read.
//   read_b32      global_load_dword, 64 lanes x 4 B per wave load
//   read_b128     global_load_dwordx4
//   read_u16      global_load_ushort
//   read_lds_b128 global_load_lds_dwordx4 (LDS-DMA, no VGPR)
//   read_stride   dword loads of 16 B windows spaced 1206 B apart (the leaf hash's access shape:
//                 one lane per symbol, 80 B per symbol per half block), every byte read once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void __launch_bounds__(256) read_b32(const uint32_t* p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
    acc ^= p[i];
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) read_b128(const uint4* p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) read_u16(const uint16_t* p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
    acc ^= p[i];
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) read_lds_b128(const uint4* p, uint64_t n, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[256 * 16];
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(p + i),
                                     (__attribute__((address_space(3))) uint8_t*)(buf + 16 * (threadIdx.x & ~63)),
                                     16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (reinterpret_cast<uint32_t*>(buf)[threadIdx.x] == 0x9E3779B9u) out[blockIdx.x] = 1;
}

// symbols of `s` bytes back to back; lane j of a wave reads 16-byte chunk c of symbol j's
// 80-byte window at byte w (w steps 64 per pass): the leaf hash's LDS window pattern
__global__ void __launch_bounds__(256) read_stride(const uint8_t* p, uint64_t n_sym, int s,
                                                   uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[4 * 64 * 80];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint64_t j0 = (uint64_t(blockIdx.x) * 4 + wv) * 64;
  if (j0 >= n_sym) return;
  const uintptr_t end = reinterpret_cast<uintptr_t>(p) + n_sym * uint64_t(s);
  for (int m = 0; m < s; m += 64) {
    for (int it = 0; it < 5; ++it) {
      const int q = l + 64 * it, jw = q / 5, c = q - jw * 5;
      const uintptr_t a = reinterpret_cast<uintptr_t>(p) + (j0 + jw) * uint64_t(s);
      const uintptr_t src = ((a + uintptr_t(m > 0 ? m - 1 : 0)) & ~uintptr_t(15)) + 16 * c;
      if (j0 + jw < n_sym && src + 16 <= end)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                         (__attribute__((address_space(3))) uint8_t*)(buf + wv * 5120 + 1024 * it),
                                         16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (reinterpret_cast<uint32_t*>(buf)[threadIdx.x] == 0x9E3779B9u) out[blockIdx.x] = 1;
}

int main() {
  const uint64_t bytes = uint64_t(256) << 20;
  uint8_t* d;
  uint32_t* o;
  hipMalloc(&d, bytes + 4096);
  hipMalloc(&o, 1 << 20);
  hipMemset(d, 1, bytes + 4096);
  const int grid = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    read_b32<<<grid, 256>>>((const uint32_t*)d, bytes / 4, o);
    read_b128<<<grid, 256>>>((const uint4*)d, bytes / 16, o);
    read_u16<<<grid, 256>>>((const uint16_t*)d, bytes / 2, o);
    read_lds_b128<<<grid, 256>>>((const uint4*)d, bytes / 16, o);
    const int s = 1206;
    const uint64_t n_sym = bytes / s;
    read_stride<<<unsigned((n_sym + 255) / 256), 256>>>(d, n_sym, s, o);
  }
  hipDeviceSynchronize();
  printf("bytes per kernel: %llu (read_stride: %llu symbols x 1206 B = %llu B)\n",
         (unsigned long long)bytes, (unsigned long long)(bytes / 1206),
         (unsigned long long)(bytes / 1206 * 1206));
  return 0;
}
