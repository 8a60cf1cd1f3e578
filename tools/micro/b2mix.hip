// Is the Blake2b compression at the floor of its instruction mix on gfx950?  (VERDICT r05
// item 4.)  A compression is 96 G functions; each G is 6 64-bit adds (v_lshl_add_u64, ~4.1
// cycles per wave64 instruction), 8 v_xor_b32 (~2.1) and 6 v_alignbit_b32 (~4.1)
// (tools/micro/valubench, profiles/r03/micro/valubench_*.txt): 66 SIMD-cycles per G, 25 G
// compressions/s on 1,024 SIMDs at 2.4 GHz if every issue slot were used.
//
//   compress   the real compression (b2bench.hip mode 0: the compiler's 64-bit adds), its
//              dependency chains as the G functions have them (4 independent G per half-round)
//   compress2  two independent compressions interleaved per lane (twice the ILP)
//   mix        the same instruction mix per G-equivalent with no dependency closer than 8
//              instructions (8 independent streams): the mix's own issue ceiling
// All at 256-thread workgroups, 8,192 workgroups (occupancy as the leaf kernels), rate in
// G compression-equivalents per second.  If compress reaches mix, the compression runs at the
// issue floor of its mix and only a different mix (fewer 4-cycle forms) can make it faster.
// Build: hipcc --offload-arch=gfx950 -O3 -o bin/b2mix b2mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <type_traits>

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) { f(std::integral_constant<int, I>{}); sfor<N, I + 1>(f); }
}
struct S { static constexpr uint8_t s[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}}; };

// rotations as the leaf kernel has them (rs2_hash.hip): two v_alignbit_b32 (32: a register swap)
template <int n>
__device__ __forceinline__ uint64_t ror(uint64_t x) {
  const uint32_t lo = uint32_t(x), hi = uint32_t(x >> 32);
  uint32_t a, b;
  if constexpr (n == 32) { a = hi; b = lo; }
  else if constexpr (n < 32) { a = __builtin_amdgcn_alignbit(hi, lo, n); b = __builtin_amdgcn_alignbit(lo, hi, n); }
  else { a = __builtin_amdgcn_alignbit(lo, hi, n - 32); b = __builtin_amdgcn_alignbit(hi, lo, n - 32); }
  return uint64_t(a) | (uint64_t(b) << 32);
}
template <int a, int b, int c, int d>
__device__ __forceinline__ void G(uint64_t (&v)[16], uint64_t x, uint64_t y) {
  v[a] = v[a] + v[b] + x; v[d] = ror<32>(v[d] ^ v[a]);
  v[c] = v[c] + v[d];     v[b] = ror<24>(v[b] ^ v[c]);
  v[a] = v[a] + v[b] + y; v[d] = ror<16>(v[d] ^ v[a]);
  v[c] = v[c] + v[d];     v[b] = ror<63>(v[b] ^ v[c]);
}
__device__ __forceinline__ void compress(uint64_t (&v)[16], const uint64_t (&m)[16]) {
  sfor<12>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    G<0, 4, 8, 12>(v, m[S::s[r][0]], m[S::s[r][1]]);
    G<1, 5, 9, 13>(v, m[S::s[r][2]], m[S::s[r][3]]);
    G<2, 6, 10, 14>(v, m[S::s[r][4]], m[S::s[r][5]]);
    G<3, 7, 11, 15>(v, m[S::s[r][6]], m[S::s[r][7]]);
    G<0, 5, 10, 15>(v, m[S::s[r][8]], m[S::s[r][9]]);
    G<1, 6, 11, 12>(v, m[S::s[r][10]], m[S::s[r][11]]);
    G<2, 7, 8, 13>(v, m[S::s[r][12]], m[S::s[r][13]]);
    G<3, 4, 9, 14>(v, m[S::s[r][14]], m[S::s[r][15]]);
  });
}

// one trip of the mix: 8 G-equivalents, one per stream (48 v_lshl_add_u64, 64 v_xor_b32,
// 48 v_alignbit_b32), consecutive instructions from different streams
__device__ __forceinline__ void mix_trip(uint64_t (&A)[8], uint32_t (&B)[8], uint32_t (&C)[8],
                                         uint64_t K) {
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(A[j]) : "v"(K));
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_xor_b32 %0, %0, %2\n v_xor_b32 %1, %1, %0" : "+v"(B[j]), "+v"(C[j]) : "v"(uint32_t(A[j])));
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(C[j]) : "v"(B[j]));
}

template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters) {
  uint64_t m[16], v[16], w[16];
  for (int i = 0; i < 16; ++i) {
    m[i] = (uint64_t(threadIdx.x * 3 + i) << 32) | (blockIdx.x + 7u * i);
    v[i] = i * 0x9E3779B97F4A7C15ull ^ threadIdx.x;
    w[i] = v[i] ^ 0x5555;
  }
  if constexpr (MODE == 0) {
    for (int it = 0; it < iters; ++it) {
      compress(v, m);
      for (int i = 0; i < 16; ++i) m[i] ^= v[i];
    }
  } else if constexpr (MODE == 1) {
    for (int it = 0; it < iters; it += 2) {  // two compressions per trip, interleaved by the compiler
      compress(v, m);
      compress(w, m);
      for (int i = 0; i < 16; ++i) m[i] ^= v[i] ^ w[i];
    }
  } else {
    // 96 G-equivalents per compression; per G: 6 v_lshl_add_u64, 8 v_xor_b32, 6 v_alignbit_b32.
    // 8 streams (j): A[j] 64-bit, B[j] / C[j] 32-bit; each trip = 8 G-equivalents (one per stream)
    uint64_t A[8];
    uint32_t B[8], C[8];
    for (int j = 0; j < 8; ++j) { A[j] = v[j]; B[j] = uint32_t(v[j + 8]); C[j] = uint32_t(m[j]); }
    const uint64_t K = m[9];
    for (int it = 0; it < iters * 12; ++it) {  // 12 trips x 8 G-eq = one compression per stream-set
      mix_trip(A, B, C, K);
    }
    for (int j = 0; j < 8; ++j) v[j] ^= A[j] ^ B[j] ^ C[j];
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= uint32_t(v[i] ^ (v[i] >> 32) ^ w[i]);
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 4 << 24);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 40, blocks = 8192;
  const char* names[3] = {"compress", "compress2 (2 interleaved)", "mix (8 independent streams)"};
  for (int mode = 0; mode < 3; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      // compression-equivalents: mode 2 runs one per 12 trips of 8 streams x 8 G... = iters per lane
      const double comp = double(blocks) * 256 * iters;
      printf("%-30s rep %d: %.3f ms  %.2f G compression-equivalents/s\n", names[mode], rep, ms,
             comp / ms / 1e6);
    }
  return 0;
}
