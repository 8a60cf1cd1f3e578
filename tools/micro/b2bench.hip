// Blake2b compression throughput on gfx950 (registers only): variants of the 64-bit add.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <type_traits>
#include <vector>

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) { f(std::integral_constant<int, I>{}); sfor<N, I + 1>(f); }
}
__constant__ uint8_t SIG[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
struct S { static constexpr uint8_t s[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}}; };

template <int n> __device__ __forceinline__ void rot(uint32_t& lo, uint32_t& hi) {
  uint32_t a, b;
  if constexpr (n == 32) { a = hi; b = lo; }
  else if constexpr (n < 32) { a = __builtin_amdgcn_alignbit(hi, lo, n); b = __builtin_amdgcn_alignbit(lo, hi, n); }
  else { a = __builtin_amdgcn_alignbit(lo, hi, n - 32); b = __builtin_amdgcn_alignbit(hi, lo, n - 32); }
  lo = a; hi = b;
}
template <int MODE> __device__ __forceinline__ void add(uint32_t& lo, uint32_t& hi, uint32_t blo, uint32_t bhi) {
  if constexpr (MODE == 0) {
    uint64_t r = ((uint64_t(hi) << 32) | lo) + ((uint64_t(bhi) << 32) | blo);
    lo = uint32_t(r); hi = uint32_t(r >> 32);
  } else if constexpr (MODE == 1) {
    uint32_t c;
    asm("v_add_co_u32_e64 %0, %2, %0, %3\n v_addc_co_u32_e64 %1, %2, %1, %4, %2"
        : "+v"(lo), "+v"(hi), "=&s"(*(uint64_t*)&c) : "v"(blo), "v"(bhi));
  } else if constexpr (MODE == 2) {
    // full-rate forms only: carry = msb((a & b) | ((a | b) & ~sum)) (bitop3 0xD4)
    uint32_t s, t;
    asm("v_add_u32 %2, %0, %4\n"
        "v_bitop3_b32 %3, %0, %4, %2 bitop3:0xD4\n"
        "v_lshrrev_b32 %3, 31, %3\n"
        "v_add_u32 %1, %1, %5\n"
        "v_add_u32 %1, %1, %3\n"
        "v_mov_b32 %0, %2\n"
        : "+v"(lo), "+v"(hi), "=&v"(s), "=&v"(t) : "v"(blo), "v"(bhi));
  } else {
    asm("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&lo) : "v"(uint64_t(blo) | (uint64_t(bhi) << 32)));
    (void)hi;
  }
}
template <int MODE, int a, int b, int c, int d>
__device__ __forceinline__ void G(uint32_t (&L)[16], uint32_t (&H)[16], uint32_t xl, uint32_t xh, uint32_t yl, uint32_t yh) {
  add<MODE>(L[a], H[a], L[b], H[b]); add<MODE>(L[a], H[a], xl, xh);
  L[d] ^= L[a]; H[d] ^= H[a]; rot<32>(L[d], H[d]);
  add<MODE>(L[c], H[c], L[d], H[d]);
  L[b] ^= L[c]; H[b] ^= H[c]; rot<24>(L[b], H[b]);
  add<MODE>(L[a], H[a], L[b], H[b]); add<MODE>(L[a], H[a], yl, yh);
  L[d] ^= L[a]; H[d] ^= H[a]; rot<16>(L[d], H[d]);
  add<MODE>(L[c], H[c], L[d], H[d]);
  L[b] ^= L[c]; H[b] ^= H[c]; rot<63>(L[b], H[b]);
}
template <int MODE>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters) {
  uint32_t ml[16], mh[16], L[16], H[16];
  for (int i = 0; i < 16; ++i) { ml[i] = threadIdx.x * 3 + i; mh[i] = blockIdx.x + 7 * i; L[i] = i * 0x9E3779B9u; H[i] = threadIdx.x ^ i; }
  for (int it = 0; it < iters; ++it) {
    sfor<12>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      G<MODE, 0, 4, 8, 12>(L, H, ml[S::s[r][0]], mh[S::s[r][0]], ml[S::s[r][1]], mh[S::s[r][1]]);
      G<MODE, 1, 5, 9, 13>(L, H, ml[S::s[r][2]], mh[S::s[r][2]], ml[S::s[r][3]], mh[S::s[r][3]]);
      G<MODE, 2, 6, 10, 14>(L, H, ml[S::s[r][4]], mh[S::s[r][4]], ml[S::s[r][5]], mh[S::s[r][5]]);
      G<MODE, 3, 7, 11, 15>(L, H, ml[S::s[r][6]], mh[S::s[r][6]], ml[S::s[r][7]], mh[S::s[r][7]]);
      G<MODE, 0, 5, 10, 15>(L, H, ml[S::s[r][8]], mh[S::s[r][8]], ml[S::s[r][9]], mh[S::s[r][9]]);
      G<MODE, 1, 6, 11, 12>(L, H, ml[S::s[r][10]], mh[S::s[r][10]], ml[S::s[r][11]], mh[S::s[r][11]]);
      G<MODE, 2, 7, 8, 13>(L, H, ml[S::s[r][12]], mh[S::s[r][12]], ml[S::s[r][13]], mh[S::s[r][13]]);
      G<MODE, 3, 4, 9, 14>(L, H, ml[S::s[r][14]], mh[S::s[r][14]], ml[S::s[r][15]], mh[S::s[r][15]]);
    });
    for (int i = 0; i < 16; ++i) ml[i] ^= L[i];
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= L[i] ^ H[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}
int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 4 << 24);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int iters = 40;
  for (int blocks : {4096, 8192}) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
        else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
        else hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        {
          static std::vector<uint32_t> ref;
          std::vector<uint32_t> h(size_t(blocks) * 256);
          (void)hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
          if (mode == 0) ref = h;
          else if (h != ref) printf("  MISMATCH mode %d\n", mode);
        }
        double comp = double(blocks) * 256 * iters;
        printf("blocks %d mode %d: %.3f ms  %.2f G compressions/s\n", blocks, mode, ms, comp / ms / 1e6);
      }
    }
  }
  return 0;
}
