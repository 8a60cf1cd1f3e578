// Micro-benchmark: what bounds the codec's GF(2^16) table multiply on gfx950 -- the LDS pipe or
// the VALU?  One 16-wave workgroup per CU (140 KiB of LDS declared, as the codec kernels), and
// every kernel times itself with s_memtime (shader clock), so rates are per CU-cycle.
//   u16    12 ds_read_u16 per step, addresses fixed (pure LDS issue)
//   b32    12 ds_read_b32 per step
//   valu   the gf_mul2 address math with no LDS reads (pure VALU)
//   mul2   the codec's gf_mul2 (15 VALU + 6 ds_read_u16 per element pair) in butterflies
//   mulb2  the two-lookup (8/8-bit) form: 10 VALU + 4 ds_read_u16 per pair
// Build: hipcc --offload-arch=gfx950 -O3 -o ldsbench ldsbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define AS3 __attribute__((address_space(3)))
constexpr int kLds = 140 * 1024;
constexpr int kIters = 256;

#define SDWA_ADD(dst, w, sel) \
  "v_add_u32_sdwa " dst ", %[tb], " w " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" sel "\n"
#define MUL_ADDR(Y)                                \
  "v_lshlrev_b32 %[w0], 1, " Y "\n"                \
  "v_lshrrev_b32 %[w1], 5, " Y "\n"                \
  "v_lshrrev_b32 %[w2], 2, " Y "\n"                \
  "v_and_b32 %[w0], 0x007e007e, %[w0]\n"           \
  "v_and_b32 %[w1], 0x003e003e, %[w1]\n"           \
  "v_and_or_b32 %[w1], %[w2], %[m2], %[w1]\n"

template <int OFF1, int OFF2>
__device__ __forceinline__ void gf_mul2(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                        uint32_t tb) {
  uint32_t w0, w1, w2, a0, a1, a2, a3, a4, a5, c2, c3, c4;
  asm volatile(MUL_ADDR("%[y1]")
               SDWA_ADD("%[a0]", "%[w0]", "WORD_0")
               SDWA_ADD("%[a1]", "%[w0]", "WORD_1")
               SDWA_ADD("%[a2]", "%[w1]", "BYTE_0")
               SDWA_ADD("%[a3]", "%[w1]", "BYTE_2")
               SDWA_ADD("%[a4]", "%[w1]", "BYTE_1")
               SDWA_ADD("%[a5]", "%[w1]", "BYTE_3")
               "ds_read_u16 %[a0], %[a0] offset:%[p0]\n"
               "ds_read_u16_d16_hi %[a1], %[a1] offset:%[p0]\n"
               "ds_read_u16 %[a2], %[a2] offset:%[p1]\n"
               "ds_read_u16_d16_hi %[a3], %[a3] offset:%[p1]\n"
               "ds_read_u16 %[a4], %[a4] offset:%[p2]\n"
               "ds_read_u16_d16_hi %[a5], %[a5] offset:%[p2]\n"
               MUL_ADDR("%[y2]")
               SDWA_ADD("%[w2]", "%[w0]", "WORD_0")
               SDWA_ADD("%[w0]", "%[w0]", "WORD_1")
               SDWA_ADD("%[c2]", "%[w1]", "BYTE_0")
               SDWA_ADD("%[c3]", "%[w1]", "BYTE_2")
               SDWA_ADD("%[c4]", "%[w1]", "BYTE_1")
               SDWA_ADD("%[w1]", "%[w1]", "BYTE_3")
               "ds_read_u16 %[w2], %[w2] offset:%[q0]\n"
               "ds_read_u16_d16_hi %[w0], %[w0] offset:%[q0]\n"
               "ds_read_u16 %[c2], %[c2] offset:%[q1]\n"
               "ds_read_u16_d16_hi %[c3], %[c3] offset:%[q1]\n"
               "ds_read_u16 %[c4], %[c4] offset:%[q2]\n"
               "ds_read_u16_d16_hi %[w1], %[w1] offset:%[q2]\n"
               "s_waitcnt lgkmcnt(6)\n"
               "v_bitop3_b32 %[x1], %[x1], %[a0], %[a1] bitop3:0x96\n"
               "v_bitop3_b32 %[x1], %[x1], %[a2], %[a3] bitop3:0x96\n"
               "v_bitop3_b32 %[x1], %[x1], %[a4], %[a5] bitop3:0x96\n"
               "s_waitcnt lgkmcnt(0)\n"
               "v_bitop3_b32 %[x2], %[x2], %[w2], %[w0] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[c2], %[c3] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[c4], %[w1] bitop3:0x96\n"
               : [x1] "+v"(x1), [x2] "+v"(x2), [w0] "=&v"(w0), [w1] "=&v"(w1), [w2] "=&v"(w2),
                 [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4),
                 [a5] "=&v"(a5), [c2] "=&v"(c2), [c3] "=&v"(c3), [c4] "=&v"(c4)
               : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [m2] "s"(0x3e003e00u), [p0] "i"(OFF1),
                 [p1] "i"(OFF1 + 128), [p2] "i"(OFF1 + 192), [q0] "i"(OFF2), [q1] "i"(OFF2 + 128),
                 [q2] "i"(OFF2 + 192));
}

// the same VALU stream with every ds_read replaced by a v_mov (no LDS)
__device__ __forceinline__ void valu_mul2(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                          uint32_t tb) {
  uint32_t w0, w1, w2, a0, a1, a2, a3, a4, a5, c2, c3, c4;
  asm volatile(MUL_ADDR("%[y1]")
               SDWA_ADD("%[a0]", "%[w0]", "WORD_0")
               SDWA_ADD("%[a1]", "%[w0]", "WORD_1")
               SDWA_ADD("%[a2]", "%[w1]", "BYTE_0")
               SDWA_ADD("%[a3]", "%[w1]", "BYTE_2")
               SDWA_ADD("%[a4]", "%[w1]", "BYTE_1")
               SDWA_ADD("%[a5]", "%[w1]", "BYTE_3")
               MUL_ADDR("%[y2]")
               SDWA_ADD("%[w2]", "%[w0]", "WORD_0")
               SDWA_ADD("%[w0]", "%[w0]", "WORD_1")
               SDWA_ADD("%[c2]", "%[w1]", "BYTE_0")
               SDWA_ADD("%[c3]", "%[w1]", "BYTE_2")
               SDWA_ADD("%[c4]", "%[w1]", "BYTE_1")
               SDWA_ADD("%[w1]", "%[w1]", "BYTE_3")
               "v_bitop3_b32 %[x1], %[x1], %[a0], %[a1] bitop3:0x96\n"
               "v_bitop3_b32 %[x1], %[x1], %[a2], %[a3] bitop3:0x96\n"
               "v_bitop3_b32 %[x1], %[x1], %[a4], %[a5] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[w2], %[w0] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[c2], %[c3] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[c4], %[w1] bitop3:0x96\n"
               : [x1] "+v"(x1), [x2] "+v"(x2), [w0] "=&v"(w0), [w1] "=&v"(w1), [w2] "=&v"(w2),
                 [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4),
                 [a5] "=&v"(a5), [c2] "=&v"(c2), [c3] "=&v"(c3), [c4] "=&v"(c4)
               : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [m2] "s"(0x3e003e00u));
}

// two-lookup form: 256-entry u16 sub-tables for the low / high operand byte
template <int OFF>
__device__ __forceinline__ void gf_mulb2(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                         uint32_t tb) {
  uint32_t w0, w1, a0, a1, a2, a3, c0, c1, c2, c3;
  asm volatile(
      "v_lshlrev_b32 %[w0], 1, %[y1]\n"
      "v_lshrrev_b32 %[w1], 7, %[y1]\n"
      "v_and_b32 %[w0], 0x01fe01fe, %[w0]\n"
      "v_and_b32 %[w1], 0x01fe01fe, %[w1]\n"
      SDWA_ADD("%[a0]", "%[w0]", "WORD_0") SDWA_ADD("%[a1]", "%[w0]", "WORD_1")
      SDWA_ADD("%[a2]", "%[w1]", "WORD_0") SDWA_ADD("%[a3]", "%[w1]", "WORD_1")
      "ds_read_u16 %[a0], %[a0] offset:%[p0]\n"
      "ds_read_u16_d16_hi %[a1], %[a1] offset:%[p0]\n"
      "ds_read_u16 %[a2], %[a2] offset:%[p1]\n"
      "ds_read_u16_d16_hi %[a3], %[a3] offset:%[p1]\n"
      "v_lshlrev_b32 %[w0], 1, %[y2]\n"
      "v_lshrrev_b32 %[w1], 7, %[y2]\n"
      "v_and_b32 %[w0], 0x01fe01fe, %[w0]\n"
      "v_and_b32 %[w1], 0x01fe01fe, %[w1]\n"
      SDWA_ADD("%[c0]", "%[w0]", "WORD_0") SDWA_ADD("%[c1]", "%[w0]", "WORD_1")
      SDWA_ADD("%[c2]", "%[w1]", "WORD_0") SDWA_ADD("%[c3]", "%[w1]", "WORD_1")
      "ds_read_u16 %[c0], %[c0] offset:%[p0]\n"
      "ds_read_u16_d16_hi %[c1], %[c1] offset:%[p0]\n"
      "ds_read_u16 %[c2], %[c2] offset:%[p1]\n"
      "ds_read_u16_d16_hi %[c3], %[c3] offset:%[p1]\n"
      "s_waitcnt lgkmcnt(4)\n"
      "v_bitop3_b32 %[x1], %[x1], %[a0], %[a1] bitop3:0x96\n"
      "v_bitop3_b32 %[x1], %[x1], %[a2], %[a3] bitop3:0x96\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_bitop3_b32 %[x2], %[x2], %[c0], %[c1] bitop3:0x96\n"
      "v_bitop3_b32 %[x2], %[x2], %[c2], %[c3] bitop3:0x96\n"
      : [x1] "+v"(x1), [x2] "+v"(x2), [w0] "=&v"(w0), [w1] "=&v"(w1), [a0] "=&v"(a0),
        [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [c0] "=&v"(c0), [c1] "=&v"(c1),
        [c2] "=&v"(c2), [c3] "=&v"(c3)
      : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [p0] "i"(OFF), [p1] "i"(OFF + 512));
}

// shift form: 5 shifts (half-rate) + fast ops; field k of the pair at bits [1, 7) or [1, 6)
// of t_k, then (t_k & mask) | tb by one v_bitop3 (truth table 0xEA = (S0 & S1) | S2), or
// (kNoTb) a plain v_and with the table base folded into the DS offset.
template <int OFF1, int OFF2, bool kNoTb>
__device__ __forceinline__ void gf_mul2n(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                         uint32_t tb) {
  uint32_t a0, a1, a2, a3, a4, a5, c0, c1, c2, c3, c4, c5;
#define N_ADDR(Y, A0, A1, A2, A3, A4, A5)                          \
  "v_add_u32 " A0 ", " Y ", " Y "\n"                               \
  "v_lshrrev_b32 " A1 ", 5, " Y "\n"                               \
  "v_lshrrev_b32 " A2 ", 10, " Y "\n"                              \
  "v_lshrrev_b32 " A3 ", 15, " Y "\n"                              \
  "v_lshrrev_b32 " A4 ", 21, " Y "\n"                              \
  "v_lshrrev_b32 " A5 ", 26, " Y "\n"
#define N_MASK3(A, M) "v_bitop3_b32 " A ", " A ", " M ", %[tb] bitop3:0xEA\n"
#define N_MASK2(A, M) "v_and_b32 " A ", " M ", " A "\n"
#define N_READS(A0, A1, A2, A3, A4, A5, P0, P1, P2)           \
  "ds_read_u16 " A0 ", " A0 " offset:" P0 "\n"                \
  "ds_read_u16 " A1 ", " A1 " offset:" P1 "\n"                \
  "ds_read_u16 " A2 ", " A2 " offset:" P2 "\n"                \
  "ds_read_u16_d16_hi " A3 ", " A3 " offset:" P0 "\n"         \
  "ds_read_u16_d16_hi " A4 ", " A4 " offset:" P1 "\n"         \
  "ds_read_u16_d16_hi " A5 ", " A5 " offset:" P2 "\n"
#define N_BODY(MASK)                                                                         \
  N_ADDR("%[y1]", "%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]")                     \
  MASK("%[a0]", "%[m7]") MASK("%[a1]", "%[m3]") MASK("%[a2]", "%[m3]")                       \
  MASK("%[a3]", "%[m7]") MASK("%[a4]", "%[m3]") MASK("%[a5]", "%[m3]")                       \
  N_READS("%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[p0]", "%[p1]", "%[p2]")   \
  N_ADDR("%[y2]", "%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]")                     \
  MASK("%[c0]", "%[m7]") MASK("%[c1]", "%[m3]") MASK("%[c2]", "%[m3]")                       \
  MASK("%[c3]", "%[m7]") MASK("%[c4]", "%[m3]") MASK("%[c5]", "%[m3]")                       \
  N_READS("%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]", "%[q0]", "%[q1]", "%[q2]")   \
  "s_waitcnt lgkmcnt(6)\n"                                                                   \
  "v_bitop3_b32 %[x1], %[x1], %[a0], %[a1] bitop3:0x96\n"                                    \
  "v_bitop3_b32 %[x1], %[x1], %[a2], %[a3] bitop3:0x96\n"                                    \
  "v_bitop3_b32 %[x1], %[x1], %[a4], %[a5] bitop3:0x96\n"                                    \
  "s_waitcnt lgkmcnt(0)\n"                                                                   \
  "v_bitop3_b32 %[x2], %[x2], %[c0], %[c1] bitop3:0x96\n"                                    \
  "v_bitop3_b32 %[x2], %[x2], %[c2], %[c3] bitop3:0x96\n"                                    \
  "v_bitop3_b32 %[x2], %[x2], %[c4], %[c5] bitop3:0x96\n"
  if constexpr (kNoTb) {
    asm volatile(N_BODY(N_MASK2)
                 : [x1] "+v"(x1), [x2] "+v"(x2), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2),
                   [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [c0] "=&v"(c0), [c1] "=&v"(c1),
                   [c2] "=&v"(c2), [c3] "=&v"(c3), [c4] "=&v"(c4), [c5] "=&v"(c5)
                 : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [m7] "s"(0x7eu), [m3] "s"(0x3eu),
                   [p0] "i"(OFF1), [p1] "i"(OFF1 + 128), [p2] "i"(OFF1 + 192), [q0] "i"(OFF2),
                   [q1] "i"(OFF2 + 128), [q2] "i"(OFF2 + 192));
  } else {
    asm volatile(N_BODY(N_MASK3)
                 : [x1] "+v"(x1), [x2] "+v"(x2), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2),
                   [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [c0] "=&v"(c0), [c1] "=&v"(c1),
                   [c2] "=&v"(c2), [c3] "=&v"(c3), [c4] "=&v"(c4), [c5] "=&v"(c5)
                 : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [m7] "s"(0x7eu), [m3] "s"(0x3eu),
                   [p0] "i"(OFF1), [p1] "i"(OFF1 + 128), [p2] "i"(OFF1 + 192), [q0] "i"(OFF2),
                   [q1] "i"(OFF2 + 128), [q2] "i"(OFF2 + 192));
  }
}

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

__device__ __forceinline__ void fence(uint32_t (&X)[32]) {
#pragma unroll
  for (int i = 0; i < 32; ++i) asm volatile("" : "+v"(X[i]));
}

// one in-wave layer set (d = 1..16) over 32 registers: 80 butterflies, table slot per group
template <int MODE>
__device__ __forceinline__ void layers(uint32_t (&X)[32], uint32_t tb) {
  sfor<5>([&](auto kk) {
    constexpr int k = decltype(kk)::value;
    constexpr int d = 1 << k;
    sfor<8>([&](auto qq) {
      constexpr int b1 = 2 * decltype(qq)::value, b2 = b1 + 1;
      constexpr int i1 = 2 * d * (b1 / d) + b1 % d, i2 = 2 * d * (b2 / d) + b2 % d;
      constexpr int t1 = ((32 - 32 / d + b1 / d) % 31) * 256, t2 = ((32 - 32 / d + b2 / d) % 31) * 256;
      X[i1 + d] ^= X[i1];
      X[i2 + d] ^= X[i2];
      if constexpr (MODE == 0) gf_mul2<t1, t2>(X[i1], X[i1 + d], X[i2], X[i2 + d], tb);
      else if constexpr (MODE == 1) valu_mul2(X[i1], X[i1 + d], X[i2], X[i2 + d], tb);
      else if constexpr (MODE == 2) gf_mulb2<(t1 % 8192) * 4>(X[i1], X[i1 + d], X[i2], X[i2 + d], tb);
      else if constexpr (MODE == 3) gf_mul2n<t1, t2, false>(X[i1], X[i1 + d], X[i2], X[i2 + d], tb);
      else gf_mul2n<t1, t2, true>(X[i1], X[i1 + d], X[i2], X[i2 + d], tb);
    });
    fence(X);
  });
}

__device__ __forceinline__ void record(uint64_t* cyc, uint64_t t0) {
  if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
}

template <int MODE>
__global__ void __launch_bounds__(1024, 1) k_mul(uint32_t* out, uint64_t* cyc, const uint16_t* tabs) {
  __shared__ __attribute__((aligned(16))) uint8_t sm[kLds];
  for (int i = threadIdx.x; i < kLds / 4; i += blockDim.x)
    reinterpret_cast<uint32_t*>(sm)[i] = reinterpret_cast<const uint32_t*>(tabs)[i % 2048];
  __syncthreads();
  uint32_t X[32];
  for (int i = 0; i < 32; ++i) X[i] = threadIdx.x * 7919u + i * 104729u;
  const uint32_t tb = uint32_t(reinterpret_cast<uintptr_t>((AS3 uint8_t*)sm)) + (threadIdx.x >> 6) * 128;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) layers<MODE>(X, tb);
  __syncthreads();
  record(cyc, t0);
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) r ^= X[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// pure LDS: 12 ds_read_u16 (or b32) per step from fixed in-table addresses
template <bool kB32>
__global__ void __launch_bounds__(1024, 1) k_lds(uint32_t* out, uint64_t* cyc, const uint16_t* tabs) {
  __shared__ __attribute__((aligned(16))) uint8_t sm[kLds];
  for (int i = threadIdx.x; i < kLds / 4; i += blockDim.x)
    reinterpret_cast<uint32_t*>(sm)[i] = reinterpret_cast<const uint32_t*>(tabs)[i % 2048];
  __syncthreads();
  const uint32_t base = uint32_t(reinterpret_cast<uintptr_t>((AS3 uint8_t*)sm));
  uint32_t a[12];
  for (int k = 0; k < 12; ++k) a[k] = base + k * 256 + ((threadIdx.x * 37 + k * 11) & 62);
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters * 40; ++it) {
    uint32_t r[12];
    if constexpr (kB32) {
#pragma unroll
      for (int k = 0; k < 12; ++k)
        asm volatile("ds_read_b32 %0, %1 offset:0" : "=v"(r[k]) : "v"(a[k] & ~3u));
    } else {
#pragma unroll
      for (int k = 0; k < 12; ++k) asm volatile("ds_read_u16 %0, %1" : "=v"(r[k]) : "v"(a[k]));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 12; ++k) acc ^= r[k];
  }
  __syncthreads();
  record(cyc, t0);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int blocks = 256, threads = 1024;
  uint32_t* out;
  uint64_t* cyc;
  uint16_t* tabs;
  hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
  hipMalloc(&cyc, sizeof(uint64_t) * blocks);
  hipMalloc(&tabs, 8192);
  std::vector<uint16_t> h(4096);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint16_t(i * 40503u + 11);
  hipMemcpy(tabs, h.data(), 8192, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"mul2 (15 VALU + 6 u16 / pair)", "valu-only mul2", "mulb2 (10 VALU + 4 u16)",
                         "u16 reads", "b32 reads", "mul2n (shifts + bitop3 OR tb)", "mul2n (shifts + and, tb in offset)"};
  for (int mode = 0; mode < 7; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_mul<0>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
        case 1: hipLaunchKernelGGL(k_mul<1>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
        case 2: hipLaunchKernelGGL(k_mul<2>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
        case 5: hipLaunchKernelGGL(k_mul<3>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
        case 6: hipLaunchKernelGGL(k_mul<4>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
        case 3: hipLaunchKernelGGL(k_lds<false>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
        default: hipLaunchKernelGGL(k_lds<true>, dim3(blocks), dim3(threads), 0, 0, out, cyc, tabs); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<uint64_t> c(blocks);
      hipMemcpy(c.data(), cyc, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost);
      double mc = 0;
      for (auto v : c) mc += double(v);
      mc /= blocks;
      const double waves = 16.0;
      if (mode <= 2 || mode >= 5) {
        const double wmuls = waves * kIters * 80;  // wave-level pair multiplies per WG
        printf("%-32s %.3f ms  %.0f cyc/WG  %.3f cyc per wave-mult per CU  %.2f T elem-mult/s\n",
               names[mode], ms, mc, mc / wmuls, wmuls * 128 * blocks / (ms * 1e-3) / 1e12);
      } else {
        const double lds = waves * kIters * 40 * 12;
        printf("%-32s %.3f ms  %.0f cyc/WG  %.3f cyc per LDS wave-instr per CU\n", names[mode], ms, mc,
               mc / lds);
      }
    }
  }
  return 0;
}
