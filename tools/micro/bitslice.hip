// Micro-benchmark: an LDS-free, bit-sliced GF(2^16) multiply by a
// wave-uniform constant against the codec's table multiply, per CU-cycle (s_memtime), on gfx950.
//
// Multiplying by a constant c is a GF(2)-linear map: a 16x16 bit matrix M_c.  Bit-sliced, a
// lane holds 32 elements of one codeword position as 16 bit-planes (plane b = bit b of the 32
// elements), and y = M_c x is, per output plane i, the XOR of the input planes j with
// M_c[i][j] = 1.  The constant is wave-uniform but not known at compile time, so the XOR network
// is chosen at run time "Four-Russians" style: the 16 input planes in 4 groups of 4; per group
// the 16 XOR combinations T[0..15] of its planes (11 XORs + 4 copies), then per output plane one
// XOR of T[nibble(i, g)] -- a register indexed by a wave-uniform value (M0-relative v_movrels /
// s_set_gpr_idx, chosen by the compiler from a readfirstlane index).  Per 32 elements:
// 4 x (15 + 16) = 124 VALU + 64 SALU index writes, no LDS.
//
//   prod    the codec's gf_mul2 (rs2_codec.hip): 17 VALU + 6 ds_read_u16 per element pair,
//           butterflies over 32 packed registers, tables in LDS
//   bs4r    bit-sliced Four-Russians butterflies over 4 positions x 16 planes per lane
//   conv    the bit-plane conversion a bit-sliced transform adds at its load and store: 16 packed
//           registers (32 elements) <-> 16 planes, 5 delta-swap stages each way (round trip)
//   check   bs4r's multiply against a host evaluation of the same bit matrices (correctness)
// Build: hipcc --offload-arch=gfx950 -O3 -o bitslice bitslice.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>
#include <vector>

constexpr int kLds = 140 * 1024;  // one 16-wave workgroup per CU, as the codec kernels
constexpr int kIters = 256;
constexpr int NCONST = 64;

// ---- the codec's table multiply (rs2_codec.hip RS2_GF_ADDR / RS2_GF_READS, 3 lookups) ----
#define GF_ADDR(Y, A0, A1, A2, A3, A4, A5)                      \
  "v_add_u32 " A0 ", " Y ", " Y "\n"                             \
  "v_lshrrev_b32 " A1 ", 15, " Y "\n"                            \
  "v_lshrrev_b32 " A2 ", 5, " Y "\n"                             \
  "v_lshrrev_b32 " A3 ", 21, " Y "\n"                            \
  "v_lshrrev_b32 " A4 ", 10, " Y "\n"                            \
  "v_lshrrev_b32 " A5 ", 26, " Y "\n"                            \
  "v_and_b32 " A0 ", 0x7e, " A0 "\n"                             \
  "v_and_b32 " A1 ", 0x7e, " A1 "\n"                             \
  "v_or_b32 " A0 ", " A0 ", %[tb]\n"                             \
  "v_or_b32 " A1 ", " A1 ", %[tb]\n"                             \
  "v_bitop3_b32 " A2 ", " A2 ", 62, %[tb] bitop3:0xEA\n"         \
  "v_bitop3_b32 " A3 ", " A3 ", 62, %[tb] bitop3:0xEA\n"         \
  "v_bitop3_b32 " A4 ", " A4 ", 62, %[tb] bitop3:0xEA\n"         \
  "v_bitop3_b32 " A5 ", " A5 ", 62, %[tb] bitop3:0xEA\n"
#define GF_READS(A0, A1, A2, A3, A4, A5, O0, O1, O2)            \
  "ds_read_u16 " A0 ", " A0 " offset:" O0 "\n"                   \
  "ds_read_u16_d16_hi " A1 ", " A1 " offset:" O0 "\n"            \
  "ds_read_u16 " A2 ", " A2 " offset:" O1 "\n"                   \
  "ds_read_u16_d16_hi " A3 ", " A3 " offset:" O1 "\n"            \
  "ds_read_u16 " A4 ", " A4 " offset:" O2 "\n"                   \
  "ds_read_u16_d16_hi " A5 ", " A5 " offset:" O2 "\n"

template <int OFF1, int OFF2>
__device__ __forceinline__ void gf_mul2(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                        uint32_t tb) {
  uint32_t a0, a1, a2, a3, a4, a5, c0, c1, c2, c3, c4, c5;
  asm volatile(GF_ADDR("%[y1]", "%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]")
               GF_READS("%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[p0]", "%[p1]", "%[p2]")
               GF_ADDR("%[y2]", "%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]")
               GF_READS("%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]", "%[q0]", "%[q1]", "%[q2]")
               "s_waitcnt lgkmcnt(6)\n"
               "v_bitop3_b32 %[x1], %[x1], %[a0], %[a1] bitop3:0x96\n"
               "v_bitop3_b32 %[x1], %[x1], %[a2], %[a3] bitop3:0x96\n"
               "v_bitop3_b32 %[x1], %[x1], %[a4], %[a5] bitop3:0x96\n"
               "s_waitcnt lgkmcnt(0)\n"
               "v_bitop3_b32 %[x2], %[x2], %[c0], %[c1] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[c2], %[c3] bitop3:0x96\n"
               "v_bitop3_b32 %[x2], %[x2], %[c4], %[c5] bitop3:0x96\n"
               : [x1] "+v"(x1), [x2] "+v"(x2), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2),
                 [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [c0] "=&v"(c0), [c1] "=&v"(c1),
                 [c2] "=&v"(c2), [c3] "=&v"(c3), [c4] "=&v"(c4), [c5] "=&v"(c5)
               : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [p0] "i"(OFF1), [p1] "i"(OFF1 + 128),
                 [p2] "i"(OFF1 + 192), [q0] "i"(OFF2), [q1] "i"(OFF2 + 128), [q2] "i"(OFF2 + 192));
}

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

// 32 packed registers (64 elements), butterflies (i, i+1) then (i, i+2), 16 multiplies per
// sweep, table slot rotating over 32 tables of 256 B
__global__ void __launch_bounds__(1024) k_prod(uint64_t* cyc, uint32_t* out, const uint16_t* tabs) {
  extern __shared__ __attribute__((aligned(128))) uint8_t smem[];
  for (int i = threadIdx.x; i < 32 * 128; i += blockDim.x)
    reinterpret_cast<uint16_t*>(smem)[i] = tabs[i % (NCONST * 128)];
  __syncthreads();
  uint32_t x[32];
  for (int i = 0; i < 32; ++i) x[i] = threadIdx.x * 7919u + i * 104729u;
  const uint32_t tb = uint32_t(reinterpret_cast<uintptr_t>(smem));
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    sfor<8>([&](auto qq) {
      constexpr int q = decltype(qq)::value;
      constexpr int i = 4 * q;
      gf_mul2<(q * 2 % 32) * 256, ((q * 2 + 1) % 32) * 256>(x[i], x[i + 1], x[i + 2], x[i + 3], tb);
      x[i + 1] ^= x[i];
      x[i + 3] ^= x[i + 2];
      gf_mul2<((q * 2 + 16) % 32) * 256, ((q * 2 + 17) % 32) * 256>(x[i], x[i + 2], x[i + 1], x[i + 3], tb);
      x[i + 2] ^= x[i];
      x[i + 3] ^= x[i + 1];
    });
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// ---- bit-sliced multiply ------------------------------------------------------------------
// acc ^= M y for 16 planes.  M as 64 nibble indices, dword [g*16 + i] = the nibble of row i over
// input planes 4g .. 4g+3 (wave-uniform, scalar loads).  Per group: the 16 XOR combinations of
// its 4 planes into v112..v127 (T[0] = 0, 4 copies, 11 XORs), then acc[i] ^= T[idx] with
// M0-relative SRC0 (s_set_gpr_idx_on / _idx / _off): 16 VALU + 17 SALU per 16 rows.
#define BS_ACC(i) "v_xor_b32 %[a" #i "], v112, %[a" #i "]\n"
#define BS_IDX(i) "s_set_gpr_idx_idx %[s" #i "]\n"
__device__ __forceinline__ void bs_group(uint32_t (&a)[16], uint32_t y0, uint32_t y1, uint32_t y2,
                                         uint32_t y3, const uint32_t* __restrict__ sp) {
  // scalar loads (constant address space): the indices go straight to SGPRs
  typedef __attribute__((address_space(4))) const uint32_t cu32;
  cu32* cp = reinterpret_cast<cu32*>(reinterpret_cast<uintptr_t>(sp));
  uint32_t s[16];
  sfor<16>([&](auto ii) { s[decltype(ii)::value] = cp[decltype(ii)::value]; });
  asm volatile(
      "v_mov_b32 v112, 0\n"
      "v_mov_b32 v113, %[y0]\n"
      "v_mov_b32 v114, %[y1]\n"
      "v_xor_b32 v115, %[y0], %[y1]\n"
      "v_mov_b32 v116, %[y2]\n"
      "v_xor_b32 v117, %[y2], %[y0]\n"
      "v_xor_b32 v118, %[y2], %[y1]\n"
      "v_xor_b32 v119, %[y2], v115\n"
      "v_mov_b32 v120, %[y3]\n"
      "v_xor_b32 v121, %[y3], %[y0]\n"
      "v_xor_b32 v122, %[y3], %[y1]\n"
      "v_xor_b32 v123, %[y3], v115\n"
      "v_xor_b32 v124, %[y3], %[y2]\n"
      "v_xor_b32 v125, %[y3], v117\n"
      "v_xor_b32 v126, %[y3], v118\n"
      "v_xor_b32 v127, %[y3], v119\n"
      "s_set_gpr_idx_on %[s0], gpr_idx(SRC0)\n" BS_ACC(0)
      BS_IDX(1) BS_ACC(1) BS_IDX(2) BS_ACC(2) BS_IDX(3) BS_ACC(3) BS_IDX(4) BS_ACC(4)
      BS_IDX(5) BS_ACC(5) BS_IDX(6) BS_ACC(6) BS_IDX(7) BS_ACC(7) BS_IDX(8) BS_ACC(8)
      BS_IDX(9) BS_ACC(9) BS_IDX(10) BS_ACC(10) BS_IDX(11) BS_ACC(11) BS_IDX(12) BS_ACC(12)
      BS_IDX(13) BS_ACC(13) BS_IDX(14) BS_ACC(14) BS_IDX(15) BS_ACC(15)
      "s_set_gpr_idx_off\n"
      : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]),
        [a5] "+v"(a[5]), [a6] "+v"(a[6]), [a7] "+v"(a[7]), [a8] "+v"(a[8]), [a9] "+v"(a[9]),
        [a10] "+v"(a[10]), [a11] "+v"(a[11]), [a12] "+v"(a[12]), [a13] "+v"(a[13]),
        [a14] "+v"(a[14]), [a15] "+v"(a[15])
      : [y0] "v"(y0), [y1] "v"(y1), [y2] "v"(y2), [y3] "v"(y3), [s0] "s"(s[0]), [s1] "s"(s[1]),
        [s2] "s"(s[2]), [s3] "s"(s[3]), [s4] "s"(s[4]), [s5] "s"(s[5]), [s6] "s"(s[6]),
        [s7] "s"(s[7]), [s8] "s"(s[8]), [s9] "s"(s[9]), [s10] "s"(s[10]), [s11] "s"(s[11]),
        [s12] "s"(s[12]), [s13] "s"(s[13]), [s14] "s"(s[14]), [s15] "s"(s[15])
      : "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",
        "v123", "v124", "v125", "v126", "v127");
}
__device__ __forceinline__ void bs_mul(uint32_t (&acc)[16], const uint32_t (&y)[16],
                                       const uint32_t* __restrict__ idx) {
  sfor<4>([&](auto gg) {
    constexpr int g = decltype(gg)::value;
    bs_group(acc, y[4 * g], y[4 * g + 1], y[4 * g + 2], y[4 * g + 3], idx + 16 * g);
  });
}

// 4 positions x 16 planes per lane: butterflies (0,1) (2,3) (0,2) (1,3) per sweep, a new
// constant per butterfly from a rotating set of NCONST matrices (scalar loads)
__global__ void __launch_bounds__(1024) k_bs4r(uint64_t* cyc, uint32_t* out, const uint32_t* mats) {
  extern __shared__ __attribute__((aligned(128))) uint8_t smem[];  // occupancy only
  (void)smem;
  uint32_t X[4][16];
  for (int p = 0; p < 4; ++p)
    for (int b = 0; b < 16; ++b) X[p][b] = threadIdx.x * 7919u + (p * 16 + b) * 104729u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    const uint32_t* m = mats + ((it * 4) % NCONST) * 64;
    bs_mul(X[0], X[1], m);
#pragma unroll
    for (int b = 0; b < 16; ++b) X[1][b] ^= X[0][b];
    bs_mul(X[2], X[3], m + 64);
#pragma unroll
    for (int b = 0; b < 16; ++b) X[3][b] ^= X[2][b];
    bs_mul(X[0], X[2], m + 128);
#pragma unroll
    for (int b = 0; b < 16; ++b) X[2][b] ^= X[0][b];
    bs_mul(X[1], X[3], m + 192);
#pragma unroll
    for (int b = 0; b < 16; ++b) X[3][b] ^= X[1][b];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
  for (int p = 0; p < 4; ++p)
    for (int b = 0; b < 16; ++b) r ^= X[p][b];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// ---- bit-plane conversion -----------------------------------------------------------------
// Register k holds elements 2k (bits 0-15) and 2k+1 (bits 16-31).  Index bits: word k3..k0,
// bit j4..j0 (element = k:j4, element bit = j3..j0).  Five delta swaps exchange a word-index bit
// with a bit-position bit: (w3,p4) (w2,p3) (w1,p2) (w0,p1) then (w3,p0), leaving word = the
// element bit (order j0 j3 j2 j1) and bit position = the element index (order k3 k2 k1 k0 j4):
// a fixed permutation of planes and elements, which the constant matrices absorb.
template <int WB, int PB>
__device__ __forceinline__ void delta_swap(uint32_t (&r)[16]) {
  constexpr int wd = 1 << WB, sh = 1 << PB;
  constexpr uint32_t mask = [] {
    uint32_t m = 0;
    for (int i = 0; i < 32; ++i)
      if (!((i >> PB) & 1)) m |= 1u << i;
    return m;
  }();
  sfor<16>([&](auto kk) {
    constexpr int k = decltype(kk)::value;
    if constexpr (!((k >> WB) & 1)) {
      // word k (w bit 0) keeps its p-bit-0 half; exchanges its p-bit-1 half with word k+wd's
      // p-bit-0 half
      const uint32_t t = ((r[k] >> sh) ^ r[k + wd]) & mask;
      r[k + wd] ^= t;
      r[k] ^= t << sh;
    }
  });
}
__device__ __forceinline__ void to_planes(uint32_t (&r)[16]) {
  delta_swap<3, 4>(r);
  delta_swap<2, 3>(r);
  delta_swap<1, 2>(r);
  delta_swap<0, 1>(r);
  delta_swap<3, 0>(r);
}
__device__ __forceinline__ void from_planes(uint32_t (&r)[16]) {  // the swaps are involutions
  delta_swap<3, 0>(r);
  delta_swap<0, 1>(r);
  delta_swap<1, 2>(r);
  delta_swap<2, 3>(r);
  delta_swap<3, 4>(r);
}
__global__ void __launch_bounds__(1024) k_conv(uint64_t* cyc, uint32_t* out) {
  extern __shared__ __attribute__((aligned(128))) uint8_t smem[];
  (void)smem;
  uint32_t r[2][16];
  for (int q = 0; q < 2; ++q)
    for (int b = 0; b < 16; ++b) r[q][b] = threadIdx.x * 7919u + (q * 16 + b) * 104729u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    to_planes(r[0]);
    to_planes(r[1]);
    r[0][it & 15] ^= r[1][(it + 3) & 15];  // keep the round trips from folding away
    from_planes(r[0]);
    from_planes(r[1]);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int q = 0; q < 2; ++q)
    for (int b = 0; b < 16; ++b) x ^= r[q][b];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// correctness: acc = M y on lane-packed data converted to planes and back
__global__ void k_check(const uint32_t* in, const uint32_t* mats, uint32_t* out) {
  uint32_t y[16], acc[16];
  for (int b = 0; b < 16; ++b) {
    y[b] = in[threadIdx.x * 16 + b];
    acc[b] = 0;
  }
  to_planes(y);
  bs_mul(acc, y, mats);
  from_planes(acc);
  for (int b = 0; b < 16; ++b) out[threadIdx.x * 16 + b] = acc[b];
}

// host: plane p after to_planes holds element bit plane_bit[p]; element e of the lane sits at
// bit position elem_pos[e] (computed by applying the same swaps to index labels)
int main() {
  const int blocks = 256, threads = 1024;
  uint64_t* d_cyc;
  uint32_t* d_out;
  uint16_t* d_tabs;
  uint32_t* d_mats;
  hipMalloc(&d_cyc, blocks * 8);
  hipMalloc(&d_out, size_t(blocks) * threads * 4 * 16);
  hipMalloc(&d_tabs, NCONST * 256);
  hipMalloc(&d_mats, (NCONST + 4) * 64 * 4);
  std::vector<uint8_t> h(NCONST * 256);
  srand(7);
  for (auto& v : h) v = uint8_t(rand());
  hipMemcpy(d_tabs, h.data(), h.size(), hipMemcpyHostToDevice);
  std::vector<uint32_t> mats((NCONST + 4) * 64);  // [constant][group][row] nibble indices
  for (auto& v : mats) v = uint32_t(rand()) & 15u;
  hipMemcpy(d_mats, mats.data(), mats.size() * 4, hipMemcpyHostToDevice);

  // ---- correctness of the bit-sliced multiply (M given by its nibble indices) ----
  {
    // plane p (after to_planes) <-> element bit, by the index-bit mapping in the comment
    // above: word bits (w3 w2 w1 w0) = (j0 j3 j2 j1) -> element bit j = j3 j2 j1 j0
    auto plane_bit = [](int w) { return ((w & 7) << 1) | (w >> 3); };
    std::vector<uint32_t> in(64 * 16), got(64 * 16);
    for (auto& v : in) v = uint32_t(rand()) ^ (uint32_t(rand()) << 16);
    uint32_t* d_in;
    hipMalloc(&d_in, in.size() * 4);
    hipMemcpy(d_in, in.data(), in.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d_in, d_mats, d_out);
    hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost);
    // M[i][j] over planes: row i, input plane j = bit (j%4) of nibble idx[16*(j/4) + i]
    int bad = 0;
    for (int lane = 0; lane < 64; ++lane)
      for (int e = 0; e < 32; ++e) {
        const uint32_t xe = (in[lane * 16 + e / 2] >> (16 * (e & 1))) & 0xFFFFu;
        const uint32_t ge = (got[lane * 16 + e / 2] >> (16 * (e & 1))) & 0xFFFFu;
        uint32_t want = 0;
        for (int i = 0; i < 16; ++i) {
          uint32_t bit = 0;
          for (int j = 0; j < 16; ++j) {
            const uint32_t mij = (mats[16 * (j / 4) + i] >> (j % 4)) & 1u;
            bit ^= mij & ((xe >> plane_bit(j)) & 1u);
          }
          want |= bit << plane_bit(i);
        }
        bad += want != ge;
      }
    printf("check: %d of %d elements differ\n", bad, 64 * 32);
    hipFree(d_in);
  }

  std::vector<uint64_t> cyc(blocks);
  auto run = [&](const char* name, auto launch, double elem_mults_per_lane_iter) {
    for (int rep = 0; rep < 3; ++rep) {
      launch();
      hipDeviceSynchronize();
      hipMemcpy(cyc.data(), d_cyc, blocks * 8, hipMemcpyDeviceToHost);
      double avg = 0;
      for (auto c : cyc) avg += double(c);
      avg /= blocks;
      // s_memtime counts at the shader clock; per CU: 16 waves x 64 lanes
      const double per_cu = 16.0 * 64 * kIters * elem_mults_per_lane_iter;
      printf("%-5s rep %d: %.0f CU-cycles, %.3f element-mults per CU-cycle, %.2f CU-cycles per "
             "wave-level pair multiply\n", name, rep, avg, per_cu / avg, avg / (per_cu / 128.0));
    }
  };
  // prod: 16 gf multiplies per sweep per lane, 2 elements each
  run("prod", [&] { hipLaunchKernelGGL(k_prod, dim3(blocks), dim3(threads), kLds, 0, d_cyc, d_out, d_tabs); }, 32.0);
  // bs4r: 4 multiplies of 32 elements per sweep per lane
  run("bs4r", [&] { hipLaunchKernelGGL(k_bs4r, dim3(blocks), dim3(threads), kLds, 0, d_cyc, d_out, d_mats); }, 128.0);
  // conv: 2 round trips of 32 elements per iteration (reported per converted element, one way
  // = half a round trip)
  run("conv", [&] { hipLaunchKernelGGL(k_conv, dim3(blocks), dim3(threads), kLds, 0, d_cyc, d_out); }, 128.0);
  return 0;
}
