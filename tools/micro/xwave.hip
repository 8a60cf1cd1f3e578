// Prototype: the decode's cross-wave transform layers run bit-sliced, with
// the data regrouped between layers through LDS so that every wave holds whole groups of
// positions under one constant, against the codec's table multiply + transposes.
//
// One 16-wave workgroup per CU (1,024 lanes, ~144 KiB LDS), every lane holding 32 codeword-pair
// registers X of one 512-position block in the codec's "A" layout (position 32 w + i in register
// i of wave w), as rs2_codec.hip holds a block after its in-wave layers d = 1 .. 8.  One
// iteration is a round trip through the layers the codec runs across waves or on a wave-wide
// constant -- IFFT d = 16 .. 256, then FFT d = 256 .. 16 -- ending in the A layout again:
//
//   table (the codec today)  d = 16 in the A layout (one constant per wave), A -> B transpose
//      through LDS, d = 32 .. 256 in the B layout (position 16 i + w; rs2_codec.hip phase_b), the
//      FFT back the same way, B -> A transpose; every multiply is gf_mul2 (3 LDS lookups per
//      element into a 256-byte table, 15.5 VALU + 6 ds_read_u16 per register pair).
//   sliced  the 32 registers become two bit-sliced sets of 16 planes (set s = position bit 4, a
//      plane holds one element bit of the 16 positions x 2 lines of its set), so a layer whose
//      butterfly partner is the other set and whose constant is uniform over the wave is ONE
//      Four-Russians multiply of 16 planes (124 VALU + 68 SALU, tools/micro/bitslice.hip) for
//      32 elements per lane.  Layout L_k (k = 4 .. 8) keeps position bit k as the set index and
//      the other four of bits 4 .. 8 as the wave index, so layer 2^k is in-lane with the wave's
//      own constant (group = wave >> (k - 4)); L_k -> L_k+1 swaps one wave bit with the set
//      index: waves w and w ^ 2^(k-4) trade one set of 16 planes through LDS (4 ds_write_b128 +
//      4 ds_read_b128 per lane, one barrier, double-buffered).  4 such exchanges per direction,
//      2 plane conversions (5 delta-swap stages, 16 registers each) at each end.
//
// Both paths apply the same GF(2)-linear maps (random 16x16 bit matrices standing for the
// field constants; the sliced path's nibble indices are the same matrices with the planes'
// bit order folded in), so their outputs must agree bit for bit; the check runs first.
// Variants for the breakdown (timing only): sliced without the exchanges' LDS traffic
// (barriers kept), table without the transposes' LDS traffic.
// No layer is pruned here (the codec skips zero / unstored groups): this measures the layers'
// full cost per CU-cycle, s_memtime per workgroup, on 256 workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 -o bin/xwave xwave.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

constexpr int kIters = 64;
constexpr int kLds = 144 * 1024;  // table area 16 KiB + 128 KiB union, as the codec's C = 512 kernel
constexpr int kTabOff = 0;        // 62 tables of 256 B (IFFT 31, FFT 31)
constexpr int kUnion = 16 * 1024; // transpose buffer / exchange buffers (2 x 64 KiB)

typedef __attribute__((address_space(3))) uint32_t lds32;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u lds128;

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

// ---- the codec's table multiply (rs2_codec.hip RS2_GF_ADDR / RS2_GF_READS, mask register) ----
#define GF_ADDR(Y, A0, A1, A2, A3, A4, A5, M)                   \
  "v_add_u32 " A0 ", " Y ", " Y "\n"                             \
  "v_lshrrev_b32 " A1 ", 15, " Y "\n"                            \
  "v_bitop3_b32 " A0 ", " A0 ", " M ", %[tb] bitop3:0xEA\n"       \
  "v_bitop3_b32 " A1 ", " A1 ", " M ", %[tb] bitop3:0xEA\n"       \
  "v_lshrrev_b32 " A2 ", 5, " Y "\n"                             \
  "v_lshrrev_b32 " A3 ", 21, " Y "\n"                            \
  "v_lshrrev_b32 " A4 ", 10, " Y "\n"                            \
  "v_lshrrev_b32 " A5 ", 26, " Y "\n"                            \
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

// x1 ^= y1 * t, x2 ^= y2 * t (t = table at LDS byte address tb, 128-byte aligned)
__device__ __forceinline__ void gf_mul2(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                        uint32_t tb) {
  uint32_t a0, a1, a2, a3, a4, a5, c0, c1, c2, c3, c4, c5;
  asm volatile("v_mov_b32 %[c5], 0x7e\n"
               GF_ADDR("%[y1]", "%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[c5]")
               GF_READS("%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "0", "128", "192")
               GF_ADDR("%[y2]", "%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]", "%[c5]")
               GF_READS("%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]", "0", "128", "192")
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
               : [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb));
}

// table slots: direction dir (0 IFFT, 1 FFT) x layer k = 4 .. 8 x group g:
//   k = 4: 16 groups (one per wave), 5: 8, 6: 4, 7: 2, 8: 1 -> 31 per direction
__host__ __device__ constexpr int slot_of(int dir, int k, int g) {
  return dir * 31 + (k == 4 ? 0 : k == 5 ? 16 : k == 6 ? 24 : k == 7 ? 28 : 30) + g;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return uint32_t(uintptr_t(p)); }
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

// d = 16 in the A layout: registers i and i + 16, the wave's own constant
template <bool kFft>
__device__ __forceinline__ void layer_a16(uint32_t (&X)[32], uint32_t tb) {
  sfor<8>([&](auto qq) {
    constexpr int j = 2 * decltype(qq)::value;
    if constexpr (!kFft) {
      X[j + 16] ^= X[j];
      X[j + 17] ^= X[j + 1];
    }
    gf_mul2(X[j], X[j + 16], X[j + 1], X[j + 17], tb);
    if constexpr (kFft) {
      X[j + 16] ^= X[j];
      X[j + 17] ^= X[j + 1];
    }
  });
}

// d = 32 .. 256 in the B layout (register i = position 16 i + w): layer k, half-distance
// dr = 2^(k-4) registers, group g = registers [2 dr g, 2 dr (g + 1))
template <bool kFft, int k>
__device__ __forceinline__ void layer_b(uint32_t (&X)[32], uint32_t tabs, int dir) {
  constexpr int dr = 1 << (k - 4);
  sfor<16 / dr>([&](auto gg) {
    constexpr int g = decltype(gg)::value;
    const uint32_t tb = tabs + uint32_t(slot_of(dir, k, g)) * 256u;
    sfor<dr / 2>([&](auto qq) {
      constexpr int i = 2 * dr * g + 2 * decltype(qq)::value;
      if constexpr (!kFft) {
        X[i + dr] ^= X[i];
        X[i + 1 + dr] ^= X[i + 1];
      }
      gf_mul2(X[i], X[i + dr], X[i + 1], X[i + 1 + dr], opaque(tb));
      if constexpr (kFft) {
        X[i + dr] ^= X[i];
        X[i + 1 + dr] ^= X[i + 1];
      }
    });
  });
}

// A <-> B through the union region: word (w*32 + i)*64 + l (A) / (16 i + w)*64 + l (B)
template <bool kAtoB, bool kNoTx>
__device__ __forceinline__ void transpose(uint32_t (&X)[32], lds32* sU, int w, int l) {
  __syncthreads();
  lds32* pa = sU + w * 32 * 64 + l;
  lds32* pb = sU + w * 64 + l;
  if constexpr (!kNoTx)
    sfor<32>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      if constexpr (kAtoB) pa[i * 64] = X[i]; else pb[i * 16 * 64] = X[i];
    });
  __syncthreads();
  if constexpr (!kNoTx)
    sfor<32>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      if constexpr (kAtoB) X[i] = pb[i * 16 * 64]; else X[i] = pa[i * 64];
    });
}

// ---- bit-sliced multiply (tools/micro/bitslice.hip) ----------------------------------------
#define BS_ACC(i) "v_xor_b32 %[a" #i "], v112, %[a" #i "]\n"
#define BS_IDX(i) "s_set_gpr_idx_idx %[s" #i "]\n"
typedef __attribute__((address_space(4))) const uint32_t cu32;
__device__ __forceinline__ void bs_group(uint32_t* a, uint32_t y0, uint32_t y1, uint32_t y2,
                                         uint32_t y3, const uint32_t* sp) {
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
        "v123", "v124", "v125", "v126", "v127", "m0");
}
// acc (16 planes) ^= M y (16 planes); M as 64 nibble indices at idx
__device__ __forceinline__ void bs_mul(uint32_t* acc, const uint32_t* y, const uint32_t* idx) {
  sfor<4>([&](auto gg) {
    constexpr int g = decltype(gg)::value;
    bs_group(acc, y[4 * g], y[4 * g + 1], y[4 * g + 2], y[4 * g + 3], idx + 16 * g);
  });
}

// 16 registers (elements 2k | 2k+1 << 16) <-> 16 planes (bitslice.hip): plane p = element bit
// ((p & 7) << 1) | (p >> 3); element (register k, half j4) at bit (k3 k2 k1 k0 j4)
template <int WB, int PB>
__device__ __forceinline__ void delta_swap(uint32_t* r) {
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
      const uint32_t t = ((r[k] >> sh) ^ r[k + wd]) & mask;
      r[k + wd] ^= t;
      r[k] ^= t << sh;
    }
  });
}
__device__ __forceinline__ void to_planes(uint32_t* r) {
  delta_swap<3, 4>(r);
  delta_swap<2, 3>(r);
  delta_swap<1, 2>(r);
  delta_swap<0, 1>(r);
  delta_swap<3, 0>(r);
}
__device__ __forceinline__ void from_planes(uint32_t* r) {
  delta_swap<3, 0>(r);
  delta_swap<0, 1>(r);
  delta_swap<1, 2>(r);
  delta_swap<2, 3>(r);
  delta_swap<3, 4>(r);
}

// sliced layer k in L_k: set 0 = a (position bit k clear), set 1 = b; group = w >> (k - 4)
template <bool kFft>
__device__ __forceinline__ void layer_s(uint32_t (&X)[32], const uint32_t* idx) {
  if constexpr (!kFft) sfor<16>([&](auto ii) { X[16 + decltype(ii)::value] ^= X[decltype(ii)::value]; });
  bs_mul(X, X + 16, idx);
  if constexpr (kFft) sfor<16>([&](auto ii) { X[16 + decltype(ii)::value] ^= X[decltype(ii)::value]; });
}

// L_k <-> L_k+1: waves w and w ^ 2^m trade one set; the wave whose bit m is b sends set 1 - b
// and receives the partner's set b into its set 1 - b (buffer buf: 64 KiB, wave slot 4 KiB)
template <int m, bool kNoX>
__device__ __forceinline__ void exchange(uint32_t (&X)[32], lds32* sU, int w, int l, int buf) {
  const int b = (w >> m) & 1;
  lds128* mine = (lds128*)(sU + buf * 16384 + w * 1024) + l;
  lds128* part = (lds128*)(sU + buf * 16384 + (w ^ (1 << m)) * 1024) + l;
  auto body = [&](auto set) {
    constexpr int o = decltype(set)::value * 16;
    if constexpr (!kNoX)
      sfor<4>([&](auto qq) {
        constexpr int q = decltype(qq)::value;
        v4u v;
        v.x = X[o + 4 * q];
        v.y = X[o + 4 * q + 1];
        v.z = X[o + 4 * q + 2];
        v.w = X[o + 4 * q + 3];
        mine[q * 64] = v;
      });
    __syncthreads();
    if constexpr (!kNoX)
      sfor<4>([&](auto qq) {
        constexpr int q = decltype(qq)::value;
        const v4u v = part[q * 64];
        X[o + 4 * q] = v.x;
        X[o + 4 * q + 1] = v.y;
        X[o + 4 * q + 2] = v.z;
        X[o + 4 * q + 3] = v.w;
      });
  };
  if (b) body(std::integral_constant<int, 0>{}); else body(std::integral_constant<int, 1>{});
}

// sliced constants: [dir][k - 4][group][64] nibble indices (group < 16 >> (k - 4))
__device__ __forceinline__ const uint32_t* bs_idx(const uint32_t* mats, int dir, int k, int g) {
  return mats + size_t(slot_of(dir, k, g)) * 64;
}

// MODE 0 table, 1 sliced, 2 sliced without exchange traffic, 3 table without transposes;
// kLiveA: 32 more registers live across the loop (the decode's accumulator during its IFFTs)
template <int MODE, bool kLiveA = true>
__global__ void __launch_bounds__(1024) k_xwave(const uint32_t* in, uint32_t* out, uint64_t* cyc,
                                                const uint16_t* tabs, const uint32_t* mats,
                                                int iters) {
  __shared__ __attribute__((aligned(128))) uint8_t smem[kLds];
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // tables into LDS (62 x 256 B)
  for (int i = tid; i < 62 * 128; i += 1024)
    ((__attribute__((address_space(3))) uint16_t*)(smem + kTabOff))[i] = tabs[i];
  __syncthreads();
  lds32* sU = (lds32*)(smem + kUnion);
  const uint32_t tabs_l = lds_addr(smem + kTabOff);
  uint32_t X[32], A[32];
  const size_t base = (size_t(blockIdx.x) * 1024 + tid) * 32;
  sfor<32>([&](auto ii) {
    X[decltype(ii)::value] = in[base + decltype(ii)::value];
    A[decltype(ii)::value] = kLiveA ? in[base + decltype(ii)::value] * 2654435761u : 0u;
  });
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0 || MODE == 3) {
      constexpr bool nt = MODE == 3;
      layer_a16<false>(X, opaque(tabs_l + uint32_t(slot_of(0, 4, w)) * 256u));
      transpose<true, nt>(X, sU, w, l);
      layer_b<false, 5>(X, tabs_l, 0);
      layer_b<false, 6>(X, tabs_l, 0);
      layer_b<false, 7>(X, tabs_l, 0);
      layer_b<false, 8>(X, tabs_l, 0);
      layer_b<true, 8>(X, tabs_l, 1);
      layer_b<true, 7>(X, tabs_l, 1);
      layer_b<true, 6>(X, tabs_l, 1);
      layer_b<true, 5>(X, tabs_l, 1);
      transpose<false, nt>(X, sU, w, l);
      layer_a16<true>(X, opaque(tabs_l + uint32_t(slot_of(1, 4, w)) * 256u));
    } else {
      constexpr bool nx = MODE == 2;
      to_planes(X);
      to_planes(X + 16);
      layer_s<false>(X, bs_idx(mats, 0, 4, w));
      exchange<0, nx>(X, sU, w, l, 0);
      layer_s<false>(X, bs_idx(mats, 0, 5, w >> 1));
      exchange<1, nx>(X, sU, w, l, 1);
      layer_s<false>(X, bs_idx(mats, 0, 6, w >> 2));
      exchange<2, nx>(X, sU, w, l, 0);
      layer_s<false>(X, bs_idx(mats, 0, 7, w >> 3));
      exchange<3, nx>(X, sU, w, l, 1);
      layer_s<false>(X, bs_idx(mats, 0, 8, 0));
      layer_s<true>(X, bs_idx(mats, 1, 8, 0));
      exchange<3, nx>(X, sU, w, l, 0);
      layer_s<true>(X, bs_idx(mats, 1, 7, w >> 3));
      exchange<2, nx>(X, sU, w, l, 1);
      layer_s<true>(X, bs_idx(mats, 1, 6, w >> 2));
      exchange<1, nx>(X, sU, w, l, 0);
      layer_s<true>(X, bs_idx(mats, 1, 5, w >> 1));
      exchange<0, nx>(X, sU, w, l, 1);
      layer_s<true>(X, bs_idx(mats, 1, 4, w));
      from_planes(X);
      from_planes(X + 16);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sfor<32>([&](auto ii) {
    if constexpr (kLiveA) asm volatile("" : "+v"(A[decltype(ii)::value]));
    out[base + decltype(ii)::value] = X[decltype(ii)::value] ^ (A[decltype(ii)::value] & 0u);
  });
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

// ---- host -----------------------------------------------------------------------------------
static uint32_t rnd32() { return (uint32_t(rand()) << 16) ^ uint32_t(rand()); }
static int parity(uint32_t v) { return __builtin_popcount(v) & 1; }

int main() {
  const int blocks = 256, lanes = blocks * 1024;
  srand(11);
  // 62 random 16x16 bit matrices G[slot][r] = row r (mask over input element bits)
  std::vector<uint16_t> G(62 * 16);
  for (auto& v : G) v = uint16_t(rnd32());
  auto apply = [&](int slot, uint32_t x) {
    uint32_t y = 0;
    for (int r = 0; r < 16; ++r) y |= uint32_t(parity(G[slot * 16 + r] & x)) << r;
    return y;
  };
  // tables (rs2_engine.cpp nib_table layout): bits 0-5, 6-10, 11-15
  std::vector<uint16_t> tabs(62 * 128);
  for (int t = 0; t < 62; ++t) {
    for (int j = 0; j < 64; ++j) tabs[t * 128 + j] = uint16_t(apply(t, uint32_t(j)));
    for (int j = 0; j < 32; ++j) tabs[t * 128 + 64 + j] = uint16_t(apply(t, uint32_t(j) << 6));
    for (int j = 0; j < 32; ++j) tabs[t * 128 + 96 + j] = uint16_t(apply(t, uint32_t(j) << 11));
  }
  // sliced nibble indices: M[i][j] = G[pb(i)][pb(j)], idx[16 g + i] = sum_b M[i][4g + b] << b
  auto pb = [](int p) { return ((p & 7) << 1) | (p >> 3); };
  std::vector<uint32_t> mats(62 * 64);
  for (int t = 0; t < 62; ++t)
    for (int g = 0; g < 4; ++g)
      for (int i = 0; i < 16; ++i) {
        uint32_t v = 0;
        for (int b = 0; b < 4; ++b) v |= uint32_t((G[t * 16 + pb(i)] >> pb(4 * g + b)) & 1) << b;
        mats[t * 64 + 16 * g + i] = v;
      }
  std::vector<uint32_t> in(size_t(lanes) * 32), o0(in.size()), o1(in.size());
  for (auto& v : in) v = rnd32();
  uint32_t *d_in, *d_out, *d_mats;
  uint16_t* d_tabs;
  uint64_t* d_cyc;
  hipMalloc(&d_in, in.size() * 4);
  hipMalloc(&d_out, in.size() * 4);
  hipMalloc(&d_tabs, tabs.size() * 2);
  hipMalloc(&d_mats, mats.size() * 4);
  hipMalloc(&d_cyc, blocks * 8);
  hipMemcpy(d_in, in.data(), in.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_tabs, tabs.data(), tabs.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(d_mats, mats.data(), mats.size() * 4, hipMemcpyHostToDevice);
  // correctness: one iteration of each path, same input
  hipLaunchKernelGGL((k_xwave<0, true>), dim3(blocks), dim3(1024), 0, 0, d_in, d_out, d_cyc, d_tabs, d_mats, 1);
  hipMemcpy(o0.data(), d_out, o0.size() * 4, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL((k_xwave<1, true>), dim3(blocks), dim3(1024), 0, 0, d_in, d_out, d_cyc, d_tabs, d_mats, 1);
  hipMemcpy(o1.data(), d_out, o1.size() * 4, hipMemcpyDeviceToHost);
  size_t bad = 0, same_in = 0;
  for (size_t i = 0; i < o0.size(); ++i) {
    bad += o0[i] != o1[i];
    same_in += o0[i] == in[i];
  }
  printf("check: %zu of %zu words differ between the table and sliced paths (%zu equal to the input)\n",
         bad, o0.size(), same_in);
  const char* names[6] = {"table (gf_mul2 + transposes)", "sliced (Four-Russians + exchanges)",
                          "sliced, no exchange traffic", "table, no transpose traffic",
                          "table, accumulator not live", "sliced, accumulator not live"};
  std::vector<uint64_t> cyc(blocks);
  for (int mode = 0; mode < 6; ++mode)
    for (int rep = 0; rep < 3; ++rep) {
#define XW(M, A) hipLaunchKernelGGL((k_xwave<M, A>), dim3(blocks), dim3(1024), 0, 0, d_in, d_out, d_cyc, d_tabs, d_mats, kIters)
      if (mode == 0) XW(0, true);
      if (mode == 1) XW(1, true);
      if (mode == 2) XW(2, true);
      if (mode == 3) XW(3, true);
      if (mode == 4) XW(0, false);
      if (mode == 5) XW(1, false);
      hipDeviceSynchronize();
      hipMemcpy(cyc.data(), d_cyc, blocks * 8, hipMemcpyDeviceToHost);
      double avg = 0;
      for (auto c : cyc) avg += double(c);
      avg /= blocks;
      printf("%-38s rep %d: %8.0f CU-cycles per round trip (IFFT d=16..256 + FFT d=256..16, 16 waves)\n",
             names[mode], rep, avg / kIters);
    }
  return bad ? 1 : 0;
}
