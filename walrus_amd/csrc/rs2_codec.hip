// Block codec kernel of the MI355X Red Stuff engine (gfx950): batched GF(2^16) additive-FFT
// Reed-Solomon encode/decode with reed-solomon-simd 3.1.0 semantics (oracle/rs2_oracle.py).
//
// Compiled once per block size:  hipcc -DRS2_C=<C> rs2_codec.hip  (C = 1, 2, ..., 512).
//
// Mapping
//   lane   one "codeword pair": two adjacent GF(2^16) elements of a symbol, packed in a u32
//   wave   PPW = min(C, kPpwTarget) codeword positions held in VGPRs, "A" layout: p = w*PPW + i
//   block  NW = C/PPW waves.  Layers whose butterfly partner sits in another wave run after an
//          in-place LDS transpose into the "B" layout p = NW*i + w.
// Every butterfly constant depends only on the position, so it is uniform across the wave: a
// multiply is 3 lookups per element into one 256-byte table in LDS (u16 sub-tables of 64, 32
// and 32 entries for operand bits 0-5, 6-10, 11-15: at most 32 dwords each, conflict-free).
// No MFMA: no step of an additive FFT is a dense matrix product.
//
// LDS: one 128 KiB union region (C = 512) time-shared by the in-place transpose buffer and one
// private 8 KiB slab per wave, which holds either the wave's in-wave layer tables or its
// per-position multiplier tables; plus the small cross-wave-layer and mixing tables.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "rs2_device.h"

#ifndef RS2_C
#error "compile with -DRS2_C=<block size>"
#endif

namespace rs2 {
namespace {

// Explicit address spaces: every table lookup must be a ds_read and every symbol access a
// global_load/store (generic flat pointers cost 64-bit address VGPRs and flat instructions).
#if defined(__HIP_DEVICE_COMPILE__)
#define RS2_AS(n) __attribute__((address_space(n)))
#else
#define RS2_AS(n)
#endif
typedef RS2_AS(3) uint16_t lds16;
typedef RS2_AS(3) uint32_t lds32;
typedef RS2_AS(3) uint4 lds128;
typedef RS2_AS(1) uint8_t g8;
typedef RS2_AS(1) uint16_t g16;
typedef RS2_AS(1) const uint4 gc128;
typedef RS2_AS(1) const int64_t gci64;

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

#define RS2_INL __attribute__((always_inline))

// The lane id, recomputed (2 VALU) where it is used: a volatile asm is never CSE'd, so the
// transposes' LDS addresses built from it are not computed once at kernel entry and kept live
// through the transforms (in the decode kernel they were spill slots)
__device__ __forceinline__ int fresh_lane() {
  uint32_t v;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
  return int(v);
}
// Diagnostic ablation knobs (variant builds only, tools/build_variant.sh; outputs are wrong in
// such builds; every other build of this file is the product kernel):
//   RS2_ABL_NOLOAD   skip the symbol loads   RS2_ABL_NOPHASE  skip the butterfly layers
//   RS2_ABL_NOSTAGE  skip the table staging  RS2_ABL_NOSTORE  skip the symbol stores
#ifndef RS2_ABL_NOLOAD
#define RS2_ABL_NOLOAD 0
#endif
#ifndef RS2_ABL_NOPHASE
#define RS2_ABL_NOPHASE 0
#endif
#ifndef RS2_ABL_NOSTAGE
#define RS2_ABL_NOSTAGE 0
#endif
#ifndef RS2_ABL_NOSTORE
#define RS2_ABL_NOSTORE 0
#endif
#ifndef RS2_ABL_NOPRE  // skip the decode's per-position pre / post multiplies
#define RS2_ABL_NOPRE 0
#endif
#ifndef RS2_ABL_NOTX  // skip the transposes' LDS data movement (barriers kept)
#define RS2_ABL_NOTX 0
#endif
#ifndef RS2_ABL_NOCOPY  // skip the fused copy-outs of the pipelined encode kernels
#define RS2_ABL_NOCOPY 0
#endif

#ifndef RS2_STAMPS
#define RS2_STAMPS 0
#endif
// (stamps only in the C = 512 kernels: the diagnostic stores change the smaller kernels' code
// enough to hit a gfx950 backend error on an LDS null check)
#define RS2_STAMPS_ON (RS2_STAMPS && RS2_C == 512)
// butterflies between scheduling barriers (bounds VGPR pressure; windows 2..8 within 0.2 %)
constexpr int kWin = 4;

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

constexpr int kPreOut = 3;  // output-table slots (0 = stage per output block)

template <int C_, int P_ = kPpwTarget>
struct Geo {
  static constexpr int C = C_;
  static constexpr int NW = C >= P_ ? C / P_ : 1;     // waves per workgroup
  static constexpr int PPW = C / NW;                  // positions (VGPRs) per wave
  static constexpr int LOGC = ilog2(C);
  static constexpr int LOGP = ilog2(PPW);
  static constexpr int LOGW = LOGC - LOGP;
  static constexpr int NTA = PPW > 1 ? PPW - 1 : 0;   // in-wave layer tables per wave
  static constexpr int NTB = NW - 1;                  // cross-wave layer tables
  static constexpr int THREADS = NW * 64;
  static constexpr int TAB_BYTES = kTabU16 * 2;
  static constexpr int TABB_BYTES = kTabU16 * 2;                     // cross-wave tables
  // union region (u32 words): the full transpose buffer (C*64 words), or one private slab per
  // wave holding either its NTA in-wave layer tables or its PPW per-position tables
  static constexpr int SLAB_WORDS = cmax(PPW, NTA) * kTabU16 / 2;
  static constexpr int U_WORDS = cmax(NW > 1 ? C * 64 : 0, NW * SLAB_WORDS + 4);
  // one LDS array: small constant tables first (addresses fit the 16-bit DS offset field,
  // so their lookups need no base VGPR), then the union region
  static constexpr int OFF_TB = 0;                                   // cross-wave tables
  static constexpr int TB_SLOT = ((NTB * TABB_BYTES + 15) / 16) * 16;
  // the output blocks' cross-wave FFT tables, staged once with the first input block (jobs of
  // at most kPreOut output blocks per workgroup), so an FFT starts without a table wait --
  // a wait that would also drain the previous output block's stores (vmcnt counts them)
  static constexpr int OFF_TO = OFF_TB + TB_SLOT;
  static constexpr int OFF_TM = OFF_TO + kPreOut * TB_SLOT;          // mixing tables
  // decode block pairs (CodecJob::pair_p): the second block's cross-wave and mixing tables
  static constexpr int OFF_TQ = OFF_TM + 2 * kTabU16 * 2;
  static constexpr int OFF_TMQ = OFF_TQ + TB_SLOT;
  static constexpr int OFF_U = OFF_TMQ + 2 * kTabU16 * 2;            // union region
  static constexpr int LDS_BYTES = OFF_U + U_WORDS * 4;
  // every table base is OR-ed into its lookup addresses (gf_mul): 128-byte aligned
  static_assert(OFF_TO % 128 == 0 && OFF_TM % 128 == 0 && OFF_TQ % 128 == 0 &&
                    OFF_TMQ % 128 == 0 && OFF_U % 128 == 0 && (SLAB_WORDS * 4) % 128 == 0 &&
                    TB_SLOT % 128 == 0,
                "LDS table bases must be 128-byte aligned");
};

// x * c for both packed elements of v; t = c's 256-byte table in LDS (reference form, kept for
// the reading of the algorithm; the kernel uses gf_mul below).
__device__ __forceinline__ uint32_t tab_mul(uint32_t v, const lds16* t) {
  const uint32_t a = uint32_t(t[v & 63u]) ^ t[64 + ((v >> 6) & 31u)] ^ t[96 + ((v >> 11) & 31u)];
  const uint32_t b = uint32_t(t[(v >> 16) & 63u]) ^ t[64 + ((v >> 22) & 31u)] ^
                     t[96 + (v >> 27)];
  return a | (b << 16);
}

// x (^)= y * c with c's 256-byte table at LDS byte address tb + OFF (tb 128-byte aligned).
// y = [e0 lo, e0 hi, e1 lo, e1 hi].  The six table addresses are 2 * (a field of e0 / e1) OR tb:
//   e0 bits 0-5: (y + y) & 0x7e        e1 bits 0-5: (y >> 15) & 0x7e     (sub-table at +0)
//   e0 bits 6-10: (y >> 5) & 0x3e      e1 bits 6-10: (y >> 21) & 0x3e    (+128)
//   e0 bits 11-15: (y >> 10) & 0x3e    e1 bits 11-15: (y >> 26) & 0x3e   (+192)
// Only full-rate VALU forms (tools/micro/valubench.hip, 4 waves/SIMD: v_add / v_or / v_and /
// right shifts ~2.1 cycles, v_bitop3 with VGPR / inline operands 2.35): SDWA, left shifts,
// v_and_or, v_perm and any SGPR operand issue at half rate (~4.1), and the SDWA form of this
// multiply cost 53 SIMD-cycles per element pair against 34 here.  The multiply is then bound by
// its 6 ds_read_u16 (2.23 CU-cycles each, tools/micro/ldsbench.hip: 16.8 -> 14.3 CU-cycles per
// wave-level pair multiply).  e0's entries load with ds_read_u16 (zero-extended), e1's with
// ds_read_u16_d16_hi, which on gfx950 fills the high half and ZEROES the low half
// (tools/micro/mulcheck.hip), so the 6 registers XOR straight into the packed product.  Loads
// land in their own address registers: a DS instruction reads its address VGPR at issue.
// 0x7e is not an inline constant and gfx950 VOP3 takes no literal, so the two 6-bit fields'
// masks come from a register M holding 0x7e (one v_mov per multiply block, shared by both
// multiplies of gf_mul2): every address is one shift (or add) and one v_bitop3, 12 VALU per
// element pair instead of 14 with separate v_and / v_or.  M may be A5: its own shift comes after
// the masks' last use.
#define RS2_GF_ADDR(Y, A0, A1, A2, A3, A4, A5, M)               \
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
#define RS2_GF_READS(A0, A1, A2, A3, A4, A5, O0, O1, O2)        \
  "ds_read_u16 " A0 ", " A0 " offset:" O0 "\n"                   \
  "ds_read_u16_d16_hi " A1 ", " A1 " offset:" O0 "\n"            \
  "ds_read_u16 " A2 ", " A2 " offset:" O1 "\n"                   \
  "ds_read_u16_d16_hi " A3 ", " A3 " offset:" O1 "\n"            \
  "ds_read_u16 " A4 ", " A4 " offset:" O2 "\n"                   \
  "ds_read_u16_d16_hi " A5 ", " A5 " offset:" O2 "\n"
#define RS2_GF_MUL_BODY                                                          \
  "v_mov_b32 %[a5], 0x7e\n"                                                       \
  RS2_GF_ADDR("%[y]", "%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[a5]") \
  RS2_GF_READS("%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[o0]", "%[o1]", "%[o2]") \
  "s_waitcnt lgkmcnt(0)\n"

template <int OFF, bool kAcc>
__device__ __forceinline__ void gf_mul(uint32_t& x, uint32_t y, uint32_t tb) {
  static_assert(OFF >= 0 && OFF + 192 < 65536, "DS offset field is 16 bits");
  uint32_t a0, a1, a2, a3, a4, a5;
  if constexpr (kAcc) {
    asm volatile(RS2_GF_MUL_BODY
                 "v_bitop3_b32 %[x], %[x], %[a0], %[a1] bitop3:0x96\n"
                 "v_bitop3_b32 %[x], %[x], %[a2], %[a3] bitop3:0x96\n"
                 "v_bitop3_b32 %[x], %[x], %[a4], %[a5] bitop3:0x96\n"
                 : [x] "+v"(x), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3),
                   [a4] "=&v"(a4), [a5] "=&v"(a5)
                 : [y] "v"(y), [tb] "v"(tb), [o0] "i"(OFF), [o1] "i"(OFF + 128),
                   [o2] "i"(OFF + 192));
  } else {
    asm volatile(RS2_GF_MUL_BODY
                 "v_bitop3_b32 %[x], %[a0], %[a1], %[a2] bitop3:0x96\n"
                 "v_bitop3_b32 %[x], %[x], %[a3], %[a4] bitop3:0x96\n"
                 "v_xor_b32 %[x], %[x], %[a5]\n"
                 : [x] "=&v"(x), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3),
                   [a4] "=&v"(a4), [a5] "=&v"(a5)
                 : [y] "v"(y), [tb] "v"(tb), [o0] "i"(OFF), [o1] "i"(OFF + 128),
                   [o2] "i"(OFF + 192));
  }
}

// Two independent multiplies in one block: both sets of table reads are in flight before the
// first result is waited for (lgkmcnt(6): LDS returns in order), which halves the exposed LDS
// latency per multiply.  12 temporaries.
template <int OFF1, int OFF2, bool kAcc>
__device__ __forceinline__ void gf_mul2(uint32_t& x1, uint32_t y1, uint32_t& x2, uint32_t y2,
                                        uint32_t tb) {
  static_assert(OFF1 >= 0 && OFF1 + 192 < 65536 && OFF2 >= 0 && OFF2 + 192 < 65536,
                "DS offset field is 16 bits");
  uint32_t a0, a1, a2, a3, a4, a5, c0, c1, c2, c3, c4, c5;
#define RS2_GF_MUL2_BODY                                                              \
  "v_mov_b32 %[c5], 0x7e\n"                                                             \
  RS2_GF_ADDR("%[y1]", "%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[c5]")  \
  RS2_GF_READS("%[a0]", "%[a1]", "%[a2]", "%[a3]", "%[a4]", "%[a5]", "%[p0]", "%[p1]", "%[p2]") \
  RS2_GF_ADDR("%[y2]", "%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]", "%[c5]")  \
  RS2_GF_READS("%[c0]", "%[c1]", "%[c2]", "%[c3]", "%[c4]", "%[c5]", "%[q0]", "%[q1]", "%[q2]") \
  "s_waitcnt lgkmcnt(6)\n"
#define RS2_GF_MUL2_OPS                                                                     \
  [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4),            \
      [a5] "=&v"(a5), [c0] "=&v"(c0), [c1] "=&v"(c1), [c2] "=&v"(c2), [c3] "=&v"(c3),        \
      [c4] "=&v"(c4), [c5] "=&v"(c5)
#define RS2_GF_MUL2_INS                                                                     \
  [y1] "v"(y1), [y2] "v"(y2), [tb] "v"(tb), [p0] "i"(OFF1), [p1] "i"(OFF1 + 128),            \
      [p2] "i"(OFF1 + 192), [q0] "i"(OFF2), [q1] "i"(OFF2 + 128), [q2] "i"(OFF2 + 192)
  if constexpr (kAcc) {
    asm volatile(RS2_GF_MUL2_BODY
                 "v_bitop3_b32 %[x1], %[x1], %[a0], %[a1] bitop3:0x96\n"
                 "v_bitop3_b32 %[x1], %[x1], %[a2], %[a3] bitop3:0x96\n"
                 "v_bitop3_b32 %[x1], %[x1], %[a4], %[a5] bitop3:0x96\n"
                 "s_waitcnt lgkmcnt(0)\n"
                 "v_bitop3_b32 %[x2], %[x2], %[c0], %[c1] bitop3:0x96\n"
                 "v_bitop3_b32 %[x2], %[x2], %[c2], %[c3] bitop3:0x96\n"
                 "v_bitop3_b32 %[x2], %[x2], %[c4], %[c5] bitop3:0x96\n"
                 : [x1] "+v"(x1), [x2] "+v"(x2), RS2_GF_MUL2_OPS
                 : RS2_GF_MUL2_INS);
  } else {
    asm volatile(RS2_GF_MUL2_BODY
                 "v_bitop3_b32 %[x1], %[a0], %[a1], %[a2] bitop3:0x96\n"
                 "v_bitop3_b32 %[x1], %[x1], %[a3], %[a4] bitop3:0x96\n"
                 "v_xor_b32 %[x1], %[x1], %[a5]\n"
                 "s_waitcnt lgkmcnt(0)\n"
                 "v_bitop3_b32 %[x2], %[c0], %[c1], %[c2] bitop3:0x96\n"
                 "v_bitop3_b32 %[x2], %[x2], %[c3], %[c4] bitop3:0x96\n"
                 "v_xor_b32 %[x2], %[x2], %[c5]\n"
                 : [x1] "=&v"(x1), [x2] "=&v"(x2), RS2_GF_MUL2_OPS
                 : RS2_GF_MUL2_INS);
  }
#undef RS2_GF_MUL2_BODY
#undef RS2_GF_MUL2_OPS
#undef RS2_GF_MUL2_INS
}

// Bijection workgroup id -> tile id that gives each XCD a contiguous tile range (see codec_body).
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t xcd_tile(uint32_t bid, uint32_t n) {
  const uint32_t x = bid % kXcds, k = bid / kXcds, q = n / kXcds, r = n % kXcds;
  return x * q + (x < r ? x : r) + k;
}

// Wave-private LDS handoff: every earlier LDS access of this wave -- including the reads inside
// the gf_mul asm blocks, which the compiler does not track -- completes before any later one,
// and the compiler moves no memory access across it.
__device__ __forceinline__ void wave_lds_handoff() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return uint32_t(reinterpret_cast<uintptr_t>(p));
}

// Global -> LDS without VGPRs (gfx950 global_load_lds_dwordx4): each lane's 16 bytes land at
// the wave-uniform LDS base + 16*lane, 1 KiB per wave-instruction, and every chunk of a table
// is in flight at once (a register copy loop waits out one L2 round trip per chunk).  The data
// is usable after lds_dma_wait() -- plus a barrier when other waves read it.  LDS-DMA loads
// count in vmcnt and return in order with the symbol loads, so waiting for a later symbol load
// also covers them.
typedef RS2_AS(3) void lds_void;
// Wave-uniform symbol base pinned in an SGPR pair: `ubase + lane_offset_u32` then selects
// global_load/store's saddr form (no per-lane 64-bit address arithmetic).
template <typename T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
  uint64_t v = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+s"(v));
  return reinterpret_cast<T*>(v);
}

// Chunk k of a transfer: the wave-uniform source base stays in SGPRs and the lane's 32-bit
// offset selects the saddr form (no per-lane 64-bit address add); only a transfer's partial
// last chunk tests the lane against its end.
template <int NBYTES, int k>
__device__ __forceinline__ void dma_chunk(lds_void* dst, const uint8_t* sbase, uint32_t lo, int l) {
  if ((k + 1) * 1024 <= NBYTES || k * 1024 + l * 16 < NBYTES)
    __builtin_amdgcn_global_load_lds(sbase + (uint32_t(k * 1024) + lo),
                                     reinterpret_cast<RS2_AS(3) uint8_t*>(dst) + k * 1024, 16, 0, 0);
}
template <int NBYTES, bool kRev = false>
__device__ __forceinline__ void dma_wave(lds_void* dst, const void* src, int l) {
  static_assert(NBYTES % 16 == 0, "16-byte chunks");
  if constexpr (RS2_ABL_NOSTAGE) return;
  constexpr int NCH = (NBYTES + 1023) / 1024;
  const uint8_t* sb = sgpr_ptr(reinterpret_cast<const uint8_t*>(src));
  const uint32_t lo = uint32_t(l) * 16u;
  sfor<NCH>([&](auto kk) RS2_INL {
    constexpr int k = kRev ? NCH - 1 - decltype(kk)::value : decltype(kk)::value;
    dma_chunk<NBYTES, k>(dst, sb, lo, l);
  });
}
// chunks [K0, K1) only (in order) of the same transfer
template <int NBYTES, int K0, int K1>
__device__ __forceinline__ void dma_wave_range(lds_void* dst, const void* src, int l) {
  static_assert(NBYTES % 16 == 0 && K0 <= K1, "16-byte chunks");
  if constexpr (RS2_ABL_NOSTAGE) return;
  const uint8_t* sb = sgpr_ptr(reinterpret_cast<const uint8_t*>(src));
  const uint32_t lo = uint32_t(l) * 16u;
  sfor<K1 - K0>([&](auto kk) RS2_INL { dma_chunk<NBYTES, K0 + decltype(kk)::value>(dst, sb, lo, l); });
}
// a table shared by the workgroup: wave w moves 1 KiB chunks w, w + NW, ...
template <int NBYTES, int NW>
__device__ __forceinline__ void dma_group(lds_void* dst, const void* src, int w, int l) {
  static_assert(NBYTES % 16 == 0, "16-byte chunks");
  if constexpr (RS2_ABL_NOSTAGE) return;
  const uint8_t* sb = sgpr_ptr(reinterpret_cast<const uint8_t*>(src));
  const uint32_t lo = uint32_t(l) * 16u;
  sfor<(NBYTES + 1023) / 1024>([&](auto kk) RS2_INL {
    constexpr int k = decltype(kk)::value;
    if (k % NW == w) dma_chunk<NBYTES, k>(dst, sb, lo, l);
  });
}
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// symbol bytes <-> packed element pair (reed-solomon-simd shard layout)
//   full 64-byte chunk q: element 32q+j = b[64q+j] | b[64q+32+j] << 8
//   tail t = s % 64:      element 32Q+j = b[64Q+j] | b[64Q+t/2+j] << 8
struct PairLoc {
  int lo, hi;
  bool fast, v0, v1;
};

__device__ __forceinline__ PairLoc pair_loc(int pair, int s) {
  PairLoc L;
  const int E = s >> 1, e0 = pair * 2;
  L.v0 = e0 < E;
  L.v1 = e0 + 1 < E;
  const int Q = s >> 6, th = (s & 63) >> 1, q = e0 >> 5, j = e0 & 31;
  if (q < Q) {
    L.lo = 64 * q + j;
    L.hi = L.lo + 32;
    L.fast = true;
  } else {
    L.lo = 64 * Q + j;
    L.hi = 64 * Q + th + j;
    L.fast = false;
  }
  return L;
}

__device__ __forceinline__ uint32_t load_pair(const g8* sym, const PairLoc& L) {
  if (L.fast) {
    const uint32_t lo = *reinterpret_cast<const g16*>(sym + L.lo);
    const uint32_t hi = *reinterpret_cast<const g16*>(sym + L.hi);
    return (lo & 0xFFu) | ((hi & 0xFFu) << 8) | ((lo & 0xFF00u) << 8) | ((hi & 0xFF00u) << 16);
  }
  uint32_t r = 0;
  if (L.v0) r = uint32_t(sym[L.lo]) | (uint32_t(sym[L.hi]) << 8);
  if (L.v1) r |= (uint32_t(sym[L.lo + 1]) << 16) | (uint32_t(sym[L.hi + 1]) << 24);
  return r;
}

__device__ __forceinline__ void store_pair(g8* sym, int64_t off, int64_t limit,
                                           const PairLoc& L, uint32_t v) {
  if (L.fast && off + L.hi + 2 <= limit) {
    *reinterpret_cast<g16*>(sym + L.lo) = uint16_t((v & 0xFFu) | ((v >> 8) & 0xFF00u));
    *reinterpret_cast<g16*>(sym + L.hi) = uint16_t(((v >> 8) & 0xFFu) | ((v >> 16) & 0xFF00u));
    return;
  }
  if (L.v0) {
    if (off + L.lo < limit) sym[L.lo] = uint8_t(v);
    if (off + L.hi < limit) sym[L.hi] = uint8_t(v >> 8);
  }
  if (L.v1) {
    if (off + L.lo + 1 < limit) sym[L.lo + 1] = uint8_t(v >> 16);
    if (off + L.hi + 1 < limit) sym[L.hi + 1] = uint8_t(v >> 24);
  }
}

// ---- symbol I/O ---------------------------------------------------------------------------
// Lanes 2m and 2m+1 hold element pairs (4m', 4m'+1) and (4m'+2, 4m'+3) of one 64-byte chunk
// (m' = m mod 8): the even lane moves the chunk's lo-byte dword of those 4 elements, the odd
// lane the hi-byte dword; a DPP quad swap and one v_perm convert between that and the packed
// pairs.  One dword per lane per position, a wave covering 4 whole chunks (256 contiguous bytes).
// Full chunks use (possibly 2-byte-misaligned) dword accesses; the tail chunk of a symbol
// (t = s % 64 bytes: t/2 lo bytes then t/2 hi bytes) uses two aligned dword loads and an
// alignbyte, never touching a dword that holds no byte of the symbol.
typedef RS2_AS(1) uint32_t g32;
typedef RS2_AS(1) const uint32_t gc32;

// Symbol stores (outputs and fused copy-outs).  (Rejected: non-temporal stores -- row codec
// 0.413 -> 0.375 ms but cols_sys 0.804 -> 0.857, step 82.0 vs 82.4 GiB/s, profiles/r03/exp/ntstore/.)
__device__ __forceinline__ void st32(g32* p, uint32_t v) { *p = v; }

__device__ __forceinline__ uint32_t swap_adjacent(uint32_t v) {  // value of lane l ^ 1
  return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t lane_odd() {
  uint32_t v = __lane_id() & 1u;
  asm volatile("" : "+v"(v));
  return v;
}
// (partner dword, own dword) -> own packed pair;  (partner pair, own pair) -> own dword
__device__ __forceinline__ uint32_t sel_load() { return lane_odd() ? 0x03070206u : 0x05010400u; }
__device__ __forceinline__ uint32_t sel_store() { return lane_odd() ? 0x03010705u : 0x06040200u; }

// A value read across lanes (readlane) inside lane-divergent code must stay live in EVERY lane
// through that code: the register allocator tracks liveness per lane, so a value whose last use
// is inside a branch may have its register reused for the lanes the branch excludes -- which a
// readlane of one of those lanes then returns (seen as wild store addresses).  A use at full exec
// after the branch keeps it live in every lane.
__device__ __forceinline__ void keep_live(int64_t v) {
  asm volatile("" ::"v"(uint32_t(v)), "v"(uint32_t(uint64_t(v) >> 32)));
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(v), lane);
  const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(uint64_t(v) >> 32), lane);
  return int64_t(uint64_t(lo) | (uint64_t(hi) << 32));
}


// Opaque copy of an LDS pointer: stops LICM from hoisting the (many) per-table addresses
// derived from it out of the block / output loops, which would pin ~4 VGPRs per table.
__device__ __forceinline__ const lds16* launder(const lds16* p) {
  uint32_t v = uint32_t(reinterpret_cast<uintptr_t>(p));
  asm volatile("" : "+v"(v));
  return reinterpret_cast<const lds16*>(uintptr_t(v));
}
__device__ __forceinline__ lds32* launder32(lds32* p) {
  uint32_t v = uint32_t(reinterpret_cast<uintptr_t>(p));
  asm volatile("" : "+v"(v));
  return reinterpret_cast<lds32*>(uintptr_t(v));
}

// Opaque register values: stops instcombine/reassociate from flattening the XOR chains of
// consecutive transform phases into long trees that keep every earlier value alive.
template <int N>
__device__ __forceinline__ void fence_regs(uint32_t (&X)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(X[i]));
}

// In-wave layers d = 1 .. PPW/2 (A layout).  Table slot of group g at half-distance d:
// PPW - PPW/d + g  (sd_stream order in rs2_engine.cpp).
// kStaged: the wave's layer tables are still arriving by LDS-DMA, 1 KiB chunks issued in slot
// order for the IFFT (whose first layer, d = 1, reads slots 0 .. PPW/2-1) and in reverse order
// for the FFT (whose first layer reads the last slot); each layer waits only for the chunks
// holding its own slots (s_waitcnt vmcnt(n) counts the chunks still allowed in flight; VMEM
// operations complete in issue order), so the later chunks land under the earlier layers.
// KLO / KHI: only layers k in [KLO, KHI) (table slots counted from SLOT0: a wave's slab holds
// one stage of its tables at a time when all of them do not fit; git history: rs2_cols2)
template <class G, bool kFft, bool kStaged = false, int KLO = 0, int KHI = G::LOGP, int SLOT0 = 0,
          int EXTRA = 0>
__device__ __forceinline__ void phase_a(uint32_t (&X)[G::PPW], const lds16* tabw_in) {
  const uint32_t tabw = lds_addr(launder(tabw_in));
  fence_regs(X);
  if constexpr (RS2_ABL_NOPHASE) return;
  sfor<KHI - KLO>([&](auto kk) RS2_INL {
    constexpr int k = KLO + decltype(kk)::value;
    constexpr int d = kFft ? (G::PPW >> (k + 1)) : (1 << k);
    if constexpr (kStaged) {
      constexpr int chunks = (G::NTA * G::TAB_BYTES + 1023) / 1024;
      constexpr int lo = G::PPW - G::PPW / d, hi = G::PPW - G::PPW / (2 * d) - 1;  // slots
      constexpr int in_flight = kFft ? (lo * G::TAB_BYTES) / 1024
                                     : chunks - 1 - (hi * G::TAB_BYTES + G::TAB_BYTES - 1) / 1024;
      // EXTRA: younger VMEM operations issued after the table chunks (the post tables' DMA)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(in_flight + EXTRA) : "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    constexpr int NB = G::PPW / 2;  // butterflies in the layer: bf = g*d + j, x register 2dg + j
    auto xreg = [](int bf) constexpr { return 2 * d * (bf / d) + bf % d; };
    auto toff = [](int bf) constexpr {
      return (G::PPW - G::PPW / d + bf / d - SLOT0) * G::TAB_BYTES;
    };
    sfor<(NB + 1) / 2>([&](auto qq) RS2_INL {
      constexpr int b1 = 2 * decltype(qq)::value, b2 = b1 + 1;
      constexpr int i1 = xreg(b1), t1 = toff(b1);
      if constexpr (b2 < NB) {
        constexpr int i2 = xreg(b2), t2 = toff(b2);
        if constexpr (kFft) {
          gf_mul2<t1, t2, true>(X[i1], X[i1 + d], X[i2], X[i2 + d], tabw);
          X[i1 + d] ^= X[i1];
          X[i2 + d] ^= X[i2];
        } else {
          X[i1 + d] ^= X[i1];
          X[i2 + d] ^= X[i2];
          gf_mul2<t1, t2, true>(X[i1], X[i1 + d], X[i2], X[i2 + d], tabw);
        }
      } else if constexpr (kFft) {
        gf_mul<t1, true>(X[i1], X[i1 + d], tabw);
        X[i1 + d] ^= X[i1];
      } else {
        X[i1 + d] ^= X[i1];
        gf_mul<t1, true>(X[i1], X[i1 + d], tabw);
      }
      if constexpr ((b2 % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
    });
  });
  fence_regs(X);
}

// Cross-wave layers d = PPW .. C/2 (B layout, register i holds position NW*i + w).
// Table slot of group g at half-distance d: NW - C/d + g; the group's x registers are
// i = 2*dr*g + j (j < dr), its y registers i + dr.
// Pruning (wave-uniform, so plain scalar branches):
//   bound    IFFT: positions >= bound are zero on input, so before layer d everything at or past
//            roundup(bound, d) is still zero and a group starting there is skipped;
//            FFT: only outputs < bound are stored, and a group starting at or past bound feeds
//            nothing below it, so it is skipped.
//   zero_g0  skew offset 0: group 0 of every layer has constant skew[d - 1] = log 0, i.e. it
//            multiplies by zero and its butterflies are a bare XOR.
template <class G, bool kFft>
__device__ __forceinline__ void phase_b(uint32_t (&Y)[G::PPW], const lds16* tabB_in,
                                        int bound, bool zero_g0) {
  constexpr int C = G::C;
  const uint32_t tabB = lds_addr(launder(tabB_in));
  fence_regs(Y);
  if constexpr (RS2_ABL_NOPHASE) return;
  sfor<G::LOGW>([&](auto kk) RS2_INL {
    constexpr int k = decltype(kk)::value;
    constexpr int d = kFft ? (C >> (k + 1)) : (G::PPW << k);
    constexpr int dr = d / G::NW;
    const int lim = kFft ? bound : ((bound + d - 1) & ~(d - 1));
    sfor<C / (2 * d)>([&](auto gg) RS2_INL {
      constexpr int g = decltype(gg)::value;
      constexpr int toff = (G::NW - C / d + g) * G::TABB_BYTES;
      auto group = [&](auto with_mul) RS2_INL {
        constexpr bool kMul = decltype(with_mul)::value;
        sfor<(dr + 1) / 2>([&](auto qq) RS2_INL {
          constexpr int j1 = 2 * decltype(qq)::value, j2 = j1 + 1;
          constexpr int i1 = 2 * dr * g + j1, i2 = i1 + 1;
          if constexpr (j2 < dr) {
            if constexpr (!kFft) {
              Y[i1 + dr] ^= Y[i1];
              Y[i2 + dr] ^= Y[i2];
            }
            if constexpr (kMul) gf_mul2<toff, toff, true>(Y[i1], Y[i1 + dr], Y[i2], Y[i2 + dr], tabB);
            if constexpr (kFft) {
              Y[i1 + dr] ^= Y[i1];
              Y[i2 + dr] ^= Y[i2];
            }
          } else {
            if constexpr (!kFft) Y[i1 + dr] ^= Y[i1];
            if constexpr (kMul) gf_mul<toff, true>(Y[i1], Y[i1 + dr], tabB);
            if constexpr (kFft) Y[i1 + dr] ^= Y[i1];
          }
          constexpr int bf = g * dr + j2;  // butterfly index in the layer
          if constexpr ((bf % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
        });
      };
      if (2 * d * g < lim) {
        if constexpr (g == 0) {
          if (zero_g0) group(std::false_type{}); else group(std::true_type{});
        } else {
          group(std::true_type{});
        }
      }
    });
  });
  fence_regs(Y);
}

// In-place layout change through the LDS union region (all waves write, then all read):
// word (w*PPW + i)*64 + l (A) / (NW*i + w)*64 + l (B), one dword per access.
// kSync: barrier before the writes.  A -> B writes only the wave's own A region (= its slab),
// whose last other-wave access (B -> A writes) an earlier barrier already ordered, so it needs
// only its own LDS reads drained; B -> A writes every wave's region and needs the barrier unless
// the caller has just passed one with no union-region access since.
// (Rejected: b64 slots holding a position pair per lane, 16 + 16 instead of 32 + 32 DS
// instructions per wave and direction -- step 70.8 vs 82.1 GiB/s, profiles/r03/exp/tx64/.)
template <class G, bool kAtoB, bool kSync = !kAtoB>
__device__ __forceinline__ void transpose(uint32_t (&X)[G::PPW], lds32* sU, int w, int l) {
  if constexpr (kSync)
    __syncthreads();
  else
    wave_lds_handoff();
  constexpr int IW = cmax(1, 65536 / (G::NW * 256));   // B registers per 64 KiB window
  constexpr int NWIN = (G::PPW + IW - 1) / IW;
  (void)l;
  const int lf = fresh_lane();
  lds32* pa = launder32(sU + w * G::PPW * 64 + lf);
  lds32* pb[NWIN];
  sfor<NWIN>([&](auto kk) RS2_INL {
    constexpr int k = decltype(kk)::value;
    pb[k] = launder32(sU + (G::NW * k * IW + w) * 64 + lf);
  });
  auto bref = [&](auto ii) RS2_INL -> lds32& {
    constexpr int i = decltype(ii)::value;
    return pb[i / IW][(i % IW) * G::NW * 64];
  };
  if constexpr (!RS2_ABL_NOTX)
    sfor<G::PPW>([&](auto ii) RS2_INL {
      constexpr int i = decltype(ii)::value;
      if constexpr (kAtoB) pa[i * 64] = X[i]; else bref(ii) = X[i];
    });
  __syncthreads();
  if constexpr (!RS2_ABL_NOTX)
    sfor<G::PPW>([&](auto ii) RS2_INL {
      constexpr int i = decltype(ii)::value;
      if constexpr (kAtoB) X[i] = bref(ii); else X[i] = pa[i * 64];
    });
}

// A-layout write of wave w's registers into its region (the first half of an A -> B pass)
template <class G>
__device__ __forceinline__ void write_a(uint32_t (&X)[G::PPW], lds32* sU, int w) {
  lds32* pa = launder32(sU + w * G::PPW * 64 + fresh_lane());
  if constexpr (!RS2_ABL_NOTX)
    sfor<G::PPW>([&](auto ii) RS2_INL { pa[decltype(ii)::value * 64] = X[decltype(ii)::value]; });
}

// B-layout read of a block whose A-layout data sits in the union region from word `base`
// (its wave regions written, and a barrier passed, before): register i <- position NW*i + w;
// registers i >= nreg (positions past the block's waves) are zero.
template <class G>
__device__ __forceinline__ void read_b(uint32_t (&X)[G::PPW], lds32* sU, int base, int nreg,
                                       int w, int l) {
  constexpr int IW = cmax(1, 65536 / (G::NW * 256));
  constexpr int NWIN = (G::PPW + IW - 1) / IW;
  (void)l;
  lds32* pb[NWIN];
  sfor<NWIN>([&](auto kk) RS2_INL {
    constexpr int k = decltype(kk)::value;
    pb[k] = launder32(sU + base + (G::NW * k * IW + w) * 64 + fresh_lane());
  });
  sfor<G::PPW>([&](auto ii) RS2_INL {
    constexpr int i = decltype(ii)::value;
    if constexpr (RS2_ABL_NOTX)
      X[i] = i < nreg ? X[i] : 0u;
    else
      X[i] = i < nreg ? pb[i / IW][(i % IW) * G::NW * 64] : 0u;
  });
}

// in-wave part of the formal derivative, in place (A layout), identity term excluded:
//   X[i] <- xor_{t < LOGP, bit t of i clear} X[i | 2^t]
template <class G>
__device__ __forceinline__ void deriv_a(uint32_t (&X)[G::PPW]) {
  sfor<G::PPW>([&](auto ii) RS2_INL {
    constexpr int i = decltype(ii)::value;
    uint32_t v = 0;
    sfor<G::LOGP>([&](auto tt) RS2_INL {
      constexpr int t = decltype(tt)::value;
      if constexpr (((i >> t) & 1) == 0) v ^= X[i | (1 << t)];
    });
    X[i] = v;
  });
}

// identity + cross-wave part of the formal derivative for register i (B layout)
template <class G, int i>
__device__ __forceinline__ uint32_t deriv_b_term(const uint32_t (&Y)[G::PPW]) {
  uint32_t v = Y[i];
  sfor<G::LOGW>([&](auto tt) RS2_INL {
    // position bit LOGP + t; in the B layout p = NW*i + w, so it is register bit LOGP-LOGW+t
    constexpr int ib = G::LOGP - G::LOGW + decltype(tt)::value;
    if constexpr (((i >> ib) & 1) == 0) v ^= Y[i | (1 << ib)];
  });
  return v;
}

// acc[i] ^= kind==1 ? v[i] : v[i]*t   (branch hoisted out of the unrolled loop so the table
// lookups are never speculated for all PPW registers at once)
template <int OFF, int PPW, typename F>
__device__ __forceinline__ void mix_into(uint32_t (&acc)[PPW], int kind, uint32_t t, F&& val) {
  if (kind == 1) {
    sfor<PPW>([&](auto ii) RS2_INL { acc[decltype(ii)::value] ^= val(ii); });
  } else {
    sfor<(PPW + 1) / 2>([&](auto qq) RS2_INL {
      constexpr int i1 = 2 * decltype(qq)::value, i2 = i1 + 1;
      if constexpr (i2 < PPW)
        gf_mul2<OFF, OFF, true>(acc[i1], val(std::integral_constant<int, i1>{}), acc[i2],
                                val(std::integral_constant<int, i2>{}), t);
      else
        gf_mul<OFF, true>(acc[i1], val(std::integral_constant<int, i1>{}), t);
      if constexpr ((i2 % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
    });
  }
}

// X[i] *= c for every register, c's table at LDS byte address t + OFF (wave-uniform)
template <int OFF, int PPW>
__device__ __forceinline__ void mul_uniform(uint32_t (&X)[PPW], uint32_t t) {
  sfor<(PPW + 1) / 2>([&](auto qq) RS2_INL {
    constexpr int i1 = 2 * decltype(qq)::value, i2 = i1 + 1;
    if constexpr (i2 < PPW)
      gf_mul2<OFF, OFF, false>(X[i1], X[i1], X[i2], X[i2], t);
    else
      gf_mul<OFF, false>(X[i1], X[i1], t);
    if constexpr ((i2 % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
  });
}

// X[i] *= (per-position table i at LDS byte address pw + i*256) for the registers of pairs
// [Q0, Q1); registers whose bit in the wave-uniform mask pm is clear are left alone (absent
// decode inputs are zero; unstored decode outputs are dropped)
template <int PPW, int Q0, int Q1>
__device__ __forceinline__ void mul_present(uint32_t (&X)[PPW], uint32_t pw, uint64_t pm) {
  constexpr int TB = kTabU16 * 2;
  if constexpr (RS2_ABL_NOPRE) return;
  sfor<Q1 - Q0>([&](auto qq) RS2_INL {
    constexpr int i1 = 2 * (Q0 + decltype(qq)::value), i2 = i1 + 1;
    const bool p1 = (pm >> i1) & 1u;
    if constexpr (i2 < PPW) {
      const bool p2 = (pm >> i2) & 1u;
      if (p1 && p2)
        gf_mul2<i1 * TB, i2 * TB, false>(X[i1], X[i1], X[i2], X[i2], pw);
      else if (p1)
        gf_mul<i1 * TB, false>(X[i1], X[i1], pw);
      else if (p2)
        gf_mul<i2 * TB, false>(X[i2], X[i2], pw);
    } else if (p1) {
      gf_mul<i1 * TB, false>(X[i1], X[i1], pw);
    }
    if constexpr ((i2 % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
  });
}

// grid: x = ceil(n_pairs / 64) element-pair tiles, y = lines, z = output block (or 1)
//   kModeRows    mixing path, no per-position multipliers (high-rate encode)
//   kModeCols    shared-input path: one IFFT, every output block an FFT of it (low rate)
//   kModeDecode  mixing path with formal derivative and per-position pre/post multipliers
template <int C, int MODE, bool kPersist = false, class Job = CodecJob>
__device__ __forceinline__ void codec_body(const Job& job) {
  using G = Geo<C>;
  constexpr int PPW = G::PPW;
  // the decode kernel is instantiated as kDecodeRt: decode plus a (never taken) runtime
  // shared-input branch -- that control flow happens to give the register allocator a
  // schedule with far fewer spills (56 vs 140 bytes/lane, measured 1.83 vs 1.96 ms)
  constexpr int kDecodeRt = 3;
  constexpr bool kDec = MODE == kModeDecode || MODE == kDecodeRt;
  __shared__ __attribute__((aligned(128))) uint8_t smem_[G::LDS_BYTES];
  lds16* sTabB = (lds16*)(smem_ + G::OFF_TB);
  lds16* sTabO = (lds16*)(smem_ + G::OFF_TO);
  lds16* sTabM = (lds16*)(smem_ + G::OFF_TM);
  // output FFT tables staged up front (see Geo::OFF_TO): every output block of the shared-input
  // path, or this workgroup's one output block (blockIdx.z) of the mixing path
  const bool shared_path = MODE == kModeCols || (MODE == kDecodeRt && job.shared_in);
  const int n_pre = shared_path ? job.n_out : 1;
  // (not in the decode kernel: its one output's table wait is short, and the extra live state
  // there costs register spills)
  const bool pre_out = !kDec && G::NW > 1 && G::NTB > 0 && n_pre <= kPreOut;
  bool pre_out_pending = pre_out;  // staged with the first input block
  lds32* sU = (lds32*)(smem_ + G::OFF_U);

  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63;
  // the DMA helpers' lane id: recomputed per call in the decode kernel, where a kept
  // 16 * lane id was a spill slot (the encode kernels keep theirs: cheaper there)
  auto dma_lane = [&]() RS2_INL { return kDec ? fresh_lane() : l; };
  const int s = job.symbol_size;
  // phase stamps (diagnostic builds, -DRS2_STAMPS=1): every wave records the shader clock at
  // each boundary (vector store from lane 0)
  int n_stamp = 0;
  uint64_t* const stamps = job.stamps;
  auto stamp = [&]() RS2_INL {
    if (RS2_STAMPS_ON && stamps) {
      if (l == 0 && n_stamp < kStamps)
        reinterpret_cast<RS2_AS(1) uint64_t*>(reinterpret_cast<uintptr_t>(stamps))[
            (int64_t(blockIdx.x + gridDim.x * blockIdx.z) * G::NW + w) * kStamps + n_stamp] =
            __builtin_amdgcn_s_memtime();
      ++n_stamp;
    }
  };
  stamp();
  // Lanes walk a flattened (line, pair) space with `pairs_span` (even) pairs per line, so one
  // workgroup may finish one line and start the next and no lane idles on a symbol's partial
  // last tile.  Symbol addresses stay a wave-uniform SGPR base (the workgroup's first line)
  // plus a 32-bit per-lane offset that carries the lane's line step `dl` (the host keeps
  // 64 * line stride below 2^31, else makes pairs_span a multiple of 64 so dl == 0).
  const int P2 = job.pairs_span;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (workgroup i runs
  // on XCD i % 8), so XCD x takes the contiguous tile range [start(x), start(x) + count(x)).
  // Neighbouring tiles share the partial 128-byte lines at their edges (a 64-pair tile covers
  // 256 bytes of a symbol at 2-byte alignment); on one XCD those lines meet in one L2 instead
  // of being fetched, and partly written back, by two.
  // kPersist: one workgroup per CU walks the XCD's contiguous tile range interleaved with the
  // XCD's other workgroups (as pipe_body), so a launch holds at most one workgroup per CU and its
  // per-workgroup start-up is paid once per range instead of once per tile
  auto tile_body = [&](uint32_t tile) RS2_INL {
  // blob batches: this workgroup's blob, whose symbols sit a fixed stride past blob 0's
  int64_t bo_in = 0, bo_out = 0, bo_cp = 0;
  if (job.tiles_per_blob > 0) {
    const uint32_t blob = tile / uint32_t(job.tiles_per_blob);
    tile -= blob * uint32_t(job.tiles_per_blob);
    bo_in = int64_t(blob) * job.in_blob_stride;
    bo_out = int64_t(blob) * job.out_blob_stride;
    bo_cp = int64_t(blob) * job.copy_blob_stride;
  }
  const int64_t g0 = int64_t(tile) * 64;
  const int lrel0 = int(g0 / P2);
  const int line0 = job.line_base + lrel0;  // wave-uniform
  const uint32_t r0 = uint32_t(g0 - int64_t(lrel0) * P2);
  // the largest line step of any lane: bounds every lane's own limit in the stores' and
  // copy-outs' wave-uniform fast test
  const uint32_t dl_max = (r0 + 63u) / uint32_t(P2);
  // Per-lane symbol I/O geometry.  Recomputed at each load / store phase from a laundered lane
  // id, so that its dozen values (and their lane masks, which are SGPR pairs) are not kept live
  // through the transforms, where registers are the binding resource.
  struct LaneGeo {
    uint32_t dl;       // lane's line step from line0 (invalid lanes read line0)
    uint32_t ld_off;   // byte of its dword in the symbol (clamped to s - 4)
    uint32_t ld_sh;    // right shift of a clamped dword
    bool line_ok, lane_ok, full_lane, ld_live;
    PairLoc L;
  };
  auto lane_geo = [&]() RS2_INL {
    uint32_t lv = uint32_t(l);
    asm volatile("" : "+v"(lv));
    LaneGeo q;
    const uint32_t dlr = (r0 + lv) / uint32_t(P2);
    const int pair = int(r0 + lv - dlr * uint32_t(P2));
    q.line_ok = lrel0 + int(dlr) < job.n_lines;
    q.dl = q.line_ok ? dlr : 0u;
    q.L = pair_loc(pair, s);
    q.lane_ok = q.L.v0 && q.line_ok;
    // dword I/O geometry (see "symbol I/O"): the tile is "fast" when all its lanes lie in full
    // chunks; its lanes then move one dword each at byte `dw` of the symbol.
    const int Qf = s >> 6, th = (s & 63) >> 1;
    const int e0 = pair * 2;
    const bool odd_l = (lv & 1) != 0;
    q.full_lane = (e0 >> 5) < Qf;
    const int dw = q.full_lane ? 64 * (e0 >> 5) + ((e0 & 31) & ~3) + (odd_l ? 32 : 0)
                               : 64 * Qf + ((e0 & 31) & ~3) + (odd_l ? th : 0);
    // loads never cross the symbol end: a dword that would is loaded from s-4 and shifted down
    // (its missing top bytes belong to elements past the symbol, which are never stored)
    // (unsigned: every symbol access is a wave-uniform 64-bit base in SGPRs plus this 32-bit
    // lane offset, which selects the saddr form of global_load/store -- no 64-bit VALU math)
    q.ld_off = uint32_t(dw + 4 <= s ? dw : s - 4);
    q.ld_sh = dw + 4 <= s ? 0u : uint32_t(8 * (dw + 4 - s));
    q.ld_live = dw < s && q.line_ok;
    return q;
  };
  // this wave's private slab: its in-wave layer tables, or its per-position tables
  lds16* tabw = (lds16*)(sU + w * G::SLAB_WORDS);
  const lds16* sP = tabw;

  uint32_t X[PPW], A[PPW];
  // per-position tables time-share the wave's slab with its in-wave layer tables in halves of
  // whole 1 KiB DMA chunks (PPW >= 8): pre tables of registers < PPW/2 and the first IFFT layer
  // (slots < PPW/2) in the first half, the rest in the second
  constexpr bool kSplitSlab = kDec && G::NTA > 0 && PPW >= 8;
  constexpr int kHalfCh = PPW * G::TAB_BYTES / 2 / 1024;
  constexpr int kInCh = (G::NTA * G::TAB_BYTES + 1023) / 1024;
  constexpr int kPostCh = PPW * G::TAB_BYTES / 1024;

  // Decode block pair (CodecJob::pair_p): block P = pair_p and block Q = the last input block,
  // whose active waves fit the workgroup together, load, pre-multiply and run their in-wave
  // IFFT layers side by side -- P on waves [0, nwp), Q on the rest -- instead of each leaving
  // most waves idle in a pass of its own (n = 1000: 334 of block 0's positions, 154 of block
  // 2's).  One A -> B pass writes both; Q's positions are read back first, finish their IFFT
  // and are XORed into the accumulator (the host pairs only a Q mixed with coefficient 1 and
  // no formal derivative), then P's continue as a single block's.  P's cross-wave tables go to
  // sTabB as usual, Q's to sTabQ.
  const int pair_p =
      (kDec && !shared_path && job.pair_nw[blockIdx.z] > 0) ? int(job.pair_p[blockIdx.z]) : -1;
  const int pair_nw = pair_p >= 0 ? int(job.pair_nw[blockIdx.z]) : G::NW;
  lds16* sTabQ = (lds16*)(smem_ + G::OFF_TQ);

  // load input block b (A layout), pre-multiply, IFFT -> X (B layout)
  auto load_ifft = [&](int b, const uint16_t* m1, const uint16_t* m2) RS2_INL {
    const bool paired = b == pair_p;
    const int bq = job.n_in - 1;
    const bool in_q = paired && w >= pair_nw;
    const int wl = in_q ? w - pair_nw : w;  // this wave's index within its block
    const InBlock ib = job.in[in_q ? bq : b];
    const bool pre = kDec && ib.pre_tab != nullptr;
    const int count = ib.count;
    const bool active = wl * PPW < count;
    // This wave's position offsets (and fused copy-out offsets), one per lane, broadcast with
    // readlane.  They are loaded before the barrier and before the table DMA: their latency
    // hides in the barrier wait, and the symbol loads that need them never wait behind the
    // DMA in the in-order vmcnt (stamped: the issue phase was a quarter of the decode).
    gci64* pos_off = (gci64*)ib.pos_off;
    const bool do_copy = MODE != kModeRows && ib.copy_off != nullptr && s >= 4;
    const int64_t voff = (active && l < PPW) ? pos_off[wl * PPW + l] : int64_t(-1);
    const int64_t vcp =
        (do_copy && active && l < PPW) ? ((gci64*)ib.copy_off)[wl * PPW + l] : int64_t(-1);
    __syncthreads();
    // table DMA next; the symbol loads below overlap it, and one wait + barrier covers both.
    // The slab first holds the per-position pre tables (decode), else the in-wave layer tables
    // (a wave past its block's count stages nothing: its slab is never read).
    if (active) {
      if (pre)
        dma_wave<PPW * G::TAB_BYTES>((lds_void*)tabw,
                                     ib.pre_tab + int64_t(blockIdx.z) * job.pre_z_stride +
                                         wl * PPW * kTabU16, dma_lane());
      else if constexpr (G::NTA > 0)
        dma_wave<G::NTA * G::TAB_BYTES>((lds_void*)tabw, ib.sd_tab + wl * G::NTA * kTabU16, dma_lane());
    }
    if constexpr (G::NTB > 0) {
      dma_group<G::NTB * G::TABB_BYTES, G::NW>((lds_void*)sTabB,
                                               job.in[b].sd_tab + G::NW * G::NTA * kTabU16, w, dma_lane());
      if (paired)
        dma_group<G::NTB * G::TABB_BYTES, G::NW>((lds_void*)sTabQ,
                                                 job.in[bq].sd_tab + G::NW * G::NTA * kTabU16, w, dma_lane());
      if (pre_out_pending) {
        pre_out_pending = false;
        for (int q = 0; q < n_pre; ++q) {
          const OutBlock& oq = job.out[shared_path ? q : int(blockIdx.z)];
          dma_group<G::NTB * G::TABB_BYTES, G::NW>(
              (lds_void*)((uint8_t RS2_AS(3)*)sTabO + q * G::TB_SLOT),
              oq.sd_tab + G::NW * G::NTA * kTabU16, w, dma_lane());
        }
      }
    }
    if (m1 && w == 0) dma_wave<G::TAB_BYTES>((lds_void*)sTabM, m1, dma_lane());
    if (m2 && w == G::NW - 1) dma_wave<G::TAB_BYTES>((lds_void*)(sTabM + kTabU16), m2, dma_lane());
    const int64_t lofs = bo_in + int64_t(line0) * ib.line_stride;
    const g8* base = (const g8*)ib.base + lofs;
    // split input (InBlock::alt_base, s >= 4 only): positions >= alt_from read from alt_base
    const int alt_from = MODE == kModeCols && ib.alt_base ? ib.alt_from : 0x7fffffff;
    const g8* abase = (const g8*)ib.alt_base + lofs;
    const LaneGeo lg = lane_geo();
    const uint32_t dl = lg.dl, ld_off = lg.ld_off, ld_sh = lg.ld_sh;
    const bool ld_live = lg.ld_live, lane_ok = lg.lane_ok;
    const PairLoc& L = lg.L;
    const uint32_t ld_off_l = ld_off + dl * uint32_t(ib.line_stride);
    // present positions (a wave-uniform bit mask: each position's test is a scalar bit test,
    // not a 64-bit vector compare of its readlane'd offset)
    const uint64_t pm_in = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0);
    if (active) {
      if (s >= 4) {
        // issue every load (a uniform skip for absent positions); combined after the wait
        sfor<PPW>([&](auto ii) RS2_INL {
          constexpr int i = decltype(ii)::value;
          const g8* src = wl * PPW + i >= alt_from ? abase : base;  // wave-uniform
          X[i] = 0u;
          if ((pm_in >> i) & 1u)
            X[i] = *reinterpret_cast<gc32*>(sgpr_ptr(src + readlane64(voff, i)) + ld_off_l);
        });
      } else {
        // 2-byte symbols: per-lane byte-exact loads.  The offset is read across lanes at full
        // exec under the wave-uniform mask test, only the load is lane-divergent (lane_ok), and
        // voff is kept live past the loop (the divergent-readlane rule at keep_live)
        sfor<PPW>([&](auto ii) RS2_INL {
          constexpr int i = decltype(ii)::value;
          uint32_t v = 0;
          if ((pm_in >> i) & 1u) {
            const int64_t off = readlane64(voff, i);  // wave-uniform
            if (lane_ok) v = load_pair(base + off + dl * ib.line_stride, L);
          }
          X[i] = v;
        });
        keep_live(voff);  // keep voff: 2-byte input offsets (loads divergent on lane_ok)
      }
      if constexpr (RS2_ABL_NOLOAD) {
        sfor<PPW>([&](auto ii) RS2_INL { X[decltype(ii)::value] = uint32_t(voff) + decltype(ii)::value; });
      }
    } else {
      sfor<PPW>([&](auto ii) RS2_INL { X[decltype(ii)::value] = 0u; });
    }
    stamp();  // loads + DMA issued
    lds_dma_wait();
    __syncthreads();
    stamp();  // loads landed, workgroup joined
    if (active && s >= 4) {
      if (MODE == kModeCols && ib.copy2_base) {
        // second copy-out at the input's own offsets (raw dwords, as the copy below)
        g8* c2base = (g8*)ib.copy2_base + lofs;
        if (ld_live)
          sfor<PPW>([&](auto ii) RS2_INL {
            constexpr int i = decltype(ii)::value;
            if ((pm_in >> i) & 1u)
              st32(reinterpret_cast<g32*>(sgpr_ptr(c2base + readlane64(voff, i)) + ld_off_l), X[i]);
            if constexpr ((i % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
          });
        keep_live(voff);  // keep voff: copy2 store offsets (region divergent on ld_live)
      }
      if (do_copy) {
        // fused copy-out of the raw symbol dwords (every byte of a symbol is covered by some
        // lane's dword; clamped tail dwords rewrite identical bytes), issued once the loads
        // have landed so it adds no wait of its own
        const int64_t cl = int64_t(line0) * ib.copy_line_stride;
        g8* cbase = (g8*)ib.copy_base + bo_cp + cl;
        const uint32_t cdl = dl * uint32_t(ib.copy_line_stride);
        const uint32_t c_off = ld_off + cdl;
        const int64_t climit = ib.copy_limit - int64_t(cdl);  // per lane: its own line
        // copied positions, and those whose symbol ends below every lane's limit (fast)
        const int64_t cfast =
            ib.copy_limit - int64_t(dl_max * uint32_t(ib.copy_line_stride)) - cl - s;
        const uint64_t cpm = __builtin_amdgcn_ballot_w64(l < PPW && vcp >= 0);
        const uint64_t cfm = __builtin_amdgcn_ballot_w64(l < PPW && vcp >= 0 && vcp <= cfast);
        // whole symbols below every lane's limit: one divergent region (keep_live)
        if (ld_live)
          sfor<PPW>([&](auto ii) RS2_INL {
            constexpr int i = decltype(ii)::value;
            if ((cfm >> i) & 1u)
              st32(reinterpret_cast<g32*>(sgpr_ptr(cbase + readlane64(vcp, i)) + c_off), X[i]);
            if constexpr ((i % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
          });
        keep_live(vcp);  // keep vcp: fused copy-out offsets (region divergent on ld_live)
        if (cpm != cfm)  // symbols reaching a lane's limit
          sfor<PPW>([&](auto ii) RS2_INL {
            constexpr int i = decltype(ii)::value;
            if (((cpm & ~cfm) >> i) & 1u) {
              const int64_t co = readlane64(vcp, i);  // wave-uniform
              g8* dst = sgpr_ptr(cbase + co);
              // bytes of this symbol left before the lane's limit
              const int64_t room = climit - (cl + co);
              if (room >= s) {
                if (ld_live) st32(reinterpret_cast<g32*>(dst + c_off), X[i]);
              } else if (room > 0 && ld_live) {
                for (uint32_t b = 0; b < 4; ++b)
                  if (int64_t(ld_off + b) < room) dst[c_off + b] = uint8_t(X[i] >> (8 * b));
              }
            }
          });
      }
      // (selector and liveness mask once per phase, not per position)
      const uint32_t sel = sel_load(), live = ld_live ? ~0u : 0u;
      sfor<PPW>([&](auto ii) RS2_INL {
        constexpr int i = decltype(ii)::value;
        const uint32_t t = (X[i] >> ld_sh) & live;
        X[i] = __builtin_amdgcn_perm(swap_adjacent(t), t, sel);
      });
    }
    if (pre && active) {
      // absent positions hold zero: their multiplies are skipped (wave-uniform branches on the
      // wave's presence mask; a random K_p subset leaves about 2/3 of the decode's positions
      // absent)
      const uint64_t pm = pm_in;
      if constexpr (kSplitSlab) {
        // the slab's first half (pre tables of registers < PPW/2) takes the first IFFT layer's
        // tables (slots < PPW/2, the same bytes) as soon as those registers are multiplied, so
        // their DMA lands under the second half's multiplies instead of in front of the layer
        mul_present<PPW, 0, PPW / 4>(X, lds_addr(launder(sP)), pm);
        wave_lds_handoff();
        dma_wave_range<G::NTA * G::TAB_BYTES, 0, kHalfCh>((lds_void*)tabw,
                                                          ib.sd_tab + wl * G::NTA * kTabU16,
                                                          dma_lane());
        mul_present<PPW, PPW / 4, PPW / 2>(X, lds_addr(launder(sP)), pm);
        wave_lds_handoff();
        dma_wave_range<G::NTA * G::TAB_BYTES, kHalfCh, kInCh>((lds_void*)tabw,
                                                              ib.sd_tab + wl * G::NTA * kTabU16,
                                                              dma_lane());
      } else {
        mul_present<PPW, 0, (PPW + 1) / 2>(X, lds_addr(launder(sP)), pm);
      }
    }
    stamp();  // pre-multiply
    if constexpr (G::NTA > 0) {
      if (pre && active) {  // the slab now takes the in-wave layer tables, layer by layer
        if constexpr (!kSplitSlab) {
          wave_lds_handoff();
          dma_wave<G::NTA * G::TAB_BYTES>((lds_void*)tabw, ib.sd_tab + wl * G::NTA * kTabU16,
                                          dma_lane());
        }
        phase_a<G, false, true>(X, tabw);
      } else if (active) {
        phase_a<G, false>(X, tabw);
      }
    } else if (active) {
      phase_a<G, false>(X, tabw);
    }
    stamp();  // in-wave IFFT layers
    if constexpr (G::NW > 1) {
      // A -> B as transpose<G, true>; a pair reads Q's positions first (they sit past P's nwp
      // wave regions): Q's cross-wave layers, XOR into the accumulator, then P's read
      wave_lds_handoff();
      write_a<G>(X, sU, w);
      __syncthreads();
#pragma clang loop unroll(disable)
      for (int h = paired ? 0 : 1; h < 2; ++h) {
        const bool hq = h == 0;
        read_b<G>(X, sU, hq ? pair_nw * PPW * 64 : 0,
                  hq ? (G::NW - pair_nw) * PPW / G::NW : paired ? pair_nw * PPW / G::NW : PPW,
                  w, l);
        stamp();  // transpose A -> B
        const InBlock& ih = job.in[hq ? bq : b];
        phase_b<G, false>(X, hq ? sTabQ : sTabB, ih.count, ih.zero_first != 0);
        stamp();  // cross-wave IFFT layers
        if (hq) sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] ^= X[decltype(ii)::value]; });
      }
    }
  };

  // FFT of A (B layout) with output block o's constants, post-multiply, store
  auto fft_store = [&](int o) RS2_INL {
    const OutBlock ob = job.out[o];
    // output offsets first, so their latency hides under the transform (read after it)
    gci64* pos_off = (gci64*)ob.pos_off;
    const int64_t voff = (w * PPW < ob.trunc && l < PPW) ? pos_off[w * PPW + l] : int64_t(-1);
    if constexpr (G::NW > 1) {
      // tables staged with the first input block: no wait, the stores of the previous output
      // block drain under this block's cross-wave layers (no input block staged them when every
      // mixing coefficient of this output is zero: then the per-output staging below)
      if (pre_out && !pre_out_pending) {
        stamp();
        const lds16* to = (const lds16*)((const uint8_t RS2_AS(3)*)sTabO +
                                         (shared_path ? o : 0) * G::TB_SLOT);
        phase_b<G, true>(A, to, ob.trunc, ob.zero_first != 0);
        stamp();  // cross-wave FFT layers
        transpose<G, false, true>(A, sU, w, l);
      } else {
        __syncthreads();
        dma_group<G::NTB * G::TABB_BYTES, G::NW>((lds_void*)sTabB,
                                                 ob.sd_tab + G::NW * G::NTA * kTabU16, w, dma_lane());
        lds_dma_wait();
        __syncthreads();
        stamp();  // FFT cross-wave tables landed
        phase_b<G, true>(A, sTabB, ob.trunc, ob.zero_first != 0);
        stamp();  // cross-wave FFT layers
        transpose<G, false, false>(A, sU, w, l);  // barrier above, no union access since
      }
      stamp();  // transpose B -> A
    }
    // the slab below is this wave's own A region, which it has just read
    if constexpr (G::NW > 1)
      wave_lds_handoff();
    else
      __syncthreads();
    // the FFT's first in-wave layer reads the last slot: its tables arrive in reverse order and
    // each layer waits for its own chunks only (the slab is private to this wave)
    const bool post = kDec && ob.post_tab != nullptr;
    const int trunc = ob.trunc;
    const bool active = w * PPW < trunc;
    if constexpr (G::NTA > 0)
      if (active)
        dma_wave<G::NTA * G::TAB_BYTES, true>((lds_void*)tabw, ob.sd_tab + w * G::NTA * kTabU16, dma_lane());
    bool split_post = false;
    if constexpr (kSplitSlab) {
      split_post = post && active;
      if (split_post) {
        // every layer but the last (slots >= PPW/2: the slab's second half) first; then the
        // post tables of registers >= PPW/2 go there under the last layer (slots < PPW/2), and
        // those of registers < PPW/2 into the first half once it is done
        phase_a<G, true, true, 0, G::LOGP - 1>(A, tabw);
        wave_lds_handoff();
        dma_wave_range<PPW * G::TAB_BYTES, kHalfCh, kPostCh>(
            (lds_void*)tabw, ob.post_tab + w * PPW * kTabU16, dma_lane());
        phase_a<G, true, true, G::LOGP - 1, G::LOGP, 0, kPostCh - kHalfCh>(A, tabw);
        wave_lds_handoff();
        dma_wave_range<PPW * G::TAB_BYTES, 0, kHalfCh>(
            (lds_void*)tabw, ob.post_tab + w * PPW * kTabU16, dma_lane());
      } else if (active) {
        phase_a<G, true, true>(A, tabw);
      }
    } else {
      if (active) phase_a<G, true, (G::NTA > 0)>(A, tabw);
    }
    stamp();  // in-wave FFT layers
    if (!split_post) {
      lds_dma_wait();
      if (post && active) {  // the slab now takes the per-position post tables
        wave_lds_handoff();
        dma_wave<PPW * G::TAB_BYTES>((lds_void*)tabw, ob.post_tab + w * PPW * kTabU16, dma_lane());
      }
    }
    const int64_t lbase = int64_t(line0) * ob.line_stride;
    g8* obase = (g8*)ob.base + bo_out + lbase;
    const LaneGeo lg = lane_geo();
    const uint32_t dl = lg.dl, ld_off = lg.ld_off;
    const bool full_lane = lg.full_lane, line_ok = lg.line_ok, lane_ok = lg.lane_ok;
    const PairLoc& L = lg.L;
    const uint32_t odl = dl * uint32_t(ob.line_stride);
    const uint32_t st_off = ld_off + odl;
    const int64_t limit = ob.limit - int64_t(odl);  // per lane: its own line
    // stored positions, and those whose symbol ends below every lane's limit (fast)
    const int64_t sfast = ob.limit - int64_t(dl_max * uint32_t(ob.line_stride)) - lbase - s;
    const uint64_t spm = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0);
    if (split_post) {
      // only stored positions are multiplied (the others are dropped below); the second half's
      // tables were issued first
      const uint64_t pm = spm;
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kHalfCh) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      mul_present<PPW, PPW / 4, PPW / 2>(A, lds_addr(launder(sP)), pm);
      lds_dma_wait();
      __builtin_amdgcn_sched_barrier(0);
      mul_present<PPW, 0, PPW / 4>(A, lds_addr(launder(sP)), pm);
    } else if (post && active) {
      const uint64_t pm = spm;
      const uint32_t pw = lds_addr(launder(sP));
      sfor<(PPW + 1) / 2>([&](auto qq) RS2_INL {
        constexpr int i1 = 2 * decltype(qq)::value, i2 = i1 + 1;
        // the tables arrive in position order, 1 KiB chunks: wait only for this pair's chunk
        constexpr int NCH = (PPW * G::TAB_BYTES + 1023) / 1024;
        constexpr int need = ((i2 < PPW ? i2 : i1) * G::TAB_BYTES + G::TAB_BYTES - 1) / 1024;
        if constexpr (i1 == 0 || (i1 * G::TAB_BYTES) / 1024 != ((i1 - 2) * G::TAB_BYTES) / 1024) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NCH - 1 - need) : "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
        // only stored positions are multiplied (the others are dropped below)
        const bool p1 = (pm >> i1) & 1u;
        if constexpr (i2 < PPW) {
          const bool p2 = (pm >> i2) & 1u;
          if (p1 && p2)
            gf_mul2<i1 * G::TAB_BYTES, i2 * G::TAB_BYTES, false>(A[i1], A[i1], A[i2], A[i2], pw);
          else if (p1)
            gf_mul<i1 * G::TAB_BYTES, false>(A[i1], A[i1], pw);
          else if (p2)
            gf_mul<i2 * G::TAB_BYTES, false>(A[i2], A[i2], pw);
        } else if (p1) {
          gf_mul<i1 * G::TAB_BYTES, false>(A[i1], A[i1], pw);
        }
        if constexpr ((i2 % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
      });
    }
    stamp();  // post-multiply
    if (active) {
      // Cross-lane reads (readlane, DPP) stay outside lane-divergent code: the register
      // allocator tracks liveness per lane, so inside a branch it may already have reused the
      // registers of lanes that branch excludes
      const uint64_t sfm = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0 && voff <= sfast);
      const bool full = full_lane && line_ok;  // ld_off == dw on full-chunk lanes
      // full-chunk lanes: their dword (own and partner pair, DPP at full exec) in place; the
      // tail chunk's lanes keep their packed pair (identity selector)
      const uint32_t sel = full ? sel_store() : 0x03020100u;
      sfor<PPW>([&](auto ii) RS2_INL {
        constexpr int i = decltype(ii)::value;
        A[i] = __builtin_amdgcn_perm(swap_adjacent(A[i]), A[i], sel);
      });
      if (full) {
        sfor<PPW>([&](auto ii) RS2_INL {
          constexpr int i = decltype(ii)::value;
          if ((spm >> i) & 1u) {
            const int64_t off = readlane64(voff, i);
            g8* dst = sgpr_ptr(obase + off);
            if constexpr (RS2_ABL_NOSTORE) {
              if (A[i] == 0x9E3779B9u) dst[st_off] = 0;
            } else if ((sfm >> i) & 1u) {  // the whole symbol below every lane's limit
              st32(reinterpret_cast<g32*>(dst + st_off), A[i]);
            } else {
              const int64_t room = limit - (lbase + off);  // symbol bytes before the limit
              if (room >= s) {
                st32(reinterpret_cast<g32*>(dst + st_off), A[i]);
              } else {
                for (uint32_t b = 0; b < 4; ++b)
                  if (int64_t(ld_off + b) < room) dst[st_off + b] = uint8_t(A[i] >> (8 * b));
              }
            }
          }
        });
      } else if (lane_ok) {
        sfor<PPW>([&](auto ii) RS2_INL {
          constexpr int i = decltype(ii)::value;
          if ((spm >> i) & 1u) {
            const int64_t off = readlane64(voff, i);
            store_pair(obase + off + odl, lbase + off, limit, L, A[i]);
          }
        });
      }
      keep_live(voff);  // keep voff: output store offsets (regions divergent on full / lane_ok)
    }
  };

  if (MODE == kModeCols || (MODE == kDecodeRt && job.shared_in)) {
    // low-rate encode: one IFFT, every output block an FFT of the same coefficients
    load_ifft(0, nullptr, nullptr);
    const int n_out = job.n_out;
    for (int o = 0; o < n_out; ++o) {
      sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] = X[decltype(ii)::value]; });
      fft_store(o);
      stamp();  // stores issued
    }
    return;
  }

  const int o = blockIdx.z;
  sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] = 0u; });
  const int n_in = job.n_in - (pair_p >= 0 ? 1 : 0);  // a pair's Q runs inside load_ifft(P)
  for (int b = 0; b < n_in; ++b) {
    const int k1 = kDec ? job.m1_kind[o][b] : 0;
    const int k2 = job.m2_kind[o][b];
    if (k1 == 0 && k2 == 0) continue;
    const uint16_t* mt = job.mix_tab + ((o * Job::kBlocks + b) * 2) * kTabU16;
    load_ifft(b, k1 == 2 ? mt : nullptr, k2 == 2 ? mt + kTabU16 : nullptr);
    const uint32_t tm = lds_addr(launder(sTabM));
    if (k2) mix_into<kTabU16 * 2>(A, k2, tm, [&](auto ii) RS2_INL { return X[decltype(ii)::value]; });
    if (kDec && k1) {
      // Dw(X) = X + S_B(X) + S_A(X)   (in-block formal derivative).  The mixing coefficient is
      // one scalar per block and Dw is linear, so X is scaled once up front (k1 * Dw(X) =
      // Dw(k1 * X)) and every derivative term is a bare XOR: one multiply pass instead of two,
      // and no multiply temporaries live beside X and A around the transposes
      if (k1 == 2) mul_uniform<0, PPW>(X, tm);
      sfor<PPW>([&](auto ii) RS2_INL {
        A[decltype(ii)::value] ^= deriv_b_term<G, decltype(ii)::value>(X);
      });
      if constexpr (G::NW > 1) transpose<G, false>(X, sU, w, l);
      deriv_a<G>(X);
      if constexpr (G::NW > 1) transpose<G, true>(X, sU, w, l);
      sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] ^= X[decltype(ii)::value]; });
    }
    stamp();  // block mixing (+ formal derivative)
  }
  fft_store(o);
  stamp();  // stores issued
  };  // tile_body

  if constexpr (kPersist) {
    const uint32_t n_tiles = uint32_t(job.n_tiles);
    const uint32_t n_xcd = gridDim.x < kXcds ? gridDim.x : kXcds;
    const uint32_t xcd = blockIdx.x % n_xcd, k_in_xcd = blockIdx.x / n_xcd;
    const uint32_t nx = (gridDim.x - xcd + n_xcd - 1) / n_xcd;
    const uint32_t q_t = n_tiles / n_xcd, r_t = n_tiles % n_xcd;
    const uint32_t x_start = xcd * q_t + (xcd < r_t ? xcd : r_t);
    const uint32_t t_end = x_start + q_t + (xcd < r_t ? 1u : 0u);
#pragma clang loop unroll(disable)
    for (uint32_t t = x_start + k_in_xcd; t < t_end; t += nx) tile_body(t);
  } else {
    tile_body(xcd_tile(blockIdx.x, gridDim.x));
  }
}


// Persistent, tile-pipelined encode.  Each workgroup walks a contiguous tile range (XCD-ordered
// like the one-tile kernels).  The tile's first ("head") input block sits at the TOP of the
// workgroup -- its nwl = ceil(count / PPW) active waves are waves [NW - nwl, NW) -- for its
// load, copies and in-wave IFFT layers, and in the same phase the waves below finish the
// previous tile's last output block: its in-wave FFT layers under the loads, its stores beside
// the IFFT.  The launcher pipelines only when that block's active waves fit below, e.g. n = 1000:
//   kShared (low-rate column code, one IFFT, every output an FFT of it): 334 input positions on
//     11 waves, the last output's 154 positions on 5;
//   mixing (high-rate row code, the head is the short input block, job.pipe_head): 155 input
//     positions on 5 waves, the output's 333 positions on 11.
// Otherwise both phases leave most of the workgroup idle (the one-tile kernel's stamps: about a
// quarter of a tile).  The other input blocks of a mixing job load on every wave as usual.
template <int C, bool kShared>
__device__ __forceinline__ void pipe_body(const CodecJob& job_arg) {
  // job fields are read through a pointer laundered once per block, so the compiler reloads
  // them (scalar loads from the kernel arguments) instead of pinning dozens of SGPRs for the
  // whole loop, which spilled 172 of them into VGPR lanes
  typedef RS2_AS(4) const CodecJob kjob;
  // (the job is the kernel's only argument: it starts the kernarg segment)
  kjob* jp = (kjob*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)job_arg;
#define job (*jp)
  using G = Geo<C>;
  constexpr int PPW = G::PPW, NW = G::NW;
  static_assert(NW > 1, "pipelining needs cross-wave layers");
  __shared__ __attribute__((aligned(128))) uint8_t smem_[G::LDS_BYTES];
  lds16* sTabB = (lds16*)(smem_ + G::OFF_TB);
  lds16* sTabO = (lds16*)(smem_ + G::OFF_TO);
  lds16* sTabM = (lds16*)(smem_ + G::OFF_TM);
  lds32* sU = (lds32*)(smem_ + G::OFF_U);
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63;
  const int s = job.symbol_size;
  const int P2 = job.pairs_span;
  const int n_in = kShared ? 1 : job.n_in;
  const int head = kShared ? 0 : job.pipe_head;
  const int n_out = job.n_out, last = n_out - 1;
  const int head_wl0 = NW - (job.in[head].count + PPW - 1) / PPW;  // first loading wave
  lds16* tabw = (lds16*)(sU + w * G::SLAB_WORDS);

  // tiles of this workgroup: XCD x (= blockIdx.x % 8, the round-robin dispatch) owns the
  // contiguous range xcd_tile gives it, and its nx workgroups interleave over that range
  // (tile start + k, start + k + nx, ...), so the workgroups running at once on one XCD hold
  // neighbouring tiles, whose shared partial lines meet in that XCD's L2 (a contiguous range
  // per workgroup reads them ~one tile-time apart, after eviction: +50 % HBM reads measured)
  const uint32_t n_tiles = uint32_t(job.n_tiles);
  const uint32_t n_xcd = gridDim.x < kXcds ? gridDim.x : kXcds;  // XCDs with a workgroup
  const uint32_t xcd = blockIdx.x % n_xcd, k_in_xcd = blockIdx.x / n_xcd;
  const uint32_t nx = (gridDim.x - xcd + n_xcd - 1) / n_xcd;  // workgroups on this XCD
  const uint32_t q_t = n_tiles / n_xcd, r_t = n_tiles % n_xcd;
  const uint32_t x_start = xcd * q_t + (xcd < r_t ? xcd : r_t);
  const uint32_t t_begin = x_start + k_in_xcd;
  const uint32_t t_end = x_start + q_t + (xcd < r_t ? 1u : 0u);

  struct TileGeo {
    int line0, lrel0;
    uint32_t r0;
    int64_t bo_in, bo_out, bo_cp;
  };
  // the largest line step of any lane of a tile (see codec_body)
  auto dl_max_of = [&](const TileGeo& t) RS2_INL { return (t.r0 + 63u) / uint32_t(P2); };
  auto tile_geo = [&](uint32_t tile) RS2_INL {
    TileGeo t;
    t.bo_in = t.bo_out = t.bo_cp = 0;
    if (job.tiles_per_blob > 0) {
      const uint32_t blob = tile / uint32_t(job.tiles_per_blob);
      tile -= blob * uint32_t(job.tiles_per_blob);
      t.bo_in = int64_t(blob) * job.in_blob_stride;
      t.bo_out = int64_t(blob) * job.out_blob_stride;
      t.bo_cp = int64_t(blob) * job.copy_blob_stride;
    }
    const int64_t g0 = int64_t(tile) * 64;
    t.lrel0 = int(g0 / P2);
    t.line0 = job.line_base + t.lrel0;
    t.r0 = uint32_t(g0 - int64_t(t.lrel0) * P2);
    return t;
  };
  struct LaneGeo {
    uint32_t dl, ld_off, ld_sh;
    bool line_ok, lane_ok, full_lane, ld_live;
    PairLoc L;
  };
  // per-lane symbol I/O geometry of a tile (as codec_body's lane_geo)
  auto lane_geo = [&](const TileGeo& t) RS2_INL {
    uint32_t lv = uint32_t(l);
    asm volatile("" : "+v"(lv));
    LaneGeo q;
    const uint32_t dlr = (t.r0 + lv) / uint32_t(P2);
    const int pair = int(t.r0 + lv - dlr * uint32_t(P2));
    q.line_ok = t.lrel0 + int(dlr) < job.n_lines;
    q.dl = q.line_ok ? dlr : 0u;
    q.L = pair_loc(pair, s);
    q.lane_ok = q.L.v0 && q.line_ok;
    const int Qf = s >> 6, th = (s & 63) >> 1;
    const int e0 = pair * 2;
    const bool odd_l = (lv & 1) != 0;
    q.full_lane = (e0 >> 5) < Qf;
    const int dw = q.full_lane ? 64 * (e0 >> 5) + ((e0 & 31) & ~3) + (odd_l ? 32 : 0)
                               : 64 * Qf + ((e0 & 31) & ~3) + (odd_l ? th : 0);
    q.ld_off = uint32_t(dw + 4 <= s ? dw : s - 4);
    q.ld_sh = dw + 4 <= s ? 0u : uint32_t(8 * (dw + 4 - s));
    q.ld_live = dw < s && q.line_ok;
    return q;
  };

  uint32_t X[PPW], A[PPW];
  // phase stamps (diagnostic builds, -DRS2_STAMPS=1): every wave records the shader clock at
  // each boundary of its first tiles (vector store from lane 0; kStamps slots)
  int n_stamp = 0;
  auto stamp = [&]() RS2_INL {
    if (RS2_STAMPS_ON && job.stamps) {
      if (l == 0 && n_stamp < kStamps)
        reinterpret_cast<RS2_AS(1) uint64_t*>(reinterpret_cast<uintptr_t>(job.stamps))[
            (int64_t(blockIdx.x) * NW + w) * kStamps + n_stamp] = __builtin_amdgcn_s_memtime();
      ++n_stamp;
    }
  };

  // cross-wave tables of every output block, once per workgroup (and of the one IFFT)
  for (int q = 0; q < n_out; ++q)
    dma_group<G::NTB * G::TABB_BYTES, G::NW>(
        (lds_void*)((uint8_t RS2_AS(3)*)sTabO + q * G::TB_SLOT),
        job.out[q].sd_tab + G::NW * G::NTA * kTabU16, w, l);
  if constexpr (kShared)
    dma_group<G::NTB * G::TABB_BYTES, G::NW>((lds_void*)sTabB,
                                             job.in[0].sd_tab + G::NW * G::NTA * kTabU16, w, l);

  // the in-wave FFT tables of output o into this wave's slab (its own A region, which it has
  // read), reverse order: the first layer reads the last slot
  auto tail_tables = [&](int o) RS2_INL {
    wave_lds_handoff();
    if constexpr (G::NTA > 0)
      dma_wave<G::NTA * G::TAB_BYTES, true>((lds_void*)tabw,
                                            job.out[o].sd_tab + w * G::NTA * kTabU16, l);
  };
  // in-wave FFT layers of output o (A layout in A), by the waves holding positions < trunc
  auto tail_fft = [&](int o, bool staged) RS2_INL {
    if (w * PPW >= job.out[o].trunc) return;
    if (!staged) tail_tables(o);
    phase_a<G, true, (G::NTA > 0)>(A, tabw);
  };
  // stores of output o of tile t
  auto tail_store = [&](int o, uint32_t t) RS2_INL {
    const OutBlock& ob = job.out[o];
    if (w * PPW >= ob.trunc) return;
    if constexpr (RS2_ABL_NOSTORE) return;
    gci64* pos_off = (gci64*)ob.pos_off;
    const int64_t voff = l < PPW ? pos_off[w * PPW + l] : int64_t(-1);
    const TileGeo tg = tile_geo(t);
    const LaneGeo lg = lane_geo(tg);
    const int64_t lbase = int64_t(tg.line0) * ob.line_stride;
    g8* obase = (g8*)ob.base + tg.bo_out + lbase;
    const uint32_t odl = lg.dl * uint32_t(ob.line_stride);
    const uint32_t st_off = lg.ld_off + odl;
    const int64_t limit = ob.limit - int64_t(odl);  // per lane: its own line
    // stored positions, and those whose symbol ends below every lane's limit (as codec_body)
    const int64_t sfast = ob.limit - int64_t(dl_max_of(tg) * uint32_t(ob.line_stride)) - lbase - s;
    const uint64_t spm = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0);
    const uint64_t sfm = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0 && voff <= sfast);
    // (as codec_body's stores: DPP at full exec, one divergent region per lane class)
    const bool full = lg.full_lane && lg.line_ok;
    const uint32_t sel = full ? sel_store() : 0x03020100u;
    sfor<PPW>([&](auto ii) RS2_INL {
      constexpr int i = decltype(ii)::value;
      A[i] = __builtin_amdgcn_perm(swap_adjacent(A[i]), A[i], sel);
    });
    if (full) {
      sfor<PPW>([&](auto ii) RS2_INL {
        constexpr int i = decltype(ii)::value;
        if ((spm >> i) & 1u) {
          const int64_t off = readlane64(voff, i);
          g8* dst = sgpr_ptr(obase + off);
          if ((sfm >> i) & 1u) {
            st32(reinterpret_cast<g32*>(dst + st_off), A[i]);
          } else {
            const int64_t room = limit - (lbase + off);
            if (room >= s) {
              st32(reinterpret_cast<g32*>(dst + st_off), A[i]);
            } else {
              for (uint32_t b = 0; b < 4; ++b)
                if (int64_t(lg.ld_off + b) < room) dst[st_off + b] = uint8_t(A[i] >> (8 * b));
            }
          }
        }
      });
    } else if (lg.lane_ok) {
      sfor<PPW>([&](auto ii) RS2_INL {
        constexpr int i = decltype(ii)::value;
        if ((spm >> i) & 1u) {
          const int64_t off = readlane64(voff, i);
          store_pair(obase + off + odl, lbase + off, limit, lg.L, A[i]);
        }
      });
    }
    keep_live(voff);  // keep voff: output store offsets (regions divergent on full / lane_ok)
  };

  // dynamic tile order (CodecJob::tile_ctr): wave 0's lane 0 takes the next tile with a device
  // atomic issued before the output blocks and resolved under their first cross-wave FFT, and
  // publishes it in LDS before that block's transpose barrier; every wave reads it at the end of
  // the tile.  Static order: t_begin, t_begin + nx, ... < t_end.
  uint32_t* const ctr = job.tile_ctr;
  const bool dyn = ctr != nullptr;
  constexpr uint32_t kNoTile = 0xFFFFFFFFu;
  __shared__ uint32_t s_tile[2];
  auto take = [&](uint32_t x) RS2_INL {
    return __hip_atomic_fetch_add(ctr + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // tile of the count k taken from XCD x's range, else the other XCDs' leftovers (or none)
  auto resolve = [&](uint32_t k) RS2_INL {
    if (k < q_t + (xcd < r_t ? 1u : 0u)) return x_start + k;
    for (uint32_t d = 1; d < n_xcd; ++d) {
      const uint32_t x = (xcd + d) % n_xcd;
      const uint32_t kx = take(x);
      if (kx < q_t + (x < r_t ? 1u : 0u)) return x * q_t + (x < r_t ? x : r_t) + kx;
    }
    return kNoTile;
  };
  uint32_t t = t_begin, it = 0;
  if (dyn) {
    if (w == 0 && l == 0) s_tile[0] = resolve(take(xcd));
    __syncthreads();
    t = s_tile[0];
  }
  bool tail = false;  // the previous tile's last output block waits for its in-wave part
  uint32_t tail_tile = 0;
  while (dyn ? t != kNoTile : t < t_end) {
    stamp();  // tile start
    // input blocks, the head first: on the head, the waves below it carry the previous tile's
    // tail; the other blocks load on every wave
#pragma clang loop unroll(disable)
    for (int bi = 0; bi < n_in; ++bi) {
      asm volatile("" : "+s"(jp));
      const bool is_head = bi == 0;
      const int b = is_head ? head : (bi <= head ? bi - 1 : bi);
      const int wl0 = is_head ? head_wl0 : 0;
      const bool loader = w >= wl0;
      const int wl = w - wl0;  // position group of a loading wave
      const TileGeo tg = tile_geo(t);
#define ib (job.in[b])
      const int k2 = kShared ? 0 : int(job.m2_kind[0][b]);
      gci64* pos_off = (gci64*)ib.pos_off;
      const bool do_copy = kShared && ib.copy_off != nullptr && s >= 4;
      const bool active = loader && wl * PPW < ib.count;
      const int64_t voff = (active && l < PPW) ? pos_off[wl * PPW + l] : int64_t(-1);
      const int64_t vcp =
          (do_copy && active && l < PPW) ? ((gci64*)ib.copy_off)[wl * PPW + l] : int64_t(-1);
      __syncthreads();  // the union region's and the shared tables' earlier readers are done
      if constexpr (!kShared) {
        dma_group<G::NTB * G::TABB_BYTES, G::NW>((lds_void*)sTabB,
                                                 ib.sd_tab + G::NW * G::NTA * kTabU16, w, l);
        if (k2 == 2 && w == G::NW - 1)
          dma_wave<G::TAB_BYTES>((lds_void*)(sTabM + kTabU16),
                                 job.mix_tab + (b * 2 + 1) * kTabU16, l);
      }
      // X is dead on the tail waves and A on the loading ones (only on the head: later blocks
      // mix into A): zeroing them says so to the register allocator
      if (loader) {
        if (is_head) sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] = 0u; });
        if (active) {
          if constexpr (G::NTA > 0)
            dma_wave<G::NTA * G::TAB_BYTES>((lds_void*)tabw, ib.sd_tab + wl * G::NTA * kTabU16,
                                            l);
          const LaneGeo lg = lane_geo(tg);
          const int64_t lofs = tg.bo_in + int64_t(tg.line0) * ib.line_stride;
          const g8* base = (const g8*)ib.base + lofs;
          const int alt_from = kShared && ib.alt_base ? ib.alt_from : 0x7fffffff;
          const g8* abase = (const g8*)ib.alt_base + lofs;
          const uint32_t ld_off_l = lg.ld_off + lg.dl * uint32_t(ib.line_stride);
          // present positions: scalar bit tests (see codec_body)
          const uint64_t pm_in = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0);
          if (s >= 4) {
            sfor<PPW>([&](auto ii) RS2_INL {
              constexpr int i = decltype(ii)::value;
              const g8* src = wl * PPW + i >= alt_from ? abase : base;  // wave-uniform
              X[i] = 0u;
              if ((pm_in >> i) & 1u)
                X[i] = *reinterpret_cast<gc32*>(sgpr_ptr(src + readlane64(voff, i)) + ld_off_l);
            });
          } else {
            // readlane at full exec, only the load lane-divergent (see codec_body)
            sfor<PPW>([&](auto ii) RS2_INL {
              constexpr int i = decltype(ii)::value;
              uint32_t v = 0;
              if ((pm_in >> i) & 1u) {
                const int64_t off = readlane64(voff, i);  // wave-uniform
                if (lg.lane_ok) v = load_pair(base + off + lg.dl * ib.line_stride, lg.L);
              }
              X[i] = v;
            });
            keep_live(voff);  // keep voff: 2-byte input offsets (loads divergent on lane_ok)
          }
        } else {
          sfor<PPW>([&](auto ii) RS2_INL { X[decltype(ii)::value] = 0u; });
        }
      } else {
        sfor<PPW>([&](auto ii) RS2_INL { X[decltype(ii)::value] = 0u; });
        if (tail) tail_fft(last, true);  // under the loads
      }
      stamp();  // loads issued (tail: its in-wave FFT)
      lds_dma_wait();
      __syncthreads();
      stamp();  // loads landed
      if (!loader && tail) tail_store(last, tail_tile);  // beside the copies and the IFFT
      if (active) {
        if (s >= 4) {
          const LaneGeo lg = lane_geo(tg);
          const int64_t lofs = tg.bo_in + int64_t(tg.line0) * ib.line_stride;
          const uint32_t ld_off_l = lg.ld_off + lg.dl * uint32_t(ib.line_stride);
          if (kShared && ib.copy2_base && !RS2_ABL_NOCOPY) {
            // second copy-out at the input's own offsets (systematic primary slivers)
            g8* c2base = (g8*)ib.copy2_base + lofs;
            const uint64_t pm_in = __builtin_amdgcn_ballot_w64(l < PPW && voff >= 0);
            if (lg.ld_live)
              sfor<PPW>([&](auto ii) RS2_INL {
                constexpr int i = decltype(ii)::value;
                if ((pm_in >> i) & 1u)
                  st32(reinterpret_cast<g32*>(sgpr_ptr(c2base + readlane64(voff, i)) + ld_off_l), X[i]);
                if constexpr ((i % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
              });
            keep_live(voff);  // keep voff: copy2 store offsets (region divergent on ld_live)
          }
          if (do_copy && !RS2_ABL_NOCOPY) {
            const int64_t cl = int64_t(tg.line0) * ib.copy_line_stride;
            g8* cbase = (g8*)ib.copy_base + tg.bo_cp + cl;
            const uint32_t cdl = lg.dl * uint32_t(ib.copy_line_stride);
            const uint32_t c_off = lg.ld_off + cdl;
            const int64_t climit = ib.copy_limit - int64_t(cdl);
            const int64_t cfast =
                ib.copy_limit - int64_t(dl_max_of(tg) * uint32_t(ib.copy_line_stride)) - cl - s;
            const uint64_t cpm = __builtin_amdgcn_ballot_w64(l < PPW && vcp >= 0);
            const uint64_t cfm = __builtin_amdgcn_ballot_w64(l < PPW && vcp >= 0 && vcp <= cfast);
            if (lg.ld_live)
              sfor<PPW>([&](auto ii) RS2_INL {
                constexpr int i = decltype(ii)::value;
                if ((cfm >> i) & 1u)
                  st32(reinterpret_cast<g32*>(sgpr_ptr(cbase + readlane64(vcp, i)) + c_off), X[i]);
                if constexpr ((i % kWin) == kWin - 1) __builtin_amdgcn_sched_barrier(0);
              });
            keep_live(vcp);  // keep vcp: fused copy-out offsets (region divergent on ld_live)
            if (cpm != cfm)
              sfor<PPW>([&](auto ii) RS2_INL {
                constexpr int i = decltype(ii)::value;
                if (((cpm & ~cfm) >> i) & 1u) {
                  const int64_t co = readlane64(vcp, i);
                  g8* dst = sgpr_ptr(cbase + co);
                  const int64_t room = climit - (cl + co);
                  if (room >= s) {
                    if (lg.ld_live) st32(reinterpret_cast<g32*>(dst + c_off), X[i]);
                  } else if (room > 0 && lg.ld_live) {
                    for (uint32_t b2 = 0; b2 < 4; ++b2)
                      if (int64_t(lg.ld_off + b2) < room) dst[c_off + b2] = uint8_t(X[i] >> (8 * b2));
                  }
                }
              });
          }
          const uint32_t sel = sel_load(), live = lg.ld_live ? ~0u : 0u;
          sfor<PPW>([&](auto ii) RS2_INL {
            constexpr int i = decltype(ii)::value;
            const uint32_t v = (X[i] >> lg.ld_sh) & live;
            X[i] = __builtin_amdgcn_perm(swap_adjacent(v), v, sel);
          });
        }
        phase_a<G, false>(X, tabw);
      }
      stamp();  // copies, in-wave IFFT (tail: its stores)
      if (loader) {
        // A -> B: the block's waves write their regions (their last other-wave access, B -> A
        // writes, was ordered by the barriers above)
        wave_lds_handoff();
        write_a<G>(X, sU, w);
      }
      __syncthreads();
      read_b<G>(X, sU, wl0 * PPW * 64, (NW - wl0) * PPW / NW, w, l);
      phase_b<G, false>(X, sTabB, ib.count, ib.zero_first != 0);
      if constexpr (!kShared) {
        if (is_head) sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] = 0u; });
        if (k2)
          mix_into<kTabU16 * 2>(A, k2, lds_addr(launder(sTabM)),
                                [&](auto ii) RS2_INL { return X[decltype(ii)::value]; });
      }
#undef ib
      stamp();  // transpose, cross-wave IFFT, mixing
      if (is_head) tail = false;  // (its stores are issued)
    }
    uint32_t k_next = 0;
    if (dyn && w == 0 && l == 0) k_next = take(xcd);
    for (int o = 0; o < n_out; ++o) {
      if constexpr (kShared)
        sfor<PPW>([&](auto ii) RS2_INL { A[decltype(ii)::value] = X[decltype(ii)::value]; });
      const OutBlock& ob = job.out[o];
      phase_b<G, true>(A, (const lds16*)((const uint8_t RS2_AS(3)*)sTabO + o * G::TB_SLOT),
                       ob.trunc, ob.zero_first != 0);
      stamp();  // cross-wave FFT
      // (the transpose's first barrier publishes it)
      if (dyn && o == 0 && w == 0 && l == 0) s_tile[(it + 1) & 1] = resolve(k_next);
      transpose<G, false, true>(A, sU, w, l);
      stamp();  // transpose B -> A
      if (o < last) {
        tail_fft(o, false);
        tail_store(o, t);
        stamp();  // in-wave FFT + stores
      }
    }
    // the last output's tables are issued now, ahead of the next tile's loads, so that its
    // in-wave layers run while those loads are in flight
    if (w * PPW < job.out[last].trunc) tail_tables(last);
    tail = true;
    tail_tile = t;
    if (dyn) {
      ++it;
      t = s_tile[it & 1];
    } else {
      t += nx;
    }
  }
  if (tail) {
    tail_fft(last, true);
    tail_store(last, tail_tile);
  }
  if (dyn && w == 0 && l == 0) {
    // the last workgroup to finish zeroes the counters for the next launch on them (every
    // workgroup's last take has returned: no other workgroup touches them any more)
    const uint32_t done =
        __hip_atomic_fetch_add(ctr + kXcds, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1)
      for (uint32_t x = 0; x <= kXcds; ++x)
        __hip_atomic_store(ctr + x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#undef job
}

}  // namespace

// One kernel per mode so rocprofv3 attributes time per stage.
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4) rs2_encode_mixed_kernel(const CodecJob job) {
  codec_body<C, kModeRows>(job);
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4) rs2_encode_shared_kernel(const CodecJob job) {
  codec_body<C, kModeCols>(job);
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4) rs2_encode_shared_pipe_kernel(
    const CodecJob job) {
  if constexpr (Geo<C>::NW > 1) pipe_body<C, true>(job);
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4) rs2_encode_mixed_pipe_kernel(
    const CodecJob job) {
  if constexpr (Geo<C>::NW > 1) pipe_body<C, false>(job);
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4) rs2_decode_kernel(const CodecJob job) {
  codec_body<C, 3>(job);  // kDecodeRt (see codec_body)
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4) rs2_decode_persist_kernel(const CodecJob job) {
  codec_body<C, 3, true>(job);
}

// Jobs of more than kMaxBlocks blocks (n_shards above about 24,580), read from device memory
// (the same bodies; one-tile kernels only, C = 512).
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4)
    rs2_encode_mixed_big_kernel(const CodecJobBig* __restrict__ job) {
  codec_body<C, kModeRows, false, CodecJobBig>(*job);
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4)
    rs2_encode_shared_big_kernel(const CodecJobBig* __restrict__ job) {
  codec_body<C, kModeCols, false, CodecJobBig>(*job);
}
template <int C>
__global__ void __launch_bounds__(Geo<C>::THREADS, 4)
    rs2_decode_big_kernel(const CodecJobBig* __restrict__ job) {
  codec_body<C, 3, false, CodecJobBig>(*job);
}

}  // namespace rs2

#define RS2_CAT2(a, b) a##b
#define RS2_CAT(a, b) RS2_CAT2(a, b)

extern "C" hipError_t RS2_CAT(rs2k_launch_codec_, RS2_C)(const rs2::CodecJob* job, int n_tiles,
                                                         int n_lines, int n_z, int mode,
                                                         hipStream_t stream) {
  const dim3 grid(n_tiles, n_lines, n_z), block(rs2::Geo<RS2_C>::THREADS);
  switch (mode) {
    case rs2::kModeRows:
      hipLaunchKernelGGL(rs2::rs2_encode_mixed_kernel<RS2_C>, grid, block, 0, stream, *job);
      break;
    case rs2::kModeCols:
      hipLaunchKernelGGL(rs2::rs2_encode_shared_kernel<RS2_C>, grid, block, 0, stream, *job);
      break;
    case rs2::kModeDecode:
      hipLaunchKernelGGL(rs2::rs2_decode_kernel<RS2_C>, grid, block, 0, stream, *job);
      break;
    case rs2::kModeDecodePersist:
      hipLaunchKernelGGL(rs2::rs2_decode_persist_kernel<RS2_C>, grid, block, 0, stream, *job);
      break;
    case rs2::kModeColsPipe:
      if constexpr (rs2::Geo<RS2_C>::NW > 1) {
        hipLaunchKernelGGL(rs2::rs2_encode_shared_pipe_kernel<RS2_C>, grid, block, 0, stream,
                           *job);
        break;
      }
      return hipErrorInvalidValue;
    case rs2::kModeRowsPipe:
      if constexpr (rs2::Geo<RS2_C>::NW > 1) {
        hipLaunchKernelGGL(rs2::rs2_encode_mixed_pipe_kernel<RS2_C>, grid, block, 0, stream,
                           *job);
        break;
      }
      return hipErrorInvalidValue;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#if RS2_C == 512
// CodecJobBig jobs (device memory): modes kModeRows / kModeCols / kModeDecode only
extern "C" hipError_t rs2k_launch_codec_big_512(const rs2::CodecJobBig* d_job, int n_tiles,
                                                int n_lines, int n_z, int mode,
                                                hipStream_t stream) {
  const dim3 grid(n_tiles, n_lines, n_z), block(rs2::Geo<512>::THREADS);
  switch (mode) {
    case rs2::kModeRows:
      hipLaunchKernelGGL(rs2::rs2_encode_mixed_big_kernel<512>, grid, block, 0, stream, d_job);
      break;
    case rs2::kModeCols:
      hipLaunchKernelGGL(rs2::rs2_encode_shared_big_kernel<512>, grid, block, 0, stream, d_job);
      break;
    case rs2::kModeDecode:
      hipLaunchKernelGGL(rs2::rs2_decode_big_kernel<512>, grid, block, 0, stream, d_job);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
#endif
