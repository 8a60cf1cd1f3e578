// Micro-benchmark: issue cost of the VALU instruction forms the codec uses, on gfx950.
// Each kernel runs 8 independent chains of one instruction form, unrolled, at 4 or 8 waves per
// SIMD; s_memtime gives cycles per wave-instruction per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o valubench valubench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

constexpr int kIters = 2048;

#define REP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

#define K_BODY(NAME, INSN)                                                            \
  template <int WPS>                                                                   \
  __global__ void __launch_bounds__(1024, WPS / 4) NAME(uint32_t* out, uint64_t* cyc) { \
    uint32_t r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11,    \
             r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19;                                 \
    uint32_t s = threadIdx.x * 0x9E3779B9u, t = s ^ 0x12345678u;                       \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                  \
    for (int it = 0; it < kIters; ++it) {                                              \
      asm volatile(INSN INSN INSN INSN                                                 \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),       \
                     "+v"(r6), "+v"(r7)                                                \
                   : "v"(s), "v"(t), "s"(0x7eu));                                                   \
    }                                                                                  \
    __syncthreads();                                                                   \
    if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7; \
  }

// 64-bit operands: eight independent register pairs
#define K_BODY64(NAME, INSN)                                                          \
  template <int WPS>                                                                   \
  __global__ void __launch_bounds__(1024, WPS / 4) NAME(uint32_t* out, uint64_t* cyc) { \
    uint64_t r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11,    \
             r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19;                                 \
    uint64_t s = threadIdx.x * 0x9E3779B97F4A7C15ull;                                  \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                  \
    for (int it = 0; it < kIters; ++it) {                                              \
      asm volatile(INSN INSN INSN INSN                                                 \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),       \
                     "+v"(r6), "+v"(r7)                                                \
                   : "v"(s));                                                          \
    }                                                                                  \
    __syncthreads();                                                                   \
    if (threadIdx.x == 0) cyc[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = uint32_t(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7); \
  }

#define X8(FMT) \
  FMT("%0") FMT("%1") FMT("%2") FMT("%3") FMT("%4") FMT("%5") FMT("%6") FMT("%7")

#define F_XOR(R) "v_xor_b32 " R ", " R ", %8\n"
#define F_BITOP3(R) "v_bitop3_b32 " R ", " R ", %8, %9 bitop3:0x96\n"
#define F_SDWA(R) "v_add_u32_sdwa " R ", %8, " R " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
#define F_LSHL(R) "v_lshlrev_b32 " R ", 1, " R "\n"
#define F_ANDOR(R) "v_and_or_b32 " R ", " R ", %8, %9\n"
#define F_PERM(R) "v_perm_b32 " R ", " R ", %8, %9\n"
#define F_ADD(R) "v_add_u32 " R ", " R ", %8\n"
#define F_LSHLADD(R) "v_lshl_add_u32 " R ", " R ", 1, %8\n"
#define F_BFE(R) "v_bfe_u32 " R ", " R ", 5, 6\n"
#define F_ANDK(R) "v_and_b32 " R ", 0x007e007e, " R "\n"
#define F_DPP(R) "v_mov_b32_dpp " R ", " R " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define F_PKADD(R) "v_pk_add_u16 " R ", " R ", %8\n"

#define F_MULHI24(R) "v_mul_hi_u32_u24 " R ", " R ", %8\n"
#define F_MULHI(R) "v_mul_hi_u32 " R ", " R ", %8\n"
#define F_MUL24(R) "v_mul_u32_u24 " R ", " R ", %8\n"
#define F_ASHR(R) "v_ashrrev_i32 " R ", 3, " R "\n"
#define F_LSHR16(R) "v_lshrrev_b16 " R ", 3, " R "\n"
#define F_OR(R) "v_or_b32 " R ", " R ", %8\n"
#define F_SUB(R) "v_sub_u32 " R ", " R ", %8\n"
#define F_CND(R) "v_cndmask_b32 " R ", " R ", %8, vcc\n"
#define F_MAX(R) "v_max_u32 " R ", " R ", %8\n"
#define F_BFI(R) "v_bfi_b32 " R ", " R ", %8, %9\n"
#define F_ALIGNB(R) "v_alignbyte_b32 " R ", " R ", %8, 2\n"
#define F_ANDS(R) "v_and_b32 " R ", s0, " R "\n"
#define F_MOV(R) "v_mov_b32 " R ", %8\n"
#define F_LSHLREV16(R) "v_lshlrev_b16 " R ", 3, " R "\n"
#define F_XORVOP3(R) "v_xor_b32_e64 " R ", " R ", %8\n"
#define F_ADD3(R) "v_add3_u32 " R ", " R ", %8, %9\n"
#define F_LSHRK(R) "v_lshrrev_b32_e64 " R ", 5, " R "\n"

#define F_LSHR5(R) "v_lshrrev_b32 " R ", 5, " R "\n"
#define F_LSHL1E64(R) "v_lshlrev_b32_e64 " R ", 1, " R "\n"
#define F_LSHR5V(R) "v_lshrrev_b32 " R ", %8, " R "\n"
#define F_LSHL1X(R) "v_lshlrev_b32 " R ", 1, %8\n"
#define F_LSHR5X(R) "v_lshrrev_b32 " R ", 5, %8\n"
#define F_LSHR5XE(R) "v_lshrrev_b32_e64 " R ", 5, %8\n"
#define F_ADDYY(R) "v_add_u32 " R ", %8, %8\n"
#define F_ANDS2(R) "v_and_b32 " R ", %10, %8\n"
#define F_BITOP3S(R) "v_bitop3_b32 " R ", %8, %10, %9 bitop3:0xEA\n"

#define F_ALIGNBIT(R) "v_alignbit_b32 " R ", " R ", %8, 24\n"
#define F_PACK(R) "v_pack_b32_f16 " R ", " R ", %8 op_sel:[1,0]\n"
#define F_ADDCO(R) "v_add_co_u32 " R ", vcc, " R ", %8\n"
#define F_LSHLADD64(R) "v_lshl_add_u64 " R ", " R ", 0, %8\n"
#define F_MOV64(R) "v_mov_b64 " R ", %8\n"

K_BODY(k_xor, X8(F_XOR))
K_BODY(k_bitop3, X8(F_BITOP3))
K_BODY(k_sdwa, X8(F_SDWA))
K_BODY(k_lshl, X8(F_LSHL))
K_BODY(k_andor, X8(F_ANDOR))
K_BODY(k_perm, X8(F_PERM))
K_BODY(k_add, X8(F_ADD))
K_BODY(k_lshladd, X8(F_LSHLADD))
K_BODY(k_bfe, X8(F_BFE))
K_BODY(k_andk, X8(F_ANDK))
K_BODY(k_dpp, X8(F_DPP))
K_BODY(k_pkadd, X8(F_PKADD))

K_BODY(k_mulhi24, X8(F_MULHI24))
K_BODY(k_mulhi, X8(F_MULHI))
K_BODY(k_mul24, X8(F_MUL24))
K_BODY(k_ashr, X8(F_ASHR))
K_BODY(k_lshr16, X8(F_LSHR16))
K_BODY(k_or, X8(F_OR))
K_BODY(k_sub, X8(F_SUB))
K_BODY(k_cnd, X8(F_CND))
K_BODY(k_max, X8(F_MAX))
K_BODY(k_bfi, X8(F_BFI))
K_BODY(k_alignb, X8(F_ALIGNB))
K_BODY(k_mov, X8(F_MOV))
K_BODY(k_lshl16, X8(F_LSHLREV16))
K_BODY(k_xorvop3, X8(F_XORVOP3))
K_BODY(k_add3, X8(F_ADD3))
K_BODY(k_lshrk, X8(F_LSHRK))


__global__ void k_check(uint32_t* out) {
  const uint32_t a = 0xF0F0F0F0u ^ threadIdx.x, b = 0xCCCCCCCCu, c = 0xAAAAAAAAu;
  uint32_t d;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xEA" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  out[threadIdx.x] = d ^ ((a & b) | c);  // 0 iff 0xEA = (S0 & S1) | S2
}

K_BODY(k_lshr5, X8(F_LSHR5))
K_BODY(k_lshl1e64, X8(F_LSHL1E64))
K_BODY(k_lshr5v, X8(F_LSHR5V))
K_BODY(k_lshl1x, X8(F_LSHL1X))
K_BODY(k_lshr5x, X8(F_LSHR5X))
K_BODY(k_lshr5xe, X8(F_LSHR5XE))
K_BODY(k_addyy, X8(F_ADDYY))
K_BODY(k_ands2, X8(F_ANDS2))
K_BODY(k_bitop3s, X8(F_BITOP3S))

K_BODY(k_alignbit, X8(F_ALIGNBIT))
K_BODY(k_pack, X8(F_PACK))
K_BODY(k_addco, X8(F_ADDCO))
K_BODY64(k_lshladd64, X8(F_LSHLADD64))
K_BODY64(k_mov64, X8(F_MOV64))

typedef void (*KFn)(uint32_t*, uint64_t*);

int main() {
  uint32_t* out;
  uint64_t* cyc;
  hipMalloc(&out, sizeof(uint32_t) * 512 * 1024);
  hipMalloc(&cyc, sizeof(uint64_t) * 512);
  {
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, out);
    uint32_t h[64];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    uint32_t bad = 0;
    for (int i = 0; i < 64; ++i) bad |= h[i];
    printf("bitop3 0xEA == (S0 & S1) | S2: %s (diff bits %08x)\n", bad ? "NO" : "yes", bad);
  }
  struct K { const char* name; KFn f4, f8; };
  K ks[] = {
      {"v_alignbit_b32", k_alignbit<4>, k_alignbit<8>},
      {"v_pack_b32_f16", k_pack<4>, k_pack<8>},
      {"v_add_co_u32 (vcc)", k_addco<4>, k_addco<8>},
      {"lshrrev 5,R (e32)", k_lshr5<4>, k_lshr5<8>},
      {"lshlrev_e64 1,R", k_lshl1e64<4>, k_lshl1e64<8>},
      {"lshrrev vS,R (e32)", k_lshr5v<4>, k_lshr5v<8>},
      {"lshlrev 1,y (indep)", k_lshl1x<4>, k_lshl1x<8>},
      {"lshrrev 5,y (indep)", k_lshr5x<4>, k_lshr5x<8>},
      {"lshrrev_e64 5,y (indep)", k_lshr5xe<4>, k_lshr5xe<8>},
      {"add y,y (indep)", k_addyy<4>, k_addyy<8>},
      {"and s,y (indep)", k_ands2<4>, k_ands2<8>},
      {"bitop3 y,s,t 0xEA", k_bitop3s<4>, k_bitop3s<8>},
      {"v_xor_b32 (VOP2)", k_xor<4>, k_xor<8>},
      {"v_bitop3_b32", k_bitop3<4>, k_bitop3<8>},
      {"v_add_u32_sdwa", k_sdwa<4>, k_sdwa<8>},
      {"v_lshlrev_b32", k_lshl<4>, k_lshl<8>},
      {"v_and_or_b32", k_andor<4>, k_andor<8>},
      {"v_perm_b32", k_perm<4>, k_perm<8>},
      {"v_add_u32", k_add<4>, k_add<8>},
      {"v_lshl_add_u32", k_lshladd<4>, k_lshladd<8>},
      {"v_bfe_u32", k_bfe<4>, k_bfe<8>},
      {"v_and_b32 literal", k_andk<4>, k_andk<8>},
      {"v_mov_b32_dpp", k_dpp<4>, k_dpp<8>},
      {"v_pk_add_u16", k_pkadd<4>, k_pkadd<8>},
      {"v_mul_hi_u32_u24", k_mulhi24<4>, k_mulhi24<8>},
      {"v_mul_hi_u32", k_mulhi<4>, k_mulhi<8>},
      {"v_mul_u32_u24", k_mul24<4>, k_mul24<8>},
      {"v_ashrrev_i32", k_ashr<4>, k_ashr<8>},
      {"v_lshrrev_b16", k_lshr16<4>, k_lshr16<8>},
      {"v_or_b32", k_or<4>, k_or<8>},
      {"v_sub_u32", k_sub<4>, k_sub<8>},
      {"v_cndmask_b32", k_cnd<4>, k_cnd<8>},
      {"v_max_u32", k_max<4>, k_max<8>},
      {"v_bfi_b32", k_bfi<4>, k_bfi<8>},
      {"v_alignbyte_b32", k_alignb<4>, k_alignb<8>},
      {"v_mov_b32", k_mov<4>, k_mov<8>},
      {"v_lshlrev_b16", k_lshl16<4>, k_lshl16<8>},
      {"v_xor_b32_e64", k_xorvop3<4>, k_xorvop3<8>},
      {"v_add3_u32", k_add3<4>, k_add3<8>},
      {"v_lshrrev_b32_e64", k_lshrk<4>, k_lshrk<8>},
      {"v_alignbit_b32", k_alignbit<4>, k_alignbit<8>},
      {"v_add_co_u32 (vcc)", k_addco<4>, k_addco<8>},
      {"v_lshl_add_u64", k_lshladd64<4>, k_lshladd64<8>},
      {"v_mov_b64", k_mov64<4>, k_mov64<8>},
  };
  for (const K& k : ks) {
    for (int wps : {4}) {
      const int blocks = 256 * (wps / 4);
      double best = 1e30;
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(wps == 4 ? k.f4 : k.f8, dim3(blocks), dim3(1024), 0, 0, out, cyc);
        hipDeviceSynchronize();
        std::vector<uint64_t> c(blocks);
        hipMemcpy(c.data(), cyc, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost);
        double m = 0;
        for (auto v : c) m += double(v);
        m /= blocks;
        best = m < best ? m : best;
      }
      // per SIMD: wps waves x kIters x 32 instructions
      const double per = best / (double(wps) * kIters * 32);
      printf("%-22s %d waves/SIMD: %.2f cycles per wave-instruction per SIMD\n", k.name, wps, per);
    }
  }
  return 0;
}
