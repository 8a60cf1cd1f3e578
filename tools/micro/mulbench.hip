// Micro-benchmark: GF(2^16) multiply-by-uniform-constant throughput on gfx950.
//   mode 0: pair lane (u32 = 2 elements), 4 nibble lookups per element in a 128-B LDS table
//   mode 1: quad lane (2 x u32 byte planes = 4 elements), v_perm_b32 3/3/2-bit lookups from
//           uniform (SGPR) tables, no LDS
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define AS3 __attribute__((address_space(3)))
typedef AS3 uint16_t lds16;

__device__ __forceinline__ uint32_t tab_mul(uint32_t v, const lds16* t) {
  const uint32_t a = uint32_t(t[v & 15u]) ^ t[16 + ((v >> 4) & 15u)] ^ t[32 + ((v >> 8) & 15u)] ^
                     t[48 + ((v >> 12) & 15u)];
  const uint32_t b = uint32_t(t[(v >> 16) & 15u]) ^ t[16 + ((v >> 20) & 15u)] ^
                     t[32 + ((v >> 24) & 15u)] ^ t[48 + (v >> 28)];
  return a | (b << 16);
}

constexpr int NREG = 16;
constexpr int NCONST = 64;

__global__ void __launch_bounds__(1024) k_lds(uint32_t* out, const uint16_t* tabs, int iters) {
  __shared__ uint16_t st[NCONST * 64];
  for (int i = threadIdx.x; i < NCONST * 64; i += blockDim.x) st[i] = tabs[i];
  __syncthreads();
  uint32_t x[NREG];
  for (int i = 0; i < NREG; ++i) x[i] = threadIdx.x * 7919u + i * 104729u;
  const lds16* t = (const lds16*)st;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NREG; i += 2) {
      const lds16* tt = t + ((it * NREG + i) % NCONST) * 64;
      x[i] ^= tab_mul(x[i + 1], tt);
      x[i + 1] ^= x[i];
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < NREG; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// T: 20 dwords: lo-plane chunk tables then hi-plane; per chunk {lo-out, hi-out};
// 8-entry tables = 2 dwords (entries 0-3, 4-7), 4-entry = 1 dword
__device__ __forceinline__ void qmul(uint32_t lo, uint32_t hi, const uint32_t* __restrict__ T,
                                     uint32_t& plo, uint32_t& phi) {
  const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
  const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
  plo ^= perm(T[1], T[0], a0) ^ perm(T[5], T[4], a1) ^ perm(0, T[8], a2) ^
         perm(T[11], T[10], b0) ^ perm(T[15], T[14], b1) ^ perm(0, T[18], b2);
  phi ^= perm(T[3], T[2], a0) ^ perm(T[7], T[6], a1) ^ perm(0, T[9], a2) ^
         perm(T[13], T[12], b0) ^ perm(T[17], T[16], b1) ^ perm(0, T[19], b2);
}

__global__ void __launch_bounds__(1024) k_perm(uint32_t* out, const uint32_t* __restrict__ tabs, int iters) {
  uint32_t xl[NREG], xh[NREG];
  for (int i = 0; i < NREG; ++i) {
    xl[i] = threadIdx.x * 7919u + i * 104729u;
    xh[i] = threadIdx.x * 31u + i * 1299709u;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NREG; i += 2) {
      const uint32_t* T = tabs + ((it * NREG + i) % NCONST) * 20;
      qmul(xl[i + 1], xh[i + 1], T, xl[i], xh[i]);
      xl[i + 1] ^= xl[i];
      xh[i + 1] ^= xh[i];
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < NREG; ++i) r ^= xl[i] ^ xh[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}


__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ void qmul3(uint32_t lo, uint32_t hi, const uint32_t* __restrict__ T,
                                      uint32_t& plo, uint32_t& phi) {
  const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
  const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
  plo = x3(x3(x3(plo, perm(T[1], T[0], a0), perm(T[5], T[4], a1)), perm(0, T[8], a2),
              perm(T[11], T[10], b0)), perm(T[15], T[14], b1), perm(0, T[18], b2));
  phi = x3(x3(x3(phi, perm(T[3], T[2], a0), perm(T[7], T[6], a1)), perm(0, T[9], a2),
              perm(T[13], T[12], b0)), perm(T[17], T[16], b1), perm(0, T[19], b2));
}
// 2-bit chunks: 8 per element, 4-entry tables (1 dword) -> T: 16 chunks... [plane][chunk][out]
__device__ __forceinline__ void qmul2(uint32_t lo, uint32_t hi, const uint32_t* __restrict__ T,
                                      uint32_t& plo, uint32_t& phi) {
  uint32_t c[8];
  c[0] = lo & 0x03030303u; c[1] = (lo >> 2) & 0x03030303u; c[2] = (lo >> 4) & 0x03030303u;
  c[3] = (lo >> 6) & 0x03030303u;
  c[4] = hi & 0x03030303u; c[5] = (hi >> 2) & 0x03030303u; c[6] = (hi >> 4) & 0x03030303u;
  c[7] = (hi >> 6) & 0x03030303u;
  uint32_t a = plo, b = phi;
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    a = x3(a, perm(0, T[2 * k], c[k]), perm(0, T[2 * k + 2], c[k + 1]));
    b = x3(b, perm(0, T[2 * k + 1], c[k]), perm(0, T[2 * k + 3], c[k + 1]));
  }
  plo = a; phi = b;
}
template <int MODE>
__global__ void __launch_bounds__(1024) k_permv(uint32_t* out, const uint32_t* __restrict__ tabs, int iters) {
  uint32_t xl[NREG], xh[NREG];
  for (int i = 0; i < NREG; ++i) {
    xl[i] = threadIdx.x * 7919u + i * 104729u;
    xh[i] = threadIdx.x * 31u + i * 1299709u;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NREG; i += 2) {
      const uint32_t* T = tabs + ((it * NREG + i) % NCONST) * 20;
      if (MODE == 2) qmul3(xl[i + 1], xh[i + 1], T, xl[i], xh[i]);
      else qmul2(xl[i + 1], xh[i + 1], T, xl[i], xh[i]);
      xl[i + 1] ^= xl[i];
      xh[i + 1] ^= xh[i];
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < NREG; ++i) r ^= xl[i] ^ xh[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}


typedef unsigned short us2 __attribute__((ext_vector_type(2)));
// v = [e0 lo, e0 hi, e1 lo, e1 hi] bytes; table at LDS byte address tb: [k][16] u16
__device__ __forceinline__ uint32_t tab_mul4(uint32_t v, uint32_t tb) {
  const uint32_t w0 = (v << 1) & 0x1E1E1E1Eu;  // bytes: 2*n0(e0) 2*n2(e0) 2*n0(e1) 2*n2(e1)
  const uint32_t w1 = (v >> 3) & 0x1E1E1E1Eu;  // bytes: 2*n1(e0) 2*n3(e0) 2*n1(e1) 2*n3(e1)
  const lds16* T = (const lds16*)(uintptr_t)0;
  us2 r0, r1, r2, r3;
  r0.x = T[(tb + (w0 & 0xFFu)) >> 1];
  r0.y = T[(tb + ((w0 >> 16) & 0xFFu)) >> 1];
  r1.x = T[(tb + 32 + (w1 & 0xFFu)) >> 1];
  r1.y = T[(tb + 32 + ((w1 >> 16) & 0xFFu)) >> 1];
  r2.x = T[(tb + 64 + ((w0 >> 8) & 0xFFu)) >> 1];
  r2.y = T[(tb + 64 + (w0 >> 24)) >> 1];
  r3.x = T[(tb + 96 + ((w1 >> 8) & 0xFFu)) >> 1];
  r3.y = T[(tb + 96 + (w1 >> 24)) >> 1];
  us2 r = r0 ^ r1 ^ r2 ^ r3;
  return __builtin_bit_cast(uint32_t, r);
}
__global__ void __launch_bounds__(1024) k_lds4(uint32_t* out, const uint16_t* tabs, int iters) {
  __shared__ uint16_t st[NCONST * 64];
  for (int i = threadIdx.x; i < NCONST * 64; i += blockDim.x) st[i] = tabs[i];
  __syncthreads();
  uint32_t x[NREG];
  for (int i = 0; i < NREG; ++i) x[i] = threadIdx.x * 7919u + i * 104729u;
  const uint32_t tb0 = (uint32_t)(uintptr_t)(lds16*)st;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NREG; i += 2) {
      const uint32_t tb = tb0 + ((it * NREG + i) % NCONST) * 128;
      x[i] ^= tab_mul4(x[i + 1], tb);
      x[i + 1] ^= x[i];
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < NREG; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}


#define SDWA_ADD(dst, b, w, sel) "v_add_u32_sdwa " dst ", " b ", " w " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" sel "\n"
// x ^= y * c, table of c at LDS byte address tb ([k][16] u16)
__device__ __forceinline__ void amul1(uint32_t& x, uint32_t y, uint32_t tb) {
  uint32_t w0, w1, a0, a1, a2, a3, a4, a5, a6, a7, r0, r1, r2, r3;
  asm volatile(
      "v_lshlrev_b32 %[w0], 1, %[y]\n"
      "v_lshrrev_b32 %[w1], 3, %[y]\n"
      "v_and_b32 %[w0], 0x1e1e1e1e, %[w0]\n"
      "v_and_b32 %[w1], 0x1e1e1e1e, %[w1]\n"
      SDWA_ADD("%[a0]", "%[tb]", "%[w0]", "BYTE_0")
      SDWA_ADD("%[a1]", "%[tb]", "%[w0]", "BYTE_2")
      SDWA_ADD("%[a2]", "%[tb]", "%[w1]", "BYTE_0")
      SDWA_ADD("%[a3]", "%[tb]", "%[w1]", "BYTE_2")
      SDWA_ADD("%[a4]", "%[tb]", "%[w0]", "BYTE_1")
      SDWA_ADD("%[a5]", "%[tb]", "%[w0]", "BYTE_3")
      SDWA_ADD("%[a6]", "%[tb]", "%[w1]", "BYTE_1")
      SDWA_ADD("%[a7]", "%[tb]", "%[w1]", "BYTE_3")
      "ds_read_u16_d16 %[r0], %[a0]\n"
      "ds_read_u16_d16_hi %[r0], %[a1]\n"
      "ds_read_u16_d16 %[r1], %[a2] offset:32\n"
      "ds_read_u16_d16_hi %[r1], %[a3] offset:32\n"
      "ds_read_u16_d16 %[r2], %[a4] offset:64\n"
      "ds_read_u16_d16_hi %[r2], %[a5] offset:64\n"
      "ds_read_u16_d16 %[r3], %[a6] offset:96\n"
      "ds_read_u16_d16_hi %[r3], %[a7] offset:96\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_bitop3_b32 %[x], %[x], %[r0], %[r1] bitop3:0x96\n"
      "v_bitop3_b32 %[x], %[x], %[r2], %[r3] bitop3:0x96\n"
      : [x] "+v"(x), [w0] "=&v"(w0), [w1] "=&v"(w1), [a0] "=&v"(a0), [a1] "=&v"(a1),
        [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6),
        [a7] "=&v"(a7), [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3)
      : [y] "v"(y), [tb] "v"(tb));
}
__global__ void __launch_bounds__(1024) k_asm1(uint32_t* out, const uint16_t* tabs, int iters) {
  __shared__ uint16_t st[NCONST * 64];
  for (int i = threadIdx.x; i < NCONST * 64; i += blockDim.x) st[i] = tabs[i];
  __syncthreads();
  uint32_t x[NREG];
  for (int i = 0; i < NREG; ++i) x[i] = threadIdx.x * 7919u + i * 104729u;
  const uint32_t tb0 = (uint32_t)(uintptr_t)(lds16*)st;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NREG; i += 2) {
      const uint32_t tb = tb0 + ((it * NREG + i) % NCONST) * 128;
      amul1(x[i], x[i + 1], tb);
      x[i + 1] ^= x[i];
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < NREG; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  const int blocks = 256 * 4, threads = 1024, iters = 512;  // 16 waves per WG
  uint32_t* out;
  uint16_t* t16;
  uint32_t* t32;
  hipMalloc(&out, sizeof(uint32_t) * blocks * threads);
  hipMalloc(&t16, NCONST * 128);
  hipMalloc(&t32, NCONST * 80 + 256);
  std::vector<uint8_t> h(NCONST * 128);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t(i * 37 + 11);
  hipMemcpy(t16, h.data(), NCONST * 128, hipMemcpyHostToDevice);
  std::vector<uint8_t> h2(NCONST * 80);
  for (size_t i = 0; i < h2.size(); ++i) h2[i] = uint8_t((i * 13 + 5) & 0x7F) & 0xFF;  // no perm special selectors needed: tables are data
  hipMemcpy(t32, h2.data(), NCONST * 80, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 6; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(threads), 0, 0, out, t16, iters);
      else if (mode == 1) hipLaunchKernelGGL(k_perm, dim3(blocks), dim3(threads), 0, 0, out, t32, iters);
      else if (mode == 2) hipLaunchKernelGGL(k_permv<2>, dim3(blocks), dim3(threads), 0, 0, out, t32, iters);
      else if (mode == 3) hipLaunchKernelGGL(k_permv<3>, dim3(blocks), dim3(threads), 0, 0, out, t32, iters);
      else if (mode == 4) hipLaunchKernelGGL(k_lds4, dim3(blocks), dim3(threads), 0, 0, out, t16, iters);
      else hipLaunchKernelGGL(k_asm1, dim3(blocks), dim3(threads), 0, 0, out, t16, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double lanes = double(blocks) * threads;
      double mults = lanes * iters * (NREG / 2) * ((mode == 0 || mode >= 4) ? 2 : 4);  // element multiplies
      printf("mode %d (%s): %.3f ms, %.1f G element-mults/s\n", mode, (const char*[]){"lds-pair","perm332","perm332-x3","perm2-x3","lds-pair-d16","lds-asm1"}[mode], ms,
             mults / ms / 1e6);
    }
  }
  return 0;
}
