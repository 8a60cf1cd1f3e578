// Correctness probe for the inline-asm GF multiply forms (vs the C nibble-table form).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
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
#define SDWA_ADD(dst, w, sel) "v_add_u32_sdwa " dst ", %[tb], " w " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" sel "\n"
#define ADDRS                                   \
  "v_lshlrev_b32 %[w0], 1, %[y]\n"               \
  "v_lshrrev_b32 %[w1], 3, %[y]\n"               \
  "v_and_b32 %[w0], 0x1e1e1e1e, %[w0]\n"         \
  "v_and_b32 %[w1], 0x1e1e1e1e, %[w1]\n"         \
  SDWA_ADD("%[a0]", "%[w0]", "BYTE_0")           \
  SDWA_ADD("%[a1]", "%[w0]", "BYTE_2")           \
  SDWA_ADD("%[a2]", "%[w1]", "BYTE_0")           \
  SDWA_ADD("%[a3]", "%[w1]", "BYTE_2")           \
  SDWA_ADD("%[a4]", "%[w0]", "BYTE_1")           \
  SDWA_ADD("%[a5]", "%[w0]", "BYTE_3")           \
  SDWA_ADD("%[a6]", "%[w1]", "BYTE_1")           \
  SDWA_ADD("%[a7]", "%[w1]", "BYTE_3")

// variant 0: d16/d16_hi merge into the same registers (as in the codec)
__device__ uint32_t m0(uint32_t y, uint32_t tb) {
  uint32_t x = 0, w0, w1, a0, a1, a2, a3, a4, a5, a6, a7;
  asm volatile(ADDRS
      "ds_read_u16_d16 %[w0], %[a0]\n"
      "ds_read_u16_d16_hi %[w0], %[a1]\n"
      "ds_read_u16_d16 %[w1], %[a2] offset:32\n"
      "ds_read_u16_d16_hi %[w1], %[a3] offset:32\n"
      "ds_read_u16_d16 %[a0], %[a4] offset:64\n"
      "ds_read_u16_d16_hi %[a0], %[a5] offset:64\n"
      "ds_read_u16_d16 %[a1], %[a6] offset:96\n"
      "ds_read_u16_d16_hi %[a1], %[a7] offset:96\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_bitop3_b32 %[x], %[w0], %[w1], %[a0] bitop3:0x96\n"
      "v_xor_b32 %[x], %[x], %[a1]\n"
      : [x] "=&v"(x), [w0] "=&v"(w0), [w1] "=&v"(w1), [a0] "=&v"(a0), [a1] "=&v"(a1),
        [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7)
      : [y] "v"(y), [tb] "v"(tb));
  return x;
}
// variant 1: plain u16 loads into 8 registers, then pack (checks the address math alone)
__device__ uint32_t m1(uint32_t y, uint32_t tb) {
  uint32_t w0, w1, a0, a1, a2, a3, a4, a5, a6, a7;
  asm volatile(ADDRS
      "ds_read_u16 %[a0], %[a0]\n"
      "ds_read_u16 %[a1], %[a1]\n"
      "ds_read_u16 %[a2], %[a2] offset:32\n"
      "ds_read_u16 %[a3], %[a3] offset:32\n"
      "ds_read_u16 %[a4], %[a4] offset:64\n"
      "ds_read_u16 %[a5], %[a5] offset:64\n"
      "ds_read_u16 %[a6], %[a6] offset:96\n"
      "ds_read_u16 %[a7], %[a7] offset:96\n"
      "s_waitcnt lgkmcnt(0)\n"
      : [w0] "=&v"(w0), [w1] "=&v"(w1), [a0] "=&v"(a0), [a1] "=&v"(a1),
        [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7)
      : [y] "v"(y), [tb] "v"(tb));
  return (a0 ^ a2 ^ a4 ^ a6) | ((a1 ^ a3 ^ a5 ^ a7) << 16);
}
// variant 2: d16 merge, but hi loads into fresh zeroed registers
__device__ uint32_t m2(uint32_t y, uint32_t tb) {
  uint32_t w0, w1, a0, a1, a2, a3, a4, a5, a6, a7, r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  asm volatile(ADDRS
      "ds_read_u16_d16 %[r0], %[a0]\n"
      "s_waitcnt lgkmcnt(0)\n"
      "ds_read_u16_d16_hi %[r0], %[a1]\n"
      "ds_read_u16_d16 %[r1], %[a2] offset:32\n"
      "s_waitcnt lgkmcnt(0)\n"
      "ds_read_u16_d16_hi %[r1], %[a3] offset:32\n"
      "ds_read_u16_d16 %[r2], %[a4] offset:64\n"
      "s_waitcnt lgkmcnt(0)\n"
      "ds_read_u16_d16_hi %[r2], %[a5] offset:64\n"
      "ds_read_u16_d16 %[r3], %[a6] offset:96\n"
      "s_waitcnt lgkmcnt(0)\n"
      "ds_read_u16_d16_hi %[r3], %[a7] offset:96\n"
      "s_waitcnt lgkmcnt(0)\n"
      : [w0] "=&v"(w0), [w1] "=&v"(w1), [a0] "=&v"(a0), [a1] "=&v"(a1),
        [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7),
        [r0] "+v"(r0), [r1] "+v"(r1), [r2] "+v"(r2), [r3] "+v"(r3)
      : [y] "v"(y), [tb] "v"(tb));
  return r0 ^ r1 ^ r2 ^ r3;
}


// variant 3: element 0 via ds_read_u16 (zero-extended), element 1 via ds_read_u16_d16_hi
// (low half zero-filled on gfx950) into the address registers themselves; XOR all 8.
__device__ uint32_t m3(uint32_t y, uint32_t tb) {
  uint32_t x = 0x12345678u, w0, w1, a0, a1, a2, a3, a4, a5, a6, a7;
  asm volatile(ADDRS
      "ds_read_u16 %[a0], %[a0]\n"
      "ds_read_u16_d16_hi %[a1], %[a1]\n"
      "ds_read_u16 %[a2], %[a2] offset:32\n"
      "ds_read_u16_d16_hi %[a3], %[a3] offset:32\n"
      "ds_read_u16 %[a4], %[a4] offset:64\n"
      "ds_read_u16_d16_hi %[a5], %[a5] offset:64\n"
      "ds_read_u16 %[a6], %[a6] offset:96\n"
      "ds_read_u16_d16_hi %[a7], %[a7] offset:96\n"
      "s_waitcnt lgkmcnt(0)\n"
      "v_bitop3_b32 %[x], %[x], %[a0], %[a1] bitop3:0x96\n"
      "v_bitop3_b32 %[x], %[x], %[a2], %[a3] bitop3:0x96\n"
      "v_bitop3_b32 %[x], %[x], %[a4], %[a5] bitop3:0x96\n"
      "v_bitop3_b32 %[x], %[x], %[a6], %[a7] bitop3:0x96\n"
      : [x] "+v"(x), [w0] "=&v"(w0), [w1] "=&v"(w1), [a0] "=&v"(a0), [a1] "=&v"(a1),
        [a2] "=&v"(a2), [a3] "=&v"(a3), [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7)
      : [y] "v"(y), [tb] "v"(tb));
  return x ^ 0x12345678u;
}

__global__ void check(const uint16_t* tabs, const uint32_t* in, uint32_t* out, int n) {
  __shared__ uint16_t st[8 * 64];
  for (int i = threadIdx.x; i < 8 * 64; i += blockDim.x) st[i] = tabs[i];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = i & 7;
  const lds16* t = (const lds16*)st + c * 64;
  const uint32_t tb = (uint32_t)(uintptr_t)t;
  const uint32_t y = in[i];
  out[4 * i + 0] = tab_mul(y, t);
  out[4 * i + 1] = m0(y, tb);
  out[4 * i + 2] = m1(y, tb);
  out[4 * i + 3] = m3(y, tb);
}

int main() {
  const int n = 1 << 16;
  std::vector<uint16_t> tabs(8 * 64);
  for (auto& v : tabs) v = uint16_t(rand());
  std::vector<uint32_t> in(n);
  for (auto& v : in) v = uint32_t(rand()) ^ (uint32_t(rand()) << 16);
  uint16_t* dt; uint32_t *di, *dout;
  (void)hipMalloc(&dt, tabs.size() * 2); (void)hipMalloc(&di, n * 4); (void)hipMalloc(&dout, n * 16);
  (void)hipMemcpy(dt, tabs.data(), tabs.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(di, in.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, dim3(n / 256), dim3(256), 0, 0, dt, di, dout, n);
  std::vector<uint32_t> out(4 * n);
  (void)hipMemcpy(out.data(), dout, n * 16, hipMemcpyDeviceToHost);
  int bad[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    // host reference
    const uint16_t* t = &tabs[(i & 7) * 64];
    uint32_t v = in[i], a = 0, b = 0;
    for (int k = 0; k < 4; ++k) { a ^= t[16 * k + ((v >> (4 * k)) & 15)]; b ^= t[16 * k + ((v >> (16 + 4 * k)) & 15)]; }
    const uint32_t ref = a | (b << 16);
    for (int m = 0; m < 4; ++m) if (out[4 * i + m] != ref) { if (bad[m] < 3) printf("variant %d i=%d in=%08x got %08x want %08x\n", m - 1, i, v, out[4 * i + m], ref); bad[m]++; }
  }
  printf("mismatches: ctab %d  v0(d16 merge) %d  v1(u16) %d  v3(u16 + d16_hi, 8 regs) %d\n", bad[0], bad[1], bad[2], bad[3]);
  return 0;
}
