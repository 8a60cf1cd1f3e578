// Hashing and data-movement kernels of the MI355X Red Stuff engine (gfx950).
//
// leaf_hash_kernel   Blake2b-256(0x00 || symbol) for every expanded symbol (merkle.rs:313-321),
//                    one lane per symbol, message blocks staged through LDS with coalesced loads.
// merkle_*_kernel    level-synchronous Blake2b trees in LDS, one workgroup per tree
//                    (merkle.rs:226-266), and the pair-leaf root + BlobId (metadata.rs:571-578,
//                    lib.rs:159-176).
// symbol_copy_kernel strided symbol copies (transposed systematic slivers, decode copies).
// build_mul_tables   per-position GF multiplier nibble tables for the decoder.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "rs2_device.h"

namespace rs2 {

template <int N, int I = 0, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<N, I + 1>(f);
  }
}

// ------------------------------------------------------------------------------------------
// Blake2b-256
// ------------------------------------------------------------------------------------------
struct B2 {
  static constexpr uint8_t sigma[12][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
  static constexpr uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                     0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                     0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                     0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
};

// 64-bit rotate right on the two 32-bit halves: 2 v_alignbit_b32 (n != 32), 0 for n == 32.
template <int n, bool kAdd = true>
__device__ __forceinline__ uint64_t rotr64(uint64_t x) {
  const uint32_t lo = uint32_t(x), hi = uint32_t(x >> 32);
  uint32_t rlo, rhi;
  if constexpr (n == 63 && kAdd) {
    // rotate left by one as (x << 1) + (x >> 63): one v_lshl_add_u64 and one 32-bit shift
    uint64_t r;
    const uint64_t t = uint64_t(hi >> 31);
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(x), "v"(t));
    return r;
  } else if constexpr (n == 32) {
    rlo = hi;
    rhi = lo;
  } else if constexpr (n < 32) {
    rlo = __builtin_amdgcn_alignbit(hi, lo, n);
    rhi = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return uint64_t(rlo) | (uint64_t(rhi) << 32);
}

template <int a, int b, int c, int d, bool kAdd>
__device__ __forceinline__ void b2_g(uint64_t (&v)[16], uint64_t x, uint64_t y) {
  v[a] = v[a] + v[b] + x;
  v[d] = rotr64<32, kAdd>(v[d] ^ v[a]);
  v[c] = v[c] + v[d];
  v[b] = rotr64<24, kAdd>(v[b] ^ v[c]);
  v[a] = v[a] + v[b] + y;
  v[d] = rotr64<16, kAdd>(v[d] ^ v[a]);
  v[c] = v[c] + v[d];
  v[b] = rotr64<63, kAdd>(v[b] ^ v[c]);
}

__device__ __forceinline__ void b2_init(uint64_t (&h)[8]) {
  sfor<8>([&](auto ii) { h[decltype(ii)::value] = B2::iv[decltype(ii)::value]; });
  h[0] ^= 0x01010020ULL;  // digest 32, no key, fanout 1, depth 1
}

// kAdd: rotate left by one as one v_lshl_add_u64 + one shift instead of two v_alignbit_b32 (4
// SIMD cycles fewer per G): C3 20.9 -> 21.4 GiB/s through the small-leaf and tree kernels, but
// 1.7 % slower in leaf_hash_kernel, which keeps the alignbits (profiles/r03/exp/rotl/)
template <bool kAdd = true>
__device__ __forceinline__ void b2_compress(uint64_t (&h)[8], const uint64_t (&m)[16], uint64_t t,
                                            bool last) {
  uint64_t v[16];
  sfor<8>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    v[i] = h[i];
    v[i + 8] = B2::iv[i];
  });
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  sfor<12>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    b2_g<0, 4, 8, 12, kAdd>(v, m[B2::sigma[r][0]], m[B2::sigma[r][1]]);
    b2_g<1, 5, 9, 13, kAdd>(v, m[B2::sigma[r][2]], m[B2::sigma[r][3]]);
    b2_g<2, 6, 10, 14, kAdd>(v, m[B2::sigma[r][4]], m[B2::sigma[r][5]]);
    b2_g<3, 7, 11, 15, kAdd>(v, m[B2::sigma[r][6]], m[B2::sigma[r][7]]);
    b2_g<0, 5, 10, 15, kAdd>(v, m[B2::sigma[r][8]], m[B2::sigma[r][9]]);
    b2_g<1, 6, 11, 12, kAdd>(v, m[B2::sigma[r][10]], m[B2::sigma[r][11]]);
    b2_g<2, 7, 8, 13, kAdd>(v, m[B2::sigma[r][12]], m[B2::sigma[r][13]]);
    b2_g<3, 4, 9, 14, kAdd>(v, m[B2::sigma[r][14]], m[B2::sigma[r][15]]);
  });
  sfor<8>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    h[i] ^= v[i] ^ v[i + 8];
  });
}

// Blake2b-256(prefix || 64 bytes given as 16 dwords) -- inner nodes and pair leaves (65 bytes).
__device__ __forceinline__ void b2_hash65(uint32_t prefix, const uint32_t (&d)[16],
                                          uint32_t (&out)[8]) {
  uint32_t M[18];
  M[0] = prefix | (d[0] << 8);
  sfor<15>([&](auto ii) {
    constexpr int t = decltype(ii)::value + 1;
    M[t] = (d[t - 1] >> 24) | (d[t] << 8);
  });
  M[16] = d[15] >> 24;
  M[17] = 0;
  uint64_t m[16];
  sfor<9>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    m[i] = uint64_t(M[2 * i]) | (uint64_t(M[2 * i + 1]) << 32);
  });
  sfor<7>([&](auto ii) { m[9 + decltype(ii)::value] = 0; });
  uint64_t h[8];
  b2_init(h);
  b2_compress(h, m, 65, true);
  sfor<4>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    out[2 * i] = uint32_t(h[i]);
    out[2 * i + 1] = uint32_t(h[i] >> 32);
  });
}

// Leaf hashes of whole runs of symbols that are contiguous in memory.  A workgroup hashes 256
// consecutive symbols of one run, one lane per symbol; every wave stages its own 64 symbols.
// Message block k is staged whole: the wave's LDS buffer gets, per symbol, the 9 x 16 B
// (16-byte aligned) that cover message bytes [128k, 128k+128) (= symbol bytes from 128k-1), in
// chunk order, by LDS-DMA (global_load_lds_dwordx4, no VGPRs).  A symbol's 9 chunks sit in
// neighbouring lanes of one or two DMA instructions (9 DMA instructions per block; round 2's
// two 80-byte half-block windows took 10).  The memory side still reads 1.44x the symbol bytes
// (tools/pmc_reqsize.sh): the line a block's window shares with the next block's is often gone
// from the XCD's L2 a compression later (Leaf hashing).  The next block's DMA is issued as soon as the current block's message words are in registers, so
// its HBM latency hides under the current compression.  Each lane then rebuilds its message
// words from LDS with one alignbyte per dword.
//   mode 0: the n x n expanded matrix as three runs (SymbolMap):
//     A  rows r < n, columns c < K_s   primary + (r*K_s + c)*s           (n*K_s symbols)
//     B  columns c >= K_s, rows r < K_p secondary + (c*K_p + r)*s         ((n-K_s)*K_p)
//     C  rows r >= K_p, columns c >= K_s both + ((r-K_p)*(n-K_s) + c-K_s)*s ((n-K_p)*(n-K_s))
//     leaf (r, c) -> out + (r*n + c)*32
//   mode 1: `count` contiguous symbols at map.primary -> out + idx*32
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Diagnostic ablation knobs (variant builds only, outputs are wrong): no message staging DMA /
// no message words from LDS either (constant messages) -- the hash rate of the bare loop
#ifndef RS2_ABL_LEAF_NOISSUE
#define RS2_ABL_LEAF_NOISSUE 0
#endif
#ifndef RS2_ABL_LEAF_NOBUILD
#define RS2_ABL_LEAF_NOBUILD 0
#endif
// RS2_ABL_LEAF_LINE: every block's window after the first DMA'd from the 128-byte line holding
// its first message byte (its 9th chunk repeats the 8th), so consecutive blocks never share a
// line: the same DMA, LDS and VALU work without the L2 re-fetch -- what the kernel would take
// without its 1.43x traffic
#ifndef RS2_ABL_LEAF_LINE
#define RS2_ABL_LEAF_LINE 0
#endif
constexpr int kLeafThreads = 256;
constexpr int kWinPad = 16;                           // block 0 of an aligned symbol reads the
                                                      // dword before its window (masked off)
// NBW message blocks per staged window: 16 * (8 NBW + 1) bytes per symbol (one 16-byte chunk
// of alignment slack), one wave's windows 64 x that
template <int NBW>
struct LeafWin {
  static constexpr int kChunks = 8 * NBW + 1;
  static constexpr int kWaveBytes = 64 * kChunks * 16;
  static constexpr int kLdsBytes = kWinPad + kLeafThreads / 64 * kWaveBytes;
};

// kLeafWaves: minimum waves per SIMD the register allocation must admit.  3 (145 VGPRs, no
// spills) beat 4 (<= 128 VGPRs, 20 B/lane of spills) and round 2's 123-VGPR half-block kernel:
// leaf hashing 0.413 / 0.446 / 0.425 ms sequential (profiles/r03/exp/leafwin/).  Padding the LDS
// to 2 / 1 workgroups per CU cut the L2 re-fetch (1.40x / 1.17x) but hashed slower
// (profiles/r03/exp/leafocc/).
constexpr int kLeafWaves = 3;
// (two-block windows: 69.6 KiB of LDS per workgroup admit two workgroups per CU, so two waves per
// SIMD is all the occupancy there is to ask for)
template <int NBW>
__global__ void __launch_bounds__(kLeafThreads, NBW == 1 ? kLeafWaves : 2)
    leaf_hash_kernel(SymbolMap map, int mode, int64_t count, int64_t tilesA, int64_t tilesB,
                     int64_t tile0, uint8_t* __restrict__ out) {
  constexpr int kWinChunks = LeafWin<NBW>::kChunks, kWaveBytes = LeafWin<NBW>::kWaveBytes;
  __shared__ __attribute__((aligned(16))) uint8_t win[LeafWin<NBW>::kLdsBytes];
  const int tid = threadIdx.x;
  const int s = map.s;
  const int64_t n = map.n, kp = map.kp, ks = map.ks;
  // run selection (wave-uniform)
  int64_t tile = blockIdx.x + tile0;  // tile0: a launch over the later runs only
  const uint8_t* base;
  int64_t run_len;
  int run;
  const int64_t blob = blockIdx.y;  // blob batches: blob y's symbols and leaves are strided
  if (mode == 1) {
    run = 3;
    base = map.primary;
    run_len = count;
  } else if (mode == 2) {
    // verifier layout (rs2k_launch_leaf_hash mode 4): map.kp rows (slivers) of map.ks systematic
    // symbols back to back at map.primary, then their n - ks repair symbols back to back at
    // map.secondary; leaf (row, c) -> out + (row * n + c) * 32
    if (tile < tilesA) {
      run = 4;
      base = map.primary;
      run_len = kp * ks;
    } else {
      run = 5;
      tile -= tilesA;
      base = map.secondary;
      run_len = kp * (n - ks);
    }
  } else if (tile < tilesA) {
    run = 0;
    base = map.primary + blob * map.primary_stride;
    run_len = n * ks;
  } else if (tile < tilesA + tilesB) {
    run = 1;
    tile -= tilesA;
    base = map.secondary + blob * map.secondary_stride + ks * kp * s;
    run_len = (n - ks) * kp;
  } else {
    run = 2;
    tile -= tilesA + tilesB;
    base = map.both + blob * map.both_stride;
    run_len = (n - kp) * (n - ks);
  }
  out += blob * map.leaf_stride;
  const int64_t j0 = tile * kLeafThreads;
  const int cnt = int(run_len - j0 < kLeafThreads ? run_len - j0 : kLeafThreads);
  const uint8_t* tile_base = base + j0 * s;
  // windows may run past this tile's symbols into the run's next ones (those bytes are masked
  // off the messages); only the run's end bounds them
  const int64_t rend_rel = (run_len - j0) * s;  // run end relative to tile_base
  const uintptr_t end = reinterpret_cast<uintptr_t>(tile_base) + uintptr_t(rend_rel);

  const int lm = s + 1;                 // message length: 0x00 || symbol
  const int nb = (lm + 127) >> 7;
  const bool mine = tid < cnt;
  // this lane's symbol: absolute address a = tile_base + tid*s
  const uintptr_t a = reinterpret_cast<uintptr_t>(tile_base) + uintptr_t(tid) * s;
  uint64_t h[8];
  b2_init(h);
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), wl = tid & 63, wj0 = wv * 64;
  const int wcnt = cnt - wj0 < 0 ? 0 : (cnt - wj0 < 64 ? cnt - wj0 : 64);
  uint8_t* const wbuf = win + kWinPad + wv * kWaveBytes;

  // Fast path: a lane's nine window starts (chunk q = wl + 64 it -> symbol jw = q / 9, piece
  // c = q % 9) as 32-bit offsets from tile_base for M > 0 -- ((a_j + M - 1) & ~15) + 16c is
  // ((a_j - 1) & ~15) + 16c + M since M is a multiple of 128 -- and the extra 16 of block 0
  // (no prefix byte before it) when a_j is 16-byte aligned.  Blocks whose windows all end
  // inside the run (every block but the run's last few bytes) issue the DMAs with no per-lane
  // bounds test.
  const uint32_t tb_lo = uint32_t(reinterpret_cast<uintptr_t>(tile_base)) & 15u;
  const uint8_t* const tb_al = tile_base - tb_lo;  // offsets below are from this 16-B boundary
  int32_t wo[kWinChunks];
  uint32_t aligned_mask = 0;  // bit it: chunk it's symbol starts 16-byte aligned
  sfor<kWinChunks>([&](auto ii) {
    constexpr int it = decltype(ii)::value;
    const int q = wl + 64 * it, jw = q / kWinChunks, c = q - jw * kWinChunks;
    const int32_t rel = (wj0 + jw) * s;
    wo[it] = int32_t((tb_lo + uint32_t(rel) - 1u) & ~15u) + 16 * c;  // -16 only for M > 0 use
    if (((tb_lo + uint32_t(rel)) & 15u) == 0) aligned_mask |= 1u << it;
  });
  const int32_t wo_max = int32_t((tb_lo + uint32_t((wj0 + 63) * s) - 1u) & ~15u) +
                         16 * (kWinChunks - 1);
  // largest M with every window inside the run (16 more for block 0's aligned shift)
  const int64_t fast_lim = rend_rel + tb_lo - 16 - wo_max - 16;
  // stage block k: chunk q = (symbol q / 9, piece q % 9) -> wave buffer + 16q
  auto issue = [&](int k) __attribute__((always_inline)) {
    if (RS2_ABL_LEAF_NOISSUE || RS2_ABL_LEAF_NOBUILD) return;
    const int M = 128 * k;
    if (RS2_ABL_LEAF_LINE && M > 0 && wcnt == 64 && int64_t(M) <= fast_lim) {
      // blocks k >= 1 only: the line holding message byte M (symbol byte M - 1) starts at or
      // after the symbol's own first byte and ends before the standard window's end, so every
      // read stays inside the checked fast-path range
      sfor<kWinChunks>([&](auto ii) {
        constexpr int it = decltype(ii)::value;
        const int q = wl + 64 * it, jw = q / kWinChunks, c = q - jw * kWinChunks;
        const uintptr_t aj = reinterpret_cast<uintptr_t>(tile_base) + uintptr_t(wj0 + jw) * s;
        const uintptr_t line = (aj + uintptr_t(M - 1)) & ~uintptr_t(127);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(line + 16 * (c < 8 ? c : 7)),
                                         (__attribute__((address_space(3))) uint8_t*)(wbuf + 1024 * it),
                                         16, 0, 0);
      });
      return;
    }
    if (wcnt == 64 && int64_t(M) <= fast_lim) {
      sfor<kWinChunks>([&](auto ii) {
        constexpr int it = decltype(ii)::value;
        // block 0 has no prefix byte before it: a window of an aligned symbol starts at the
        // symbol, 16 bytes after the other blocks' rule (exact in 32-bit wrap-around: the sum
        // is never negative)
        const uint32_t off = uint32_t(wo[it] + M) + (M == 0 ? ((aligned_mask >> it) & 1u) * 16u : 0u);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(tb_al + off),
                                         (__attribute__((address_space(3))) uint8_t*)(wbuf + 1024 * it),
                                         16, 0, 0);
      });
      return;
    }
    const int back = M > 0 ? 1 : 0;
    for (int it = 0; it < kWinChunks; ++it) {
      const int q = wl + 64 * it, jw = q / kWinChunks, c = q - jw * kWinChunks;
      if (jw >= wcnt) continue;
      const uintptr_t aj = reinterpret_cast<uintptr_t>(tile_base) + uintptr_t(wj0 + jw) * s;
      const uintptr_t src = ((aj + uintptr_t(M - back)) & ~uintptr_t(15)) + 16 * c;
      if (src + 16 <= end) {
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                         (__attribute__((address_space(3))) uint8_t*)(wbuf + 1024 * it),
                                         16, 0, 0);
      } else {
        // the run's last bytes: 2-byte loads (symbols are 2-byte aligned), never past the end
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int bb = 0; bb < 16 && src + bb < end; bb += 2)
          w[bb >> 2] |= uint32_t(*reinterpret_cast<const uint16_t*>(src + bb)) << (8 * (bb & 3));
        *reinterpret_cast<uint4*>(wbuf + 16 * q) = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  };

  issue(0);
  for (int k = 0; k < nb; ++k) {
    const int kw = k - k % NBW;  // first block of the staged window
    if (k == kw) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this window's DMA has landed
      wave_lds_sync();
    }
    uint64_t m[16];
    const bool edge = k == 0 || k == nb - 1;  // only these blocks need byte masking
    if (RS2_ABL_LEAF_NOBUILD) {
      sfor<16>([&](auto ii) { m[decltype(ii)::value] = uint64_t(tid) * (decltype(ii)::value + 1) + k; });
    } else if (mine) {
      const int M = 128 * k, MW = 128 * kw, back = MW > 0 ? 1 : 0;
      const uintptr_t A = a + uintptr_t(M) - 1;  // message byte M (a - 1 is the prefix)
      const uintptr_t ws = (a + uintptr_t(MW - back)) & ~uintptr_t(15);
      const int o = int(intptr_t(A - ws));       // -1 .. 15, + 128 per block into the window
      const int di = o >> 2;                     // -1 .. 3 (+ 32 per block; arithmetic shift)
      const int sh = o & 3;
      const uint32_t* L = reinterpret_cast<const uint32_t*>(wbuf + wl * kWinChunks * 16) + di;
      auto build = [&](auto masked) __attribute__((always_inline)) {
        uint32_t lo = L[0];
        sfor<16>([&](auto ii) {
          constexpr int i = decltype(ii)::value;
          uint32_t pr[2];
          sfor<2>([&](auto qq_) {
            constexpr int qq = decltype(qq_)::value;
            constexpr int w = 2 * i + qq;
            const uint32_t hi = L[w + 1];
            uint32_t mm = __builtin_amdgcn_alignbyte(hi, lo, sh);
            lo = hi;
            if constexpr (decltype(masked)::value) {
              const int t = k * 32 + w;
              if (t == 0) mm &= 0xFFFFFF00u;  // message byte 0 is the 0x00 leaf prefix
              const int keep = lm - 4 * t;
              if (keep < 4) mm = keep <= 0 ? 0u : (mm & ((1u << (8 * keep)) - 1u));
            }
            pr[qq] = mm;
          });
          m[i] = uint64_t(pr[0]) | (uint64_t(pr[1]) << 32);
        });
      };
      if (edge)
        build(std::true_type{});
      else
        build(std::false_type{});
    }
    // the window's last message words are in registers: the buffers take the next window
    // while this block hashes
    if (k % NBW == NBW - 1 || k + 1 == nb) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wave_lds_sync();
      if (k + 1 < nb) issue(k + 1);
    }
    if (mine) {
      const bool last = k == nb - 1;
      b2_compress<false>(h, m, last ? uint64_t(lm) : uint64_t(128) * (k + 1), last);
    }
  }
  if (!mine) return;
  const int64_t idx = j0 + tid;
  int64_t leaf;
  if (run == 3) {
    leaf = idx;
  } else if (run == 4) {
    leaf = (idx / ks) * n + idx % ks;
  } else if (run == 5) {
    leaf = (idx / (n - ks)) * n + ks + idx % (n - ks);
  } else if (run == 0) {
    leaf = (idx / ks) * n + idx % ks;
  } else if (run == 1) {
    leaf = (idx % kp) * n + ks + idx / kp;
  } else {
    leaf = (kp + idx / (n - ks)) * n + ks + idx % (n - ks);
  }
  uint4* o = reinterpret_cast<uint4*>(out + leaf * 32);
  o[0] = make_uint4(uint32_t(h[0]), uint32_t(h[0] >> 32), uint32_t(h[1]), uint32_t(h[1] >> 32));
  o[1] = make_uint4(uint32_t(h[2]), uint32_t(h[2] >> 32), uint32_t(h[3]), uint32_t(h[3] >> 32));
}

// Leaf hashes of symbols whose message (0x00 || symbol) fits one 128-byte Blake2b block
// (s <= 126; C3's 4 MiB blobs at n = 1000 have s = 20): one lane per symbol, its bytes loaded
// straight into registers -- no LDS windows, whose 144-byte staging per 128 message bytes and
// 36 KiB per workgroup cost more than these short messages carry.  Same runs, tiles and leaf
// order as leaf_hash_kernel.  Dwords are loaded from the symbol's 4-byte-aligned start, never
// below it (the prefix byte is synthesized) and never past the run's end (2-byte loads there).
// NZ: message words (8 bytes) that can be non-zero, ceil((s + 1) / 8): the others are constant
// zeros, so the compression's additions of them fold away (C3's s = 20: 3 of 16 words)
template <int NZ>
__global__ void __launch_bounds__(kLeafThreads)
    leaf_hash_small_kernel(SymbolMap map, int mode, int64_t count, int64_t tilesA,
                           int64_t tilesB, int64_t tile0, uint8_t* __restrict__ out) {
  const int tid = threadIdx.x;
  const int s = map.s;
  const int64_t n = map.n, kp = map.kp, ks = map.ks;
  int64_t tile = blockIdx.x + tile0;
  const uint8_t* base;
  int64_t run_len;
  int run;
  const int64_t blob = blockIdx.y;
  if (mode == 1) {
    run = 3;
    base = map.primary;
    run_len = count;
  } else if (mode == 2) {
    // verifier layout (rs2k_launch_leaf_hash mode 4): map.kp rows (slivers) of map.ks systematic
    // symbols back to back at map.primary, then their n - ks repair symbols back to back at
    // map.secondary; leaf (row, c) -> out + (row * n + c) * 32
    if (tile < tilesA) {
      run = 4;
      base = map.primary;
      run_len = kp * ks;
    } else {
      run = 5;
      tile -= tilesA;
      base = map.secondary;
      run_len = kp * (n - ks);
    }
  } else if (tile < tilesA) {
    run = 0;
    base = map.primary + blob * map.primary_stride;
    run_len = n * ks;
  } else if (tile < tilesA + tilesB) {
    run = 1;
    tile -= tilesA;
    base = map.secondary + blob * map.secondary_stride + ks * kp * s;
    run_len = (n - ks) * kp;
  } else {
    run = 2;
    tile -= tilesA + tilesB;
    base = map.both + blob * map.both_stride;
    run_len = (n - kp) * (n - ks);
  }
  out += blob * map.leaf_stride;
  const int64_t idx = tile * kLeafThreads + tid;
  if (idx >= run_len) return;
  const uintptr_t end = reinterpret_cast<uintptr_t>(base) + uintptr_t(run_len * s);
  const uintptr_t a = reinterpret_cast<uintptr_t>(base) + uintptr_t(idx * s);
  const uintptr_t A = a & ~uintptr_t(3);
  const int off = int(a - A);  // 0 .. 3 (s may be odd through rs2_merkle_root)
  const int lm = s + 1;
  // E[k] = dword at A + 4k (k < 33 covers s <= 126 plus the alignment)
  auto dword_at = [&](uintptr_t p) -> uint32_t {
    if (p + 4 <= end) return *reinterpret_cast<const uint32_t*>(p);
    uint32_t v = 0;
    for (int b = 0; b < 3; ++b)
      if (p + b < end) v |= uint32_t(*reinterpret_cast<const uint8_t*>(p + b)) << (8 * b);
    return v;
  };
  const int need = (off + s + 3) >> 2;  // dwords holding the symbol
  uint32_t E[33];
  sfor<33>([&](auto kk) {
    constexpr int k = decltype(kk)::value;
    E[k] = k < need ? dword_at(A + 4 * k) : 0u;
  });
  // message word t = bytes A + off - 1 + 4t .. +3: off >= 1 -> alignbyte(E[t+1], E[t], off - 1);
  // off = 0 -> alignbyte(E[t], E[t-1], 3) with E[-1] = 0 (byte 0 is the prefix either way)
  uint32_t M[32];
  sfor<32>([&](auto tt) {
    constexpr int t = decltype(tt)::value;
    uint32_t w;
    if (off != 0) {
      w = __builtin_amdgcn_alignbyte(t + 1 < 33 ? E[t + 1] : 0u, E[t], uint32_t(off - 1));
    } else {
      w = __builtin_amdgcn_alignbyte(E[t], t > 0 ? E[t > 0 ? t - 1 : 0] : 0u, 3);
    }
    if (t == 0) w &= 0xFFFFFF00u;  // message byte 0 is the 0x00 leaf prefix
    const int keep = lm - 4 * t;
    if (keep < 4) w = keep <= 0 ? 0u : (w & ((1u << (8 * keep)) - 1u));
    M[t] = w;
  });
  uint64_t m[16];
  sfor<16>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    if constexpr (i < NZ)
      m[i] = uint64_t(M[2 * i]) | (uint64_t(M[2 * i + 1]) << 32);
    else
      m[i] = 0;
  });
  uint64_t h[8];
  b2_init(h);
  b2_compress(h, m, uint64_t(lm), true);
  int64_t leaf;
  if (run == 3) {
    leaf = idx;
  } else if (run == 4) {
    leaf = (idx / ks) * n + idx % ks;
  } else if (run == 5) {
    leaf = (idx / (n - ks)) * n + ks + idx % (n - ks);
  } else if (run == 0) {
    leaf = (idx / ks) * n + idx % ks;
  } else if (run == 1) {
    leaf = (idx % kp) * n + ks + idx / kp;
  } else {
    leaf = (kp + idx / (n - ks)) * n + ks + idx % (n - ks);
  }
  uint4* o = reinterpret_cast<uint4*>(out + leaf * 32);
  o[0] = make_uint4(uint32_t(h[0]), uint32_t(h[0] >> 32), uint32_t(h[1]), uint32_t(h[1] >> 32));
  o[1] = make_uint4(uint32_t(h[2]), uint32_t(h[2] >> 32), uint32_t(h[3]), uint32_t(h[3] >> 32));
}

// ------------------------------------------------------------------------------------------
// Merkle trees (merkle.rs:226-266): odd levels padded with an all-zero node.
// ------------------------------------------------------------------------------------------
constexpr int kMerkleMax = 4096;  // leaves of one tree (n_shards) in the tree / root kernels
constexpr int kMerkleThreads = 512;

// In place over one buffer of cnt + 1 nodes: chunk i0 reads nodes [2*i0, 2*i0 + 2T) into
// registers, a barrier, then writes [i0, i0 + T); later chunks only read past 2*(i0 + T).
__device__ void merkle_reduce(uint32_t (*buf)[8], int cnt, int tid, uint32_t (&root)[8]) {
  while (cnt > 1) {
    if (cnt & 1) {
      if (tid < 8) buf[cnt][tid] = 0u;
      ++cnt;
    }
    __syncthreads();
    const int half = cnt >> 1;
    for (int i0 = 0; i0 < half; i0 += kMerkleThreads) {
      const int i = i0 + tid;
      uint32_t o[8];
      if (i < half) {
        uint32_t d[16];
        sfor<8>([&](auto jj) {
          constexpr int j = decltype(jj)::value;
          d[j] = buf[2 * i][j];
          d[j + 8] = buf[2 * i + 1][j];
        });
        b2_hash65(1u, d, o);
      }
      __syncthreads();
      if (i < half) sfor<8>([&](auto jj) { buf[i][decltype(jj)::value] = o[decltype(jj)::value]; });
      __syncthreads();
    }
    cnt = half;
  }
  sfor<8>([&](auto jj) { root[decltype(jj)::value] = buf[0][decltype(jj)::value]; });
}

// One WAVE per tree (up to 4 or kTreeWaves trees per workgroup: blockDim.x / 64, fewer when the
// slabs of 4 would not fit the LDS), no workgroup barriers.  Tree t is over
// leaf hashes leaves + base_t + j * stride_t (j < n):
//   t <  n_row_trees: base = t * row_base, stride = row_stride          (rows)
//   else            : base = (n-1-u) * col_base, stride = col_stride    (columns, u = t - n_rows)
// root -> out + u * out_stride + (t < n_row_trees ? 0 : 32).
// Level 0 hashes leaf pairs straight from HBM into the wave's LDS slab ((n+1)/2 nodes); every
// later level runs in place in that slab, 64 nodes per round: a round reads nodes
// [128k, 128k+128) and writes [64k, 64k+64), so once its reads are in registers its writes
// never clobber a node a later round still needs.
// Trees (waves) per workgroup: 4, or 8 for launches of many trees (blob batches: wave 0 then
// finishes the top levels of 8 trees in one pass -- C3 22.1 vs 21.8 GiB/s -- while one blob's
// 2n trees keep 4, as 8 leaves CUs without a workgroup: step 87.7 vs 87.9 GiB/s,
// profiles/r05/exp/treewaves8/)
constexpr int kTreeWaves = 8;
constexpr int kTreeManyTrees = 16384;  // launches of at least this many trees take 8 per workgroup


// nodes != null: tree t also stores all its nodes at nodes + t * nodes_stride in the reference's
// MerkleTree::nodes order (merkle.rs:226-266): level by level from the leaf hashes, every level
// of more than one node padded to even with the all-zero node, the root last -- the array
// MerkleTree::get_proof (merkle.rs:281-309) reads sibling paths from.
__global__ void __launch_bounds__(64 * kTreeWaves)
    merkle_trees_kernel(const uint8_t* __restrict__ leaves, int n, int n_trees, int n_row_trees,
                        int64_t row_base, int64_t row_stride, int64_t col_base, int64_t col_stride,
                        uint8_t* __restrict__ out, int64_t out_stride,
                        uint8_t* __restrict__ nodes, int64_t nodes_stride,
                        int64_t leaves_blob_stride, int64_t out_blob_stride) {
  extern __shared__ uint32_t tree_slab[];
  // blob batches: blob y's leaves and roots are strided (nodes are never requested then)
  leaves += int64_t(blockIdx.y) * leaves_blob_stride;
  out += int64_t(blockIdx.y) * out_blob_stride;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x * int(blockDim.x >> 6) + wv;
  if (t >= n_trees) return;
  const int half0 = (n + 1) >> 1;
  // roots only: the first two hash levels are fused in registers (a lane hashes 4 consecutive
  // leaves into 2 + 1 nodes), so the LDS levels start at the second level's (half0 + 1) / 2
  // nodes: half the slab of one tree, twice the resident waves (the launcher sizes the slab)
  const bool fused = nodes == nullptr && n > 2;
  const int slab_nodes = fused ? ((half0 + 1) >> 1) + 1 : half0 + 1;
  uint32_t(*buf)[8] = reinterpret_cast<uint32_t(*)[8]>(tree_slab + wv * slab_nodes * 8);
  const bool is_row = t < n_row_trees;
  const int u = is_row ? t : t - n_row_trees;
  const int64_t base = is_row ? int64_t(u) * row_base : int64_t(n - 1 - u) * col_base;
  const int64_t stride = is_row ? row_stride : col_stride;
  uint32_t* tn = nodes ? reinterpret_cast<uint32_t*>(nodes + int64_t(t) * nodes_stride) : nullptr;
  auto store_node = [&](int64_t at, const uint32_t (&v)[8]) {
    uint4* q = reinterpret_cast<uint4*>(tn + 8 * at);
    q[0] = make_uint4(v[0], v[1], v[2], v[3]);
    q[1] = make_uint4(v[4], v[5], v[6], v[7]);
  };
  uint32_t root[8];
  if (tn) {  // level 0: the leaf hashes themselves (+ the padding node)
    for (int i = lane; i < n; i += 64) {
      const uint4* a = reinterpret_cast<const uint4*>(leaves + base + int64_t(i) * stride);
      uint4* q = reinterpret_cast<uint4*>(tn + 8 * int64_t(i));
      q[0] = a[0];
      q[1] = a[1];
    }
    if (n > 1 && (n & 1) && lane == 0) {
      const uint32_t z[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      store_node(n, z);
    }
  }
  int64_t lvl_base = n > 1 ? n + (n & 1) : n;  // first node of the level being produced
  if (n == 1) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(leaves + base);
    sfor<8>([&](auto jj) { root[decltype(jj)::value] = src[decltype(jj)::value]; });
  } else {
    int cnt = half0;
    auto load_leaf = [&](int j, uint32_t* d) {
      if (j < n) {
        const uint4* a = reinterpret_cast<const uint4*>(leaves + base + int64_t(j) * stride);
        const uint4 a0 = a[0], a1 = a[1];
        d[0] = a0.x; d[1] = a0.y; d[2] = a0.z; d[3] = a0.w;
        d[4] = a1.x; d[5] = a1.y; d[6] = a1.z; d[7] = a1.w;
      } else {
        sfor<8>([&](auto jj) { d[decltype(jj)::value] = 0u; });
      }
    };
    if (fused) {
      // node 2i of the first level = inner(leaf 4i, leaf 4i+1), node 2i+1 = inner(leaf 4i+2,
      // leaf 4i+3) when 2i+1 < half0 (else the zero node); missing leaves are the zero node
      cnt = (half0 + 1) >> 1;
      for (int i = lane; i < cnt; i += 64) {
        uint32_t d[16], e[16], o[8];
        load_leaf(4 * i, d);
        load_leaf(4 * i + 1, d + 8);
        const bool has_b = 2 * i + 1 < half0;
        if (has_b) {
          load_leaf(4 * i + 2, e);
          load_leaf(4 * i + 3, e + 8);
        }
        b2_hash65(1u, d, o);
        sfor<8>([&](auto jj) { d[decltype(jj)::value] = o[decltype(jj)::value]; });
        if (has_b) {
          b2_hash65(1u, e, o);
          sfor<8>([&](auto jj) { d[8 + decltype(jj)::value] = o[decltype(jj)::value]; });
        } else {
          sfor<8>([&](auto jj) { d[8 + decltype(jj)::value] = 0u; });
        }
        b2_hash65(1u, d, o);
        sfor<8>([&](auto jj) { buf[i][decltype(jj)::value] = o[decltype(jj)::value]; });
      }
    }
    // level 0: leaf pairs from HBM (the odd last leaf pairs with the all-zero node)
    for (int i = lane; i < (fused ? 0 : half0); i += 64) {
      uint32_t d[16], o[8];
      const uint4* a = reinterpret_cast<const uint4*>(leaves + base + int64_t(2 * i) * stride);
      const uint4 a0 = a[0], a1 = a[1];
      uint4 b0 = make_uint4(0u, 0u, 0u, 0u), b1 = b0;
      if (2 * i + 1 < n) {
        const uint4* b = reinterpret_cast<const uint4*>(leaves + base + int64_t(2 * i + 1) * stride);
        b0 = b[0];
        b1 = b[1];
      }
      d[0] = a0.x; d[1] = a0.y; d[2] = a0.z; d[3] = a0.w;
      d[4] = a1.x; d[5] = a1.y; d[6] = a1.z; d[7] = a1.w;
      d[8] = b0.x; d[9] = b0.y; d[10] = b0.z; d[11] = b0.w;
      d[12] = b1.x; d[13] = b1.y; d[14] = b1.z; d[15] = b1.w;
      b2_hash65(1u, d, o);
      sfor<8>([&](auto jj) { buf[i][decltype(jj)::value] = o[decltype(jj)::value]; });
      if (tn) store_node(lvl_base + i, o);
    }
    // each wave alone while a level has more than 64 nodes; below that wave 0 finishes every
    // tree of the workgroup (a level of 32 nodes would keep 4 waves half idle)
    while (cnt > 64) {
      wave_lds_sync();
      if (cnt & 1) {
        if (lane < 8) buf[cnt][lane] = 0u;
        if (tn && lane == 0) {
          const uint32_t z[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
          store_node(lvl_base + cnt, z);
        }
        ++cnt;
        wave_lds_sync();
      }
      const int half = cnt >> 1;
      lvl_base += cnt;
      for (int i0 = 0; i0 < half; i0 += 64) {
        const int i = i0 + lane;
        uint32_t d[16], o[8];
        if (i < half) {
          sfor<8>([&](auto jj) {
            constexpr int j = decltype(jj)::value;
            d[j] = buf[2 * i][j];
            d[j + 8] = buf[2 * i + 1][j];
          });
          b2_hash65(1u, d, o);
          if (tn) store_node(lvl_base + i, o);
        }
        wave_lds_sync();
        if (i < half) sfor<8>([&](auto jj) { buf[i][decltype(jj)::value] = o[decltype(jj)::value]; });
      }
      cnt = half;
    }
    if (cnt > 1) {
      // the top levels of the workgroup's trees (same n, so the same shape) by wave 0: lane g of
      // a round takes tree g / half, node g % half
      const int nt = min(int(blockDim.x >> 6), n_trees - int(blockIdx.x) * int(blockDim.x >> 6));
      __syncthreads();
      if (wv != 0) return;
      uint32_t(*all)[8] = reinterpret_cast<uint32_t(*)[8]>(tree_slab);
      auto tree_nodes = [&](int q) -> uint32_t* {
        return nodes ? reinterpret_cast<uint32_t*>(nodes + int64_t(blockIdx.x * (blockDim.x >> 6) + q) *
                                                           nodes_stride)
                     : nullptr;
      };
      while (cnt > 1) {
        if (cnt & 1) {
          for (int g = lane; g < nt * 8; g += 64) all[(g >> 3) * slab_nodes + cnt][g & 7] = 0u;
          if (nodes && lane < nt) {
            const uint32_t z[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
            uint4* q = reinterpret_cast<uint4*>(tree_nodes(lane) + 8 * (lvl_base + cnt));
            q[0] = make_uint4(z[0], z[1], z[2], z[3]);
            q[1] = make_uint4(z[4], z[5], z[6], z[7]);
          }
          ++cnt;
          wave_lds_sync();
        }
        const int half = cnt >> 1;
        lvl_base += cnt;
        for (int g0 = 0; g0 < nt * half; g0 += 64) {
          const int g = g0 + lane;
          const int q = g / half, i = g - q * half;
          uint32_t d[16], o[8];
          if (g < nt * half) {
            uint32_t(*tb)[8] = all + q * slab_nodes;
            sfor<8>([&](auto jj) {
              constexpr int j = decltype(jj)::value;
              d[j] = tb[2 * i][j];
              d[j + 8] = tb[2 * i + 1][j];
            });
            b2_hash65(1u, d, o);
            if (nodes) {
              uint4* qq = reinterpret_cast<uint4*>(tree_nodes(q) + 8 * (lvl_base + i));
              qq[0] = make_uint4(o[0], o[1], o[2], o[3]);
              qq[1] = make_uint4(o[4], o[5], o[6], o[7]);
            }
          }
          wave_lds_sync();
          if (g < nt * half)
            sfor<8>([&](auto jj) { all[q * slab_nodes + i][decltype(jj)::value] = o[decltype(jj)::value]; });
        }
        cnt = half;
      }
      wave_lds_sync();
      // roots: lane q writes tree q's
      if (lane < nt) {
        const int tq = blockIdx.x * int(blockDim.x >> 6) + lane;
        const bool row_q = tq < n_row_trees;
        const int uq = row_q ? tq : tq - n_row_trees;
        uint32_t* o = reinterpret_cast<uint32_t*>(out + int64_t(uq) * out_stride + (row_q ? 0 : 32));
        sfor<8>([&](auto jj) { o[decltype(jj)::value] = all[lane * slab_nodes][decltype(jj)::value]; });
      }
      return;
    }
    wave_lds_sync();
    sfor<8>([&](auto jj) { root[decltype(jj)::value] = buf[0][decltype(jj)::value]; });
  }
  if (lane == 0) {
    uint32_t* o = reinterpret_cast<uint32_t*>(out + int64_t(u) * out_stride + (is_row ? 0 : 32));
    sfor<8>([&](auto jj) { o[decltype(jj)::value] = root[decltype(jj)::value]; });
  }
}

// One level of a Merkle tree of any width: out[i] = inner(in[2i], in[2i+1] or the zero node).
__global__ void __launch_bounds__(256)
    merkle_level_kernel(const uint8_t* __restrict__ in, int64_t cnt, uint8_t* __restrict__ out) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= (cnt + 1) / 2) return;
  uint32_t d[16], o[8];
  const uint32_t* a = reinterpret_cast<const uint32_t*>(in + 64 * i);
  sfor<8>([&](auto jj) { d[decltype(jj)::value] = a[decltype(jj)::value]; });
  if (2 * i + 1 < cnt) {
    sfor<8>([&](auto jj) { d[8 + decltype(jj)::value] = a[8 + decltype(jj)::value]; });
  } else {
    sfor<8>([&](auto jj) { d[8 + decltype(jj)::value] = 0u; });
  }
  b2_hash65(1u, d, o);
  uint32_t* p = reinterpret_cast<uint32_t*>(out + 32 * i);
  sfor<8>([&](auto jj) { p[decltype(jj)::value] = o[decltype(jj)::value]; });
}

// Full node arrays (MerkleTree::nodes order, merkle.rs:226-266) of trees too wide for one wave's
// LDS slab (n > kMerkleMax), one level per launch through HBM: node j of the destination level
// of tree t (total = trees * dst_cnt lanes).  Level 0 (src == null): leaf j of the tree kernel's
// addressing (rows t * row_base + j * row_stride, columns (n - 1 - u) * col_base + j * col_stride);
// later levels: inner(src[2j], src[2j + 1]) from the previous level of the same array, which the
// previous launch padded to even.  `pad`: the level's count is odd and above one, so node dst_cnt
// is the zero node (written by lane j == dst_cnt).  The one-node level is the root, also
// written to out + u * out_stride (+ 32 for column trees).
__global__ void __launch_bounds__(256)
    merkle_nodes_level_kernel(const uint8_t* __restrict__ leaves, int n, int n_row_trees,
                              int64_t row_base, int64_t row_stride, int64_t col_base,
                              int64_t col_stride, uint8_t* __restrict__ nodes,
                              int64_t nodes_stride, int64_t src_off, int64_t dst_off,
                              int64_t dst_cnt, int pad, int64_t total,
                              uint8_t* __restrict__ out, int64_t out_stride) {
  const int64_t g = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (g >= total) return;
  const int64_t w = dst_cnt + pad;
  const int64_t t = g / w, j = g - t * w;
  uint8_t* tn = nodes + t * nodes_stride;
  uint32_t o[8];
  if (j == dst_cnt) {
    sfor<8>([&](auto jj) { o[decltype(jj)::value] = 0u; });
  } else if (src_off < 0) {
    const bool row = t < n_row_trees;
    const int64_t base = row ? t * row_base : (n - 1 - (t - n_row_trees)) * col_base;
    const uint32_t* a = reinterpret_cast<const uint32_t*>(
        leaves + base + j * (row ? row_stride : col_stride));
    sfor<8>([&](auto jj) { o[decltype(jj)::value] = a[decltype(jj)::value]; });
  } else {
    uint32_t d[16];
    const uint32_t* a = reinterpret_cast<const uint32_t*>(tn + (src_off + 2 * j) * 32);
    sfor<16>([&](auto jj) { d[decltype(jj)::value] = a[decltype(jj)::value]; });
    b2_hash65(1u, d, o);
  }
  uint32_t* p = reinterpret_cast<uint32_t*>(tn + (dst_off + j) * 32);
  sfor<8>([&](auto jj) { p[decltype(jj)::value] = o[decltype(jj)::value]; });
  if (dst_cnt == 1 && src_off >= 0) {
    const bool row = t < n_row_trees;
    uint32_t* r = reinterpret_cast<uint32_t*>(out + (row ? t : t - n_row_trees) * out_stride +
                                              (row ? 0 : 32));
    sfor<8>([&](auto jj) { r[decltype(jj)::value] = o[decltype(jj)::value]; });
  }
}

// Node j of level L (L >= 1) of a tree over n leaf digests at leaves + base + i * stride: the
// level-(L-1) nodes 2j and 2j + 1 hashed together, the right one the zero node when 2j + 1 is
// past level L-1's count ceil(n / 2^(L-1)) (odd levels padded, merkle.rs:226-266); computed in
// registers from its 2^L leaves.
template <int L>
__device__ __forceinline__ void fold_node(const uint8_t* __restrict__ leaves, int64_t base,
                                          int64_t stride, int64_t n, int64_t j,
                                          uint32_t (&out)[8]) {
  uint32_t d[16];
  if constexpr (L == 1) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(leaves + base + 2 * j * stride);
    sfor<8>([&](auto jj) { d[decltype(jj)::value] = a[decltype(jj)::value]; });
    if (2 * j + 1 < n) {
      const uint32_t* b = reinterpret_cast<const uint32_t*>(leaves + base + (2 * j + 1) * stride);
      sfor<8>([&](auto jj) { d[8 + decltype(jj)::value] = b[decltype(jj)::value]; });
    } else {
      sfor<8>([&](auto jj) { d[8 + decltype(jj)::value] = 0u; });
    }
  } else {
    const int64_t below = (n + (int64_t(1) << (L - 1)) - 1) >> (L - 1);  // level L-1's count
    uint32_t l[8], r[8];
    fold_node<L - 1>(leaves, base, stride, n, 2 * j, l);
    if (2 * j + 1 < below) {
      fold_node<L - 1>(leaves, base, stride, n, 2 * j + 1, r);
    } else {
      sfor<8>([&](auto jj) { r[decltype(jj)::value] = 0u; });
    }
    sfor<8>([&](auto jj) {
      d[decltype(jj)::value] = l[decltype(jj)::value];
      d[8 + decltype(jj)::value] = r[decltype(jj)::value];
    });
  }
  b2_hash65(1u, d, out);
}

// Level L of `n_trees` trees of n > kMerkleMax leaves (rs2k_launch_merkle_trees beyond one
// workgroup's LDS), L the smallest with ceil(n / 2^L) <= kMerkleMax: node j of tree t folded
// from its 2^L leaves with the tree kernel's leaf addressing (rows: t * row_base + j * row_stride;
// columns, u = t - n_row_trees: (n - 1 - u) * col_base + j * col_stride), written to
// out + (t * m + j) * 32, m = ceil(n / 2^L).  One lane per node; the trees kernel then reduces
// the m-node levels.  (Round 4 built levels 1 and 2 by a launch each into twice the scratch.)
template <int L>
__global__ void __launch_bounds__(256)
    merkle_fold_kernel(const uint8_t* __restrict__ leaves, int n, int n_row_trees,
                       int64_t row_base, int64_t row_stride, int64_t col_base,
                       int64_t col_stride, int64_t total, uint8_t* __restrict__ out) {
  const int64_t g = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (g >= total) return;
  const int64_t m = (int64_t(n) + (int64_t(1) << L) - 1) >> L;
  const int64_t t = g / m, j = g - t * m;
  const int64_t base = t < n_row_trees ? t * row_base : (n - 1 - (t - n_row_trees)) * col_base;
  const int64_t stride = t < n_row_trees ? row_stride : col_stride;
  uint32_t o[8];
  fold_node<L>(leaves, base, stride, n, j, o);
  uint32_t* p = reinterpret_cast<uint32_t*>(out + g * 32);
  sfor<8>([&](auto jj) { p[decltype(jj)::value] = o[decltype(jj)::value]; });
}

// MerkleTree::get_proof (merkle.rs:281-309) + the symbol it authenticates, for request r:
// tree r's sibling path of leaf targets[r] (path_len nodes of 32 B) and symbol targets[r] of
// the r-th expanded sliver (the recovery symbol, slivers.rs:180-213): a systematic symbol
// (t < k) from the sliver itself (sys: back-to-back slivers of k symbols), a repair one from
// rep ([r][n - k][s]).  One workgroup per request.
__global__ void __launch_bounds__(64)
    proof_gather_kernel(const uint8_t* __restrict__ sys, const uint8_t* __restrict__ rep, int n,
                        int k, int s, const uint8_t* __restrict__ nodes, int64_t nodes_stride,
                        const uint16_t* __restrict__ targets, int path_len,
                        uint8_t* __restrict__ sym_out, uint8_t* __restrict__ proof_out) {
  const int r = blockIdx.x, lane = threadIdx.x;
  const int t = targets[r];
  const uint8_t* sp = t < k ? sys + (int64_t(r) * k + t) * s
                            : rep + (int64_t(r) * (n - k) + (t - k)) * s;
  const uint16_t* src = reinterpret_cast<const uint16_t*>(sp);
  uint16_t* dst = reinterpret_cast<uint16_t*>(sym_out + int64_t(r) * s);
  for (int k = lane; k < s / 2; k += 64) dst[k] = src[k];
  // path: level l's sibling of the node on the path (levels padded to even, merkle.rs:293-305)
  for (int e = lane; e < 8 * path_len; e += 64) {
    const int l = e >> 3, w = e & 7;
    int64_t lvl_base = 0, cnt = n;
    int idx = t;
    for (int k = 0; k < l; ++k) {
      cnt += cnt & 1;
      lvl_base += cnt;
      cnt >>= 1;
      idx >>= 1;
    }
    const int64_t sib = lvl_base + (idx ^ 1);
    const uint32_t* tn = reinterpret_cast<const uint32_t*>(nodes + int64_t(r) * nodes_stride);
    reinterpret_cast<uint32_t*>(proof_out + (int64_t(r) * path_len + l) * 32)[w] = tn[8 * sib + w];
  }
}

// MerkleProof::compute_root (merkle.rs:150-169) for `count` proofs: start from leaf digest r,
// climb path r (path_len nodes) by leaf_index[r]'s bits: inner(cur, sib) when the level index
// is even, inner(sib, cur) when odd.  One lane per proof.
__global__ void __launch_bounds__(64)
    proof_root_kernel(const uint8_t* __restrict__ leaf_digests, const uint32_t* __restrict__ leaf_index,
                      const uint8_t* __restrict__ paths, int path_len, int count,
                      uint8_t* __restrict__ roots) {
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= count) return;
  uint32_t cur[8];
  const uint32_t* lf = reinterpret_cast<const uint32_t*>(leaf_digests + int64_t(r) * 32);
  sfor<8>([&](auto jj) { cur[decltype(jj)::value] = lf[decltype(jj)::value]; });
  uint32_t idx = leaf_index[r];
  for (int l = 0; l < path_len; ++l) {
    const uint32_t* sb = reinterpret_cast<const uint32_t*>(paths + (int64_t(r) * path_len + l) * 32);
    uint32_t d[16], o[8];
    const bool right = idx & 1u;
    sfor<8>([&](auto jj) {
      constexpr int j = decltype(jj)::value;
      d[j] = right ? sb[j] : cur[j];
      d[j + 8] = right ? cur[j] : sb[j];
    });
    b2_hash65(1u, d, o);
    sfor<8>([&](auto jj) { cur[decltype(jj)::value] = o[decltype(jj)::value]; });
    idx >>= 1;
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(roots + int64_t(r) * 32);
  sfor<8>([&](auto jj) { o[decltype(jj)::value] = cur[decltype(jj)::value]; });
}

// Node j of level L of the tree over n pair leaves (pair q = 64 bytes at pair_hashes + 64 q,
// leaf-hashed with prefix 0x00), computed in registers (see fold_node).
template <int L>
__device__ __forceinline__ void pair_node(const uint8_t* __restrict__ pair_hashes, int n, int j,
                                          uint32_t (&out)[8]) {
  uint32_t d[16];
  if constexpr (L == 0) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(pair_hashes + int64_t(j) * 64);
    sfor<16>([&](auto jj) { d[decltype(jj)::value] = src[decltype(jj)::value]; });
    b2_hash65(0u, d, out);
  } else {
    const int below = (n + (1 << (L - 1)) - 1) >> (L - 1);
    uint32_t l[8], r[8];
    pair_node<L - 1>(pair_hashes, n, 2 * j, l);
    if (2 * j + 1 < below) {
      pair_node<L - 1>(pair_hashes, n, 2 * j + 1, r);
    } else {
      sfor<8>([&](auto jj) { r[decltype(jj)::value] = 0u; });
    }
    sfor<8>([&](auto jj) {
      d[decltype(jj)::value] = l[decltype(jj)::value];
      d[8 + decltype(jj)::value] = r[decltype(jj)::value];
    });
    b2_hash65(1u, d, out);
  }
}

// Root over the n pair leaves (primary || secondary, leaf prefix 0x00) and the blob id
// Blake2b-256(0x01 || u64le(blob_len) || root)   (metadata.rs:571-578, lib.rs:159-176).
// Blob batches: workgroup b takes pair_hashes + b*n*64 and writes blob_id_out + b*32, with
// blob length blob_lens[b] (device array) or blob_len for every blob when blob_lens is null.
__global__ void __launch_bounds__(kMerkleThreads)
    merkle_root_kernel(const uint8_t* __restrict__ pair_hashes, int n, uint64_t blob_len,
                       uint8_t* __restrict__ blob_id_out, const uint64_t* __restrict__ blob_lens) {
  __shared__ uint32_t bufA[kMerkleMax + 2][8];
  const int tid = threadIdx.x;
  pair_hashes += int64_t(blockIdx.x) * n * 64;
  blob_id_out += int64_t(blockIdx.x) * 32;
  if (blob_lens) blob_len = blob_lens[blockIdx.x];
  // n > kMerkleMax (up to 16 times that): the first lv inner levels are built while the pair
  // leaves are hashed (pair_node), so the LDS holds at most kMerkleMax nodes (odd levels padded
  // with the zero node, as merkle_reduce does)
  int lv = 0;
  while (((n + (1 << lv) - 1) >> lv) > kMerkleMax) ++lv;
  const int m = (n + (1 << lv) - 1) >> lv;
  for (int i = tid; i < m; i += kMerkleThreads) {
    uint32_t o[8];
    switch (lv) {
      case 0: pair_node<0>(pair_hashes, n, i, o); break;
      case 1: pair_node<1>(pair_hashes, n, i, o); break;
      case 2: pair_node<2>(pair_hashes, n, i, o); break;
      case 3: pair_node<3>(pair_hashes, n, i, o); break;
      default: pair_node<4>(pair_hashes, n, i, o); break;
    }
    sfor<8>([&](auto jj) { bufA[i][decltype(jj)::value] = o[decltype(jj)::value]; });
  }
  uint32_t root[8];
  if (n == 0) {
    sfor<8>([&](auto jj) { root[decltype(jj)::value] = 0u; });
  } else {
    merkle_reduce(bufA, m, tid, root);
  }
  if (tid == 0) {
    // message: 0x01 | blob_len (8 bytes LE) | root (32 bytes) = 41 bytes
    uint32_t M[12];
    const uint32_t lo = uint32_t(blob_len), hi = uint32_t(blob_len >> 32);
    M[0] = 1u | (lo << 8);
    M[1] = (lo >> 24) | (hi << 8);
    M[2] = (hi >> 24) | (root[0] << 8);
    sfor<7>([&](auto jj) {
      constexpr int j = decltype(jj)::value + 3;
      M[j] = (root[j - 3] >> 24) | (root[j - 2] << 8);
    });
    M[10] = root[7] >> 24;
    M[11] = 0;
    uint64_t m[16];
    sfor<6>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      m[i] = uint64_t(M[2 * i]) | (uint64_t(M[2 * i + 1]) << 32);
    });
    sfor<10>([&](auto ii) { m[6 + decltype(ii)::value] = 0; });
    uint64_t h[8];
    b2_init(h);
    b2_compress(h, m, 41, true);
    uint32_t* o = reinterpret_cast<uint32_t*>(blob_id_out);
    sfor<4>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      o[2 * i] = uint32_t(h[i]);
      o[2 * i + 1] = uint32_t(h[i] >> 32);
    });
  }
}

// ------------------------------------------------------------------------------------------
// symbol copies (transposed systematic slivers, present originals of a decode)
//   dst + a*dsa + b*dsb  <-  src + a*ssa + b*ssb   (s bytes, u16 granularity), a = blockIdx.y
//   bytes at dst offset >= dst_limit are not written
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    symbol_copy_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ src_a,
                       int64_t ssb, uint8_t* __restrict__ dst, const int64_t* __restrict__ dst_a,
                       int64_t dsb, int count_b, int s, int64_t dst_limit) {
  const int a = blockIdx.y;
  const int64_t so = src_a[a], dof = dst_a[a];
  const int hw = s >> 1;
  const int64_t total = int64_t(count_b) * hw;
  for (int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * 256) {
    const int b = int(idx / hw), k = int(idx % hw);
    const int64_t d = dof + b * dsb + 2 * k;
    const uint16_t v = *reinterpret_cast<const uint16_t*>(src + so + b * ssb + 2 * k);
    if (d + 2 <= dst_limit) {
      *reinterpret_cast<uint16_t*>(dst + d) = v;
    } else if (d < dst_limit) {
      dst[d] = uint8_t(v);
    }
  }
}

// Segment copies (the partitioned encode's exchange packing, partition.py): segment (a, b) is
// `len` bytes from src + src_a[a] + b*ssb to dst + dst_a[a] + b*dsb.  Lanes take consecutive
// U-byte units of consecutive segments, so a wave moves 64 units of one or more contiguous
// segments per instruction; the launcher picks the widest U that divides every offset, stride,
// length and base (U = 16 for the 4 GiB C4 blob's s = 19,280).  Unit -> (segment, a, b) uses
// multiply-high division by host-made constants (flat index < 2^31 per launch).
struct FastDiv {
  uint32_t m, l, d;
};
__device__ __forceinline__ uint32_t fast_div(uint32_t x, FastDiv f) {
  return uint32_t((uint64_t(__umulhi(x, f.m)) + x) >> f.l);
}
template <int U>
struct UnitT;
template <> struct UnitT<1> { using T = uint8_t; };
template <> struct UnitT<2> { using T = uint16_t; };
template <> struct UnitT<4> { using T = uint32_t; };
template <> struct UnitT<8> { using T = uint2; };
template <> struct UnitT<16> { using T = uint4; };

// long segments (>= 256 units): one workgroup per 1024-unit chunk of one segment, so the
// segment's offsets are workgroup-uniform (scalar loads) and every lane moves 4 units
template <int U>
__global__ void __launch_bounds__(256)
    segment_copy_wide_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                             const int64_t* __restrict__ src_a, const int64_t* __restrict__ dst_a,
                             int64_t ssb, int64_t dsb, FastDiv chunks, FastDiv per_a, uint32_t ups) {
  using T = typename UnitT<U>::T;
  const uint32_t seg = fast_div(blockIdx.x, chunks), c = blockIdx.x - seg * chunks.d;
  const uint32_t a = fast_div(seg, per_a), b = seg - a * per_a.d;
  const uint8_t* sp = src + src_a[a] + int64_t(b) * ssb;
  uint8_t* dp = dst + dst_a[a] + int64_t(b) * dsb;
  const uint32_t u0 = c * 1024u + threadIdx.x;
  T v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (u0 + 256u * k < ups) v[k] = *reinterpret_cast<const T*>(sp + int64_t(u0 + 256u * k) * U);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (u0 + 256u * k < ups) *reinterpret_cast<T*>(dp + int64_t(u0 + 256u * k) * U) = v[k];
}

template <int U>
__global__ void __launch_bounds__(256)
    segment_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                        const int64_t* __restrict__ src_a, const int64_t* __restrict__ dst_a,
                        int64_t ssb, int64_t dsb, FastDiv per_seg, FastDiv per_a, uint32_t total) {
  using T = typename UnitT<U>::T;
  for (uint32_t f = blockIdx.x * 256u + threadIdx.x; f < total; f += gridDim.x * 256u) {
    const uint32_t seg = fast_div(f, per_seg), u = f - seg * per_seg.d;
    const uint32_t a = fast_div(seg, per_a), b = seg - a * per_a.d;
    const T v = *reinterpret_cast<const T*>(src + src_a[a] + int64_t(b) * ssb + int64_t(u) * U);
    *reinterpret_cast<T*>(dst + dst_a[a] + int64_t(b) * dsb + int64_t(u) * U) = v;
  }
}

// Quilt V1 column fill (quilt_encoding.rs:1447-1528): quilt symbol (r, c) <- payload bytes
// [r*s, r*s + s) of column c's run (zero past the column's length).  One thread per aligned
// 16-byte piece of the quilt (a plain vector store); its 8 u16 elements are gathered from the
// column runs (symbols are only 2-byte aligned, and an even s never splits an element).
__global__ void __launch_bounds__(256)
    quilt_layout_kernel(const uint8_t* __restrict__ payload, const int64_t* __restrict__ col_off,
                        const uint32_t* __restrict__ col_len, int n_cols, int s, int64_t total,
                        uint8_t* __restrict__ quilt) {
  const int64_t row_bytes = int64_t(n_cols) * s;
  const int64_t pieces = (total + 15) >> 4;
  for (int64_t t = int64_t(blockIdx.x) * 256 + threadIdx.x; t < pieces;
       t += int64_t(gridDim.x) * 256) {
    const int64_t g = t << 4;
    int64_t r = g / row_bytes;
    const int64_t x = g - r * row_bytes;
    int c = int(x / s);
    int k = int(x - int64_t(c) * s);
    uint32_t w[4];
    sfor<8>([&](auto ee) {
      constexpr int e = decltype(ee)::value;
      uint32_t v = 0;
      if (g + 2 * e < total) {
        const int64_t at = r * s + k;  // byte of column c's run
        const int64_t len = col_len[c];
        const uint8_t* src = payload + col_off[c] + at;
        if (at + 2 <= len) {
          v = *reinterpret_cast<const uint16_t*>(src);
        } else if (at < len) {
          v = src[0];
        }
      }
      if constexpr ((e & 1) == 0) {
        w[e >> 1] = v;
      } else {
        w[e >> 1] |= v << 16;
      }
      k += 2;
      if (k == s) {
        k = 0;
        if (++c == n_cols) {
          c = 0;
          ++r;
        }
      }
    });
    if (g + 16 <= total) {
      *reinterpret_cast<uint4*>(quilt + g) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (int e = 0; 2 * e < int(total - g); ++e)
        *reinterpret_cast<uint16_t*>(quilt + g + 2 * e) = uint16_t(w[e >> 1] >> (16 * (e & 1)));
    }
  }
}

// Blob batches: the message of blob y (its blob_lens[y] bytes at src + y*src_stride, zero-filled
// to msg bytes) -> dst + y*dst_stride, the blob's systematic primary slivers.  One thread per
// 16-byte piece; aligned whole pieces move as one vector load / store.
__global__ void __launch_bounds__(256)
    batch_blob_copy_kernel(const uint8_t* __restrict__ src, int64_t src_stride,
                           const uint64_t* __restrict__ blob_lens, int64_t msg,
                           uint8_t* __restrict__ dst, int64_t dst_stride) {
  const int64_t y = blockIdx.y;
  const int64_t len = int64_t(blob_lens[y]);
  const uint8_t* sp0 = src + y * src_stride;
  uint8_t* dp0 = dst + y * dst_stride;
  for (int64_t t = int64_t(blockIdx.x) * 256 + threadIdx.x; t * 16 < msg;
       t += int64_t(gridDim.x) * 256) {
    const int64_t g = t * 16;
    const uint8_t* sp = sp0 + g;
    uint8_t* dp = dp0 + g;
    const bool aligned = ((reinterpret_cast<uintptr_t>(sp) | reinterpret_cast<uintptr_t>(dp)) & 15) == 0;
    if (aligned && g + 16 <= len && g + 16 <= msg) {
      *reinterpret_cast<uint4*>(dp) = *reinterpret_cast<const uint4*>(sp);
    } else if (aligned && g >= len && g + 16 <= msg) {
      *reinterpret_cast<uint4*>(dp) = make_uint4(0u, 0u, 0u, 0u);
    } else {
      for (int e = 0; e < 16 && g + e < msg; ++e) dp[e] = g + e < len ? sp[e] : uint8_t(0);
    }
  }
}

// Per-position multiplier tables (rs2_engine.cpp nib_table layout): out[i][e] = x(e) * exp(logs[i])
// with x(e) = e (e < 64), (e - 64) << 6 (e < 96), (e - 96) << 11  (log 65535 == 0).
__global__ void __launch_bounds__(256)
    build_mul_tables_kernel(const uint16_t* __restrict__ exp_t, const uint16_t* __restrict__ log_t,
                            const uint16_t* __restrict__ logs, int count,
                            uint16_t* __restrict__ out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= count * kTabU16) return;
  const int i = idx / kTabU16, e = idx % kTabU16;
  const uint32_t x = e < 64 ? uint32_t(e) : (e < 96 ? uint32_t(e - 64) << 6 : uint32_t(e - 96) << 11);
  uint16_t r = 0;
  if (x) {
    const uint32_t sum = uint32_t(log_t[x]) + logs[i];
    r = exp_t[(sum + (sum >> 16)) & 0xFFFFu];
  }
  out[idx] = r;
}

// Row gather (the device Default check's unverified rows, rs2_engine.cpp default_check): row a
// of `row_bytes` bytes from src + src_off[a] to dst + a * row_bytes.  Rows are only 2-byte
// aligned (K_s * s bytes), so each thread writes one 4-byte-aligned destination dword from two
// aligned source dwords and an alignbyte; the dwords at a row's two ends are written bytewise.
// grid (ceil(dwords per row / 256), rows).
__global__ void __launch_bounds__(256) row_gather_kernel(const uint8_t* __restrict__ src,
                                                         const int64_t* __restrict__ src_off,
                                                         uint8_t* __restrict__ dst,
                                                         int64_t row_bytes) {
  const int64_t a = blockIdx.y;
  const uintptr_t d0 = reinterpret_cast<uintptr_t>(dst) + uintptr_t(a * row_bytes);
  const uintptr_t d1 = d0 + uintptr_t(row_bytes);
  const uintptr_t s0 = reinterpret_cast<uintptr_t>(src) + uintptr_t(src_off[a]);
  const uintptr_t D = (d0 & ~uintptr_t(3)) + 4 * (uintptr_t(blockIdx.x) * 256 + threadIdx.x);
  if (D >= d1) return;
  if (D >= d0 && D + 4 <= d1) {
    const uintptr_t S = s0 + (D - d0);
    const uintptr_t Sa = S & ~uintptr_t(3);
    const uint32_t sh = uint32_t(S & 3);
    const uint32_t lo = *reinterpret_cast<const uint32_t*>(Sa);
    // the second dword only when the bytes span it (never read past the source row's end)
    const uint32_t hi = sh ? *reinterpret_cast<const uint32_t*>(Sa + 4) : 0u;
    *reinterpret_cast<uint32_t*>(D) = __builtin_amdgcn_alignbyte(hi, lo, sh);
    return;
  }
  for (uintptr_t x = D; x < D + 4; ++x)
    if (x >= d0 && x < d1)
      *reinterpret_cast<uint8_t*>(x) = *reinterpret_cast<const uint8_t*>(s0 + (x - d0));
}

// Small host -> device uploads (rs2_engine.cpp UploadSlots): the kernel reads the pinned,
// device-mapped host slot over PCIe and writes the device buffer, in stream order like any
// launch -- no DMA-engine copy, whose cross-engine dependency on the stream's earlier kernels
// made the issuing thread wait for them (6-28 ms stalls, gpurun_out/r05c traces).  16 bytes
// per lane when both ends are 16-byte aligned, else bytes.
// Completion is reported to the host without an event: a copy with a completion word runs as
// ONE workgroup (a lane per 16 bytes, striding; the slot uploads are a few KiB, <= 512 KiB),
// whose lane 0, once every lane's loads of the slot have returned (the barrier), stores `gen`
// into the slot's word of a coherent, mapped host array; the host reuses the slot once it reads
// that generation.  So a slot's reuse depends on nothing but this kernel having read it -- not on
// the lifetime of the stream it ran on (a plan, verifier or caller stream torn down since).  The
// store is relaxed: the host reads nothing else the GPU wrote, so no release (whose L2
// write-back on gfx950 every other kernel on the XCD would pay for) is needed.
// done == nullptr: no report, a 16-byte chunk per lane over as many workgroups as it takes.
__global__ void __launch_bounds__(256) host_upload_kernel(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, int64_t n,
                                                          uint64_t* done, uint64_t gen) {
  const bool aligned =
      ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  auto chunk = [&](int64_t i) {
    if (i + 16 <= n && aligned) {
      *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
      for (int b = 0; b < 16 && i + b < n; ++b) dst[i + b] = src[i + b];
    }
  };
  if (done) {
    for (int64_t i = int64_t(threadIdx.x) * 16; i < n; i += 256 * 16) chunk(i);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const int64_t i = (int64_t(blockIdx.x) * 256 + threadIdx.x) * 16;
  if (i < n) chunk(i);
}

// The job ring's completion report (UploadSlots::launch_with_job): queued behind the consumer
// kernel that reads the job, one lane stores the generation (stream order: the consumer is done;
// relaxed, as host_upload_kernel's).
__global__ void __launch_bounds__(64) upload_signal_kernel(uint64_t* done, uint64_t gen) {
  if (threadIdx.x == 0) __hip_atomic_store(done, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The encode's padded tail rows (rs2_engine.cpp encode_device): dst[i] = i < have ? src[i] : 0
// for i < total, 4 bytes per thread (byte loads: src is only 2-byte aligned), one launch in place
// of a D2D copy plus a memset (which the runtime splits into three fill kernels on unaligned
// ranges) on the encode's critical path.
__global__ void __launch_bounds__(256) tail_rows_kernel(const uint8_t* __restrict__ src, int64_t have,
                                                        uint8_t* __restrict__ dst, int64_t total) {
  const int64_t i = (int64_t(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i >= total) return;
  if (i + 4 <= have) {
    const uint32_t v = uint32_t(src[i]) | (uint32_t(src[i + 1]) << 8) |
                       (uint32_t(src[i + 2]) << 16) | (uint32_t(src[i + 3]) << 24);
    if (i + 4 <= total && ((reinterpret_cast<uintptr_t>(dst) + uintptr_t(i)) & 3u) == 0) {
      *reinterpret_cast<uint32_t*>(dst + i) = v;
      return;
    }
  }
  for (int b = 0; b < 4 && i + b < total; ++b) dst[i + b] = i + b < have ? src[i + b] : uint8_t(0);
}

}  // namespace rs2

// ------------------------------------------------------------------------------------------
// launchers (called from rs2_engine.cpp)
// ------------------------------------------------------------------------------------------
extern "C" {

// mode 0: every expanded symbol; 1: `count` contiguous symbols; 2: run A only (the primary
// slivers' systematic columns, final after the systematic-column codec); 3: runs B and C
hipError_t rs2k_launch_leaf_hash(rs2::SymbolMap map, int mode, int64_t count, int n_blobs,
                                 uint8_t* d_out, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  if (n_blobs < 1 || n_blobs > 65535 || ((mode == 1 || mode == 4) && n_blobs != 1) || mode < 0 ||
      mode > 4)
    return hipErrorInvalidValue;
  const int64_t T = rs2::kLeafThreads;
  int64_t tilesA = 0, tilesB = 0, tiles, tile0 = 0;
  if (mode == 1) {
    tiles = (count + T - 1) / T;
  } else if (mode == 4) {
    // verifier layout: map.kp rows, map.ks systematic + (n - ks) repair symbols each (kernel
    // mode 2); `count` = all their symbols (rows * n)
    const int64_t n = map.n, rows = map.kp, ks = map.ks;
    tilesA = (rows * ks + T - 1) / T;
    // (no map.secondary: the rows' systematic symbols only -- compute_metadata's run A pieces)
    tilesB = map.secondary ? (rows * (n - ks) + T - 1) / T : 0;
    tiles = tilesA + tilesB;
    mode = 2;
  } else {
    const int64_t n = map.n, kp = map.kp, ks = map.ks;
    tilesA = (n * ks + T - 1) / T;
    tilesB = ((n - ks) * kp + T - 1) / T;
    const int64_t tilesC = ((n - kp) * (n - ks) + T - 1) / T;
    tiles = mode == 2 ? tilesA : mode == 3 ? tilesB + tilesC : tilesA + tilesB + tilesC;
    if (mode == 3) tile0 = tilesA;
    mode = 0;
  }
  if (tiles == 0) return hipSuccess;
  static const bool no_small = [] {  // A/B knob: RS2_SMALL_LEAF=0 keeps the LDS-window kernel
    const char* e = std::getenv("RS2_SMALL_LEAF");
    return e && std::atoi(e) == 0;
  }();
  if (map.s + 1 <= 128 && !no_small) {
    const int nz = (map.s + 1 + 7) / 8;  // 1 .. 16
#define RS2_SMALL(NZ)                                                                          \
  case NZ:                                                                                     \
    hipLaunchKernelGGL(rs2::leaf_hash_small_kernel<NZ>, dim3(unsigned(tiles), unsigned(n_blobs)), \
                       dim3(rs2::kLeafThreads), 0, stream, map, mode, count, tilesA, tilesB,  \
                       tile0, d_out);                                                          \
    break;
    switch (nz) {
      RS2_SMALL(1) RS2_SMALL(2) RS2_SMALL(3) RS2_SMALL(4) RS2_SMALL(5) RS2_SMALL(6)
      RS2_SMALL(7) RS2_SMALL(8) RS2_SMALL(9) RS2_SMALL(10) RS2_SMALL(11) RS2_SMALL(12)
      RS2_SMALL(13) RS2_SMALL(14) RS2_SMALL(15) RS2_SMALL(16)
      default: return hipErrorInvalidValue;
    }
#undef RS2_SMALL
    return hipGetLastError();
  }
  static const int nbw = [] {  // A/B knob: RS2_LEAF_WIN=2 stages two message blocks per window
    const char* e = std::getenv("RS2_LEAF_WIN");
    return e && std::atoi(e) == 2 ? 2 : 1;
  }();
  if (nbw == 2)
    hipLaunchKernelGGL(rs2::leaf_hash_kernel<2>, dim3(unsigned(tiles), unsigned(n_blobs)),
                       dim3(rs2::kLeafThreads), 0, stream, map, mode, count, tilesA, tilesB, tile0,
                       d_out);
  else
    hipLaunchKernelGGL(rs2::leaf_hash_kernel<1>, dim3(unsigned(tiles), unsigned(n_blobs)),
                       dim3(rs2::kLeafThreads), 0, stream, map, mode, count, tilesA, tilesB, tile0,
                       d_out);
  return hipGetLastError();
}

hipError_t rs2k_launch_merkle_trees(const uint8_t* d_leaves, int n, int n_row_trees,
                                    int n_col_trees, int64_t row_base, int64_t row_stride,
                                    int64_t col_base, int64_t col_stride, uint8_t* d_out,
                                    int64_t out_stride, hipStream_t stream,
                                    uint8_t* d_nodes = nullptr, int64_t nodes_stride = 0,
                                    int n_blobs = 1, int64_t leaves_blob_stride = 0,
                                    int64_t out_blob_stride = 0, uint8_t* d_scratch = nullptr) {
  if (n > rs2::kMerkleMax && d_nodes) {
    // full node arrays: one launch per level through HBM (merkle_nodes_level_kernel)
    const int trees = n_row_trees + n_col_trees;
    if (n_blobs != 1 || n > 65535) return hipErrorInvalidValue;
    if (trees == 0) return hipSuccess;
    int64_t cnt = n, src = -1, dst = 0;
    for (;;) {
      const int pad = cnt > 1 && (cnt & 1) ? 1 : 0;
      const int64_t total = int64_t(trees) * (cnt + pad);
      hipLaunchKernelGGL(rs2::merkle_nodes_level_kernel, dim3(unsigned((total + 255) / 256)),
                         dim3(256), 0, stream, d_leaves, n, n_row_trees, row_base, row_stride,
                         col_base, col_stride, d_nodes, nodes_stride, src, dst, cnt, pad, total,
                         d_out, out_stride);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess || cnt == 1) return e;
      src = dst;
      dst += cnt + pad;
      cnt = (cnt + pad) / 2;
    }
  }
  if (n > rs2::kMerkleMax && n <= 16 * rs2::kMerkleMax) {
    // level L (ceil(n / 2^L) <= kMerkleMax) folded straight from the leaves into d_scratch
    // (trees * ceil(n / 2^L) nodes), then trees over it: roots only, one blob
    if (!d_scratch || d_nodes || n_blobs != 1) return hipErrorInvalidValue;
    const int trees = n_row_trees + n_col_trees;
    if (trees == 0) return hipSuccess;
    int L = 1;
    while (((int64_t(n) + (int64_t(1) << L) - 1) >> L) > rs2::kMerkleMax) ++L;
    const int m = int((int64_t(n) + (int64_t(1) << L) - 1) >> L);
    const int64_t total = int64_t(trees) * m;
    const dim3 grid(unsigned((total + 255) / 256)), block(256);
#define RS2_FOLD(LL)                                                                           \
  case LL:                                                                                     \
    hipLaunchKernelGGL(rs2::merkle_fold_kernel<LL>, grid, block, 0, stream, d_leaves, n,       \
                       n_row_trees, row_base, row_stride, col_base, col_stride, total, d_scratch); \
    break;
    switch (L) {
      RS2_FOLD(1) RS2_FOLD(2) RS2_FOLD(3) RS2_FOLD(4)
      default: return hipErrorInvalidValue;
    }
#undef RS2_FOLD
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n_row_trees > 0) {
      e = rs2k_launch_merkle_trees(d_scratch, m, n_row_trees, 0, int64_t(m) * 32, 32, 0, 0, d_out,
                                   out_stride, stream);
      if (e != hipSuccess) return e;
    }
    if (n_col_trees > 0)
      e = rs2k_launch_merkle_trees(d_scratch + int64_t(n_row_trees) * m * 32, m, n_col_trees, 0,
                                   int64_t(m) * 32, 32, 0, 0, d_out + 32, out_stride, stream);
    return e;
  }
  if (n > rs2::kMerkleMax || n < 1) return hipErrorInvalidValue;
  if (n_blobs < 1 || n_blobs > 65535 || (n_blobs > 1 && d_nodes)) return hipErrorInvalidValue;
  const int trees = n_row_trees + n_col_trees;
  if (trees == 0) return hipSuccess;
  // one wave's level buffer (merkle_trees_kernel: roots-only trees fuse the first two levels)
  const size_t slab = size_t(!d_nodes && n > 2 ? ((n + 1) / 2 + 1) / 2 + 1 : (n + 1) / 2 + 1) * 32;
  const int want = int64_t(trees) * n_blobs >= rs2::kTreeManyTrees ? rs2::kTreeWaves : 4;
  const int waves = int(std::min<size_t>(size_t(want), size_t(160 * 1024) / slab));
  const int wgs = (trees + waves - 1) / waves;
  const size_t lds = size_t(waves) * slab;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&rs2::merkle_trees_kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(rs2::merkle_trees_kernel, dim3(wgs, unsigned(n_blobs)),
                     dim3(64 * waves), lds, stream, d_leaves, n, trees, n_row_trees,
                     row_base, row_stride, col_base, col_stride, d_out, out_stride, d_nodes,
                     nodes_stride, leaves_blob_stride, out_blob_stride);
  return hipGetLastError();
}

hipError_t rs2k_launch_proof_gather(const uint8_t* d_sys, const uint8_t* d_rep, int n, int k,
                                    int s, const uint8_t* d_nodes, int64_t nodes_stride,
                                    const uint16_t* d_targets, int count, int path_len,
                                    uint8_t* d_sym, uint8_t* d_proof, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(rs2::proof_gather_kernel, dim3(unsigned(count)), dim3(64), 0, stream, d_sys,
                     d_rep, n, k, s, d_nodes, nodes_stride, d_targets, path_len, d_sym, d_proof);
  return hipGetLastError();
}

hipError_t rs2k_launch_proof_roots(const uint8_t* d_leaf_digests, const uint32_t* d_leaf_index,
                                   const uint8_t* d_paths, int path_len, int count,
                                   uint8_t* d_roots, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(rs2::proof_root_kernel, dim3(unsigned((count + 63) / 64)), dim3(64), 0, stream,
                     d_leaf_digests, d_leaf_index, d_paths, path_len, count, d_roots);
  return hipGetLastError();
}

hipError_t rs2k_launch_merkle_level(const uint8_t* d_in, int64_t cnt, uint8_t* d_out,
                                    hipStream_t stream) {
  const int64_t half = (cnt + 1) / 2;
  if (half <= 0) return hipSuccess;
  hipLaunchKernelGGL(rs2::merkle_level_kernel, dim3(unsigned((half + 255) / 256)), dim3(256), 0,
                     stream, d_in, cnt, d_out);
  return hipGetLastError();
}

hipError_t rs2k_launch_merkle_root(const uint8_t* d_pair_hashes, int n, uint64_t blob_len,
                                   uint8_t* d_blob_id, hipStream_t stream, int n_blobs = 1,
                                   const uint64_t* d_blob_lens = nullptr) {
  if (n > 16 * rs2::kMerkleMax || n_blobs < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rs2::merkle_root_kernel, dim3(unsigned(n_blobs)), dim3(rs2::kMerkleThreads), 0,
                     stream, d_pair_hashes, n, blob_len, d_blob_id, d_blob_lens);
  return hipGetLastError();
}

hipError_t rs2k_launch_symbol_copy(const uint8_t* src, const int64_t* d_src_a, int64_t ssb,
                                   uint8_t* dst, const int64_t* d_dst_a, int64_t dsb, int count_a,
                                   int count_b, int s, int64_t dst_limit, hipStream_t stream) {
  if (count_a <= 0 || count_b <= 0) return hipSuccess;
  const int64_t total = int64_t(count_b) * (s >> 1);
  unsigned bx = unsigned((total + 255) / 256);
  if (bx > 64) bx = 64;
  hipLaunchKernelGGL(rs2::symbol_copy_kernel, dim3(bx, count_a), dim3(256), 0, stream, src,
                     d_src_a, ssb, dst, d_dst_a, dsb, count_b, s, dst_limit);
  return hipGetLastError();
}

static rs2::FastDiv make_fast_div(uint32_t d) {
  uint32_t l = 0;
  while ((uint64_t(1) << l) < d) ++l;
  const uint32_t m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1);
  return rs2::FastDiv{m, l, d};
}

hipError_t rs2k_launch_segment_copy(const uint8_t* src, uint8_t* dst, uint32_t count_a,
                                    const int64_t* d_src_a, const int64_t* d_dst_a, uint32_t count_b,
                                    int64_t ssb, int64_t dsb, uint32_t len, int unit,
                                    hipStream_t stream) {
  if (count_a == 0 || count_b == 0 || len == 0) return hipSuccess;
  const uint32_t ups = len / uint32_t(unit);
  if (ups >= 256) {
    const uint32_t chunks = (ups + 1023) / 1024;
    const uint64_t blocks = uint64_t(count_a) * count_b * chunks;
    if (blocks >= (uint64_t(1) << 31)) return hipErrorInvalidValue;
    const rs2::FastDiv fc = make_fast_div(chunks), fa = make_fast_div(count_b);
#define RS2_SEGW(UU)                                                                           \
  hipLaunchKernelGGL(rs2::segment_copy_wide_kernel<UU>, dim3(unsigned(blocks)), dim3(256), 0,  \
                     stream, src, dst, d_src_a, d_dst_a, ssb, dsb, fc, fa, ups)
    switch (unit) {
      case 16: RS2_SEGW(16); break;
      case 8: RS2_SEGW(8); break;
      case 4: RS2_SEGW(4); break;
      case 2: RS2_SEGW(2); break;
      default: RS2_SEGW(1); break;
    }
#undef RS2_SEGW
    return hipGetLastError();
  }
  const uint64_t per_a = uint64_t(count_b) * ups;
  // a-ranges of at most 2^31 units per launch
  const uint32_t a_step = uint32_t(std::max<uint64_t>(1, (uint64_t(1) << 31) / per_a));
  for (uint32_t a0 = 0; a0 < count_a; a0 += a_step) {
    const uint32_t na = std::min(a_step, count_a - a0);
    const uint64_t total = uint64_t(na) * per_a;
    if (total >= (uint64_t(1) << 32)) return hipErrorInvalidValue;  // one segment row > 2^32 units
    const unsigned grid = unsigned(std::min<uint64_t>((total + 255) / 256, 256 * 64));
    const rs2::FastDiv fs = make_fast_div(ups), fa = make_fast_div(count_b);
#define RS2_SEG(UU)                                                                          \
  hipLaunchKernelGGL(rs2::segment_copy_kernel<UU>, dim3(grid), dim3(256), 0, stream, src, dst, \
                     d_src_a + a0, d_dst_a + a0, ssb, dsb, fs, fa, uint32_t(total))
    switch (unit) {
      case 16: RS2_SEG(16); break;
      case 8: RS2_SEG(8); break;
      case 4: RS2_SEG(4); break;
      case 2: RS2_SEG(2); break;
      default: RS2_SEG(1); break;
    }
#undef RS2_SEG
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t rs2k_launch_quilt_layout(int n_rows, int n_cols, int s, const uint8_t* payload,
                                    const int64_t* col_off, const uint32_t* col_len,
                                    uint8_t* quilt, hipStream_t stream) {
  if (n_rows <= 0 || n_cols <= 0 || s <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(quilt) & 15) return hipErrorInvalidValue;
  const int64_t total = int64_t(n_rows) * n_cols * s;
  int64_t blocks = (((total + 15) >> 4) + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(rs2::quilt_layout_kernel, dim3(unsigned(blocks)), dim3(256), 0, stream,
                     payload, col_off, col_len, n_cols, s, total, quilt);
  return hipGetLastError();
}

hipError_t rs2k_launch_batch_blob_copy(const uint8_t* src, int64_t src_stride,
                                       const uint64_t* d_blob_lens, int64_t msg, uint8_t* dst,
                                       int64_t dst_stride, int n_blobs, hipStream_t stream) {
  if (n_blobs <= 0 || msg <= 0) return hipSuccess;
  if (n_blobs > 65535) return hipErrorInvalidValue;
  const int64_t pieces = (msg + 15) / 16;
  const unsigned bx = unsigned(std::min<int64_t>((pieces + 255) / 256, 4096));
  hipLaunchKernelGGL(rs2::batch_blob_copy_kernel, dim3(bx, unsigned(n_blobs)), dim3(256), 0, stream,
                     src, src_stride, d_blob_lens, msg, dst, dst_stride);
  return hipGetLastError();
}

hipError_t rs2k_launch_build_mul_tables(const uint16_t* d_exp, const uint16_t* d_log,
                                        const uint16_t* d_logs, int count, uint16_t* d_out,
                                        hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  const unsigned blocks = unsigned((count * rs2::kTabU16 + 255) / 256);
  hipLaunchKernelGGL(rs2::build_mul_tables_kernel, dim3(blocks), dim3(256), 0, stream, d_exp,
                     d_log, d_logs, count, d_out);
  return hipGetLastError();
}

hipError_t rs2k_launch_row_gather(const uint8_t* src, const int64_t* d_src_off, uint8_t* dst,
                                  int64_t row_bytes, int rows, hipStream_t stream) {
  if (rows <= 0 || row_bytes <= 0) return hipSuccess;
  const int64_t words = row_bytes / 4 + 2;  // the aligned span of a row
  const int64_t bx = (words + 255) / 256;
  if (bx >= (int64_t(1) << 31) || rows > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rs2::row_gather_kernel, dim3(unsigned(bx), unsigned(rows)), dim3(256), 0,
                     stream, src, d_src_off, dst, row_bytes);
  return hipGetLastError();
}

hipError_t rs2k_launch_host_upload(const void* src, void* dst, int64_t n, uint64_t* done,
                                   uint64_t gen, hipStream_t stream) {
  if (n <= 0 && !done) return hipSuccess;
  // with a completion word: one workgroup (see host_upload_kernel)
  const int64_t blocks = done ? 1 : (n + 4095) / 4096;
  if (blocks >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rs2::host_upload_kernel, dim3(unsigned(blocks)), dim3(256), 0, stream,
                     static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), n, done, gen);
  return hipGetLastError();
}

hipError_t rs2k_launch_upload_signal(uint64_t* done, uint64_t gen, hipStream_t stream) {
  hipLaunchKernelGGL(rs2::upload_signal_kernel, dim3(1), dim3(64), 0, stream, done, gen);
  return hipGetLastError();
}

hipError_t rs2k_launch_tail_rows(const uint8_t* src, int64_t have, uint8_t* dst, int64_t total,
                                 hipStream_t stream) {
  if (total <= 0) return hipSuccess;
  const int64_t blocks = (total + 1023) / 1024;
  if (blocks >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rs2::tail_rows_kernel, dim3(unsigned(blocks)), dim3(256), 0, stream, src,
                     have, dst, total);
  return hipGetLastError();
}

}  // extern "C"
