// Host side of the MI355X Red Stuff engine: GF(2^16) constant tables, codec job planning,
// blob plans and the C ABI declared in include/walrus_rs2.h.
//
// Reference semantics (paths relative to the reference checkout):
//   encoding/blob_encoding.rs:277-368  encode_with_metadata    -> rs2_encode_device_async
//   encoding/blob_encoding.rs:888-993  BlobDecoder::decode      -> rs2_decode_device_async
//   encoding/basic_encoding.rs:107-429 ReedSolomonEncoder/Decoder -> rs2_encode_1d / rs2_decode_1d
//   reed-solomon-simd 3.1.0 (Cargo.lock:8813): GF tables, skew, rates -- restated in
//   oracle/rs2_oracle.py, mirrored here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <map>
#include <set>
#include <tuple>
#include <memory>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/walrus_rs2.h"
#include "rs2_device.h"

// ---- kernel launchers (rs2_codec.hip per block size, rs2_hash.hip) --------------------------
extern "C" {
#define RS2_DECL(CC)                                                                      \
  hipError_t rs2k_launch_codec_##CC(const rs2::CodecJob* job, int n_tiles, int n_lines, \
                                    int n_z, int mode, hipStream_t stream);
RS2_DECL(1)
RS2_DECL(2)
RS2_DECL(4)
RS2_DECL(8)
RS2_DECL(16)
RS2_DECL(32)
RS2_DECL(64)
RS2_DECL(128)
RS2_DECL(256)
RS2_DECL(512)
#undef RS2_DECL
hipError_t rs2k_launch_leaf_hash(rs2::SymbolMap map, int mode, int64_t count, int n_blobs,
                                 uint8_t* d_out, hipStream_t stream);
hipError_t rs2k_launch_merkle_trees(const uint8_t* d_leaves, int n, int n_row_trees,
                                    int n_col_trees, int64_t row_base, int64_t row_stride,
                                    int64_t col_base, int64_t col_stride, uint8_t* d_out,
                                    int64_t out_stride, hipStream_t stream,
                                    uint8_t* d_nodes = nullptr, int64_t nodes_stride = 0,
                                    int n_blobs = 1, int64_t leaves_blob_stride = 0,
                                    int64_t out_blob_stride = 0, uint8_t* d_scratch = nullptr);
hipError_t rs2k_launch_batch_blob_copy(const uint8_t* src, int64_t src_stride,
                                       const uint64_t* d_blob_lens, int64_t msg, uint8_t* dst,
                                       int64_t dst_stride, int n_blobs, hipStream_t stream);
hipError_t rs2k_launch_proof_gather(const uint8_t* d_sys, const uint8_t* d_rep, int n, int k,
                                    int s, const uint8_t* d_nodes, int64_t nodes_stride,
                                    const uint16_t* d_targets, int count, int path_len,
                                    uint8_t* d_sym, uint8_t* d_proof, hipStream_t stream);
hipError_t rs2k_launch_proof_roots(const uint8_t* d_leaf_digests, const uint32_t* d_leaf_index,
                                   const uint8_t* d_paths, int path_len, int count,
                                   uint8_t* d_roots, hipStream_t stream);
hipError_t rs2k_launch_merkle_root(const uint8_t* d_pair_hashes, int n, uint64_t blob_len,
                                   uint8_t* d_blob_id, hipStream_t stream, int n_blobs = 1,
                                   const uint64_t* d_blob_lens = nullptr);
hipError_t rs2k_launch_merkle_level(const uint8_t* d_in, int64_t cnt, uint8_t* d_out,
                                    hipStream_t stream);
hipError_t rs2k_launch_symbol_copy(const uint8_t* src, const int64_t* d_src_a, int64_t ssb,
                                   uint8_t* dst, const int64_t* d_dst_a, int64_t dsb, int count_a,
                                   int count_b, int s, int64_t dst_limit, hipStream_t stream);
hipError_t rs2k_launch_segment_copy(const uint8_t* src, uint8_t* dst, uint32_t count_a,
                                    const int64_t* d_src_a, const int64_t* d_dst_a, uint32_t count_b,
                                    int64_t ssb, int64_t dsb, uint32_t len, int unit,
                                    hipStream_t stream);
hipError_t rs2k_launch_quilt_layout(int n_rows, int n_cols, int s, const uint8_t* payload,
                                    const int64_t* col_off, const uint32_t* col_len,
                                    uint8_t* quilt, hipStream_t stream);
hipError_t rs2k_launch_host_upload(const void* src, void* dst, int64_t n, uint64_t* done,
                                   uint64_t gen, hipStream_t stream);
hipError_t rs2k_launch_upload_signal(uint64_t* done, uint64_t gen, hipStream_t stream);
hipError_t rs2k_launch_codec_big_512(const rs2::CodecJobBig* d_job, int n_tiles, int n_lines,
                                     int n_z, int mode, hipStream_t stream);
hipError_t rs2k_launch_tail_rows(const uint8_t* src, int64_t have, uint8_t* dst, int64_t total,
                                 hipStream_t stream);
hipError_t rs2k_launch_row_gather(const uint8_t* src, const int64_t* d_src_off, uint8_t* dst,
                                  int64_t row_bytes, int rows, hipStream_t stream);
hipError_t rs2k_launch_build_mul_tables(const uint16_t* d_exp, const uint16_t* d_log,
                                        const uint16_t* d_logs, int count, uint16_t* d_out,
                                        hipStream_t stream);
}

namespace rs2 {
namespace {

// ---------------------------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------------------------
thread_local std::string g_last_error = "ok";

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(RS2_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));    \
  } while (0)

// Diagnostic: RS2_HOST_TRACE=<path> appends one "name ms" line per host-timed section (the
// decode's per-pattern setup), so the cost of individual calls can be read, not only the mean.
void host_trace(const char* name, double ms) {
  static FILE* f = [] {
    const char* e = std::getenv("RS2_HOST_TRACE");
    return e ? std::fopen(e, "a") : nullptr;
  }();
  if (!f) return;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  std::fprintf(f, "%s %.4f\n", name, ms);
  std::fflush(f);
}

// ---------------------------------------------------------------------------------------------
// GF(2^16) tables (reed-solomon-simd engine/tables.rs restated; see oracle/rs2_oracle.py)
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kOrder = 65536, kModulus = 65535, kPoly = 0x1002D;
constexpr uint16_t kCantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                  0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

struct Gf {
  std::vector<uint16_t> exp, log, skew;
  Gf() : exp(kOrder), log(kOrder), skew(kModulus) {
    std::vector<uint32_t> e(kOrder), l(kOrder);
    uint32_t state = 1;
    for (uint32_t i = 0; i < kModulus; ++i) {
      e[state] = i;
      state <<= 1;
      if (state >= kOrder) state ^= kPoly;
    }
    e[0] = kModulus;
    l[0] = 0;
    for (int i = 0; i < 16; ++i) {
      const uint32_t width = 1u << i;
      for (uint32_t j = 0; j < width; ++j) l[j + width] = l[j] ^ kCantor[i];
    }
    for (uint32_t i = 0; i < kOrder; ++i) l[i] = e[l[i]];
    for (uint32_t i = 0; i < kOrder; ++i) e[l[i]] = i;
    e[kModulus] = e[0];
    for (uint32_t i = 0; i < kOrder; ++i) {
      exp[i] = uint16_t(e[i]);
      log[i] = uint16_t(l[i]);
    }
    // skew LUT
    std::vector<uint32_t> sk(kModulus, 0);
    uint32_t temp[15];
    for (int i = 1; i < 16; ++i) temp[i - 1] = 1u << i;
    for (int m = 0; m < 15; ++m) {
      const uint32_t step = 1u << (m + 1);
      sk[(1u << m) - 1] = 0;
      for (int i = m; i < 15; ++i) {
        const uint32_t s = 1u << (i + 1);
        for (uint32_t j = (1u << m) - 1; j < s; j += step) sk[j + s] = sk[j] ^ temp[i];
      }
      temp[m] = kModulus - log[mul(temp[m], log[temp[m] ^ 1])];
      for (int i = m + 1; i < 15; ++i) temp[i] = mul(temp[i], add_mod(log[temp[i] ^ 1], temp[m]));
    }
    for (uint32_t i = 0; i < kModulus; ++i) skew[i] = log[sk[i]];
  }
  static uint32_t add_mod(uint32_t a, uint32_t b) {
    const uint32_t s = a + b;
    return (s + (s >> 16)) & 0xFFFFu;
  }
  // x * exp(log_m) with the generic semantics (log_m == 65535 is log 0, i.e. times one)
  uint32_t mul(uint32_t x, uint32_t log_m) const {
    return x == 0 ? 0 : exp[add_mod(log[x], log_m)];
  }
};

const Gf& gf() {
  static const Gf g;
  return g;
}

// 256-byte multiplier table of exp(log_m), one sub-table per bit field of the operand
// (rs2_device.h kTabU16): out[f] = f * m (bits 0-5, 64 entries), out[64 + f] = (f << 6) * m
// (bits 6-10), out[96 + f] = (f << 11) * m (bits 11-15).  Multiplication by a constant is
// GF(2)-linear, so x * m is the XOR of the three entries its fields select.  Each sub-table
// spans at most 32 dwords, so a wave's lookups into it never bank-conflict.
// fft_zero: a butterfly constant log_m == 65535 means multiply by ZERO (engine special case).
void nib_table(uint32_t log_m, bool fft_zero, uint16_t* out) {
  const Gf& g = gf();
  const bool zero = fft_zero && log_m == kModulus;
  for (uint32_t e = 0; e < uint32_t(kTabU16); ++e) {
    const uint32_t x = e < 64 ? e : (e < 96 ? (e - 64) << 6 : (e - 96) << 11);
    out[e] = zero ? 0 : uint16_t(g.mul(x, log_m));
  }
}

// Constant tables of a size-C transform with skew offset sd, in kernel consumption order
// (rs2_codec.hip: A slots PPW - PPW/d + g per wave, then B slots NW - C/d + g).
std::vector<uint16_t> sd_stream(int C, int sd, int ppw = kPpwTarget) {
  const Gf& g = gf();
  const int NW = C >= ppw ? C / ppw : 1, PPW = C / NW;
  std::vector<uint16_t> out;
  out.reserve(size_t(std::max(C - 1, 0)) * kTabU16);
  uint16_t t[kTabU16];
  for (int w = 0; w < NW; ++w)
    for (int d = 1; d < PPW; d *= 2)
      for (int gi = 0; gi < PPW / (2 * d); ++gi) {
        const int r = w * PPW + 2 * d * gi;
        nib_table(g.skew[r + d + sd - 1], true, t);
        out.insert(out.end(), t, t + kTabU16);
      }
  for (int d = PPW; d < C; d *= 2)
    for (int gi = 0; gi < C / (2 * d); ++gi) {
      const int r = 2 * d * gi;
      nib_table(g.skew[r + d + sd - 1], true, t);
      out.insert(out.end(), t, t + kTabU16);
    }
  return out;
}

// 1 when group 0 of every cross-wave layer of a size-C transform with skew offset sd multiplies
// by zero (skew[d + sd - 1] is log 0, which holds for sd = 0): the kernel then skips those
// multiplies (rs2_codec.hip phase_b).
int group0_zero(int C, int sd, int ppw = kPpwTarget) {
  const Gf& g = gf();
  const int NW = C >= ppw ? C / ppw : 1, PPW = C / NW;
  if (NW == 1) return 0;
  for (int d = PPW; d < C; d *= 2)
    if (g.skew[d + sd - 1] != kModulus) return 0;
  return 1;
}

uint32_t next_pow2(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// reed-solomon-simd DefaultRate: high rate iff pow2(recovery) <= pow2(original)
bool use_high_rate(uint32_t k, uint32_t r) { return next_pow2(r) <= next_pow2(k); }

bool rate_supported(uint32_t k, uint32_t r) {
  if (k == 0 || r == 0 || k >= kOrder || r >= kOrder) return false;
  return std::min(next_pow2(k), next_pow2(r)) + std::max(k, r) <= kOrder;
}

// ---------------------------------------------------------------------------------------------
// device context: per-device constant tables and a cache of transform table streams
// ---------------------------------------------------------------------------------------------
// Device memory arena, one per device: every DevBuf of plans, codecs, verifiers and contexts is
// a range of a few large hipMalloc'd segments (best fit over the free ranges, 256-byte
// granularity, neighbours coalesced on release), so plans created and destroyed for every new
// blob length -- the reference builds an encoder per call (config.rs:545-567) -- reuse device
// memory instead of calling hipMalloc / hipFree.  A segment is added only when no free range
// fits: max(request, reserved / 2, 256 MiB) rounded to 64 MiB, so the reserve grows
// geometrically and stops once it covers the workload's peak.  RS2_ARENA_RESERVE_MIB reserves
// a first segment up front (a hard budget: peak device memory = that reserve as long as the
// live buffers fit).  A range released by an owner that has quiesced its streams first (plan /
// codec / verifier destroy) is free at once; one released while work may still read it (a
// buffer outgrowing itself) waits in quarantine until a miss synchronizes the device.  Fully
// free segments beyond RS2_ARENA_CACHE_MIB of reserve (default 8192: the 256 MiB workload's
// double-buffered plans fit, a transient 4 GiB blob's do not stay) go back to hipFree, and
// rs2_device_memory_trim hands every wholly free segment back on request.
thread_local bool t_quiesced = false;  // the releasing owner has drained its streams

struct DevArena {
  static constexpr size_t kGrain = 256;
  struct Seg {
    uint8_t* base;
    size_t size;
    size_t used = 0;
    std::map<size_t, size_t> free_;  // offset -> length
  };
  std::mutex mu;
  std::vector<std::unique_ptr<Seg>> segs;
  std::set<std::tuple<size_t, size_t, size_t>> by_size;  // (length, segment, offset)
  std::vector<std::pair<void*, size_t>> quarantine_;
  size_t reserved = 0;
  uint64_t mallocs = 0, frees = 0, syncs = 0;
  int64_t live = 0, peak = 0;

  static size_t env_mib(const char* name, size_t dflt) {
    const char* e = std::getenv(name);
    return size_t(e ? std::max(0, std::atoi(e)) : int(dflt)) << 20;
  }
  static size_t cap() {
    static const size_t c = env_mib("RS2_ARENA_CACHE_MIB", 8192);
    return c;
  }
  size_t seg_of(const void* p) const {
    for (size_t k = 0; k < segs.size(); ++k)
      if (segs[k] && p >= segs[k]->base && p < segs[k]->base + segs[k]->size) return k;
    return SIZE_MAX;
  }
  void add_free(size_t k, size_t off, size_t len) {  // coalesces with both neighbours
    Seg& sg = *segs[k];
    auto nx = sg.free_.lower_bound(off);
    if (nx != sg.free_.end() && off + len == nx->first) {
      by_size.erase({nx->second, k, nx->first});
      len += nx->second;
      nx = sg.free_.erase(nx);
    }
    if (nx != sg.free_.begin()) {
      auto pv = std::prev(nx);
      if (pv->first + pv->second == off) {
        by_size.erase({pv->second, k, pv->first});
        off = pv->first;
        len += pv->second;
        sg.free_.erase(pv);
      }
    }
    sg.free_[off] = len;
    by_size.insert({len, k, off});
  }
  bool carve(size_t c, void** out) {
    auto it = by_size.lower_bound({c, 0, 0});
    if (it == by_size.end()) return false;
    const auto [len, k, off] = *it;
    by_size.erase(it);
    Seg& sg = *segs[k];
    sg.free_.erase(off);
    if (len > c) {
      sg.free_[off + c] = len - c;
      by_size.insert({len - c, k, off + c});
    }
    sg.used += c;
    *out = sg.base + off;
    return true;
  }
  hipError_t grow(size_t want) {
    uint8_t* p = nullptr;
    const hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want);
    if (e != hipSuccess) return e;
    ++mallocs;
    size_t k = 0;
    while (k < segs.size() && segs[k]) ++k;
    if (k == segs.size()) segs.emplace_back();
    segs[k].reset(new Seg{p, want});
    reserved += want;
    add_free(k, 0, want);
    return hipSuccess;
  }
  hipError_t get(size_t n, void** out, size_t* got) {
    const size_t c = (std::max<size_t>(n, 1) + kGrain - 1) / kGrain * kGrain;
    std::unique_lock<std::mutex> lk(mu);
    if (reserved == 0) {
      static const size_t first = env_mib("RS2_ARENA_RESERVE_MIB", 0);
      if (first) {
        const hipError_t e = grow((first + (size_t(64) << 20) - 1) >> 26 << 26);
        if (e != hipSuccess) return e;
      }
    }
    bool ok = carve(c, out);
    if (!ok && !quarantine_.empty()) {
      // only the ranges quarantined before the synchronize are safe to release after it: take
      // them now, so a range another thread quarantines meanwhile stays quarantined
      std::vector<std::pair<void*, size_t>> q;
      q.swap(quarantine_);
      lk.unlock();
      const hipError_t e = hipDeviceSynchronize();
      lk.lock();
      if (e != hipSuccess) {
        quarantine_.insert(quarantine_.end(), q.begin(), q.end());
        return e;
      }
      ++syncs;
      std::vector<std::pair<void*, size_t>> to_free;  // segments past the cap
      for (auto& b : q) release_locked(b.first, b.second, &to_free);
      if (!to_free.empty()) {  // their hipFree outside the lock
        lk.unlock();
        for (auto& f : to_free) (void)hipFree(f.first);
        lk.lock();
      }
      ok = carve(c, out);
    }
    if (!ok) {
      size_t want = std::max({c, reserved / 2, size_t(256) << 20});
      want = (want + (size_t(64) << 20) - 1) >> 26 << 26;
      hipError_t e = grow(want);
      if (e != hipSuccess && want > c) e = grow((c + (size_t(2) << 20) - 1) >> 21 << 21);
      if (e != hipSuccess) return e;
      ok = carve(c, out);
      if (!ok) return hipErrorOutOfMemory;
    }
    live += int64_t(c);
    peak = std::max(peak, live);
    *got = c;
    return hipSuccess;
  }
  // Return a range to its segment.  A segment that falls wholly free past the cap leaves the
  // arena here, but its hipFree (which synchronizes the device) is the caller's, after the lock
  // is released, so other threads' allocations do not wait behind it.
  void release_locked(void* p, size_t c, std::vector<std::pair<void*, size_t>>* to_free) {
    const size_t k = seg_of(p);
    if (k == SIZE_MAX) return;
    Seg& sg = *segs[k];
    add_free(k, size_t(static_cast<uint8_t*>(p) - sg.base), c);
    sg.used -= c;
    if (sg.used == 0 && reserved > cap()) {  // trim a wholly free segment past the cap
      by_size.erase({sg.size, k, 0});
      reserved -= sg.size;
      ++frees;
      to_free->push_back({sg.base, sg.size});
      segs[k].reset();
    }
  }
  void put(void* p, size_t c, bool quiesced) {
    std::vector<std::pair<void*, size_t>> to_free;
    {
      std::lock_guard<std::mutex> lk(mu);
      live -= int64_t(c);
      if (quiesced)
        release_locked(p, c, &to_free);
      else
        quarantine_.push_back({p, c});
    }
    for (auto& f : to_free) (void)hipFree(f.first);
  }
  // every wholly free segment back to hipFree (quarantined ranges first released after a device
  // synchronize); returns the bytes handed back
  hipError_t trim(uint64_t* released) {
    std::unique_lock<std::mutex> lk(mu);
    std::vector<std::pair<void*, size_t>> to_free;
    if (!quarantine_.empty()) {
      std::vector<std::pair<void*, size_t>> q;  // snapshot before the synchronize (see get)
      q.swap(quarantine_);
      lk.unlock();
      const hipError_t e = hipDeviceSynchronize();
      lk.lock();
      if (e != hipSuccess) {
        quarantine_.insert(quarantine_.end(), q.begin(), q.end());
        return e;
      }
      ++syncs;
      for (auto& b : q) release_locked(b.first, b.second, &to_free);
    }
    uint64_t got = 0;
    for (auto& f : to_free) got += f.second;  // past the cap while leaving quarantine
    for (size_t k = 0; k < segs.size(); ++k) {
      if (!segs[k] || segs[k]->used) continue;
      Seg& sg = *segs[k];
      by_size.erase({sg.size, k, 0});
      reserved -= sg.size;
      got += sg.size;
      ++frees;
      to_free.push_back({sg.base, sg.size});
      segs[k].reset();
    }
    lk.unlock();
    for (auto& f : to_free) (void)hipFree(f.first);
    if (released) *released = got;
    return hipSuccess;
  }
};

DevArena& dev_arena(int device) {
  // never destroyed: buffers of objects torn down at process exit (the contexts) still return here
  static DevArena* arenas = new DevArena[64];
  return arenas[std::min(std::max(device, 0), 63)];
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;  // usable bytes (the arena range is bytes + 256, a multiple of 256)
  size_t cls = 0;
  int dev = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) dev_arena(dev).put(p, cls, t_quiesced);
    p = nullptr;
    bytes = 0;
    cls = 0;
  }
  hipError_t ensure(size_t n) {
    if (bytes >= n && p) return hipSuccess;
    release();
    // 256 bytes of slack: kernels may read whole dwords past a symbol's last byte
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    size_t got = 0;
    e = dev_arena(dev).get(n + 256, &p, &got);
    if (e == hipSuccess) {
      bytes = got - 256;
      cls = got;
    } else {
      p = nullptr;
    }
    return e;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

std::atomic<uint64_t> g_pinned_allocs{0};

struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t n) {
    if (bytes >= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
    if (e == hipSuccess) {
      bytes = n;
      g_pinned_allocs.fetch_add(1, std::memory_order_relaxed);
    }
    return e;
  }
};

// Host worker threads for the pinned staging of the host-buffer ABI: copies between the
// caller's pageable buffers and pinned slots run on several cores while the DMA engine moves
// the previous slot (one core's memcpy would cap the path at ~10 GB/s).  Shared by every plan
// of a device; run() is re-entrant (each call waits only for its own tasks).
class HostPool {
 public:
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() {
    start();
    return int(th_.size()) + 1;
  }
  // Run every task (the calling thread takes a share) and return when all have finished.
  void run(std::vector<std::function<void()>>& tasks) {
    start();
    if (tasks.empty()) return;
    struct Latch {
      std::mutex m;
      std::condition_variable cv;
      size_t left;
    };
    auto latch = std::make_shared<Latch>();
    latch->left = tasks.size();
    auto finish = [latch]() {
      std::lock_guard<std::mutex> lk(latch->m);
      if (--latch->left == 0) latch->cv.notify_all();
    };
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (size_t i = 1; i < tasks.size(); ++i) {
        std::function<void()> t = std::move(tasks[i]);
        q_.emplace_back([t, finish]() {
          t();
          finish();
        });
      }
    }
    cv_.notify_all();
    tasks[0]();
    finish();
    std::unique_lock<std::mutex> lk(latch->m);
    latch->cv.wait(lk, [&] { return latch->left == 0; });
  }

 private:
  void start() {
    std::call_once(once_, [this] {
      int n = int(std::thread::hardware_concurrency());
      const char* e = std::getenv("RS2_HOST_THREADS");
      int want = e ? std::atoi(e) : 16;
      want = std::max(1, std::min(want, std::max(n, 1)));
      for (int i = 0; i + 1 < want; ++i) th_.emplace_back([this] { loop(); });
    });
  }
  void loop() {
    for (;;) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        t = std::move(q_.front());
        q_.pop_front();
      }
      t();
    }
  }
  std::once_flag once_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
};

// One piece of a host <-> device transfer: `len` bytes between host `h` and device `d`.
struct Seg {
  uint8_t* h;
  uint8_t* d;
  size_t len;
};

// memcpy of many segments split evenly over the pool's threads (dst/src per direction)
void par_copy(HostPool& pool, const std::vector<Seg>& segs, bool to_host) {
  size_t total = 0;
  for (const auto& g : segs) total += g.len;
  if (total == 0) return;
  const int T = int(std::min<size_t>(size_t(pool.threads()), (total + (1 << 20) - 1) >> 20));
  const size_t per = (total + T - 1) / T;
  std::vector<std::vector<Seg>> parts(T);
  size_t acc = 0;
  for (const auto& g : segs) {
    size_t off = 0;
    while (off < g.len) {
      const int t = int(std::min<size_t>(acc / per, size_t(T - 1)));
      const size_t room = (size_t(t) + 1) * per - acc;
      const size_t take = std::min(g.len - off, t == T - 1 ? g.len - off : room);
      parts[t].push_back({g.h + off, g.d + off, take});
      off += take;
      acc += take;
    }
  }
  std::vector<std::function<void()>> tasks;
  for (auto& part : parts) {
    if (part.empty()) continue;
    tasks.emplace_back([&part, to_host] {
      for (const auto& g : part) {
        if (to_host)
          std::memcpy(g.h, g.d, g.len);
        else
          std::memcpy(g.d, g.h, g.len);
      }
    });
  }
  pool.run(tasks);
}

// Pinned slots for the small per-call uploads (a decode's position offsets, mixing tables and
// multiplier logs, copy lists, verifier targets).  A hipMemcpyAsync host -> device on a stream
// that has kernels queued can block the issuing thread until they have run (the copy engine's
// dependency on the compute queue): the bench's timed decodes 4 and 6 stalled 6-7 ms each that
// way in every run, whatever its length, from pageable sources (gpurun_out/r05a traces: the
// 0.6 ms per step the 20-step driver run showed as dec_plan_host) and 15-28 ms from pinned ones
// (gpurun_out/r05c).  So the data goes into a pinned, device-mapped slot and a copy kernel
// (rs2_hash.hip host_upload_kernel) moves it in stream order like any other launch.  kSlots
// slots of kSlotBytes, pinned once per device at first use and never grown; uploads take them
// round-robin.
//
// Reuse of a slot.  Every use of slot k carries a generation number; the kernel that last reads
// the slot stores that generation into word k of a coherent, device-mapped host array when it
// has finished (rs2_hash.hip host_upload_kernel / upload_signal_kernel),
// and the host rewrites the slot only once it reads that generation there.  No HIP event is
// involved, so the wait depends on nothing but the copy having run -- not on the stream it ran
// on still existing (plans, verifiers and caller streams come and go between uploads; an event
// recorded on a destroyed stream is refused by the runtime) -- and it never waits for more than
// that one copy (no device-wide synchronize).  With 64 slots the wait is reached only with 64
// uploads still queued (rs2_upload_stats counts the waits).  Both rings are allocated coherent
// (fine-grained), so the copy kernel's reads of a rewritten slot never depend on GPU cache state.
// Larger uploads (n_shards in the thousands) keep the runtime's path.
std::atomic<uint64_t> g_upload_calls{0}, g_upload_waits{0}, g_upload_jobs{0};

class UploadSlots {
 public:
  static constexpr int kSlots = 64;
  static constexpr size_t kSlotBytes = size_t(512) << 10;
  // (lives as long as its Context, i.e. to process exit: the pinned blocks are left to the process
  // teardown rather than freed while the runtime may already be going down)
  hipError_t upload(void* dst, const void* src, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (n > kSlotBytes) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
    std::lock_guard<std::mutex> lk(mu_);
    hipError_t e = init_locked();
    if (e != hipSuccess) return e;
    if (!base_) {
      e = pin(&base_, &dev_base_, kSlots * kSlotBytes);
      if (e != hipSuccess) return e;
    }
    const int k = next_;
    next_ = (next_ + 1) % kSlots;
    if ((e = wait_locked(k)) != hipSuccess) return e;
    uint8_t* slot = base_ + size_t(k) * kSlotBytes;
    std::memcpy(slot, src, n);
    const uint64_t g = ++gen_counter_;
    // a copy kernel reading the mapped slot, not hipMemcpyAsync (rs2_hash.hip host_upload_kernel);
    // its one workgroup reports generation g in word k once every load of the slot has returned
    e = rs2k_launch_host_upload(dev_base_ + size_t(k) * kSlotBytes, dst, int64_t(n),
                                done_dev_ + k, g, st);
    if (e != hipSuccess) return e;  // not launched: the slot stays free (want_ unchanged)
    want_[k] = g;
    g_upload_calls.fetch_add(1, std::memory_order_relaxed);
    return hipSuccess;
  }

  // A CodecJobBig for one launch: staged into a pinned slot, copied by the copy kernel into a
  // device slot of its own, `launch(device pointer)` enqueues the consumer on st, and a signal
  // kernel queued behind the consumer reports the slot pair free.  (Jobs of more than kMaxBlocks
  // blocks: n_shards above about 24,580.)
  template <class F>
  hipError_t launch_with_job(const void* src, size_t n, hipStream_t st, F launch) {
    if (n > kSlotBytes) return hipErrorInvalidValue;
    std::lock_guard<std::mutex> lk(mu_);
    hipError_t e = init_locked();
    if (e != hipSuccess) return e;
    if (!jbase_) {
      if ((e = pin(&jbase_, &jdev_host_, kJobSlots * kSlotBytes)) != hipSuccess) return e;
      if ((e = jdev_.ensure(kJobSlots * kSlotBytes)) != hipSuccess) return e;
    }
    const int k = jnext_;
    jnext_ = (jnext_ + 1) % kJobSlots;
    const int w = kSlots + k;  // completion word of job slot k
    if ((e = wait_locked(w)) != hipSuccess) return e;
    std::memcpy(jbase_ + size_t(k) * kSlotBytes, src, n);
    uint8_t* d = jdev_.as<uint8_t>() + size_t(k) * kSlotBytes;
    const uint64_t g = ++gen_counter_;
    e = rs2k_launch_host_upload(jdev_host_ + size_t(k) * kSlotBytes, d, int64_t(n), nullptr, 0,
                                st);
    if (e != hipSuccess) return e;
    const hipError_t le = launch(d);
    // reported whether or not the consumer launched: the copy above did, and reads the slot
    e = rs2k_launch_upload_signal(done_dev_ + w, g, st);
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(st);  // no report coming: the copy (and consumer) have run
      return le != hipSuccess ? le : e;
    }
    want_[w] = g;
    g_upload_jobs.fetch_add(1, std::memory_order_relaxed);
    return le;
  }

 private:
  static constexpr int kJobSlots = 16;
  static constexpr int kWords = kSlots + kJobSlots;
  static hipError_t pin(uint8_t** host, uint8_t** dev, size_t bytes) {
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    g_pinned_allocs.fetch_add(1, std::memory_order_relaxed);
    void* dp = nullptr;
    if ((e = hipHostGetDevicePointer(&dp, p, 0)) != hipSuccess) return e;
    *host = static_cast<uint8_t*>(p);
    *dev = static_cast<uint8_t*>(dp);
    return hipSuccess;
  }
  // the completion words (coherent host memory, device-mapped)
  hipError_t init_locked() {
    if (done_host_) return hipSuccess;
    uint8_t *h = nullptr, *d = nullptr;
    hipError_t e = pin(&h, &d, kWords * sizeof(uint64_t));
    if (e != hipSuccess) return e;
    std::memset(h, 0, kWords * sizeof(uint64_t));
    done_host_ = reinterpret_cast<uint64_t*>(h);
    done_dev_ = reinterpret_cast<uint64_t*>(d);
    return hipSuccess;
  }
  // Wait (spinning, then yielding) until word w reports the generation its slot was last used
  // with.  A copy that never runs (a faulted device) ends the wait with an error after 120 s.
  hipError_t wait_locked(int w) {
    const uint64_t want = want_[w];
    if (want == 0 || __atomic_load_n(done_host_ + w, __ATOMIC_ACQUIRE) >= want) return hipSuccess;
    g_upload_waits.fetch_add(1, std::memory_order_relaxed);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0; __atomic_load_n(done_host_ + w, __ATOMIC_ACQUIRE) < want; ++spin) {
      if (spin < 4096) continue;
      std::this_thread::yield();
      if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        return hipErrorLaunchTimeOut;
    }
    return hipSuccess;
  }
  std::mutex mu_;
  uint64_t* done_host_ = nullptr;  // [kWords] completion words as the host reads them
  uint64_t* done_dev_ = nullptr;   // the same words as the device addresses them
  uint64_t gen_counter_ = 0;
  uint64_t want_[kWords] = {};     // generation of each slot's last use (0 = never used)
  uint8_t* base_ = nullptr;
  uint8_t* dev_base_ = nullptr;    // the same slots as the device addresses them
  int next_ = 0;
  uint8_t* jbase_ = nullptr;
  uint8_t* jdev_host_ = nullptr;
  DevBuf jdev_;
  int jnext_ = 0;
};

struct Dec1D;  // rs2_decode_1d's pooled state (below)

struct Context {
  int device = 0;
  HostPool pool;
  DevBuf exp_t, log_t;
  std::mutex mu;
  std::map<std::tuple<int, int, int>, std::unique_ptr<DevBuf>> streams;
  hipStream_t util_stream = nullptr;
  UploadSlots uploads;
  hipError_t upload(void* dst, const void* src, size_t n, hipStream_t st) {
    return uploads.upload(dst, src, n, st);
  }
  // Pooled helpers of the host-buffer single-sliver entry points (SliverData::verify /
  // get_merkle_root, recovery symbols, the 1D decode of a sliver recovery): a storage node calls
  // them one sliver at a time, so a verifier (stream, encode plan, device buffers, pinned
  // staging) or a 1D decoder is checked out of a pool per parameter set instead of being built
  // and torn down per call (a fresh stream and plan cost more than the work at n = 1000).
  std::mutex pool_mu;
  std::map<std::tuple<int, int, int>, std::vector<::rs2_verifier*>> verifier_pool;
  std::map<std::tuple<int, int, int>, std::vector<Dec1D*>> dec1d_pool;
  static constexpr size_t kPoolKeep = 8;  // idle objects kept per parameter set

  int init(int dev) {
    device = dev;
    HIP_TRY(hipSetDevice(dev));
    const Gf& g = gf();
    HIP_TRY(exp_t.ensure(kOrder * 2));
    HIP_TRY(log_t.ensure(kOrder * 2));
    HIP_TRY(hipMemcpy(exp_t.p, g.exp.data(), kOrder * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(log_t.p, g.log.data(), kOrder * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipStreamCreateWithFlags(&util_stream, hipStreamNonBlocking));
    return RS2_OK;
  }

  // device table stream for a size-C transform with skew offset sd, laid out for `ppw`
  // positions per wave (built once, cached)
  const uint16_t* stream(int C, int sd, int ppw) {
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(C, sd, ppw);
    auto it = streams.find(key);
    if (it != streams.end()) return it->second->as<uint16_t>();
    std::vector<uint16_t> host = sd_stream(C, sd, ppw);
    auto buf = std::make_unique<DevBuf>();
    if (buf->ensure(std::max<size_t>(host.size() * 2, 16)) != hipSuccess) return nullptr;
    if (!host.empty() &&
        hipMemcpy(buf->p, host.data(), host.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
      return nullptr;
    const uint16_t* p = buf->as<uint16_t>();
    streams.emplace(key, std::move(buf));
    return p;
  }
};

std::mutex g_ctx_mu;
std::map<int, std::unique_ptr<Context>> g_ctx;
thread_local int g_device = 0;

int get_context(Context** out) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto it = g_ctx.find(g_device);
  if (it != g_ctx.end()) {
    *out = it->second.get();
    return hipSetDevice(g_device) == hipSuccess ? RS2_OK : fail(RS2_E_DEVICE, "hipSetDevice");
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= g_device)
    return fail(RS2_E_DEVICE, "no HIP device available");
  auto ctx = std::make_unique<Context>();
  const int rc = ctx->init(g_device);
  if (rc != RS2_OK) return rc;
  *out = ctx.get();
  g_ctx.emplace(g_device, std::move(ctx));
  return RS2_OK;
}

// Diagnostic phase stamps (a library built with -DRS2_STAMPS=1 and $RS2_STAMP_FILE set): every
// codec launch runs synchronously and appends {mode, C, tiles, n_z, kStamps, waves} + the stamps
// of every wave of every workgroup to the file (tools/stamps_summary.py reads it).
hipError_t stamp_dump(int C, int mode, int tiles, int n_z, uint64_t* d, hipStream_t st) {
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  hipError_t e = hipStreamSynchronize(st);
  if (e != hipSuccess) return e;
  const int nw = std::max(1, C / kPpwTarget);
  std::vector<uint64_t> h(size_t(tiles) * n_z * nw * kStamps);
  e = hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return e;
  if (FILE* f = std::fopen(std::getenv("RS2_STAMP_FILE"), "ab")) {
    const int32_t hdr[6] = {mode, C, tiles, n_z, kStamps, nw};
    std::fwrite(hdr, sizeof hdr, 1, f);
    std::fwrite(h.data(), 8, h.size(), f);
    std::fclose(f);
  }
  return hipSuccess;
}

// n_blobs > 1: the same job over a batch of blobs whose symbols lie in_bs / out_bs / cp_bs
// bytes apart (CodecJob::tiles_per_blob); the grid holds every blob's tiles.
// tile_ctr: kTileCtrWords zeroed words owned by this launch site (CodecJob::tile_ctr), used when
// the job runs as a pipelined kernel and RS2_PIPE_DYN=1; null = static tile ranges.
// The job as the kernels' by-value argument: every scalar field at once (CodecScalars), the
// block arrays and mixing kinds cut to kMaxBlocks (the caller checked that n_in, n_out <=
// kMaxBlocks); rs2_device.h static_asserts that the arrays listed here are all there is.
void narrow_job(const CodecJobBig& b, CodecJob& s) {
  static_cast<CodecScalars&>(s) = static_cast<const CodecScalars&>(b);
  std::copy(b.in, b.in + kMaxBlocks, s.in);
  std::copy(b.out, b.out + kMaxBlocks, s.out);
  for (int o = 0; o < kMaxBlocks; ++o) {
    std::memcpy(s.m1_kind[o], b.m1_kind[o], kMaxBlocks);
    std::memcpy(s.m2_kind[o], b.m2_kind[o], kMaxBlocks);
  }
  std::copy(b.pair_p, b.pair_p + kMaxBlocks, s.pair_p);
  std::copy(b.pair_q, b.pair_q + kMaxBlocks, s.pair_q);
  std::copy(b.pair_nw, b.pair_nw + kMaxBlocks, s.pair_nw);
}

hipError_t launch_codec_big(const CodecJobBig& job_in, int n_lines, int n_z, int mode,
                            hipStream_t st, int n_blobs, int64_t in_bs, int64_t out_bs,
                            int64_t cp_bs);

hipError_t launch_codec_c(int C, const CodecJobBig& job_big, int n_lines, int n_z, int mode,
                          hipStream_t st, int n_blobs = 1, int64_t in_bs = 0, int64_t out_bs = 0,
                          int64_t cp_bs = 0, uint32_t* tile_ctr = nullptr) {
  if (job_big.n_pairs <= 0 || n_lines <= 0 || job_big.pairs_span < job_big.n_pairs) return hipSuccess;
  if (n_blobs < 1) return hipErrorInvalidValue;
  if (job_big.n_in > kMaxBlocks || job_big.n_out > kMaxBlocks) {
    // more blocks than the kernel argument holds (n_shards above about 24,580)
    if (C != kMaxC) return hipErrorInvalidValue;
    return launch_codec_big(job_big, n_lines, n_z, mode, st, n_blobs, in_bs, out_bs, cp_bs);
  }
  CodecJob job;
  narrow_job(job_big, job);
  job.n_lines = n_lines;
  const int64_t per_blob = (int64_t(n_lines) * job.pairs_span + 63) / 64;
  const int64_t tiles64 = per_blob * n_blobs;
  if (tiles64 > 0x7FFFFFFF) return hipErrorInvalidValue;
  const int tiles = int(tiles64);
  job.tiles_per_blob = n_blobs > 1 ? int(per_blob) : 0;
  job.in_blob_stride = in_bs;
  job.out_blob_stride = out_bs;
  job.copy_blob_stride = cp_bs;
  n_lines = 1;  // lines are folded into grid.x
  job.stamps = nullptr;
  // Shared-input jobs whose last output block's active waves fit below the input's run as the
  // persistent tile-pipelined kernel (rs2_codec.hip cols_pipe_body): one workgroup per CU, each
  // walking a contiguous tile range.  RS2_PIPE=0: never (A/B knob).
  int grid_tiles = tiles;
  if (((mode == kModeCols && job.shared_in && job.n_out <= 3) ||
       (mode == kModeRows && !job.shared_in && job.n_out == 1)) &&
      n_z == 1 && job.n_out >= 1 && C >= 2 * kPpwTarget) {
    static const int pipe_wgs = [] {
      const char* e = std::getenv("RS2_PIPE");
      if (e && std::atoi(e) == 0) return 0;
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
      const int k = e ? std::max(1, std::atoi(e)) : 1;  // RS2_PIPE=k: k workgroups per CU
      const char* nw_env = std::getenv("RS2_PIPE_WGS");   // A/B: an absolute workgroup count
      if (nw_env && std::atoi(nw_env) > 0) return std::atoi(nw_env);
      return cus * k;
    }();
    const int nw = C / kPpwTarget;
    auto waves = [](int count) { return (count + kPpwTarget - 1) / kPpwTarget; };
    const int tail_waves = waves(job.out[job.n_out - 1].trunc);
    // the head input block: the shared input, or the mixing job's shortest block (every block
    // of a pipelined mixing job must carry a nonzero coefficient)
    int head = 0;
    bool ok = pipe_wgs > 0;
    if (mode == kModeRows)
      for (int b = 0; b < job.n_in && ok; ++b) {
        ok = job.m2_kind[0][b] != 0 && job.m1_kind[0][b] == 0;
        if (job.in[b].count < job.in[head].count) head = b;
      }
    if (ok && waves(job.in[head].count) + tail_waves <= nw) {
      mode = mode == kModeCols ? kModeColsPipe : kModeRowsPipe;
      job.n_tiles = tiles;
      job.pipe_head = head;
      grid_tiles = std::min(tiles, pipe_wgs);
      // RS2_PIPE_DYN=1: dynamic tile order (A/B knob; static ranges measured 82.5 vs 81.4 GiB/s,
      // and with a high-priority decode stream 63.0 vs 63.2: profiles/r03/exp/dyn/)
      static const bool dyn = [] {
        const char* e = std::getenv("RS2_PIPE_DYN");
        return e && std::atoi(e) != 0;
      }();
      job.tile_ctr = dyn ? tile_ctr : nullptr;
    }
  }
  // The decode as one persistent workgroup per CU (kModeDecodePersist) when RS2_DEC_PERSIST=k
  // (k workgroups per CU) is set: A/B knob
  if (mode == kModeDecode && n_z == 1) {
    static const int dec_wgs = [] {
      const char* e = std::getenv("RS2_DEC_PERSIST");
      if (!e || std::atoi(e) <= 0) return 0;
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
      return cus * std::atoi(e);
    }();
    if (dec_wgs > 0 && tiles > dec_wgs) {
      mode = kModeDecodePersist;
      job.n_tiles = tiles;
      grid_tiles = dec_wgs;
    }
  }
  static const bool stamping = std::getenv("RS2_STAMP_FILE") != nullptr;
  if (stamping) {
    const size_t n_st = size_t(tiles) * n_z * std::max(1, C / kPpwTarget) * kStamps;
    hipError_t e = hipMalloc(&job.stamps, n_st * 8);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(job.stamps, 0, n_st * 8, st);
    if (e != hipSuccess) return e;
  }
  hipError_t le = hipSuccess;
  switch (C) {
    case 1: le = rs2k_launch_codec_1(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 2: le = rs2k_launch_codec_2(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 4: le = rs2k_launch_codec_4(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 8: le = rs2k_launch_codec_8(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 16: le = rs2k_launch_codec_16(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 32: le = rs2k_launch_codec_32(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 64: le = rs2k_launch_codec_64(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 128: le = rs2k_launch_codec_128(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 256: le = rs2k_launch_codec_256(&job, grid_tiles, n_lines, n_z, mode, st); break;
    case 512: le = rs2k_launch_codec_512(&job, grid_tiles, n_lines, n_z, mode, st); break;
    default: le = hipErrorInvalidValue;
  }
  if (le != hipSuccess || !stamping) return le;
  return stamp_dump(C, mode, grid_tiles, n_z, job.stamps, st);
}

int get_context(Context** out);

// A job of more than kMaxBlocks blocks (C = 512): one-tile kernels reading the job from device
// memory (no pipelined / persistent variants, no stamps).
hipError_t launch_codec_big(const CodecJobBig& job_in, int n_lines, int n_z, int mode,
                            hipStream_t st, int n_blobs, int64_t in_bs, int64_t out_bs,
                            int64_t cp_bs) {
  if (mode != kModeRows && mode != kModeCols && mode != kModeDecode) return hipErrorInvalidValue;
  auto job = std::make_unique<CodecJobBig>(job_in);
  job->n_lines = n_lines;
  const int64_t per_blob = (int64_t(n_lines) * job->pairs_span + 63) / 64;
  const int64_t tiles64 = per_blob * n_blobs;
  if (tiles64 > 0x7FFFFFFF) return hipErrorInvalidValue;
  job->tiles_per_blob = n_blobs > 1 ? int(per_blob) : 0;
  job->in_blob_stride = in_bs;
  job->out_blob_stride = out_bs;
  job->copy_blob_stride = cp_bs;
  job->stamps = nullptr;
  job->tile_ctr = nullptr;
  Context* ctx = nullptr;
  if (get_context(&ctx) != RS2_OK) return hipErrorInvalidDevice;
  const int tiles = int(tiles64);
  return ctx->uploads.launch_with_job(job.get(), sizeof(CodecJobBig), st, [&](uint8_t* d) {
    return rs2k_launch_codec_big_512(reinterpret_cast<const CodecJobBig*>(d), tiles, 1, n_z, mode,
                                     st);
  });
}

// ---------------------------------------------------------------------------------------------
// codec job planning
// ---------------------------------------------------------------------------------------------
// A planned job: the CodecJob plus host copies of its per-position offset arrays.  Pointer
// fields that reference per-job device arrays are filled by bind() once those are uploaded.
struct PlannedJob {
  CodecJobBig job{};                 // narrowed to CodecJob at launch when it has <= 64 blocks
  int mix_stride = kMaxBlocks;       // mixing-table row length (kMaxBlocksBig for big jobs)
  int C = 1;
  int n_z = 1;
  int mode = kModeRows;              // kernel variant (rs2_device.h CodecMode)
  int ppw = kPpwTarget;              // positions per wave of the variant's table stream
  std::vector<int64_t> offs;         // (n_in + n_out) blocks x C
  std::vector<int64_t> copy_offs;    // n_in blocks x C fused copy-out offsets, or empty
  uint8_t* copy_base = nullptr;
  int64_t copy_ls = 0, copy_limit = INT64_MAX;
  std::vector<uint16_t> pre_logs;    // per in-block C logs (decode), empty if none
  std::vector<uint16_t> post_logs;   // per out-block C logs (decode)
  std::vector<uint16_t> mix;         // mix_stride^2 * 2 tables (block mixing tables)
  std::vector<uint16_t> logs;        // pre ++ post logs as uploaded (kept alive for async H2D)
  std::vector<int> in_sd, out_sd;    // skew offset of each block's in-block transform
  std::vector<uint32_t> in_first;    // code position (source index) of each in-block's slot 0
  bool has_pre = false, has_post = false, has_mix = false;

  size_t in_off(int b) const { return size_t(b) * C; }
  size_t out_off(int o) const { return size_t(job.n_in + o) * C; }
  // lines are folded into grid.x with the element pairs (CodecJob::pairs_span)
  hipError_t launch(int n_lines, hipStream_t st, uint32_t* tile_ctr = nullptr) const {
    return launch_codec_c(C, job, n_lines, n_z, mode, st, 1, 0, 0, 0, tile_ctr);
  }
};

// Device memory holding a planned job's arrays.
struct JobMem {
  DevBuf offs, pre_tab, post_tab, mix, logs;
};

// rs2_decode_1d's state per (k, n_shards, symbol size), pooled in the Context (a sliver
// recovery decodes one codeword of K symbols per call): its stream, device buffers, pinned
// staging and the planned decode job's device arrays.
struct Dec1D {
  hipStream_t st = nullptr;
  DevBuf din, dout;
  PinnedBuf hin, hout;
  PlannedJob pj;
  JobMem mem;
};

// checkout / return of a pooled Dec1D (returned with its stream drained: rs2_decode_1d
// synchronizes before it returns)
struct Dec1DLease {
  Context* ctx = nullptr;
  std::tuple<int, int, int> key;
  Dec1D* d = nullptr;
  Dec1DLease(Context* c, int k, int n, int s) : ctx(c), key(k, n, s) {}
  Dec1DLease(const Dec1DLease&) = delete;
  Dec1DLease& operator=(const Dec1DLease&) = delete;
  hipError_t get() {
    {
      std::lock_guard<std::mutex> lk(ctx->pool_mu);
      auto& free_ = ctx->dec1d_pool[key];
      if (!free_.empty()) {
        d = free_.back();
        free_.pop_back();
        return hipSuccess;
      }
    }
    auto nd = std::make_unique<Dec1D>();
    hipError_t e = hipStreamCreateWithFlags(&nd->st, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    d = nd.release();
    return hipSuccess;
  }
  ~Dec1DLease() {
    if (!d) return;
    // drained before it goes back: an error return may leave its H2D copy of hin (or the
    // decode) queued, and the next holder rewrites hin / grows it (PinnedBuf::ensure frees it)
    (void)hipStreamSynchronize(d->st);
    {
      std::lock_guard<std::mutex> lk(ctx->pool_mu);
      auto& free_ = ctx->dec1d_pool[key];
      if (free_.size() < Context::kPoolKeep) {
        free_.push_back(d);
        return;
      }
    }
    (void)hipStreamSynchronize(d->st);
    (void)hipStreamDestroy(d->st);
    const bool prev = t_quiesced;
    t_quiesced = true;  // drained above: its ranges may be reused at once
    delete d;
    t_quiesced = prev;
  }
};

int plan_fail_unsupported(const std::string& what) { return fail(RS2_E_UNSUPPORTED, what); }

// Largest transform block held on chip.  RS2_BLOCK_MAX (a power of two <= kMaxC) lowers it for
// experiments: smaller blocks mean smaller workgroups (C/32 waves) and more of them per CU, at
// the price of more block-level mixing.
std::atomic<uint32_t> g_block_max{0};
uint32_t block_max() {
  uint32_t v = g_block_max.load(std::memory_order_relaxed);
  if (v) return v;
  const char* e = std::getenv("RS2_BLOCK_MAX");
  uint32_t x = e ? uint32_t(std::atoi(e)) : uint32_t(kMaxC);
  if (x < 1 || x > uint32_t(kMaxC) || (x & (x - 1))) x = uint32_t(kMaxC);
  g_block_max.store(x, std::memory_order_relaxed);
  return x;
}

// Blocks a job of block size C may have: jobs beyond kMaxBlocks run from device memory
// (CodecJobBig), for which only C = 512 kernels are built.
int max_blocks(int C) { return C == kMaxC ? kMaxBlocksBig : kMaxBlocks; }

// Symbolic block-level transform layers.  A "slot" is one block of C positions; its value is a
// linear combination (GF(2^16) coefficients) of the jobs' input blocks after their in-block
// IFFTs.  Layers whose butterfly distance is >= C have one constant per block pair, so on whole
// blocks they are scalar operations (same constants as the element-level transforms).
using Coef = std::vector<uint32_t>;

void coef_xor(Coef& y, const Coef& x) {
  for (size_t i = 0; i < y.size(); ++i) y[i] ^= x[i];
}
void coef_mul_xor(Coef& y, const Coef& x, uint32_t log_c) {
  const Gf& g = gf();
  for (size_t i = 0; i < y.size(); ++i) y[i] ^= g.mul(x[i], log_c);
}
// IFFT layers d = C .. span/2 of a size-`span` transform with skew offset sd
void sym_ifft_top(std::vector<Coef>& V, uint32_t C, uint32_t span, uint32_t sd) {
  const Gf& g = gf();
  for (uint32_t d = C; d < span; d *= 2)
    for (uint32_t r = 0; r < span; r += 2 * d) {
      const uint32_t c = g.skew[r + d + sd - 1];
      for (uint32_t j = 0; j < d / C; ++j) {
        const uint32_t x = r / C + j, y = x + d / C;
        coef_xor(V[y], V[x]);
        if (c != kModulus) coef_mul_xor(V[x], V[y], c);
      }
    }
}
// FFT layers d = span/2 .. C of a size-`span` transform with skew offset sd
void sym_fft_top(std::vector<Coef>& V, uint32_t C, uint32_t span, uint32_t sd) {
  const Gf& g = gf();
  for (uint32_t d = span / 2; d >= C && d > 0; d /= 2) {
    for (uint32_t r = 0; r < span; r += 2 * d) {
      const uint32_t c = g.skew[r + d + sd - 1];
      for (uint32_t j = 0; j < d / C; ++j) {
        const uint32_t x = r / C + j, y = x + d / C;
        if (c != kModulus) coef_mul_xor(V[x], V[y], c);
        coef_xor(V[y], V[x]);
      }
    }
    if (d == C) break;
  }
}

// Mixing kinds and tables of output block oi from its coefficient vectors (M1 may be empty).
void set_mixing(PlannedJob& pj, int oi, const Coef* m1, const Coef& m2) {
  const Gf& g = gf();
  CodecJobBig& j = pj.job;
  const size_t ms = size_t(pj.mix_stride);
  if (pj.mix.empty()) pj.mix.assign(ms * ms * 2 * kTabU16, 0);
  for (int bi = 0; bi < j.n_in; ++bi) {
    const uint32_t c1 = m1 ? (*m1)[bi] : 0u, c2 = m2[bi];
    j.m1_kind[oi][bi] = uint8_t(c1 == 0 ? 0 : (c1 == 1 ? 1 : 2));
    j.m2_kind[oi][bi] = uint8_t(c2 == 0 ? 0 : (c2 == 1 ? 1 : 2));
    uint16_t* t = pj.mix.data() + (size_t(oi) * ms + bi) * 2 * kTabU16;
    if (c1 > 1) {
      nib_table(g.log[c1], false, t);
      pj.has_mix = true;
    }
    if (c2 > 1) {
      nib_table(g.log[c2], false, t + kTabU16);
      pj.has_mix = true;
    }
  }
}

// Encode K source symbols into R recovery symbols for every line (reed-solomon-simd encoders,
// oracle rs_encode_elems).  src(i) / dst(j): byte offsets relative to the base (before the line
// stride).  Transforms larger than the block size C are split into blocks of C with the
// top layers applied as block mixing.
template <class SrcF, class DstF>
int plan_encode(uint32_t K, uint32_t R, int symbol_size, const uint8_t* src_base,
                int64_t src_ls, SrcF src, uint8_t* dst_base, int64_t dst_ls, DstF dst,
                int64_t dst_limit, PlannedJob& pj) {
  if (!rate_supported(K, R)) return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "unsupported shard count");
  CodecJobBig& j = pj.job;
  j = CodecJobBig{};
  pj.mix.clear();
  pj.has_mix = false;
  pj.in_sd.clear();
  pj.out_sd.clear();
  pj.in_first.clear();
  j.symbol_size = symbol_size;
  j.n_pairs = (symbol_size + 3) / 4;
  const bool high = use_high_rate(K, R);
  const uint32_t cs = high ? next_pow2(R) : next_pow2(K);
  const uint32_t C = std::min(cs, block_max());
  const uint32_t nb = cs / C;
  pj.C = int(C);
  // input blocks
  struct Blk { uint32_t first, count; int sd; };
  std::vector<Blk> in, out;
  if (high) {
    for (uint32_t k = 0; k * cs < K; ++k)
      for (uint32_t b = 0; b < nb && k * cs + b * C < K; ++b)
        in.push_back({k * cs + b * C, std::min(C, K - k * cs - b * C), int((k + 1) * cs + b * C)});
  } else {
    for (uint32_t b = 0; b < nb && b * C < K; ++b)
      in.push_back({b * C, std::min(C, K - b * C), int(b * C)});
  }
  if (in.size() > size_t(max_blocks(C))) return plan_fail_unsupported("too many input blocks");
  j.n_in = int(in.size());
  // block mixing: coefficient vectors of each output block's pre-FFT slot
  std::vector<Coef> outs;
  const size_t ni = in.size();
  if (high) {
    std::vector<Coef> acc(nb, Coef(ni, 0));
    size_t bi = 0;
    for (uint32_t k = 0; k * cs < K; ++k) {
      std::vector<Coef> V(nb, Coef(ni, 0));
      for (uint32_t b = 0; b < nb && k * cs + b * C < K; ++b) V[b][bi++] = 1;
      sym_ifft_top(V, C, cs, (k + 1) * cs);
      for (uint32_t b = 0; b < nb; ++b) coef_xor(acc[b], V[b]);
    }
    sym_fft_top(acc, C, cs, 0);
    for (uint32_t b = 0; b < nb && b * C < R; ++b) {
      out.push_back({b * C, std::min(C, R - b * C), int(b * C)});
      outs.push_back(acc[b]);
    }
  } else {
    std::vector<Coef> V(nb, Coef(ni, 0));
    for (size_t bi = 0; bi < ni; ++bi) V[bi][bi] = 1;
    sym_ifft_top(V, C, cs, 0);
    for (uint32_t k = 0; k * cs < R; ++k) {
      std::vector<Coef> Wk = V;
      sym_fft_top(Wk, C, cs, (k + 1) * cs);
      for (uint32_t b = 0; b < nb && k * cs + b * C < R; ++b) {
        out.push_back({k * cs + b * C, std::min(C, R - k * cs - b * C), int((k + 1) * cs + b * C)});
        outs.push_back(Wk[b]);
      }
    }
  }
  if (out.size() > size_t(max_blocks(C))) return plan_fail_unsupported("too many output blocks");
  j.n_out = int(out.size());
  pj.mix_stride = std::max(in.size(), out.size()) > size_t(kMaxBlocks) ? kMaxBlocksBig : kMaxBlocks;
  // one shared IFFT when a single input block feeds every output unmixed (low rate, C == cs)
  j.shared_in = (!high && nb == 1) ? 1 : 0;
  pj.n_z = j.shared_in ? 1 : j.n_out;
  pj.mode = j.shared_in ? kModeCols : kModeRows;
  pj.ppw = kPpwTarget;
  pj.copy_offs.clear();
  pj.offs.assign(size_t(j.n_in + j.n_out) * C, -1);
  for (int bi = 0; bi < j.n_in; ++bi) {
    InBlock& ib = j.in[bi];
    ib.base = src_base;
    ib.line_stride = src_ls;
    ib.count = int(in[bi].count);
    for (uint32_t p = 0; p < in[bi].count; ++p) pj.offs[pj.in_off(bi) + p] = src(in[bi].first + p);
    pj.in_sd.push_back(in[bi].sd);
    pj.in_first.push_back(in[bi].first);
  }
  for (int oi = 0; oi < j.n_out; ++oi) {
    OutBlock& ob = j.out[oi];
    ob.base = dst_base;
    ob.line_stride = dst_ls;
    ob.trunc = int(out[oi].count);
    ob.limit = dst_limit;
    for (uint32_t p = 0; p < out[oi].count; ++p) pj.offs[pj.out_off(oi) + p] = dst(out[oi].first + p);
    pj.out_sd.push_back(out[oi].sd);
    if (!j.shared_in) set_mixing(pj, oi, nullptr, outs[oi]);
  }
  return RS2_OK;
}

// Fused copy-out of a job's loaded source symbols: source index q (a loaded position) is
// also written to base + line*ls + f(q) (f(q) < 0: not copied).  Needs whole-dword symbol
// I/O (s >= 4); the caller keeps a separate copy pass otherwise.
template <class F>
void set_copy(PlannedJob& pj, uint8_t* base, int64_t ls, int64_t limit, F f) {
  pj.copy_base = base;
  pj.copy_ls = ls;
  pj.copy_limit = limit;
  pj.copy_offs.assign(size_t(pj.job.n_in) * pj.C, -1);
  for (int b = 0; b < pj.job.n_in; ++b)
    for (int p = 0; p < pj.job.in[b].count; ++p)
      pj.copy_offs[size_t(b) * pj.C + p] = f(pj.in_first[b] + uint32_t(p));
}

// True when every in-block that carries copy positions is loaded by at least one output
// block (the kernel skips in-blocks whose mixing coefficients are all zero); otherwise the
// copy is dropped and the caller falls back to a separate copy pass.
bool copy_covered(PlannedJob& pj) {
  if (pj.copy_offs.empty()) return false;
  if (pj.mode == kModeRows) {  // the mixed-encode kernel has no copy-out (register budget)
    pj.copy_offs.clear();
    return false;
  }
  const CodecJobBig& j = pj.job;
  for (int b = 0; b < j.n_in; ++b) {
    bool any_copy = false;
    for (int p = 0; p < pj.C; ++p) any_copy |= pj.copy_offs[size_t(b) * pj.C + p] >= 0;
    if (!any_copy || j.shared_in) continue;
    bool loaded = false;
    for (int o = 0; o < j.n_out; ++o)
      loaded |= j.m2_kind[o][b] != 0 || (pj.mode == kModeDecode && j.m1_kind[o][b] != 0);
    if (!loaded) {
      pj.copy_offs.clear();
      return false;
    }
  }
  return true;
}

// Attach sd tables, upload the offsets and mixing tables.  Must follow plan_encode / plan_decode.
int bind_job(Context* ctx, PlannedJob& pj, JobMem& mem, hipStream_t st) {
  CodecJobBig& j = pj.job;
  // flattened lane space: pairs rounded up to even (lane pairs share a 64-byte chunk); lines may
  // then share a workgroup, whose per-lane line step must fit the kernel's 32-bit offsets
  int64_t max_ls = std::max<int64_t>(pj.copy_ls, 0);
  for (int b = 0; b < j.n_in; ++b) max_ls = std::max(max_ls, std::abs(j.in[b].line_stride));
  for (int o = 0; o < j.n_out; ++o) max_ls = std::max(max_ls, std::abs(j.out[o].line_stride));
  j.pairs_span = (j.n_pairs + 1) & ~1;
  if (64 * max_ls + 65536 >= (int64_t(1) << 31)) j.pairs_span = (j.n_pairs + 63) & ~63;
  // position offsets, then the fused copy-out offsets (if any), in one upload
  const size_t n_off = pj.offs.size();
  if (!pj.copy_offs.empty()) pj.offs.insert(pj.offs.end(), pj.copy_offs.begin(), pj.copy_offs.end());
  auto t0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* name) {
    const auto t1 = std::chrono::steady_clock::now();
    host_trace(name, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  };
  HIP_TRY(mem.offs.ensure(pj.offs.size() * 8));
  lap("bind_offs_ensure");
  HIP_TRY(ctx->upload(mem.offs.p, pj.offs.data(), pj.offs.size() * 8, st));
  lap("bind_offs_copy");
  for (int b = 0; b < j.n_in; ++b) {
    if (!pj.copy_offs.empty()) {
      j.in[b].copy_base = pj.copy_base;
      j.in[b].copy_off = mem.offs.as<int64_t>() + n_off + size_t(b) * pj.C;
      j.in[b].copy_line_stride = pj.copy_ls;
      j.in[b].copy_limit = pj.copy_limit;
    } else {
      j.in[b].copy_off = nullptr;
    }
    j.in[b].pos_off = mem.offs.as<int64_t>() + pj.in_off(b);
    j.in[b].sd_tab = ctx->stream(pj.C, pj.in_sd[b], pj.ppw);
    if (!j.in[b].sd_tab) return fail(RS2_E_DEVICE, "table upload failed");
    j.in[b].zero_first = group0_zero(pj.C, pj.in_sd[b], pj.ppw);
  }
  for (int o = 0; o < j.n_out; ++o) {
    j.out[o].pos_off = mem.offs.as<int64_t>() + pj.out_off(o);
    j.out[o].sd_tab = ctx->stream(pj.C, pj.out_sd[o], pj.ppw);
    if (!j.out[o].sd_tab) return fail(RS2_E_DEVICE, "table upload failed");
    j.out[o].zero_first = group0_zero(pj.C, pj.out_sd[o], pj.ppw);
  }
  lap("bind_sd_tables");
  if (pj.has_mix) {
    // the tables of output blocks o < n_out only (rows of mix_stride * 2 tables)
    const size_t used = std::min(pj.mix.size(), size_t(j.n_out) * pj.mix_stride * 2 * kTabU16);
    HIP_TRY(mem.mix.ensure(pj.mix.size() * 2));
    HIP_TRY(ctx->upload(mem.mix.p, pj.mix.data(), used * 2, st));
    j.mix_tab = mem.mix.as<uint16_t>();
    lap("bind_mix_copy");
  }
  return RS2_OK;
}

int bind_encode(Context* ctx, PlannedJob& pj, JobMem& mem, hipStream_t st) {
  return bind_job(ctx, pj, mem, st);
}

// ---------------------------------------------------------------------------------------------
// decode planning: erasure locator logs (FWHT), per-block IFFTs, block mixing matrices
// ---------------------------------------------------------------------------------------------
// XOR-convolution of the erasure indicator with LOG over the decoder's subspace of size W:
//   L[p] = sum_{e erased} LOG[p ^ e]  (mod 65535),  via FWHT (W^-1 = 2^(16 - log W)).
// Arithmetic mod 65535 on 16-bit values as reed-solomon-simd does it (65535 aliases 0): the
// FWHT butterflies are one add and one fold each, no division.
inline uint32_t add_mod16(uint32_t a, uint32_t b) {
  const uint32_t t = a + b;
  return (t + (t >> 16)) & 0xFFFFu;
}
inline uint32_t sub_mod16(uint32_t a, uint32_t b) {
  const uint32_t d = a - b;
  return (d + (d >> 16)) & 0xFFFFu;
}
void fwht16(uint32_t* a, uint32_t W) {
  for (uint32_t h = 1; h < W; h <<= 1)
    for (uint32_t i = 0; i < W; i += 2 * h)
      for (uint32_t j = i; j < i + h; ++j) {
        const uint32_t x = a[j], y = a[j + h];
        a[j] = add_mod16(x, y);
        a[j + h] = sub_mod16(x, y);
      }
}
// FWHT of LOG over the first W entries: the same for every erasure pattern of a size, so it is
// computed once per W (reed-solomon-simd keeps the 65536-point one, LOG_WALSH, as a table)
const std::vector<uint32_t>& log_walsh(uint32_t W) {
  static std::mutex mu;
  static std::map<uint32_t, std::vector<uint32_t>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(W);
  if (it != cache.end()) return it->second;
  const Gf& g = gf();
  std::vector<uint32_t> lg(W);
  for (uint32_t i = 0; i < W; ++i) lg[i] = g.log[i] % kModulus;  // LOG[0] = 65535 == 0
  fwht16(lg.data(), W);
  return cache.emplace(W, std::move(lg)).first->second;
}
// Erasure locator logs, the decoder's eval_poly restricted to its W-point subspace:
//   L[p] = sum_{e erased} LOG[p ^ e]  (mod 65535)  = FWHT^-1(FWHT(erased) * FWHT(LOG)),
// with FWHT^-1 = FWHT / W and 1/W = 2^(16 - log W) mod 65535 (2^16 == 1): a 16-bit rotate.
std::vector<uint32_t> erasure_logs(const std::vector<uint8_t>& erased, uint32_t W) {
  const std::vector<uint32_t>& lw = log_walsh(W);
  std::vector<uint32_t> a(W);
  for (uint32_t i = 0; i < W; ++i) a[i] = erased[i] ? 1u : 0u;
  fwht16(a.data(), W);
  for (uint32_t i = 0; i < W; ++i) {
    const uint32_t x = a[i] == 0xFFFFu ? 0u : a[i], y = lw[i] == 0xFFFFu ? 0u : lw[i];
    a[i] = x * y % kModulus;  // < 65535^2 < 2^32
  }
  fwht16(a.data(), W);
  uint32_t logW = 0;
  while ((1u << logW) < W) ++logW;
  const uint32_t k = (16 - logW) & 15;
  for (uint32_t i = 0; i < W; ++i) {
    uint32_t x = a[i] == 0xFFFFu ? 0u : a[i];
    x = ((x << k) | (x >> (16 - k))) & 0xFFFFu;  // x * 2^k mod 65535 (k = 0: x)
    a[i] = x == 0xFFFFu ? 0u : x;
  }
  return a;
}

// Block-level mixing: out block o = FFT_o( sum_b M1[o][b] Dw(X_b) + M2[o][b] X_b ).
void mixing_matrices(int m, uint32_t cs, uint32_t W, std::vector<std::vector<uint32_t>>& M1,
                     std::vector<std::vector<uint32_t>>& M2) {
  const Gf& g = gf();
  std::vector<std::vector<uint32_t>> Va(m, std::vector<uint32_t>(m, 0)), Vb = Va;
  for (int i = 0; i < m; ++i) Va[i][i] = 1;
  auto xor_into = [&](std::vector<uint32_t>& a, const std::vector<uint32_t>& b) {
    for (int i = 0; i < m; ++i) a[i] ^= b[i];
  };
  auto mul_into = [&](std::vector<uint32_t>& a, const std::vector<uint32_t>& b, uint32_t c) {
    for (int i = 0; i < m; ++i) a[i] ^= g.mul(b[i], c);
  };
  for (uint32_t d = cs; d < W; d *= 2)
    for (uint32_t r = 0; r < W; r += 2 * d) {
      const uint32_t c = g.skew[r + d - 1];
      for (uint32_t j = 0; j < d / cs; ++j) {
        const int x = int(r / cs + j), y = int(x + d / cs);
        xor_into(Va[y], Va[x]);
        xor_into(Vb[y], Vb[x]);
        if (c != kModulus) {
          mul_into(Va[x], Va[y], c);
          mul_into(Vb[x], Vb[y], c);
        }
      }
    }
  // formal derivative: in-block part (Dw) moves alpha to beta; cross-block bits add blocks
  std::vector<std::vector<uint32_t>> nVa(m, std::vector<uint32_t>(m, 0));
  for (int i = 0; i < m; ++i)
    for (int t = 0; (1 << t) < m; ++t)
      if (!((i >> t) & 1) && (i | (1 << t)) < m) xor_into(nVa[i], Va[i | (1 << t)]);
  Vb = Va;
  Va = nVa;
  for (uint32_t d = W / 2; d >= cs && d > 0; d /= 2) {
    for (uint32_t r = 0; r < W; r += 2 * d) {
      const uint32_t c = g.skew[r + d - 1];
      for (uint32_t j = 0; j < d / cs; ++j) {
        const int x = int(r / cs + j), y = int(x + d / cs);
        if (c != kModulus) {
          mul_into(Va[x], Va[y], c);
          mul_into(Vb[x], Vb[y], c);
        }
        xor_into(Va[y], Va[x]);
        xor_into(Vb[y], Vb[x]);
      }
    }
    if (d == cs) break;
  }
  M1 = Vb;
  M2 = Va;
}

// Symbols of a 1D decode: present[q] = source offset (or -1) for shard index q < n;
// dst(i) = destination offset of source symbol i (only erased originals are written here).
struct DecodeSpec {
  uint32_t K = 0, R = 0;
  std::vector<int64_t> present;        // size K + R
  const uint8_t* src_base = nullptr;
  int64_t src_ls = 0;
  uint8_t* dst_base = nullptr;
  int64_t dst_ls = 0;
  std::vector<int64_t> dst;            // size K: destination offset of source symbol i
  int64_t dst_limit = INT64_MAX;
  int symbol_size = 0;
  bool copy_present = false;           // also write present originals to dst (fused copy)
};

int plan_decode(const DecodeSpec& sp, PlannedJob& pj) {
  const uint32_t K = sp.K, R = sp.R;
  if (!rate_supported(K, R)) return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "unsupported shard count");
  const bool high = use_high_rate(K, R);
  const uint32_t cs0 = high ? next_pow2(R) : next_pow2(K);
  const uint32_t end = high ? cs0 + K : cs0 + R;
  const uint32_t W = next_pow2(end);
  // blocks of C positions over the whole W-point transform (the chunk size cs0 only fixes
  // where originals and recovery shards sit)
  const uint32_t cs = std::min(cs0, block_max());
  const int m = int(W / cs);
  pj.in_sd.clear();
  pj.out_sd.clear();
  pj.in_first.clear();
  pj.copy_offs.clear();
  pj.mix.clear();
  pj.has_mix = false;
  pj.mode = kModeDecode;
  auto opos = [&](uint32_t i) { return high ? cs0 + i : i; };
  auto rpos = [&](uint32_t j) { return high ? j : cs0 + j; };
  std::vector<uint8_t> erased(W, 0);
  std::vector<int64_t> src_at(W, -1);
  for (uint32_t i = 0; i < K; ++i) {
    if (sp.present[i] >= 0) src_at[opos(i)] = sp.present[i];
    else erased[opos(i)] = 1;
  }
  for (uint32_t j = 0; j < R; ++j) {
    if (sp.present[K + j] >= 0) src_at[rpos(j)] = sp.present[K + j];
    else erased[rpos(j)] = 1;
  }
  if (high)
    for (uint32_t p = R; p < cs0; ++p) erased[p] = 1;
  else
    for (uint32_t p = end; p < W; ++p) erased[p] = 1;
  const std::vector<uint32_t> L = erasure_logs(erased, W);
  std::vector<std::vector<uint32_t>> M1, M2;
  mixing_matrices(m, cs, W, M1, M2);

  CodecJobBig& j = pj.job;
  j = CodecJobBig{};
  j.symbol_size = sp.symbol_size;
  j.n_pairs = (sp.symbol_size + 3) / 4;
  j.shared_in = 0;
  pj.C = int(cs);
  // input blocks with at least one present position
  std::vector<int> in_blocks, out_blocks;
  for (int b = 0; b < m; ++b) {
    bool any = false;
    for (uint32_t p = 0; p < cs; ++p) any |= src_at[b * cs + p] >= 0;
    if (any) in_blocks.push_back(b);
  }
  for (int b = 0; b < m; ++b) {
    bool any = false;
    for (uint32_t i = 0; i < K; ++i)
      any |= sp.present[i] < 0 && opos(i) / cs == uint32_t(b);
    if (any) out_blocks.push_back(b);
  }
  if (in_blocks.size() > size_t(max_blocks(int(cs))) || out_blocks.size() > size_t(max_blocks(int(cs))))
    return plan_fail_unsupported("too many decode blocks");
  pj.mix_stride = std::max(in_blocks.size(), out_blocks.size()) > size_t(kMaxBlocks) ? kMaxBlocksBig
                                                                                     : kMaxBlocks;
  // Block pair (rs2_codec.hip load_ifft, CodecJob::pair_p): with one output block, an input
  // block Q mixed with M1 = 0 (coefficient 1 once folded below) and another block P whose
  // active waves (ceil(count / ppw)) fit the workgroup together run their loads and in-wave
  // IFFT layers in one pass.  Q moves to the end of the input list (the kernel's convention).
  const int ppw = std::min<int>(int(cs), kPpwTarget), nw = int(cs) / ppw;
  auto block_waves = [&](int b) {
    int count = 0;
    for (uint32_t p = 0; p < cs; ++p)
      if (src_at[b * cs + p] >= 0) count = int(p) + 1;
    return (count + ppw - 1) / ppw;
  };
  int pair_p = -1, pair_nw = 0;
  static const bool no_pair = [] {
    const char* e = std::getenv("RS2_PAIR");  // A/B knob: 0 = never pair
    return e && std::atoi(e) == 0;
  }();
  if (!no_pair && nw > 1 && out_blocks.size() == 1) {
    const int o = out_blocks[0];
    for (size_t qi = 0; qi < in_blocks.size() && pair_p < 0; ++qi) {
      const int q = in_blocks[qi];
      if (M1[o][q] != 0 || M2[o][q] == 0) continue;
      for (size_t pi = 0; pi < in_blocks.size(); ++pi) {
        const int p = in_blocks[pi];
        if (p == q || (M1[o][p] == 0 && M2[o][p] == 0)) continue;
        if (block_waves(p) + block_waves(q) > nw) continue;
        in_blocks.erase(in_blocks.begin() + qi);
        in_blocks.push_back(q);
        pair_p = int(std::find(in_blocks.begin(), in_blocks.end(), p) - in_blocks.begin());
        pair_nw = block_waves(p);
        break;
      }
    }
  }
  std::fill(std::begin(j.pair_p), std::end(j.pair_p), int8_t(-1));
  std::fill(std::begin(j.pair_q), std::end(j.pair_q), int8_t(-1));
  std::fill(std::begin(j.pair_nw), std::end(j.pair_nw), int8_t(0));
  if (pair_p >= 0) {
    j.pair_p[0] = int8_t(pair_p);
    j.pair_q[0] = int8_t(in_blocks.size() - 1);
    j.pair_nw[0] = int8_t(pair_nw);
  }
  j.n_in = int(in_blocks.size());
  j.n_out = int(out_blocks.size());
  pj.n_z = j.n_out;
  pj.offs.assign(size_t(j.n_in + j.n_out) * cs, -1);
  pj.pre_logs.assign(size_t(j.n_out) * j.n_in * cs, 0);
  pj.post_logs.assign(size_t(j.n_out) * cs, 0);
  pj.has_pre = pj.has_post = true;
  for (int bi = 0; bi < j.n_in; ++bi) {
    const int b = in_blocks[bi];
    InBlock& ib = j.in[bi];
    ib.base = sp.src_base;
    ib.line_stride = sp.src_ls;
    int count = 0;
    for (uint32_t p = 0; p < cs; ++p) {
      const uint32_t gp = b * cs + p;
      if (src_at[gp] >= 0) {
        pj.offs[pj.in_off(bi) + p] = src_at[gp];
        count = int(p) + 1;
      }
    }
    ib.count = count;
    pj.in_sd.push_back(int(b * cs));
    pj.in_first.push_back(uint32_t(b * cs));
  }
  if (sp.copy_present) {
    pj.copy_base = sp.dst_base;
    pj.copy_ls = sp.dst_ls;
    pj.copy_limit = sp.dst_limit;
    pj.copy_offs.assign(size_t(j.n_in) * cs, -1);
    for (int bi = 0; bi < j.n_in; ++bi)
      for (uint32_t i = 0; i < K; ++i)
        if (sp.present[i] >= 0 && opos(i) / cs == uint32_t(in_blocks[bi]))
          pj.copy_offs[size_t(bi) * cs + opos(i) % cs] = sp.dst[i];
  }
  for (int oi = 0; oi < j.n_out; ++oi) {
    const int o = out_blocks[oi];
    OutBlock& ob = j.out[oi];
    ob.base = sp.dst_base;
    ob.line_stride = sp.dst_ls;
    ob.limit = sp.dst_limit;
    int trunc = 0;
    for (uint32_t i = 0; i < K; ++i) {
      if (sp.present[i] >= 0) continue;
      const uint32_t gp = opos(i);
      if (gp / cs != uint32_t(o)) continue;
      const uint32_t p = gp % cs;
      pj.offs[pj.out_off(oi) + p] = sp.dst[i];
      pj.post_logs[size_t(oi) * cs + p] = uint16_t(kModulus - L[gp]);  // 65535 == times one
      trunc = std::max(trunc, int(p) + 1);
    }
    ob.trunc = trunc;
    pj.out_sd.push_back(int(o * cs));
    // Fold one mixing coefficient of every input block into its pre-multiplier (the decoder
    // scales each loaded symbol by exp(L[p]) anyway).  With f = M1 (or M2 when M1 is zero) and
    // X'_b = IFFT_b(f * exp(L) * in_b) = f * X_b (IFFT and Dw are GF-linear):
    //   M1 Dw(X_b) + M2 X_b = Dw(X'_b) + (M2 / M1) X'_b
    // so the block costs at most one table multiply per position instead of three.  Each output
    // block folds its own coefficients, hence per-output pre tables (CodecJob::pre_z_stride).
    const Gf& g = gf();
    Coef c1(j.n_in), c2(j.n_in);
    for (int bi = 0; bi < j.n_in; ++bi) {
      const int b = in_blocks[bi];
      c1[bi] = M1[o][b];
      c2[bi] = M2[o][b];
      const uint32_t f = c1[bi] ? c1[bi] : c2[bi];
      if (f == 0) continue;  // this output does not use the block
      const uint32_t lf = g.log[f];
      if (c1[bi]) {
        c2[bi] = c2[bi] ? g.mul(c2[bi], kModulus - lf) : 0u;
        c1[bi] = 1;
      } else {
        c2[bi] = 1;
      }
      uint16_t* pl = pj.pre_logs.data() + (size_t(oi) * j.n_in + bi) * cs;
      for (uint32_t p = 0; p < cs; ++p)
        if (src_at[b * cs + p] >= 0) pl[p] = uint16_t(Gf::add_mod(L[b * cs + p], lf));
    }
    set_mixing(pj, oi, &c1, c2);
  }
  return RS2_OK;
}

// Upload a decode job's arrays and build its per-position tables on the device.
int bind_decode(Context* ctx, PlannedJob& pj, JobMem& mem, hipStream_t st) {
  CodecJobBig& j = pj.job;
  const int rc = bind_job(ctx, pj, mem, st);
  if (rc != RS2_OK) return rc;
  const size_t npre = pj.pre_logs.size(), npost = pj.post_logs.size();
  std::vector<uint16_t>& logs = pj.logs;
  logs.resize(npre + npost);
  std::copy(pj.pre_logs.begin(), pj.pre_logs.end(), logs.begin());
  std::copy(pj.post_logs.begin(), pj.post_logs.end(), logs.begin() + npre);
  HIP_TRY(mem.logs.ensure(std::max<size_t>(logs.size() * 2, 16)));
  HIP_TRY(mem.pre_tab.ensure(std::max<size_t>((npre + npost) * kTabU16 * 2, 16)));
  if (!logs.empty()) {
    HIP_TRY(ctx->upload(mem.logs.p, logs.data(), logs.size() * 2, st));
    HIP_TRY(rs2k_launch_build_mul_tables(ctx->exp_t.as<uint16_t>(), ctx->log_t.as<uint16_t>(),
                                         mem.logs.as<uint16_t>(), int(logs.size()),
                                         mem.pre_tab.as<uint16_t>(), st));
  }
  for (int b = 0; b < j.n_in; ++b)
    j.in[b].pre_tab = mem.pre_tab.as<uint16_t>() + size_t(b) * pj.C * kTabU16;
  j.pre_z_stride = int64_t(j.n_in) * pj.C * kTabU16;
  for (int o = 0; o < j.n_out; ++o)
    j.out[o].post_tab = mem.pre_tab.as<uint16_t>() + (npre + size_t(o) * pj.C) * kTabU16;
  return RS2_OK;
}

constexpr int kMerkleMaxLeaves = 4096;  // rs2_hash.hip kMerkleMax (one-wave / one-WG trees)
// n_shards above that: the trees' level L (the first with ceil(n / 2^L) <= 4,096 nodes) is
// folded straight from the leaves by a kernel of its own into a scratch buffer
// (rs2k_launch_merkle_trees d_scratch) and the pair-leaf root folds its first L levels into its
// loads (L <= 4); the codec plans take up to 128 blocks of 512 (W <= 65536; jobs above 64 blocks
// run from device memory, CodecJobBig).  That covers every n_shards reed-solomon-simd admits for
// both codes (up to 49,155, the reference's own bound, config.rs:446-460); beyond,
// RS2_E_INCOMPATIBLE_PARAMETERS from the rate check.  Full node arrays (recovery-symbol proofs)
// of wider trees are built one level per launch through HBM; blob batches run their wide trees
// a blob at a time.
constexpr int kMaxShards = 16 * kMerkleMaxLeaves - 1;  // n_shards is a u16
// scratch bytes of the trees' folded level for `trees` trees of n leaves (0 when not needed)
size_t tree_scratch_bytes(int64_t trees, int64_t n) {
  if (n <= kMerkleMaxLeaves) return 0;
  int L = 1;
  while (((n + (int64_t(1) << L) - 1) >> L) > kMerkleMaxLeaves) ++L;
  return size_t(trees) * size_t((n + (int64_t(1) << L) - 1) >> L) * 32;
}

// Root of n leaf digests (32 B each, contiguous) by one level launch per tree level
// (merkle.rs:226-266: odd levels padded with the zero node; one leaf is its own root).
int device_merkle_root(const uint8_t* d_digests, uint64_t n, DevBuf& tmp, uint8_t* d_root,
                       hipStream_t st) {
  if (n == 0) {
    HIP_TRY(hipMemsetAsync(d_root, 0, 32, st));
    return RS2_OK;
  }
  const uint64_t half = (n + 1) / 2;
  HIP_TRY(tmp.ensure(size_t(2 * half * 32)));
  uint8_t* a = tmp.as<uint8_t>();
  uint8_t* b = a + half * 32;
  const uint8_t* src = d_digests;
  uint8_t* dst = a;
  for (uint64_t cnt = n; cnt > 1; cnt = (cnt + 1) / 2) {
    HIP_TRY(rs2k_launch_merkle_level(src, int64_t(cnt), dst, st));
    src = dst;
    dst = dst == a ? b : a;
  }
  HIP_TRY(hipMemcpyAsync(d_root, src, 32, hipMemcpyDeviceToDevice, st));
  return RS2_OK;
}

// Pinned staging ring of the host-buffer ABI.  A transfer is cut into slot-sized pieces: the
// DMA of one piece overlaps the host copies (context worker pool) of the others.  Contiguous
// device ranges of a piece move with one hipMemcpyAsync.  A slot is reused only after the event
// of its last DMA, so consecutive calls need no extra synchronisation.
struct Stager {
  static constexpr int kSlots = 4;
  size_t slot_bytes = size_t(32) << 20;
  PinnedBuf ring;
  hipEvent_t ev[kSlots] = {};
  Stager() = default;
  Stager(const Stager&) = delete;
  Stager& operator=(const Stager&) = delete;
  ~Stager() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
  int init() {
    if (ring.p) return RS2_OK;
    HIP_TRY(ring.ensure(slot_bytes * kSlots));
    for (auto& e : ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return RS2_OK;
  }
  uint8_t* slot(int k) { return static_cast<uint8_t*>(ring.p) + size_t(k % kSlots) * slot_bytes; }
};

// Pinned staging rings are leased per host-buffer call from a per-device pool (a plan no
// longer owns one): 128 MiB of pinned memory is not re-pinned for every new plan, and the rings
// pinned at once are bounded by the host calls in flight, not by the plans alive.
// RS2_STAGING_RINGS (default 0, at most 16) pins that many rings at the first lease, for a
// fixed pinned budget from the start.
struct StagerPool {
  std::mutex mu;
  bool primed = false;
  std::vector<std::unique_ptr<Stager>> free;
};
StagerPool& stager_pool(int device) {
  // never destroyed: pinned rings outlive the HIP runtime's own teardown at process exit
  static StagerPool* pools = new StagerPool[64];
  return pools[std::min(std::max(device, 0), 63)];
}
struct StagerLease {
  int dev;
  std::unique_ptr<Stager> st;
  explicit StagerLease(int device) : dev(device) {
    StagerPool& pool = stager_pool(dev);
    std::lock_guard<std::mutex> lk(pool.mu);
    if (!pool.primed) {
      pool.primed = true;
      const char* e = std::getenv("RS2_STAGING_RINGS");
      for (int i = 0, k = e ? std::min(16, std::atoi(e)) : 0; i < k; ++i) {
        auto sg = std::make_unique<Stager>();
        if (sg->init() != RS2_OK) break;
        pool.free.push_back(std::move(sg));
      }
    }
    if (!pool.free.empty()) {
      st = std::move(pool.free.back());
      pool.free.pop_back();
    } else {
      st = std::make_unique<Stager>();
    }
  }
  ~StagerLease() {
    StagerPool& pool = stager_pool(dev);
    std::lock_guard<std::mutex> lk(pool.mu);
    if (pool.free.size() < 16) pool.free.push_back(std::move(st));  // else unpinned here
  }
  StagerLease(const StagerLease&) = delete;
  StagerLease& operator=(const StagerLease&) = delete;
};

struct Piece {
  std::vector<Seg> frags;  // h / d of each fragment; the slot holds them back to back
};

std::vector<Piece> cut_pieces(const std::vector<Seg>& segs, size_t slot) {
  std::vector<Piece> out;
  size_t fill = slot;
  for (const auto& g : segs) {
    size_t off = 0;
    while (off < g.len) {
      if (fill == slot) {
        out.emplace_back();
        fill = 0;
      }
      const size_t take = std::min(g.len - off, slot - fill);
      out.back().frags.push_back({g.h + off, g.d + off, take});
      off += take;
      fill += take;
    }
  }
  return out;
}

// one hipMemcpyAsync per run of fragments that are contiguous on the device
hipError_t piece_dma(const Piece& pc, uint8_t* slot, bool to_host, hipStream_t st) {
  size_t o = 0;
  for (size_t i = 0; i < pc.frags.size();) {
    size_t j = i + 1, len = pc.frags[i].len;
    while (j < pc.frags.size() && pc.frags[j].d == pc.frags[j - 1].d + pc.frags[j - 1].len) {
      len += pc.frags[j].len;
      ++j;
    }
    const hipError_t e =
        to_host ? hipMemcpyAsync(slot + o, pc.frags[i].d, len, hipMemcpyDeviceToHost, st)
                : hipMemcpyAsync(pc.frags[i].d, slot + o, len, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    o += len;
    i = j;
  }
  return hipSuccess;
}

std::vector<Seg> slot_view(const Piece& pc, uint8_t* slot) {
  std::vector<Seg> v;
  size_t o = 0;
  for (const auto& f : pc.frags) {
    v.push_back({f.h, slot + o, f.len});
    o += f.len;
  }
  return v;
}

// Caller buffers page-locked with rs2_host_register: start -> length.  A transfer segment whose
// host range lies wholly inside one moves by DMA straight from / to it, without the ring.
std::mutex g_reg_mu;
std::map<uintptr_t, size_t> g_reg;

bool host_registered(const uint8_t* h, size_t len) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(h);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.upper_bound(p);
  if (it == g_reg.begin()) return false;
  --it;
  return p >= it->first && p + len <= it->first + it->second;
}

// Runs of segments contiguous on both sides (a caller's sliver rows laid out back to back, as
// on the device) that lie in registered host memory and reach kDirectMin bytes -> one
// hipMemcpyAsync each on st; the rest returned for the ring (a DMA call per scattered sliver
// costs more than staging it: decode inputs of randomly chosen slivers stay staged).
constexpr size_t kDirectMin = size_t(4) << 20;
std::vector<Seg> issue_direct(const std::vector<Seg>& segs, bool to_host, hipStream_t st,
                              hipError_t* err, bool* any) {
  std::vector<Seg> staged;
  *err = hipSuccess;
  *any = false;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (g_reg.empty()) return segs;
  }
  std::vector<Seg> runs;
  std::vector<std::pair<size_t, size_t>> span;  // [first, last) segment index of each run
  for (size_t i = 0; i < segs.size(); ++i) {
    const Seg& g = segs[i];
    if (!runs.empty() && g.h == runs.back().h + runs.back().len &&
        g.d == runs.back().d + runs.back().len) {
      runs.back().len += g.len;
      span.back().second = i + 1;
    } else {
      runs.push_back(g);
      span.push_back({i, i + 1});
    }
  }
  for (size_t r = 0; r < runs.size(); ++r) {
    const Seg& g = runs[r];
    if (g.len < kDirectMin || !host_registered(g.h, g.len)) {
      for (size_t i = span[r].first; i < span[r].second; ++i) staged.push_back(segs[i]);
      continue;
    }
    *any = true;
    const hipError_t e = to_host ? hipMemcpyAsync(g.h, g.d, g.len, hipMemcpyDeviceToHost, st)
                                 : hipMemcpyAsync(g.d, g.h, g.len, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) {
      *err = e;
      break;
    }
  }
  return staged;
}

// host -> device, enqueued on st (the host copies are done when this returns; the DMA is not;
// registered caller memory is read by the DMA itself, which every host-buffer call waits for
// before it returns)
int stage_h2d(Context* ctx, Stager& sg, const std::vector<Seg>& segs_all, hipStream_t st) {
  int rc = sg.init();
  if (rc != RS2_OK) return rc;
  hipError_t de;
  bool any;
  const std::vector<Seg> segs = issue_direct(segs_all, false, st, &de, &any);
  HIP_TRY(de);
  const std::vector<Piece> pcs = cut_pieces(segs, sg.slot_bytes);
  for (size_t k = 0; k < pcs.size(); ++k) {
    const int sl = int(k % Stager::kSlots);
    HIP_TRY(hipEventSynchronize(sg.ev[sl]));
    par_copy(ctx->pool, slot_view(pcs[k], sg.slot(sl)), false);
    HIP_TRY(piece_dma(pcs[k], sg.slot(sl), false, st));
    HIP_TRY(hipEventRecord(sg.ev[sl], st));
  }
  return RS2_OK;
}

// device -> host after the work queued on st; returns when every byte is in the host buffers
int stage_d2h(Context* ctx, Stager& sg, const std::vector<Seg>& segs_all, hipStream_t st) {
  int rc = sg.init();
  if (rc != RS2_OK) return rc;
  hipError_t de;
  bool any;
  const std::vector<Seg> segs = issue_direct(segs_all, true, st, &de, &any);
  HIP_TRY(de);
  if (segs.empty()) {
    if (any) HIP_TRY(hipStreamSynchronize(st));
    return RS2_OK;
  }
  const std::vector<Piece> pcs = cut_pieces(segs, sg.slot_bytes);
  auto issue = [&](size_t k) -> int {
    const int sl = int(k % Stager::kSlots);
    HIP_TRY(hipEventSynchronize(sg.ev[sl]));
    HIP_TRY(piece_dma(pcs[k], sg.slot(sl), true, st));
    HIP_TRY(hipEventRecord(sg.ev[sl], st));
    return RS2_OK;
  };
  for (size_t k = 0; k < pcs.size() && k < size_t(Stager::kSlots); ++k)
    if ((rc = issue(k)) != RS2_OK) return rc;
  for (size_t k = 0; k < pcs.size(); ++k) {
    const int sl = int(k % Stager::kSlots);
    HIP_TRY(hipEventSynchronize(sg.ev[sl]));
    par_copy(ctx->pool, slot_view(pcs[k], sg.slot(sl)), true);
    if (k + Stager::kSlots < pcs.size() && (rc = issue(k + Stager::kSlots)) != RS2_OK) return rc;
  }
  return RS2_OK;
}

}  // namespace
}  // namespace rs2

using namespace rs2;

// =============================================================================================
// plans
// =============================================================================================
struct rs2_plan {
  Context* ctx = nullptr;
  hipStream_t stream = nullptr;
  // the systematic-column codec runs beside the row codec on `side` (fork / join events)
  hipStream_t side = nullptr;
  // the same role for split encodes (rs2_encode_device_split_async), at the device's greatest
  // stream priority; created on first use
  hipStream_t side_hi = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr, copy_ev = nullptr;
  // the row codec's padded tail rows (a few workgroups) beside its main launch; created on
  // first use
  hipStream_t aux = nullptr;
  hipEvent_t aux_ev = nullptr;
  hipEvent_t leaf_ev = nullptr;        // the side stream's leaf hashes (run A) are done
  hipEvent_t enc_done = nullptr;       // the last encode's work (guards re-binding its arrays)
  uint16_t n = 0, kp = 0, ks = 0, s = 0;
  uint64_t blob_len = 0;
  // encode
  PlannedJob row, col_sys, col_rep;
  JobMem row_mem, col_sys_mem, col_rep_mem;
  DevBuf both, leaves, pairs, blob_id, sys_a_src, sys_a_dst;
  DevBuf int_primary, int_secondary;   // internal sliver buffers (compute_metadata / host API)
  DevBuf dev_blob;                     // host-API staging of the blob / decode output
  const void* bound_primary = nullptr;
  const void* bound_secondary = nullptr;
  bool sys_fused = false;              // systematic secondary slivers written by col_sys
  // the systematic primary slivers (= the blob's zero-padded rows) written by col_sys from its
  // own loads of the blob (InBlock::copy2_base); the padded last rows come from tail_rows
  bool prim_fused = false;
  DevBuf tail_rows;
  DevBuf tree_scratch;                 // n_shards > 4096: the trees' first level
  DevBuf tile_ctr;                     // pipelined codec launch sites' tile counters (kCtr*)
  const void* bound_both = nullptr;
  // blob batches (rs2_encode_batch_*): per-blob repair quadrants and leaf digests, the blob
  // lengths on the device (and the host copy they were uploaded from), the host-buffer form's
  // device blobs / slivers
  DevBuf batch_both, batch_leaves, batch_lens, batch_blob, batch_primary, batch_secondary,
      batch_hashes, batch_ids;
  std::vector<uint64_t> batch_lens_h;
  // decode (two slots so back-to-back async decodes never overwrite live arrays)
  PlannedJob dec_job[2];
  JobMem dec_mem[2];
  DevBuf dec_copy_src[2], dec_copy_dst[2];
  std::vector<int64_t> dec_copy_src_h[2], dec_copy_dst_h[2];  // alive until dec_done[slot]
  hipEvent_t dec_done[2] = {nullptr, nullptr};
  int dec_slot = 0;
  // the erasure pattern / buffers a slot's decode job was planned for: a repeat decode with the
  // same key reuses the slot's tables and offsets on the device instead of re-planning
  std::vector<int64_t> dec_key[2];
  bool dec_fused[2] = {false, false};
  // host-buffer API: pinned staging ring, a copy stream for the sliver D2H (released by a split
  // encode as soon as the primary slivers are final), row gather offsets of the Default check
  Stager* stage = nullptr;  // the pinned ring leased for the host-buffer call in progress
  hipStream_t io = nullptr;
  rs2_verifier* check_v = nullptr;
  DevBuf check_src, check_rows, check_roots;
  std::vector<int64_t> check_src_h;
  // opt-in stage profiler: events recorded between consecutive launches on the stream
  struct Prof {
    bool on = false;
    std::vector<hipEvent_t> free_events;
    std::vector<std::pair<std::string, hipEvent_t>> pending;  // "" = start mark
    std::map<std::string, std::pair<double, uint32_t>> acc;   // name -> (total ms, launches)
    std::vector<std::string> order;
  } prof;
  ~rs2_plan() {
    for (auto& e : dec_done)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : prof.free_events) (void)hipEventDestroy(e);
    for (auto& pe : prof.pending) (void)hipEventDestroy(pe.second);
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (join_ev) (void)hipEventDestroy(join_ev);
    if (copy_ev) (void)hipEventDestroy(copy_ev);
    if (aux_ev) (void)hipEventDestroy(aux_ev);
    if (leaf_ev) (void)hipEventDestroy(leaf_ev);
    if (aux) (void)hipStreamDestroy(aux);
    if (enc_done) (void)hipEventDestroy(enc_done);
    if (side) (void)hipStreamDestroy(side);
    if (side_hi) (void)hipStreamDestroy(side_hi);
    if (io) (void)hipStreamDestroy(io);
    if (check_v) rs2_verifier_destroy(check_v);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// Batched sliver verification state (no reference counterpart: the storage node verifies
// slivers one by one on a thread pool, walrus-service/src/node.rs:2615-2633).
struct rs2_verifier {
  Context* ctx = nullptr;
  hipStream_t stream = nullptr;
  uint16_t n = 0, k = 0, s = 0;
  PlannedJob job;
  JobMem mem;
  DevBuf input, leaves, roots;
  DevBuf repair;  // the slivers' repair symbols, [count][n - k][s]
  DevBuf tree_scratch;  // n > 4096: the trees' first level
  // recovery symbols with proofs: full trees, targets, outputs of the host-buffer form
  DevBuf nodes, targets, sym_out, proof_out;
  PinnedBuf h_in, h_out;  // host-buffer forms: slivers in, roots / symbols / proofs out
  int axis = 0;
  std::vector<uint16_t> targets_h;  // alive until the upload of the last call has landed
  // recorded on the caller's stream after each *_device_async call: destroy waits on it before
  // its buffers go back to the arena as quiesced (they may be handed out again at once)
  hipEvent_t done = nullptr;
  ~rs2_verifier() {
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// Device 1D codec over many independent codewords ("lines") with strided layouts: the
// building block of the partitioned (multi-GPU) 2D code and of batched recovery symbols.
// The encode job is planned once per layout and re-based per call (the base pointers travel
// in the kernel argument); decodes are planned per erasure pattern in two slots, each
// guarded by an event so an in-flight launch never sees its arrays rewritten.
struct rs2_codec {
  Context* ctx = nullptr;
  uint16_t n = 0, k = 0, s = 0;
  PlannedJob enc;
  JobMem enc_mem;
  int64_t enc_key[4] = {-1, -1, -1, -1};
  hipEvent_t enc_done = nullptr;
  PlannedJob dec[2];
  JobMem dec_mem[2];
  DevBuf copy_src[2], copy_dst[2];
  std::vector<int64_t> copy_src_h[2], copy_dst_h[2];
  hipEvent_t dec_done[2] = {nullptr, nullptr};
  int dec_slot = 0;
  ~rs2_codec() {
    if (enc_done) (void)hipEventDestroy(enc_done);
    for (auto& e : dec_done)
      if (e) (void)hipEventDestroy(e);
  }
};

namespace {

// Record a stage boundary on `st` (no-op unless profiling).  The stage's time is the span
// from the previous mark on this plan; a mark named "" only starts a span.
void mark(rs2_plan* p, const char* name, hipStream_t st) {
  auto& pr = p->prof;
  if (!pr.on) return;
  hipEvent_t e;
  if (!pr.free_events.empty()) {
    e = pr.free_events.back();
    pr.free_events.pop_back();
  } else if (hipEventCreate(&e) != hipSuccess) {
    return;
  }
  (void)hipEventRecord(e, st);
  pr.pending.emplace_back(name, e);
}

// host time since t0 under `name` (profiling on): the erasure-pattern planning of a decode
void prof_host(rs2_plan* p, const char* name, std::chrono::steady_clock::time_point t0) {
  auto& pr = p->prof;
  if (!pr.on) return;
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  host_trace(name, ms);
  auto it = pr.acc.find(name);
  if (it == pr.acc.end()) {
    pr.order.push_back(name);
    it = pr.acc.emplace(name, std::make_pair(0.0, 0u)).first;
  }
  it->second.first += ms;
  it->second.second += 1;
}

void prof_collect(rs2_plan* p) {
  auto& pr = p->prof;
  hipEvent_t prev = nullptr;
  for (auto& pe : pr.pending) {
    (void)hipEventSynchronize(pe.second);
    if (prev && !pe.first.empty()) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, prev, pe.second) == hipSuccess) {
        auto it = pr.acc.find(pe.first);
        if (it == pr.acc.end()) {
          pr.order.push_back(pe.first);
          it = pr.acc.emplace(pe.first, std::make_pair(0.0, 0u)).first;
        }
        it->second.first += ms;
        it->second.second += 1;
      }
    }
    prev = pe.second;
  }
  for (auto& pe : pr.pending) pr.free_events.push_back(pe.second);
  pr.pending.clear();
}

int64_t primary_len(const rs2_plan* p) { return int64_t(p->ks) * p->s; }
int64_t secondary_len(const rs2_plan* p) { return int64_t(p->kp) * p->s; }

// (Re)build the three encode jobs for the given device sliver buffers.  The offset / mixing
// uploads go on `st`, the stream the codecs are launched on next, so they land before the
// kernels read them; the device arrays are shared by every encode of the plan, so an encode
// still in flight on another stream is waited for before they are rewritten.
int bind_encode_buffers(rs2_plan* p, uint8_t* d_primary, uint8_t* d_secondary, hipStream_t st,
                        uint8_t* d_both = nullptr) {
  if (!d_both) d_both = p->both.as<uint8_t>();
  if (p->bound_primary == d_primary && p->bound_secondary == d_secondary &&
      p->bound_both == d_both)
    return RS2_OK;
  if (p->enc_done) HIP_TRY(hipEventSynchronize(p->enc_done));
  p->bound_primary = p->bound_secondary = p->bound_both = nullptr;  // valid after a full rebind
  const int64_t s = p->s, n = p->n, kp = p->kp, ks = p->ks;
  int rc;
  // rows: secondary encoding (K = K_s) of primary slivers 0..K_p -> secondary slivers K_s..n
  rc = plan_encode(
      uint32_t(ks), uint32_t(n - ks), int(s), d_primary, ks * s, [&](uint32_t c) { return int64_t(c) * s; },
      d_secondary, s, [&](uint32_t j) { return (ks + int64_t(j)) * kp * s; }, INT64_MAX, p->row);
  if (rc != RS2_OK) return rc;
  rc = bind_encode(p->ctx, p->row, p->row_mem, st);
  if (rc != RS2_OK) return rc;
  // systematic columns c < K_s: primary encoding (K = K_p) -> primary slivers K_p..n, column c
  rc = plan_encode(
      uint32_t(kp), uint32_t(n - kp), int(s), d_primary, s, [&](uint32_t r) { return int64_t(r) * ks * s; },
      d_primary, s, [&](uint32_t j) { return (kp + int64_t(j)) * ks * s; }, INT64_MAX, p->col_sys);
  if (rc != RS2_OK) return rc;
  // the column loads are exactly the systematic secondary slivers (secondary c, row r =
  // primary r, column c): write them out from the same loads instead of a transpose pass
  p->sys_fused = false;
  if (s >= 4) {
    set_copy(p->col_sys, d_secondary, kp * s, INT64_MAX, [&](uint32_t r) { return int64_t(r) * s; });
    p->sys_fused = copy_covered(p->col_sys);
  }
  rc = bind_encode(p->ctx, p->col_sys, p->col_sys_mem, st);
  if (rc != RS2_OK) return rc;
  // the column loads are also every byte of the blob: when one shared-input block holds the
  // K_p rows in order (position r at r * K_s * s), col_sys reads the blob in place and writes
  // the systematic primary slivers itself instead of a separate blob copy
  p->prim_fused = false;
  static const bool fuse_env = [] {  // RS2_FUSE_BLOB=0: the separate blob copy (A/B knob)
    const char* e = std::getenv("RS2_FUSE_BLOB");
    return !(e && std::atoi(e) == 0);
  }();
  if (fuse_env && p->sys_fused && p->col_sys.mode == kModeCols && p->col_sys.job.n_in == 1 &&
      p->col_sys.job.in[0].count == int(kp)) {
    bool in_order = true;
    for (int64_t r = 0; r < kp; ++r) in_order &= p->col_sys.offs[size_t(r)] == r * ks * s;
    const int64_t r_full = std::min<int64_t>(kp, int64_t(p->blob_len) / (ks * s));
    if (in_order && r_full < kp) HIP_TRY(p->tail_rows.ensure(size_t((kp - r_full) * ks * s)));
    p->prim_fused = in_order;
  }
  // repair columns c >= K_s: from secondary slivers K_s..n -> the both-repair quadrant
  rc = plan_encode(
      uint32_t(kp), uint32_t(n - kp), int(s), d_secondary + ks * kp * s, kp * s,
      [&](uint32_t r) { return int64_t(r) * s; }, d_both, s,
      [&](uint32_t j) { return int64_t(j) * (n - ks) * s; }, INT64_MAX, p->col_rep);
  if (rc != RS2_OK) return rc;
  rc = bind_encode(p->ctx, p->col_rep, p->col_rep_mem, st);
  if (rc != RS2_OK) return rc;
  p->bound_primary = d_primary;
  p->bound_secondary = d_secondary;
  p->bound_both = d_both;
  return RS2_OK;
}

// messages at least this large (K_p * K_s * s bytes) get the extra stream overlap in
// encode_device (tail rows beside the main row launch, leaf hashes split across streams)
constexpr int64_t kBigMessage = int64_t(64) << 20;

int encode_device(rs2_plan* p, const uint8_t* d_blob, uint8_t* d_primary, uint8_t* d_secondary,
                  uint8_t* d_hashes, uint8_t* d_blob_id, hipStream_t st, bool need_slivers,
                  hipStream_t prim_st = nullptr) {
  const int64_t s = p->s, n = p->n, kp = p->kp, ks = p->ks;
  const int64_t msg = kp * ks * s;
  int rc = bind_encode_buffers(p, d_primary, d_secondary, st);
  if (rc != RS2_OK) return rc;
  // The plan's buffers (repair quadrant, leaves, tile counters) serve one encode at a time: an
  // encode queued on another stream than the previous one's runs after it on the device.
  if (p->enc_done) HIP_TRY(hipStreamWaitEvent(st, p->enc_done, 0));
  // A split encode's primary slivers (blob copy + systematic-column codec on the side stream)
  // are the critical path of the caller's next step (a decode, a send).  Round 1 ran them on a
  // high-priority side stream; with the bench's steps correctly ordered (round 2: each encode
  // waits for the last reader of its buffers) that costs 3.73 -> 4.10 ms per step, so the side
  // stream keeps the default priority unless RS2_SIDE_PRIORITY=1 (A/B knob).
  hipStream_t side = p->side;
  static const char* pri_env = std::getenv("RS2_SIDE_PRIORITY");
  if (prim_st && pri_env && std::atoi(pri_env) != 0) {
    if (!p->side_hi) {
      int lo_pri = 0, hi_pri = 0;
      HIP_TRY(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
      HIP_TRY(hipStreamCreateWithPriority(&p->side_hi, hipStreamNonBlocking, hi_pri));
    }
    side = p->side_hi;
  }
  // tile counters of the pipelined codec launches below, one set per launch site (they may run
  // at once on different streams); zeroed once, and re-zeroed by each launch's last workgroup
  if (!p->tile_ctr.p) {
    HIP_TRY(p->tile_ctr.ensure(4 * kTileCtrWords * 4));
    HIP_TRY(hipMemsetAsync(p->tile_ctr.p, 0, 4 * kTileCtrWords * 4, st));
  }
  uint32_t* const ctr = p->tile_ctr.as<uint32_t>();
  mark(p, "", st);
  // Two streams.  Side: the systematic-column codec, which reads the blob's rows in place and
  // (fused, prim_fused) writes the systematic primary slivers (= the zero-padded blob rows) from
  // the same loads; else a D2D copy makes those slivers first.  Caller's stream: the row codec
  // -- rows that lie wholly inside the blob straight from d_blob, the padded tail rows from the
  // tail buffer (or, unfused, from the copied slivers) -- then the repair-column codec.  The
  // codec grids fill each other's last, partly empty rounds of workgroups; stage times overlap
  // and each is its own span.
  // The blob's partial last row (and any rows past its end), zero-padded, in a small buffer that
  // both codecs read in place of the missing rows (fused path).
  const int64_t r_full = std::min<int64_t>(kp, int64_t(p->blob_len) / (ks * s));
  // BlobEncoder::compute_metadata (blob_encoding.rs:406-486) keeps no sliver: with the blob read
  // in place (fused) the systematic slivers are never materialised, only hashed
  const bool meta_only = !need_slivers && p->prim_fused && p->sys_fused;
  const uint8_t* tail_base = nullptr;
  if (p->prim_fused && r_full < kp) {
    const int64_t have = int64_t(p->blob_len) - r_full * ks * s;
    HIP_TRY(p->tail_rows.ensure(size_t((kp - r_full) * ks * s)));  // the plan may have been rebound
    uint8_t* tail = p->tail_rows.as<uint8_t>();
    HIP_TRY(rs2k_launch_tail_rows(d_blob + r_full * ks * s, have, tail, (kp - r_full) * ks * s, st));
    mark(p, "enc_tail_rows", st);
    tail_base = tail - r_full * ks * s;  // row r >= r_full at tail_base + r * K_s * s
  }
  HIP_TRY(hipEventRecord(p->fork_ev, st));
  HIP_TRY(hipStreamWaitEvent(side, p->fork_ev, 0));
  mark(p, "", side);
  if (p->prim_fused) {
    CodecJobBig cj = p->col_sys.job;
    cj.in[0].base = d_blob;
    cj.in[0].copy2_base = d_primary;
    if (r_full < kp) {
      cj.in[0].alt_base = tail_base;
      cj.in[0].alt_from = int(r_full);
    }
    if (meta_only) {
      // compute_metadata: no systematic sliver is written (neither the secondary copy-out nor
      // the primary one); their leaves are hashed from the blob and the tail buffer below
      cj.in[0].copy_off = nullptr;
      cj.in[0].copy2_base = nullptr;
    }
    HIP_TRY(launch_codec_c(p->col_sys.C, cj, int(ks), p->col_sys.n_z, p->col_sys.mode, side, 1, 0,
                           0, 0, ctr));
  } else {
    if (p->blob_len)
      HIP_TRY(hipMemcpyAsync(d_primary, d_blob, p->blob_len, hipMemcpyDeviceToDevice, side));
    if (uint64_t(msg) > p->blob_len)
      HIP_TRY(hipMemsetAsync(d_primary + p->blob_len, 0, msg - p->blob_len, side));
    mark(p, "enc_blob_copy", side);
    HIP_TRY(hipEventRecord(p->copy_ev, side));
    HIP_TRY(p->col_sys.launch(int(ks), side, ctr));
  }
  mark(p, "enc_cols_sys_codec", side);
  HIP_TRY(hipEventRecord(p->join_ev, side));
  // all primary slivers are final here (systematic rows + the column code's repair rows):
  // work the caller queues on prim_st next (a decode, a D2H to the NIC) starts now, beside
  // the secondary codecs and the hashing still running on st
  if (prim_st) HIP_TRY(hipStreamWaitEvent(prim_st, p->join_ev, 0));
  // RS2_TAIL_AUX=1 (A/B): the padded tail rows (a few workgroups) on a stream of their own
  // beside the main row launch instead of after it, the repair-column codec waiting for both.
  // Off by default since round 5: beside the persistent row kernel the tail's workgroups wait
  // for CUs anyway (the kernel trace shows them finishing with it), and the step is 88.1-88.3
  // vs 87.7-87.9 GiB/s without them on their own stream (five interleaved pairs,
  // profiles/r05/exp/tailaux/)
  static const bool tail_aux = [] {
    const char* e = std::getenv("RS2_TAIL_AUX");
    return e && std::atoi(e) == 1;
  }();
  // (large blobs only: for small ones the extra stream and launch cost more than the tail, and
  // many plans encoding at once share the device's few hardware queues: C3's 16 plans on 16
  // streams measured 12.1 vs 13.6 GiB/s with it)
  const bool big = msg >= kBigMessage;
  const bool aux_tail = p->prim_fused && r_full < kp && r_full > 0 && tail_aux && big;
  if (aux_tail) {
    if (!p->aux) {
      HIP_TRY(hipStreamCreateWithFlags(&p->aux, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&p->aux_ev, hipEventDisableTiming));
    }
    HIP_TRY(hipStreamWaitEvent(p->aux, p->fork_ev, 0));
    mark(p, "", p->aux);
    CodecJobBig tail = p->row.job;
    tail.line_base = int(r_full);
    for (int b = 0; b < tail.n_in; ++b) tail.in[b].base = tail_base;
    HIP_TRY(launch_codec_c(p->row.C, tail, int(kp - r_full), p->row.n_z, p->row.mode, p->aux, 1,
                           0, 0, 0, ctr + 2 * kTileCtrWords));
    mark(p, "enc_rows_tail", p->aux);
    HIP_TRY(hipEventRecord(p->aux_ev, p->aux));
  }
  mark(p, "", st);
  if (r_full > 0) {
    CodecJobBig from_blob = p->row.job;  // same layout: blob row r is primary sliver r
    for (int b = 0; b < from_blob.n_in; ++b) from_blob.in[b].base = d_blob;
    HIP_TRY(launch_codec_c(p->row.C, from_blob, int(r_full), p->row.n_z, p->row.mode, st, 1, 0, 0,
                           0, ctr + kTileCtrWords));
  }
  if (aux_tail) {
    HIP_TRY(hipStreamWaitEvent(st, p->aux_ev, 0));
  } else if (r_full < kp) {
    CodecJobBig tail = p->row.job;
    tail.line_base = int(r_full);
    if (p->prim_fused)  // the padded rows from the tail buffer (filled above, on st)
      for (int b = 0; b < tail.n_in; ++b) tail.in[b].base = tail_base;
    else  // from the systematic primary slivers once the side stream's copy has landed
      HIP_TRY(hipStreamWaitEvent(st, p->copy_ev, 0));
    HIP_TRY(launch_codec_c(p->row.C, tail, int(kp - r_full), p->row.n_z, p->row.mode, st, 1, 0, 0,
                           0, ctr + 2 * kTileCtrWords));
  }
  mark(p, "enc_rows_codec", st);
  HIP_TRY(p->col_rep.launch(int(n - ks), st, ctr + 3 * kTileCtrWords));
  mark(p, "enc_cols_rep_codec", st);
  // leaf hashes of all n x n symbols, 2n Merkle trees, root and blob id.  The primary slivers'
  // leaves (run A) are hashed on the side stream as soon as the systematic-column codec is done,
  // beside the row / repair-column codecs; the secondary-side runs B and C here after them.
  SymbolMap map{d_primary, d_secondary, p->both.as<uint8_t>(), int(n), int(kp), int(ks), int(s)};
  static const bool split_leaf = [] {  // RS2_SPLIT_LEAF=0: one leaf launch after the join (A/B)
    const char* e = std::getenv("RS2_SPLIT_LEAF");
    return !(e && std::atoi(e) == 0);
  }();
  const bool split = split_leaf && p->sys_fused && big;  // (C3 streams: 11.1 vs 13.6 GiB/s)
  if (meta_only) {
    // run A (rows of K_s symbols, leaf (r, c) at r*n + c) from where the rows are: the blob's
    // whole rows in place, its zero-padded tail rows in the tail buffer, the repair rows K_p..n
    // in the primary scratch; then runs B and C (the secondary side) as below
    hipStream_t sa = split ? side : st;
    if (!split) HIP_TRY(hipStreamWaitEvent(st, p->join_ev, 0));
    mark(p, "", sa);
    auto rows_run = [&](const uint8_t* base, int64_t r0, int64_t rows) -> int {
      if (rows <= 0) return RS2_OK;
      SymbolMap rm{base, nullptr, nullptr, int(n), int(rows), int(ks), int(s)};
      HIP_TRY(rs2k_launch_leaf_hash(rm, 4, rows * n, 1, p->leaves.as<uint8_t>() + r0 * n * 32, sa));
      return RS2_OK;
    };
    int rc2 = rows_run(d_blob, 0, r_full);
    if (rc2 == RS2_OK && r_full < kp) rc2 = rows_run(tail_base + r_full * ks * s, r_full, kp - r_full);
    if (rc2 == RS2_OK) rc2 = rows_run(d_primary + kp * ks * s, kp, n - kp);
    if (rc2 != RS2_OK) return rc2;
    mark(p, "enc_leaf_hash_a", sa);
    if (split) HIP_TRY(hipEventRecord(p->leaf_ev, side));
    mark(p, "", st);
    HIP_TRY(rs2k_launch_leaf_hash(map, 3, n * n, 1, p->leaves.as<uint8_t>(), st));
    mark(p, "enc_leaf_hash", st);
    if (split) HIP_TRY(hipStreamWaitEvent(st, p->leaf_ev, 0));
  } else if (split) {
    mark(p, "", side);
    HIP_TRY(rs2k_launch_leaf_hash(map, 2, n * n, 1, p->leaves.as<uint8_t>(), side));
    mark(p, "enc_leaf_hash_a", side);
    HIP_TRY(hipEventRecord(p->leaf_ev, side));
    mark(p, "", st);
    HIP_TRY(rs2k_launch_leaf_hash(map, 3, n * n, 1, p->leaves.as<uint8_t>(), st));
    mark(p, "enc_leaf_hash", st);
    HIP_TRY(hipStreamWaitEvent(st, p->leaf_ev, 0));  // after join_ev on the side stream
  } else {
    HIP_TRY(hipStreamWaitEvent(st, p->join_ev, 0));
    mark(p, "", st);
    if (!p->sys_fused) {
      // systematic secondary slivers: secondary c, row r = primary r, column c (c < K_s)
      HIP_TRY(rs2k_launch_symbol_copy(d_primary, p->sys_a_src.as<int64_t>(), ks * s, d_secondary,
                                      p->sys_a_dst.as<int64_t>(), s, int(ks), int(kp), int(s),
                                      INT64_MAX, st));
      mark(p, "enc_sys_transpose", st);
    }
    HIP_TRY(rs2k_launch_leaf_hash(map, 0, n * n, 1, p->leaves.as<uint8_t>(), st));
    mark(p, "enc_leaf_hash", st);
  }
  mark(p, "", st);
  uint8_t* pairs = d_hashes ? d_hashes : p->pairs.as<uint8_t>();
  uint8_t* scratch = nullptr;
  if (const size_t sb = tree_scratch_bytes(2 * n, n)) {
    HIP_TRY(p->tree_scratch.ensure(sb));
    scratch = p->tree_scratch.as<uint8_t>();
  }
  HIP_TRY(rs2k_launch_merkle_trees(p->leaves.as<uint8_t>(), int(n), int(n), int(n), n * 32, 32,
                                   32, n * 32, pairs, 64, st, nullptr, 0, 1, 0, 0, scratch));
  mark(p, "enc_merkle_trees", st);
  HIP_TRY(rs2k_launch_merkle_root(pairs, int(n), p->blob_len,
                                  d_blob_id ? d_blob_id : p->blob_id.as<uint8_t>(), st));
  mark(p, "enc_merkle_root", st);
  HIP_TRY(hipEventRecord(p->enc_done, st));  // st has joined the side stream above
  return RS2_OK;
}

// Blob batch (the upload relay's many-blob encode, walrus-upload-relay/src/controller.rs:177;
// the client's encode_blobs_as, node_client.rs:3156-3221): n_blobs blobs of this plan's symbol
// size, blob b at d_blobs + b*blob_stride (lens[b] bytes, or the plan's blob_len for all), its
// slivers at d_primary + b*p_stride / d_secondary + b*s_stride (the single-blob layouts), its
// pair hashes at d_hashes + b*64n and BlobId at d_blob_ids + b*32.  Every stage is ONE launch
// over all blobs (the codec grids hold every blob's tiles, the hash grids a blob per grid.y),
// so many small blobs cost no more launches than one large one.
int encode_batch_device(rs2_plan* p, uint32_t n_blobs, const uint8_t* d_blobs, int64_t blob_stride,
                        const uint64_t* lens, uint8_t* d_primary, int64_t p_stride,
                        uint8_t* d_secondary, int64_t s_stride, uint8_t* d_hashes,
                        uint8_t* d_blob_ids, hipStream_t st) {
  const int64_t s = p->s, n = p->n, kp = p->kp, ks = p->ks;
  const int64_t msg = kp * ks * s, pl = ks * s, sl = kp * s;
  if (n_blobs == 0) return RS2_OK;
  if (n_blobs > 65535) return fail(RS2_E_INVALID_ARGUMENT, "more than 65535 blobs in a batch");
  if (!d_primary || !d_secondary || !d_hashes || !d_blob_ids)
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (p_stride < n * pl || s_stride < n * sl)
    return fail(RS2_E_INVALID_ARGUMENT, "sliver stride smaller than a blob's slivers");
  std::vector<uint64_t> lv(n_blobs, p->blob_len);
  uint64_t max_len = 0;
  for (uint32_t b = 0; b < n_blobs; ++b) {
    if (lens) lv[b] = lens[b];
    uint16_t sb = 0;
    int rc = rs2_symbol_size_for_blob(p->n, lv[b], &sb);
    if (rc != RS2_OK) return rc;
    if (sb != p->s) return fail(RS2_E_INVALID_ARGUMENT, "blob length outside the plan's symbol size");
    max_len = std::max(max_len, lv[b]);
  }
  if (max_len && !d_blobs) return fail(RS2_E_INVALID_ARGUMENT, "null blobs");
  if (n_blobs > 1 && int64_t(max_len) > blob_stride)
    return fail(RS2_E_INVALID_ARGUMENT, "blob stride smaller than a blob");
  const int64_t both_b = (n - kp) * (n - ks) * s, leaves_b = n * n * 32;
  HIP_TRY(p->batch_both.ensure(size_t(n_blobs) * both_b));
  HIP_TRY(p->batch_leaves.ensure(size_t(n_blobs) * leaves_b));
  int rc = bind_encode_buffers(p, d_primary, d_secondary, st, p->batch_both.as<uint8_t>());
  if (rc != RS2_OK) return rc;
  if (lv != p->batch_lens_h) {  // upload the lengths (the host copy stays alive until it lands)
    if (p->enc_done) HIP_TRY(hipEventSynchronize(p->enc_done));
    p->batch_lens_h = lv;
    HIP_TRY(p->batch_lens.ensure(lv.size() * 8));
    HIP_TRY(p->ctx->upload(p->batch_lens.p, p->batch_lens_h.data(), lv.size() * 8, st));
  }
  const uint64_t* d_lens = p->batch_lens.as<uint64_t>();
  const int B = int(n_blobs);
  mark(p, "", st);
  HIP_TRY(rs2k_launch_batch_blob_copy(d_blobs, blob_stride, d_lens, msg, d_primary, p_stride, B, st));
  mark(p, "enc_blob_copy", st);
  HIP_TRY(launch_codec_c(p->col_sys.C, p->col_sys.job, int(ks), p->col_sys.n_z, p->col_sys.mode,
                         st, B, p_stride, p_stride, s_stride));
  mark(p, "enc_cols_sys_codec", st);
  HIP_TRY(launch_codec_c(p->row.C, p->row.job, int(kp), p->row.n_z, p->row.mode, st, B, p_stride,
                         s_stride, 0));
  mark(p, "enc_rows_codec", st);
  HIP_TRY(launch_codec_c(p->col_rep.C, p->col_rep.job, int(n - ks), p->col_rep.n_z,
                         p->col_rep.mode, st, B, s_stride, both_b, 0));
  mark(p, "enc_cols_rep_codec", st);
  if (!p->sys_fused)
    for (int b = 0; b < B; ++b)
      HIP_TRY(rs2k_launch_symbol_copy(d_primary + b * p_stride, p->sys_a_src.as<int64_t>(), ks * s,
                                      d_secondary + b * s_stride, p->sys_a_dst.as<int64_t>(), s,
                                      int(ks), int(kp), int(s), INT64_MAX, st));
  SymbolMap map{d_primary, d_secondary, p->batch_both.as<uint8_t>(), int(n), int(kp), int(ks),
                int(s), p_stride, s_stride, both_b, leaves_b};
  HIP_TRY(rs2k_launch_leaf_hash(map, 0, n * n, B, p->batch_leaves.as<uint8_t>(), st));
  mark(p, "enc_leaf_hash", st);
  if (const size_t sb = tree_scratch_bytes(2 * n, n)) {
    // trees wider than one wave's slab: a blob at a time through the plan's fold scratch
    // (launches on one stream, so the scratch is reused in order)
    HIP_TRY(p->tree_scratch.ensure(sb));
    for (int b = 0; b < B; ++b)
      HIP_TRY(rs2k_launch_merkle_trees(p->batch_leaves.as<uint8_t>() + b * leaves_b, int(n),
                                       int(n), int(n), n * 32, 32, 32, n * 32, d_hashes + b * n * 64,
                                       64, st, nullptr, 0, 1, 0, 0, p->tree_scratch.as<uint8_t>()));
  } else {
    HIP_TRY(rs2k_launch_merkle_trees(p->batch_leaves.as<uint8_t>(), int(n), int(n), int(n), n * 32,
                                     32, 32, n * 32, d_hashes, 64, st, nullptr, 0, B, leaves_b,
                                     n * 64));
  }
  mark(p, "enc_merkle_trees", st);
  HIP_TRY(rs2k_launch_merkle_root(d_hashes, int(n), p->blob_len, d_blob_ids, st, B, d_lens));
  mark(p, "enc_merkle_root", st);
  HIP_TRY(hipEventRecord(p->enc_done, st));
  return RS2_OK;
}

// Select the slivers a BlobDecoder would use (blob_encoding.rs:904-951): walk the input in
// order, stop once `need` slivers are taken (the item that finds the workspace full has been
// pulled from the iterator: it still counts for the Default check, config.rs:621-640), skip a
// repeated index, drop a sliver of the wrong length or symbol size (lens / sym_sizes may be
// null).  An index >= n_shards is taken like any other -- the reference's BTreeSet accepts any
// u16 -- and makes the column decodes fail with NotEnoughShards later (basic_encoding.rs:
// 400-410: reed-solomon-simd rejects the shard, the error is ignored, decode() then has too
// few).  *pulled = number of input slivers consumed.
int select_slivers(const rs2_plan* p, int axis, uint32_t count, const uint16_t* idx,
                   const uint64_t* lens, const uint16_t* sym_sizes,
                   std::vector<std::pair<uint16_t, uint32_t>>& chosen, uint32_t* pulled = nullptr) {
  const uint32_t need = axis == RS2_AXIS_PRIMARY ? p->kp : p->ks;
  const uint64_t want_len = uint64_t(axis == RS2_AXIS_PRIMARY ? primary_len(p) : secondary_len(p));
  std::vector<uint8_t> seen(65536, 0);
  chosen.clear();
  uint32_t i = 0;
  for (; i < count; ++i) {
    if (chosen.size() == need) {
      ++i;  // pulled, then dropped as surplus
      break;
    }
    const uint16_t q = idx[i];
    if (seen[q]) continue;
    if (lens && lens[i] != want_len) continue;
    if (sym_sizes && sym_sizes[i] != p->s) continue;
    seen[q] = 1;
    chosen.emplace_back(q, i);
  }
  if (pulled) *pulled = std::min(i, count);
  if (chosen.size() != need) return fail(RS2_E_DECODING_UNSUCCESSFUL, "not enough slivers");
  for (const auto& c : chosen)
    if (c.first >= p->n) return fail(RS2_E_NOT_ENOUGH_SHARDS, "not enough shards (sliver index out of range)");
  return RS2_OK;
}

// Decode from chosen device slivers: sliver i at base + off[i].
int decode_device(rs2_plan* p, int axis, const std::vector<std::pair<uint16_t, uint32_t>>& chosen,
                  const uint8_t* base, const uint64_t* off, uint8_t* d_out, hipStream_t st) {
  const int64_t s = p->s, n = p->n, kp = p->kp, ks = p->ks;
  const bool prim = axis == RS2_AXIS_PRIMARY;
  const uint32_t K = prim ? uint32_t(kp) : uint32_t(ks);
  const int slot = p->dec_slot;
  p->dec_slot ^= 1;
  const auto wait_t0 = std::chrono::steady_clock::now();
  if (p->dec_done[slot]) HIP_TRY(hipEventSynchronize(p->dec_done[slot]));
  prof_host(p, "dec_host_slotwait", wait_t0);
  DecodeSpec sp;
  sp.K = K;
  sp.R = uint32_t(n) - K;
  sp.symbol_size = int(s);
  sp.present.assign(n, -1);
  sp.src_base = base;
  sp.src_ls = s;  // line = column c (primary) / row r (secondary): symbol c of the sliver
  sp.dst_base = d_out;
  sp.dst_limit = int64_t(p->blob_len);
  sp.dst.resize(K);
  for (uint32_t i = 0; i < K; ++i) sp.dst[i] = prim ? int64_t(i) * ks * s : int64_t(i) * s;
  sp.dst_ls = prim ? s : ks * s;
  std::vector<int64_t>& copy_src = p->dec_copy_src_h[slot];
  std::vector<int64_t>& copy_dst = p->dec_copy_dst_h[slot];
  copy_src.clear();
  copy_dst.clear();
  for (auto& c : chosen) {
    sp.present[c.first] = int64_t(off[c.second]);
    if (c.first < K) {
      copy_src.push_back(int64_t(off[c.second]));
      copy_dst.push_back(sp.dst[c.first]);
    }
  }
  mark(p, "", st);
  const bool run_codec = copy_src.size() < K;
  PlannedJob& pj = p->dec_job[slot];
  std::vector<int64_t> key;
  key.reserve(size_t(n) + 4);
  key.push_back(axis);
  key.push_back(int64_t(block_max()));
  key.push_back(int64_t(p->blob_len));  // sp.dst_limit: rebind keeps the plan, not the limit
  key.push_back(int64_t(reinterpret_cast<uintptr_t>(base)));
  key.push_back(int64_t(reinterpret_cast<uintptr_t>(d_out)));
  key.insert(key.end(), sp.present.begin(), sp.present.end());
  const bool cached = key == p->dec_key[slot];
  p->dec_key[slot].clear();  // valid again only once this call has re-planned successfully
  bool fused = cached && p->dec_fused[slot];
  const auto host_t0 = std::chrono::steady_clock::now();
  if (run_codec && !cached) {
    // present originals are written by the decode kernel from its own loads when it can
    static const bool no_fuse = [] {  // A/B knob: RS2_DEC_NOFUSE=1
      const char* e = std::getenv("RS2_DEC_NOFUSE");
      return e && std::atoi(e) != 0;
    }();
    sp.copy_present = !copy_src.empty() && s >= 4 && !no_fuse;
    int rc = plan_decode(sp, pj);
    if (rc != RS2_OK) return rc;
    fused = sp.copy_present && copy_covered(pj);
    prof_host(p, "dec_host_plan", host_t0);
  }
  // present originals: straight copies into the blob (when not fused into the decode)
  if (!copy_src.empty() && !fused) {
    if (!cached) {
      HIP_TRY(p->dec_copy_src[slot].ensure(copy_src.size() * 8));
      HIP_TRY(p->dec_copy_dst[slot].ensure(copy_dst.size() * 8));
      HIP_TRY(p->ctx->upload(p->dec_copy_src[slot].p, copy_src.data(), copy_src.size() * 8, st));
      HIP_TRY(p->ctx->upload(p->dec_copy_dst[slot].p, copy_dst.data(), copy_dst.size() * 8, st));
    }
    const int count_b = prim ? int(ks) : int(kp);
    HIP_TRY(rs2k_launch_symbol_copy(base, p->dec_copy_src[slot].as<int64_t>(), s, d_out,
                                    p->dec_copy_dst[slot].as<int64_t>(), prim ? s : ks * s,
                                    int(copy_src.size()), count_b, int(s), int64_t(p->blob_len),
                                    st));
    mark(p, "dec_copy_present", st);
  }
  if (run_codec) {
    if (!cached) {
      const auto bind_t0 = std::chrono::steady_clock::now();
      // (on st, behind its wait for the slivers: the same setup on a stream of its own, so the
      // decode starts the moment the primary slivers are final, measured 81.8 vs 87.4 GiB/s --
      // a decode that takes the CUs earlier delays the encode's chain)
      int rc = bind_decode(p->ctx, pj, p->dec_mem[slot], st);
      if (rc != RS2_OK) return rc;
      prof_host(p, "dec_host_bind", bind_t0);
      prof_host(p, "dec_plan_host", host_t0);
    }
    mark(p, "dec_setup", st);
    const int lines = prim ? int(ks) : int(kp);
    HIP_TRY(pj.launch(lines, st));
    mark(p, "dec_codec", st);
  }
  if (!p->dec_done[slot]) HIP_TRY(hipEventCreateWithFlags(&p->dec_done[slot], hipEventDisableTiming));
  HIP_TRY(hipEventRecord(p->dec_done[slot], st));
  p->dec_key[slot] = std::move(key);
  p->dec_fused[slot] = fused;
  return RS2_OK;
}

// Stream argument of the plan / verifier ABI: NULL = the object's own stream,
// RS2_STREAM_LEGACY ((void*)1) = the HIP null stream (torch's default stream), else a
// hipStream_t.
hipStream_t abi_stream(void* stream, hipStream_t own) {
  if (!stream) return own;
  if (stream == RS2_STREAM_LEGACY) return nullptr;
  return reinterpret_cast<hipStream_t>(stream);
}

hipStream_t pick_stream(rs2_plan* p, void* stream) {
  return abi_stream(stream, p->stream);
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

int rs2_source_symbols_for_n_shards(uint16_t n_shards, uint16_t* n_primary, uint16_t* n_secondary) {
  if (n_shards == 0 || !n_primary || !n_secondary)
    return fail(RS2_E_INVALID_ARGUMENT, "n_shards must be non-zero");
  const uint16_t f = uint16_t((n_shards - 1) / 3);
  *n_secondary = uint16_t(n_shards - f);
  *n_primary = uint16_t(n_shards - 2 * f);
  return RS2_OK;
}

int rs2_symbol_size_for_blob(uint16_t n_shards, uint64_t blob_len, uint16_t* symbol_size) {
  uint16_t kp, ks;
  int rc = rs2_source_symbols_for_n_shards(n_shards, &kp, &ks);
  if (rc != RS2_OK) return rc;
  const uint64_t n_sym = uint64_t(kp) * ks;
  const uint64_t len = std::max<uint64_t>(blob_len, 1);
  uint64_t sz = (len + n_sym - 1) / n_sym;
  sz = (sz + 1) / 2 * 2;
  if (sz > 0xFFFF) return fail(RS2_E_DATA_TOO_LARGE, "blob too large for the symbol size");
  *symbol_size = uint16_t(sz);
  return RS2_OK;
}

int rs2_encoded_blob_length(uint16_t n_shards, uint64_t blob_len, uint64_t* encoded_len) {
  uint16_t kp, ks, s;
  int rc = rs2_source_symbols_for_n_shards(n_shards, &kp, &ks);
  if (rc != RS2_OK) return rc;
  rc = rs2_symbol_size_for_blob(n_shards, blob_len, &s);
  if (rc != RS2_OK) return rc;
  const uint64_t slivers = uint64_t(n_shards) * (uint64_t(kp) + ks) * s;
  const uint64_t meta = uint64_t(n_shards) * (uint64_t(n_shards) * 64 + 32);
  *encoded_len = slivers + meta;
  return RS2_OK;
}

int rs2_set_device(int device) {
  g_device = device;
  return RS2_OK;
}

const char* rs2_last_error(void) { return g_last_error.c_str(); }

int rs2_device_available(void) {
  int n = 0;
  return (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
}

int rs2_set_block_limit(uint32_t max_block) {
  if (max_block < 1 || max_block > uint32_t(kMaxC) || (max_block & (max_block - 1)))
    return fail(RS2_E_INVALID_ARGUMENT, "block limit must be a power of two <= 512");
  g_block_max.store(max_block, std::memory_order_relaxed);
  return RS2_OK;
}

int rs2_plan_create(uint16_t n_shards, uint64_t blob_len, rs2_plan** out) {
  if (!out) return fail(RS2_E_INVALID_ARGUMENT, "null plan pointer");
  *out = nullptr;
  uint16_t kp, ks, s;
  int rc = rs2_source_symbols_for_n_shards(n_shards, &kp, &ks);
  if (rc != RS2_OK) return rc;
  rc = rs2_symbol_size_for_blob(n_shards, blob_len, &s);
  if (rc != RS2_OK) return rc;
  if (kp == n_shards || ks == n_shards)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "n_shards too small for a recovery code");
  if (n_shards > kMaxShards) return fail(RS2_E_UNSUPPORTED, "n_shards above 65535");
  Context* ctx = nullptr;
  rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  auto p = std::make_unique<rs2_plan>();
  p->ctx = ctx;
  p->n = n_shards;
  p->kp = kp;
  p->ks = ks;
  p->s = s;
  p->blob_len = blob_len;
  HIP_TRY(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&p->fork_ev, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&p->join_ev, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&p->copy_ev, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&p->leaf_ev, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&p->enc_done, hipEventDisableTiming));
  const int64_t n = n_shards;
  HIP_TRY(p->both.ensure(size_t(n - kp) * (n - ks) * s));
  HIP_TRY(p->leaves.ensure(size_t(n) * n * 32));
  HIP_TRY(p->pairs.ensure(size_t(n) * 64));
  HIP_TRY(p->blob_id.ensure(32));
  // systematic secondary copy offsets: a = column c
  std::vector<int64_t> sa(ks), da(ks);
  for (int64_t c = 0; c < ks; ++c) {
    sa[c] = c * s;
    da[c] = c * kp * s;
  }
  HIP_TRY(p->sys_a_src.ensure(sa.size() * 8));
  HIP_TRY(p->sys_a_dst.ensure(da.size() * 8));
  HIP_TRY(hipMemcpy(p->sys_a_src.p, sa.data(), sa.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(p->sys_a_dst.p, da.data(), da.size() * 8, hipMemcpyHostToDevice));
  *out = p.release();
  return RS2_OK;
}

int rs2_plan_info_get(const rs2_plan* plan, rs2_plan_info* info) {
  if (!plan || !info) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  info->n_shards = plan->n;
  info->n_primary = plan->kp;
  info->n_secondary = plan->ks;
  info->symbol_size = plan->s;
  info->blob_len = plan->blob_len;
  info->primary_sliver_len = uint64_t(primary_len(plan));
  info->secondary_sliver_len = uint64_t(secondary_len(plan));
  return RS2_OK;
}

void rs2_plan_destroy(rs2_plan* plan) {
  if (!plan) return;
  (void)hipSetDevice(plan->ctx->device);
  // every stream and event the plan's work may still run behind (no device-wide synchronize):
  // its buffers then go straight back to the device arena for the next plan
  for (hipStream_t st : {plan->stream, plan->side, plan->side_hi, plan->aux, plan->io})
    if (st) (void)hipStreamSynchronize(st);
  for (hipEvent_t ev : {plan->enc_done, plan->dec_done[0], plan->dec_done[1], plan->leaf_ev})
    if (ev) (void)hipEventSynchronize(ev);
  const bool prev = t_quiesced;
  t_quiesced = true;
  delete plan;
  t_quiesced = prev;
}

int rs2_plan_rebind(rs2_plan* plan, uint64_t blob_len) {
  if (!plan) return fail(RS2_E_INVALID_ARGUMENT, "null plan");
  uint16_t s = 0;
  const int rc = rs2_symbol_size_for_blob(plan->n, blob_len, &s);
  if (rc != RS2_OK) return rc;
  if (s != plan->s)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "blob length needs another symbol size than the plan's");
  plan->blob_len = blob_len;
  return RS2_OK;
}

int rs2_host_register(void* ptr, uint64_t len) {
  if (!ptr || !len) return fail(RS2_E_INVALID_ARGUMENT, "null or empty range");
  const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.lower_bound(p);
  if (it != g_reg.end() && it->first < p + len)
    return fail(RS2_E_INVALID_ARGUMENT, "range overlaps a registered range");
  if (it != g_reg.begin() && std::prev(it)->first + std::prev(it)->second > p)
    return fail(RS2_E_INVALID_ARGUMENT, "range overlaps a registered range");
  HIP_TRY(hipHostRegister(ptr, size_t(len), hipHostRegisterPortable));
  g_reg.emplace(p, size_t(len));
  return RS2_OK;
}

int rs2_host_unregister(void* ptr) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_reg.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == g_reg.end()) return fail(RS2_E_INVALID_ARGUMENT, "pointer was not registered");
  g_reg.erase(it);
  HIP_TRY(hipHostUnregister(ptr));
  return RS2_OK;
}

int rs2_device_memory_stats(int device, uint64_t* stats_out) {
  if (!stats_out) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  DevArena& a = dev_arena(device);
  std::lock_guard<std::mutex> lk(a.mu);
  stats_out[0] = a.mallocs;
  stats_out[1] = a.frees;
  stats_out[2] = uint64_t(a.live);
  stats_out[3] = a.reserved;
  stats_out[4] = uint64_t(a.peak);
  stats_out[5] = a.syncs;
  stats_out[6] = g_pinned_allocs.load(std::memory_order_relaxed);
  return RS2_OK;
}

int rs2_upload_stats(uint64_t* stats_out) {
  if (!stats_out) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  stats_out[0] = g_upload_calls.load(std::memory_order_relaxed);
  stats_out[1] = g_upload_jobs.load(std::memory_order_relaxed);
  stats_out[2] = g_upload_waits.load(std::memory_order_relaxed);
  return RS2_OK;
}

int rs2_device_memory_trim(int device, uint64_t* released_bytes) {
  if (released_bytes) *released_bytes = 0;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(RS2_E_INVALID_ARGUMENT, "bad device");
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(device));
  const hipError_t e = dev_arena(device).trim(released_bytes);
  (void)hipSetDevice(prev);
  HIP_TRY(e);
  return RS2_OK;
}

int rs2_encode_device_async(rs2_plan* plan, const void* d_blob, void* d_primary, void* d_secondary,
                            void* d_hashes, void* d_blob_id, void* stream) {
  if (!plan || !d_primary || !d_secondary || (!d_blob && plan->blob_len))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  return encode_device(plan, reinterpret_cast<const uint8_t*>(d_blob),
                       reinterpret_cast<uint8_t*>(d_primary), reinterpret_cast<uint8_t*>(d_secondary),
                       reinterpret_cast<uint8_t*>(d_hashes), reinterpret_cast<uint8_t*>(d_blob_id),
                       pick_stream(plan, stream), true);
}

int rs2_compute_metadata_device_async(rs2_plan* plan, const void* d_blob, void* d_hashes,
                                      void* d_blob_id, void* stream) {
  if (!plan || !d_hashes || !d_blob_id || (!d_blob && plan->blob_len))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  const int64_t n = plan->n;
  HIP_TRY(plan->int_primary.ensure(size_t(n) * primary_len(plan)));
  HIP_TRY(plan->int_secondary.ensure(size_t(n) * secondary_len(plan)));
  return encode_device(plan, reinterpret_cast<const uint8_t*>(d_blob),
                       plan->int_primary.as<uint8_t>(), plan->int_secondary.as<uint8_t>(),
                       reinterpret_cast<uint8_t*>(d_hashes), reinterpret_cast<uint8_t*>(d_blob_id),
                       pick_stream(plan, stream), false);
}

int rs2_encode_device_split_async(rs2_plan* plan, const void* d_blob, void* d_primary,
                                  void* d_secondary, void* d_hashes, void* d_blob_id, void* stream,
                                  void* primary_stream) {
  if (!plan || !d_primary || !d_secondary || (!d_blob && plan->blob_len) || !primary_stream)
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  hipStream_t st = pick_stream(plan, stream);
  hipStream_t pst = abi_stream(primary_stream, nullptr);
  if (pst == st || pst == plan->side || pst == plan->side_hi)
    return fail(RS2_E_INVALID_ARGUMENT, "primary_stream must differ from stream");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  return encode_device(plan, reinterpret_cast<const uint8_t*>(d_blob),
                       reinterpret_cast<uint8_t*>(d_primary), reinterpret_cast<uint8_t*>(d_secondary),
                       reinterpret_cast<uint8_t*>(d_hashes), reinterpret_cast<uint8_t*>(d_blob_id),
                       st, true, pst);
}

int rs2_decode_device_async(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                            const void* d_slivers_base, const uint64_t* sliver_off,
                            void* d_blob_out, void* stream) {
  if (!plan || !sliver_idx || !sliver_off || !d_slivers_base || !d_blob_out)
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (axis != RS2_AXIS_PRIMARY && axis != RS2_AXIS_SECONDARY)
    return fail(RS2_E_INVALID_ARGUMENT, "bad axis");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  std::vector<std::pair<uint16_t, uint32_t>> chosen;
  int rc = select_slivers(plan, axis, count, sliver_idx, nullptr, nullptr, chosen);
  if (rc != RS2_OK) return rc;
  return decode_device(plan, axis, chosen, reinterpret_cast<const uint8_t*>(d_slivers_base),
                       sliver_off, reinterpret_cast<uint8_t*>(d_blob_out), pick_stream(plan, stream));
}

int rs2_profile_enable(rs2_plan* plan, int enable) {
  if (!plan) return fail(RS2_E_INVALID_ARGUMENT, "null plan");
  plan->prof.on = enable != 0;
  return RS2_OK;
}

int rs2_profile_read(rs2_plan* plan, uint32_t max_stages, char* names, double* total_ms,
                     uint32_t* launches, uint32_t* n_stages) {
  if (!plan || !n_stages) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  (void)hipSetDevice(plan->ctx->device);
  prof_collect(plan);
  auto& pr = plan->prof;
  uint32_t k = 0;
  for (const auto& name : pr.order) {
    if (k >= max_stages) break;
    const auto& v = pr.acc[name];
    if (names) {
      std::memset(names + 32 * size_t(k), 0, 32);
      std::strncpy(names + 32 * size_t(k), name.c_str(), 31);
    }
    if (total_ms) total_ms[k] = v.first;
    if (launches) launches[k] = v.second;
    ++k;
  }
  *n_stages = k;
  pr.acc.clear();
  pr.order.clear();
  return RS2_OK;
}

int rs2_sync(rs2_plan* plan, void* stream) {
  if (!plan) return fail(RS2_E_INVALID_ARGUMENT, "null plan");
  HIP_TRY(hipStreamSynchronize(pick_stream(plan, stream)));
  return RS2_OK;
}

namespace {
// a pinned ring leased to `plan` for one host-buffer call
struct RingGuard {
  rs2_plan* p;
  StagerLease lease;
  explicit RingGuard(rs2_plan* plan) : p(plan), lease(plan->ctx->device) { p->stage = lease.st.get(); }
  ~RingGuard() {
    // the ring's slot events were recorded on this plan's streams, which may be destroyed before
    // the next lease waits on them: drain them and move them to the context's stream
    for (hipEvent_t ev : lease.st->ev)
      if (ev) {
        (void)hipEventSynchronize(ev);
        (void)hipEventRecord(ev, p->ctx->util_stream);
      }
    p->stage = nullptr;
  }
};
}  // namespace

int rs2_encode_with_metadata(rs2_plan* plan, const uint8_t* blob, uint8_t* const* primary_out,
                             uint8_t* const* secondary_out, uint8_t* hashes_out,
                             uint8_t* blob_id_out) {
  if (!plan || (!blob && plan->blob_len)) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  RingGuard ring(plan);
  Context* ctx = plan->ctx;
  const int64_t n = plan->n, pl = primary_len(plan), sl = secondary_len(plan);
  // the message size (not blob_len): a plan rebound to another length of its symbol size keeps it
  HIP_TRY(plan->dev_blob.ensure(std::max<uint64_t>(uint64_t(plan->kp) * plan->ks * plan->s, 16)));
  HIP_TRY(plan->int_primary.ensure(size_t(n) * pl));
  HIP_TRY(plan->int_secondary.ensure(size_t(n) * sl));
  if (!plan->io) HIP_TRY(hipStreamCreateWithFlags(&plan->io, hipStreamNonBlocking));
  hipStream_t st = plan->stream, io = plan->io;
  int rc = RS2_OK;
  // the blob in through the pinned ring (host copies of piece k+1 under the DMA of piece k)
  if (plan->blob_len &&
      (rc = stage_h2d(ctx, *plan->stage, {{const_cast<uint8_t*>(blob), plan->dev_blob.as<uint8_t>(),
                                          size_t(plan->blob_len)}}, st)) != RS2_OK)
    return rc;
  uint8_t* dp = plan->int_primary.as<uint8_t>();
  uint8_t* ds = plan->int_secondary.as<uint8_t>();
  const bool slivers = primary_out || secondary_out;
  // split encode: `io` is released once the primary slivers are final, so their D2H overlaps the
  // secondary codecs and the hashing still running on st
  rc = encode_device(plan, plan->dev_blob.as<uint8_t>(), dp, ds, plan->pairs.as<uint8_t>(),
                     plan->blob_id.as<uint8_t>(), st, slivers, slivers ? io : nullptr);
  if (rc != RS2_OK) return rc;
  std::vector<Seg> segs;
  for (int64_t i = 0; primary_out && i < n; ++i)
    if (primary_out[i]) segs.push_back({primary_out[i], dp + i * pl, size_t(pl)});
  if (!segs.empty() && (rc = stage_d2h(ctx, *plan->stage, segs, io)) != RS2_OK) return rc;
  segs.clear();
  for (int64_t i = 0; secondary_out && i < n; ++i)
    if (secondary_out[i]) segs.push_back({secondary_out[i], ds + i * sl, size_t(sl)});
  if (hashes_out) segs.push_back({hashes_out, plan->pairs.as<uint8_t>(), size_t(n) * 64});
  if (blob_id_out) segs.push_back({blob_id_out, plan->blob_id.as<uint8_t>(), 32});
  HIP_TRY(hipStreamWaitEvent(io, plan->enc_done, 0));
  if (!segs.empty() && (rc = stage_d2h(ctx, *plan->stage, segs, io)) != RS2_OK) return rc;
  HIP_TRY(hipStreamSynchronize(io));
  HIP_TRY(hipStreamSynchronize(st));
  return RS2_OK;
}

int rs2_compute_metadata(rs2_plan* plan, const uint8_t* blob, uint8_t* hashes_out,
                         uint8_t* blob_id_out) {
  return rs2_encode_with_metadata(plan, blob, nullptr, nullptr, hashes_out, blob_id_out);
}

int rs2_encode_batch_device_async(rs2_plan* plan, uint32_t n_blobs, const void* d_blobs,
                                  uint64_t blob_stride, const uint64_t* blob_lens, void* d_primary,
                                  uint64_t primary_stride, void* d_secondary,
                                  uint64_t secondary_stride, void* d_hashes, void* d_blob_ids,
                                  void* stream) {
  if (!plan) return fail(RS2_E_INVALID_ARGUMENT, "null plan");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  return encode_batch_device(plan, n_blobs, reinterpret_cast<const uint8_t*>(d_blobs),
                             int64_t(blob_stride), blob_lens, reinterpret_cast<uint8_t*>(d_primary),
                             int64_t(primary_stride), reinterpret_cast<uint8_t*>(d_secondary),
                             int64_t(secondary_stride), reinterpret_cast<uint8_t*>(d_hashes),
                             reinterpret_cast<uint8_t*>(d_blob_ids), pick_stream(plan, stream));
}

int rs2_encode_batch_with_metadata(rs2_plan* plan, uint32_t n_blobs, const uint8_t* const* blobs,
                                   const uint64_t* blob_lens, uint8_t* const* primary_out,
                                   uint8_t* const* secondary_out, uint8_t* hashes_out,
                                   uint8_t* blob_ids_out) {
  if (!plan) return fail(RS2_E_INVALID_ARGUMENT, "null plan");
  if (n_blobs == 0) return RS2_OK;
  if (n_blobs > 65535) return fail(RS2_E_INVALID_ARGUMENT, "more than 65535 blobs in a batch");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  RingGuard ring(plan);
  Context* ctx = plan->ctx;
  const int64_t n = plan->n, pl = primary_len(plan), sl = secondary_len(plan);
  const size_t B = n_blobs;
  uint64_t max_len = 0;
  for (size_t b = 0; b < B; ++b) {
    const uint64_t len = blob_lens ? blob_lens[b] : plan->blob_len;
    if (len && (!blobs || !blobs[b])) return fail(RS2_E_INVALID_ARGUMENT, "null blob");
    max_len = std::max(max_len, len);
  }
  const int64_t bstride = int64_t((std::max<uint64_t>(max_len, 1) + 255) / 256 * 256);
  HIP_TRY(plan->batch_blob.ensure(B * size_t(bstride)));
  HIP_TRY(plan->batch_primary.ensure(B * size_t(n * pl)));
  HIP_TRY(plan->batch_secondary.ensure(B * size_t(n * sl)));
  HIP_TRY(plan->batch_hashes.ensure(B * size_t(n) * 64));
  HIP_TRY(plan->batch_ids.ensure(B * 32));
  hipStream_t st = plan->stream;
  uint8_t* db = plan->batch_blob.as<uint8_t>();
  uint8_t* dp = plan->batch_primary.as<uint8_t>();
  uint8_t* ds = plan->batch_secondary.as<uint8_t>();
  uint8_t* dh = plan->batch_hashes.as<uint8_t>();
  uint8_t* di = plan->batch_ids.as<uint8_t>();
  std::vector<Seg> segs;
  for (size_t b = 0; b < B; ++b) {
    const uint64_t len = blob_lens ? blob_lens[b] : plan->blob_len;
    if (len) segs.push_back({const_cast<uint8_t*>(blobs[b]), db + b * bstride, size_t(len)});
  }
  int rc = stage_h2d(ctx, *plan->stage, segs, st);
  if (rc != RS2_OK) return rc;
  rc = encode_batch_device(plan, n_blobs, db, bstride, blob_lens, dp, n * pl, ds, n * sl, dh, di, st);
  if (rc != RS2_OK) return rc;
  segs.clear();
  for (size_t b = 0; b < B; ++b)
    for (int64_t i = 0; i < n; ++i) {
      if (primary_out && primary_out[b * n + i])
        segs.push_back({primary_out[b * n + i], dp + (b * n + i) * pl, size_t(pl)});
      if (secondary_out && secondary_out[b * n + i])
        segs.push_back({secondary_out[b * n + i], ds + (b * n + i) * sl, size_t(sl)});
    }
  if (hashes_out) segs.push_back({hashes_out, dh, B * size_t(n) * 64});
  if (blob_ids_out) segs.push_back({blob_ids_out, di, B * 32});
  if (!segs.empty() && (rc = stage_d2h(ctx, *plan->stage, segs, st)) != RS2_OK) return rc;
  HIP_TRY(hipStreamSynchronize(st));
  return RS2_OK;
}

namespace {

// Host slivers -> decoded blob in plan->dev_blob (blob_len bytes, zero up to the K_p*K_s*s
// message size so its rows are the zero-padded systematic primary slivers), enqueued on the
// plan stream.  *pulled: input slivers consumed (select_slivers).
int decode_host(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                const uint8_t* const* slivers, const uint64_t* sliver_len,
                const uint16_t* sliver_symbol_size, uint32_t* pulled) {
  if (count && (!sliver_idx || !slivers || !sliver_len))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (axis != RS2_AXIS_PRIMARY && axis != RS2_AXIS_SECONDARY)
    return fail(RS2_E_INVALID_ARGUMENT, "bad axis");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  std::vector<std::pair<uint16_t, uint32_t>> chosen;
  int rc = select_slivers(plan, axis, count, sliver_idx, sliver_len, sliver_symbol_size, chosen,
                          pulled);
  if (rc != RS2_OK) return rc;
  for (const auto& c : chosen)
    if (!slivers[c.second]) return fail(RS2_E_INVALID_ARGUMENT, "null sliver");
  const int64_t len = axis == RS2_AXIS_PRIMARY ? primary_len(plan) : secondary_len(plan);
  const int64_t msg = int64_t(plan->kp) * plan->ks * plan->s;
  hipStream_t st = plan->stream;
  // the chosen slivers, back to back on the device, through the pinned ring
  DevBuf& stage = axis == RS2_AXIS_PRIMARY ? plan->int_primary : plan->int_secondary;
  HIP_TRY(stage.ensure(size_t(plan->n) * len));  // the encoder's size: never re-allocated
  std::vector<uint64_t> off(count, 0);
  std::vector<Seg> segs;
  for (size_t i = 0; i < chosen.size(); ++i) {
    off[chosen[i].second] = uint64_t(i) * len;
    segs.push_back({const_cast<uint8_t*>(slivers[chosen[i].second]),
                    stage.as<uint8_t>() + i * len, size_t(len)});
  }
  HIP_TRY(plan->dev_blob.ensure(size_t(std::max<int64_t>(msg, 16))));
  if ((rc = stage_h2d(plan->ctx, *plan->stage, segs, st)) != RS2_OK) return rc;
  if (uint64_t(msg) > plan->blob_len)
    HIP_TRY(hipMemsetAsync(plan->dev_blob.as<uint8_t>() + plan->blob_len, 0,
                           size_t(msg - plan->blob_len), st));
  return decode_device(plan, axis, chosen, stage.as<uint8_t>(), off.data(),
                       plan->dev_blob.as<uint8_t>(), st);
}

// Default consistency check (blob_encoding.rs:579-612) on a decoded blob on the device (`blob`,
// `blob_valid` bytes of it written: plan->dev_blob of the host path holds the whole zero-padded
// message, a caller's device buffer only blob_len bytes): every systematic primary sliver
// i < K_p not marked in `verified` is re-expanded with the secondary code, its n symbols
// leaf-hashed and Merkle-reduced on the device, and the root compared with the metadata's
// primary hash of pair i.
int default_check(rs2_plan* plan, const std::vector<uint8_t>& verified, const uint8_t* hashes,
                  const uint8_t* blob, int64_t blob_valid, hipStream_t st) {
  const int64_t kp = plan->kp, ks = plan->ks, s = plan->s, row = ks * s;
  std::vector<uint16_t> rows;
  for (int64_t i = 0; i < kp; ++i)
    if (!verified[size_t(i)]) rows.push_back(uint16_t(i));
  if (rows.empty()) return RS2_OK;
  if (!plan->check_v) {
    int rc = rs2_verifier_create(plan->n, plan->s, RS2_AXIS_PRIMARY, &plan->check_v);
    if (rc != RS2_OK) return rc;
  }
  const uint8_t* src = blob;
  // rows past the written bytes (the zero-padded tail of the message) are rebuilt in the gather
  // buffer: zeros, then the row's written prefix
  std::vector<size_t> partial;
  for (size_t a = 0; a < rows.size(); ++a)
    if (int64_t(rows[a] + 1) * row > blob_valid) partial.push_back(a);
  if (int64_t(rows.size()) < kp || !partial.empty()) {  // gather the unverified rows back to back
    plan->check_src_h.assign(rows.size(), 0);
    for (size_t a = 0; a < rows.size(); ++a) plan->check_src_h[a] = int64_t(rows[a]) * row;
    HIP_TRY(plan->check_src.ensure(rows.size() * 8));
    HIP_TRY(plan->check_rows.ensure(rows.size() * size_t(row)));
    HIP_TRY(plan->ctx->upload(plan->check_src.p, plan->check_src_h.data(), rows.size() * 8, st));
    const int full = int(rows.size() - partial.size());  // partial rows are the last ones
    if (full > 0)  // row a of the gather buffer at a * row
      HIP_TRY(rs2k_launch_row_gather(src, plan->check_src.as<int64_t>(),
                                     plan->check_rows.as<uint8_t>(), row, full, st));
    for (size_t a : partial) {
      uint8_t* dst = plan->check_rows.as<uint8_t>() + a * row;
      HIP_TRY(hipMemsetAsync(dst, 0, size_t(row), st));
      const int64_t have = std::max<int64_t>(0, blob_valid - int64_t(rows[a]) * row);
      if (have > 0)
        HIP_TRY(hipMemcpyAsync(dst, src + int64_t(rows[a]) * row, size_t(have),
                               hipMemcpyDeviceToDevice, st));
    }
    src = plan->check_rows.as<uint8_t>();
  }
  HIP_TRY(plan->check_roots.ensure(rows.size() * 32));
  // (st nullptr is the HIP null stream here; at the ABI NULL would mean the verifier's own
  // stream, unordered with the decode that wrote `blob`)
  int rc = rs2_verifier_roots_device_async(plan->check_v, uint32_t(rows.size()), src,
                                           plan->check_roots.p,
                                           st ? static_cast<void*>(st) : RS2_STREAM_LEGACY);
  if (rc != RS2_OK) return rc;
  std::vector<uint8_t> roots(rows.size() * 32);
  HIP_TRY(hipMemcpyAsync(roots.data(), plan->check_roots.p, roots.size(), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (size_t a = 0; a < rows.size(); ++a)
    if (std::memcmp(roots.data() + 32 * a, hashes + 64 * size_t(rows[a]), 32) != 0)
      return fail(RS2_E_VERIFICATION, "primary sliver hash mismatch");
  return RS2_OK;
}

// Strict consistency check (config.rs:164-172): the metadata of the decoded blob (blob_len bytes
// on the device), re-derived on the device, must give the same blob id.
int strict_check(rs2_plan* plan, const uint8_t* blob_id, const uint8_t* blob, hipStream_t st) {
  const int64_t n = plan->n;
  HIP_TRY(plan->int_primary.ensure(size_t(n) * primary_len(plan)));
  HIP_TRY(plan->int_secondary.ensure(size_t(n) * secondary_len(plan)));
  int rc = encode_device(plan, blob, plan->int_primary.as<uint8_t>(),
                         plan->int_secondary.as<uint8_t>(), plan->pairs.as<uint8_t>(),
                         plan->blob_id.as<uint8_t>(), st, false);
  if (rc != RS2_OK) return rc;
  uint8_t bid[32];
  HIP_TRY(hipMemcpyAsync(bid, plan->blob_id.p, 32, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (std::memcmp(bid, blob_id, 32) != 0) return fail(RS2_E_VERIFICATION, "blob id mismatch");
  return RS2_OK;
}

int blob_to_host(rs2_plan* plan, uint8_t* blob_out) {
  if (plan->blob_len) {
    int rc = stage_d2h(plan->ctx, *plan->stage,
                       {{blob_out, plan->dev_blob.as<uint8_t>(), size_t(plan->blob_len)}},
                       plan->stream);
    if (rc != RS2_OK) return rc;
  }
  HIP_TRY(hipStreamSynchronize(plan->stream));
  return RS2_OK;
}

}  // namespace

int rs2_decode_blob(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                    const uint8_t* const* slivers, const uint64_t* sliver_len,
                    const uint16_t* sliver_symbol_size, uint8_t* blob_out) {
  if (!plan || (!blob_out && plan->blob_len)) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  RingGuard ring(plan);
  int rc = decode_host(plan, axis, count, sliver_idx, slivers, sliver_len, sliver_symbol_size,
                       nullptr);
  if (rc != RS2_OK) return rc;
  return blob_to_host(plan, blob_out);
}

int rs2_decode_and_verify(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                          const uint8_t* const* slivers, const uint64_t* sliver_len,
                          const uint16_t* sliver_symbol_size, const uint8_t* hashes,
                          const uint8_t* blob_id, int consistency_check, uint8_t* blob_out) {
  if (!plan || (!blob_out && plan->blob_len)) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (!hashes || !blob_id) return fail(RS2_E_INVALID_ARGUMENT, "null metadata");
  if (consistency_check != RS2_CHECK_SKIP && consistency_check != RS2_CHECK_DEFAULT &&
      consistency_check != RS2_CHECK_STRICT)
    return fail(RS2_E_INVALID_ARGUMENT, "bad consistency check");
  RingGuard ring(plan);
  uint32_t pulled = 0;
  int rc = decode_host(plan, axis, count, sliver_idx, slivers, sliver_len, sliver_symbol_size,
                       &pulled);
  if (rc != RS2_OK) return rc;
  if (consistency_check == RS2_CHECK_DEFAULT) {
    // config.rs:621-640: with primary slivers, every systematic index the decoder pulled from
    // the input counts as already verified (the caller verified each sliver on receipt); with
    // secondary slivers none does
    std::vector<uint8_t> verified(plan->kp, 0);
    if (axis == RS2_AXIS_PRIMARY)
      for (uint32_t i = 0; i < pulled; ++i)
        if (sliver_idx[i] < plan->kp) verified[sliver_idx[i]] = 1;
    rc = default_check(plan, verified, hashes, plan->dev_blob.as<uint8_t>(),
                       int64_t(plan->kp) * plan->ks * plan->s, plan->stream);
  } else if (consistency_check == RS2_CHECK_STRICT) {
    rc = strict_check(plan, blob_id, plan->dev_blob.as<uint8_t>(), plan->stream);
  }
  if (rc != RS2_OK) return rc;
  return blob_to_host(plan, blob_out);
}

int rs2_decode_and_verify_device(rs2_plan* plan, int axis, uint32_t count,
                                 const uint16_t* sliver_idx, const void* d_slivers_base,
                                 const uint64_t* sliver_off, const uint8_t* hashes,
                                 const uint8_t* blob_id, int consistency_check, void* d_blob_out,
                                 void* stream) {
  if (!plan || !sliver_idx || !sliver_off || !d_slivers_base || !d_blob_out)
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (!hashes || !blob_id) return fail(RS2_E_INVALID_ARGUMENT, "null metadata");
  if (axis != RS2_AXIS_PRIMARY && axis != RS2_AXIS_SECONDARY)
    return fail(RS2_E_INVALID_ARGUMENT, "bad axis");
  if (consistency_check != RS2_CHECK_SKIP && consistency_check != RS2_CHECK_DEFAULT &&
      consistency_check != RS2_CHECK_STRICT)
    return fail(RS2_E_INVALID_ARGUMENT, "bad consistency check");
  HIP_TRY(hipSetDevice(plan->ctx->device));
  std::vector<std::pair<uint16_t, uint32_t>> chosen;
  uint32_t pulled = 0;
  int rc = select_slivers(plan, axis, count, sliver_idx, nullptr, nullptr, chosen, &pulled);
  if (rc != RS2_OK) return rc;
  hipStream_t st = pick_stream(plan, stream);
  uint8_t* out = reinterpret_cast<uint8_t*>(d_blob_out);
  rc = decode_device(plan, axis, chosen, reinterpret_cast<const uint8_t*>(d_slivers_base),
                     sliver_off, out, st);
  if (rc != RS2_OK) return rc;
  if (consistency_check == RS2_CHECK_DEFAULT) {
    std::vector<uint8_t> verified(plan->kp, 0);  // as rs2_decode_and_verify
    if (axis == RS2_AXIS_PRIMARY)
      for (uint32_t i = 0; i < pulled; ++i)
        if (sliver_idx[i] < plan->kp) verified[sliver_idx[i]] = 1;
    rc = default_check(plan, verified, hashes, out, int64_t(plan->blob_len), st);
  } else if (consistency_check == RS2_CHECK_STRICT) {
    rc = strict_check(plan, blob_id, out, st);
  }
  if (rc != RS2_OK) return rc;
  HIP_TRY(hipStreamSynchronize(st));
  return RS2_OK;
}

int rs2_encode_1d(uint16_t k, uint16_t n_shards, uint16_t symbol_size, uint32_t batch,
                  const uint8_t* data, uint8_t* out_all) {
  if (!data || !out_all) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (symbol_size == 0 || symbol_size % 2)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "symbol_size must be a multiple of the required alignment");
  if (n_shards < k || k == 0)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "n_shards must be at least n_source_symbols");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  const int64_t s = symbol_size, K = k, N = n_shards;
  const size_t in_bytes = size_t(batch) * K * s, out_bytes = size_t(batch) * N * s;
  for (uint32_t b = 0; b < batch; ++b) std::memcpy(out_all + b * N * s, data + b * K * s, K * s);
  if (N == K || batch == 0) return RS2_OK;
  DevBuf din, dout;
  HIP_TRY(din.ensure(in_bytes));
  HIP_TRY(dout.ensure(out_bytes));
  hipStream_t st = ctx->util_stream;
  HIP_TRY(hipMemcpyAsync(din.p, data, in_bytes, hipMemcpyHostToDevice, st));
  PlannedJob pj;
  JobMem mem;
  rc = plan_encode(uint32_t(K), uint32_t(N - K), int(s), din.as<uint8_t>(), K * s,
                   [&](uint32_t i) { return int64_t(i) * s; }, dout.as<uint8_t>(), N * s,
                   [&](uint32_t j) { return (K + int64_t(j)) * s; }, INT64_MAX, pj);
  if (rc != RS2_OK) return rc;
  rc = bind_encode(ctx, pj, mem, st);
  if (rc != RS2_OK) return rc;
  HIP_TRY(pj.launch(int(batch), st));
  HIP_TRY(hipStreamSynchronize(st));
  for (uint32_t b = 0; b < batch; ++b)
    HIP_TRY(hipMemcpy(out_all + b * N * s + K * s, dout.as<uint8_t>() + b * N * s + K * s,
                      (N - K) * s, hipMemcpyDeviceToHost));
  return RS2_OK;
}

int rs2_decode_1d(uint16_t k, uint16_t n_shards, uint16_t symbol_size, uint32_t count,
                  const uint16_t* idx, const uint8_t* const* symbols, uint8_t* out_source) {
  if (!out_source || (count && (!idx || !symbols))) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (symbol_size == 0 || symbol_size % 2 || n_shards <= k || k == 0)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "incompatible parameters");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  const int64_t s = symbol_size, K = k, N = n_shards;
  std::vector<int64_t> present(N, -1);
  std::vector<uint32_t> order;
  for (uint32_t i = 0; i < count; ++i) {
    if (idx[i] >= N) continue;  // invalid indices are ignored by the crate
    if (present[idx[i]] >= 0) continue;
    present[idx[i]] = int64_t(order.size()) * s;
    order.push_back(i);
  }
  if (order.size() < size_t(K)) return fail(RS2_E_NOT_ENOUGH_SHARDS, "not enough shards");
  // any K shards determine the codeword; use the first K distinct ones
  for (size_t i = size_t(K); i < order.size(); ++i) present[idx[order[i]]] = -1;
  order.resize(size_t(K));
  bool all_src = true;
  for (int64_t i = 0; i < K; ++i) all_src &= present[i] >= 0;
  if (all_src) {
    for (int64_t i = 0; i < K; ++i) {
      const uint32_t src = order[size_t(present[i] / s)];
      std::memcpy(out_source + i * s, symbols[src], s);
    }
    return RS2_OK;
  }
  Dec1DLease lease(ctx, int(K), int(N), int(s));
  HIP_TRY(lease.get());
  Dec1D& D = *lease.d;
  DevBuf& din = D.din;
  DevBuf& dout = D.dout;
  HIP_TRY(din.ensure(order.size() * s));
  HIP_TRY(dout.ensure(K * s));
  hipStream_t st = D.st;
  // the symbols gathered into pinned staging: one DMA instead of K pageable copies
  HIP_TRY(D.hin.ensure(order.size() * s));
  HIP_TRY(D.hout.ensure(size_t(K) * s));
  for (size_t i = 0; i < order.size(); ++i)
    std::memcpy(static_cast<uint8_t*>(D.hin.p) + i * s, symbols[order[i]], s);
  HIP_TRY(hipMemcpyAsync(din.p, D.hin.p, order.size() * s, hipMemcpyHostToDevice, st));
  DecodeSpec sp;
  sp.K = uint32_t(K);
  sp.R = uint32_t(N - K);
  sp.symbol_size = int(s);
  sp.present = present;
  sp.src_base = din.as<uint8_t>();
  sp.src_ls = 0;
  sp.dst_base = dout.as<uint8_t>();
  sp.dst_ls = 0;
  sp.dst.resize(K);
  for (int64_t i = 0; i < K; ++i) sp.dst[i] = i * s;
  rc = plan_decode(sp, D.pj);
  if (rc != RS2_OK) return rc;
  rc = bind_decode(ctx, D.pj, D.mem, st);
  if (rc != RS2_OK) return rc;
  HIP_TRY(D.pj.launch(1, st));
  HIP_TRY(hipMemcpyAsync(D.hout.p, dout.p, size_t(K) * s, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint8_t* dec = static_cast<const uint8_t*>(D.hout.p);
  for (int64_t i = 0; i < K; ++i) {
    if (present[i] >= 0)
      std::memcpy(out_source + i * s, symbols[order[size_t(present[i] / s)]], s);
    else
      std::memcpy(out_source + i * s, dec + i * s, s);
  }
  return RS2_OK;
}

// ---- sliver verification, Merkle roots, blob ids: all hashing on the device ----------------

int rs2_verifier_create(uint16_t n_shards, uint16_t symbol_size, int axis, rs2_verifier** out) {
  if (!out) return fail(RS2_E_INVALID_ARGUMENT, "null verifier pointer");
  *out = nullptr;
  if (axis != RS2_AXIS_PRIMARY && axis != RS2_AXIS_SECONDARY)
    return fail(RS2_E_INVALID_ARGUMENT, "bad axis");
  if (symbol_size == 0 || symbol_size % 2)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "symbol_size must be a multiple of the required alignment");
  uint16_t kp, ks;
  int rc = rs2_source_symbols_for_n_shards(n_shards, &kp, &ks);
  if (rc != RS2_OK) return rc;
  if (n_shards > kMaxShards) return fail(RS2_E_UNSUPPORTED, "n_shards above 65535");
  Context* ctx = nullptr;
  rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  auto v = std::make_unique<rs2_verifier>();
  v->ctx = ctx;
  v->n = n_shards;
  v->k = axis == RS2_AXIS_PRIMARY ? ks : kp;  // a primary sliver expands with the secondary code
  v->s = symbol_size;
  v->axis = axis;
  HIP_TRY(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
  *out = v.release();
  return RS2_OK;
}

void rs2_verifier_destroy(rs2_verifier* v) {
  if (!v) return;
  (void)hipSetDevice(v->ctx->device);
  if (v->stream) (void)hipStreamSynchronize(v->stream);
  if (v->done) (void)hipEventSynchronize(v->done);  // work queued on a caller's stream
  const bool prev = t_quiesced;
  t_quiesced = true;
  delete v;
  t_quiesced = prev;
}

namespace {
// A pooled verifier for one host-buffer call (Context::verifier_pool); returned on scope exit
// with its stream drained (every host-buffer call synchronizes before returning).
struct VerifierLease {
  Context* ctx = nullptr;
  rs2_verifier* v = nullptr;
  VerifierLease() = default;
  VerifierLease(const VerifierLease&) = delete;
  VerifierLease& operator=(const VerifierLease&) = delete;
  int get(uint16_t n_shards, uint16_t symbol_size, int axis) {
    int rc = get_context(&ctx);
    if (rc != RS2_OK) return rc;
    {
      std::lock_guard<std::mutex> lk(ctx->pool_mu);
      auto& free_ = ctx->verifier_pool[std::make_tuple(int(n_shards), int(symbol_size), axis)];
      if (!free_.empty()) {
        v = free_.back();
        free_.pop_back();
        return RS2_OK;
      }
    }
    return rs2_verifier_create(n_shards, symbol_size, axis, &v);
  }
  ~VerifierLease() {
    if (!v) return;
    // drained before it goes back: an error return may leave the h_in -> input copy queued on
    // its stream, and the next holder rewrites h_in / grows it (PinnedBuf::ensure frees it)
    (void)hipStreamSynchronize(v->stream);
    if (v->done) (void)hipEventSynchronize(v->done);
    {
      std::lock_guard<std::mutex> lk(ctx->pool_mu);
      auto& free_ = ctx->verifier_pool[std::make_tuple(int(v->n), int(v->s), v->axis)];
      if (free_.size() < Context::kPoolKeep) {
        free_.push_back(v);
        return;
      }
    }
    rs2_verifier_destroy(v);
  }
};

// path length and node count of a MerkleTree over n leaves (merkle.rs path_length / n_nodes)
int merkle_path_len(uint64_t n) {
  int l = 0;
  while (n > 1) {
    n = (n + 1) / 2;
    ++l;
  }
  return l;
}
uint64_t merkle_n_nodes(uint64_t n) {
  uint64_t tot = 0;
  while (n > 1) {
    n += n & 1;
    tot += n;
    n /= 2;
  }
  return tot + n;
}

// Expand `count` back-to-back slivers on the orthogonal axis (their n - k repair symbols each,
// in v->repair) and leaf-hash all n symbols of each (v->leaves), on st.
int verifier_leaves(rs2_verifier* v, uint32_t count, const uint8_t* din, hipStream_t st);

// the verifier's last work on st (any caller stream): rs2_verifier_destroy waits for it
int verifier_mark_done(rs2_verifier* v, hipStream_t st) {
  if (!v->done) HIP_TRY(hipEventCreateWithFlags(&v->done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(v->done, st));
  return RS2_OK;
}
}  // namespace

int rs2_verifier_roots_device_async(rs2_verifier* v, uint32_t count, const void* d_slivers,
                                    void* d_roots, void* stream) {
  if (!v || (count && (!d_slivers || !d_roots))) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (count == 0) return RS2_OK;
  HIP_TRY(hipSetDevice(v->ctx->device));
  hipStream_t st = abi_stream(stream, v->stream);
  int rc = verifier_leaves(v, count, reinterpret_cast<const uint8_t*>(d_slivers), st);
  if (rc != RS2_OK) return rc;
  uint8_t* scratch = nullptr;
  if (const size_t sb = tree_scratch_bytes(count, v->n)) {
    HIP_TRY(v->tree_scratch.ensure(sb));
    scratch = v->tree_scratch.as<uint8_t>();
  }
  HIP_TRY(rs2k_launch_merkle_trees(v->leaves.as<uint8_t>(), int(v->n), int(count), 0,
                                   int64_t(v->n) * 32, 32, 0, 0,
                                   reinterpret_cast<uint8_t*>(d_roots), 32, st, nullptr, 0, 1, 0,
                                   0, scratch));
  return verifier_mark_done(v, st);
}

int rs2_verifier_recovery_symbols_device_async(rs2_verifier* v, uint32_t count,
                                               const void* d_slivers,
                                               const uint16_t* target_sliver_index,
                                               void* d_symbols, void* d_proofs, void* d_nodes,
                                               void* stream) {
  if (!v || (count && (!d_slivers || !target_sliver_index || !d_symbols || !d_proofs)))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  for (uint32_t i = 0; i < count; ++i)
    if (target_sliver_index[i] >= v->n)  // slivers.rs check_index -> RecoverySymbolError::IndexTooLarge
      return fail(RS2_E_INVALID_ARGUMENT, "target index too large");
  if (count == 0) return RS2_OK;
  HIP_TRY(hipSetDevice(v->ctx->device));
  hipStream_t st = abi_stream(stream, v->stream);
  int rc = verifier_leaves(v, count, reinterpret_cast<const uint8_t*>(d_slivers), st);
  if (rc != RS2_OK) return rc;
  const int64_t n = v->n, nn = int64_t(merkle_n_nodes(uint64_t(n)));
  uint8_t* nodes = reinterpret_cast<uint8_t*>(d_nodes);
  if (!nodes) {
    HIP_TRY(v->nodes.ensure(size_t(count) * nn * 32));
    nodes = v->nodes.as<uint8_t>();
  }
  HIP_TRY(v->roots.ensure(size_t(count) * 32));
  HIP_TRY(rs2k_launch_merkle_trees(v->leaves.as<uint8_t>(), int(n), int(count), 0, n * 32, 32, 0, 0,
                                   v->roots.as<uint8_t>(), 32, st, nodes, nn * 32));
  // the targets go up through a pinned upload slot (no host copy to keep alive); the device
  // buffer is rewritten in stream order after the previous call's gather (verifier calls on
  // different streams are ordered by verifier_mark_done)
  v->targets_h.assign(target_sliver_index, target_sliver_index + count);
  HIP_TRY(v->targets.ensure(size_t(count) * 2));
  HIP_TRY(v->ctx->upload(v->targets.p, v->targets_h.data(), size_t(count) * 2, st));
  HIP_TRY(rs2k_launch_proof_gather(reinterpret_cast<const uint8_t*>(d_slivers),
                                   v->repair.as<uint8_t>(), int(n), int(v->k), int(v->s), nodes,
                                   nn * 32, v->targets.as<uint16_t>(), int(count),
                                   merkle_path_len(n), reinterpret_cast<uint8_t*>(d_symbols),
                                   reinterpret_cast<uint8_t*>(d_proofs), st));
  return verifier_mark_done(v, st);
}

int rs2_merkle_tree_shape(uint32_t n_leaves, uint32_t* path_len, uint64_t* n_nodes) {
  if (path_len) *path_len = uint32_t(merkle_path_len(n_leaves));
  if (n_nodes) *n_nodes = merkle_n_nodes(n_leaves);
  return RS2_OK;
}

int rs2_recovery_symbols(uint16_t n_shards, uint16_t symbol_size, int axis, uint32_t count,
                         const uint8_t* const* slivers, const uint64_t* sliver_len,
                         const uint16_t* target_sliver_index, uint8_t* symbols_out,
                         uint8_t* proofs_out) {
  if (count && (!slivers || !sliver_len || !target_sliver_index || !symbols_out || !proofs_out))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  VerifierLease lease;
  int rc = lease.get(n_shards, symbol_size, axis);
  if (rc != RS2_OK) return rc;
  rs2_verifier* v = lease.v;
  const uint64_t len = uint64_t(v->k) * symbol_size;
  for (uint32_t i = 0; i < count; ++i)
    if (!slivers[i] || sliver_len[i] != len)
      return fail(RS2_E_INCORRECT_DATA_LENGTH, "sliver length does not match the encoder");
  // every argument checked before any work is queued (a target is remote input on a node)
  for (uint32_t i = 0; i < count; ++i)
    if (target_sliver_index[i] >= n_shards)  // slivers.rs check_index -> IndexTooLarge
      return fail(RS2_E_INVALID_ARGUMENT, "target index too large");
  if (count == 0) return RS2_OK;
  HIP_TRY(hipSetDevice(v->ctx->device));
  const int L = merkle_path_len(n_shards);
  const size_t sym_b = size_t(count) * symbol_size, prf_b = size_t(count) * L * 32;
  HIP_TRY(v->input.ensure(size_t(count) * len));
  HIP_TRY(v->sym_out.ensure(sym_b));
  HIP_TRY(v->proof_out.ensure(size_t(count) * std::max(L, 1) * 32));
  HIP_TRY(v->h_in.ensure(size_t(count) * len));
  HIP_TRY(v->h_out.ensure(sym_b + prf_b));
  for (uint32_t i = 0; i < count; ++i)
    std::memcpy(static_cast<uint8_t*>(v->h_in.p) + size_t(i) * len, slivers[i], len);
  HIP_TRY(hipMemcpyAsync(v->input.p, v->h_in.p, size_t(count) * len, hipMemcpyHostToDevice,
                         v->stream));
  rc = rs2_verifier_recovery_symbols_device_async(v, count, v->input.p, target_sliver_index,
                                                  v->sym_out.p, v->proof_out.p, nullptr, nullptr);
  if (rc != RS2_OK) return rc;
  uint8_t* ho = static_cast<uint8_t*>(v->h_out.p);
  HIP_TRY(hipMemcpyAsync(ho, v->sym_out.p, sym_b, hipMemcpyDeviceToHost, v->stream));
  if (L) HIP_TRY(hipMemcpyAsync(ho + sym_b, v->proof_out.p, prf_b, hipMemcpyDeviceToHost, v->stream));
  HIP_TRY(hipStreamSynchronize(v->stream));
  std::memcpy(symbols_out, ho, sym_b);
  if (L) std::memcpy(proofs_out, ho + sym_b, prf_b);
  return RS2_OK;
}

int rs2_merkle_proof_roots(uint32_t count, const uint8_t* leaves, uint32_t leaf_len,
                           const uint32_t* leaf_index, const uint8_t* paths, uint32_t path_len,
                           uint8_t* roots_out) {
  if (count && (!leaves || !leaf_index || !roots_out || (path_len && !paths)))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (leaf_len % 2) return fail(RS2_E_INVALID_ARGUMENT, "leaf length must be even (symbols are)");
  if (count == 0) return RS2_OK;
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  hipStream_t st = ctx->util_stream;
  DevBuf dl, dd, di, dp, dr;
  HIP_TRY(dl.ensure(std::max<size_t>(size_t(count) * leaf_len, 16)));
  HIP_TRY(dd.ensure(size_t(count) * 32));
  HIP_TRY(di.ensure(size_t(count) * 4));
  HIP_TRY(dp.ensure(std::max<size_t>(size_t(count) * path_len * 32, 16)));
  HIP_TRY(dr.ensure(size_t(count) * 32));
  if (leaf_len)
    HIP_TRY(hipMemcpyAsync(dl.p, leaves, size_t(count) * leaf_len, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(di.p, leaf_index, size_t(count) * 4, hipMemcpyHostToDevice, st));
  if (path_len)
    HIP_TRY(hipMemcpyAsync(dp.p, paths, size_t(count) * path_len * 32, hipMemcpyHostToDevice, st));
  SymbolMap map{dl.as<uint8_t>(), nullptr, nullptr, 0, 0, 0, int(leaf_len)};
  HIP_TRY(rs2k_launch_leaf_hash(map, 1, count, 1, dd.as<uint8_t>(), st));
  HIP_TRY(rs2k_launch_proof_roots(dd.as<uint8_t>(), di.as<uint32_t>(), dp.as<uint8_t>(),
                                  int(path_len), int(count), dr.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(roots_out, dr.p, size_t(count) * 32, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return RS2_OK;
}

namespace {

// The n leaf hashes of every sliver without an expanded copy: the repair symbols go to a
// compact [count][n - k][s] buffer (v->repair) and the leaf kernel reads each sliver's
// systematic symbols in place (rs2k_launch_leaf_hash mode 4); recovery symbols gather from
// the same two places (proof_gather_kernel).
int verifier_leaves(rs2_verifier* v, uint32_t count, const uint8_t* din, hipStream_t st) {
  const int64_t n = v->n, K = v->k, s = v->s;
  // a previous call on another stream still owns the scratch buffers: order after it, so the
  // done event recorded at the end of this call also covers that one
  if (v->done) HIP_TRY(hipStreamWaitEvent(st, v->done, 0));
  HIP_TRY(v->leaves.ensure(size_t(count) * n * 32));
  uint8_t* rep = nullptr;
  if (n > K) {
    HIP_TRY(v->repair.ensure(size_t(count) * (n - K) * s));
    rep = v->repair.as<uint8_t>();
    int rc = plan_encode(uint32_t(K), uint32_t(n - K), int(s), din, K * s,
                         [&](uint32_t i) { return int64_t(i) * s; }, rep, (n - K) * s,
                         [&](uint32_t j) { return int64_t(j) * s; }, INT64_MAX, v->job);
    if (rc != RS2_OK) return rc;
    rc = bind_encode(v->ctx, v->job, v->mem, st);
    if (rc != RS2_OK) return rc;
    HIP_TRY(v->job.launch(int(count), st));
  }
  SymbolMap map{din, rep, nullptr, int(n), int(count), int(K), int(s)};
  HIP_TRY(rs2k_launch_leaf_hash(map, 4, int64_t(count) * n, 1, v->leaves.as<uint8_t>(), st));
  return RS2_OK;
}
}  // namespace

int rs2_sliver_merkle_roots(uint16_t n_shards, uint16_t symbol_size, int axis, uint32_t count,
                            const uint8_t* const* slivers, const uint64_t* sliver_len,
                            uint8_t* roots_out) {
  if (count && (!slivers || !sliver_len || !roots_out))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  VerifierLease lease;
  int rc = lease.get(n_shards, symbol_size, axis);
  if (rc != RS2_OK) return rc;
  rs2_verifier* v = lease.v;
  const uint64_t len = uint64_t(v->k) * symbol_size;
  for (uint32_t i = 0; i < count; ++i)
    if (!slivers[i] || sliver_len[i] != len)
      return fail(RS2_E_INCORRECT_DATA_LENGTH, "sliver length does not match the encoder");
  if (count == 0) return RS2_OK;
  HIP_TRY(hipSetDevice(v->ctx->device));
  HIP_TRY(v->input.ensure(size_t(count) * len));
  HIP_TRY(v->roots.ensure(size_t(count) * 32));
  // the slivers gathered into pinned staging: one DMA instead of one pageable copy per sliver
  HIP_TRY(v->h_in.ensure(size_t(count) * len));
  HIP_TRY(v->h_out.ensure(size_t(count) * 32));
  for (uint32_t i = 0; i < count; ++i)
    std::memcpy(static_cast<uint8_t*>(v->h_in.p) + size_t(i) * len, slivers[i], len);
  HIP_TRY(hipMemcpyAsync(v->input.p, v->h_in.p, size_t(count) * len, hipMemcpyHostToDevice,
                         v->stream));
  rc = rs2_verifier_roots_device_async(v, count, v->input.p, v->roots.p, nullptr);
  if (rc != RS2_OK) return rc;
  HIP_TRY(hipMemcpyAsync(v->h_out.p, v->roots.p, size_t(count) * 32, hipMemcpyDeviceToHost,
                         v->stream));
  HIP_TRY(hipStreamSynchronize(v->stream));
  std::memcpy(roots_out, v->h_out.p, size_t(count) * 32);
  return RS2_OK;
}

int rs2_sliver_merkle_root(uint16_t n_shards, uint16_t symbol_size, int axis, const uint8_t* sliver,
                           uint64_t sliver_len, uint8_t root_out[32]) {
  if (!sliver || !root_out || symbol_size == 0) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  return rs2_sliver_merkle_roots(n_shards, symbol_size, axis, 1, &sliver, &sliver_len, root_out);
}

int rs2_merkle_root(const uint8_t* leaves, uint32_t n_leaves, uint32_t leaf_len, uint8_t root_out[32]) {
  if ((!leaves && n_leaves) || !root_out) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (n_leaves == 0) {  // merkle.rs: an empty tree's root is the all-zero node
    std::memset(root_out, 0, 32);
    return RS2_OK;
  }
  if (leaf_len > 0x7FFFFFFFu / 2) return fail(RS2_E_UNSUPPORTED, "leaf too large");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  hipStream_t st = ctx->util_stream;
  DevBuf din, digests, tmp, root;
  HIP_TRY(din.ensure(size_t(n_leaves) * leaf_len));
  HIP_TRY(digests.ensure(size_t(n_leaves) * 32));
  HIP_TRY(root.ensure(32));
  if (leaf_len)
    HIP_TRY(hipMemcpyAsync(din.p, leaves, size_t(n_leaves) * leaf_len, hipMemcpyHostToDevice, st));
  SymbolMap map{din.as<uint8_t>(), nullptr, nullptr, 0, 0, 0, int(leaf_len)};
  HIP_TRY(rs2k_launch_leaf_hash(map, 1, n_leaves, 1, digests.as<uint8_t>(), st));
  rc = device_merkle_root(digests.as<uint8_t>(), n_leaves, tmp, root.as<uint8_t>(), st);
  if (rc != RS2_OK) return rc;
  HIP_TRY(hipMemcpyAsync(root_out, root.p, 32, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return RS2_OK;
}

// ---- device 1D codec over strided lines, device hashing primitives -------------------------

int rs2_codec_create(uint16_t k, uint16_t n_shards, uint16_t symbol_size, rs2_codec** out) {
  if (!out) return fail(RS2_E_INVALID_ARGUMENT, "null codec pointer");
  *out = nullptr;
  if (symbol_size == 0 || symbol_size % 2)
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "symbol_size must be a multiple of the required alignment");
  if (k == 0 || n_shards <= k) return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "need 0 < k < n_shards");
  if (!rate_supported(k, uint32_t(n_shards) - k))
    return fail(RS2_E_INCOMPATIBLE_PARAMETERS, "unsupported shard count");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  auto c = std::make_unique<rs2_codec>();
  c->ctx = ctx;
  c->n = n_shards;
  c->k = k;
  c->s = symbol_size;
  *out = c.release();
  return RS2_OK;
}

void rs2_codec_destroy(rs2_codec* c) {
  if (!c) return;
  (void)hipSetDevice(c->ctx->device);
  if (c->enc_done) (void)hipEventSynchronize(c->enc_done);
  for (auto& e : c->dec_done)
    if (e) (void)hipEventSynchronize(e);
  const bool prev = t_quiesced;
  t_quiesced = true;
  delete c;
  t_quiesced = prev;
}

int rs2_codec_encode_device_async(rs2_codec* c, uint32_t lines, const void* d_src,
                                  uint64_t src_sym_stride, uint64_t src_line_stride,
                                  void* d_repair, uint64_t repair_sym_stride,
                                  uint64_t repair_line_stride, void* stream) {
  if (!c || (lines && (!d_src || !d_repair))) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (lines == 0) return RS2_OK;
  if (src_sym_stride < c->s || repair_sym_stride < c->s)
    return fail(RS2_E_INVALID_ARGUMENT, "symbol stride smaller than the symbol");
  HIP_TRY(hipSetDevice(c->ctx->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t key[4] = {int64_t(src_sym_stride), int64_t(src_line_stride),
                          int64_t(repair_sym_stride), int64_t(repair_line_stride)};
  const uint8_t* src = reinterpret_cast<const uint8_t*>(d_src);
  uint8_t* dst = reinterpret_cast<uint8_t*>(d_repair);
  if (!std::equal(key, key + 4, c->enc_key)) {
    if (c->enc_done) HIP_TRY(hipEventSynchronize(c->enc_done));  // old arrays may be in use
    const int64_t ss = key[0], rs = key[2];
    int rc = plan_encode(uint32_t(c->k), uint32_t(c->n - c->k), int(c->s), src, key[1],
                         [&](uint32_t i) { return int64_t(i) * ss; }, dst, key[3],
                         [&](uint32_t j) { return int64_t(j) * rs; }, INT64_MAX, c->enc);
    if (rc != RS2_OK) return rc;
    rc = bind_encode(c->ctx, c->enc, c->enc_mem, st);
    if (rc != RS2_OK) return rc;
    std::copy(key, key + 4, c->enc_key);
  }
  for (int b = 0; b < c->enc.job.n_in; ++b) c->enc.job.in[b].base = src;
  for (int o = 0; o < c->enc.job.n_out; ++o) c->enc.job.out[o].base = dst;
  HIP_TRY(c->enc.launch(int(lines), st));
  if (!c->enc_done) HIP_TRY(hipEventCreateWithFlags(&c->enc_done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(c->enc_done, st));
  return RS2_OK;
}

int rs2_codec_decode_device_async(rs2_codec* c, uint32_t lines, uint32_t count,
                                  const uint16_t* idx, const void* d_base, const uint64_t* sym_off,
                                  uint64_t line_stride, void* d_out, uint64_t out_sym_stride,
                                  uint64_t out_line_stride, uint64_t out_limit, void* stream) {
  if (!c || (count && (!idx || !sym_off)) || (lines && (!d_base || !d_out)))
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (out_sym_stride < c->s) return fail(RS2_E_INVALID_ARGUMENT, "symbol stride smaller than the symbol");
  const int64_t K = c->k, N = c->n, s = c->s;
  // the first K distinct valid indices (the crate ignores duplicates and invalid indices)
  std::vector<int64_t> present(N, -1);
  uint32_t got = 0;
  for (uint32_t i = 0; i < count && got < K; ++i) {
    if (idx[i] >= N || present[idx[i]] >= 0) continue;
    present[idx[i]] = int64_t(sym_off[i]);
    ++got;
  }
  if (got < K) return fail(RS2_E_NOT_ENOUGH_SHARDS, "not enough shards");
  if (lines == 0) return RS2_OK;
  HIP_TRY(hipSetDevice(c->ctx->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int slot = c->dec_slot;
  c->dec_slot ^= 1;
  if (c->dec_done[slot]) HIP_TRY(hipEventSynchronize(c->dec_done[slot]));
  const uint8_t* base = reinterpret_cast<const uint8_t*>(d_base);
  uint8_t* out = reinterpret_cast<uint8_t*>(d_out);
  std::vector<int64_t>& cs = c->copy_src_h[slot];
  std::vector<int64_t>& cd = c->copy_dst_h[slot];
  cs.clear();
  cd.clear();
  for (int64_t i = 0; i < K; ++i)
    if (present[i] >= 0) {
      cs.push_back(present[i]);
      cd.push_back(i * int64_t(out_sym_stride));
    }
  const bool run_codec = cs.size() < size_t(K);
  bool fused = false;
  PlannedJob& pj = c->dec[slot];
  if (run_codec) {
    DecodeSpec sp;
    sp.K = uint32_t(K);
    sp.R = uint32_t(N - K);
    sp.symbol_size = int(s);
    sp.present = present;
    sp.src_base = base;
    sp.src_ls = int64_t(line_stride);
    sp.dst_base = out;
    sp.dst_ls = int64_t(out_line_stride);
    sp.dst_limit = int64_t(std::min<uint64_t>(out_limit, uint64_t(INT64_MAX)));
    sp.dst.resize(K);
    for (int64_t i = 0; i < K; ++i) sp.dst[i] = i * int64_t(out_sym_stride);
    sp.copy_present = !cs.empty() && s >= 4;
    int rc = plan_decode(sp, pj);
    if (rc != RS2_OK) return rc;
    fused = sp.copy_present && copy_covered(pj);
  }
  if (!cs.empty() && !fused) {
    HIP_TRY(c->copy_src[slot].ensure(cs.size() * 8));
    HIP_TRY(c->copy_dst[slot].ensure(cd.size() * 8));
    HIP_TRY(c->ctx->upload(c->copy_src[slot].p, cs.data(), cs.size() * 8, st));
    HIP_TRY(c->ctx->upload(c->copy_dst[slot].p, cd.data(), cd.size() * 8, st));
    HIP_TRY(rs2k_launch_symbol_copy(base, c->copy_src[slot].as<int64_t>(), int64_t(line_stride), out,
                                    c->copy_dst[slot].as<int64_t>(), int64_t(out_line_stride),
                                    int(cs.size()), int(lines), int(s),
                                    int64_t(std::min<uint64_t>(out_limit, uint64_t(INT64_MAX))), st));
  }
  if (run_codec) {
    int rc = bind_decode(c->ctx, pj, c->dec_mem[slot], st);
    if (rc != RS2_OK) return rc;
    HIP_TRY(pj.launch(int(lines), st));
  }
  if (!c->dec_done[slot]) HIP_TRY(hipEventCreateWithFlags(&c->dec_done[slot], hipEventDisableTiming));
  HIP_TRY(hipEventRecord(c->dec_done[slot], st));
  return RS2_OK;
}

int rs2_copy_segments_device_async(const void* d_src, void* d_dst, uint32_t count_a,
                                   const int64_t* d_src_a, const int64_t* d_dst_a, uint32_t count_b,
                                   int64_t src_b_stride, int64_t dst_b_stride, uint32_t seg_len,
                                   uint32_t unit, void* stream) {
  if (count_a == 0 || count_b == 0 || seg_len == 0) return RS2_OK;
  if (!d_src || !d_dst || !d_src_a || !d_dst_a) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (unit != 1 && unit != 2 && unit != 4 && unit != 8 && unit != 16)
    return fail(RS2_E_INVALID_ARGUMENT, "unit must be 1, 2, 4, 8 or 16");
  const auto misaligned = [&](int64_t v) { return v % int64_t(unit) != 0; };
  if (misaligned(int64_t(seg_len)) || misaligned(src_b_stride) || misaligned(dst_b_stride) ||
      misaligned(int64_t(reinterpret_cast<uintptr_t>(d_src))) ||
      misaligned(int64_t(reinterpret_cast<uintptr_t>(d_dst))))
    return fail(RS2_E_INVALID_ARGUMENT, "length, strides or bases not multiples of unit");
  HIP_TRY(rs2k_launch_segment_copy(static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst),
                                   count_a, d_src_a, d_dst_a, count_b, src_b_stride, dst_b_stride,
                                   seg_len, int(unit), static_cast<hipStream_t>(stream)));
  return RS2_OK;
}

int rs2_leaf_hashes_device_async(const void* d_symbols, uint64_t count, uint16_t symbol_size,
                                 void* d_leaves, void* stream) {
  if (count && (!d_symbols || !d_leaves)) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (symbol_size % 2) return fail(RS2_E_INVALID_ARGUMENT, "symbol_size must be even");
  if (count == 0) return RS2_OK;
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  SymbolMap map{reinterpret_cast<const uint8_t*>(d_symbols), nullptr, nullptr, 0, 0, 0, int(symbol_size)};
  HIP_TRY(rs2k_launch_leaf_hash(map, 1, int64_t(count), 1, reinterpret_cast<uint8_t*>(d_leaves),
                                reinterpret_cast<hipStream_t>(stream)));
  return RS2_OK;
}

int rs2_merkle_roots_device_async(const void* d_leaves, uint32_t n_trees, uint32_t n_leaves,
                                  uint64_t tree_stride, uint64_t leaf_stride, void* d_roots,
                                  uint64_t root_stride, void* stream) {
  if (n_trees && (!d_leaves || !d_roots)) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (n_leaves == 0 || n_leaves > uint32_t(kMaxShards))
    return fail(RS2_E_UNSUPPORTED, "trees of 1..65535 leaves supported by this build");
  if (leaf_stride % 16 || tree_stride % 16 || root_stride % 4)
    return fail(RS2_E_INVALID_ARGUMENT, "leaf/tree strides must be multiples of 16 bytes");
  if (n_trees == 0) return RS2_OK;
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  // above 4,096 leaves the folded level goes to scratch; the arena quarantines the range when
  // this buffer is released, so the queued launches keep it until the next device sync
  DevBuf scratch;
  if (n_leaves > uint32_t(kMerkleMaxLeaves))
    HIP_TRY(scratch.ensure(tree_scratch_bytes(n_trees, n_leaves)));
  HIP_TRY(rs2k_launch_merkle_trees(reinterpret_cast<const uint8_t*>(d_leaves), int(n_leaves),
                                   int(n_trees), 0, int64_t(tree_stride), int64_t(leaf_stride), 0, 0,
                                   reinterpret_cast<uint8_t*>(d_roots), int64_t(root_stride),
                                   reinterpret_cast<hipStream_t>(stream), nullptr, 0, 1, 0, 0,
                                   scratch.as<uint8_t>()));
  return RS2_OK;
}

int rs2_blob_id_device_async(const void* d_hashes, uint16_t n_shards, uint64_t blob_len,
                             void* d_blob_id, void* stream) {
  if (!d_blob_id || (n_shards && !d_hashes)) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (n_shards > kMaxShards) return fail(RS2_E_UNSUPPORTED, "n_shards above 65535");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  HIP_TRY(rs2k_launch_merkle_root(reinterpret_cast<const uint8_t*>(d_hashes), n_shards, blob_len,
                                  reinterpret_cast<uint8_t*>(d_blob_id),
                                  reinterpret_cast<hipStream_t>(stream)));
  return RS2_OK;
}

int rs2_blob_id_from_hashes(const uint8_t* hashes, uint16_t n_shards, uint64_t blob_len,
                            uint8_t blob_id_out[32]) {
  if (!hashes || !blob_id_out) return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  if (n_shards > kMaxShards) return fail(RS2_E_UNSUPPORTED, "n_shards above 65535");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  hipStream_t st = ctx->util_stream;
  DevBuf dh, bid;
  HIP_TRY(dh.ensure(size_t(n_shards) * 64));
  HIP_TRY(bid.ensure(32));
  if (n_shards)
    HIP_TRY(hipMemcpyAsync(dh.p, hashes, size_t(n_shards) * 64, hipMemcpyHostToDevice, st));
  HIP_TRY(rs2k_launch_merkle_root(dh.as<uint8_t>(), n_shards, blob_len, bid.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(blob_id_out, bid.p, 32, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return RS2_OK;
}

int rs2_quilt_layout_device_async(uint16_t n_rows, uint16_t n_cols, uint16_t symbol_size,
                                  const void* d_payload, const int64_t* d_col_off,
                                  const uint32_t* d_col_len, void* d_quilt, void* stream) {
  if (!n_rows || !n_cols || !symbol_size) return fail(RS2_E_INVALID_ARGUMENT, "empty quilt");
  if (symbol_size & 1) return fail(RS2_E_INVALID_ARGUMENT, "symbol size must be even");
  if (!d_payload || !d_col_off || !d_col_len || !d_quilt)
    return fail(RS2_E_INVALID_ARGUMENT, "null argument");
  Context* ctx = nullptr;
  int rc = get_context(&ctx);
  if (rc != RS2_OK) return rc;
  HIP_TRY(rs2k_launch_quilt_layout(n_rows, n_cols, symbol_size,
                                   reinterpret_cast<const uint8_t*>(d_payload), d_col_off, d_col_len,
                                   reinterpret_cast<uint8_t*>(d_quilt),
                                   reinterpret_cast<hipStream_t>(stream)));
  return RS2_OK;
}

}  // extern "C"
