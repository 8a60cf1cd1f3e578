/*
 * rs2_cpu.c -- CPU restatement of the Red Stuff (RS2) path: TEST INFRASTRUCTURE / CPU BASELINE.
 *
 * Not product code: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it (as the checker and as the timed CPU reference).  It restates, in C with AVX2:
 *   - reed-solomon-simd 3.1.0 (Cargo.lock:8813): GF(2^16) Cantor-basis tables, skew LUT,
 *     additive FFT/IFFT, high/low-rate encoders, the erasure decoder with its per-call
 *     eval_poly (FWHT over the whole field), and the 64-byte lo/hi shard layout, with the
 *     crate's AVX2 technique (vpshufb nibble tables, 32 elements per 64-byte chunk);
 *   - walrus-core: encode_with_metadata (blob_encoding.rs:277-368), leaf hashes + Merkle
 *     trees + BlobId (blob_encoding.rs:161-196, merkle.rs:216-332, lib.rs:159-176),
 *     BlobDecoder::decode (blob_encoding.rs:888-993);
 *   - blake2b-256 (RustCrypto blake2 0.10.6 portable path).
 * Like the reference, one blob is encoded/decoded on one thread.
 *
 * Build: make -C oracle  ->  oracle/build/librs2cpu.so, oracle/build/rs2_cpu_bench
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------------------------
 * GF(2^16) tables
 * ---------------------------------------------------------------------------------------- */
#define ORDER 65536u
#define MODULUS 65535u
static uint16_t EXP[ORDER], LOG[ORDER], SKEW[MODULUS];
static int64_t LOG_WALSH[ORDER];
static int g_init = 0;

static uint32_t add_mod(uint32_t a, uint32_t b) {
  uint32_t s = a + b;
  return (s + (s >> 16)) & 0xFFFF;
}
static uint32_t gmul(uint32_t x, uint32_t log_m) { return x ? EXP[add_mod(LOG[x], log_m)] : 0; }

static void fwht(int64_t* a, uint32_t n, uint32_t trunc);

void rs2cpu_init(void) {
  if (g_init) return;
  static const uint16_t cantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E,
                                      0x914C, 0x4012, 0x6C98, 0x10D8, 0x6A72, 0xB900,
                                      0xFDB8, 0xFB34, 0xFF38, 0x991E};
  static uint32_t e[ORDER], l[ORDER];
  uint32_t state = 1;
  for (uint32_t i = 0; i < MODULUS; i++) {
    e[state] = i;
    state <<= 1;
    if (state >= ORDER) state ^= 0x1002D;
  }
  e[0] = MODULUS;
  l[0] = 0;
  for (int i = 0; i < 16; i++)
    for (uint32_t j = 0; j < (1u << i); j++) l[j + (1u << i)] = l[j] ^ cantor[i];
  for (uint32_t i = 0; i < ORDER; i++) l[i] = e[l[i]];
  for (uint32_t i = 0; i < ORDER; i++) e[l[i]] = i;
  e[MODULUS] = e[0];
  for (uint32_t i = 0; i < ORDER; i++) {
    EXP[i] = (uint16_t)e[i];
    LOG[i] = (uint16_t)l[i];
  }
  static uint32_t sk[MODULUS];
  uint32_t temp[15];
  for (int i = 1; i < 16; i++) temp[i - 1] = 1u << i;
  for (int m = 0; m < 15; m++) {
    uint32_t step = 1u << (m + 1);
    sk[(1u << m) - 1] = 0;
    for (int i = m; i < 15; i++) {
      uint32_t s = 1u << (i + 1);
      for (uint32_t j = (1u << m) - 1; j < s; j += step) sk[j + s] = sk[j] ^ temp[i];
    }
    temp[m] = MODULUS - LOG[gmul(temp[m], LOG[temp[m] ^ 1])];
    for (int i = m + 1; i < 15; i++) temp[i] = gmul(temp[i], add_mod(LOG[temp[i] ^ 1], temp[m]));
  }
  for (uint32_t i = 0; i < MODULUS; i++) SKEW[i] = LOG[sk[i]];
  for (uint32_t i = 0; i < ORDER; i++) LOG_WALSH[i] = LOG[i];
  LOG_WALSH[0] = 0;
  fwht(LOG_WALSH, ORDER, ORDER);
  g_init = 1;
}

/* ------------------------------------------------------------------------------------------
 * shards: `chunks` x 64-byte chunks; element j of chunk q = lo[j] | hi[j] << 8
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  __m256i t[8]; /* [k][byte]: nibble k -> lo / hi byte of (n << 4k) * c, both 128-bit lanes */
} MulTab;

static void make_tab(uint32_t log_m, MulTab* mt) {
  uint8_t b[8][16];
  for (int k = 0; k < 4; k++)
    for (int n = 0; n < 16; n++) {
      uint32_t v = gmul((uint32_t)n << (4 * k), log_m);
      b[2 * k][n] = (uint8_t)v;
      b[2 * k + 1][n] = (uint8_t)(v >> 8);
    }
  for (int i = 0; i < 8; i++) {
    __m128i x = _mm_loadu_si128((const __m128i*)b[i]);
    mt->t[i] = _mm256_broadcastsi128_si256(x);
  }
}

/* x ^= y * c  over `chunks` chunks */
static void mul_add(uint8_t* x, const uint8_t* y, const MulTab* mt, size_t chunks) {
  const __m256i m = _mm256_set1_epi8(0x0F);
  for (size_t q = 0; q < chunks; q++) {
    __m256i lo = _mm256_loadu_si256((const __m256i*)(y + 64 * q));
    __m256i hi = _mm256_loadu_si256((const __m256i*)(y + 64 * q + 32));
    __m256i l0 = _mm256_and_si256(lo, m), l1 = _mm256_and_si256(_mm256_srli_epi64(lo, 4), m);
    __m256i h0 = _mm256_and_si256(hi, m), h1 = _mm256_and_si256(_mm256_srli_epi64(hi, 4), m);
    __m256i plo = _mm256_xor_si256(
        _mm256_xor_si256(_mm256_shuffle_epi8(mt->t[0], l0), _mm256_shuffle_epi8(mt->t[2], l1)),
        _mm256_xor_si256(_mm256_shuffle_epi8(mt->t[4], h0), _mm256_shuffle_epi8(mt->t[6], h1)));
    __m256i phi = _mm256_xor_si256(
        _mm256_xor_si256(_mm256_shuffle_epi8(mt->t[1], l0), _mm256_shuffle_epi8(mt->t[3], l1)),
        _mm256_xor_si256(_mm256_shuffle_epi8(mt->t[5], h0), _mm256_shuffle_epi8(mt->t[7], h1)));
    __m256i* xl = (__m256i*)(x + 64 * q);
    __m256i* xh = (__m256i*)(x + 64 * q + 32);
    _mm256_storeu_si256(xl, _mm256_xor_si256(_mm256_loadu_si256(xl), plo));
    _mm256_storeu_si256(xh, _mm256_xor_si256(_mm256_loadu_si256(xh), phi));
  }
}

/* x = x * c (in place) */
static void mul_inplace(uint8_t* x, const MulTab* mt, size_t chunks, uint8_t* tmp) {
  memcpy(tmp, x, 64 * chunks);
  memset(x, 0, 64 * chunks);
  mul_add(x, tmp, mt, chunks);
}

static void xor_into(uint8_t* x, const uint8_t* y, size_t chunks) {
  for (size_t i = 0; i < 2 * chunks; i++) {
    __m256i* a = (__m256i*)(x + 32 * i);
    _mm256_storeu_si256(a, _mm256_xor_si256(_mm256_loadu_si256(a),
                                            _mm256_loadu_si256((const __m256i*)(y + 32 * i))));
  }
}

/* table cache per log value (built lazily; thread-safe: a table is published with a release
   compare-and-swap after it is complete, a racing builder frees its copy) */
static MulTab* g_tabs[ORDER];
static const MulTab* tab_for(uint32_t log_m) {
  MulTab* cur = __atomic_load_n(&g_tabs[log_m], __ATOMIC_ACQUIRE);
  if (cur) return cur;
  MulTab* t = (MulTab*)aligned_alloc(32, sizeof(MulTab));
  make_tab(log_m, t);
  MulTab* expected = NULL;
  if (__atomic_compare_exchange_n(&g_tabs[log_m], &expected, t, 0, __ATOMIC_RELEASE,
                                  __ATOMIC_ACQUIRE))
    return t;
  free(t);
  return expected;
}

/* FFT / IFFT on shards work[pos..pos+size) (radix-2 statement of the crate's engine) */
static void fft(uint8_t** w, size_t chunks, uint32_t pos, uint32_t size, uint32_t trunc,
                uint32_t sd) {
  for (uint32_t d = size >> 1; d >= 1; d >>= 1) {
    for (uint32_t r = 0; r < trunc; r += 2 * d) {
      uint32_t lm = SKEW[r + d + sd - 1];
      const MulTab* mt = lm == MODULUS ? NULL : tab_for(lm);
      for (uint32_t i = r; i < r + d; i++) {
        uint8_t* x = w[pos + i];
        uint8_t* y = w[pos + i + d];
        if (mt) mul_add(x, y, mt, chunks);
        xor_into(y, x, chunks);
      }
    }
    if (d == 1) break;
  }
}

static void ifft(uint8_t** w, size_t chunks, uint32_t pos, uint32_t size, uint32_t trunc,
                 uint32_t sd) {
  for (uint32_t d = 1; d < size; d <<= 1) {
    for (uint32_t r = 0; r < trunc; r += 2 * d) {
      uint32_t lm = SKEW[r + d + sd - 1];
      const MulTab* mt = lm == MODULUS ? NULL : tab_for(lm);
      for (uint32_t i = r; i < r + d; i++) {
        uint8_t* x = w[pos + i];
        uint8_t* y = w[pos + i + d];
        xor_into(y, x, chunks);
        if (mt) mul_add(x, y, mt, chunks);
      }
    }
  }
}

static uint32_t pow2(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
static int high_rate(uint32_t k, uint32_t r) { return pow2(r) <= pow2(k); }

/* shard byte layout <-> chunk layout (reed-solomon-simd Shards::insert / undo_last_chunk) */
static void to_chunks(const uint8_t* sym, uint32_t s, uint8_t* dst) {
  uint32_t full = s / 64 * 64, t = s % 64;
  memcpy(dst, sym, full);
  if (t) {
    uint8_t* c = dst + full;
    memset(c, 0, 64);
    memcpy(c, sym + full, t / 2);
    memcpy(c + 32, sym + full + t / 2, t / 2);
  }
}
static void from_chunks(const uint8_t* src, uint32_t s, uint8_t* sym) {
  uint32_t full = s / 64 * 64, t = s % 64;
  memcpy(sym, src, full);
  if (t) {
    memcpy(sym + full, src + full, t / 2);
    memcpy(sym + full + t / 2, src + full + 32, t / 2);
  }
}

typedef struct {
  uint32_t k, r, s, chunks, cap;
  uint8_t* mem;  /* cap shards */
  uint8_t** w;
  uint8_t* tmp;
} Codec;

static void codec_init(Codec* c, uint32_t k, uint32_t r, uint32_t s) {
  c->k = k;
  c->r = r;
  c->s = s;
  c->chunks = (s + 63) / 64;
  uint32_t cs = high_rate(k, r) ? pow2(r) : pow2(k);
  uint32_t end = high_rate(k, r) ? cs + k : cs + r;
  uint32_t w = pow2(end);
  c->cap = w > 2 * cs ? w : 2 * cs;
  if (c->cap < k + cs) c->cap = pow2(k + cs);
  size_t shard = 64 * (size_t)c->chunks;
  c->mem = (uint8_t*)aligned_alloc(64, shard * c->cap);
  c->w = (uint8_t**)malloc(sizeof(uint8_t*) * c->cap);
  for (uint32_t i = 0; i < c->cap; i++) c->w[i] = c->mem + shard * i;
  c->tmp = (uint8_t*)aligned_alloc(64, shard);
}
static void codec_free(Codec* c) {
  free(c->mem);
  free(c->w);
  free(c->tmp);
}

/* encode: src[i] (i < k) symbol pointers -> rec[j] (j < r) symbol pointers */
static void codec_encode(Codec* c, const uint8_t* const* src, uint8_t* const* rec) {
  const uint32_t k = c->k, r = c->r, ch = c->chunks;
  const size_t shard = 64 * (size_t)ch;
  uint8_t** w = c->w;
  if (high_rate(k, r)) {
    const uint32_t cs = pow2(r);
    memset(w[0], 0, shard * cs);
    for (uint32_t start = 0; start < k; start += cs) {
      uint32_t cnt = k - start < cs ? k - start : cs;
      uint8_t** blk = w + cs;
      memset(blk[0], 0, shard * cs);
      for (uint32_t i = 0; i < cnt; i++) to_chunks(src[start + i], c->s, blk[i]);
      ifft(blk, ch, 0, cs, cnt, start + cs);
      for (uint32_t i = 0; i < cs; i++) xor_into(w[i], blk[i], ch);
    }
    fft(w, ch, 0, cs, r, 0);
    for (uint32_t j = 0; j < r; j++) from_chunks(w[j], c->s, rec[j]);
  } else {
    const uint32_t cs = pow2(k);
    memset(w[0], 0, shard * cs);
    for (uint32_t i = 0; i < k; i++) to_chunks(src[i], c->s, w[i]);
    ifft(w, ch, 0, cs, k, 0);
    uint8_t** cp = w + cs;
    for (uint32_t start = 0; start < r; start += cs) {
      uint32_t cnt = r - start < cs ? r - start : cs;
      memcpy(cp[0], w[0], shard * cs);
      fft(cp, ch, 0, cs, cnt, start + cs);
      for (uint32_t j = 0; j < cnt; j++) from_chunks(cp[j], c->s, rec[start + j]);
    }
  }
}

/* FWHT mod 65535 over n points (first layers truncated to `trunc` non-zero inputs) */
static void fwht(int64_t* a, uint32_t n, uint32_t trunc) {
  (void)trunc;
  for (uint32_t h = 1; h < n; h <<= 1)
    for (uint32_t i = 0; i < n; i += 2 * h)
      for (uint32_t j = i; j < i + h; j++) {
        int64_t x = a[j], y = a[j + h];
        int64_t s = x + y, d = x - y;
        a[j] = (s + (s >> 16)) & 0xFFFF;
        d &= 0xFFFFFFFF;
        a[j + h] = (d + (d >> 16)) & 0xFFFF;
      }
}

/* decode: `present[q]` symbol pointer or NULL for q < k+r; writes the k originals to out[i]
 * (originals that were present are copied).  eval_poly is recomputed per call over the whole
 * field, as the crate's decoder does. */
static int codec_decode(Codec* c, const uint8_t* const* present, uint8_t* const* out) {
  const uint32_t k = c->k, r = c->r, ch = c->chunks;
  const size_t shard = 64 * (size_t)ch;
  uint32_t have = 0, all_orig = 1;
  for (uint32_t q = 0; q < k + r; q++) have += present[q] != NULL;
  for (uint32_t i = 0; i < k; i++) all_orig &= present[i] != NULL;
  if (have < k) return -1;
  for (uint32_t i = 0; i < k; i++)
    if (present[i]) memcpy(out[i], present[i], c->s);
  if (all_orig) return 0;
  const int hi = high_rate(k, r);
  const uint32_t cs = hi ? pow2(r) : pow2(k);
  const uint32_t end = hi ? cs + k : cs + r;
  const uint32_t W = pow2(end);
  static __thread int64_t er[ORDER];  /* per thread: the CPU baseline runs one blob per thread */
  memset(er, 0, sizeof(er));
  for (uint32_t i = 0; i < k; i++)
    if (!present[i]) er[hi ? cs + i : i] = 1;
  for (uint32_t j = 0; j < r; j++)
    if (!present[k + j]) er[hi ? j : cs + j] = 1;
  if (hi) {
    for (uint32_t p = r; p < cs; p++) er[p] = 1;
  } else {
    for (uint32_t p = end; p < W; p++) er[p] = 1;
  }
  /* eval_poly: FWHT, multiply by FWHT(log), FWHT -> log of the locator (mod 65535) */
  fwht(er, ORDER, hi ? end : ORDER);
  for (uint32_t i = 0; i < ORDER; i++) er[i] = (er[i] * LOG_WALSH[i]) % MODULUS;
  fwht(er, ORDER, ORDER);
  uint8_t** w = c->w;
  memset(w[0], 0, shard * W);
  for (uint32_t q = 0; q < k + r; q++) {
    if (!present[q]) continue;
    uint32_t p = q < k ? (hi ? cs + q : q) : (hi ? q - k : cs + (q - k));
    to_chunks(present[q], c->s, w[p]);
    uint32_t lm = (uint32_t)er[p];
    mul_inplace(w[p], tab_for(lm == MODULUS ? 0 : lm), ch, c->tmp);
  }
  ifft(w, ch, 0, W, end, 0);
  for (uint32_t i = 1; i < W; i++) {
    uint32_t width = i & (~i + 1);
    for (uint32_t j = 0; j < width; j++) xor_into(w[i - width + j], w[i + j], ch);
  }
  fft(w, ch, 0, W, hi ? end : k, 0);
  for (uint32_t i = 0; i < k; i++) {
    if (present[i]) continue;
    uint32_t p = hi ? cs + i : i;
    uint32_t lm = MODULUS - (uint32_t)(er[p] % MODULUS);
    mul_inplace(w[p], tab_for(lm == MODULUS ? 0 : lm), ch, c->tmp);
    from_chunks(w[p], c->s, out[i]);
  }
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * Blake2b-256
 * ---------------------------------------------------------------------------------------- */
static const uint64_t B2IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint8_t SIG[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
#define ROTR(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
#define G(a, b, c, d, x, y)     \
  do {                          \
    v[a] = v[a] + v[b] + (x);   \
    v[d] = ROTR(v[d] ^ v[a], 32); \
    v[c] = v[c] + v[d];         \
    v[b] = ROTR(v[b] ^ v[c], 24); \
    v[a] = v[a] + v[b] + (y);   \
    v[d] = ROTR(v[d] ^ v[a], 16); \
    v[c] = v[c] + v[d];         \
    v[b] = ROTR(v[b] ^ v[c], 63); \
  } while (0)

static void b2_compress(uint64_t h[8], const uint8_t blk[128], uint64_t t, int last) {
  uint64_t m[16], v[16];
  memcpy(m, blk, 128);
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = B2IV[i];
  }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = SIG[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

/* Blake2b-256(prefix || data) */
static void b2_prefixed(uint8_t prefix, const uint8_t* data, size_t len, uint8_t out[32]) {
  uint64_t h[8];
  for (int i = 0; i < 8; i++) h[i] = B2IV[i];
  h[0] ^= 0x01010020ULL;
  uint8_t blk[128];
  size_t total = len + 1, done = 0;
  size_t pos = 0; /* bytes of data consumed */
  int first = 1;
  while (1) {
    size_t fill = 0;
    if (first) {
      blk[0] = prefix;
      fill = 1;
      first = 0;
    }
    size_t take = len - pos < 128 - fill ? len - pos : 128 - fill;
    memcpy(blk + fill, data + pos, take);
    pos += take;
    fill += take;
    done += fill;
    int last = done == total;
    if (last) {
      memset(blk + fill, 0, 128 - fill);
      b2_compress(h, blk, done, 1);
      break;
    }
    b2_compress(h, blk, done, 0);
  }
  memcpy(out, h, 32);
}

static void merkle_root(uint8_t (*nodes)[32], size_t n, uint8_t out[32]) {
  if (n == 0) {
    memset(out, 0, 32);
    return;
  }
  uint8_t buf[64];
  while (n > 1) {
    if (n & 1) memset(nodes[n++], 0, 32);
    for (size_t i = 0; i < n / 2; i++) {
      memcpy(buf, nodes[2 * i], 32);
      memcpy(buf + 32, nodes[2 * i + 1], 32);
      b2_prefixed(1, buf, 64, nodes[i]);
    }
    n /= 2;
  }
  memcpy(out, nodes[0], 32);
}

/* ------------------------------------------------------------------------------------------
 * 2D Red Stuff
 * ---------------------------------------------------------------------------------------- */
void rs2cpu_params(uint32_t n, uint64_t blob_len, uint32_t* kp, uint32_t* ks, uint32_t* s) {
  uint32_t f = (n - 1) / 3;
  *ks = n - f;
  *kp = n - 2 * f;
  uint64_t ns = (uint64_t)(*kp) * (*ks), len = blob_len ? blob_len : 1;
  uint64_t sz = (len + ns - 1) / ns;
  *s = (uint32_t)((sz + 1) / 2 * 2);
}

/* encode_with_metadata: primary [n][ks*s], secondary [n][kp*s], hashes [n][64], blob_id 32 */
int rs2cpu_encode(uint32_t n, const uint8_t* blob, uint64_t blob_len, uint8_t* primary,
                  uint8_t* secondary, uint8_t* hashes, uint8_t* blob_id) {
  rs2cpu_init();
  uint32_t kp, ks, s;
  rs2cpu_params(n, blob_len, &kp, &ks, &s);
  const size_t pl = (size_t)ks * s, sl = (size_t)kp * s;
  const size_t msg = (size_t)kp * pl;
  memset(primary, 0, msg);
  memcpy(primary, blob, blob_len);
  /* rows (secondary encoding) -> secondary slivers ks..n at row r */
  Codec row;
  codec_init(&row, ks, n - ks, s);
  const uint8_t** src = (const uint8_t**)malloc(sizeof(uint8_t*) * n);
  uint8_t** dst = (uint8_t**)malloc(sizeof(uint8_t*) * n);
  for (uint32_t r = 0; r < kp; r++) {
    for (uint32_t c = 0; c < ks; c++) src[c] = primary + r * pl + (size_t)c * s;
    for (uint32_t j = 0; j < n - ks; j++) dst[j] = secondary + (size_t)(ks + j) * sl + (size_t)r * s;
    codec_encode(&row, src, dst);
  }
  codec_free(&row);
  /* systematic secondary slivers */
  for (uint32_t c = 0; c < ks; c++)
    for (uint32_t r = 0; r < kp; r++)
      memcpy(secondary + (size_t)c * sl + (size_t)r * s, primary + r * pl + (size_t)c * s, s);
  /* columns (primary encoding), leaf hashes */
  uint8_t(*leaf)[32] = (uint8_t(*)[32])malloc((size_t)n * n * 32);
  uint8_t* colbuf = (uint8_t*)malloc((size_t)(n - kp) * s);
  Codec col;
  codec_init(&col, kp, n - kp, s);
  for (uint32_t c = 0; c < n; c++) {
    for (uint32_t r = 0; r < kp; r++) src[r] = secondary + (size_t)c * sl + (size_t)r * s;
    for (uint32_t j = 0; j < n - kp; j++)
      dst[j] = c < ks ? primary + (size_t)(kp + j) * pl + (size_t)c * s : colbuf + (size_t)j * s;
    codec_encode(&col, src, dst);
    for (uint32_t r = 0; r < n; r++) {
      const uint8_t* sym = r < kp ? src[r] : dst[r - kp];
      b2_prefixed(0, sym, s, leaf[(size_t)r * n + c]);
    }
  }
  codec_free(&col);
  /* 2n trees, root, blob id */
  uint8_t(*nodes)[32] = (uint8_t(*)[32])malloc((size_t)(n + 1) * 32);
  for (uint32_t i = 0; i < n; i++) {
    memcpy(nodes, leaf[(size_t)i * n], (size_t)n * 32);
    merkle_root(nodes, n, hashes + 64 * (size_t)i);
    for (uint32_t r = 0; r < n; r++) memcpy(nodes[r], leaf[(size_t)r * n + (n - 1 - i)], 32);
    merkle_root(nodes, n, hashes + 64 * (size_t)i + 32);
  }
  for (uint32_t i = 0; i < n; i++) b2_prefixed(0, hashes + 64 * (size_t)i, 64, nodes[i]);
  uint8_t root[32], idmsg[40];
  merkle_root(nodes, n, root);
  for (int i = 0; i < 8; i++) idmsg[i] = (uint8_t)(blob_len >> (8 * i));
  memcpy(idmsg + 8, root, 32);
  b2_prefixed(1, idmsg, 40, blob_id);
  free(nodes);
  free(leaf);
  free(colbuf);
  free(src);
  free(dst);
  return 0;
}

/* BlobDecoder::decode from primary slivers: `count` slivers with indices idx[], data[i] */
int rs2cpu_decode_primary(uint32_t n, uint64_t blob_len, uint32_t count, const uint16_t* idx,
                          const uint8_t* const* data, uint8_t* blob_out) {
  rs2cpu_init();
  uint32_t kp, ks, s;
  rs2cpu_params(n, blob_len, &kp, &ks, &s);
  const uint8_t** present = (const uint8_t**)calloc(n, sizeof(uint8_t*));
  const uint8_t** sliver = (const uint8_t**)calloc(n, sizeof(uint8_t*));
  uint32_t got = 0;
  for (uint32_t i = 0; i < count && got < kp; i++) {
    if (idx[i] >= n || sliver[idx[i]]) continue;
    sliver[idx[i]] = data[i];
    got++;
  }
  if (got < kp) {
    free(present);
    free(sliver);
    return -1;
  }
  const size_t pl = (size_t)ks * s;
  uint8_t* mat = (uint8_t*)malloc((size_t)kp * pl);
  uint8_t** out = (uint8_t**)malloc(sizeof(uint8_t*) * kp);
  Codec col;
  codec_init(&col, kp, n - kp, s);
  int rc = 0;
  for (uint32_t c = 0; c < ks && rc == 0; c++) {
    for (uint32_t q = 0; q < n; q++) present[q] = sliver[q] ? sliver[q] + (size_t)c * s : NULL;
    for (uint32_t r = 0; r < kp; r++) out[r] = mat + r * pl + (size_t)c * s;
    rc = codec_decode(&col, present, out);
  }
  codec_free(&col);
  if (rc == 0) memcpy(blob_out, mat, blob_len);
  free(mat);
  free(out);
  free(present);
  free(sliver);
  return rc;
}

/* ------------------------------------------------------------------------------------------
 * encode_with_metadata on T threads without the n x n leaf array (golden cases at large
 * n_shards, where n^2 leaf digests no longer fit in memory).  Same bytes as rs2cpu_encode:
 *   - rows (secondary code) in parallel; systematic secondary slivers;
 *   - columns in T chunks of CS = pow2(ceil(n / T)) columns (chunk t = [t CS, (t+1) CS)): each
 *     column is encoded (primary code), its n leaves hashed, its tree (the secondary hash of pair
 *     n-1-c) built at once, and every row's leaf pushed into that row's streaming Merkle stack;
 *   - a chunk ends with every row's level-k node of the chunk (k = log2 CS; a complete aligned
 *     subtree, or for the last chunk the padded one -- the global odd-level padding happens
 *     inside it), and each row's tree is finished over its chunks' nodes (merkle.rs:226-266).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  uint32_t n, kp, ks, s, T, t, CS, k;
  uint8_t *primary, *secondary, *hashes;
  uint8_t (*chunk_nodes)[32]; /* [n_chunks][n] */
  int phase;
} MtJob;

static void node_pair(const uint8_t l[32], const uint8_t r[32], uint8_t out[32]) {
  uint8_t buf[64];
  memcpy(buf, l, 32);
  memcpy(buf + 32, r, 32);
  b2_prefixed(1, buf, 64, out);
}

static void* mt_job(void* arg) {
  MtJob* j = (MtJob*)arg;
  const uint32_t n = j->n, kp = j->kp, ks = j->ks, s = j->s;
  const size_t pl = (size_t)ks * s, sl = (size_t)kp * s;
  if (j->phase == 0) { /* rows r = t, t + T, ...: repair symbols of the row code */
    Codec row;
    codec_init(&row, ks, n - ks, s);
    const uint8_t** src = (const uint8_t**)malloc(sizeof(uint8_t*) * n);
    uint8_t** dst = (uint8_t**)malloc(sizeof(uint8_t*) * n);
    for (uint32_t r = j->t; r < kp; r += j->T) {
      for (uint32_t c = 0; c < ks; c++) src[c] = j->primary + r * pl + (size_t)c * s;
      for (uint32_t q = 0; q < n - ks; q++) dst[q] = j->secondary + (size_t)(ks + q) * sl + (size_t)r * s;
      codec_encode(&row, src, dst);
    }
    codec_free(&row);
    free(src);
    free(dst);
    return 0;
  }
  if (j->phase == 1) { /* systematic secondary slivers c = t, t + T, ... */
    for (uint32_t c = j->t; c < ks; c += j->T)
      for (uint32_t r = 0; r < kp; r++)
        memcpy(j->secondary + (size_t)c * sl + (size_t)r * s, j->primary + r * pl + (size_t)c * s, s);
    return 0;
  }
  /* phase 2: the columns of chunk t */
  const uint32_t c0 = j->t * j->CS, c1 = c0 + j->CS < n ? c0 + j->CS : n;
  if (c0 >= n) return 0;
  const uint32_t K = j->k + 1; /* stack levels 0..k */
  uint8_t(*stk)[32] = (uint8_t(*)[32])malloc((size_t)n * K * 32);
  uint32_t* occ = (uint32_t*)calloc(n, sizeof(uint32_t)); /* bit l: level l holds a node */
  uint8_t(*leaf)[32] = (uint8_t(*)[32])malloc(((size_t)n + 1) * 32);
  uint8_t* colbuf = (uint8_t*)malloc((size_t)(n - kp) * s);
  const uint8_t** src = (const uint8_t**)malloc(sizeof(uint8_t*) * n);
  uint8_t** dst = (uint8_t**)malloc(sizeof(uint8_t*) * n);
  Codec col;
  codec_init(&col, kp, n - kp, s);
  static const uint8_t Z[32] = {0};
  uint8_t cur[32];
  for (uint32_t c = c0; c < c1; c++) {
    for (uint32_t r = 0; r < kp; r++) src[r] = j->secondary + (size_t)c * sl + (size_t)r * s;
    for (uint32_t q = 0; q < n - kp; q++)
      dst[q] = c < ks ? j->primary + (size_t)(kp + q) * pl + (size_t)c * s : colbuf + (size_t)q * s;
    codec_encode(&col, src, dst);
    for (uint32_t r = 0; r < n; r++) {
      const uint8_t* sym = r < kp ? src[r] : dst[r - kp];
      b2_prefixed(0, sym, s, leaf[r]);
      /* row r's stack: carry the leaf up while the level is occupied */
      memcpy(cur, leaf[r], 32);
      uint32_t l = 0;
      while (occ[r] >> l & 1u) {
        node_pair(stk[(size_t)r * K + l], cur, cur);
        occ[r] &= ~(1u << l);
        l++;
      }
      memcpy(stk[(size_t)r * K + l], cur, 32);
      occ[r] |= 1u << l;
    }
    merkle_root(leaf, n, j->hashes + 64 * (size_t)(n - 1 - c) + 32); /* column tree */
  }
  /* each row's level-k node of this chunk (padded when the chunk is the last, partial one) */
  for (uint32_t r = 0; r < n; r++) {
    int have = 0;
    for (uint32_t l = 0; l < j->k; l++) {
      const int p = occ[r] >> l & 1u;
      if (p && have) {
        node_pair(stk[(size_t)r * K + l], cur, cur);
      } else if (p) {
        node_pair(stk[(size_t)r * K + l], Z, cur);
        have = 1;
      } else if (have) {
        node_pair(cur, Z, cur);
      }
    }
    if (occ[r] >> j->k & 1u) memcpy(cur, stk[(size_t)r * K + j->k], 32); /* a full chunk */
    memcpy(j->chunk_nodes[(size_t)j->t * n + r], cur, 32);
  }
  codec_free(&col);
  free(stk); free(occ); free(leaf); free(colbuf); free(src); free(dst);
  return 0;
}

int rs2cpu_encode_mt(uint32_t n, const uint8_t* blob, uint64_t blob_len, uint8_t* primary,
                     uint8_t* secondary, uint8_t* hashes, uint8_t* blob_id, int threads) {
  rs2cpu_init();
  if (threads < 2) return rs2cpu_encode(n, blob, blob_len, primary, secondary, hashes, blob_id);
  uint32_t kp, ks, s;
  rs2cpu_params(n, blob_len, &kp, &ks, &s);
  const size_t pl = (size_t)ks * s, msg = (size_t)kp * pl;
  memset(primary, 0, msg);
  memcpy(primary, blob, blob_len);
  const uint32_t T = (uint32_t)threads;
  uint32_t CS = 1, k = 0;
  while (CS < (n + T - 1) / T) CS <<= 1, k++;
  const uint32_t n_chunks = (n + CS - 1) / CS;
  uint8_t(*chunk_nodes)[32] = (uint8_t(*)[32])malloc((size_t)n_chunks * n * 32);
  MtJob* jobs = (MtJob*)calloc(T, sizeof(MtJob));
  pthread_t* th = (pthread_t*)calloc(T, sizeof(pthread_t));
  for (int phase = 0; phase < 3; phase++) {
    for (uint32_t t = 0; t < T; t++) {
      MtJob z = {n, kp, ks, s, T, t, CS, k, primary, secondary, hashes, chunk_nodes, phase};
      jobs[t] = z;
      pthread_create(&th[t], 0, mt_job, &jobs[t]);
    }
    for (uint32_t t = 0; t < T; t++) pthread_join(th[t], 0);
  }
  /* rows: the tree over each row's chunk nodes (level k upward) */
  uint8_t(*nodes)[32] = (uint8_t(*)[32])malloc(((size_t)(n_chunks > n ? n_chunks : n) + 1) * 32);
  for (uint32_t r = 0; r < n; r++) {
    for (uint32_t q = 0; q < n_chunks; q++) memcpy(nodes[q], chunk_nodes[(size_t)q * n + r], 32);
    merkle_root(nodes, n_chunks, hashes + 64 * (size_t)r);
  }
  for (uint32_t i = 0; i < n; i++) b2_prefixed(0, hashes + 64 * (size_t)i, 64, nodes[i]);
  uint8_t root[32], idmsg[40];
  merkle_root(nodes, n, root);
  for (int i = 0; i < 8; i++) idmsg[i] = (uint8_t)(blob_len >> (8 * i));
  memcpy(idmsg + 8, root, 32);
  b2_prefixed(1, idmsg, 40, blob_id);
  free(nodes); free(chunk_nodes); free(jobs); free(th);
  return 0;
}

/* 1D encode_all over `batch` codewords (data stride k*s, out stride n*s) */
int rs2cpu_encode_1d(uint32_t k, uint32_t n, uint32_t s, uint32_t batch, const uint8_t* data,
                     uint8_t* out) {
  rs2cpu_init();
  Codec c;
  codec_init(&c, k, n - k, s);
  const uint8_t** src = (const uint8_t**)malloc(sizeof(uint8_t*) * k);
  uint8_t** dst = (uint8_t**)malloc(sizeof(uint8_t*) * (n - k));
  for (uint32_t b = 0; b < batch; b++) {
    const uint8_t* d = data + (size_t)b * k * s;
    uint8_t* o = out + (size_t)b * n * s;
    memcpy(o, d, (size_t)k * s);
    for (uint32_t i = 0; i < k; i++) src[i] = d + (size_t)i * s;
    for (uint32_t j = 0; j < n - k; j++) dst[j] = o + (size_t)(k + j) * s;
    codec_encode(&c, src, dst);
  }
  codec_free(&c);
  free(src);
  free(dst);
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * Storage-node side: what walrus-service runs per sliver on its CPU pools --
 * SliverData::verify (slivers.rs:100-135, node.rs:2615-2633), recovery_symbol_for_sliver with
 * its Merkle proof (slivers.rs:180-213, recovery_symbol_service.rs:161-235) and sliver recovery
 * from decoding symbols (slivers.rs:246-379, request_futures.rs:436-497).  axis 0 = primary
 * (K_s symbols, expanded with the secondary code), 1 = secondary (K_p symbols, primary code).
 * A per-thread cache keeps the codec of the last two (k, n, s), as the node keeps its encoders.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  uint32_t k, n, s;
  int live;
  Codec c;
} CodecSlot;
static __thread CodecSlot t_codec[2];
static __thread uint8_t* t_buf;  /* n expanded symbols */
static __thread uint8_t (*t_nodes)[32];
static __thread size_t t_buf_len, t_nodes_len;

static Codec* codec_for(uint32_t k, uint32_t n, uint32_t s) {
  for (int i = 0; i < 2; i++)
    if (t_codec[i].live && t_codec[i].k == k && t_codec[i].n == n && t_codec[i].s == s)
      return &t_codec[i].c;
  if (t_codec[1].live) codec_free(&t_codec[1].c);
  t_codec[1] = t_codec[0];
  codec_init(&t_codec[0].c, k, n - k, s);
  t_codec[0].k = k;
  t_codec[0].n = n;
  t_codec[0].s = s;
  t_codec[0].live = 1;
  return &t_codec[0].c;
}

static uint32_t axis_k(uint32_t n, int axis) {
  uint32_t kp, ks, s;
  rs2cpu_params(n, 1, &kp, &ks, &s);
  return axis == 0 ? ks : kp;
}

/* the sliver's n recovery symbols (slivers.rs:169-178) into t_buf, their leaf hashes into
 * t_nodes[0..n) */
static void expand_and_hash(uint32_t n, uint32_t s, int axis, const uint8_t* sliver) {
  const uint32_t k = axis_k(n, axis);
  if (t_buf_len < (size_t)n * s) {
    free(t_buf);
    t_buf = (uint8_t*)malloc((size_t)n * s);
    t_buf_len = (size_t)n * s;
  }
  if (t_nodes_len < (size_t)2 * n + 2) {
    free(t_nodes);
    t_nodes = (uint8_t(*)[32])malloc(((size_t)2 * n + 2) * 32);
    t_nodes_len = (size_t)2 * n + 2;
  }
  memcpy(t_buf, sliver, (size_t)k * s);
  if (n > k) {
    const uint8_t* src[n];
    uint8_t* dst[n];
    for (uint32_t i = 0; i < k; i++) src[i] = t_buf + (size_t)i * s;
    for (uint32_t j = 0; j < n - k; j++) dst[j] = t_buf + (size_t)(k + j) * s;
    codec_encode(codec_for(k, n, s), src, dst);
  }
  for (uint32_t i = 0; i < n; i++) b2_prefixed(0, t_buf + (size_t)i * s, s, t_nodes[i]);
}

/* SliverData::get_merkle_root (slivers.rs:387-392) */
int rs2cpu_sliver_root(uint32_t n, uint32_t s, int axis, const uint8_t* sliver, uint8_t root[32]) {
  rs2cpu_init();
  expand_and_hash(n, s, axis, sliver);
  merkle_root(t_nodes, n, root);
  return 0;
}

/* recovery_symbol_for_sliver: expanded symbol `target` and MerkleTree::get_proof(target)
 * (merkle.rs:281-309: sibling path leaf -> root, odd levels padded with the zero node);
 * proof_out holds path_len * 32 bytes; returns path_len */
int rs2cpu_recovery_symbol(uint32_t n, uint32_t s, int axis, const uint8_t* sliver,
                           uint32_t target, uint8_t* sym_out, uint8_t* proof_out) {
  rs2cpu_init();
  if (target >= n) return -1;
  expand_and_hash(n, s, axis, sliver);
  memcpy(sym_out, t_buf + (size_t)target * s, s);
  uint8_t buf[64];
  uint32_t cnt = n, idx = target, len = 0;
  while (cnt > 1) {
    if (cnt & 1) memset(t_nodes[cnt++], 0, 32);
    memcpy(proof_out + 32 * (size_t)len++, t_nodes[idx ^ 1], 32);
    for (uint32_t i = 0; i < cnt / 2; i++) {
      memcpy(buf, t_nodes[2 * i], 32);
      memcpy(buf + 32, t_nodes[2 * i + 1], 32);
      b2_prefixed(1, buf, 64, t_nodes[i]);
    }
    cnt /= 2;
    idx /= 2;
  }
  return (int)len;
}

/* recover_sliver (slivers.rs:246-289) of `axis` from `count` decoding symbols (symbol i has
 * index idx[i] on the orthogonal axis, its bytes at symbols + i*s; the first k distinct
 * in-range indices are used), then its Merkle root for the verify against the metadata
 * (slivers.rs:341-379).  Returns 0, or -1 when too few symbols. */
int rs2cpu_recover_sliver(uint32_t n, uint32_t s, int axis, uint32_t count, const uint16_t* idx,
                          const uint8_t* symbols, uint8_t* sliver_out, uint8_t root[32]) {
  rs2cpu_init();
  const uint32_t k = axis_k(n, axis);
  const uint8_t* present[n];
  uint8_t* out[k];
  memset(present, 0, sizeof(present));
  uint32_t got = 0;
  for (uint32_t i = 0; i < count && got < k; i++) {
    if (idx[i] >= n || present[idx[i]]) continue;
    present[idx[i]] = symbols + (size_t)i * s;
    got++;
  }
  if (got < k) return -1;
  for (uint32_t i = 0; i < k; i++) out[i] = sliver_out + (size_t)i * s;
  if (codec_decode(codec_for(k, n, s), present, out) != 0) return -1;
  return rs2cpu_sliver_root(n, s, axis, sliver_out, root);
}

/* ------------------------------------------------------------------------------------------
 * CPU baseline driver: encode + decode (random K_p primary subset) of one blob per thread.
 * The reference encodes a blob on one thread and parallelises over blobs at its call sites
 * (rayon over blobs, walrus-sdk/src/node_client.rs:3182), so T threads = T independent blobs.
 *   rs2_cpu_bench N_SHARDS BLOB_BYTES [THREADS]
 * ---------------------------------------------------------------------------------------- */
#ifdef RS2CPU_MAIN
static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static uint64_t rnd(uint64_t* xs) {
  *xs ^= *xs << 13;
  *xs ^= *xs >> 7;
  *xs ^= *xs << 17;
  return *xs;
}
typedef struct {
  uint32_t n;
  uint64_t len, seed;
  double enc_s, dec_s;
  int ok;
} Job;
static void* run_job(void* arg) {
  Job* j = (Job*)arg;
  const uint32_t n = j->n;
  const uint64_t len = j->len;
  uint64_t xs = j->seed;
  uint32_t kp, ks, s;
  rs2cpu_params(n, len, &kp, &ks, &s);
  uint8_t* blob = (uint8_t*)malloc(len);
  for (uint64_t i = 0; i < len; i++) blob[i] = (uint8_t)rnd(&xs);
  uint8_t* prim = (uint8_t*)malloc((size_t)n * ks * s);
  uint8_t* sec = (uint8_t*)malloc((size_t)n * kp * s);
  uint8_t* hashes = (uint8_t*)malloc((size_t)n * 64);
  uint8_t id[32];
  double t0 = now();
  rs2cpu_encode(n, blob, len, prim, sec, hashes, id);
  double t1 = now();
  uint16_t* idx = (uint16_t*)malloc(sizeof(uint16_t) * n);
  for (uint32_t i = 0; i < n; i++) idx[i] = (uint16_t)i;
  for (uint32_t i = n - 1; i > 0; i--) {
    uint32_t k = (uint32_t)(rnd(&xs) % (i + 1));
    uint16_t t = idx[i];
    idx[i] = idx[k];
    idx[k] = t;
  }
  const uint8_t** data = (const uint8_t**)malloc(sizeof(uint8_t*) * kp);
  for (uint32_t i = 0; i < kp; i++) data[i] = prim + (size_t)idx[i] * ks * s;
  uint8_t* dec = (uint8_t*)malloc(len);
  double t2 = now();
  int rc = rs2cpu_decode_primary(n, len, kp, idx, data, dec);
  double t3 = now();
  j->ok = rc == 0 && memcmp(dec, blob, len) == 0;
  j->enc_s = t1 - t0;
  j->dec_s = t3 - t2;
  free(blob); free(prim); free(sec); free(hashes); free(idx); free(data); free(dec);
  return 0;
}
/* node mode: one blob encoded (untimed), then T threads share the storage node's per-sliver
 * work: (1) SliverData::verify of every primary and secondary sliver, (2) one recovery symbol
 * with proof per primary sliver (target pair (i * 7 + 3) mod n), (3) recover_sliver of
 * `recovers` primary slivers from K_s recovery symbols each (the symbols of the expanded row,
 * from secondary slivers n-1, n-2, ...), each verified against the metadata. */
typedef struct {
  uint32_t n, s, kp, ks, T, t, recovers;
  const uint8_t *prim, *sec, *hashes;
  int phase, ok;
  double secs;
} NodeJob;
static void* node_job(void* arg) {
  NodeJob* j = (NodeJob*)arg;
  const uint32_t n = j->n, s = j->s, ks = j->ks, kp = j->kp;
  const size_t pl = (size_t)ks * s, sl = (size_t)kp * s;
  uint8_t root[32];
  j->ok = 1;
  double t0 = now();
  if (j->phase == 0) {
    for (uint32_t q = j->t; q < 2 * n; q += j->T) {
      const int axis = q < n ? 0 : 1;
      const uint32_t i = q < n ? q : q - n;
      rs2cpu_sliver_root(n, s, axis, axis ? j->sec + i * sl : j->prim + i * pl, root);
      const uint32_t pair = axis ? n - 1 - i : i;
      j->ok &= memcmp(root, j->hashes + 64 * (size_t)pair + 32 * axis, 32) == 0;
    }
  } else if (j->phase == 1) {
    uint8_t sym[65536], proof[64 * 32];
    for (uint32_t i = j->t; i < n; i += j->T) {
      const uint32_t target = (i * 7 + 3) % n;
      j->ok &= rs2cpu_recovery_symbol(n, s, 0, j->prim + i * pl, target, sym, proof) > 0;
    }
  } else {
    uint8_t* syms = (uint8_t*)malloc((size_t)ks * s);
    uint8_t* out = (uint8_t*)malloc(pl);
    uint16_t* idx = (uint16_t*)malloc(sizeof(uint16_t) * ks);
    uint8_t proof[64 * 32];
    for (uint32_t r = j->t; r < j->recovers; r += j->T) {
      const uint32_t target = (r * 131) % n;
      /* recovery symbols for primary sliver `target` from secondary slivers c = n-1, n-2, ...:
         symbol c of the target row's expansion (the row code's codeword position c) */
      double u0 = now();
      for (uint32_t q = 0; q < ks; q++) {
        const uint32_t c = n - 1 - q;
        idx[q] = (uint16_t)c;
        rs2cpu_recovery_symbol(n, s, 1, j->sec + c * sl, target, syms + (size_t)q * s, proof);
      }
      j->secs -= now() - u0;  /* symbol generation is the other nodes' work: not timed */
      j->ok &= rs2cpu_recover_sliver(n, s, 0, ks, idx, syms, out, root) == 0 &&
               memcmp(out, j->prim + target * pl, pl) == 0 &&
               memcmp(root, j->hashes + 64 * (size_t)target, 32) == 0;
    }
    free(syms);
    free(out);
    free(idx);
  }
  j->secs += now() - t0;
  return 0;
}
static int node_main(int argc, char** argv) {
  const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000;
  const uint64_t len = argc > 3 ? strtoull(argv[3], 0, 10) : (256u << 20);
  int T = argc > 4 ? atoi(argv[4]) : 1;
  const uint32_t recovers = argc > 5 ? (uint32_t)atoi(argv[5]) : 16;
  if (T < 1) T = 1;
  rs2cpu_init();
  uint32_t kp, ks, s;
  rs2cpu_params(n, len, &kp, &ks, &s);
  uint64_t xs = 0x9E3779B97F4A7C15ULL;
  uint8_t* blob = (uint8_t*)malloc(len);
  for (uint64_t i = 0; i < len; i++) blob[i] = (uint8_t)rnd(&xs);
  uint8_t* prim = (uint8_t*)malloc((size_t)n * ks * s);
  uint8_t* sec = (uint8_t*)malloc((size_t)n * kp * s);
  uint8_t* hashes = (uint8_t*)malloc((size_t)n * 64);
  uint8_t id[32];
  rs2cpu_encode(n, blob, len, prim, sec, hashes, id);
  NodeJob* jobs = (NodeJob*)calloc((size_t)T, sizeof(NodeJob));
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  double wall[3];
  int ok = 1;
  for (int phase = 0; phase < 3; phase++) {
    for (int t = 0; t < T; t++) {
      NodeJob z = {n, s, kp, ks, (uint32_t)T, (uint32_t)t, recovers, prim, sec, hashes, phase, 1, 0.0};
      jobs[t] = z;
    }
    for (int t = 0; t < T; t++) pthread_create(&th[t], 0, node_job, &jobs[t]);
    for (int t = 0; t < T; t++) pthread_join(th[t], 0);
    wall[phase] = 0;
    for (int t = 0; t < T; t++) {
      ok &= jobs[t].ok;
      wall[phase] = wall[phase] > jobs[t].secs ? wall[phase] : jobs[t].secs;  /* slowest thread */
    }
  }
  const double vbytes = (double)n * (ks + kp) * s;
  const uint32_t per_thread = (recovers + T - 1) / T;
  printf("{\"cores\": %d, \"n\": %u, \"symbol_size\": %u, "
         "\"verify_slivers_per_s\": %.2f, \"verify_gibs\": %.6f, \"verify_s\": %.4f, "
         "\"recovery_symbols_per_s\": %.2f, \"recovery_symbols_s\": %.4f, "
         "\"recover_sliver_ms\": %.4f, \"recovers\": %u, \"ok\": %s, "
         "\"sample\": \"C/AVX2 restatement (oracle/rs2_cpu.c), %d thread(s), one %.1f MiB blob at "
         "n=%u (s=%u): verify of all %u primary + %u secondary slivers, %u recovery symbols with "
         "proofs, %u primary-sliver recoveries from K_s symbols (each verified)\"}\n",
         T, n, s, 2.0 * n / wall[0], vbytes / wall[0] / (1u << 30), wall[0], n / wall[1], wall[1],
         wall[2] / per_thread * 1e3, recovers, ok ? "true" : "false", T, len / 1048576.0, n, s, n,
         n, n, recovers);
  free(blob); free(prim); free(sec); free(hashes); free(jobs); free(th);
  return ok ? 0 : 1;
}

/* c3 mode (BASELINE config C3's CPU twin): `blobs` independent blobs of `len` bytes, generated
 * untimed, then T threads encode_with_metadata them, thread t taking blobs t, t + T, ... one at a
 * time -- the reference's rayon over blobs (walrus-sdk/src/node_client.rs:3182, into_par_iter
 * over the blobs, each encoded on one thread).  Timed: the wall time of the encodes.  Every
 * BlobId is checked against a serial re-encode of the same blob after the timed region. */
typedef struct {
  uint32_t n, t, T, blobs;
  uint64_t len;
  const uint8_t* data;
  uint8_t* ids;
} C3Job;
static void* c3_job(void* arg) {
  C3Job* j = (C3Job*)arg;
  uint32_t kp, ks, s;
  rs2cpu_params(j->n, j->len, &kp, &ks, &s);
  uint8_t* prim = (uint8_t*)malloc((size_t)j->n * ks * s);
  uint8_t* sec = (uint8_t*)malloc((size_t)j->n * kp * s);
  uint8_t* hashes = (uint8_t*)malloc((size_t)j->n * 64);
  for (uint32_t b = j->t; b < j->blobs; b += j->T)
    rs2cpu_encode(j->n, j->data + (size_t)b * j->len, j->len, prim, sec, hashes, j->ids + 32 * (size_t)b);
  free(prim); free(sec); free(hashes);
  return 0;
}
static int c3_main(int argc, char** argv) {
  const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000;
  const uint64_t len = argc > 3 ? strtoull(argv[3], 0, 10) : (4u << 20);
  const uint32_t blobs = argc > 4 ? (uint32_t)atoi(argv[4]) : 128;
  int T = argc > 5 ? atoi(argv[5]) : 1;
  if (T < 1) T = 1;
  if ((uint32_t)T > blobs) T = (int)blobs;
  rs2cpu_init();
  uint32_t kp, ks, s;
  rs2cpu_params(n, len, &kp, &ks, &s);
  uint8_t* data = (uint8_t*)malloc((size_t)blobs * len);
  uint64_t xs = 0x243F6A8885A308D3ULL;
  for (uint64_t i = 0; i < (uint64_t)blobs * len; i++) data[i] = (uint8_t)rnd(&xs);
  uint8_t* ids = (uint8_t*)calloc(blobs, 32);
  C3Job* jobs = (C3Job*)calloc((size_t)T, sizeof(C3Job));
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  const double w0 = now();
  for (int t = 0; t < T; t++) {
    C3Job z = {n, (uint32_t)t, (uint32_t)T, blobs, len, data, ids};
    jobs[t] = z;
    pthread_create(&th[t], 0, c3_job, &jobs[t]);
  }
  for (int t = 0; t < T; t++) pthread_join(th[t], 0);
  const double secs = now() - w0;
  /* check: the first and last blobs' ids from a serial re-encode (untimed) */
  int ok = 1;
  {
    uint8_t* prim = (uint8_t*)malloc((size_t)n * ks * s);
    uint8_t* sec = (uint8_t*)malloc((size_t)n * kp * s);
    uint8_t* hashes = (uint8_t*)malloc((size_t)n * 64);
    uint8_t id[32];
    const uint32_t check[2] = {0, blobs - 1};
    for (int c = 0; c < 2; c++) {
      rs2cpu_encode(n, data + (size_t)check[c] * len, len, prim, sec, hashes, id);
      ok &= memcmp(id, ids + 32 * (size_t)check[c], 32) == 0;
    }
    free(prim); free(sec); free(hashes);
  }
  printf("{\"encode_gibs\": %.6f, \"cores\": %d, \"blobs\": %u, \"blob_bytes\": %llu, "
         "\"symbol_size\": %u, \"wall_s\": %.4f, \"ok\": %s, \"sample\": \"C/AVX2 restatement "
         "(oracle/rs2_cpu.c), %d thread(s), %u blobs of %.1f MiB at n=%u (s=%u), one blob per thread "
         "at a time (rayon over blobs): encode_with_metadata\"}\n",
         (double)blobs * len / (1u << 30) / secs, T, blobs, (unsigned long long)len, s, secs,
         ok ? "true" : "false", T, blobs, len / 1048576.0, n, s);
  free(data); free(ids); free(jobs); free(th);
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "node") == 0) return node_main(argc, argv);
  if (argc > 1 && strcmp(argv[1], "c3") == 0) return c3_main(argc, argv);
  uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
  uint64_t len = argc > 2 ? strtoull(argv[2], 0, 10) : (16u << 20);
  int threads = argc > 3 ? atoi(argv[3]) : 1;
  if (threads < 1) threads = 1;
  rs2cpu_init();
  uint32_t kp, ks, s;
  rs2cpu_params(n, len, &kp, &ks, &s);
  Job* jobs = (Job*)calloc((size_t)threads, sizeof(Job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t].n = n;
    jobs[t].len = len;
    jobs[t].seed = 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL * (uint64_t)t;
  }
  double w0 = now();
  if (threads == 1) {
    run_job(&jobs[0]);
  } else {
    for (int t = 0; t < threads; t++) pthread_create(&th[t], 0, run_job, &jobs[t]);
    for (int t = 0; t < threads; t++) pthread_join(th[t], 0);
  }
  double w1 = now();
  int ok = 1;
  double enc = 0, dec = 0;
  for (int t = 0; t < threads; t++) {
    ok &= jobs[t].ok;
    enc += jobs[t].enc_s;
    dec += jobs[t].dec_s;
  }
  double gib = (double)len * threads / (1u << 30);
  /* one thread: the timed encode + decode alone (blob generation excluded); several: wall time
     of all threads, each generating, encoding and decoding its own blob, minus the mean
     generation time (enc/dec of the slowest thread bound the wall) */
  double secs = threads == 1 ? jobs[0].enc_s + jobs[0].dec_s : (w1 - w0);
  if (threads > 1) {
    double work = 0;
    for (int t = 0; t < threads; t++) work = work > jobs[t].enc_s + jobs[t].dec_s ? work : jobs[t].enc_s + jobs[t].dec_s;
    secs = work;  /* the slowest thread's timed encode + decode (all ran concurrently) */
  }
  printf("{\"gibs\": %.6f, \"cores\": %d, \"encode_s\": %.4f, \"decode_s\": %.4f, \"ok\": %s, "
         "\"wall_s\": %.3f, \"sample\": \"C/AVX2 restatement (oracle/rs2_cpu.c), %d thread(s), "
         "one %.1f MiB blob per thread at n=%u (s=%u): encode_with_metadata + primary decode from "
         "%u random slivers\"}\n",
         gib / secs, threads, enc / threads, dec / threads, ok ? "true" : "false", w1 - w0, threads,
         len / 1048576.0, n, s, kp);
  free(jobs);
  free(th);
  return ok ? 0 : 1;
}
#endif
