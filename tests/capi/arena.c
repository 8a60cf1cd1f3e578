/* Plan churn through the C ABI without device allocations: a blob store's encode / decode
 * traffic is blobs of every length, and the reference builds a BlobEncoder / BlobDecoder per
 * call (config.rs:545-567, 591-603).  Here T OS threads share one plan cache keyed by symbol
 * size (plans rebound per call with rs2_plan_rebind, least-recently-used plans destroyed past
 * CACHE entries) and run encode_with_metadata + decode_and_verify (Default, from a rotating
 * K_p subset of primary slivers) over L distinct blob lengths, log-spaced from 1 KiB to
 * max_bytes, in waves of T (one length per thread, a barrier between waves).
 *
 * The first pass warms the device arena and the pinned staging pool; further passes over the
 * same lengths follow until one calls hipMalloc zero times and pins no host memory
 * (rs2_device_memory_stats) -- at most `warm` more: the threads' interleaving decides which
 * blocks are live together, so an early pass may still meet a new combination.  Every decoded
 * blob must equal its input and every blob id the first pass's.  Every pass starts from an
 * empty plan cache.  Prints the arena's peak live bytes and its reserve (the bounded device
 * footprint: cached plans plus calls in flight, within the reserved segments).
 *
 *   usage: arena [threads=8] [lengths=200] [n_shards=1000] [max_bytes=268435456] [cache=8]
 *                [warm=6] [churn]
 *   prints "arena ok ..." and exits 0, or "FAIL ..." and exits 1.
 *
 * `churn` (more device memory live than the arena keeps cached, RS2_ARENA_CACHE_MIB,
 * default 8 GiB): exactly warm + 1 passes, no allocation-free pass expected; instead the live
 * peak must pass the cap, segments that fall wholly free past it must have gone back to hipFree
 * during the passes (their hipFree runs outside the arena lock while the other threads keep
 * allocating), the reserve must end below the peak, and every blob id / decode must still
 * match.  Prints "arena churn ok ...".
 */
#include <pthread.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/walrus_rs2.h"

typedef struct {
  uint16_t s;
  rs2_plan* plan;
  pthread_mutex_t lock; /* one call at a time per plan (include/walrus_rs2.h threading rule) */
  int refs;
  uint64_t last_use;
} Entry;

static struct {
  pthread_mutex_t mu;
  Entry* e[64];
  int count, cap;
  uint64_t clock;
} g_cache = {PTHREAD_MUTEX_INITIALIZER, {0}, 0, 8, 0};

static uint16_t g_n;
static int g_threads, g_lengths, g_pass;
static uint64_t* g_len;   /* lengths, processing order */
static uint8_t (*g_ids)[32];
static pthread_barrier_t g_bar;
static int g_failed;
static char g_why[512];
static pthread_mutex_t g_fail_mu = PTHREAD_MUTEX_INITIALIZER;

static void fail(const char* msg, uint64_t len, int rc) {
  pthread_mutex_lock(&g_fail_mu);
  if (!g_failed) snprintf(g_why, sizeof g_why, "%s (len %llu, rc %d: %s)", msg,
                          (unsigned long long)len, rc, rs2_last_error());
  g_failed = 1;
  pthread_mutex_unlock(&g_fail_mu);
}

/* the cached plan of len's symbol size, locked and rebound to len (NULL on error) */
static Entry* acquire(uint64_t len, int* rc) {
  uint16_t s = 0;
  if ((*rc = rs2_symbol_size_for_blob(g_n, len, &s)) != RS2_OK) return NULL;
  Entry* victims[64];
  int nv = 0;
  Entry* hit = NULL;
  pthread_mutex_lock(&g_cache.mu);
  for (int i = 0; i < g_cache.count; ++i)
    if (g_cache.e[i]->s == s) hit = g_cache.e[i];
  if (!hit) {
    hit = (Entry*)calloc(1, sizeof(Entry));
    hit->s = s;
    pthread_mutex_init(&hit->lock, NULL);
    g_cache.e[g_cache.count++] = hit;
  }
  hit->refs++;
  hit->last_use = ++g_cache.clock;
  while (g_cache.count > g_cache.cap) { /* evict the least recently used idle plan */
    int v = -1;
    for (int i = 0; i < g_cache.count; ++i)
      if (g_cache.e[i]->refs == 0 && (v < 0 || g_cache.e[i]->last_use < g_cache.e[v]->last_use))
        v = i;
    if (v < 0) break;
    victims[nv++] = g_cache.e[v];
    g_cache.e[v] = g_cache.e[--g_cache.count];
  }
  pthread_mutex_unlock(&g_cache.mu);
  for (int i = 0; i < nv; ++i) {
    rs2_plan_destroy(victims[i]->plan);
    pthread_mutex_destroy(&victims[i]->lock);
    free(victims[i]);
  }
  pthread_mutex_lock(&hit->lock);
  *rc = hit->plan ? rs2_plan_rebind(hit->plan, len) : rs2_plan_create(g_n, len, &hit->plan);
  if (*rc != RS2_OK) {
    pthread_mutex_unlock(&hit->lock);
    pthread_mutex_lock(&g_cache.mu);
    hit->refs--;
    pthread_mutex_unlock(&g_cache.mu);
    return NULL;
  }
  return hit;
}

static void release(Entry* e) {
  pthread_mutex_unlock(&e->lock);
  pthread_mutex_lock(&g_cache.mu);
  e->refs--;
  pthread_mutex_unlock(&g_cache.mu);
}

static void fill(uint8_t* p, uint64_t len, uint64_t seed) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  uint64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    memcpy(p + i, &x, 8);
  }
  for (; i < len; ++i) p[i] = (uint8_t)(x >> (8 * (i & 7)));
}

static int g_trace;

static void one(uint64_t len, int item) {
  int rc = 0;
  if (g_trace) {
    printf("start pass %d item %d len %llu\n", g_pass, item, (unsigned long long)len);
    fflush(stdout);
  }
  uint8_t *blob = NULL, *prim = NULL, *out = NULL;
  uint8_t** pp = NULL;
  const uint8_t** sl = NULL;
  uint16_t *idx = NULL, *syms = NULL;
  uint64_t* lens = NULL;
  uint8_t id[32];
  Entry* e = acquire(len, &rc);
  if (!e) {
    fail("plan", len, rc);
    return;
  }
  rs2_plan_info info;
  rs2_plan_info_get(e->plan, &info);
  const uint16_t n = info.n_shards, kp = info.n_primary;
  const uint64_t pl = info.primary_sliver_len;
  blob = (uint8_t*)malloc(len ? len : 1);
  prim = (uint8_t*)malloc((size_t)n * pl);
  out = (uint8_t*)malloc(len ? len : 1);
  pp = (uint8_t**)malloc(n * sizeof *pp);
  sl = (const uint8_t**)malloc(kp * sizeof *sl);
  idx = (uint16_t*)malloc(kp * sizeof *idx);
  syms = (uint16_t*)malloc(kp * sizeof *syms);
  lens = (uint64_t*)malloc(kp * sizeof *lens);
  uint8_t* hashes = (uint8_t*)malloc((size_t)n * 64);
  if (!blob || !prim || !out || !pp || !sl || !idx || !syms || !lens || !hashes) {
    fail("host allocation", len, 0);
    goto done;
  }
  fill(blob, len, len);
  for (int i = 0; i < n; ++i) pp[i] = prim + (size_t)i * pl;
  /* primary slivers only: the secondary codecs still run (their hashes are in the metadata) */
  if ((rc = rs2_encode_with_metadata(e->plan, blob, pp, NULL, hashes, id)) != RS2_OK) {
    fail("encode_with_metadata", len, rc);
    goto done;
  }
  const uint16_t rot = (uint16_t)((item * 97) % n);
  for (int i = 0; i < kp; ++i) {
    idx[i] = (uint16_t)((rot + i) % n);
    sl[i] = pp[idx[i]];
    lens[i] = pl;
    syms[i] = info.symbol_size;
  }
  rc = rs2_decode_and_verify(e->plan, RS2_AXIS_PRIMARY, kp, idx, sl, lens, syms, hashes, id,
                             RS2_CHECK_DEFAULT, out);
  if (rc != RS2_OK) {
    fail("decode_and_verify", len, rc);
    goto done;
  }
  if (len && memcmp(out, blob, len) != 0) {
    fail("decoded blob differs", len, 0);
    goto done;
  }
  if (g_pass == 0)
    memcpy(g_ids[item], id, 32);
  else if (memcmp(g_ids[item], id, 32) != 0)
    fail("blob id differs from pass 1", len, 0);
done:
  release(e);
  free(blob), free(prim), free(out), free(pp), free(sl), free(idx), free(syms), free(lens);
  free(hashes);
}

static void* worker(void* arg) {
  const int t = (int)(intptr_t)arg;
  for (int w = 0; w * g_threads < g_lengths; ++w) {
    const int item = w * g_threads + t;
    if (item < g_lengths && !g_failed) one(g_len[item], item);
    pthread_barrier_wait(&g_bar);
  }
  return NULL;
}

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void clear_cache(void) {
  for (int i = 0; i < g_cache.count; ++i) {
    rs2_plan_destroy(g_cache.e[i]->plan);
    pthread_mutex_destroy(&g_cache.e[i]->lock);
    free(g_cache.e[i]);
  }
  g_cache.count = 0;
}

static int run_pass(int pass) {
  g_pass = pass;
  pthread_t th[64];
  pthread_barrier_init(&g_bar, NULL, (unsigned)g_threads);
  for (int t = 0; t < g_threads; ++t) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < g_threads; ++t) pthread_join(th[t], NULL);
  pthread_barrier_destroy(&g_bar);
  clear_cache();
  return !g_failed;
}

int main(int argc, char** argv) {
  g_threads = argc > 1 ? atoi(argv[1]) : 8;
  g_lengths = argc > 2 ? atoi(argv[2]) : 200;
  g_n = (uint16_t)(argc > 3 ? atoi(argv[3]) : 1000);
  const uint64_t max_bytes = argc > 4 ? strtoull(argv[4], NULL, 10) : (uint64_t)256 << 20;
  g_cache.cap = argc > 5 ? atoi(argv[5]) : 8;
  g_trace = getenv("ARENA_TRACE") != NULL;
  setvbuf(stdout, NULL, _IOLBF, 0);
  if (g_threads < 1 || g_threads > 64 || g_lengths < 2 || g_cache.cap < 1 || g_cache.cap > 32) {
    printf("FAIL bad arguments\n");
    return 1;
  }
  g_len = (uint64_t*)malloc(g_lengths * sizeof *g_len);
  g_ids = malloc((size_t)g_lengths * 32);
  /* distinct log-spaced lengths (odd offsets keep them off round sizes), then a fixed shuffle
   * so every wave mixes large and small blobs */
  const double lo = log(1024.0), hi = log((double)max_bytes);
  uint64_t prev = 0;
  for (int i = 0; i < g_lengths; ++i) {
    uint64_t v = (uint64_t)exp(lo + (hi - lo) * i / (g_lengths - 1)) - (uint64_t)(i % 7) * 3;
    if (v <= prev) v = prev + 1;
    if (v > max_bytes) v = max_bytes;
    g_len[i] = prev = v;
  }
  uint64_t x = 0x243F6A8885A308D3ull;
  for (int i = g_lengths - 1; i > 0; --i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const int j = (int)(x % (uint64_t)(i + 1));
    const uint64_t tmp = g_len[i];
    g_len[i] = g_len[j], g_len[j] = tmp;
  }
  const int warm = argc > 6 ? atoi(argv[6]) : 6;
  const int churn = argc > 7 && strcmp(argv[7], "churn") == 0;
  uint64_t s0[7], a[7], b[7];
  rs2_device_memory_stats(0, s0);
  const double t0 = now();
  int clean = -1;
  for (int pass = 0; pass <= warm && (clean < 0 || churn); ++pass) {
    rs2_device_memory_stats(0, a);
    const double ta = now();
    if (!run_pass(pass)) {
      printf("FAIL pass %d: %s\n", pass + 1, g_why);
      return 1;
    }
    rs2_device_memory_stats(0, b);
    printf("pass %d: %.2f s, %llu hipMalloc, %llu hipFree, %llu pinned allocs, %llu quarantine "
           "syncs\n", pass + 1, now() - ta, (unsigned long long)(b[0] - a[0]),
           (unsigned long long)(b[1] - a[1]), (unsigned long long)(b[6] - a[6]),
           (unsigned long long)(b[5] - a[5]));
    if (pass > 0 && b[0] == a[0] && b[6] == a[6]) clean = pass;
  }
  printf("%.2f s, %llu hipMalloc in all; peak live %.1f MiB, reserved %.1f MiB, live with "
         "every plan destroyed %.1f MiB (device context tables)\n", now() - t0,
         (unsigned long long)(b[0] - s0[0]), b[4] / 1048576.0, b[3] / 1048576.0,
         b[2] / 1048576.0);
  if (churn) {
    const char* e = getenv("RS2_ARENA_CACHE_MIB");
    const uint64_t cap = (uint64_t)(e ? atoi(e) : 8192) << 20;
    const uint64_t frees = b[1] - s0[1];
    if (b[4] <= cap || frees == 0 || b[3] >= b[4]) {
      printf("FAIL churn: peak live %llu vs cap %llu, %llu hipFree, reserved %llu\n",
             (unsigned long long)b[4], (unsigned long long)cap, (unsigned long long)frees,
             (unsigned long long)b[3]);
      return 1;
    }
    printf("arena churn ok threads=%d lengths=%d passes=%d peak_mib=%.1f cap_mib=%.1f "
           "hipFree=%llu reserved_mib=%.1f\n", g_threads, g_lengths, warm + 1,
           b[4] / 1048576.0, cap / 1048576.0, (unsigned long long)frees, b[3] / 1048576.0);
    return 0;
  }
  if (clean < 0) {
    printf("FAIL no pass without allocations after %d warm-up passes\n", warm);
    return 1;
  }
  printf("arena ok threads=%d lengths=%d n=%u max=%llu warm_passes=%d peak_mib=%.1f\n",
         g_threads, g_lengths, (unsigned)g_n, (unsigned long long)max_bytes, clean,
         b[4] / 1048576.0);
  return 0;
}
