/* Threading contract of the C ABI as a Rust caller would exercise it: plain C against
 * include/walrus_rs2.h, linked to libwalrus_rs2.so with the system ROCm runtime (no torch, no
 * Python in the process).  T OS threads each create their own plan and, R times, encode a
 * blob of their own with encode_with_metadata, decode it back from a random K_p subset of its
 * primary slivers, run decode_and_verify (Default and Strict) and verify a batch of slivers
 * with rs2_sliver_merkle_roots -- all concurrently, as rayon / tokio blocking threads call the
 * reference (walrus-sdk/src/node_client.rs:3182, walrus-service/src/node.rs:2615-2633).
 * Afterwards the main thread re-encodes every thread's blobs serially and checks the blob ids.
 *
 *   usage: threads [threads=6] [rounds=3] [n_shards=1000] [blob_bytes=4194304]
 *   prints one line "threads ok ..." and exits 0, or "FAIL ..." and exits 1.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/walrus_rs2.h"

typedef struct {
  int id, rounds;
  uint16_t n;
  uint64_t len;
  uint8_t blob_ids[16][32];
  int failed;
  char why[256];
} Job;

static uint64_t next(uint64_t* x) {
  *x ^= *x << 13;
  *x ^= *x >> 7;
  *x ^= *x << 17;
  return *x;
}

static void fill(uint8_t* p, uint64_t len, uint64_t seed) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  for (uint64_t i = 0; i < len; ++i) p[i] = (uint8_t)(next(&x) >> 24);
}

#define CHECK(cond, ...)                               \
  do {                                                 \
    if (!(cond)) {                                     \
      snprintf(job->why, sizeof job->why, __VA_ARGS__); \
      job->failed = 1;                                 \
      goto done;                                       \
    }                                                  \
  } while (0)

static void* worker(void* arg) {
  Job* job = (Job*)arg;
  rs2_plan* plan = NULL;
  rs2_plan_info info;
  uint8_t *blob = NULL, *prim = NULL, *sec = NULL, *out = NULL, *roots = NULL;
  uint8_t** pp = NULL;
  uint8_t** sp = NULL;
  const uint8_t** sl = NULL;
  uint16_t* idx = NULL;
  uint64_t* lens = NULL;
  uint8_t hashes[2048 * 64], bid[32];
  int rc = rs2_plan_create(job->n, job->len, &plan);
  CHECK(rc == RS2_OK, "plan_create rc=%d %s", rc, rs2_last_error());
  rs2_plan_info_get(plan, &info);
  const uint16_t n = info.n_shards, kp = info.n_primary;
  const uint64_t pl = info.primary_sliver_len, sll = info.secondary_sliver_len;
  blob = malloc(job->len);
  prim = malloc(n * pl);
  sec = malloc(n * sll);
  out = malloc(job->len);
  roots = malloc((size_t)n * 32);
  pp = malloc(n * sizeof *pp);
  sp = malloc(n * sizeof *sp);
  sl = malloc(n * sizeof *sl);
  idx = malloc(n * sizeof *idx);
  lens = malloc(n * sizeof *lens);
  for (int i = 0; i < n; ++i) {
    pp[i] = prim + i * pl;
    sp[i] = sec + i * sll;
  }
  uint64_t rng = 12345 + job->id;
  for (int r = 0; r < job->rounds; ++r) {
    fill(blob, job->len, (uint64_t)job->id * 100 + r);
    rc = rs2_encode_with_metadata(plan, blob, pp, sp, hashes, bid);
    CHECK(rc == RS2_OK, "encode rc=%d %s", rc, rs2_last_error());
    memcpy(job->blob_ids[r], bid, 32);
    /* random K_p primary slivers */
    for (int i = 0; i < n; ++i) idx[i] = (uint16_t)i;
    for (int i = n - 1; i > 0; --i) {
      int j = (int)(next(&rng) % (uint64_t)(i + 1));
      uint16_t t = idx[i];
      idx[i] = idx[j];
      idx[j] = t;
    }
    for (int i = 0; i < kp; ++i) {
      sl[i] = pp[idx[i]];
      lens[i] = pl;
    }
    memset(out, 0, job->len);
    rc = rs2_decode_blob(plan, RS2_AXIS_PRIMARY, kp, idx, sl, lens, NULL, out);
    CHECK(rc == RS2_OK && memcmp(out, blob, job->len) == 0, "decode rc=%d", rc);
    for (int check = RS2_CHECK_DEFAULT; check <= RS2_CHECK_STRICT; ++check) {
      memset(out, 0, job->len);
      rc = rs2_decode_and_verify(plan, RS2_AXIS_PRIMARY, kp, idx, sl, lens, NULL, hashes, bid,
                                 check, out);
      CHECK(rc == RS2_OK && memcmp(out, blob, job->len) == 0, "decode_and_verify(%d) rc=%d",
            check, rc);
    }
    /* the node's sliver verification: every primary sliver's root = its metadata hash */
    for (int i = 0; i < n; ++i) lens[i] = pl;
    rc = rs2_sliver_merkle_roots(n, info.symbol_size, RS2_AXIS_PRIMARY, n,
                                 (const uint8_t* const*)pp, lens, roots);
    CHECK(rc == RS2_OK, "sliver roots rc=%d", rc);
    for (int i = 0; i < n; ++i)
      CHECK(memcmp(roots + 32 * i, hashes + 64 * i, 32) == 0, "sliver %d root mismatch", i);
  }
done:
  if (plan) rs2_plan_destroy(plan);
  free(blob);
  free(prim);
  free(sec);
  free(out);
  free(roots);
  free(pp);
  free(sp);
  free(sl);
  free(idx);
  free(lens);
  return NULL;
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 6;
  const int R = argc > 2 ? atoi(argv[2]) : 3;
  const uint16_t n = (uint16_t)(argc > 3 ? atoi(argv[3]) : 1000);
  const uint64_t len = argc > 4 ? strtoull(argv[4], NULL, 10) : (4u << 20);
  if (T < 1 || T > 64 || R < 1 || R > 16) return 2;
  if (!rs2_device_available()) {
    printf("FAIL no device\n");
    return 1;
  }
  Job* jobs = calloc((size_t)T, sizeof *jobs);
  pthread_t* th = malloc((size_t)T * sizeof *th);
  for (int t = 0; t < T; ++t) {
    jobs[t].id = t;
    jobs[t].rounds = R;
    jobs[t].n = n;
    jobs[t].len = len + (uint64_t)t * 4099; /* a different blob size (plan) per thread */
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  int bad = 0;
  for (int t = 0; t < T; ++t)
    if (jobs[t].failed) {
      printf("FAIL thread %d: %s\n", t, jobs[t].why);
      bad = 1;
    }
  /* serial re-encode: the concurrent blob ids were the deterministic ones */
  for (int t = 0; t < T && !bad; ++t) {
    rs2_plan* plan = NULL;
    if (rs2_plan_create(n, jobs[t].len, &plan) != RS2_OK) return 1;
    uint8_t* blob = malloc(jobs[t].len);
    uint8_t bid[32];
    for (int r = 0; r < R && !bad; ++r) {
      fill(blob, jobs[t].len, (uint64_t)t * 100 + r);
      if (rs2_compute_metadata(plan, blob, NULL, bid) != RS2_OK ||
          memcmp(bid, jobs[t].blob_ids[r], 32) != 0) {
        printf("FAIL serial re-encode of thread %d round %d differs\n", t, r);
        bad = 1;
      }
    }
    free(blob);
    rs2_plan_destroy(plan);
  }
  if (!bad) printf("threads ok: %d threads x %d rounds, n=%u, %llu-byte blobs\n", T, R, n,
                   (unsigned long long)len);
  free(jobs);
  free(th);
  return bad;
}
