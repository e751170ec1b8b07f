/*
 * fpset_cpu.c — CPU COMPARATOR for the FPSet stress (TEST INFRASTRUCTURE /
 * bench.py cpu_baseline only; never part of the product).
 *
 * BASELINE.json configs[3] / SURVEY §8(d) config 4 on the host: a
 * multithreaded open-addressing fingerprint set in host RAM with the same
 * shape as the GPU FPSet (u64 slots, 0 = empty, MSB clear, linear probing,
 * insert = load then 64-bit CAS into the empty slot; TLC's in-memory FPSets
 * are built the same way [ext-TLC]).  Threads take disjoint slices of a
 * stream of distinct 63-bit fingerprints (a bijective mix of seed + i), insert
 * them into one table sized for the target load, then look up as many (half
 * present, half absent).  Reports inserts/s and lookups/s.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "kubeapi_oracle.h"

static inline uint64_t fc_mix(uint64_t z) {       /* bijective (splitmix64 finaliser) */
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
/* distinct 63-bit fingerprints: the mix is a bijection of 64-bit words, so
 * entries i != j differ; the MSB is folded into bit 0 and 0 is remapped,
 * which keeps them distinct with overwhelming probability (checked below) */
static inline uint64_t fc_fp(uint64_t seed, uint64_t i) {
  uint64_t x = fc_mix(seed + i);
  x = (x & 0x7fffffffffffffffull) ^ (x >> 63);
  return x ? x : 1;
}

typedef struct {
  uint64_t *slots, mask;
  uint64_t seed, n, lo, hi;    /* this thread's slice [lo, hi) of the stream */
  int lookup;                  /* 0 insert, 1 lookup (odd entries: absent stream) */
  uint64_t hits, fresh;
} fc_job;

static void *fc_worker(void *arg) {
  fc_job *j = (fc_job *)arg;
  uint64_t *t = j->slots, mask = j->mask;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint64_t fp = j->lookup ? ((i & 1) ? fc_fp(j->seed ^ 0xabcdef12345ull, i) : fc_fp(j->seed, i))
                                  : fc_fp(j->seed, i);
    uint64_t s = (fp * 0x9e3779b97f4a7c15ull) >> 17 & mask;
    for (;;) {
      uint64_t e = __atomic_load_n(&t[s], __ATOMIC_RELAXED);
      if (e == fp) { j->hits++; break; }
      if (e == 0) {
        if (j->lookup) break;
        uint64_t z = 0;
        if (__atomic_compare_exchange_n(&t[s], &z, fp, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) { j->fresh++; break; }
        if (z == fp) { j->hits++; break; }
      }
      s = (s + 1) & mask;
    }
  }
  return NULL;
}

static double fc_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int fc_phase(uint64_t *slots, uint64_t mask, uint64_t seed, uint64_t n, int threads, int lookup,
                    double *secs, uint64_t *hits, uint64_t *fresh) {
  pthread_t th[256];
  fc_job jobs[256];
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  const double t0 = fc_now();
  for (int k = 0; k < threads; k++) {
    jobs[k] = (fc_job){slots, mask, seed, n, n * k / threads, n * (k + 1) / threads, lookup, 0, 0};
    if (pthread_create(&th[k], NULL, fc_worker, &jobs[k]) != 0) return -1;
  }
  *hits = *fresh = 0;
  for (int k = 0; k < threads; k++) {
    pthread_join(th[k], NULL);
    *hits += jobs[k].hits;
    *fresh += jobs[k].fresh;
  }
  *secs = fc_now() - t0;
  return 0;
}

int ko_fpset_stress_cpu(uint64_t n, double load, int threads, uint64_t seed, ko_fpset_cpu_result *out) {
  memset(out, 0, sizeof *out);
  if (n == 0 || load <= 0 || load >= 1) return -1;
  uint64_t slots = 1024;
  while ((double)n / (double)slots > load) slots *= 2;
  const size_t bytes = slots * sizeof(uint64_t);
  uint64_t *t = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (t == MAP_FAILED) return -2;
  madvise(t, bytes, MADV_HUGEPAGE);
  memset(t, 0, bytes);                 /* fault the pages in before timing */
  uint64_t hits = 0, fresh = 0;
  if (fc_phase(t, slots - 1, seed, n, threads, 0, &out->insert_seconds, &hits, &fresh) != 0) {
    munmap(t, bytes);
    return -3;
  }
  out->inserted = fresh;
  out->duplicates = hits;
  if (fc_phase(t, slots - 1, seed, n, threads, 1, &out->lookup_seconds, &hits, &fresh) != 0) {
    munmap(t, bytes);
    return -3;
  }
  out->found = hits;
  out->slots = slots;
  out->threads = threads;
  out->inserts_per_s = n / out->insert_seconds;
  out->lookups_per_s = n / out->lookup_seconds;
  munmap(t, bytes);
  return 0;
}
