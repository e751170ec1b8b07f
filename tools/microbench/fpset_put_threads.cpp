// fpset_put_threads.cpp — TLC's FPSet seam as TLC drives it: T host threads
// (TLC's -workers) each calling kc_fpset_put(fp) one fingerprint at a time
// (FPSet.put(long) is per state, MC.out:5).  Concurrent calls are
// flat-combined into one batch launch (fpset.hip), so throughput grows with
// the number of callers.  Reports puts/s and fingerprints per combined batch
// at 1/4/16/64 threads.  Diagnostic; not part of the product.
//
//   g++ -O2 -std=c++17 -I include tools/microbench/fpset_put_threads.cpp \
//       -L tla-kubernetes_amd/kubecheck/lib -lkubecheck -lpthread \
//       -Wl,-rpath,$PWD/tla-kubernetes_amd/kubecheck/lib -o tools/microbench/fpset_put_threads
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "kubecheck.h"

static uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
  printf("{\"bench\": \"kc_fpset_put from T host threads (TLC FPSet.put seam)\", \"results\": [\n");
  bool first = true;
  for (int T : {1, 4, 16, 64}) {
    kc_fpset* s = nullptr;
    if (kc_fpset_create(1ull << 26, 0, &s) != 0) {
      fprintf(stderr, "kc_fpset_create: %s\n", kc_last_error());
      return 1;
    }
    // warm the combining path (keys outside every thread's stream, so the
    // size check below counts exactly the timed puts)
    int seen = 0;
    for (int i = 0; i < 100; ++i) kc_fpset_put(s, mix((0xfeedull << 48) + i), &seen);
    const uint64_t r0 = kc_fpset_combine_rounds(s), size0 = kc_fpset_size(s);
    std::vector<uint64_t> done(T, 0);
    std::vector<int> err(T, 0);
    const auto t0 = std::chrono::steady_clock::now();
    const auto stop = t0 + std::chrono::duration<double>(seconds);
    std::vector<std::thread> th;
    for (int k = 0; k < T; ++k)
      th.emplace_back([&, k] {
        uint64_t i = 0;
        int sn = 0;
        while (std::chrono::steady_clock::now() < stop) {
          for (int b = 0; b < 16; ++b, ++i)
            if (kc_fpset_put(s, mix(((uint64_t)k << 40) + i + 1000), &sn) != 0) err[k] = 1;
        }
        done[k] = i;
      });
    for (auto& x : th) x.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t n = 0;
    int bad = 0;
    for (int k = 0; k < T; ++k) n += done[k], bad |= err[k];
    const uint64_t rounds = kc_fpset_combine_rounds(s) - r0;
    const bool exact = kc_fpset_size(s) - size0 == n;
    printf("%s {\"threads\": %d, \"puts\": %llu, \"seconds\": %.3f, \"puts_per_s\": %.1f, \"batches\": %llu, "
           "\"fps_per_batch\": %.2f, \"size_exact\": %s, \"errors\": %d}\n",
           first ? " " : ",", T, (unsigned long long)n, dt, n / dt, (unsigned long long)rounds,
           rounds ? (double)n / rounds : 0.0, exact ? "true" : "false", bad);
    first = false;
    fflush(stdout);
    kc_fpset_destroy(s);
  }
  printf("]}\n");
  return 0;
}
