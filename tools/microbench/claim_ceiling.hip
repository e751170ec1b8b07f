// claim_ceiling.hip — the mixed random-operation ceiling of k_claim's claim
// protocol on MI355X (diagnostic only, not the product).
//
// k_claim's HBM work per NP=2 check (kc_result.fpset_probes, the bench
// line's op_rate block): 2.126e9 ClaimSet claims by tile representatives, of
// which 0.7406e9 insert a new fingerprint (first-slot load, CAS, and in the
// deterministic protocol the agent-scope claim store) and 1.385e9 find their
// fingerprint already there (first-slot load, compare; 1.87 per new state).
// This kernel issues exactly that mix, with the product's own ClaimSet code
// (fpset_dev.h claimset_claim_store_from / claimset_insert_from, linear
// probing included) and no successor computation, on a ClaimSet of the
// product's size (2^32 16-B slots = 64 GiB, the NP=2 table):
//
//   prefill : N0 = units / 2 fingerprints (stream A) claimed at level 1
//   timed   : `units` units at level 2; unit u claims a new fingerprint of
//             stream B and looks up 1 or 2 (mean 1.8706) stream-A
//             fingerprints, which are found (CL_OLD)
//
// Each lane takes K units and issues all their first-slot loads back to back
// before any result is used (k_claim issues two representatives' loads and
// CASes together, KC_CLAIM_BATCH); the launch has no LDS, so occupancy is
// the register file's.  The fastest K is the ceiling: the time the claim
// protocol's memory operations need when nothing else runs.  op_rate.frac =
// that time / k_claim's time (bench.py), <= 1 by construction unless
// k_claim beat its own memory operations.
//
// It also re-takes the isolated rates of the three operation kinds on the
// same 64 GiB table (random first-slot 16-B load, inserting CAS, agent-scope
// claim store), which round 2 measured on 32 GiB (pmc_calib.hip).
//
//   hipcc -O3 --offload-arch=gfx950 -I../../tla-kubernetes_amd/csrc claim_ceiling.hip -o claim_ceiling
//   ./claim_ceiling [log2 slots = 32] [units = 740607993] [probes = 2125979524]
// prints one JSON object per line; the last line is the summary.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "fpset_dev.h"

using namespace kc;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fp_a(uint64_t k) { return normalize_fp(mix(k * 2 + 1)); }
__device__ __forceinline__ uint64_t fp_b(uint64_t u) { return normalize_fp(mix(u * 2 + 0x100000000000ull)); }

struct Stats {
  unsigned long long n_new, n_old, n_other, loads;
};

__global__ void __launch_bounds__(256) k_prefill(ClaimEntry* t, uint64_t ns, uint64_t n0, Stats* st, int compact) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n0) return;
  unsigned long long* w = reinterpret_cast<unsigned long long*>(t);
  const uint64_t f = fp_a(k), b = fpslots_home(f, ns);
  const int r = compact ? fpslots_insert_pair(w, ns, f, b, fpslots_first(w, b))
                        : claimset_claim_store(t, ns, f, make_claim(1, k), 1);
  if (r != CL_NEW) atomicAdd(&st->n_other, 1ull);
}

// extras of unit u: 1 + [u's hash < thr], thr / 2^32 = the mean's fraction
__device__ __forceinline__ int extras(uint64_t u, uint32_t thr) {
  return 1 + (((uint32_t)(mix(u ^ 0x5bd1e995ull) >> 32)) < thr ? 1 : 0);
}

// FIRST = 0: the deterministic STORE-claim protocol (CAS + claim store per
// new state); 1: first-claim mode (CAS only); 2 (round 6): first-claim mode
// on the compact ClaimSet of the engine (u64 fp words from an even home
// slot, fpslots_insert_pair: one aligned 16-B load of the home pair; `t` is
// then the u64 slot array).
template <int K, int FIRST>
__global__ void __launch_bounds__(256) k_mixed(ClaimEntry* __restrict__ t, uint64_t ns, uint64_t units, uint64_t n0,
                                               uint32_t thr, Stats* st) {
  const uint64_t u0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * K;
  if (u0 >= units) return;
  constexpr int Q = 3 * K;   // at most 1 new + 2 old per unit
  uint64_t fq[Q], iq[Q];
  ulonglong2 eq[Q];
  int nq = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint64_t u = u0 + k;
    if (u >= units) break;
    const int e = extras(u, thr);
    fq[nq] = fp_b(u);
    ++nq;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (j < e) {
        fq[nq] = fp_a(__umul64hi(mix(u * 4 + 1 + j), n0));
        ++nq;
      }
  }
  // every first-slot load issued before any is used
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (q < nq) {
      iq[q] = FIRST == 2 ? fpslots_home(fq[q], ns) : bucket_of(fq[q], ns);
      eq[q] = FIRST == 2 ? fpslots_first(reinterpret_cast<const unsigned long long*>(t), iq[q])
                         : claimset_first(t, iq[q]);
    }
  unsigned long long nn = 0, no = 0, nx = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q)
    if (q < nq) {
      const int r = FIRST == 2 ? fpslots_insert_pair(reinterpret_cast<unsigned long long*>(t), ns, fq[q], iq[q], eq[q])
                  : FIRST ? claimset_insert_from(t, ns, fq[q], iq[q], eq[q].x)
                          : claimset_claim_store_from(t, ns, fq[q], make_claim(2, u0 * 4 + q), 2, iq[q], eq[q]);
      if (r == CL_NEW) ++nn;
      else if (r == CL_OLD) ++no;
      else ++nx;
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    nn += __shfl_down(nn, off, 64);
    no += __shfl_down(no, off, 64);
    nx += __shfl_down(nx, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&st[blockIdx.x & 63].n_new, nn);
    atomicAdd(&st[blockIdx.x & 63].n_old, no);
    if (nx) atomicAdd(&st[blockIdx.x & 63].n_other, nx);
  }
}

// the isolated kinds on the same table (one op per lane): first-slot load of
// a random slot, inserting CAS on a random empty slot, agent-scope store
__global__ void __launch_bounds__(256) k_iso_load(const ClaimEntry* __restrict__ t, uint64_t ns, uint64_t n,
                                                  unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ulonglong2 e = claimset_first(t, __umul64hi(mix(i + 77), ns));
  if ((e.x ^ e.y) == 0x1234567ull) out[0] = e.x;
}
__global__ void __launch_bounds__(256) k_iso_cas(ClaimEntry* __restrict__ t, uint64_t ns, uint64_t n,
                                                 unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long v = atomicCAS(&t[__umul64hi(mix(i + 99), ns)].fp, 0ull, (unsigned long long)i + 1);
  if (v == 0x1234567ull) out[0] = v;
}
__global__ void __launch_bounds__(256) k_iso_store(ClaimEntry* __restrict__ t, uint64_t ns, uint64_t n,
                                                   unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  __hip_atomic_store(&t[__umul64hi(mix(i + 123), ns)].nclaim, (unsigned long long)i, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 32;
  const uint64_t units = argc > 2 ? strtoull(argv[2], nullptr, 10) : 740607993ull;
  const uint64_t probes = argc > 3 ? strtoull(argv[3], nullptr, 10) : 2125979524ull;
  if (lg < 20 || lg > 33 || units == 0 || probes < units || probes > 3 * units) {
    fprintf(stderr, "usage: claim_ceiling [log2 slots 20..33] [units] [probes in units..3 units]\n");
    return 2;
  }
  const uint64_t ns = 1ull << lg, n0 = units / 2;
  const double extra_mean = (double)(probes - units) / (double)units;   // 1 + P(2 extras)
  const uint32_t thr = (uint32_t)((extra_mean - 1.0) * 4294967296.0);
  ClaimEntry* t = nullptr;
  Stats* st = nullptr;
  unsigned long long* out = nullptr;
  CK(hipMalloc(&t, ns * sizeof(ClaimEntry)));
  CK(hipMalloc(&st, 64 * sizeof(Stats)));
  CK(hipMalloc(&out, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](auto launch) -> double {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return (double)ms;
  };
  const uint64_t niso = 1ull << 28;
  const unsigned giso = (unsigned)(niso / 256);
  // isolated rates (table zeroed before each kind that writes)
  CK(hipMemset(t, 0, ns * sizeof(ClaimEntry)));
  CK(hipDeviceSynchronize());
  const double ms_load = timed([&] { hipLaunchKernelGGL(k_iso_load, dim3(giso), dim3(256), 0, 0, t, ns, niso, out); });
  const double ms_cas = timed([&] { hipLaunchKernelGGL(k_iso_cas, dim3(giso), dim3(256), 0, 0, t, ns, niso, out); });
  const double ms_store = timed([&] { hipLaunchKernelGGL(k_iso_store, dim3(giso), dim3(256), 0, 0, t, ns, niso, out); });
  printf("{\"isolated\": true, \"table_slots\": %llu, \"ops\": %llu, \"load_G_per_s\": %.3f, \"cas_G_per_s\": %.3f, "
         "\"store_G_per_s\": %.3f}\n",
         (unsigned long long)ns, (unsigned long long)niso, niso / ms_load / 1e6, niso / ms_cas / 1e6,
         niso / ms_store / 1e6);
  fflush(stdout);
  double best[3] = {1e30, 1e30, 1e30};
  int bestk[3] = {0, 0, 0};
  for (int first = 0; first < 3; ++first) {
    for (int K : {1, 2, 4}) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(t, 0, ns * sizeof(ClaimEntry)));
        CK(hipMemset(st, 0, 64 * sizeof(Stats)));
        hipLaunchKernelGGL(k_prefill, dim3((unsigned)((n0 + 255) / 256)), dim3(256), 0, 0, t, ns, n0, st,
                           first == 2 ? 1 : 0);
        CK(hipDeviceSynchronize());
        const unsigned g = (unsigned)((units + 256ull * K - 1) / (256ull * K));
        const double ms = timed([&] {
#define KC_MX(KK, FF) hipLaunchKernelGGL((k_mixed<KK, FF>), dim3(g), dim3(256), 0, 0, t, ns, units, n0, thr, st)
          if (first == 2) {
            if (K == 1) KC_MX(1, 2); else if (K == 2) KC_MX(2, 2); else KC_MX(4, 2);
          } else if (first) {
            if (K == 1) KC_MX(1, 1); else if (K == 2) KC_MX(2, 1); else KC_MX(4, 1);
          } else {
            if (K == 1) KC_MX(1, 0); else if (K == 2) KC_MX(2, 0); else KC_MX(4, 0);
          }
#undef KC_MX
        });
        Stats h[64];
        CK(hipMemcpy(h, st, sizeof h, hipMemcpyDeviceToHost));
        unsigned long long nn = 0, no = 0, nx = 0;
        for (int k = 0; k < 64; ++k) {
          nn += h[k].n_new;
          no += h[k].n_old;
          nx += h[k].n_other;
        }
        printf("{\"mode\": \"%s\", \"K\": %d, \"rep\": %d, \"ms\": %.3f, \"units\": %llu, \"new\": %llu, "
               "\"old\": %llu, \"other\": %llu, \"claims\": %llu, \"claims_G_per_s\": %.3f}\n",
               first == 2 ? "first_compact" : first ? "first" : "deterministic", K, rep, ms, (unsigned long long)units, nn, no, nx,
               nn + no + nx, (nn + no + nx) / ms / 1e6);
        fflush(stdout);
        if (nn != units || nx != 0) {
          fprintf(stderr, "claim_ceiling: unexpected outcomes (new %llu of %llu, other %llu)\n", nn,
                  (unsigned long long)units, nx);
          return 1;
        }
        if (ms < best[first]) {
          best[first] = ms;
          bestk[first] = K;
        }
      }
    }
  }
  printf("{\"summary\": true, \"table_slots\": %llu, \"prefill\": %llu, \"units\": %llu, \"probes\": %llu, "
         "\"deterministic_ms\": %.3f, \"deterministic_K\": %d, \"first_ms\": %.3f, \"first_K\": %d, "
         "\"first_compact_ms\": %.3f, \"first_compact_K\": %d, "
         "\"iso_load_G_per_s\": %.3f, \"iso_cas_G_per_s\": %.3f, \"iso_store_G_per_s\": %.3f}\n",
         (unsigned long long)ns, (unsigned long long)n0, (unsigned long long)units, (unsigned long long)probes,
         best[0], bestk[0], best[1], bestk[1], best[2], bestk[2], niso / ms_load / 1e6, niso / ms_cas / 1e6, niso / ms_store / 1e6);
  CK(hipFree(t));
  CK(hipFree(st));
  CK(hipFree(out));
  return 0;
}
