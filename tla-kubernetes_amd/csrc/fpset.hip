// fpset.hip — HBM FPSet: host owner, batch kernels and the kc_fpset_* C-ABI
// (drop-in for TLC's tlc2.tool.fp.FPSet put/contains/size/checkFPs; see
// include/kubecheck.h and INTEGRATION.md).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kubecheck.h"
#include "engine_kernels.h"
#include "engine_util.h"
#include "fpset_host.h"
#include "kc_common.h"

namespace kc {

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Rehash every stored fingerprint of `old` into `nw`.
__global__ void k_fpset_rehash(const unsigned long long* __restrict__ old, uint64_t old_slots,
                               unsigned long long* __restrict__ nw, uint64_t new_buckets,
                               unsigned long long* __restrict__ fail) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < old_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long fp = old[i];
    if (fp && fpset_insert(nw, new_buckets, fp) < 0) atomicAdd(fail, 1ull);
  }
}

// Insert a short list of fingerprints (init states) into the FPSet.
__global__ void k_fpset_insert_list(const uint64_t* __restrict__ fps, uint64_t n,
                                    unsigned long long* __restrict__ slots, uint64_t nbuckets,
                                    int* __restrict__ result) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int r = fpset_insert(slots, nbuckets, fps[i]);
    if (result) result[i] = r;
  }
}

void launch_fpset_insert_list(const uint64_t* d_fps, uint64_t n, const DevFpset& fs, int* d_res,
                              hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_fpset_insert_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       d_fps, n, fs.slots, fs.nbuckets, d_res);
}

int DevFpset::init(uint64_t min_slots, hipStream_t st) {
  release();
  nbuckets = (min_slots + 7) / 8;
  if (nbuckets < 8) nbuckets = 8;
  KC_HIP_TRY(hipMalloc(&slots, nbuckets * 64));
  KC_HIP_TRY(hipMemsetAsync(slots, 0, nbuckets * 64, st));
  KC_HIP_TRY(hipMalloc(&d_fail, sizeof(unsigned long long)));
  count = 0;
  return 0;
}

void DevFpset::release() {
  if (slots) (void)hipFree(slots);
  if (d_fail) (void)hipFree(d_fail);
  slots = nullptr;
  d_fail = nullptr;
  nbuckets = 0;
  count = 0;
}

int DevFpset::reserve(uint64_t extra, hipStream_t st) {
  if ((count + extra) * 4 <= capacity() * 3) return 0;
  uint64_t nb = nbuckets;
  while ((count + extra) * 4 > nb * 8 * 2) nb *= 2;  // land at <= 50% load
  unsigned long long* ns = nullptr;
  KC_HIP_TRY(hipMalloc(&ns, nb * 64));
  KC_HIP_TRY(hipMemsetAsync(ns, 0, nb * 64, st));
  KC_HIP_TRY(hipMemsetAsync(d_fail, 0, sizeof(unsigned long long), st));
  const uint64_t old_slots = capacity();
  hipLaunchKernelGGL(k_fpset_rehash, dim3(table_grid(old_slots)), dim3(256), 0, st, slots, old_slots, ns, nb, d_fail);
  KC_HIP_TRY(hipGetLastError());
  unsigned long long fail = 0;
  KC_HIP_TRY(hipMemcpyAsync(&fail, d_fail, sizeof fail, hipMemcpyDeviceToHost, st));
  KC_HIP_TRY(hipStreamSynchronize(st));
  if (fail) {
    (void)hipFree(ns);
    set_error("fpset rehash failed (%llu)", fail);
    return -ENOMEM;
  }
  KC_HIP_TRY(hipFree(slots));
  slots = ns;
  nbuckets = nb;
  return 0;
}

// ---------------------------------------------------------------- ClaimSet
// Move every entry of `old` into `nw` (fps are unique, so the claim word is
// a plain store next to the CAS'd fp).
// The per-run clear of the ClaimSet: 16-B non-temporal stores over a
// grid-stride loop of 8192 workgroups (64 GiB in 9.9-10.1 ms against 10.8-10.9
// for hipMemsetAsync, profiles/r03ap_clear.txt).
typedef unsigned int kc_u32x4 __attribute__((ext_vector_type(4)));
// (n16: the table's size in 16-B units — nslots, or nslots / 2 compact)
__global__ void __launch_bounds__(256) k_claimset_clear(ClaimEntry* __restrict__ t, uint64_t n16) {
  kc_u32x4* p = reinterpret_cast<kc_u32x4*>(t);
  const kc_u32x4 z = {0u, 0u, 0u, 0u};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(z, &p[i]);
}

__global__ void k_claimset_rehash(const ClaimEntry* __restrict__ old, uint64_t old_slots,
                                  ClaimEntry* __restrict__ nw, uint64_t new_slots,
                                  unsigned long long* __restrict__ fail) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < old_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const ClaimEntry e = old[i];
    if (!e.fp) continue;
    uint64_t k = bucket_of(e.fp, new_slots);
    bool placed = false;
    for (uint64_t probe = 0; probe < new_slots; ++probe) {
      if (nw[k].fp == 0ull && atomicCAS(&nw[k].fp, 0ull, e.fp) == 0ull) {
        nw[k].nclaim = e.nclaim;
        placed = true;
        break;
      }
      k = (k + 1 == new_slots) ? 0 : k + 1;
    }
    if (!placed) atomicAdd(fail, 1ull);
  }
}

__global__ void k_claimset_insert_list(const uint64_t* __restrict__ fps, uint64_t n,
                                       ClaimEntry* __restrict__ t, uint64_t nslots,
                                       uint32_t level, int* __restrict__ result) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int r = claimset_claim(t, nslots, fps[i], make_claim(level, i), level);
    if (result) result[i] = r;
  }
}

// the compact table's rehash and list insert (fp words only)
__global__ void k_fpslots_rehash(const unsigned long long* __restrict__ old, uint64_t old_slots,
                                 unsigned long long* __restrict__ nw, uint64_t new_slots,
                                 unsigned long long* __restrict__ fail) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < old_slots;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long fp = old[i];
    if (!fp) continue;
    const uint64_t k = fpslots_home(fp, new_slots);
    if (fpslots_insert_pair(nw, new_slots, fp, k, fpslots_first(nw, k)) != CL_NEW) atomicAdd(fail, 1ull);
  }
}
__global__ void k_fpslots_insert_list(const uint64_t* __restrict__ fps, uint64_t n, unsigned long long* __restrict__ t,
                                      uint64_t nslots, int* __restrict__ result) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const uint64_t k = fpslots_home(fps[i], nslots);
    const int r = fpslots_insert_pair(t, nslots, fps[i], k, fpslots_first(t, k));
    if (result) result[i] = r;
  }
}

void launch_claimset_insert_list(const uint64_t* d_fps, uint64_t n, const DevClaimSet& cs,
                                 uint32_t level, int* d_res, hipStream_t st) {
  if (n && cs.compact)
    hipLaunchKernelGGL(k_fpslots_insert_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       d_fps, n, cs.words(), cs.nslots, d_res);
  else if (n)
    hipLaunchKernelGGL(k_claimset_insert_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       d_fps, n, cs.t, cs.nslots, level, d_res);
}

int DevClaimSet::init(uint64_t min_slots, hipStream_t st) {
  release();
  nslots = min_slots < 64 ? 64 : min_slots;
  KC_HIP_TRY(hipMalloc(&t, nslots * slot_bytes()));
  KC_HIP_TRY(hipMemsetAsync(t, 0, nslots * slot_bytes(), st));
  KC_HIP_TRY(hipMalloc(&d_fail, sizeof(unsigned long long)));
  count = 0;
  return 0;
}

// (an 8,192-workgroup grid-stride clear kernel: 6.9 TB/s on the 64 GiB NP=2
// table against hipMemsetAsync's 6.3, round 3; on the 32 GiB
// compact table hipMemsetAsync is the faster, 5.8 against 6.5-7.3 ms,
// profiles/r06u_clear_bench.log)
int DevClaimSet::clear(hipStream_t st) {
  if (nslots < (1u << 20) || compact) {
    KC_HIP_TRY(hipMemsetAsync(t, 0, nslots * slot_bytes(), st));
  } else {
    hipLaunchKernelGGL(k_claimset_clear, dim3(8192u), dim3(256), 0, st, t, nslots * slot_bytes() / 16);
    KC_HIP_TRY(hipGetLastError());
  }
  count = 0;
  return 0;
}

void DevClaimSet::release() {
  if (t) (void)hipFree(t);
  if (d_fail) (void)hipFree(d_fail);
  t = nullptr;
  d_fail = nullptr;
  nslots = 0;
  count = 0;
}

// Linear probing: every extra probe of a chain is a dependent load the
// claim kernel waits for, so the load factor is paid in k_claim time (NP=2:
// 64 GiB at 17% load runs the check 2.3% faster than 32 GiB at 35%, its
// larger clear included).  Past 1/3 load the table grows to
// land at <= 1/4; when HBM cannot hold that, at <= 1/2.
int DevClaimSet::reserve(uint64_t extra, hipStream_t st) {
  // grow once the reserved fill would pass 1/3 of the slots, to at most 1/4
  // (round 5 A/B: growing at 1/2 halves the NP=2 table and its clear but
  // costs k_claim 7-10 ms in longer probe runs; 1/4 gives the same table)
  constexpr uint64_t ld = 3;
  const uint64_t need = count + extra;
  if (need * ld <= capacity()) return 0;
  uint64_t ns = nslots, ns_min = nslots;
  while (need * (ld + 1) > ns) ns *= 2;
  while (need * 2 > ns_min) ns_min *= 2;
  ClaimEntry* nt = nullptr;
  if (hipMalloc(&nt, ns * slot_bytes()) != hipSuccess) {
    (void)hipGetLastError();
    nt = nullptr;
    ns = ns_min;
    if (ns == nslots) return 0;                    // (still <= 1/2 after this batch)
    KC_HIP_TRY(hipMalloc(&nt, ns * slot_bytes()));
  }
  KC_HIP_TRY(hipMemsetAsync(nt, 0, ns * slot_bytes(), st));
  KC_HIP_TRY(hipMemsetAsync(d_fail, 0, sizeof(unsigned long long), st));
  if (compact)
    hipLaunchKernelGGL(k_fpslots_rehash, dim3(table_grid(nslots)), dim3(256), 0, st,
                       words(), nslots, reinterpret_cast<unsigned long long*>(nt), ns, d_fail);
  else
    hipLaunchKernelGGL(k_claimset_rehash, dim3(table_grid(nslots)), dim3(256), 0, st,
                       t, nslots, nt, ns, d_fail);
  KC_HIP_TRY(hipGetLastError());
  unsigned long long fail = 0;
  KC_HIP_TRY(hipMemcpyAsync(&fail, d_fail, sizeof fail, hipMemcpyDeviceToHost, st));
  KC_HIP_TRY(hipStreamSynchronize(st));
  if (fail) {
    (void)hipFree(nt);
    set_error("claimset rehash failed (%llu)", fail);
    return -ENOMEM;
  }
  KC_HIP_TRY(hipFree(t));
  t = nt;
  nslots = ns;
  return 0;
}

int DevBatchTable::ensure(uint64_t entries, hipStream_t st) {
  (void)st;
  if (entries <= cap) return 0;
  release();
  KC_HIP_TRY(hipMalloc(&t, entries * sizeof(BatchEntry)));
  cap = entries;
  return 0;
}

void DevBatchTable::release() {
  if (t) (void)hipFree(t);
  t = nullptr;
  cap = 0;
}

// --------------------------------------------------------------- kernels
// Batch statistics [new, full, found, -] live in STAT_ROWS 64-B rows, one
// picked per block: a per-wave atomic on one shared address serialises the
// whole grid (the same effect the engine's striped Counters avoid).
constexpr int STAT_ROWS = 64;
constexpr size_t STAT_BYTES = STAT_ROWS * 8 * sizeof(unsigned long long);
__device__ __forceinline__ unsigned long long* stat_row(unsigned long long* stats) {
  return stats + (blockIdx.x & (STAT_ROWS - 1)) * 8;
}
__global__ void k_normalize(uint64_t* __restrict__ fps, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fps[i] = normalize_fp(fps[i]);
}
__global__ void k_batch_claim(const uint64_t* __restrict__ fps, uint64_t n,
                              BatchEntry* __restrict__ bt, uint64_t mask) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) batch_insert(bt, mask, fps[i], i);
}
__global__ void k_batch_put(const uint64_t* __restrict__ fps, uint64_t n,
                            const BatchEntry* __restrict__ bt, uint64_t mask,
                            unsigned long long* __restrict__ slots, uint64_t nbuckets,
                            uint8_t* __restrict__ seen, unsigned long long* __restrict__ stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long nw = 0, full = 0;
  if (i < n) {
    const uint64_t fp = fps[i];
    uint8_t s = 1;
    if (batch_is_rep(bt, mask, fp, i)) {
      const int r = fpset_insert(slots, nbuckets, fp);
      if (r == 1) { s = 0; nw = 1; }
      else if (r < 0) full = 1;
    }
    seen[i] = s;
  }
  // one atomic per wave, into this block's stats row
  const unsigned long long bw = __ballot(nw != 0), bf = __ballot(full != 0);
  if ((threadIdx.x & 63) == 0) {
    if (bw) atomicAdd(&stat_row(stats)[0], (unsigned long long)__popcll(bw));
    if (bf) atomicAdd(&stat_row(stats)[1], (unsigned long long)__popcll(bf));
  }
}
__global__ void k_contains(const uint64_t* __restrict__ fps, uint64_t n,
                           const unsigned long long* __restrict__ slots, uint64_t nbuckets,
                           uint8_t* __restrict__ seen) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) seen[i] = (uint8_t)fpset_contains(slots, nbuckets, fps[i]);
}

// A combined round of <= SMALL_MAX single puts/contains (kc_fpset_put from
// TLC's worker threads): ONE launch of one workgroup that reads the
// fingerprints from pinned host memory and writes the answers and counts
// straight back into it, so a round costs one launch and one sync instead of
// copies, a batch table and two syncs.  Sequential semantics inside the
// round: a fingerprint equal to an earlier one of the round is "already
// present" for a put (the earlier one inserted it).
constexpr int SMALL_MAX = 1024;
__global__ void __launch_bounds__(SMALL_MAX) k_small_round(const uint64_t* __restrict__ in, uint32_t n, int op,
                                                           unsigned long long* __restrict__ slots, uint64_t nbuckets,
                                                           uint8_t* __restrict__ seen_out,
                                                           unsigned long long* __restrict__ stats_out) {
  __shared__ unsigned long long sh[SMALL_MAX];
  __shared__ unsigned int sh_new, sh_full;
  const uint32_t t = threadIdx.x;
  if (t == 0) sh_new = sh_full = 0;
  const uint64_t fp = t < n ? normalize_fp(in[t]) : 0;
  if (t < n) sh[t] = fp;
  __syncthreads();
  if (t < n) {
    bool dup = false;
    for (uint32_t j = 0; j < t && !dup; ++j) dup = sh[j] == fp;
    uint8_t seen;
    if (op == 1) {
      seen = (uint8_t)fpset_contains(slots, nbuckets, fp);
    } else if (dup) {
      seen = 1;
    } else {
      const int r = fpset_insert(slots, nbuckets, fp);
      if (r == 1) atomicAdd(&sh_new, 1u);
      if (r < 0) atomicAdd(&sh_full, 1u);
      seen = r == 0 ? 1 : 0;
    }
    seen_out[t] = seen;
  }
  __syncthreads();
  if (t == 0) {
    stats_out[0] = sh_new;
    stats_out[1] = sh_full;
  }
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// Stress fingerprints: fp = perm63(seed + i), a
// bijection of [0, 2^63) (xor-shifts and odd multiplies mod 2^63), so
// distinct stream inputs give distinct, already-normalised fingerprints
// (MSB clear, never 0 for a nonzero input).  The insert stream is inputs
// seed + [0, n_ins); a lookup j is present for even j (input seed +
// splitmix64(j) % n_ins) and absent for odd j (input seed + n_ins + j), so
// a run's size and found counts are known exactly: n_ins and ceil(n_lookup/2).
__host__ __device__ __forceinline__ uint64_t perm63(uint64_t x) {
  constexpr uint64_t M = 0x7fffffffffffffffull;
  x &= M;
  x ^= x >> 31; x = (x * 0x9e3779b97f4a7c15ull) & M;
  x ^= x >> 29; x = (x * 0xbf58476d1ce4e5b9ull) & M;
  x ^= x >> 32; x = (x * 0x94d049bb133111ebull) & M;
  return x ^ (x >> 30);
}
__host__ __device__ __forceinline__ uint64_t stress_insert_fp(uint64_t seed, uint64_t i) {
  return perm63(seed + i);
}
__host__ __device__ __forceinline__ uint64_t stress_lookup_fp(uint64_t seed, uint64_t n_ins, uint64_t j) {
  return perm63((j & 1) ? seed + n_ins + j : seed + splitmix64(j) % n_ins);
}
// Stress insert: fingerprints generated in registers (no input traffic).
__global__ void __launch_bounds__(256)
k_stress_insert(uint64_t seed, uint64_t start, uint64_t n, unsigned long long* __restrict__ slots,
                uint64_t nbuckets, unsigned long long* __restrict__ stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long nw = 0;
  if (i < n) nw = fpset_insert(slots, nbuckets, stress_insert_fp(seed, start + i)) == 1;
  const unsigned long long b = __ballot(nw != 0);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&stat_row(stats)[0], (unsigned long long)__popcll(b));
}
// Stress lookup of lookup-stream entries [start, start + n).
__global__ void __launch_bounds__(256)
k_stress_lookup(uint64_t seed, uint64_t n_ins, uint64_t start, uint64_t n,
                const unsigned long long* __restrict__ slots, uint64_t nbuckets,
                unsigned long long* __restrict__ stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long f = 0;
  if (i < n) f = fpset_contains(slots, nbuckets, stress_lookup_fp(seed, n_ins, start + i));
  const unsigned long long b = __ballot(f != 0);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&stat_row(stats)[2], (unsigned long long)__popcll(b));
}
// (Round 5 measured windowed inserts — the stream bucketed by 1 GiB table
// windows before the CASes — 4.4x slower: the bucketing pass writes and
// re-reads every fingerprint, and a 1 GiB window is no more cache-resident
// than the whole table; DESIGN §7.3.  Removed in round 6.)

// The same streams written to memory (the sharded stress exchanges them).
__global__ void k_stress_gen(uint64_t seed, int kind, uint64_t n_ins, uint64_t start, uint64_t n,
                             uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    out[i] = kind == 0 ? stress_insert_fp(seed, start + i) : stress_lookup_fp(seed, n_ins, start + i);
}
// Bulk insert / lookup of fingerprints in memory, counting new / found.
__global__ void __launch_bounds__(256)
k_insert_count(const uint64_t* __restrict__ fps, uint64_t n, unsigned long long* __restrict__ slots,
               uint64_t nbuckets, unsigned long long* __restrict__ stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int r = 0;
  if (i < n) r = fpset_insert(slots, nbuckets, normalize_fp(fps[i]));
  const unsigned long long bw = __ballot(r == 1), bf = __ballot(r < 0);
  if ((threadIdx.x & 63) == 0) {
    if (bw) atomicAdd(&stat_row(stats)[0], (unsigned long long)__popcll(bw));
    if (bf) atomicAdd(&stat_row(stats)[1], (unsigned long long)__popcll(bf));
  }
}
__global__ void __launch_bounds__(256)
k_contains_count(const uint64_t* __restrict__ fps, uint64_t n, const unsigned long long* __restrict__ slots,
                 uint64_t nbuckets, unsigned long long* __restrict__ stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int f = 0;
  if (i < n) f = fpset_contains(slots, nbuckets, normalize_fp(fps[i]));
  const unsigned long long b = __ballot(f != 0);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(&stat_row(stats)[2], (unsigned long long)__popcll(b));
}

// ------------------------------------------------------- owner partition
// Stable counting sort of a batch of fingerprints by owner rank
// floor(fp * R / 2^63) (the sharded FPSet's routing step, like the BFS
// records: engine_kernels.h owner_of).  One workgroup = PART_TILE
// consecutive fps; pass 1 counts per (owner, tile), one exclusive scan over
// the owner-major matrix gives each tile's base, pass 2 scatters in input
// order (wave ballots rank the lanes of one owner, LDS carries the running
// per-owner offset across the tile's rounds).
constexpr int PART_TILE = 4096;
constexpr int PART_MAXR = 16;
__device__ __forceinline__ uint32_t part_owner(uint64_t fp, uint32_t world) {
  return owner_of(normalize_fp(fp), world);
}
__global__ void __launch_bounds__(256)
k_part_count(const uint64_t* __restrict__ fps, uint64_t n, uint32_t world, uint32_t ntiles,
             uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[PART_MAXR];
  if (threadIdx.x < PART_MAXR) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * PART_TILE;
  for (int k = threadIdx.x; k < PART_TILE; k += 256) {
    const uint64_t i = t0 + k;
    if (i < n) atomicAdd(&h[part_owner(fps[i], world)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < world) cnt[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}
__global__ void __launch_bounds__(256)
k_part_scatter(const uint64_t* __restrict__ fps, uint64_t n, uint32_t world, uint32_t ntiles,
               const uint32_t* __restrict__ off, uint64_t* __restrict__ out) {
  __shared__ uint32_t run[PART_MAXR];
  __shared__ uint32_t wcnt[4][PART_MAXR];
  if (threadIdx.x < world) run[threadIdx.x] = off[(uint64_t)threadIdx.x * ntiles + blockIdx.x];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1;
  const uint64_t t0 = (uint64_t)blockIdx.x * PART_TILE;
  for (int k = 0; k < PART_TILE; k += 256) {
    const uint64_t i = t0 + k + threadIdx.x;
    const bool live = i < n;
    const uint64_t fp = live ? fps[i] : 0;
    const uint32_t o = live ? part_owner(fp, world) : PART_MAXR;
    uint32_t r = 0;
    for (uint32_t q = 0; q < world; ++q) {
      const uint64_t m = __ballot(o == q);
      if (o == q) r = (uint32_t)__popcll(m & lt);
      if (lane == 0) wcnt[wv][q] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (live) {
      uint32_t pos = run[o] + r;
      for (int w = 0; w < wv; ++w) pos += wcnt[w][o];
      out[pos] = fp;
    }
    __syncthreads();
    if (threadIdx.x < world)
      run[threadIdx.x] += wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] + wcnt[3][threadIdx.x];
    __syncthreads();
  }
}

__global__ void k_compact_fps(const unsigned long long* __restrict__ slots, uint64_t nslots,
                              unsigned long long* __restrict__ out, unsigned long long* __restrict__ n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x)
    if (slots[i]) out[atomicAdd(n, 1ull)] = slots[i];
}
__global__ void k_min_gap(const unsigned long long* __restrict__ s, uint64_t n,
                          unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 < n) atomicMin(out, s[i + 1] - s[i]);
}

}  // namespace kc

using namespace kc;

// Flat-combining state of the single-fingerprint put/contains (below).
struct Combiner {
  struct Req { uint64_t fp; int op; uint64_t ticket; };
  struct Res { uint8_t seen; int rc; std::string msg; };   // msg: the combiner's error text (rc < 0)
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req> pending;
  std::unordered_map<uint64_t, Res> done;
  uint64_t next_ticket = 0, rounds = 0;
  bool busy = false;
};

struct kc_fpset {
  int device = 0;
  hipStream_t stream = nullptr;
  DevFpset fs;
  DevBatchTable bt;
  uint64_t* d_fps = nullptr;
  uint8_t* d_seen = nullptr;
  uint64_t stage_cap = 0;
  unsigned long long* d_stats = nullptr;  // STAT_ROWS rows of [new, full, found, -]
  uint32_t *part_cnt = nullptr, *part_off = nullptr;   // owner partition scratch
  uint64_t part_cap = 0, part_off_cap = 0;
  uint8_t* scan_tmp = nullptr;
  uint64_t scan_cap = 0;
  uint8_t* h_small = nullptr;   // pinned: SMALL_MAX fps, SMALL_MAX answers, 2 counts (k_small_round)
  std::mutex mu;
  Combiner comb;
};

// One combined round of n <= SMALL_MAX requests (op 0 put, 1 contains).
static int small_round(kc_fpset* s, const uint64_t* fps, size_t n, int op, uint8_t* seen) {
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  if (!s->h_small) KC_HIP_TRY(hipHostMalloc(&s->h_small, SMALL_MAX * 9 + 64));
  if (op == 0) KC_TRY(s->fs.reserve(n, s->stream));
  uint64_t* hf = reinterpret_cast<uint64_t*>(s->h_small);
  uint8_t* hs = s->h_small + SMALL_MAX * 8;
  unsigned long long* hc = reinterpret_cast<unsigned long long*>(s->h_small + SMALL_MAX * 9 + 8 - (SMALL_MAX * 9) % 8);
  memcpy(hf, fps, n * 8);
  hipLaunchKernelGGL(k_small_round, dim3(1), dim3(SMALL_MAX), 0, s->stream, hf, (uint32_t)n, op, s->fs.slots,
                     s->fs.nbuckets, hs, hc);
  KC_HIP_TRY(hipGetLastError());
  KC_HIP_TRY(hipStreamSynchronize(s->stream));
  if (hc[1]) {
    set_error("fpset full");
    return -ENOMEM;
  }
  s->fs.count += hc[0];
  memcpy(seen, hs, n);
  return 0;
}

// Sum the striped stats rows (syncs the stream).
static int read_stats(kc_fpset* s, hipStream_t st, unsigned long long out[4]) {
  unsigned long long rows[STAT_ROWS * 8];
  KC_HIP_TRY(hipMemcpyAsync(rows, s->d_stats, STAT_BYTES, hipMemcpyDeviceToHost, st));
  KC_HIP_TRY(hipStreamSynchronize(st));
  for (int k = 0; k < 4; ++k) {
    out[k] = 0;
    for (int r = 0; r < STAT_ROWS; ++r) out[k] += rows[r * 8 + k];
  }
  return 0;
}

static int stage(kc_fpset* s, uint64_t n) {
  if (n <= s->stage_cap) return 0;
  if (s->d_fps) (void)hipFree(s->d_fps);
  if (s->d_seen) (void)hipFree(s->d_seen);
  s->d_fps = nullptr;
  s->d_seen = nullptr;
  s->stage_cap = 0;
  const uint64_t cap = next_pow2(n);
  KC_HIP_TRY(hipMalloc(&s->d_fps, cap * 8));
  KC_HIP_TRY(hipMalloc(&s->d_seen, cap));
  s->stage_cap = cap;
  return 0;
}

static int put_dev(kc_fpset* s, uint64_t* fps, size_t n, uint8_t* seen, hipStream_t st,
                   uint64_t* n_new) {
  if (n == 0) return 0;
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_normalize, dim3(grid), dim3(256), 0, st, fps, (uint64_t)n);
  const uint64_t cap = next_pow2(2 * (uint64_t)n + 64);
  KC_TRY(s->bt.ensure(cap, st));
  KC_HIP_TRY(hipMemsetAsync(s->bt.t, 0, cap * sizeof(BatchEntry), st));
  hipLaunchKernelGGL(k_batch_claim, dim3(grid), dim3(256), 0, st, fps, (uint64_t)n, s->bt.t, cap - 1);
  KC_TRY(s->fs.reserve(n, st));
  KC_HIP_TRY(hipMemsetAsync(s->d_stats, 0, STAT_BYTES, st));
  hipLaunchKernelGGL(k_batch_put, dim3(grid), dim3(256), 0, st, fps, (uint64_t)n, s->bt.t, cap - 1,
                     s->fs.slots, s->fs.nbuckets, seen, s->d_stats);
  KC_HIP_TRY(hipGetLastError());
  unsigned long long stats[4];
  KC_TRY(read_stats(s, st, stats));
  if (stats[1]) {
    set_error("fpset full");
    return -ENOMEM;
  }
  s->fs.count += stats[0];
  if (n_new) *n_new = stats[0];
  return 0;
}

extern "C" {

int kc_fpset_create(uint64_t capacity_fps, int device, kc_fpset** out) {
  if (!out) { set_error("kc_fpset_create: out is NULL"); return -EINVAL; }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("kc_fpset_create: no HIP device");
    return -ENODEV;
  }
  if (device < 0 || device >= ndev) { set_error("kc_fpset_create: bad device %d", device); return -EINVAL; }
  KC_HIP_TRY(hipSetDevice(device));
  auto* s = new kc_fpset();
  s->device = device;
  int rc = 0;
  // a BLOCKING stream: it orders with the legacy default stream, which is
  // where a caller's NULL-stream work (and torch's default stream) runs, so
  // a *_dev call without a stream sees the caller's earlier writes
  if (hipStreamCreate(&s->stream) != hipSuccess) rc = -EIO;
  if (!rc) rc = s->fs.init(capacity_fps * 4 / 3 + 8, s->stream);
  if (!rc && hipMalloc(&s->d_stats, STAT_BYTES) != hipSuccess) rc = -ENOMEM;
  if (!rc && hipStreamSynchronize(s->stream) != hipSuccess) rc = -EIO;
  if (rc) { kc_fpset_destroy(s); if (rc == -EIO) set_error("kc_fpset_create: HIP failure"); return rc; }
  *out = s;
  return 0;
}

void kc_fpset_destroy(kc_fpset* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  s->fs.release();
  s->bt.release();
  if (s->d_fps) (void)hipFree(s->d_fps);
  if (s->d_seen) (void)hipFree(s->d_seen);
  if (s->d_stats) (void)hipFree(s->d_stats);
  if (s->h_small) (void)hipHostFree(s->h_small);
  for (void* p : {(void*)s->part_cnt, (void*)s->part_off, (void*)s->scan_tmp})
    if (p) (void)hipFree(p);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

int kc_fpset_put_batch(kc_fpset* s, const uint64_t* fps, size_t n, uint8_t* seen_out) {
  if (!s || (n && (!fps || !seen_out))) { set_error("kc_fpset_put_batch: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  KC_TRY(stage(s, n));
  if (n == 0) return 0;
  KC_HIP_TRY(hipMemcpyAsync(s->d_fps, fps, n * 8, hipMemcpyHostToDevice, s->stream));
  KC_TRY(put_dev(s, s->d_fps, n, s->d_seen, s->stream, nullptr));
  KC_HIP_TRY(hipMemcpyAsync(seen_out, s->d_seen, n, hipMemcpyDeviceToHost, s->stream));
  KC_HIP_TRY(hipStreamSynchronize(s->stream));
  return 0;
}

int kc_fpset_contains_batch(kc_fpset* s, const uint64_t* fps, size_t n, uint8_t* seen_out) {
  if (!s || (n && (!fps || !seen_out))) { set_error("kc_fpset_contains_batch: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  KC_TRY(stage(s, n));
  if (n == 0) return 0;
  KC_HIP_TRY(hipMemcpyAsync(s->d_fps, fps, n * 8, hipMemcpyHostToDevice, s->stream));
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_normalize, dim3(grid), dim3(256), 0, s->stream, s->d_fps, (uint64_t)n);
  hipLaunchKernelGGL(k_contains, dim3(grid), dim3(256), 0, s->stream, s->d_fps, (uint64_t)n,
                     s->fs.slots, s->fs.nbuckets, s->d_seen);
  KC_HIP_TRY(hipGetLastError());
  KC_HIP_TRY(hipMemcpyAsync(seen_out, s->d_seen, n, hipMemcpyDeviceToHost, s->stream));
  KC_HIP_TRY(hipStreamSynchronize(s->stream));
  return 0;
}

int kc_fpset_put_batch_dev(kc_fpset* s, uint64_t* fps_dev, size_t n, uint8_t* seen_dev, void* hs) {
  if (!s || (n && (!fps_dev || !seen_dev))) { set_error("kc_fpset_put_batch_dev: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = hs ? (hipStream_t)hs : s->stream;
  return put_dev(s, fps_dev, n, seen_dev, st, nullptr);
}

int kc_fpset_contains_batch_dev(kc_fpset* s, uint64_t* fps_dev, size_t n, uint8_t* seen_dev, void* hs) {
  if (!s || (n && (!fps_dev || !seen_dev))) { set_error("kc_fpset_contains_batch_dev: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = hs ? (hipStream_t)hs : s->stream;
  if (n == 0) return 0;
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_normalize, dim3(grid), dim3(256), 0, st, fps_dev, (uint64_t)n);
  hipLaunchKernelGGL(k_contains, dim3(grid), dim3(256), 0, st, fps_dev, (uint64_t)n, s->fs.slots,
                     s->fs.nbuckets, seen_dev);
  KC_HIP_TRY(hipGetLastError());
  return 0;
}

uint64_t kc_fpset_size(const kc_fpset* s) { return s ? s->fs.count : 0; }
uint64_t kc_fpset_capacity(const kc_fpset* s) { return s ? s->fs.capacity() : 0; }

int kc_fpset_check_fps(kc_fpset* s, uint64_t* min_gap_out, double* prob_out) {
  if (!s) { set_error("kc_fpset_check_fps: NULL"); return -EINVAL; }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = s->stream;
  const uint64_t nslots = s->fs.capacity();
  unsigned long long *d_a = nullptr, *d_b = nullptr, *d_n = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  int rc = 0;
  unsigned long long n = 0, gap = ~0ull;
  const uint64_t cnt = s->fs.count ? s->fs.count : 1;
  if (hipMalloc(&d_a, cnt * 8) != hipSuccess || hipMalloc(&d_b, cnt * 8) != hipSuccess ||
      hipMalloc(&d_n, 16) != hipSuccess) {
    rc = -ENOMEM; set_error("kc_fpset_check_fps: out of device memory");
  }
  if (!rc) {
    (void)hipMemsetAsync(d_n, 0, 8, st);
    (void)hipMemcpyAsync(d_n + 1, &gap, 8, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_compact_fps, dim3(table_grid(nslots)), dim3(256), 0, st,
                       s->fs.slots, nslots, d_a, d_n);
    (void)hipMemcpyAsync(&n, d_n, 8, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    if (n > cnt) { rc = -EIO; set_error("kc_fpset_check_fps: count mismatch"); }
  }
  if (!rc && n > 1) {
    if (hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, d_a, d_b, (int)n, 0, 64, st) != hipSuccess) {
      rc = -EIO; set_error("kc_fpset_check_fps: sort");
    }
    if (!rc && hipMalloc(&tmp, tmp_bytes) != hipSuccess) { rc = -ENOMEM; set_error("kc_fpset_check_fps: temp"); }
    if (!rc) {
      (void)hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, d_a, d_b, (int)n, 0, 64, st);
      hipLaunchKernelGGL(k_min_gap, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_b, n, d_n + 1);
      (void)hipMemcpyAsync(&gap, d_n + 1, 8, hipMemcpyDeviceToHost, st);
      if (hipStreamSynchronize(st) != hipSuccess) { rc = -EIO; set_error("kc_fpset_check_fps: HIP"); }
    }
  }
  if (tmp) (void)hipFree(tmp);
  if (d_a) (void)hipFree(d_a);
  if (d_b) (void)hipFree(d_b);
  if (d_n) (void)hipFree(d_n);
  if (rc) return rc;
  if (min_gap_out) *min_gap_out = gap;
  if (prob_out) *prob_out = (n > 1 && gap) ? 1.0 / (double)gap : 0.0;
  return 0;
}

static bool stress_args_ok(uint64_t seed, uint64_t n, uint64_t n_lookup) {
  // every stream input seed + x (x < n + n_lookup) must lie in [1, 2^63)
  const uint64_t M = 0x7fffffffffffffffull;
  return seed >= 1 && seed <= M && n <= M - seed && n_lookup <= M - seed - n;
}

int kc_fpset_stress(kc_fpset* s, uint64_t seed, uint64_t n, uint64_t batch, uint64_t n_lookup,
                    double* insert_seconds, double* lookup_seconds, uint64_t* found_out) {
  if (!s || batch == 0 || !stress_args_ok(seed, n, n_lookup) || (n_lookup && !n)) {
    set_error("kc_fpset_stress: bad argument (batch > 0, 1 <= seed, seed + n + n_lookup < 2^63, "
              "lookups need inserts)");
    return -EINVAL;
  }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = s->stream;
  KC_TRY(s->fs.reserve(n, st));
  hipEvent_t e0, e1, e2;
  KC_HIP_TRY(hipEventCreate(&e0));
  KC_HIP_TRY(hipEventCreate(&e1));
  KC_HIP_TRY(hipEventCreate(&e2));
  KC_HIP_TRY(hipMemsetAsync(s->d_stats, 0, STAT_BYTES, st));
  KC_HIP_TRY(hipEventRecord(e0, st));
  for (uint64_t off = 0; off < n; off += batch) {
    const uint64_t m = std::min(batch, n - off);
    hipLaunchKernelGGL(k_stress_insert, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, seed,
                       off, m, s->fs.slots, s->fs.nbuckets, s->d_stats);
  }
  KC_HIP_TRY(hipEventRecord(e1, st));
  for (uint64_t off = 0; off < n_lookup; off += batch) {
    const uint64_t m = std::min(batch, n_lookup - off);
    hipLaunchKernelGGL(k_stress_lookup, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st,
                       seed, n, off, m, s->fs.slots, s->fs.nbuckets, s->d_stats);
  }
  KC_HIP_TRY(hipEventRecord(e2, st));
  KC_HIP_TRY(hipGetLastError());
  unsigned long long stats[4];
  KC_TRY(read_stats(s, st, stats));
  float ms1 = 0, ms2 = 0;
  KC_HIP_TRY(hipEventElapsedTime(&ms1, e0, e1));
  KC_HIP_TRY(hipEventElapsedTime(&ms2, e1, e2));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipEventDestroy(e2);
  s->fs.count += stats[0];
  if (insert_seconds) *insert_seconds = ms1 * 1e-3;
  if (lookup_seconds) *lookup_seconds = ms2 * 1e-3;
  if (found_out) *found_out = stats[2];
  return 0;
}

int kc_stress_fps_dev(uint64_t seed, int kind, uint64_t n_ins, uint64_t start, uint64_t n,
                      uint64_t* out_dev, void* hs) {
  if ((n && !out_dev) || (kind != 0 && kind != 1) || (kind == 1 && n_ins == 0) ||
      !stress_args_ok(seed, kind == 0 ? start + n : n_ins, kind == 0 ? 0 : start + n)) {
    set_error("kc_stress_fps_dev: bad argument");
    return -EINVAL;
  }
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_stress_gen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)hs,
                     seed, kind, n_ins, start, n, out_dev);
  KC_HIP_TRY(hipGetLastError());
  return 0;
}

uint64_t kc_stress_fp(uint64_t seed, int kind, uint64_t n_ins, uint64_t i) {
  return kind == 0 ? stress_insert_fp(seed, i) : stress_lookup_fp(seed, n_ins ? n_ins : 1, i);
}

int kc_fpset_partition_dev(kc_fpset* s, const uint64_t* fps_dev, uint64_t n, int world,
                           uint64_t* out_dev, uint64_t* counts_out, void* hs) {
  if (!s || world < 1 || world > PART_MAXR || !counts_out || (n && (!fps_dev || !out_dev)) ||
      fps_dev == out_dev) {
    set_error("kc_fpset_partition_dev: bad argument (1 <= world <= %d, distinct buffers)", PART_MAXR);
    return -EINVAL;
  }
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = hs ? (hipStream_t)hs : s->stream;
  for (int o = 0; o < world; ++o) counts_out[o] = 0;
  if (n == 0) return 0;
  const uint64_t ntiles = (n + PART_TILE - 1) / PART_TILE;
  const uint64_t cells = ntiles * (uint64_t)world;
  if (cells >= (1ull << 31) || n >= (1ull << 32)) {
    set_error("kc_fpset_partition_dev: batch too large (< 2^32 fingerprints)");
    return -EINVAL;
  }
  KC_TRY(grow_buffer(s->part_cnt, s->part_cap, cells + 1, false, st));
  KC_TRY(grow_buffer(s->part_off, s->part_off_cap, cells + 1, false, st));
  hipLaunchKernelGGL(k_part_count, dim3((unsigned)ntiles), dim3(256), 0, st, fps_dev, n, (uint32_t)world,
                     (uint32_t)ntiles, s->part_cnt);
  size_t tmp_bytes = 0;
  KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, s->part_cnt, s->part_off, (int)cells, st));
  KC_TRY(grow_buffer(s->scan_tmp, s->scan_cap, tmp_bytes + 16, false, st));
  KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(s->scan_tmp, tmp_bytes, s->part_cnt, s->part_off, (int)cells, st));
  hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)ntiles), dim3(256), 0, st, fps_dev, n, (uint32_t)world,
                     (uint32_t)ntiles, s->part_off, out_dev);
  KC_HIP_TRY(hipGetLastError());
  // per-owner totals: the owner-major scan's bases (owner o starts at
  // off[o * ntiles]); the last owner ends at n
  std::vector<uint32_t> base(world);
  for (int o = 0; o < world; ++o)
    KC_HIP_TRY(hipMemcpyAsync(&base[o], s->part_off + (uint64_t)o * ntiles, 4, hipMemcpyDeviceToHost, st));
  KC_HIP_TRY(hipStreamSynchronize(st));
  for (int o = 0; o < world; ++o)
    counts_out[o] = (o + 1 < world ? (uint64_t)base[o + 1] : n) - base[o];
  return 0;
}

static int count_dev(kc_fpset* s, const uint64_t* fps_dev, size_t n, uint64_t* out, void* hs, bool insert) {
  std::lock_guard<std::mutex> g(s->mu);
  KC_HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = hs ? (hipStream_t)hs : s->stream;
  if (insert) KC_TRY(s->fs.reserve(n, st));
  KC_HIP_TRY(hipMemsetAsync(s->d_stats, 0, STAT_BYTES, st));
  if (n) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (insert)
      hipLaunchKernelGGL(k_insert_count, dim3(grid), dim3(256), 0, st, fps_dev, (uint64_t)n, s->fs.slots,
                         s->fs.nbuckets, s->d_stats);
    else
      hipLaunchKernelGGL(k_contains_count, dim3(grid), dim3(256), 0, st, fps_dev, (uint64_t)n,
                         s->fs.slots, s->fs.nbuckets, s->d_stats);
    KC_HIP_TRY(hipGetLastError());
  }
  unsigned long long stats[4];
  KC_TRY(read_stats(s, st, stats));
  if (stats[1]) {
    set_error("fpset full");
    return -ENOMEM;
  }
  if (insert) s->fs.count += stats[0];
  *out = insert ? stats[0] : stats[2];
  return 0;
}

int kc_fpset_insert_count_dev(kc_fpset* s, const uint64_t* fps_dev, size_t n, uint64_t* n_new_out, void* hs) {
  if (!s || !n_new_out || (n && !fps_dev)) { set_error("kc_fpset_insert_count_dev: bad argument"); return -EINVAL; }
  return count_dev(s, fps_dev, n, n_new_out, hs, true);
}

int kc_fpset_contains_count_dev(kc_fpset* s, const uint64_t* fps_dev, size_t n, uint64_t* found_out, void* hs) {
  if (!s || !found_out || (n && !fps_dev)) { set_error("kc_fpset_contains_count_dev: bad argument"); return -EINVAL; }
  return count_dev(s, fps_dev, n, found_out, hs, false);
}

// ---- single-fingerprint put/contains from many host threads (flat combining)
// TLC's workers call FPSet.put(long) concurrently, one fingerprint each
// (MC.out:5 "4 workers").  A caller enqueues its request; if no batch is in
// flight it becomes the combiner: it takes every pending request (in arrival
// order), runs them as ONE put_batch launch (equal fps inside resolve in
// arrival order, as sequential puts would), publishes the results and
// repeats while requests are pending.  Other callers just wait for their
// result, so N concurrent workers cost one kernel launch per round, not N.
static int combine_one(kc_fpset* s, uint64_t fp, int op, uint8_t* result) {
  Combiner& c = s->comb;
  std::unique_lock<std::mutex> lk(c.mu);
  const uint64_t ticket = c.next_ticket++;
  c.pending.push_back({fp, op, ticket});
  for (;;) {
    auto it = c.done.find(ticket);
    if (it != c.done.end()) {
      const int rc = it->second.rc;
      *result = it->second.seen;
      // the combiner ran this request: its failure message, on this thread
      if (rc < 0) set_error("%s", it->second.msg.c_str());
      c.done.erase(it);
      return rc;
    }
    if (!c.busy) break;
    c.cv.wait(lk);
  }
  // become the combiner
  c.busy = true;
  while (!c.pending.empty()) {
    std::vector<Combiner::Req> batch;
    batch.swap(c.pending);
    lk.unlock();
    // puts and contains keep their relative order: consecutive runs of the
    // same op go out as one batch each
    std::vector<uint8_t> seen(batch.size());
    std::vector<int> rcs(batch.size(), 0);
    std::vector<std::string> msgs(batch.size());
    size_t a = 0;
    while (a < batch.size()) {
      size_t b = a;
      std::vector<uint64_t> fps;
      while (b < batch.size() && batch[b].op == batch[a].op) fps.push_back(batch[b++].fp);
      const int rc = fps.size() <= (size_t)SMALL_MAX
                         ? small_round(s, fps.data(), fps.size(), batch[a].op, seen.data() + a)
                         : batch[a].op == 0 ? kc_fpset_put_batch(s, fps.data(), fps.size(), seen.data() + a)
                                            : kc_fpset_contains_batch(s, fps.data(), fps.size(), seen.data() + a);
      const std::string m = rc < 0 ? std::string(last_error()) : std::string();
      for (size_t k = a; k < b; ++k) {
        rcs[k] = rc;
        msgs[k] = m;
      }
      a = b;
    }
    lk.lock();
    ++c.rounds;
    for (size_t k = 0; k < batch.size(); ++k) c.done[batch[k].ticket] = {seen[k], rcs[k], std::move(msgs[k])};
    c.cv.notify_all();
  }
  c.busy = false;
  auto it = c.done.find(ticket);
  const int rc = it->second.rc;
  *result = it->second.seen;
  if (rc < 0) set_error("%s", it->second.msg.c_str());
  c.done.erase(it);
  c.cv.notify_all();
  return rc;
}

int kc_fpset_put(kc_fpset* s, uint64_t fp, int* seen_out) {
  if (!s || !seen_out) { set_error("kc_fpset_put: NULL"); return -EINVAL; }
  uint8_t r = 0;
  const int rc = combine_one(s, fp, 0, &r);
  *seen_out = r;
  return rc;
}

int kc_fpset_contains(kc_fpset* s, uint64_t fp, int* seen_out) {
  if (!s || !seen_out) { set_error("kc_fpset_contains: NULL"); return -EINVAL; }
  uint8_t r = 0;
  const int rc = combine_one(s, fp, 1, &r);
  *seen_out = r;
  return rc;
}

uint64_t kc_fpset_combine_rounds(const kc_fpset* s) { return s ? s->comb.rounds : 0; }

}  // extern "C"
