// engine_spill.h — kernels of the engine's seen-set spill mode
// (kc_model_config.seen_hbm_bytes > 0; coldset.h has the cold tier).
//
// The hot tier is the ClaimSet at a fixed size.  Per chunk of parents:
//   k_tile_succ     successors per 256-parent tile, so the host can cut the
//                   level into chunks whose insertions fit the hot table;
//   k_claim / k_settle_rec / k_tile_scan as in the default path: the
//                   chunk's winners w.r.t. the HOT tier (newmask bits);
//   k_spill_queries each winner's cold key and (parent, position), at its
//                   tile offset (same wave-balanced dealing as k_emit);
//   [sort by key; ColdSet::probe]
//   k_spill_apply   winners found in the cold tier lose: newmask bit and tile
//                   count cleared, and the hot slot re-tagged "level 0" so
//                   every later copy (this level's later chunks included)
//                   reads it as old without another cold probe;
//   k_tile_scan, k_emit as usual.
// A flush (k_claimset_keys, sort, ColdSet::add_run, clear) happens between
// chunks.  Chunks of one level are processed in parent order and claims grow
// with the parent index, so a flushed claim of an earlier chunk is always the
// winner over a later chunk's copy, which now finds it in the cold tier.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "coldset.h"
#include "engine_kernels.h"
#include "fpset_dev.h"

namespace kc {

constexpr unsigned long long kClaimRetired = ~0ull;   // nclaim of a slot found in the cold tier (claim 0: level 0)

// successors per tile of 256 parents (plan totals, capped like k_claim)
template <class M>
__global__ void __launch_bounds__(256) k_tile_succ(const typename M::State* __restrict__ cur, uint64_t n, Flags f,
                                                   uint32_t* __restrict__ tsum) {
  __shared__ unsigned int sh[4];
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned int c = 0;
  if (i < n) {
    const int t = M::plan(load_state<M>(cur, i), f).total;
    c = (unsigned)(t > M::MAXSUCC ? M::MAXSUCC : t);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tsum[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// Every winner w.r.t. the hot tier -> (cold key, loc = parent-in-chunk << 5 | t),
// written at the chunk's exclusive tile offset plus the wave prefix.
template <class M>
__global__ void __launch_bounds__(256) k_spill_queries(const typename M::State* __restrict__ cur, uint64_t n, Flags f,
                                                       const uint32_t* __restrict__ newmask,
                                                       const uint32_t* __restrict__ tile_off,
                                                       uint64_t* __restrict__ qkey, uint32_t* __restrict__ qloc) {
  __shared__ unsigned int sh_wtot[4];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t mask = 0;
  uint64_t counts = 0;
  if (i < n) {
    mask = newmask[i];
    if (mask) counts = M::plan(load_state<M>(cur, i), f).counts;
  }
  const int cnt = __builtin_popcount(mask);
  const int lane = (int)(threadIdx.x & 63);
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  const int wtot = __shfl(incl, 63, 64);
  const int excl = incl - cnt;
  if (lane == 0) sh_wtot[threadIdx.x >> 6] = (unsigned int)wtot;
  __syncthreads();
  uint32_t obase = tile_off[blockIdx.x];
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) obase += sh_wtot[w];
  const uint64_t wave0 = i - (uint64_t)lane;
  for (int r = 0; r < wtot; r += 64) {
    const int g = r + lane;
    int p = 0;                                       // last lane with excl <= g
#pragma unroll
    for (int b = 32; b > 0; b >>= 1) {
      const int e = __shfl(excl, p + b, 64);
      if (e <= g) p += b;
    }
    int k = g - __shfl(excl, p, 64);
    uint32_t m = (uint32_t)__shfl((int)mask, p, 64);
    const uint64_t pc = __shfl(counts, p, 64);
    if (g >= wtot) continue;
    for (; k > 0; --k) m &= m - 1;
    const int t = __ffs(m) - 1;
    const uint64_t pi = wave0 + (uint64_t)p;
    const typename M::State s = load_state<M>(cur, pi);
    const typename M::Plan pl{pc, 0, -1, -1};
    int slot, j;
    M::locate(pl, t, slot, j);
    typename M::State x;
    M::apply(s, slot, j, f, x);
    const uint64_t o = (uint64_t)obase + (uint64_t)g;
    qkey[o] = cold_key(M::fingerprint(x));
    qloc[o] = (uint32_t)(pi << 5) | (uint32_t)t;
  }
}

// Re-tag fp's hot slot "level 0" (a claim of ~0 reads as old from every
// later level) and as already in the cold tier (flushes skip it).  False if
// fp is not in the table, which the protocol never produces.
__device__ __forceinline__ bool claimset_retire(ClaimEntry* __restrict__ cs, uint64_t nslots, uint64_t fp) {
  uint64_t s = bucket_of(fp, nslots);
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    const unsigned long long f = cs[s].fp;
    if (f == fp) {
      cs[s].nclaim = kClaimRetired;
      return true;
    }
    if (f == 0ull) break;
    s = (s + 1 == nslots) ? 0 : s + 1;
  }
  return false;
}

// Winners found in the cold tier lose (see the file comment).
static __global__ void k_spill_apply(const uint64_t* __restrict__ qkey, const uint32_t* __restrict__ qloc,
                              const uint8_t* __restrict__ found, uint64_t m, uint32_t* __restrict__ newmask,
                              uint32_t* __restrict__ tile_total, ClaimEntry* __restrict__ cs, uint64_t nslots,
                              Counters* __restrict__ C) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !found[i]) return;
  const uint32_t loc = qloc[i];
  atomicAnd(&newmask[loc >> 5], ~(1u << (loc & 31)));
  atomicSub(&tile_total[loc >> 13], 1u);              // tile = parent / 256
  if (!claimset_retire(cs, nslots, cold_unkey(qkey[i])))
    atomicAdd(&C->overflow, 1ull);                    // a winner's fp is always in the hot table
}

// Flush: the cold key of every live hot slot (retired slots are already in
// the cold tier) into a dense array; *count = how many.
static __global__ void k_claimset_keys(const ClaimEntry* __restrict__ t, uint64_t nslots, uint64_t* __restrict__ out,
                                uint64_t cap, unsigned long long* __restrict__ count) {
  // (grid-stride; the bound is uniform per wave, so the ballot sees every lane)
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < nslots; i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + threadIdx.x;
    bool live = false;
    uint64_t fp = 0;
    if (i < nslots) {
      const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(t + i);
      fp = e.x;
      live = fp != 0ull && e.y != kClaimRetired;
    }
    const unsigned long long b = __ballot(live);
    const int lane = (int)(threadIdx.x & 63);
    unsigned long long base = 0;
    if (lane == 0 && b) base = atomicAdd(count, (unsigned long long)__popcll(b));
    base = __shfl(base, 0, 64);
    if (live) {
      const uint64_t k = base + (uint64_t)__popcll(b & ((1ull << lane) - 1));
      if (k < cap) out[k] = cold_key(fp);
    }
  }
}

}  // namespace kc
