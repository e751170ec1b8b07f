// fpset_dev.h — device-side fingerprint set primitives (HBM, gfx950).
//
// Three tables:
//
//  * FPSet (the drop-in for TLC's tlc2.tool.fp.FPSet, MC.out:5
//    "OffHeapDiskFPSet"): open addressing over 64-B buckets of 8 u64 slots,
//    linear probing by bucket.  A probe is one 64-B line read (four 16-B
//    vector loads by one lane) plus, for a new fingerprint, one 64-bit
//    atomicCAS into the same line.  Slot value 0 = empty; stored
//    fingerprints have the MSB clear (TLC's disk FPSets reserve it) and are
//    never 0 (see normalize()).  Slots are never cleared, so a fingerprint
//    sits in the first slot that was empty along its probe sequence when it
//    was inserted — which makes `contains` stop at the first empty slot.
//
//  * Batch table (per BFS level chunk / per put_batch call): 16-B entries
//    {fp, ~key}.  Every candidate CAS-inserts its fp and then atomicMax'es
//    the complement of its order key, so after the pass each entry holds
//    the SMALLEST key that produced the fp: the deterministic "first
//    occurrence" a 1-worker TLC would have seen.  Only that representative
//    touches the FPSet.  Sized ~2x the batch so it stays in L2/MALL.
//    (Used by kc_fpset_put_batch and the sharded stages.)
//
//  * ClaimSet (the single-GPU engine's seen-set): the two fused — 16-B
//    {fp, ~claim} slots with linear probing, see below.
//
// Visibility: stale L1 copies can only show a slot as empty (0) that was
// filled in this launch; every such slot is re-checked by the CAS, whose
// returned value is authoritative (device-scope atomics execute at the
// memory side on gfx950).  A fingerprint is inserted by at most one lane per
// launch (the batch representative), so no duplicate can be created.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kc {

struct BatchEntry {
  unsigned long long fp;
  unsigned long long nkey;  // ~key; 0 = unclaimed (memset 0 initialises)
};

__host__ __device__ __forceinline__ uint64_t normalize_fp(uint64_t fp) {
  fp &= 0x7fffffffffffffffull;
  return fp ? fp : 1ull;
}

// KC_BUCKET_LOWBITS (A/B build switch): the bucket from the fingerprint's
// low 59 bits — the Zobrist fold, uniform on every path; the top bits are
// the sharded path's owner bits, which must not pick the bucket — with no
// remixing multiply (0: rounds 1-3's multiply-shift on a remixed fp)
#ifndef KC_BUCKET_LOWBITS
#define KC_BUCKET_LOWBITS 0
#endif
__device__ __forceinline__ uint64_t bucket_of(uint64_t fp, uint64_t nbuckets) {
#if KC_BUCKET_LOWBITS
  return __umul64hi(fp << 5, nbuckets);
#else
  // multiply-shift on a remixed fp: owner sharding uses the fp's top bits,
  // so the bucket index must not be a function of those bits alone.
  return __umul64hi(fp * 0x9e3779b97f4a7c15ull, nbuckets);
#endif
}
__device__ __forceinline__ uint64_t batch_slot(uint64_t fp, uint64_t mask) {
  uint64_t h = fp ^ (fp >> 29);
  h *= 0xbf58476d1ce4e5b9ull;
  return (h >> 21) & mask;
}

// The FPSet is one array of u64 slots (nbuckets * 8 of them; the 64-B
// "bucket" is only the allocation unit) probed linearly from
// bucket_of(fp, nslots).  Each probe step reads one aligned 16-B pair, so a
// lane issues one load per two slots instead of four per eight; at <= 1/2
// load almost every probe ends inside its first pair.
//
// Insert: 1 = newly inserted, 0 = already present, -1 = table full.
__device__ __forceinline__ int fpset_insert(unsigned long long* __restrict__ slots,
                                            uint64_t nbuckets, uint64_t fp) {
  const uint64_t ns = nbuckets * 8;
  uint64_t i = bucket_of(fp, ns);
  for (uint64_t probe = 0; probe < ns;) {
    const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(slots + (i & ~1ull));
    // slots i (and i+1 when i is even) in probe order
    for (int k = (int)(i & 1); k < 2; ++k, ++probe) {
      const unsigned long long e = k ? q.y : q.x;
      if (e == fp) return 0;
      if (e == 0ull) {
        const unsigned long long old = atomicCAS(slots + (i & ~1ull) + k, 0ull, (unsigned long long)fp);
        if (old == 0ull) return 1;
        if (old == fp) return 0;
      }
    }
    i = (i | 1ull) + 1 == ns ? 0 : (i | 1ull) + 1;
  }
  return -1;
}

// Lookup: 1 = present, 0 = absent (stops at the first empty slot).
__device__ __forceinline__ int fpset_contains(const unsigned long long* __restrict__ slots,
                                              uint64_t nbuckets, uint64_t fp) {
  const uint64_t ns = nbuckets * 8;
  uint64_t i = bucket_of(fp, ns);
  for (uint64_t probe = 0; probe < ns;) {
    const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(slots + (i & ~1ull));
    for (int k = (int)(i & 1); k < 2; ++k, ++probe) {
      const unsigned long long e = k ? q.y : q.x;
      if (e == fp) return 1;
      if (e == 0ull) return 0;
    }
    i = (i | 1ull) + 1 == ns ? 0 : (i | 1ull) + 1;
  }
  return 0;
}

// ---------------------------------------------------------------- ClaimSet
// The BFS engine's seen-set: the FPSet fused with the per-level "first
// occurrence" table.  Open addressing with linear probing over 16-B slots
// {fp, ~claim}, where claim = level << 44 | key and key = (parent index in
// level) << 8 | (successor position).  A probe is ONE 16-B load (measured on
// MI355X: one 16-B load per lane reaches ~48 G random probes/s at 16-64 GB
// tables, a lane reading a whole 64-B bucket with four loads ~20 G/s;
// tools/microbench/random_probe.hip).  Within one level every copy of a
// fingerprint does atomicMax(~claim), so after the level's claim pass the
// slot holds the SMALLEST key (the state a 1-worker TLC BFS meets first).
// Slots of older levels carry smaller levels, so a claim never changes them
// and a probe that finds one knows the state is old without any write.
// ~claim = 0 (never written) reads as "claim pending, current level".
struct ClaimEntry {
  unsigned long long fp;
  unsigned long long nclaim;  // ~(level << 44 | key); 0 = not yet set
};
constexpr int CLAIM_KEY_BITS = 44;   // key: [rank 4 |] parent index 32 | position 8
enum ClaimResult : int { CL_OLD = 0, CL_LOST = 1, CL_CUR = 2, CL_NEW = 3, CL_FULL = 4 };

__host__ __device__ __forceinline__ uint64_t make_claim(uint32_t level, uint64_t key) {
  return ((uint64_t)level << CLAIM_KEY_BITS) | key;
}

__device__ __forceinline__ int claim_settle(unsigned long long* nclaim_p, unsigned long long seen,
                                            unsigned long long nc, uint32_t level) {
  if (((~seen) >> CLAIM_KEY_BITS) < level) return CL_OLD;   // stored in an earlier level
  if (seen >= nc) return CL_LOST;                           // a smaller key is already there
  const unsigned long long prev = atomicMax(nclaim_p, nc);
  return prev < nc ? CL_CUR : CL_LOST;
}

// Claim fp for `claim` in the current `level`.  CL_NEW: inserted; CL_CUR:
// current-level entry whose claim this call lowered; CL_LOST: current-level
// entry already holding a smaller key; CL_OLD: stored by an earlier level;
// CL_FULL: no empty slot anywhere.  Stale (other-XCD L2) copies can only show
// slots as empty or claims as larger; both are settled by the atomics, whose
// returned values are authoritative.  Slots fill in probe order and are never
// cleared, so an fp is always found before the first truly empty slot.
__device__ __forceinline__ int claimset_claim(ClaimEntry* __restrict__ t, uint64_t nslots,
                                              uint64_t fp, uint64_t claim, uint32_t level) {
  const unsigned long long nc = ~(unsigned long long)claim;
  uint64_t i = bucket_of(fp, nslots);
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(t + i);
    if (e.x == fp) return claim_settle(&t[i].nclaim, e.y, nc, level);
    if (e.x == 0ull) {
      const unsigned long long old = atomicCAS(&t[i].fp, 0ull, (unsigned long long)fp);
      if (old == 0ull) {
        atomicMax(&t[i].nclaim, nc);
        return CL_NEW;
      }
      if (old == fp) return claim_settle(&t[i].nclaim, 0ull, nc, level);
    }
    i = (i + 1 == nslots) ? 0 : i + 1;
  }
  return CL_FULL;
}

// STORE-claim protocol (the single-GPU engine; one atomic per new state):
//   claim kernel — the lane whose CAS inserts fp writes its claim with a
//     PLAIN store (it is the slot's only writer in this kernel).  A lane that
//     finds fp stored by an earlier level: CL_OLD.  Finds a smaller claim
//     already stored: CL_LOST (no write).  Otherwise (claim word still 0, or
//     larger than its own): CL_CUR, a candidate, still without any write.
//   settle pass A (next kernel) — every CL_CUR candidate atomicMax'es its
//     claim into the slot (claimset_store_claim), so the slot ends with the
//     minimum over the inserter and all candidates;
//   settle pass B (next kernel) — every candidate and inserter wins iff the
//     stored claim is its own.
// The engine keeps the winners as per-parent bit masks and so re-reads only
// the displacers (engine_kernels.h, k_claim / k_settle_rec).
// Stale copies in another XCD's L2 can only show a slot empty or its claim
// word 0, which makes a lane a candidate (conservative); the CAS result is
// authoritative for the fp.
// The first probe's 16-B load split out, so a caller can issue the loads of
// several claims back to back (claimset_claim_store_from takes the slot index
// and the pair it loaded).
__device__ __forceinline__ ulonglong2 claimset_first(const ClaimEntry* __restrict__ t, uint64_t i) {
  return *reinterpret_cast<const ulonglong2*>(t + i);
}
__device__ __forceinline__ int claimset_claim_store_from(ClaimEntry* __restrict__ t, uint64_t nslots,
                                                         uint64_t fp, uint64_t claim, uint32_t level,
                                                         uint64_t i, ulonglong2 e) {
  const unsigned long long nc = ~(unsigned long long)claim;
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    if (probe) e = *reinterpret_cast<const ulonglong2*>(t + i);
    unsigned long long f = e.x, seen = e.y;
    if (f == 0ull) {
      f = atomicCAS(&t[i].fp, 0ull, (unsigned long long)fp);
      if (f == 0ull) {
        // agent-scope store: written through this XCD's L2, so claimants on
        // other XCDs see the claim (and lose at once) instead of a 0 word
        __hip_atomic_store(&t[i].nclaim, nc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return CL_NEW;
      }
      seen = 0ull;
    }
    if (f == fp) {
      if (seen != 0ull && ((~seen) >> CLAIM_KEY_BITS) < level) return CL_OLD;
      return (seen != 0ull && seen >= nc) ? CL_LOST : CL_CUR;
    }
    i = (i + 1 == nslots) ? 0 : i + 1;
  }
  return CL_FULL;
}
__device__ __forceinline__ int claimset_claim_store(ClaimEntry* __restrict__ t, uint64_t nslots,
                                                    uint64_t fp, uint64_t claim, uint32_t level) {
  const uint64_t i = bucket_of(fp, nslots);
  return claimset_claim_store_from(t, nslots, fp, claim, level, i, claimset_first(t, i));
}

// First-claim mode (k_claim FIRST): the CAS that inserts fp is the claim and
// no claim word is written.  From slot i, whose fp word the caller loaded as
// f.  CL_NEW: this call inserted fp; CL_OLD: fp is present; CL_FULL.
__device__ __forceinline__ int claimset_insert_from(ClaimEntry* __restrict__ t, uint64_t nslots, uint64_t fp,
                                                    uint64_t i, unsigned long long f) {
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    if (probe) f = t[i].fp;
    if (f == 0ull) {
      f = atomicCAS(&t[i].fp, 0ull, (unsigned long long)fp);
      if (f == 0ull) return CL_NEW;
    }
    if (f == fp) return CL_OLD;
    i = (i + 1 == nslots) ? 0 : i + 1;
  }
  return CL_FULL;
}

// Compact ClaimSet (round 6; the engine's first-claim mode, DevClaimSet::
// compact): the claim word is never read there, so a slot is the fp word
// alone — 8 B instead of 16, half the table to allocate and clear per check
// for the same slot count and load.  `t` is the u64 slot array.  A
// fingerprint's home is an even slot (fpslots_home), so the first probe is
// one aligned 16-B load of the pair {home, home + 1} (fpslots_insert_pair):
// a probe run of two slots costs one round trip instead of two.
__device__ __forceinline__ uint64_t fpslots_home(uint64_t fp, uint64_t nslots) {
  return bucket_of(fp, nslots >> 1) << 1;
}
__device__ __forceinline__ ulonglong2 fpslots_first(const unsigned long long* __restrict__ t, uint64_t home) {
  return *reinterpret_cast<const ulonglong2*>(t + home);
}
__device__ __forceinline__ int fpslots_insert_from(unsigned long long* __restrict__ t, uint64_t nslots, uint64_t fp,
                                                   uint64_t i, unsigned long long f) {
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    if (probe) f = t[i];
    if (f == 0ull) {
      f = atomicCAS(&t[i], 0ull, (unsigned long long)fp);
      if (f == 0ull) return CL_NEW;
    }
    if (f == fp) return CL_OLD;
    i = (i + 1 == nslots) ? 0 : i + 1;
  }
  return CL_FULL;
}

// From the pair e = {t[home], t[home + 1]} loaded together (home even):
// CL_OLD when either holds fp; else the CAS into the first that read empty,
// then linear probing on.  `cas` (~0: not issued) is the result of that CAS
// when the caller issued it already (fpslots_pair_target).
__device__ __forceinline__ uint64_t fpslots_pair_target(uint64_t home, ulonglong2 e, uint64_t fp) {
  if (e.x == fp || e.y == fp) return ~0ull;                       // present: no CAS
  return e.x == 0ull ? home : e.y == 0ull ? home + 1 : ~1ull;      // ~1: both held other fps
}
__device__ __forceinline__ int fpslots_insert_pair(unsigned long long* __restrict__ t, uint64_t nslots, uint64_t fp,
                                                   uint64_t home, ulonglong2 e, unsigned long long cas = ~0ull) {
  const uint64_t j = fpslots_pair_target(home, e, fp);
  if (j == ~0ull) return CL_OLD;
  if (j == ~1ull) {
    const uint64_t k = home + 2 == nslots ? 0 : home + 2;
    return fpslots_insert_from(t, nslots, fp, k, t[k]);
  }
  const unsigned long long f = cas != ~0ull ? cas : atomicCAS(&t[j], 0ull, (unsigned long long)fp);
  if (f == 0ull) return CL_NEW;
  if (f == fp) return CL_OLD;
  if (j == home) return fpslots_insert_from(t, nslots, fp, home + 1, e.y);   // (a stale e.y is re-checked by its CAS)
  const uint64_t k = j + 1 == nslots ? 0 : j + 1;
  return fpslots_insert_from(t, nslots, fp, k, t[k]);
}

// Settle pass A of a CL_CUR candidate: fold its claim into the slot.
// Returns the ~claim the slot held before (0 if fp is absent, which the
// protocol never produces).
__device__ __forceinline__ unsigned long long claimset_store_claim(ClaimEntry* __restrict__ t,
                                                                   uint64_t nslots, uint64_t fp,
                                                                   uint64_t claim) {
  uint64_t i = bucket_of(fp, nslots);
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    const unsigned long long f = t[i].fp;
    if (f == fp) return atomicMax(&t[i].nclaim, ~(unsigned long long)claim);
    if (f == 0ull) return 0ull;
    i = (i + 1 == nslots) ? 0 : i + 1;
  }
  return 0ull;
}

// ~claim stored for fp (0 if absent).  Called in a later kernel than the
// claims, so every claim is visible.
__device__ __forceinline__ unsigned long long claimset_get(const ClaimEntry* __restrict__ t,
                                                           uint64_t nslots, uint64_t fp) {
  uint64_t i = bucket_of(fp, nslots);
  for (uint64_t probe = 0; probe < nslots; ++probe) {
    const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(t + i);
    if (e.x == fp) return e.y;
    if (e.x == 0ull) return 0;
    i = (i + 1 == nslots) ? 0 : i + 1;
  }
  return 0;
}

// Batch table: record (fp, key); keeps the minimum key per fp.
__device__ __forceinline__ void batch_insert(BatchEntry* __restrict__ t, uint64_t mask,
                                             uint64_t fp, uint64_t key) {
  uint64_t i = batch_slot(fp, mask);
  for (;;) {
    unsigned long long e = t[i].fp;
    if (e == 0ull) {
      e = atomicCAS(&t[i].fp, 0ull, (unsigned long long)fp);
      if (e == 0ull) e = fp;
    }
    if (e == fp) {
      atomicMax(&t[i].nkey, ~(unsigned long long)key);
      return;
    }
    i = (i + 1) & mask;
  }
}
// After the insert pass: is `key` the smallest key recorded for fp?
__device__ __forceinline__ bool batch_is_rep(const BatchEntry* __restrict__ t, uint64_t mask,
                                             uint64_t fp, uint64_t key) {
  uint64_t i = batch_slot(fp, mask);
  for (;;) {
    const unsigned long long e = t[i].fp;
    if (e == fp) return t[i].nkey == ~(unsigned long long)key;
    if (e == 0ull) return false;  // unreachable: every fp was inserted
    i = (i + 1) & mask;
  }
}

}  // namespace kc
