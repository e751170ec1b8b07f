// fpset_host.h — host-side owner of an HBM FPSet (used by the engine and by
// the kc_fpset_* C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fpset_dev.h"

namespace kc {

// Grid of a grid-stride pass over a table of n entries (256 lanes per
// workgroup): at most 65,536 workgroups, so a table of 2^33+ slots does not
// ask for more than 2^32 lanes in one launch.
inline unsigned table_grid(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)(g < 65536 ? (g ? g : 1) : 65536);
}

struct DevFpset {
  unsigned long long* slots = nullptr;  // nbuckets * 8 u64
  uint64_t nbuckets = 0;
  uint64_t count = 0;                   // host-tracked number of stored fps
  unsigned long long* d_fail = nullptr; // rehash failure counter

  uint64_t capacity() const { return nbuckets * 8; }
  // allocate for >= min_slots slots (whole buckets), zeroed
  int init(uint64_t min_slots, hipStream_t st);
  void release();
  // grow (rehash into 2x..) so that count + extra <= 75% of capacity
  int reserve(uint64_t extra, hipStream_t st);
};

// Host owner of the engine's ClaimSet (fpset_dev.h): nslots 16-B entries,
// or (compact, the first-claim mode) nslots u64 fp words at the same address.
struct DevClaimSet {
  ClaimEntry* t = nullptr;
  uint64_t nslots = 0;
  uint64_t count = 0;                   // host-tracked number of stored fps
  unsigned long long* d_fail = nullptr;
  bool compact = false;                 // set before init(); fixed for the owner's life

  uint64_t capacity() const { return nslots; }
  uint64_t slot_bytes() const { return compact ? 8 : sizeof(ClaimEntry); }
  unsigned long long* words() const { return reinterpret_cast<unsigned long long*>(t); }
  uint32_t word_shift() const { return compact ? 0u : 1u; }   // slot i's fp word: words()[i << word_shift()]
  int init(uint64_t min_slots, hipStream_t st);
  int clear(hipStream_t st);
  void release();
  // grow (rehash) so that count + extra <= 1/2 of capacity
  int reserve(uint64_t extra, hipStream_t st);
};
// claim a device list of (normalised) fps at `level` with keys 0..n-1;
// d_res[i] = ClaimResult (may be NULL; a compact set reports CL_NEW / CL_OLD)
void launch_claimset_insert_list(const uint64_t* d_fps, uint64_t n, const DevClaimSet& cs,
                                 uint32_t level, int* d_res, hipStream_t st);

// Batch table used to dedup a batch by minimum order key.
struct DevBatchTable {
  BatchEntry* t = nullptr;
  uint64_t cap = 0;  // allocated entries (power of two)
  int ensure(uint64_t entries, hipStream_t st);  // grow allocation if needed
  void release();
};

uint64_t next_pow2(uint64_t x);
// insert a device list of (normalised) fps; d_res[i] = 1 new / 0 present (may be NULL)
void launch_fpset_insert_list(const uint64_t* d_fps, uint64_t n, const DevFpset& fs, int* d_res,
                              hipStream_t st);

}  // namespace kc
