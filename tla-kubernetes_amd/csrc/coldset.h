// coldset.h — the cold tier of the engine's seen-set (seen-set spill).
//
// The reference's run used TLC's OffHeapDiskFPSet (MC.out:5): an in-memory
// table whose contents are flushed into a sorted disk file, later lookups
// checking the table first and the sorted file second.  The engine's version
// keeps the ClaimSet in HBM as the hot tier under an HBM budget
// (kc_model_config.seen_hbm_bytes); when it fills, its fingerprints are
// flushed into a sorted RUN here.  Runs live in pinned host RAM, which the
// GPU reads directly over the host link, or, past seen_host_bytes, in files
// in spill_dir, streamed through pinned staging windows.  Each run has in HBM:
//   * a directory: dir[b] = first index whose key's top `dbits` bits are >= b
//     (about 16 keys per bucket), so a lookup reads the run near one
//     interpolated position instead of binary-searching it;
//   * optionally a blocked Bloom filter (one 64-B block per key, 6 bits), so
//     most lookups of truly new states never leave HBM.
// Runs are size-tiered: a new run is merged (on the host, by key range in
// parallel threads) with the previous one while that one is at most twice
// its size, so a query probes O(log flushes) runs.
//
// Keys are cold_key(fp): a bijective 64-bit mix of the fingerprint, uniform
// in every bit (a fingerprint's top bits are the owner bits, a projection
// hash: far from uniform), which the directory and the interpolation need.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace kc {

namespace coldmix {
constexpr uint64_t M1 = 0xbf58476d1ce4e5b9ull, M2 = 0x94d049bb133111ebull;
// multiplicative inverse mod 2^64 of an odd constant (Newton: 3 -> 96 bits)
__host__ __device__ constexpr uint64_t inv64(uint64_t a) {
  uint64_t x = a;
  for (int i = 0; i < 5; ++i) x *= 2 - a * x;
  return x;
}
constexpr uint64_t I1 = inv64(M1), I2 = inv64(M2);
static_assert(M1 * I1 == 1ull && M2 * I2 == 1ull, "inverse");
__host__ __device__ __forceinline__ uint64_t unxorshift(uint64_t y, int s) {
  uint64_t x = y;
  for (int k = s; k < 64; k += s) x = y ^ (x >> s);
  return x;
}
}  // namespace coldmix

__host__ __device__ __forceinline__ uint64_t cold_key(uint64_t fp) {
  uint64_t z = fp;
  z = (z ^ (z >> 30)) * coldmix::M1;
  z = (z ^ (z >> 27)) * coldmix::M2;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t cold_unkey(uint64_t k) {
  uint64_t z = coldmix::unxorshift(k, 31) * coldmix::I2;
  z = coldmix::unxorshift(z, 27) * coldmix::I1;
  return coldmix::unxorshift(z, 30);
}

// One sorted run of keys.
struct ColdRun {
  uint64_t n = 0;                 // keys
  uint64_t* host = nullptr;       // pinned host RAM (device-readable), or nullptr on disk
  uint64_t host_cap = 0;          // keys the pinned buffer holds (pooled: >= n)
  std::string path;               // the spill file when on disk
  uint64_t* d_dir = nullptr;      // HBM: 2^dbits + 1 entries
  int dbits = 1;
  uint32_t* d_bloom = nullptr;    // HBM: nblocks x 16 words (nullptr = no filter)
  uint64_t nblocks = 0;
  uint64_t meta_bytes = 0;        // HBM of dir + filter
  uint64_t* d_keys = nullptr;     // HBM copy of the keys (the newest runs, as the budget allows)
  // disk runs: staging windows of wkeys keys; window w holds the keys in
  // [d_wkeys[w], d_wkeys[w + 1]) (d_wkeys[0] = 0, d_wkeys[nw] = ~0: HBM)
  uint64_t wkeys = 0, nw = 0;
  uint64_t* d_wkeys = nullptr;
  uint64_t bytes() const { return n * 8; }
};

struct ColdStats {
  uint64_t runs = 0, runs_disk = 0, keys = 0;
  uint64_t host_bytes = 0, disk_bytes = 0, meta_bytes = 0, peak_meta_bytes = 0;
  uint64_t merges = 0, merged_keys = 0, disk_written = 0, disk_read = 0, windows_skipped = 0;
  uint64_t cached_runs = 0, cached_keys = 0, cache_bytes = 0, cache_uploaded = 0;
  uint64_t filter_tests = 0, filter_passed = 0;   // query x run pairs a filter saw / let through
  uint64_t merge_probes = 0;                       // (query set, run) pairs read as a streaming merge
  // host wall time: pinning buffers, CPU merges, directory/filter builds
  // (incl. the copy of a new run), writing runs to files
  double pin_seconds = 0, merge_seconds = 0, meta_seconds = 0, evict_seconds = 0;
};

class ColdSet {
 public:
  struct Config {
    int device = 0;
    uint64_t meta_hbm_bytes = 0;   // HBM for directories + filters (0 = unlimited)
    uint64_t host_bytes = 0;       // pinned host RAM for runs (0 = unlimited)
    std::string dir;               // spill directory ("" = none: past host_bytes -ENOMEM)
    uint64_t window_keys = 1ull << 23;   // disk runs: keys per staging window
    int merge_threads = 16;
    int bloom_bits = 10;           // target filter bits per key (0 = no filters)
    bool cache_keys = true;        // copy the newest runs' keys into what HBM budget is left
    // a host run probed by m >= n / merge_div sorted queries is read once,
    // sequentially, by k_cold_merge_probe instead of ~1.2 random 64-B reads
    // per query (0 = never, the default: no gain measured on NP=2 under a
    // 4 GiB seen-set; KC_COLD_MERGE_DIV overrides)
    int merge_div = 0;
  };
  ColdSet() = default;
  ~ColdSet();
  ColdSet(const ColdSet&) = delete;
  ColdSet& operator=(const ColdSet&) = delete;

  int init(const Config& c);
  void clear();                    // drop every run (files unlinked)
  uint64_t size() const { return keys_; }
  bool empty() const { return runs_.empty(); }
  // Add the n keys at d_sorted (device memory, ascending, distinct; the
  // caller may reuse the buffer once this returns) as a new run, then merge
  // and evict as the tiering and the host budget require.  Synchronous on st.
  int add_run(const uint64_t* d_sorted, uint64_t n, hipStream_t st);
  // found[i] |= key q[i] is in some run (q: device, ascending, m keys;
  // found: device u8).  Adds the hits to *d_hits (device counter).
  // Enqueued on st; synchronises only to stream disk runs.
  int probe(const uint64_t* d_q, uint64_t m, uint8_t* d_found, unsigned long long* d_hits, hipStream_t st);
  void stats(ColdStats* s) const;
  // the sorted keys of every run, merged (host; tests and checkFPs)
  int all_keys(std::vector<uint64_t>& out);

 private:
  int build_meta(ColdRun& r, const uint64_t* keys_dev_or_host, hipStream_t st);
  void free_meta(ColdRun& r);
  int merge_last_two(hipStream_t st);
  int evict_oldest_host(hipStream_t st);
  int read_window(const ColdRun& r, uint64_t w0, uint64_t w1, uint64_t* dst);
  void free_run(ColdRun& r);
  int staging(uint64_t keys);
  // HBM copies of run keys: newest runs first, within what the directories
  // and filters leave of the budget; dropped oldest-first when a new run's
  // directory and filter need the room
  int recache(hipStream_t st);
  void uncache(ColdRun& r);
  void make_room(uint64_t bytes);
  uint64_t cache_used_ = 0, cache_uploaded_ = 0;
  // pinned host buffers are pooled: pinning GBs of pages costs more than the
  // merges that use them
  int pin_get(uint64_t keys, uint64_t** p, uint64_t* cap);
  void pin_put(uint64_t* p, uint64_t cap);
  std::vector<std::pair<uint64_t*, uint64_t>> pool_;
  double t_pin_ = 0, t_merge_ = 0, t_meta_ = 0, t_evict_ = 0;

  Config cfg_;
  std::vector<ColdRun> runs_;      // oldest first
  uint64_t keys_ = 0, host_used_ = 0, disk_used_ = 0, meta_used_ = 0, peak_meta_ = 0;
  uint64_t merges_ = 0, merged_keys_ = 0, disk_written_ = 0, disk_read_ = 0, windows_skipped_ = 0;
  uint64_t merge_probes_ = 0;                  // (query set, run) pairs probed by the streaming merge
  uint64_t file_seq_ = 0, id_ = 0;
  uint64_t* stage_[2] = {nullptr, nullptr};   // pinned staging windows (disk runs)
  uint64_t stage_keys_ = 0;
  hipEvent_t stage_ev_[2] = {nullptr, nullptr};
  unsigned long long* d_stat_ = nullptr;       // [0] queries seen by filters, [1] passed
  uint64_t* d_qa_ = nullptr;                   // disk runs: first query of each window
  uint64_t* h_qa_ = nullptr;
  uint64_t qa_cap_ = 0;
};

}  // namespace kc
