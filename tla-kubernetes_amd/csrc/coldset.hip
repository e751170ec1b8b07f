// coldset.hip — the seen-set's cold tier (coldset.h): sorted fingerprint
// runs in pinned host RAM or spill files, with HBM directories and Bloom
// filters, probed by the GPU.  TLC's DiskFPSet keeps the same shape (an
// in-memory table flushed into a sorted file with an index; MC.out:5
// "OffHeapDiskFPSet"); here the lookups are batched GPU kernels over a
// level's sorted new fingerprints, and the host only merges runs and moves
// bytes to and from files.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <thread>

#include "coldset.h"
#include "kc_common.h"

namespace kc {

namespace {

constexpr int kBloomK = 6;            // bits per key, in one 512-bit block
__device__ __forceinline__ uint64_t bloom_block(uint64_t k, uint64_t nblocks) {
  return __umul64hi(k * 0x9e3779b97f4a7c15ull, nblocks);
}
__device__ __forceinline__ uint64_t bloom_hash(uint64_t k) {
  uint64_t h = (k ^ (k >> 32)) * 0xd6e8feb86659fd93ull;
  return h ^ (h >> 29);
}

__host__ __device__ __forceinline__ uint64_t dir_bucket(uint64_t k, int dbits) { return k >> (64 - dbits); }

// dir[b] = first index whose bucket is >= b (b in [0, 2^dbits]): thread i
// writes the buckets in (bucket(i-1), bucket(i)], thread n the tail.
// Directory and filter in one pass over the keys (a merged run is read
// over the host link once, not twice).
__global__ void k_run_meta(const uint64_t* __restrict__ keys, uint64_t n, uint64_t* __restrict__ dir, int dbits,
                           uint32_t* __restrict__ bloom, uint64_t nblocks) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const uint64_t nb = 1ull << dbits;
  const uint64_t k = i < n ? keys[i] : 0;
  const uint64_t hi = i < n ? dir_bucket(k, dbits) : nb;
  // the previous key's bucket: a neighbour lane's load (same line), or a load
  const uint64_t prev = __shfl_up(k, 1, 64);
  const uint64_t kp = i == 0 ? 0 : ((threadIdx.x & 63) ? prev : keys[i - 1]);
  const uint64_t lo = i > 0 ? dir_bucket(kp, dbits) + 1 : 0;
  for (uint64_t b = lo; b <= hi; ++b) dir[b] = i;
  if (bloom && i < n) {
    uint32_t* blk = bloom + bloom_block(k, nblocks) * 16;
    uint64_t h = bloom_hash(k);
    for (int j = 0; j < kBloomK; ++j, h >>= 9) atomicOr(&blk[(h >> 5) & 15], 1u << (h & 31));
  }
}

// One query against one run, restricted to the run's indices [w0, w1) held
// at win[j - w0].  The directory gives the key's bucket [lo, hi); keys in a
// bucket are uniform over its key range, so the search starts at the
// interpolated position and reads whole aligned 8-key lines (one 64-B
// request each over the host link) until the key's place is bracketed:
// about 1.2 lines per lookup.
__host__ __device__ __forceinline__ bool run_find(uint64_t k, const uint64_t* __restrict__ win, uint64_t w0, uint64_t w1,
                                         const uint64_t* __restrict__ dir, int dbits) {
  const uint64_t b = dir_bucket(k, dbits);
  const uint64_t blo = dir[b], bhi = dir[b + 1];
  const uint64_t lo = blo > w0 ? blo : w0, hi = bhi < w1 ? bhi : w1;
  if (lo >= hi) return false;
  // interpolation inside the bucket: the key's bits below the bucket bits
  const uint64_t frac = (k << dbits) >> 32;                     // 32-bit fraction
  uint64_t pos = blo + (((bhi - blo) * frac) >> 32);
  pos = pos < lo ? lo : (pos >= hi ? hi - 1 : pos);
  uint64_t a = pos & ~7ull;
  if (a < lo) a = lo;
  // walk lines away from the guess in ONE direction: a key that falls
  // between two lines' ranges is absent (turning back would loop forever)
  int way = 0;
  for (uint64_t steps = 0; steps <= (hi - lo) / 8 + 2; ++steps) {
    uint64_t e = (a | 7ull) + 1;
    if (e > hi) e = hi;
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = a + u < e ? win[a + u - w0] : ~0ull;
    if (k < v[0]) {
      if (a == lo || way > 0) return false;
      way = -1;
      a = (a - 1) & ~7ull;
      if (a < lo) a = lo;
      continue;
    }
    uint64_t last = v[0];
#pragma unroll
    for (int u = 1; u < 8; ++u) last = a + u < e ? v[u] : last;
    if (k > last) {
      if (e >= hi || way < 0) return false;
      way = 1;
      a = e;
      continue;
    }
    bool hit = false;
#pragma unroll
    for (int u = 0; u < 8; ++u) hit |= v[u] == k;
    return hit;
  }
  return false;
}

// stat[0]: filter tests (query x run), stat[1]: those it passed
__global__ void k_cold_probe(const uint64_t* __restrict__ q, uint64_t m, uint8_t* __restrict__ found,
                             const uint64_t* __restrict__ win, uint64_t w0, uint64_t w1,
                             const uint64_t* __restrict__ dir, int dbits, const uint32_t* __restrict__ bloom,
                             uint64_t nblocks, unsigned long long* __restrict__ hits,
                             unsigned long long* __restrict__ stat) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool hit = false, tested = false, passed = false;
  if (i < m && !found[i]) {
    const uint64_t k = q[i];
    bool maybe = true;
    if (bloom) {
      tested = true;
      const uint32_t* blk = bloom + bloom_block(k, nblocks) * 16;
      uint64_t h = bloom_hash(k);
#pragma unroll
      for (int j = 0; j < kBloomK; ++j, h >>= 9) maybe &= (blk[(h >> 5) & 15] >> (h & 31)) & 1u;
      passed = maybe;
    }
    if (maybe && run_find(k, win, w0, w1, dir, dbits)) {
      hit = true;
      found[i] = 1;
    }
  }
  const unsigned long long bh = __ballot(hit), bt = __ballot(tested), bp = __ballot(passed);
  if ((threadIdx.x & 63) == 0) {
    if (bh) atomicAdd(hits, (unsigned long long)__popcll(bh));
    if (bt) atomicAdd(&stat[0], (unsigned long long)__popcll(bt));
    if (bp) atomicAdd(&stat[1], (unsigned long long)__popcll(bp));
  }
}

// Streaming merge-probe of sorted queries against one run: workgroup b
// reads the run's keys [b * MSEG, (b + 1) * MSEG) once, in order (coalesced
// loads; over the host link for a pinned run), into LDS, then finds the
// queries that fall in that key range (two binary searches over the sorted
// queries) by binary search in LDS.  Reads n * 8 bytes sequentially instead
// of ~1.2 random 64-B lines per query: the better trade once queries exceed
// a few percent of the run (host link: ~56 GB/s streamed vs ~310M random
// lines/s).
constexpr int MSEG = 2048;
__device__ __forceinline__ uint64_t lower_bound_dev(const uint64_t* __restrict__ a, uint64_t n, uint64_t k) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (a[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__global__ void __launch_bounds__(256)
k_cold_merge_probe(const uint64_t* __restrict__ q, uint64_t m, uint8_t* __restrict__ found,
                   const uint64_t* __restrict__ keys, uint64_t n, unsigned long long* __restrict__ hits) {
  __shared__ uint64_t seg[MSEG];
  __shared__ uint64_t qr[2];
  const uint64_t s0 = (uint64_t)blockIdx.x * MSEG;
  const uint32_t cnt = (uint32_t)(n - s0 < (uint64_t)MSEG ? n - s0 : (uint64_t)MSEG);
  for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) seg[j] = keys[s0 + j];
  __syncthreads();
  if (threadIdx.x < 2) {
    // queries in [first key, last key] of this segment
    qr[threadIdx.x] = threadIdx.x == 0 ? lower_bound_dev(q, m, seg[0])
                                       : (seg[cnt - 1] == ~0ull ? m : lower_bound_dev(q, m, seg[cnt - 1] + 1));
  }
  __syncthreads();
  unsigned long long h = 0;
  for (uint64_t i = qr[0] + threadIdx.x; i < qr[1]; i += blockDim.x) {
    if (found[i]) continue;
    const uint64_t k = q[i];
    uint32_t lo = 0, hi = cnt;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (seg[mid] < k) lo = mid + 1;
      else hi = mid;
    }
    if (lo < cnt && seg[lo] == k) {
      found[i] = 1;
      ++h;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) h += __shfl_down(h, off, 64);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(hits, h);
}

// qa[w] = first sorted query >= bound[w] (w = 0..nw)
__global__ void k_window_ranges(const uint64_t* __restrict__ q, uint64_t m, const uint64_t* __restrict__ bound,
                                uint64_t nw, uint64_t* __restrict__ qa) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w > nw) return;
  if (w == nw) {
    qa[w] = m;
    return;
  }
  const uint64_t b = bound[w];
  uint64_t lo = 0, hi = m;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (q[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  qa[w] = lo;
}

unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

// Best fit from the pool, else a fresh pinned buffer with 1/4 slack (the
// size-tiered runs come in a few recurring sizes).
int ColdSet::pin_get(uint64_t keys, uint64_t** p, uint64_t* cap) {
  size_t best = pool_.size();
  for (size_t i = 0; i < pool_.size(); ++i)
    if (pool_[i].second >= keys && (best == pool_.size() || pool_[i].second < pool_[best].second)) best = i;
  if (best < pool_.size()) {
    *p = pool_[best].first;
    *cap = pool_[best].second;
    pool_.erase(pool_.begin() + best);
    return 0;
  }
  const double t0 = now_s();
  // power-of-two size classes: runs of the binary-counter tiering recur in
  // a few sizes, so freed buffers are reused instead of pinning new pages
  uint64_t c = 1ull << 16;
  while (c < keys) c *= 2;
  KC_HIP_TRY(hipHostMalloc(p, c * 8));
  *cap = c;
  t_pin_ += now_s() - t0;
  return 0;
}
// Back to the pool; the pool keeps its 6 largest buffers.
void ColdSet::pin_put(uint64_t* p, uint64_t cap) {
  if (!p) return;
  pool_.push_back({p, cap});
  std::sort(pool_.begin(), pool_.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
  while (pool_.size() > 6) {
    (void)hipHostFree(pool_.back().first);
    pool_.pop_back();
  }
}

ColdSet::~ColdSet() {
  clear();
  if (d_qa_) (void)hipFree(d_qa_);
  if (h_qa_) (void)hipHostFree(h_qa_);
  for (int s = 0; s < 2; ++s) {
    if (stage_[s]) (void)hipHostFree(stage_[s]);
    if (stage_ev_[s]) (void)hipEventDestroy(stage_ev_[s]);
  }
  if (d_stat_) (void)hipFree(d_stat_);
  for (auto& b : pool_) (void)hipHostFree(b.first);
  pool_.clear();
}

int ColdSet::init(const Config& c) {
  static uint64_t ids = 0;
  cfg_ = c;
  if (cfg_.window_keys < 64) cfg_.window_keys = 64;
  cfg_.window_keys &= ~7ull;
  if (cfg_.merge_threads < 1) cfg_.merge_threads = 1;
  const char* md = getenv("KC_COLD_MERGE_DIV");     // (A/B: 0 = random probes only)
  if (md) cfg_.merge_div = atoi(md);
  id_ = ++ids;
  if (!d_stat_) {
    KC_HIP_TRY(hipMalloc(&d_stat_, 16));
    KC_HIP_TRY(hipMemset(d_stat_, 0, 16));
  }
  return 0;
}

void ColdSet::free_meta(ColdRun& r) {
  if (r.d_wkeys) (void)hipFree(r.d_wkeys);
  r.d_wkeys = nullptr;
  r.nw = r.wkeys = 0;
  if (r.d_dir) (void)hipFree(r.d_dir);
  if (r.d_bloom) (void)hipFree(r.d_bloom);
  meta_used_ -= r.meta_bytes;
  r.d_dir = nullptr;
  r.d_bloom = nullptr;
  r.meta_bytes = 0;
  r.nblocks = 0;
}

void ColdSet::uncache(ColdRun& r) {
  if (!r.d_keys) return;
  (void)hipFree(r.d_keys);
  r.d_keys = nullptr;
  cache_used_ -= r.bytes();
}

// free key copies, oldest run first, until `bytes` of the budget are free
void ColdSet::make_room(uint64_t bytes) {
  if (!cfg_.meta_hbm_bytes) return;
  for (auto& r : runs_) {
    if (meta_used_ + cache_used_ + bytes <= cfg_.meta_hbm_bytes) return;
    uncache(r);
  }
}

int ColdSet::recache(hipStream_t st) {
  if (!cfg_.cache_keys) return 0;
  for (size_t k = runs_.size(); k-- > 0;) {            // newest first
    ColdRun& r = runs_[k];
    if (r.d_keys || r.n == 0) continue;
    if (cfg_.meta_hbm_bytes && meta_used_ + cache_used_ + r.bytes() > cfg_.meta_hbm_bytes) break;
    if (hipMalloc(&r.d_keys, r.bytes()) != hipSuccess) {
      r.d_keys = nullptr;
      (void)hipGetLastError();
      break;
    }
    cache_used_ += r.bytes();
    cache_uploaded_ += r.bytes();
    if (r.host) {
      KC_HIP_TRY(hipMemcpyAsync(r.d_keys, r.host, r.bytes(), hipMemcpyHostToDevice, st));
    } else {                                             // a file run: through the staging windows
      KC_TRY(staging(r.wkeys));
      for (uint64_t w0 = 0; w0 < r.n; w0 += r.wkeys) {
        const uint64_t w1 = std::min(r.n, w0 + r.wkeys);
        KC_HIP_TRY(hipStreamSynchronize(st));
        KC_TRY(read_window(r, w0, w1, stage_[0]));
        KC_HIP_TRY(hipMemcpyAsync(r.d_keys + w0, stage_[0], (w1 - w0) * 8, hipMemcpyHostToDevice, st));
      }
    }
  }
  peak_meta_ = std::max(peak_meta_, meta_used_ + cache_used_);
  KC_HIP_TRY(hipStreamSynchronize(st));
  return 0;
}

void ColdSet::free_run(ColdRun& r) {
  uncache(r);
  free_meta(r);
  if (r.host) {
    pin_put(r.host, r.host_cap);
    host_used_ -= r.bytes();
  }
  if (!r.path.empty()) {
    unlink(r.path.c_str());
    disk_used_ -= r.bytes();
  }
  keys_ -= r.n;
  r = ColdRun{};
}

void ColdSet::clear() {
  (void)hipDeviceSynchronize();
  for (auto& r : runs_) free_run(r);
  runs_.clear();
  if (d_stat_) (void)hipMemset(d_stat_, 0, 16);
  merges_ = merged_keys_ = disk_written_ = disk_read_ = windows_skipped_ = 0;
  cache_uploaded_ = 0;
  t_pin_ = t_merge_ = t_meta_ = t_evict_ = 0;
  peak_meta_ = meta_used_;
}

// Directory (mandatory) and filter (as the HBM budget allows) of run r from
// its keys (device memory or pinned host RAM: the kernels read either).
int ColdSet::build_meta(ColdRun& r, const uint64_t* keys, hipStream_t st) {
  int dbits = 1;
  while ((1ull << (dbits + 1)) * 16 <= r.n && dbits < 40) ++dbits;
  const uint64_t dir_bytes = ((1ull << dbits) + 1) * 8;
  // directories and filters come before key copies
  make_room(dir_bytes + (uint64_t)cfg_.bloom_bits * r.n / 8 + 64);
  if (cfg_.meta_hbm_bytes && meta_used_ + dir_bytes > cfg_.meta_hbm_bytes) {
    set_error("seen-set: HBM budget for cold-run directories exhausted (%llu + %llu > %llu B); raise seen_hbm_bytes",
              (unsigned long long)meta_used_, (unsigned long long)dir_bytes,
              (unsigned long long)cfg_.meta_hbm_bytes);
    return -ENOMEM;
  }
  KC_HIP_TRY(hipMalloc(&r.d_dir, dir_bytes));
  r.dbits = dbits;
  r.meta_bytes = dir_bytes;
  meta_used_ += dir_bytes;
  // filter bits per key: the target, or what the budget has left
  uint64_t bits = (uint64_t)cfg_.bloom_bits;
  if (cfg_.meta_hbm_bytes && r.n) {
    const uint64_t left = cfg_.meta_hbm_bytes - meta_used_ - cache_used_;
    bits = std::min<uint64_t>(bits, left * 8 / r.n);
  }
  if (bits >= 4 && r.n) {
    r.nblocks = std::max<uint64_t>(1, r.n * bits / 512);
    const uint64_t fb = r.nblocks * 64;
    KC_HIP_TRY(hipMalloc(&r.d_bloom, fb));
    KC_HIP_TRY(hipMemsetAsync(r.d_bloom, 0, fb, st));
    r.meta_bytes += fb;
    meta_used_ += fb;
  }
  hipLaunchKernelGGL(k_run_meta, dim3(grid_of(r.n + 1)), dim3(256), 0, st, keys, r.n, r.d_dir, dbits, r.d_bloom,
                     r.nblocks);
  KC_HIP_TRY(hipGetLastError());
  peak_meta_ = std::max(peak_meta_, meta_used_ + cache_used_);
  return 0;
}

int ColdSet::add_run(const uint64_t* d_sorted, uint64_t n, hipStream_t st) {
  if (n == 0) return 0;
  ColdRun r;
  r.n = n;
  KC_TRY(pin_get(n, &r.host, &r.host_cap));
  host_used_ += r.bytes();
  keys_ += n;
  const double t0 = now_s();
  KC_HIP_TRY(hipMemcpyAsync(r.host, d_sorted, n * 8, hipMemcpyDeviceToHost, st));
  const int rc = build_meta(r, d_sorted, st);
  runs_.push_back(r);                   // owned (and freed) by runs_ from here on
  KC_TRY(rc);
  KC_HIP_TRY(hipStreamSynchronize(st));
  t_meta_ += now_s() - t0;
  // size-tiered compaction: a binary counter of run sizes
  while (runs_.size() >= 2) {
    const ColdRun &a = runs_[runs_.size() - 2], &b = runs_.back();
    if (!a.host || !b.host) break;
    if (!(a.n * 2 <= b.n * 3 || runs_.size() > 12)) break;
    KC_TRY(merge_last_two(st));
  }
  while (cfg_.host_bytes && host_used_ > cfg_.host_bytes) {
    bool any = false;
    for (const auto& x : runs_) any |= x.host != nullptr;
    if (!any) break;
    KC_TRY(evict_oldest_host(st));
  }
  return recache(st);
}

int ColdSet::merge_last_two(hipStream_t st) {
  ColdRun& a = runs_[runs_.size() - 2];
  ColdRun& b = runs_.back();
  ColdRun c;
  c.n = a.n + b.n;
  KC_TRY(pin_get(c.n, &c.host, &c.host_cap));
  host_used_ += c.bytes();
  const double t0 = now_s();
  // the key space cut into T equal ranges, each merged by its own thread
  // (the runs are uniform, so the ranges carry equal work)
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cfg_.merge_threads, c.n / 65536 + 1));
  std::vector<uint64_t> ia(T + 1), ib(T + 1);
  ia[0] = ib[0] = 0;
  ia[T] = a.n;
  ib[T] = b.n;
  for (int t = 1; t < T; ++t) {
    const uint64_t s = (uint64_t)(((unsigned __int128)t << 64) / (unsigned)T);
    ia[t] = std::lower_bound(a.host, a.host + a.n, s) - a.host;
    ib[t] = std::lower_bound(b.host, b.host + b.n, s) - b.host;
  }
  const uint64_t *pa = a.host, *pb = b.host;
  uint64_t* pc = c.host;
  auto work = [&](int t) {
    std::merge(pa + ia[t], pa + ia[t + 1], pb + ib[t], pb + ib[t + 1], pc + ia[t] + ib[t]);
  };
  try {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  } catch (...) {
    pin_put(c.host, c.host_cap);
    host_used_ -= c.bytes();
    set_error("seen-set: cannot start merge threads");
    return -ENOMEM;
  }
  const double t1 = now_s();
  t_merge_ += t1 - t0;
  merges_ += 1;
  merged_keys_ += c.n;
  const uint64_t na = a.n, nb = b.n;
  free_run(runs_.back());
  runs_.pop_back();
  free_run(runs_.back());
  runs_.pop_back();
  keys_ += c.n;
  const int rc = build_meta(c, c.host, st);
  runs_.push_back(c);
  KC_TRY(rc);
  KC_HIP_TRY(hipStreamSynchronize(st));
  t_meta_ += now_s() - t1;
  (void)na;
  (void)nb;
  return 0;
}

int ColdSet::evict_oldest_host(hipStream_t st) {
  (void)st;
  const double t0 = now_s();
  for (auto& r : runs_) {
    if (!r.host) continue;
    if (cfg_.dir.empty()) {
      set_error("seen-set: host budget %llu B exhausted and no spill directory",
                (unsigned long long)cfg_.host_bytes);
      return -ENOMEM;
    }
    char name[80];
    snprintf(name, sizeof name, "/kcfp-%d-%llu-%llu.run", (int)getpid(), (unsigned long long)id_,
             (unsigned long long)++file_seq_);
    const std::string path = cfg_.dir + name;
    const int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (fd < 0) {
      set_error("seen-set: cannot create spill file %s", path.c_str());
      return -EIO;
    }
    const char* p = reinterpret_cast<const char*>(r.host);
    uint64_t left = r.bytes(), off = 0;
    while (left) {
      const ssize_t w = pwrite(fd, p + off, std::min<uint64_t>(left, 1ull << 30), (off_t)off);
      if (w <= 0) {
        close(fd);
        unlink(path.c_str());
        set_error("seen-set: short write to spill file %s", path.c_str());
        return -EIO;
      }
      left -= (uint64_t)w;
      off += (uint64_t)w;
    }
    if (close(fd) != 0) {
      unlink(path.c_str());
      set_error("seen-set: cannot close spill file %s", path.c_str());
      return -EIO;
    }
    // window boundary keys (HBM; a few per GiB of run)
    r.wkeys = cfg_.window_keys;
    r.nw = (r.n + r.wkeys - 1) / r.wkeys;
    std::vector<uint64_t> wk(r.nw + 1);
    wk[0] = 0;
    for (uint64_t w = 1; w < r.nw; ++w) wk[w] = r.host[w * r.wkeys];
    wk[r.nw] = ~0ull;
    KC_HIP_TRY(hipMalloc(&r.d_wkeys, (r.nw + 1) * 8));
    KC_HIP_TRY(hipMemcpy(r.d_wkeys, wk.data(), (r.nw + 1) * 8, hipMemcpyHostToDevice));
    pin_put(r.host, r.host_cap);
    r.host = nullptr;
    r.host_cap = 0;
    host_used_ -= r.bytes();
    r.path = path;
    disk_used_ += r.bytes();
    disk_written_ += r.bytes();
    t_evict_ += now_s() - t0;
    return 0;
  }
  return 0;
}

int ColdSet::staging(uint64_t keys) {
  if (keys <= stage_keys_) return 0;
  for (int s = 0; s < 2; ++s) {
    if (stage_[s]) (void)hipHostFree(stage_[s]);
    stage_[s] = nullptr;
  }
  stage_keys_ = 0;
  for (int s = 0; s < 2; ++s) {
    KC_HIP_TRY(hipHostMalloc(&stage_[s], keys * 8));
    if (!stage_ev_[s]) KC_HIP_TRY(hipEventCreateWithFlags(&stage_ev_[s], hipEventDisableTiming));
  }
  stage_keys_ = keys;
  return 0;
}

int ColdSet::read_window(const ColdRun& r, uint64_t w0, uint64_t w1, uint64_t* dst) {
  const int fd = open(r.path.c_str(), O_RDONLY);
  if (fd < 0) {
    set_error("seen-set: spill file %s missing", r.path.c_str());
    return -EIO;
  }
  char* p = reinterpret_cast<char*>(dst);
  uint64_t left = (w1 - w0) * 8, off = 0;
  while (left) {
    const ssize_t g = pread(fd, p + off, std::min<uint64_t>(left, 1ull << 30), (off_t)(w0 * 8 + off));
    if (g <= 0) {
      close(fd);
      set_error("seen-set: short read from spill file %s", r.path.c_str());
      return -EIO;
    }
    left -= (uint64_t)g;
    off += (uint64_t)g;
  }
  close(fd);
  disk_read_ += (w1 - w0) * 8;
  return 0;
}

int ColdSet::probe(const uint64_t* d_q, uint64_t m, uint8_t* d_found, unsigned long long* d_hits, hipStream_t st) {
  if (m == 0) return 0;
  for (size_t k = runs_.size(); k-- > 0;) {            // newest first
    const ColdRun& r = runs_[k];
    if (!r.d_keys && r.host && cfg_.merge_div > 0 && m >= r.n / (uint64_t)cfg_.merge_div) {
      // a dense query set against a host run: one sequential pass over it
      hipLaunchKernelGGL(k_cold_merge_probe, dim3((unsigned)((r.n + MSEG - 1) / MSEG)), dim3(256), 0, st, d_q, m,
                         d_found, r.host, r.n, d_hits);
      ++merge_probes_;
      continue;
    }
    if (r.d_keys || r.host) {         // HBM copy, else the pinned host run read over the link
      hipLaunchKernelGGL(k_cold_probe, dim3(grid_of(m)), dim3(256), 0, st, d_q, m, d_found,
                         r.d_keys ? r.d_keys : r.host, 0ull, r.n, r.d_dir, r.dbits, r.d_bloom, r.nblocks, d_hits,
                         d_stat_);
      continue;
    }
    // disk run: stream the windows holding at least one query's key range
    // through two pinned buffers (read one while the GPU probes the other);
    // each window's launch covers just its queries
    KC_TRY(staging(r.wkeys));
    if (qa_cap_ < r.nw + 1) {
      if (d_qa_) (void)hipFree(d_qa_);
      if (h_qa_) (void)hipHostFree(h_qa_);
      d_qa_ = nullptr;
      h_qa_ = nullptr;
      qa_cap_ = 0;
      KC_HIP_TRY(hipMalloc(&d_qa_, (r.nw + 1) * 8));
      KC_HIP_TRY(hipHostMalloc(&h_qa_, (r.nw + 1) * 8));
      qa_cap_ = r.nw + 1;
    }
    hipLaunchKernelGGL(k_window_ranges, dim3(grid_of(r.nw + 1)), dim3(256), 0, st, d_q, m, r.d_wkeys, r.nw, d_qa_);
    KC_HIP_TRY(hipMemcpyAsync(h_qa_, d_qa_, (r.nw + 1) * 8, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    int s = 0;
    for (uint64_t w = 0; w < r.nw; ++w) {
      const uint64_t qa = h_qa_[w], qb = h_qa_[w + 1];
      if (qb <= qa) {
        ++windows_skipped_;
        continue;
      }
      const uint64_t w0 = w * r.wkeys, w1 = std::min(r.n, w0 + r.wkeys);
      KC_HIP_TRY(hipEventSynchronize(stage_ev_[s]));  // the kernel that last read this buffer is done
      KC_TRY(read_window(r, w0, w1, stage_[s]));
      hipLaunchKernelGGL(k_cold_probe, dim3(grid_of(qb - qa)), dim3(256), 0, st, d_q + qa, qb - qa, d_found + qa,
                         stage_[s], w0, w1, r.d_dir, r.dbits, r.d_bloom, r.nblocks, d_hits, d_stat_);
      KC_HIP_TRY(hipEventRecord(stage_ev_[s], st));
      s ^= 1;
    }
  }
  KC_HIP_TRY(hipGetLastError());
  return 0;
}

void ColdSet::stats(ColdStats* s) const {
  *s = ColdStats{};
  s->runs = runs_.size();
  for (const auto& r : runs_) s->runs_disk += r.host ? 0 : 1;
  s->keys = keys_;
  s->host_bytes = host_used_;
  s->disk_bytes = disk_used_;
  s->meta_bytes = meta_used_;
  s->peak_meta_bytes = peak_meta_;
  s->merges = merges_;
  s->merged_keys = merged_keys_;
  s->disk_written = disk_written_;
  s->disk_read = disk_read_;
  s->windows_skipped = windows_skipped_;
  s->merge_probes = merge_probes_;
  for (const auto& r : runs_)
    if (r.d_keys) {
      s->cached_runs++;
      s->cached_keys += r.n;
    }
  s->cache_bytes = cache_used_;
  s->cache_uploaded = cache_uploaded_;
  s->pin_seconds = t_pin_;
  s->merge_seconds = t_merge_;
  s->meta_seconds = t_meta_;
  s->evict_seconds = t_evict_;
  unsigned long long st[2] = {0, 0};
  if (d_stat_ && hipMemcpy(st, d_stat_, 16, hipMemcpyDeviceToHost) == hipSuccess) {
    s->filter_tests = st[0];
    s->filter_passed = st[1];
  }
}

int ColdSet::all_keys(std::vector<uint64_t>& out) {
  out.clear();
  out.reserve(keys_);
  std::vector<uint64_t> buf;
  for (const auto& r : runs_) {
    const size_t at = out.size();
    if (r.host) {
      out.insert(out.end(), r.host, r.host + r.n);
    } else {
      buf.resize(r.n);
      KC_TRY(read_window(r, 0, r.n, buf.data()));
      out.insert(out.end(), buf.begin(), buf.end());
    }
    std::inplace_merge(out.begin(), out.begin() + at, out.end());
  }
  return 0;
}

}  // namespace kc

// Host self-check of the cold-run search (no GPU): n sorted random keys with
// the directory the kernels build, every key found, absent keys (including
// ones between two lines' ranges) not found, each through whole-run and
// windowed views.  Returns the number of wrong answers (0 expected).
extern "C" int64_t kc_cold_find_selftest(uint64_t n, uint64_t seed) {
  using namespace kc;
  std::vector<uint64_t> keys(n);
  uint64_t x = seed | 1;
  for (auto& k : keys) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    k = cold_key(x);
  }
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  n = keys.size();
  int dbits = 1;
  while ((1ull << (dbits + 1)) * 16 <= n && dbits < 40) ++dbits;
  std::vector<uint64_t> dir((1ull << dbits) + 1);
  for (uint64_t b = 0, i = 0; b <= (1ull << dbits); ++b) {
    while (i < n && dir_bucket(keys[i], dbits) < b) ++i;
    dir[b] = i;
  }
  int64_t bad = 0;
  const uint64_t W = 64 + (n / 7 & ~7ull);      // windows of W keys (a multiple of 8)
  auto find_any = [&](uint64_t k) {
    if (run_find(k, keys.data(), 0, n, dir.data(), dbits)) return 1;
    return 0;
  };
  auto find_win = [&](uint64_t k) {
    int hits = 0;
    for (uint64_t w0 = 0; w0 < n; w0 += W)
      hits += run_find(k, keys.data() + w0, w0, std::min(n, w0 + W), dir.data(), dbits) ? 1 : 0;
    return hits;
  };
  for (uint64_t i = 0; i < n; ++i) {
    bad += find_any(keys[i]) != 1;
    if (i % 7 == 0) bad += find_win(keys[i]) != 1;
    // absent neighbours: just above this key (inside gaps, often between lines)
    if (i + 1 < n && keys[i + 1] > keys[i] + 1) {
      const uint64_t a = keys[i] + 1 + (keys[i + 1] - keys[i] - 1) / 2;
      bad += find_any(a) != 0;
      if (i % 7 == 0) bad += find_win(a) != 0;
    }
  }
  bad += find_any(0) != (n && keys[0] == 0);
  bad += find_any(~0ull) != (n && keys[n - 1] == ~0ull);
  return bad;
}
