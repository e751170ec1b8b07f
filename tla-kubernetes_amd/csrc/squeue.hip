// squeue.hip — the StateQueue (kc_squeue_*; TLC's tlc2.tool.queue.StateQueue,
// MC.out:5 "DiskStateQueue"): segmented FIFO of packed states over HBM,
// pinned host RAM and spill files (squeue.h).  The engine keeps its
// frontiers in one of these when a frontier HBM budget is set
// (kc_model_config.frontier_hbm_bytes, engine.hip run_queued); the C-ABI
// serves callers that drive their own BFS (device-pointer enqueue/dequeue,
// in-place reserve/commit and front/pop).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <mutex>

#include "../../include/kubecheck.h"
#include "kc_common.h"
#include "squeue.h"

namespace kc {

namespace {
std::atomic<uint64_t> g_queue_ids{0};
}

SegQueue::~SegQueue() {
  (void)hipSetDevice(cfg_.device);
  (void)hipDeviceSynchronize();
  for (auto& s : segs_) (void)free_seg(s);
  segs_.clear();
  for (auto* p : pool_) (void)hipFree(p);
  pool_.clear();
  if (stage_) (void)hipHostFree(stage_);
}

int SegQueue::init(const Config& c) {
  if (c.words <= 0 || c.seg_states == 0) {
    set_error("StateQueue: bad configuration (words %d, segment %llu states)", c.words,
              (unsigned long long)c.seg_states);
    return -EINVAL;
  }
  cfg_ = c;
  id_ = ++g_queue_ids;
  return 0;
}

int SegQueue::staging(uint64_t b) {
  if (b <= stage_cap_) return 0;
  if (stage_) (void)hipHostFree(stage_);
  stage_ = nullptr;
  stage_cap_ = 0;
  KC_HIP_TRY(hipHostMalloc(&stage_, b));
  stage_cap_ = b;
  return 0;
}

void SegQueue::dev_release(uint64_t* p, uint64_t cap) {
  if (!p) return;
  if (cap == cfg_.seg_states && (cfg_.hbm_bytes == 0 || hbm_used_ <= cfg_.hbm_bytes)) {
    pool_.push_back(p);            // stream-ordered reuse: still counted in hbm_used_
    return;
  }
  (void)hipFree(p);
  hbm_used_ -= bytes(cap);
}

// One HBM buffer of `cap` states.  Over budget: free pooled buffers, then
// spill segments (never the back, never index <= keep_hi) until it fits or
// nothing is left to spill (the segments being read and written always stay).
int SegQueue::dev_alloc(uint64_t cap, uint64_t** p, hipStream_t st, int64_t keep_hi) {
  if (cap == cfg_.seg_states && !pool_.empty()) {
    *p = pool_.back();
    pool_.pop_back();
    return 0;
  }
  while (cfg_.hbm_bytes && hbm_used_ + bytes(cap) > cfg_.hbm_bytes) {
    if (!pool_.empty()) {
      (void)hipFree(pool_.back());
      pool_.pop_back();
      hbm_used_ -= bytes(cfg_.seg_states);
      continue;
    }
    bool done = false;
    KC_TRY(spill_one(st, keep_hi, &done));
    if (!done) break;
  }
  KC_HIP_TRY(hipMalloc(p, bytes(cap)));
  hbm_used_ += bytes(cap);
  peak_hbm_ = std::max(peak_hbm_, hbm_used_);
  return 0;
}

int SegQueue::spill_one(hipStream_t st, int64_t keep_hi, bool* done) {
  *done = false;
  if (segs_.size() < 2) return 0;
  for (size_t i = segs_.size() - 1; i-- > 0;) {      // nearest the tail first, never the back
    if ((int64_t)i <= keep_hi) break;
    if (segs_[i].tier != HBM) continue;
    KC_TRY(spill(segs_[i], st));
    *done = true;
    return 0;
  }
  return 0;
}

// Move a closed HBM segment's live states to host RAM (or, past the host
// budget, to a spill file) and return its HBM buffer.
int SegQueue::spill(Seg& s, hipStream_t st) {
  const uint64_t live = s.tail - s.head, b = bytes(live);
  const uint64_t* src = s.dev + s.head * cfg_.words;
  if (cfg_.host_bytes == 0 || host_used_ + b <= cfg_.host_bytes) {
    uint64_t* h = nullptr;
    KC_HIP_TRY(hipHostMalloc(&h, b ? b : 8));
    if (b) KC_HIP_TRY(hipMemcpyAsync(h, src, b, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    s.host = h;
    s.tier = HOST;
    host_used_ += b;
    spilled_host_ += b;
  } else if (!cfg_.dir.empty()) {
    KC_TRY(staging(b ? b : 8));
    if (b) KC_HIP_TRY(hipMemcpyAsync(stage_, src, b, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    char name[64];
    snprintf(name, sizeof name, "/kcsq-%d-%llu-%llu.seg", (int)getpid(), (unsigned long long)id_,
             (unsigned long long)++file_seq_);
    s.path = cfg_.dir + name;
    FILE* f = fopen(s.path.c_str(), "wb");
    if (!f) {
      set_error("StateQueue: cannot create spill file %s", s.path.c_str());
      return -EIO;
    }
    const size_t w = b ? fwrite(stage_, 1, b, f) : 0;
    const int cl = fclose(f);
    if (w != b || cl != 0) {
      set_error("StateQueue: short write to spill file %s", s.path.c_str());
      unlink(s.path.c_str());
      return -EIO;
    }
    s.tier = DISK;
    disk_used_ += b;
    spilled_disk_ += b;
  } else {
    set_error("StateQueue: HBM budget %llu B and host budget %llu B exhausted and no spill directory",
              (unsigned long long)cfg_.hbm_bytes, (unsigned long long)cfg_.host_bytes);
    return -ENOMEM;
  }
  dev_release(s.dev, s.cap);
  s.dev = nullptr;
  s.head = 0;
  s.tail = live;
  return 0;
}

// Bring segment idx back to HBM (segments 0..idx are being read: not victims).
int SegQueue::load(size_t idx, hipStream_t st) {
  Seg& s = segs_[idx];
  if (s.tier == HBM) return 0;
  uint64_t* p = nullptr;
  KC_TRY(dev_alloc(s.cap, &p, st, std::max<int64_t>(front_pin_, (int64_t)idx)));
  Seg& t = segs_[idx];                               // (deque references survive; re-read anyway)
  const uint64_t b = bytes(t.tail);
  if (t.tier == HOST) {
    if (b) KC_HIP_TRY(hipMemcpyAsync(p, t.host, b, hipMemcpyHostToDevice, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    (void)hipHostFree(t.host);
    t.host = nullptr;
    host_used_ -= b;
  } else {
    KC_TRY(staging(b ? b : 8));
    FILE* f = fopen(t.path.c_str(), "rb");
    if (!f) {
      set_error("StateQueue: spill file %s missing", t.path.c_str());
      return -EIO;
    }
    const size_t r = b ? fread(stage_, 1, b, f) : 0;
    fclose(f);
    if (r != b) {
      set_error("StateQueue: short read from spill file %s", t.path.c_str());
      return -EIO;
    }
    if (b) KC_HIP_TRY(hipMemcpyAsync(p, stage_, b, hipMemcpyHostToDevice, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    unlink(t.path.c_str());
    t.path.clear();
    disk_used_ -= b;
  }
  reloaded_ += b;
  t.dev = p;
  t.tier = HBM;
  return 0;
}

int SegQueue::free_seg(Seg& s) {
  if (s.tier == HBM) {
    dev_release(s.dev, s.cap);
  } else if (s.tier == HOST) {
    if (s.host) (void)hipHostFree(s.host);
    host_used_ -= bytes(s.tail);
  } else {
    if (!s.path.empty()) unlink(s.path.c_str());
    disk_used_ -= bytes(s.tail);
  }
  s = Seg{};
  return 0;
}

int SegQueue::new_tail(uint64_t n, hipStream_t st) {
  if (!segs_.empty() && segs_.back().tail == segs_.back().head && segs_.size() > 1 &&
      (int64_t)segs_.size() - 1 > front_pin_) {
    free_seg(segs_.back());                          // an empty back nobody reads
    segs_.pop_back();
  }
  // the new back goes in first, so the old (now closed) back may be spilled
  // to make room for it
  segs_.push_back(Seg{});
  segs_.back().cap = std::max(cfg_.seg_states, n);
  uint64_t* p = nullptr;
  const int rc = dev_alloc(segs_.back().cap, &p, st, front_pin_);
  if (rc < 0) {
    segs_.pop_back();
    return rc;
  }
  segs_.back().dev = p;
  return 0;
}

int SegQueue::reserve(uint64_t n, uint64_t** dev, hipStream_t st) {
  KC_HIP_TRY(hipSetDevice(cfg_.device));
  if (segs_.empty() || segs_.back().tier != HBM || segs_.back().cap - segs_.back().tail < n) {
    // an empty back segment without readers is simply reused from its start
    if (!segs_.empty() && segs_.back().tier == HBM && segs_.back().tail == segs_.back().head &&
        segs_.back().cap >= n && (int64_t)segs_.size() - 1 > front_pin_) {
      segs_.back().head = segs_.back().tail = 0;
    } else {
      KC_TRY(new_tail(n, st));
    }
  }
  Seg& b = segs_.back();
  *dev = b.dev + b.tail * cfg_.words;
  reserved_ = n;
  return 0;
}

int SegQueue::commit(uint64_t n, hipStream_t st) {
  (void)st;
  if (n > reserved_ || segs_.empty()) {
    set_error("StateQueue: commit of %llu states exceeds the reservation (%llu)", (unsigned long long)n,
              (unsigned long long)reserved_);
    return -EINVAL;
  }
  segs_.back().tail += n;
  size_ += n;
  reserved_ = 0;
  return 0;
}

int SegQueue::enqueue_dev(const uint64_t* src, uint64_t n, hipStream_t st) {
  uint64_t done = 0;
  while (done < n) {
    uint64_t room = 0;
    if (!segs_.empty() && segs_.back().tier == HBM) room = segs_.back().cap - segs_.back().tail;
    const uint64_t m = std::min(n - done, room ? room : cfg_.seg_states);
    uint64_t* d = nullptr;
    KC_TRY(reserve(m, &d, st));
    KC_HIP_TRY(hipMemcpyAsync(d, src + done * cfg_.words, bytes(m), hipMemcpyDeviceToDevice, st));
    KC_TRY(commit(m, st));
    done += m;
  }
  return 0;
}

int SegQueue::enqueue_host(const uint64_t* src, uint64_t n, hipStream_t st) {
  uint64_t done = 0;
  while (done < n) {
    uint64_t room = 0;
    if (!segs_.empty() && segs_.back().tier == HBM) room = segs_.back().cap - segs_.back().tail;
    const uint64_t m = std::min(n - done, room ? room : cfg_.seg_states);
    uint64_t* d = nullptr;
    KC_TRY(reserve(m, &d, st));
    KC_HIP_TRY(hipMemcpyAsync(d, src + done * cfg_.words, bytes(m), hipMemcpyHostToDevice, st));
    KC_HIP_TRY(hipStreamSynchronize(st));             // the caller's buffer may go away
    KC_TRY(commit(m, st));
    done += m;
  }
  return 0;
}

int SegQueue::front(uint64_t offset, uint64_t max_n, const uint64_t** dev, uint64_t* got, hipStream_t st) {
  KC_HIP_TRY(hipSetDevice(cfg_.device));
  *got = 0;
  *dev = nullptr;
  if (offset >= size_ || max_n == 0) return 0;
  size_t idx = 0;
  uint64_t off = offset;
  while (off >= segs_[idx].tail - segs_[idx].head) {
    off -= segs_[idx].tail - segs_[idx].head;
    ++idx;
  }
  if (segs_[idx].tier != HBM) KC_TRY(load(idx, st));
  front_pin_ = std::max<int64_t>(front_pin_, (int64_t)idx);
  const Seg& s = segs_[idx];
  *dev = s.dev + (s.head + off) * cfg_.words;
  *got = std::min(max_n, s.tail - s.head - off);
  return 0;
}

int SegQueue::pop(uint64_t n, hipStream_t st) {
  (void)st;
  if (n > size_) {
    set_error("StateQueue: pop of %llu states from a queue of %llu", (unsigned long long)n,
              (unsigned long long)size_);
    return -EINVAL;
  }
  while (n) {
    Seg& s = segs_.front();
    const uint64_t k = std::min(n, s.tail - s.head);
    s.head += k;
    size_ -= k;
    n -= k;
    if (s.head == s.tail && segs_.size() > 1) {
      free_seg(s);
      segs_.pop_front();
      if (front_pin_ >= 0) --front_pin_;
    }
  }
  if (size_ == 0) {
    front_pin_ = -1;
    if (!segs_.empty() && reserved_ == 0 && segs_.back().tier == HBM) segs_.back().head = segs_.back().tail = 0;
  }
  return 0;
}

int SegQueue::dequeue_dev(uint64_t* dst, uint64_t max_n, uint64_t* got, hipStream_t st) {
  const uint64_t want = std::min(max_n, size_);
  uint64_t done = 0;
  while (done < want) {
    const uint64_t* p = nullptr;
    uint64_t m = 0;
    KC_TRY(front(0, want - done, &p, &m, st));
    KC_HIP_TRY(hipMemcpyAsync(dst + done * cfg_.words, p, bytes(m), hipMemcpyDeviceToDevice, st));
    KC_TRY(pop(m, st));
    done += m;
  }
  *got = done;
  return 0;
}

int SegQueue::dequeue_host(uint64_t* dst, uint64_t max_n, uint64_t* got, hipStream_t st) {
  const uint64_t want = std::min(max_n, size_);
  KC_TRY(peek_host(0, want, dst, st));
  KC_TRY(pop(want, st));
  *got = want;
  return 0;
}

int SegQueue::peek_host(uint64_t offset, uint64_t n, uint64_t* dst, hipStream_t st) {
  KC_HIP_TRY(hipSetDevice(cfg_.device));
  if (offset + n > size_) {
    set_error("StateQueue: peek [%llu, %llu) beyond size %llu", (unsigned long long)offset,
              (unsigned long long)(offset + n), (unsigned long long)size_);
    return -EINVAL;
  }
  uint64_t done = 0, skip = offset;
  for (size_t i = 0; i < segs_.size() && done < n; ++i) {
    const Seg& s = segs_[i];
    const uint64_t live = s.tail - s.head;
    if (skip >= live) {
      skip -= live;
      continue;
    }
    const uint64_t m = std::min(n - done, live - skip), at = s.head + skip;
    uint64_t* out = dst + done * cfg_.words;
    if (s.tier == HBM) {
      KC_HIP_TRY(hipMemcpyAsync(out, s.dev + at * cfg_.words, bytes(m), hipMemcpyDeviceToHost, st));
      KC_HIP_TRY(hipStreamSynchronize(st));
    } else if (s.tier == HOST) {
      memcpy(out, s.host + at * cfg_.words, bytes(m));
    } else {
      FILE* f = fopen(s.path.c_str(), "rb");
      if (!f) {
        set_error("StateQueue: spill file %s missing", s.path.c_str());
        return -EIO;
      }
      const bool ok = fseeko(f, (off_t)bytes(at), SEEK_SET) == 0 && fread(out, 1, bytes(m), f) == bytes(m);
      fclose(f);
      if (!ok) {
        set_error("StateQueue: short read from spill file %s", s.path.c_str());
        return -EIO;
      }
    }
    done += m;
    skip = 0;
  }
  return 0;
}

int SegQueue::clear(hipStream_t st) {
  KC_HIP_TRY(hipSetDevice(cfg_.device));
  KC_HIP_TRY(hipStreamSynchronize(st));
  for (auto& s : segs_) free_seg(s);
  segs_.clear();
  size_ = 0;
  reserved_ = 0;
  front_pin_ = -1;
  return 0;
}

void SegQueue::stats(kc_squeue_stats* o) const {
  memset(o, 0, sizeof *o);
  o->size = size_;
  o->segments = segs_.size();
  for (const auto& s : segs_) {
    if (s.tier == HBM) ++o->seg_hbm;
    else if (s.tier == HOST) ++o->seg_host;
    else ++o->seg_disk;
  }
  o->hbm_bytes = hbm_used_;
  o->host_bytes = host_used_;
  o->disk_bytes = disk_used_;
  o->spilled_host_bytes = spilled_host_;
  o->spilled_disk_bytes = spilled_disk_;
  o->reloaded_bytes = reloaded_;
  o->peak_hbm_bytes = peak_hbm_;
}

}  // namespace kc

using namespace kc;

struct kc_squeue {
  SegQueue q;
  hipStream_t st = nullptr;       // the queue's own stream (blocking: ordered with the null stream)
  int device = 0;
  uint64_t max_states = 0;        // kc_squeue_create's capacity: a hard bound (0 = none)
  std::mutex mu;
  hipStream_t pick(void* s) const { return s ? (hipStream_t)s : st; }
  // the round-1 constructor's contract: enqueue past capacity_states fails
  int room(size_t n, const char* fn) const {
    if (max_states && q.size() + n > max_states) {
      set_error("%s: StateQueue full (%llu + %zu states > capacity %llu)", fn, (unsigned long long)q.size(), n,
                (unsigned long long)max_states);
      return -ENOMEM;
    }
    return 0;
  }
};

extern "C" {

int kc_squeue_create2(const kc_squeue_config* c, kc_squeue** out) {
  if (!c || !out || c->state_words <= 0) {
    set_error("kc_squeue_create2: bad argument");
    return -EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("kc_squeue_create: no HIP device (the StateQueue has no CPU fallback)");
    return -ENODEV;
  }
  if (c->device < 0 || c->device >= ndev) {
    set_error("kc_squeue_create: bad device %d", c->device);
    return -EINVAL;
  }
  KC_HIP_TRY(hipSetDevice(c->device));
  SegQueue::Config qc;
  qc.words = c->state_words;
  qc.device = c->device;
  qc.seg_states = c->segment_states ? c->segment_states : (1u << 20);
  qc.hbm_bytes = c->hbm_bytes;
  qc.host_bytes = c->host_bytes;
  qc.dir = c->spill_dir ? c->spill_dir : "";
  auto* q = new kc_squeue();
  q->device = c->device;
  int rc = q->q.init(qc);
  if (rc == 0 && hipStreamCreate(&q->st) != hipSuccess) {
    set_error("kc_squeue_create: stream creation failed");
    rc = -EIO;
  }
  if (rc) {
    delete q;
    return rc;
  }
  *out = q;
  return 0;
}

int kc_squeue_create(int state_words, uint64_t capacity_states, int device, kc_squeue** out) {
  kc_squeue_config c;
  memset(&c, 0, sizeof c);
  c.state_words = state_words;
  c.device = device;
  c.segment_states = capacity_states;
  if (capacity_states == 0) {
    set_error("kc_squeue_create: bad argument");
    return -EINVAL;
  }
  KC_TRY(kc_squeue_create2(&c, out));
  (*out)->max_states = capacity_states;     // a bounded queue, as this constructor always was
  return 0;
}

void kc_squeue_destroy(kc_squeue* q) {
  if (!q) return;
  {
    std::lock_guard<std::mutex> g(q->mu);
    (void)hipSetDevice(q->device);
    (void)q->q.clear(q->st);
  }
  if (q->st) (void)hipStreamDestroy(q->st);
  delete q;
}

int kc_squeue_enqueue(kc_squeue* q, const uint64_t* states, size_t n) {
  if (!q || (n && !states)) { set_error("kc_squeue_enqueue: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  KC_TRY(q->room(n, "kc_squeue_enqueue"));
  KC_HIP_TRY(hipSetDevice(q->device));
  return q->q.enqueue_host(states, n, q->st);
}

int kc_squeue_dequeue(kc_squeue* q, uint64_t* out, size_t max_n, size_t* n_out) {
  if (!q || !n_out || (max_n && !out)) { set_error("kc_squeue_dequeue: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  KC_HIP_TRY(hipSetDevice(q->device));
  uint64_t got = 0;
  KC_TRY(q->q.dequeue_host(out, max_n, &got, q->st));
  *n_out = got;
  return 0;
}

int kc_squeue_enqueue_dev(kc_squeue* q, const uint64_t* dev_states, size_t n, void* stream) {
  if (!q || (n && !dev_states)) { set_error("kc_squeue_enqueue_dev: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  KC_TRY(q->room(n, "kc_squeue_enqueue_dev"));
  KC_HIP_TRY(hipSetDevice(q->device));
  return q->q.enqueue_dev(dev_states, n, q->pick(stream));
}

int kc_squeue_dequeue_dev(kc_squeue* q, uint64_t* dev_out, size_t max_n, size_t* n_out, void* stream) {
  if (!q || !n_out || (max_n && !dev_out)) { set_error("kc_squeue_dequeue_dev: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  KC_HIP_TRY(hipSetDevice(q->device));
  uint64_t got = 0;
  KC_TRY(q->q.dequeue_dev(dev_out, max_n, &got, q->pick(stream)));
  *n_out = got;
  return 0;
}

int kc_squeue_reserve_dev(kc_squeue* q, size_t n, uint64_t** dev_ptr, void* stream) {
  if (!q || !dev_ptr || n == 0) { set_error("kc_squeue_reserve_dev: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  KC_TRY(q->room(n, "kc_squeue_reserve_dev"));
  return q->q.reserve(n, dev_ptr, q->pick(stream));
}

int kc_squeue_commit(kc_squeue* q, size_t n, void* stream) {
  if (!q) { set_error("kc_squeue_commit: NULL"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  return q->q.commit(n, q->pick(stream));
}

int kc_squeue_front_dev(kc_squeue* q, size_t offset, size_t max_n, const uint64_t** dev_ptr, size_t* n_out,
                        void* stream) {
  if (!q || !dev_ptr || !n_out) { set_error("kc_squeue_front_dev: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  uint64_t got = 0;
  KC_TRY(q->q.front(offset, max_n, dev_ptr, &got, q->pick(stream)));
  *n_out = got;
  return 0;
}

int kc_squeue_pop(kc_squeue* q, size_t n, void* stream) {
  if (!q) { set_error("kc_squeue_pop: NULL"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  return q->q.pop(n, q->pick(stream));
}

int kc_squeue_peek(kc_squeue* q, size_t offset, size_t n, uint64_t* host_out, void* stream) {
  if (!q || (n && !host_out)) { set_error("kc_squeue_peek: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  return q->q.peek_host(offset, n, host_out, q->pick(stream));
}

int kc_squeue_get_stats(kc_squeue* q, kc_squeue_stats* out) {
  if (!q || !out) { set_error("kc_squeue_get_stats: NULL"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  q->q.stats(out);
  return 0;
}

uint64_t kc_squeue_size(const kc_squeue* q) { return q ? q->q.size() : 0; }

}  // extern "C"
