// squeue.h — the StateQueue (TLC's tlc2.tool.queue.StateQueue seam; the
// recorded run used DiskStateQueue, MC.out:5): a FIFO of fixed-width packed
// states kept in segments that live in one of three tiers,
//
//   HBM   device buffers (the tail segment is always here: kernels write
//         new states into it in place, kc_squeue_reserve_dev/commit),
//   HOST  pinned host RAM (hipHostMalloc), beyond an HBM byte budget,
//   DISK  files in a spill directory, beyond a host byte budget
//         (DiskStateQueue's role).
//
// Spill order: when a new HBM segment would exceed the budget, the HBM
// segment nearest the TAIL that nothing is reading is written out first
// (it is the one dequeued last), so the head region stays resident.  A
// segment is brought back to HBM when a reader reaches it (front/peek).
// Every copy runs on the one stream the queue is driven on (the caller's,
// or the queue's own), so kernels that read a front run or write a
// reserved run are ordered with the spills and reloads without events;
// buffers are reused through a pool of standard-size segments.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <deque>
#include <string>
#include <vector>

#include "../../include/kubecheck.h"

namespace kc {

class SegQueue {
 public:
  enum Tier : int { HBM = 0, HOST = 1, DISK = 2 };
  struct Config {
    int words = 0;               // u64 words per state
    int device = 0;
    uint64_t seg_states = 1u << 20;
    uint64_t hbm_bytes = 0;      // 0 = unlimited
    uint64_t host_bytes = 0;     // 0 = unlimited
    std::string dir;             // "" = no disk tier
  };
  SegQueue() = default;
  SegQueue(const SegQueue&) = delete;
  SegQueue& operator=(const SegQueue&) = delete;
  ~SegQueue();

  int init(const Config& c);
  // Tail: a contiguous device run of n states to write (valid until the next
  // call), then commit(k <= n) appends the first k of them.
  int reserve(uint64_t n, uint64_t** dev, hipStream_t st);
  int commit(uint64_t n, hipStream_t st);
  int enqueue_dev(const uint64_t* src, uint64_t n, hipStream_t st);
  int enqueue_host(const uint64_t* src, uint64_t n, hipStream_t st);
  // Head: a contiguous device run of up to max_n states starting `offset`
  // states after the head (its segment is brought to HBM first); *got may be
  // less than max_n at a segment boundary.  pop(n) drops n head states.
  int front(uint64_t offset, uint64_t max_n, const uint64_t** dev, uint64_t* got, hipStream_t st);
  int pop(uint64_t n, hipStream_t st);
  int dequeue_dev(uint64_t* dst, uint64_t max_n, uint64_t* got, hipStream_t st);
  int dequeue_host(uint64_t* dst, uint64_t max_n, uint64_t* got, hipStream_t st);
  // copy states [offset, offset + n) after the head to host memory, from
  // whatever tier holds them (no reload, no pop)
  int peek_host(uint64_t offset, uint64_t n, uint64_t* dst, hipStream_t st);
  int clear(hipStream_t st);

  uint64_t size() const { return size_; }
  int words() const { return cfg_.words; }
  uint64_t seg_states() const { return cfg_.seg_states; }
  void stats(kc_squeue_stats* s) const;

 private:
  struct Seg {
    uint64_t cap = 0, head = 0, tail = 0;   // states
    int tier = HBM;
    uint64_t* dev = nullptr;
    uint64_t* host = nullptr;
    std::string path;
  };
  uint64_t bytes(uint64_t states) const { return states * (uint64_t)cfg_.words * 8; }
  int dev_alloc(uint64_t cap, uint64_t** p, hipStream_t st, int64_t keep_hi);
  void dev_release(uint64_t* p, uint64_t cap);
  int spill_one(hipStream_t st, int64_t keep_hi, bool* done);
  int spill(Seg& s, hipStream_t st);
  int load(size_t idx, hipStream_t st);
  int staging(uint64_t b);
  int new_tail(uint64_t n, hipStream_t st);
  int free_seg(Seg& s);

  Config cfg_;
  std::deque<Seg> segs_;
  std::vector<uint64_t*> pool_;            // free standard-size HBM buffers
  uint64_t size_ = 0;
  uint64_t reserved_ = 0;                  // states reserved in the tail
  int64_t front_pin_ = -1;                 // segments 0..front_pin_ have handed out front runs
  uint64_t hbm_used_ = 0, host_used_ = 0, disk_used_ = 0, peak_hbm_ = 0;
  uint64_t spilled_host_ = 0, spilled_disk_ = 0, reloaded_ = 0;
  uint64_t* stage_ = nullptr;              // pinned staging for the disk tier
  uint64_t stage_cap_ = 0;                 // bytes
  uint64_t file_seq_ = 0;
  uint64_t id_ = 0;
};

}  // namespace kc
