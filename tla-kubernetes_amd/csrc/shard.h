// shard.h — type-erased interface of one fingerprint-owner shard (shard.hip)
// and the kc_shard handle, shared with the native level loop
// (shard_driver.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <vector>

#include "../../include/kubecheck.h"

namespace kc {

class ShardBase {
 public:
  virtual ~ShardBase() = default;
  virtual int setup() = 0;
  virtual int set_stream(hipStream_t st) = 0;
  virtual int init(uint64_t* n_local) = 0;
  // the error key of the first Init state (in this rank's order) that
  // violates an invariant (low byte 0x12), ~0 if none: level 1's error,
  // ahead of anything expansion finds (TLC checks Init before expanding)
  virtual uint64_t init_error() const = 0;
  virtual int expand(uint64_t* counts, uint64_t* err_key) = 0;
  // expand() split around a device-side all-gather row (the native loop over
  // RCCL): expand_dev enqueues the level's claims and writes d_row[0..world)
  // = owner totals, d_row[world] = status_new, d_row[world + 1] = status_err
  // (on level 1 an Init-state invariant key instead, as the loop would),
  // d_row[world + 2] = 1 if the claims overflowed (else 0), with no host sync; expand_done, after the caller's stream sync, reports what
  // expand() reports.
  virtual int expand_dev(uint64_t status_new, uint64_t status_err, bool level1, uint64_t* d_row) = 0;
  virtual int expand_done(uint64_t* counts, uint64_t* err_key) = 0;
  virtual uint64_t record_bytes() const = 0;
  virtual int pack(void* send) = 0;
  virtual int insert(const void* recv, uint64_t n, uint64_t* n_new, uint64_t* err_key) = 0;
  virtual int advance() = 0;
  virtual int parent_key(int level, uint64_t idx, uint64_t* key) = 0;
  virtual int frontier_tuple(uint64_t idx, uint64_t* out) = 0;
  virtual int result(kc_result* r) = 0;
  virtual void claim_times(double* ms, uint64_t* launches, uint64_t* parents) = 0;
  virtual hipStream_t stream() const = 0;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual int device() const = 0;
  virtual int tuple_words() const = 0;
  virtual const kc_model_config& config() const = 0;
  // pack() without its own host sync (the caller orders the records' use)
  virtual void set_async_pack(bool on) = 0;
  // ---- the deferred frontier (round 5; the native loop's counted levels):
  // with it on, insert emits only links and parent keys, and the next
  // level's expand rebuilds the states (from this rank's previous frontier
  // or from the records this level received — the caller keeps the receive
  // buffer passed to insert intact until the next expand).  An invariant
  // violation among rebuilt states is an error of the level before: the
  // device row carries it (expand_dev), and defer_error() reports it after
  // expand_done.  materialize() builds a deferred frontier now (before a
  // narrow batch or a max_levels stop; synchronous) and returns its
  // invariant key the same way.  drop_last_insert() takes the last insert's
  // new states back out of the distinct count (a world-1 run that learns of
  // such an error only after it inserted the next level).
  virtual void set_deferred(bool on) = 0;
  virtual uint64_t defer_error() const = 0;
  virtual int materialize(uint64_t* defer_err) = 0;
  virtual void drop_last_insert() = 0;
  // (the solo path) the last deferred expand's act_gen counts go too
  virtual int drop_last_expand() = 0;
  virtual int replay(int init_idx, const std::vector<int>& ords, int kind, int pos,
                     std::vector<std::vector<uint64_t>>& tuples, int* err_action, int* err_self,
                     int* err_inv) = 0;

  // ---- TLC order (cfg.tlc_order at world > 1; counted levels with the
  // deferred frontier): every state carries G, its position in its level in
  // sequential-BFS order, and claims, records, parent keys and error keys
  // carry the parent's G instead of (rank, local index), so the first
  // discoverer of every state, the error reported and its trace are those of
  // TLC -workers 1.  After every rank's insert of a level of global width W:
  // tlc_masks() sets, per parent G, the positions of its successors this
  // rank won (*mask: W words on the device); the caller sums the masks over
  // the ranks in place; tlc_order() then gives each new state its G (the
  // winners before it in (parent G, position) order) and sorts this rank's
  // new frontier by G.  tlc_locate() finds the local index of G at a level
  // (the trace walk).
  virtual bool tlc() const = 0;
  virtual int tlc_masks(uint64_t W, uint32_t** mask) = 0;
  virtual int tlc_order(uint64_t W) = 0;
  virtual int tlc_locate(int level, uint64_t G, uint64_t* idx, bool* found) = 0;

  // ---- device-driven narrow levels (shard_narrow.h), driven by the native
  // loop: sn_setup once (the control block, scratch and the fixed exchange
  // slots: world x (slot_cap + 1) records each way), then per batch
  // sn_begin, per level sn_pre (expand, send, pack), the caller's fixed
  // exchange of the slots, sn_post (receive, claim, scan, emit), and
  // sn_end (one host sync; the levels the batch ran).
  struct SNOut {
    int levels = 0;                 // levels run (the same on every rank)
    int reason = 0;                 // SNReason (0: every level of the batch ran)
    std::vector<uint64_t> widths;   // global width of each level run
    uint64_t status_new = 0;        // this rank's width of the next level
    uint64_t status_err = ~0ull;    // the previous level's errors (the counted loop's status_err)
    uint64_t sent = 0;              // records this rank sent to other ranks in the levels run
    bool filled = false;            // sn_end read the batch's outcome (set even when it then fails)
  };
  virtual int sn_setup(uint32_t slot_cap) = 0;
  virtual uint64_t sn_slot_bytes() const = 0;
  virtual void* sn_send() = 0;
  virtual void* sn_recv() = 0;
  virtual int sn_begin(uint64_t status_new, uint64_t status_err, int batch) = 0;
  virtual int sn_pre(uint32_t lev, bool fail) = 0;
  virtual int sn_post(uint32_t lev) = 0;
  virtual int sn_end(SNOut* out) = 0;
};

// One transfer of a rank's all-to-all (shard_driver.hip exchange_plan).
struct Xfer {
  int peer;
  int send;          // 1 = send to peer, 0 = receive from peer
  uint64_t off, n;   // records: offset into the send / receive buffer, count
};
std::vector<Xfer> exchange_plan(const std::vector<std::vector<uint64_t>>& Mx, int me, uint64_t piece);

}  // namespace kc

struct kc_shard {
  std::unique_ptr<kc::ShardBase> impl;
};
