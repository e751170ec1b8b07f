// engine_kernels.h — the per-level BFS kernels of the single-GPU engine
// (gfx950): k_claim, k_settle_rec, k_emit.
//
// One lane = one parent state.  Each kernel re-derives a parent's successor
// plan from its packed words (cheap integer work) instead of materialising
// candidate states in HBM; the random HBM traffic is the ClaimSet probe of
// each tile representative and the re-read of each candidate.
//
// Order key of a successor: (parent index within the level) << 8 | t, where
// t is its position in TLC's enumeration order.  Error keys put the parent
// index in bits 16+, the successor position in bits 8-15 and the ErrKind in
// bits 0-7, so the minimum key is the error a sequential 1-worker TLC BFS
// would have hit first.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fpset_dev.h"
#include "kubeapi_spec.h"
#include "record.h"

namespace kc {

// Counters.  Totals that every workgroup adds to (per-action counts, probe
// counts, the next level's candidate count) are striped over CTR_STRIPES
// rows in separate cache lines, row = blockIdx.x % CTR_STRIPES: one hot
// address taking an atomic from every workgroup serialises at the memory
// side (it cost k_settle_rec 4/5 of its time).  The host sums the rows.
constexpr int CTR_STRIPES = 64;
constexpr int OUTDEG_BINS = 16;
struct CtrStripe {                  // 1 KiB
  unsigned long long act_gen[A_COUNT];
  unsigned long long act_dist[A_COUNT];
  unsigned long long probes;        // FPSet / ClaimSet probes
  unsigned long long settles;       // ClaimSet re-reads in k_settle_*
  unsigned long long next_cand;     // successors of the new states (cumulative)
  // TLC's outdegree (msg 2268, MC.out:1104): new states first reached from
  // a parent, histogram over the expanded parents (bin OUTDEG_BINS-1 = that
  // many or more)
  unsigned long long outdeg[OUTDEG_BINS];
  // KC_DIAG builds only: k_claim ClaimSet outcomes (CL_OLD, CL_LOST, CL_CUR,
  // CL_NEW) and CL_OLD outcomes by level distance (1, 2, 3, 4, 5-8, 9-16, 17+)
  unsigned long long claim_out[4];
  unsigned long long old_dist[8];
  unsigned long long cand_ovf;      // candidate records that went to the overflow list
  // KC_DIAG builds only: k_claim successor-loop trips, per wave the max over
  // its lanes (what the wave runs) and the sum (what its lanes need)
  // (and loop_sorted: the wave trips if each tile's parents were dealt to
  // its waves in order of successor count)
  unsigned long long loop_max, loop_sum, loop_sorted;
  unsigned long long pad[128 - 2 * A_COUNT - 19 - OUTDEG_BINS];
};
struct Counters {
  unsigned long long err_key;     // min error key of the level (~0 = none)
  unsigned long long chunk_base;  // next-frontier offset of the current chunk
  unsigned long long overflow;    // states with > MAXSUCC successors, full tables
  unsigned long long batch_used;  // >0: a batch-table probe run overflowed (retry)
  unsigned long long cand_total;  // sum of the next_cand stripes (k_advance)
  unsigned long long level_new;   // sharded insert: new states of the level (local + records)
  unsigned long long emit_done;   // sharded insert: emit workgroups done (the last one reads the totals)
  unsigned long long defer_flags; // deferred frontier (DeferArgs): DF_* bits of the level
  unsigned long long defer_inv_n; // ... ~(lowest index of a rebuilt state violating an invariant); 0 = none
                                  // (word 8: k_advance copies it to the host with the head)
  unsigned long long defer_err;   // sharded deferred frontier: min invariant key of the rebuilt states (~0 = none)
  unsigned long long head_pad[6];
  CtrStripe s[CTR_STRIPES];

  unsigned long long act_gen(int a) const { return sum(&CtrStripe::act_gen, a); }
  unsigned long long act_dist(int a) const { return sum(&CtrStripe::act_dist, a); }
  unsigned long long probes() const { return sum1(&CtrStripe::probes); }
  unsigned long long settles() const { return sum1(&CtrStripe::settles); }
  unsigned long long cand_ovf() const { return sum1(&CtrStripe::cand_ovf); }
  unsigned long long next_cand() const { return sum1(&CtrStripe::next_cand); }
  unsigned long long outdeg(int b) const {
    unsigned long long t = 0;
    for (int k = 0; k < CTR_STRIPES; ++k) t += s[k].outdeg[b];
    return t;
  }
  unsigned long long claim_out(int r) const {
    unsigned long long t = 0;
    for (int k = 0; k < CTR_STRIPES; ++k) t += s[k].claim_out[r];
    return t;
  }
  unsigned long long loop_max() const { return sum1(&CtrStripe::loop_max); }
  unsigned long long loop_sum() const { return sum1(&CtrStripe::loop_sum); }
  unsigned long long loop_sorted() const { return sum1(&CtrStripe::loop_sorted); }
  unsigned long long old_dist(int b) const {
    unsigned long long t = 0;
    for (int k = 0; k < CTR_STRIPES; ++k) t += s[k].old_dist[b];
    return t;
  }

 private:
  unsigned long long sum(unsigned long long (CtrStripe::*f)[A_COUNT], int a) const {
    unsigned long long t = 0;
    for (int k = 0; k < CTR_STRIPES; ++k) t += (s[k].*f)[a];
    return t;
  }
  unsigned long long sum1(unsigned long long CtrStripe::*f) const {
    unsigned long long t = 0;
    for (int k = 0; k < CTR_STRIPES; ++k) t += s[k].*f;
    return t;
  }
};
// bytes of the per-level head (every word before the stripes: err_key ...
// defer_err and the padding): what the host reads back after a level.  The
// engine's k_advance writes its pinned copy word by word (words 0-5, 7, 8);
// a head copy (hipMemcpy of kCtrHead bytes) takes all of them.
constexpr size_t kCtrHead = 16 * sizeof(unsigned long long);
static_assert(offsetof(Counters, defer_flags) == 7 * 8 && offsetof(Counters, defer_inv_n) == 8 * 8 &&
                  offsetof(Counters, defer_err) == 9 * 8 && offsetof(Counters, s) == kCtrHead,
              "k_advance's host copy indexes the head words; kCtrHead covers the whole head");
// defer_flags: a rebuilt frontier state violates an invariant; a level's
// links or trace entries did not fit the capacity the host estimated; (the
// sharded k_claim) a tile's records did not fit the staging buffer
constexpr unsigned long long DF_INVARIANT = 1, DF_CAPACITY = 2, DF_STAGE = 4;
__device__ __forceinline__ CtrStripe& stripe(Counters* C) {
  return C->s[blockIdx.x & (CTR_STRIPES - 1)];
}

template <class M>
__device__ __forceinline__ typename M::State load_state(const typename M::State* __restrict__ p,
                                                        uint64_t i) {
  typename M::State s;
  const ulonglong2* v = reinterpret_cast<const ulonglong2*>(p + i);
#pragma unroll
  for (int k = 0; k < M::W / 2; ++k) {
    const ulonglong2 q = v[k];
    s.w[2 * k] = q.x;
    s.w[2 * k + 1] = q.y;
  }
  return s;
}
template <class M>
__device__ __forceinline__ void store_state(typename M::State* __restrict__ p, uint64_t i,
                                            const typename M::State& s) {
  ulonglong2* v = reinterpret_cast<ulonglong2*>(p + i);
#pragma unroll
  for (int k = 0; k < M::W / 2; ++k) v[k] = make_ulonglong2(s.w[2 * k], s.w[2 * k + 1]);
}
// A record (record.h): the successor's key, then its bit-packed canonical
// state; 48 B for NP = 2.
template <class M>
__device__ __forceinline__ void load_record(const Record<M>* __restrict__ in, uint64_t i,
                                            typename M::State& x, uint64_t& key) {
  const ulonglong2* v = reinterpret_cast<const ulonglong2*>(in + i);
  uint64_t r[Record<M>::RW];
#pragma unroll
  for (int k = 0; k < Record<M>::RW / 2; ++k) {
    const ulonglong2 q = v[k];
    r[2 * k] = q.x;
    r[2 * k + 1] = q.y;
  }
  record_unpack<M>(r, x, key);
}
template <class M>
__device__ __forceinline__ void store_record(Record<M>* __restrict__ out, uint64_t i, const typename M::State& x,
                                             uint64_t key) {
  uint64_t w[Record<M>::RW];
  record_pack<M>(x, key, w);
  ulonglong2* v = reinterpret_cast<ulonglong2*>(out + i);
#pragma unroll
  for (int k = 0; k < Record<M>::RW / 2; ++k) v[k] = make_ulonglong2(w[2 * k], w[2 * k + 1]);
}

// ------------------------------------------------------------------------
// Single-GPU engine, claim path (ClaimSet, fpset_dev.h).
//
//   k_claim  : one workgroup = TILE consecutive parents.  Every successor's
//              fingerprint goes into an LDS hash table keeping the minimum
//              tile-local key (parent << 5 | position); siblings in BFS order
//              produce the same state often (diamonds: a-then-b = b-then-a),
//              so about half of all successors die here without touching HBM.
//              Then each tile representative claims its fp in the ClaimSet
//              (one 16-B slot read; a CAS only for a new fp).  The lane that
//              inserts an fp sets its bit in its parent's newmask word (a
//              provisional win).  A claimant that finds a larger claim
//              stored (or none yet) is a candidate: per tile, a list of
//              {fp, tile-local key}.
//   k_settle_rec<0> : every candidate folds its claim into its slot
//              (atomicMax).  One that displaces a claim clears the displaced
//              claim's newmask bit (its parent index and position are the
//              claim's key) and flags itself a displacer.
//   k_settle_rec<1> : every displacer wins iff the stored claim is still
//              its own -> sets its newmask bit.
// Inserters never re-read their slot: only a displacement can take their
// win away, and it clears their bit itself.  The scan then runs over
// popcount(newmask); no successor is re-derived.
// Tile-local dedup only ever discards a copy whose fp is held by a smaller
// key of the same tile, which can never be the level minimum; an LDS table
// overflow just sends the copy to the ClaimSet directly.
constexpr int CLAIM_TILE = 256;
// tile representatives whose first probe loads a lane issues together (A/B:
// build with -DKC_CLAIM_BATCH=1 for one at a time)
// k_claim deals each tile's parents to its waves by successor count (build
// with -DKC_DEAL=0 for lane = parent)
#ifndef KC_DEAL
#define KC_DEAL 1
#endif
#ifndef KC_CLAIM_BATCH
#define KC_CLAIM_BATCH 2
#endif
// KC_CLAIM_PIPE (default 1; 0 for A/B): the CASes of a group's
// representatives whose first slot read empty are issued back to back as
// well, before any result is used (one round trip for the group's inserts
// instead of one each).  Same box, NP=2: k_claim 103.2-103.9 ms per check
// against 103.9-105.3 (profiles/r04p_claim_pipe_ab.txt); with groups of 3
// 105.4 (not kept).
#ifndef KC_CLAIM_PIPE
#define KC_CLAIM_PIPE 1
#endif
constexpr int CLAIM_LDS_BITS = 11;
constexpr int CLAIM_LDS = 1 << CLAIM_LDS_BITS;   // entries (fp 8 B + key 4 B)
// Candidate records (claimants whose claim may win): fp + tile-local key
// (bit 31: set by settle pass A on a displacer).  Each tile keeps its first
// CLAIM_RCAP in its own segment (12 B per parent); the rest of a busy tile's
// go to one overflow list shared by the chunk, {fp, key, tile}, sized by the
// chunk's successor count (an exact upper bound), so it cannot overflow
// either.  (A segment of CLAIM_TILE * 32 per tile, the worst case, cost 384 B
// per parent: 6 GB at NP=2's widest level for ~0.1 candidate per parent.)
constexpr int CLAIM_RCAP = 256;
constexpr unsigned int CAND_DISPLACER = 1u << 31;
struct CandOvf {
  unsigned long long* count = nullptr;   // records pushed (may exceed cap: then C->overflow)
  unsigned long long* fp = nullptr;
  unsigned int* lk = nullptr;
  unsigned int* tile = nullptr;
  uint64_t cap = 0;
};

__device__ __forceinline__ void push_candidate(unsigned int* sh_rc, uint64_t tile,
                                               unsigned long long* __restrict__ rec_fp,
                                               unsigned int* __restrict__ rec_lk, uint64_t fp,
                                               unsigned int lk, const CandOvf& ovf, Counters* __restrict__ C) {
  const unsigned int k = atomicAdd(sh_rc, 1u);
  if (k < (unsigned)CLAIM_RCAP) {
    rec_fp[tile * CLAIM_RCAP + k] = fp;
    rec_lk[tile * CLAIM_RCAP + k] = lk;
    return;
  }
  const unsigned long long g = ovf.count ? atomicAdd(ovf.count, 1ull) : ~0ull;
  if (g < ovf.cap) {
    ovf.fp[g] = fp;
    ovf.lk[g] = lk;
    ovf.tile[g] = (unsigned int)tile;
  } else {
    atomicAdd(&C->overflow, 1ull);
  }
}

// The LDS table of the sharded variant is smaller (CLAIM_LDS_SH entries):
// its per-parent owner counts take LDS too, and 2048 entries would leave
// room for 5 workgroups per CU instead of 6 (measured: k_claim 686 vs 564 us
// per launch at RCCL world 1, r02i).
constexpr int CLAIM_LDS_SH = 1792;
static_assert(CLAIM_LDS_SH % CLAIM_TILE == 0, "whole entries per lane in the compaction");
// (KC_LDS_LOWBITS: the slot from the fingerprint's low 32 bits — the
// Zobrist fold, uniform in every bit on both paths — with no 64-bit
// multiply; A/B switch, 0 = the remixed slot of rounds 1-3)
#ifndef KC_LDS_LOWBITS
#define KC_LDS_LOWBITS 1
#endif
template <int NT = CLAIM_LDS>
__device__ __forceinline__ int lds_claim(unsigned long long* sh_fp, unsigned int* sh_key,
                                         uint64_t fp, unsigned int lk) {
  unsigned int h;
  if (KC_LDS_LOWBITS)
    h = NT == CLAIM_LDS ? (unsigned int)fp & (CLAIM_LDS - 1) : __umulhi((unsigned int)fp, (unsigned int)NT);
  else
    h = NT == CLAIM_LDS ? (unsigned int)((fp * 0xd6e8feb86659fd93ull) >> (64 - CLAIM_LDS_BITS))
                        : (unsigned int)(((fp * 0xd6e8feb86659fd93ull) >> 32) * (uint64_t)NT >> 32);
  for (int p = 0; p < NT; ++p) {
    unsigned long long e = __hip_atomic_load(&sh_fp[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (e == 0ull) {
      e = atomicCAS(&sh_fp[h], 0ull, (unsigned long long)fp);
      if (e == 0ull) e = fp;
    }
    if (e == fp) {
      atomicMin(&sh_key[h], lk);
      return (int)h;
    }
    h = (h + 1 == (unsigned int)NT) ? 0u : h + 1;
  }
  return -1;
}

// Fingerprint-owner sharding (shard.hip, SH = true): a rank claims only the
// fingerprints it owns, owner(fp) = floor(fp * R / 2^63); every other tile
// representative is marked in repmask and counted per owner for the record
// exchange.  Claim keys carry the rank above the parent index.
constexpr int CLAIM_RANK_SHIFT = 40;
// Claim keys (the ClaimSet keeps the smallest claim of a level).  Default:
// rank << 40 | parent index << 8 | position, i.e. (rank, parent, position)
// order.  TLC order (the sharded loop's tlc_order mode at world > 1): G << 12
// | position << 4 | rank, G = the parent's position in the level in
// sequential-BFS order (gpos[parent]), so the smallest claim is the first
// discovery of TLC -workers 1; a rank maps its own claims back to local
// parents with the level's rank-select map of its G values (gbits: one bit
// per G of the level; grank: the set bits before each word).
struct ClaimKeys {
  uint32_t rank = 0;
  const uint32_t* gpos = nullptr;
  const uint32_t* gbits = nullptr;
  const uint32_t* grank = nullptr;
  __host__ __device__ ClaimKeys(uint32_t r = 0) : rank(r) {}
  __device__ __forceinline__ uint64_t own(uint64_t pidx, uint32_t t) const {
    if (gpos) return ((uint64_t)gpos[pidx] << 12) | ((uint64_t)t << 4) | rank;
    return ((uint64_t)rank << CLAIM_RANK_SHIFT) | (pidx << 8) | t;
  }
  // a claim key of this rank: its parent's local index and position
  __device__ __forceinline__ bool mine(uint64_t key, uint64_t& pp, uint32_t& t) const {
    if (!gpos) {
      if ((uint32_t)(key >> CLAIM_RANK_SHIFT) != rank) return false;
      pp = (key >> 8) & 0xffffffffull;
      t = (uint32_t)(key & 31);
      return true;
    }
    if ((uint32_t)(key & 15) != rank) return false;
    const uint64_t g = key >> 12;
    const uint32_t w = gbits[g >> 5], b = 1u << (g & 31);
    pp = (w & b) ? (uint64_t)grank[g >> 5] + (uint64_t)__builtin_popcount(w & (b - 1u)) : ~0ull;
    t = (uint32_t)((key >> 4) & 31);
    return true;
  }
};
// claim key of a record key (rank << 60 | parent << 16 | position << 8 |
// action; in TLC order the parent field holds G)
__host__ __device__ __forceinline__ uint64_t record_ckey(uint64_t key, bool tlc) {
  if (tlc) return (((key >> 16) & 0xffffffffull) << 12) | (((key >> 8) & 0xff) << 4) | (key >> 60);
  return ((key >> 60) << CLAIM_RANK_SHIFT) | (((key >> 16) & 0xffffffffull) << 8) | ((key >> 8) & 0xff);
}
constexpr uint32_t CLAIM_SPREAD = 768;   // k_claim tile-order columns (spread_tile)
// (k_claim's per-launch arguments beyond the engine's: owner sharding, the
// tile order, and the candidate overflow list)
struct ShardArgs {
  uint32_t world = 1, rank = 0;
  uint32_t spread = CLAIM_SPREAD; // tile order strided by `spread` (spread_tile); 0 = block order
  uint32_t* repmask = nullptr;   // [n]: remote representatives of each parent
  uint8_t* cnt = nullptr;        // [world][n]: remote representatives per owner and parent (<= 32: 8 bits)
  CandOvf ovf;
  // Record staging (round 5; stage != nullptr): each tile writes its remote
  // representatives' records itself, grouped by owner and in (parent,
  // position) order within an owner, into a segment of the staging buffer
  // it reserves with one atomic; tcnt / stoff let k_shard_gather move the
  // segments into the owner-grouped send buffer in tile order: the order
  // k_shard_pack produced from the per-parent owner scan, with neither the
  // re-expansion nor the scan.  A tile whose segment does not fit sets
  // DF_STAGE and stages nothing; the host then packs that level the old way
  // (repmask / cnt are written either way).
  void* stage = nullptr;                      // Record<M>[stage_cap]
  unsigned long long* stage_cur = nullptr;    // records reserved this level
  uint64_t stage_cap = 0;
  uint32_t* tcnt = nullptr;                   // [world][tiles]: records per owner and tile
  unsigned long long* stoff = nullptr;        // [tiles]: the tile's first staging record (~0: none staged)
  // TLC order (ClaimKeys): G of each parent of the level; records and claims
  // then carry G instead of the local parent index
  const uint32_t* gpos = nullptr;
  // first-claim mode (k_claim FIRST; the engine, KC_FIRST_CLAIM): each tile's
  // new-state count, the input of k_tile_scan (no settle passes run)
  uint32_t* ttot = nullptr;
  // (round 6, the engine's first-claim levels) each tile's count also added
  // into its chunk of CSUM_TILES tiles: k_chunk_scan then scans T / 64 sums
  // instead of T counts, and the link emit finishes a tile's offset itself
  uint32_t* csum = nullptr;
  // (round 6, the sharded staging) each tile's per-owner record counts also
  // added into ocsum[owner][chunk of CSUM_TILES tiles]: k_owner_cscan scans
  // those, k_shard_gather finishes a tile's positions itself
  uint32_t* ocsum = nullptr;
};
constexpr uint32_t CSUM_TILES = 64;
// Tile order of k_claim.  Block b takes tile (b % S) * share + b / S: the
// workgroups resident together (~1,536: 6 per CU) work on tiles spread over
// the whole level, and each of the S columns of tiles is walked in order.
// Same-level duplicates come mostly from neighbouring parents, i.e. from
// neighbouring tiles; in block order those run at the same time and the
// later key often claims first (a settle candidate, an atomicMax); spread,
// tile t + 1 of a column runs after tile t, finds t's smaller claim and
// loses at once.  NP=2: settle candidates 440M -> 110M per check, 171 ->
// 157 ms (S = CLAIM_SPREAD = 768 measured best of 128..3072).  A bijection
// of [0, G).
__device__ __forceinline__ uint32_t spread_tile(uint32_t b, uint32_t G, uint32_t S) {
  if (S == 0 || S >= G) return b;
  const uint32_t x = b % S, k = b / S, g = G / S, rem = G % S;
  return x * g + (x < rem ? x : rem) + k;
}

__device__ __forceinline__ uint32_t owner_of(uint64_t fp, uint32_t world) {
  return (uint32_t)__umul64hi(fp << 1, (uint64_t)world);
}

// Deferred frontier (the engine's default wide path): k_emit writes only
// each new state's link (parent index in its level, successor position) —
// the trace entries — and the next level's k_claim rebuilds its parent from
// the previous frontier: load the grandparent, plan, apply the successor,
// store the state into the frontier buffer, check the invariants and count
// its action (act_dist).  That work then runs inside k_claim, whose time is
// set by its random memory operations, instead of in a k_emit of its own.
// Any invariant violation sets DF_INVARIANT: the host then re-runs the check
// on the exact (materialising) path, so error reports are unchanged.
// Per-action LDS counters of k_claim / k_materialize, ACT_STRIPES copies
// indexed by lane: the lanes of a wave mostly count the same few actions,
// and LDS atomics on one address serialise.
#ifndef KC_ACT_STRIPES
#define KC_ACT_STRIPES 4
#endif
constexpr int ACT_STRIPES = KC_ACT_STRIPES;
template <int AS = ACT_STRIPES>
__device__ __forceinline__ unsigned int act_sum(const unsigned int* sh, unsigned int a) {
  unsigned int v = 0;
#pragma unroll
  for (int k = 0; k < AS; ++k) v += sh[a * AS + k];
  return v;
}
struct DeferArgs {
  const void* prev = nullptr;                 // the previous frontier (State*); nullptr: cur holds the states
  // sharded k_claim (SH): link[i] >> 63 set = frontier state i is received
  // record link[i] & ~(1 << 63) of the previous level (prev_rec, Record<M>*);
  // else parent index << 8 | position in the previous frontier, as above
  const void* prev_rec = nullptr;
  const unsigned long long* parent = nullptr; // trace: global parent index per state (keep_trace) ...
  const uint8_t* ord = nullptr;               // ... and successor position
  const unsigned long long* link = nullptr;   // or, without a trace: parent index << 8 | position
  uint64_t gidx0 = 0;                         // global index of this frontier's state 0 (trace path)
  uint64_t prev_gidx0 = 0;                    // global index of the previous frontier's state 0
  void* out = nullptr;                        // where the rebuilt states go (State*; the frontier buffer)
  // successor plans (Plan::counts) of the previous frontier's states, as its
  // k_claim computed them (nullptr: plan the grandparent here)
  const unsigned long long* prev_counts = nullptr;
  // where k_claim writes its own parents' plans for the next level (any k_claim
  // of the engine's wide path; nullptr: not kept)
  unsigned long long* counts_out = nullptr;
  // diagnostic (sharded, KC_DEFER_CHECK=1): out already holds the states the
  // materialising emit built; each rebuilt state is compared with its slot:
  // check[0] += mismatches, check[1] = min mismatching index, check[2] = min
  // mismatching index whose link is a received record
  unsigned long long* check = nullptr;
  // TLC order: G of each state of the previous frontier (error keys by G)
  const uint32_t* prev_gpos = nullptr;
};

// Rebuild frontier state i (index within the level) from its link; stores it
// into df.out, checks the invariants and counts its action into sh_actd.
template <class M, int AS = ACT_STRIPES>
__device__ __forceinline__ typename M::State defer_rebuild(const DeferArgs& df, uint64_t i, const Flags& f,
                                                           unsigned int* sh_actd, Counters* __restrict__ C) {
  uint64_t pp;
  int t;
  if (df.link) {
    const unsigned long long lk = df.link[i];
    pp = lk >> 8;
    t = (int)(lk & 0xff);
  } else {
    pp = df.parent[df.gidx0 + i] - df.prev_gidx0;
    t = (int)df.ord[df.gidx0 + i];
  }
  const typename M::State gp = load_state<M>(reinterpret_cast<const typename M::State*>(df.prev), pp);
  const typename M::Plan pl{df.prev_counts ? df.prev_counts[pp] : M::plan(gp, f).counts, 0, -1, -1};
  int slot, j;
  M::locate(pl, t, slot, j);
  typename M::State s;
  M::apply(gp, slot, j, f, s);
  store_state<M>(reinterpret_cast<typename M::State*>(df.out), i, s);
  if (M::check(s, f.inv_mask) >= 0) {
    atomicOr(&C->defer_flags, DF_INVARIANT);
    atomicMax(&C->defer_inv_n, ~(unsigned long long)i);   // the level's first violator in BFS order
  }
  atomicAdd(&sh_actd[M::slot_action(gp, slot) * AS + (threadIdx.x & (AS - 1))], 1u);
  return s;
}

// The sharded deferred frontier (round 5): rebuild frontier state i of rank
// `rank` from its link — its own parent in the previous frontier, or a
// record it received last level (kept in that level's receive buffer) —
// store it, check the invariants (the key the materialising emit would have
// made, into C->defer_err: an error of the previous level) and count its
// action into sh_actd.
template <class M, int AS = ACT_STRIPES, bool TLC = false>
__device__ __forceinline__ typename M::State shard_rebuild(const DeferArgs& df, uint64_t i, const Flags& f,
                                                           uint64_t rank, unsigned int* sh_actd,
                                                           Counters* __restrict__ C) {
  const unsigned long long lk = df.link[i];
  typename M::State s;
  uint64_t key;
  int act;
  if (lk >> 63) {
    load_record<M>(reinterpret_cast<const Record<M>*>(df.prev_rec), lk & ~(1ull << 63), s, key);
    act = (int)(key & 0xff);
  } else {
    const uint64_t pp = lk >> 8;
    const int t = (int)(lk & 0xff);
    const typename M::State gp = load_state<M>(reinterpret_cast<const typename M::State*>(df.prev), pp);
    const typename M::Plan pl{df.prev_counts ? df.prev_counts[pp] : M::plan(gp, f).counts, 0, -1, -1};
    int slot, j;
    M::locate(pl, t, slot, j);
    M::apply(gp, slot, j, f, s);
    act = M::slot_action(gp, slot);
    key = (rank << 60) | ((TLC ? (uint64_t)df.prev_gpos[pp] : pp) << 16) | ((uint64_t)t << 8);
  }
  if (df.check) {
    const typename M::State e = load_state<M>(reinterpret_cast<const typename M::State*>(df.out), i);
    bool same = true;
#pragma unroll
    for (int k = 0; k < M::W; ++k) same &= e.w[k] == s.w[k];
    if (!same) {
      atomicAdd(&df.check[0], 1ull);
      atomicMin(&df.check[1], (unsigned long long)i);
      if (lk >> 63) atomicMin(&df.check[2], (unsigned long long)i);
    }
  }
  store_state<M>(reinterpret_cast<typename M::State*>(df.out), i, s);
  // (TLC order: errors order by G alone, no rank above it)
  if (M::check(s, f.inv_mask) >= 0)
    atomicMin(&C->defer_err, (key & (TLC ? 0x0fffffffffffff00ull : ~0xffull)) | E_INVARIANT);
  // (a record's action byte indexes LDS: anything out of range would be a
  // corrupt record, counted nowhere)
  if ((unsigned)act < (unsigned)A_COUNT) atomicAdd(&sh_actd[act * AS + (threadIdx.x & (AS - 1))], 1u);
  return s;
}

// Deferred-frontier materialisation outside k_claim (the level before a
// narrow run, a max_levels stop, a captured level): the same rebuild, plus
// the level's successor count (next_cand).
template <class M>
__global__ void __launch_bounds__(256) k_materialize(DeferArgs df, uint64_t n, Flags f, Counters* __restrict__ C) {
  __shared__ unsigned int sh_actd[A_COUNT * ACT_STRIPES];
  if (threadIdx.x < A_COUNT * ACT_STRIPES) sh_actd[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long cand = 0;
  if (i < n) {
    const typename M::State s = defer_rebuild<M>(df, i, f, sh_actd, C);
    cand = (unsigned long long)M::plan(s, f).total;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cand += __shfl_down(cand, off, 64);
  if ((threadIdx.x & 63) == 0 && cand) atomicAdd(&stripe(C).next_cand, cand);
  __syncthreads();
  if (threadIdx.x < A_COUNT) {
    const unsigned int v = act_sum(sh_actd, threadIdx.x);
    if (v) atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)v);
  }
}

// The parent chain of global state g (TLC's trace-file walk), on the
// device: one lane follows the parent pointers from g back to its Init
// state; out[k] = state index << 8 | ordinal, *len = the chain's length
// (0: longer than cap, a corrupt chain).  Writes pinned host memory.
static __global__ void k_parent_chain(const unsigned long long* __restrict__ parent, const uint8_t* __restrict__ ord,
                                      uint64_t g, uint64_t* __restrict__ out, uint32_t cap,
                                      uint64_t* __restrict__ len) {
  if (threadIdx.x != 0) return;
  uint32_t k = 0;
  for (;;) {
    if (k >= cap) {
      *len = 0;
      return;
    }
    const unsigned long long p = parent[g];
    out[k++] = (g << 8) | (uint64_t)ord[g];
    if (p == ~0ull) break;
    g = p;
  }
  *len = k;
}

// Record staging of the sharded k_claim (ShardArgs::stage): after the claim
// loop, with the per-parent remote masks (sh_rep) and per-owner counts
// (sh_cnt, 4 x 8 bits per word) complete and the LDS table free.
//   1. per owner, the exclusive prefix of the counts over the tile's parents
//      (lane = parent; two owners per word in 16-bit halves: a tile has at
//      most 256 x 32 records) -> pre[owner pair][parent]; the prefix of the
//      parents' remote-representative counts -> rbase[parent]; each dealt
//      lane leaves its parent's plan word (and fold) in LDS;
//   2. the tile's totals per owner, its segment reserved with one atomic,
//      tcnt / stoff for k_shard_gather;
//   3. the tile's remote representatives dealt out flat, one per lane per
//      round (round 5: per parent, one lane ran all of its parent's records,
//      and a wave waited for its busiest parent): lane r finds its parent
//      and position (rbase, the remote mask), reloads the parent (the
//      frontier or the rebuilt states: L2), re-applies the successor and
//      takes its owner; after a barrier, its rank among the parent's records
//      of that owner (their owners, as 4-bit codes per position in LDS, are
//      all known: the parent's lower positions are lower ranks r) places
//      the record at segment base + owner base + the parent's prefix for
//      that owner + that rank — the order the per-parent loop produced.
// At R = 2^k the owner comes from the successor's owner bits alone
// (kubeapi_spec.h owner_bits_succ), else from its fingerprint (the parent's
// fold kept in LDS).
template <class M, int NT, bool TLC = false>
__device__ __forceinline__ void stage_records(const ShardArgs& sh, bool live, uint64_t fold, uint64_t counts,
                                              uint32_t lp, Flags f, const unsigned int* sh_rep,
                                              const unsigned int* sh_cnt, const uint32_t* sh_proj,
                                              unsigned long long* sh_fp, unsigned int* sh_key, uint32_t tile,
                                              const typename M::State* __restrict__ psrc, uint64_t pbase0,
                                              uint64_t pkey0, Counters* __restrict__ C) {
  constexpr bool SWAR = KC_LOCATE_SWAR && M::CUM_OK;
  static_assert(NT * 8 >= 8 * CLAIM_TILE * 4, "pre[] needs (world + 1) / 2 x 256 words (world <= 15)");
  static_assert(NT >= 1536 && CLAIM_TILE == 256, "stage LDS layout (below)");
  const uint32_t R = sh.world, npair = (R + 1) / 2;
  // LDS (the claim table's, free now): sh_fp as u32 pre[npair][256], then
  // u64 pcnt[256] and pfold[256] (<= 8 x 128 + 512 u64 words); sh_key:
  // wsum [0, 32), tt [32, 64), seg [64, 66), rbase [128, 384), rep wave
  // totals [384, 388), owner codes onib[256][4] at [512, 1536)
  uint32_t* pre = reinterpret_cast<uint32_t*>(sh_fp);   // [npair][CLAIM_TILE]
  unsigned long long* pcnt = sh_fp + npair * (CLAIM_TILE / 2);
  unsigned long long* pfold = pcnt + CLAIM_TILE;
  unsigned int* wsum = sh_key;                          // [4 waves][8 pairs]
  unsigned int* tt = sh_key + 32;                       // [0, 16): per-owner totals; [16, 32): owner bases
  unsigned int* seg = sh_key + 64;                      // segment base, lo / hi (~0: none)
  unsigned int* rbase = sh_key + 128;
  unsigned int* rwave = sh_key + 384;
  unsigned int* onib = sh_key + 512;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (uint32_t w = 0; w < npair; ++w) {
    const uint32_t o0 = 2 * w, o1 = 2 * w + 1;
    uint32_t v = (sh_cnt[(o0 >> 2) * CLAIM_TILE + tid] >> (8 * (o0 & 3))) & 0xffu;
    if (o1 < R) v |= ((sh_cnt[(o1 >> 2) * CLAIM_TILE + tid] >> (8 * (o1 & 3))) & 0xffu) << 16;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[wv * 8 + w] = x;
    pre[w * CLAIM_TILE + tid] = x - v;
  }
  const uint32_t nrep = (uint32_t)__builtin_popcount(sh_rep[tid]);
  uint32_t rx = nrep;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(rx, d, 64);
    if (lane >= (uint32_t)d) rx += y;
  }
  if (lane == 63) rwave[wv] = rx;
#pragma unroll
  for (int q = 0; q < 4; ++q) onib[tid * 4 + q] = 0u;
  if (live) {
    pcnt[lp] = counts;
    pfold[lp] = fold;
  }
  __syncthreads();
  for (uint32_t w = 0; w < npair; ++w) {
    uint32_t b = 0;
    for (uint32_t k = 0; k < wv; ++k) b += wsum[k * 8 + w];
    pre[w * CLAIM_TILE + tid] += b;
  }
  {
    uint32_t b = 0;
    for (uint32_t k = 0; k < wv; ++k) b += rwave[k];
    rbase[tid] = b + rx - nrep;
  }
  if (tid < R) {
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < CLAIM_TILE / 64; ++k) a += wsum[k * 8 + (tid >> 1)];
    tt[tid] = (a >> (16 * (tid & 1))) & 0xffffu;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t o = 0; o < R; ++o) {
      tt[16 + o] = acc;
      acc += tt[o];
    }
    unsigned long long b = acc ? atomicAdd(sh.stage_cur, (unsigned long long)acc) : 0ull;
    if (acc && b + acc > sh.stage_cap) {
      atomicOr(&C->defer_flags, DF_STAGE);
      b = ~0ull;
    }
    seg[0] = (unsigned int)b;
    seg[1] = (unsigned int)(b >> 32);
    sh.stoff[tile] = b;
  }
  if (tid < R) {
    sh.tcnt[(uint64_t)tid * gridDim.x + tile] = tt[tid];
    if (sh.ocsum && tt[tid])
      atomicAdd(&sh.ocsum[(uint64_t)tid * ((gridDim.x + CSUM_TILES - 1) / CSUM_TILES) + tile / CSUM_TILES], tt[tid]);
  }
  __syncthreads();
  const unsigned long long sb = (unsigned long long)seg[0] | ((unsigned long long)seg[1] << 32);
  const uint32_t total = rwave[0] + rwave[1] + rwave[2] + rwave[3];
  if (sb == ~0ull || total == 0) return;                 // (uniform over the workgroup)
  Record<M>* out = reinterpret_cast<Record<M>*>(sh.stage);
  static_assert(M::OWNER_BITS == 4, "owner bits >> (4 - k) at R = 2^k");
  const int sh_pow2 = R == 1 ? 4 : R == 2 ? 3 : R == 4 ? 2 : R == 8 ? 1 : -1;
  for (uint32_t r0 = 0; r0 < total; r0 += CLAIM_TILE) {
    const uint32_t r = r0 + tid;
    const bool act = r < total;
    uint32_t p = 0, t = 0, o = 0, m = 0;
    typename M::State x;
    uint64_t key = 0;
    if (act) {
      uint32_t lo = 0, hi = CLAIM_TILE;                  // the last parent with rbase <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rbase[mid] <= r) lo = mid; else hi = mid;
      }
      p = lo;
      m = sh_rep[p];
      uint32_t mm = m;
      for (uint32_t k = r - rbase[p]; k > 0; --k) mm &= mm - 1;
      t = (uint32_t)(__ffs(mm) - 1);
      const typename M::State ps = load_state<M>(psrc, pbase0 + p);
      const uint64_t pc = pcnt[p];
      int slot, j;
      if (SWAR) {
        M::locate_cum(pc, (int)t, slot, j);
      } else {
        const typename M::Plan pl{pc, 0, -1, -1};
        M::locate(pl, (int)t, slot, j);
      }
      int who;
      M::apply(ps, slot, j, f, x, who);
      const uint32_t proj = sh_proj[p];
      o = sh_pow2 >= 0 ? (M::owner_bits_succ(ps, x, who, proj) >> sh_pow2)
                       : owner_of(M::template fingerprint_succ<1>(ps, pfold[p], x, who, proj), R);
      atomicOr(&onib[p * 4 + (t >> 3)], o << (4 * (t & 7)));
      const uint64_t pg = pkey0 + p;                     // the parent's index in the frontier
      key = ((uint64_t)sh.rank << 60) | ((TLC ? (uint64_t)sh.gpos[pg] : pg) << 16) | ((uint64_t)t << 8) |
            (uint64_t)M::slot_action(ps, slot);
    }
    __syncthreads();
    if (act) {
      // the parent's records of owner o at lower positions
      uint32_t below = 0;
      const uint32_t lower = m & ((1u << t) - 1u);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t wq = onib[p * 4 + q] ^ (o * 0x11111111u);   // nibble 0 = owner o
        const uint32_t lm = (lower >> (8 * q)) & 0xffu;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          below += (((lm >> i) & 1u) && ((wq >> (4 * i)) & 0xfu) == 0u) ? 1u : 0u;
      }
      const uint64_t pos = sb + tt[16 + o] + ((pre[(o >> 1) * CLAIM_TILE + p] >> (16 * (o & 1))) & 0xffffu) + below;
      store_record<M>(out, pos, x, key);
    }
  }
}

// ABL (diagnostic builds of the same kernel, launched on scratch buffers when
// KC_ABLATE=1): 1 = successors + LDS dedup only, 2 = successors only,
// 3 = plan + fold only (no successor), 4 = successors with an XOR of their
// words for a fingerprint (2 - 4: the fingerprint's cost), 5 = fingerprints
// of the parent with one word perturbed, no apply (2 - 5: apply's cost).
// Occupancy: the LDS table (24 KB) allows 6 workgroups = 6 waves per SIMD;
// the claims are latency-bound random probes, so the register budget is
// pinned to match (one wave less measured +15 ms per NP=2 check).
// OWN: the fingerprints' owner projection (kubeapi_spec.h; 1 on the sharded
// path, also at world 1 where it runs the SH = false variant)
// TLC (SH only): claims, records and keys by the parents' G (ClaimKeys; the
// sharded loop's tlc_order mode), a variant of its own so the default one's
// registers are untouched
// Diagnostic builds (-DKC_CLAIM_TRACE): thread 0 of every k_claim workgroup
// stamps the wall clock (100 MHz) at its phase boundaries and adds each
// phase's duration to g_ctrace[1..7] ([0] workgroups, [8] the longest
// workgroup, [9] / [10] the earliest start / latest end); the host reads and
// resets it after each launch (shard.hip).
#ifdef KC_CLAIM_TRACE
static __device__ unsigned long long g_ctrace[16];
#define KC_CT(k)                                 \
  do {                                           \
    if (threadIdx.x == 0) ct[k] = wall_clock64(); \
  } while (0)
#else
#define KC_CT(k) ((void)0)
#endif
// FIRST (the engine only): first-claim mode, TLC's -workers N semantics —
// the copy whose CAS inserts a fingerprint is its new state, every other copy
// (an earlier level's, or a later claimant's of this level) is not new; no
// candidates, no settle passes, the tile's new-state count written here.
// Counts, widths and trace lengths are the exact path's; which copy of a
// same-level duplicate wins (its parent, its action's distinct count) is
// not deterministic, as in a multi-worker TLC run.
// C8 (FIRST only): the compact ClaimSet, u64 fp words (DevClaimSet::compact;
// the engine's and the sharded loop's first-claim mode)
template <class M, int ABL = 0, bool SH = false, int OWN = SH ? 1 : 0, bool TLC = false, bool FIRST = false,
          bool C8 = false>
__global__ void __launch_bounds__(CLAIM_TILE)
__attribute__((amdgpu_waves_per_eu(6, 6)))
k_claim(const typename M::State* __restrict__ cur, uint64_t n, uint64_t base, Flags f,
        int check_deadlock, ClaimEntry* __restrict__ cs, uint64_t nbuckets, uint32_t level,
        uint32_t* __restrict__ scratch /* ABL builds only */, unsigned int* __restrict__ rcount,
        unsigned long long* __restrict__ rec_fp, unsigned int* __restrict__ rec_lk,
        uint32_t* __restrict__ newmask, Counters* __restrict__ C, ShardArgs sh, DeferArgs df = DeferArgs{}) {
  constexpr int NT = SH ? CLAIM_LDS_SH : CLAIM_LDS;
  static_assert(!C8 || (FIRST && !TLC), "the compact ClaimSet holds no claim words (first-claim mode)");
  unsigned long long* const cs8 = reinterpret_cast<unsigned long long*>(cs);
  // (one stripe of action counters on the sharded path: OWN's projections
  // take that LDS, and 6 workgroups per CU need it)
  constexpr int AS = OWN ? 1 : ACT_STRIPES;
  __shared__ unsigned long long sh_fp[NT];
  __shared__ unsigned int sh_key[NT];
  __shared__ unsigned int sh_cur[CLAIM_TILE];     // newmask of the tile's parents
  __shared__ unsigned int sh_act[A_COUNT * AS];
  __shared__ unsigned int sh_actd[A_COUNT * AS];   // deferred frontier: actions that made the parents
  __shared__ unsigned long long sh_dcand;         // deferred frontier: the parents' successor count
  __shared__ uint32_t sh_proj[OWN ? CLAIM_TILE : 1];  // OWN = 1: each parent's owner projection (kubeapi_spec.h)
  __shared__ unsigned int sh_rc;
  __shared__ unsigned int sh_nrep;                // tile representatives
  // SH only (dynamic LDS): remote representatives per parent, then their
  // counts per owner packed 4 owners x 8 bits per word (a parent has <= 32)
  extern __shared__ unsigned int sh_dyn[];
  unsigned int* sh_rep = sh_dyn;
  unsigned int* sh_cnt = sh_dyn + CLAIM_TILE;
  if (threadIdx.x == 0) {
    sh_rc = 0;
    sh_nrep = 0;
    sh_dcand = 0;
  }
  // DEAL: each tile's parents are dealt to its waves in order of successor
  // count (below), staged through the LDS table, which is cleared after that
  // (state words in sh_fp; fold and plan there too when they fit, else as
  // 32-bit halves in sh_key past the counters: the sharded table is smaller)
  constexpr bool DEAL_FP = (M::W + 2) * CLAIM_TILE <= NT;
  constexpr int DEAL_KEY0 = CLAIM_TILE + 128;             // sh_key: fold lo/hi, plan lo/hi
  constexpr bool DEAL = KC_DEAL && (DEAL_FP || (M::W * CLAIM_TILE <= NT && DEAL_KEY0 + 4 * CLAIM_TILE <= NT));
  unsigned int* const deal_cnt = sh_key + CLAIM_TILE;   // parents per successor count
  unsigned int* const deal_start = deal_cnt + 64;
  static_assert(!DEAL || CLAIM_TILE + 64 + M::MAXSUCC + 1 <= NT, "deal counters");
  if (DEAL) {
    if (threadIdx.x <= M::MAXSUCC) deal_cnt[threadIdx.x] = 0;
  } else {
    for (int k = threadIdx.x; k < NT; k += CLAIM_TILE) {
      sh_fp[k] = 0ull;
      sh_key[k] = ~0u;
    }
  }
  if (SH) {
    sh_rep[threadIdx.x] = 0;
    for (uint32_t k = threadIdx.x; k < ((sh.world + 3) / 4) * CLAIM_TILE; k += CLAIM_TILE) sh_cnt[k] = 0;
  }
  const uint64_t kbase = SH ? ((uint64_t)sh.rank << CLAIM_RANK_SHIFT) : 0ull;
  // (TLC order, SH only: claims by G; ClaimKeys)
  auto okey = [&](uint64_t pidx, uint64_t t) -> uint64_t {
    if (SH && TLC) return ((uint64_t)sh.gpos[pidx] << 12) | (t << 4) | sh.rank;
    return kbase | (pidx << 8) | t;
  };
  sh_cur[threadIdx.x] = 0;
  if (threadIdx.x < A_COUNT * AS) sh_act[threadIdx.x] = sh_actd[threadIdx.x] = 0;
#ifdef KC_CLAIM_TRACE
  unsigned long long ct[8] = {};
#endif
  KC_CT(0);
  __syncthreads();
  const uint32_t tile = spread_tile(blockIdx.x, gridDim.x, sh.spread);
#ifdef KC_DIAG
  // diagnostic builds: ClaimSet outcomes (16-bit counts per ClaimResult 0..3
  // per lane) and the level distance of CL_OLD hits (one extra probe each)
  uint64_t outc = 0;
  __shared__ unsigned int sh_odist[8];
  if (threadIdx.x < 8) sh_odist[threadIdx.x] = 0;
  __syncthreads();
#define KC_DIAG_OUT(r)                                                                        \
  do {                                                                                        \
    outc += (r) < 4 ? 1ull << (16 * (r)) : 0ull;                                              \
    if ((r) == CL_OLD) {                                                                      \
      const uint32_t lv = (uint32_t)((~claimset_get(cs, nbuckets, fp)) >> CLAIM_KEY_BITS);   \
      const uint32_t d = level - lv;                                                          \
      atomicAdd(&sh_odist[d <= 4 ? (d ? d - 1 : 7) : d <= 8 ? 4 : d <= 16 ? 5 : 6], 1u);       \
    }                                                                                         \
  } while (0)
#else
#define KC_DIAG_OUT(r) ((void)0)
#endif
  const uint64_t tile0 = (uint64_t)tile * CLAIM_TILE;
  const uint64_t i = tile0 + threadIdx.x;
  const bool live = i < n;
  unsigned probes = 0;
  typename M::State s;
  uint64_t fold = 0, counts = 0;
  int tot = 0;
  // a deferred frontier: the engine passes its previous frontier; the
  // sharded path (OWN) its links (a rank whose previous frontier was empty
  // has no previous-frontier buffer, only record links)
  const bool dfr = OWN ? df.link != nullptr : df.prev != nullptr;
  if (live) {
    if (dfr)
      s = OWN ? shard_rebuild<M, AS, TLC>(df, base + i, f, sh.rank, sh_actd, C)     // (the sharded path, any world)
              : defer_rebuild<M, AS>(df, base + i, f, sh_actd, C);
    else
      s = load_state<M>(cur, i);
    const typename M::Plan pl = M::plan(s, f);
    if (df.counts_out) df.counts_out[base + i] = pl.counts;
    // (an LDS total, not a register live through the kernel: k_claim sits at
    // its 80-VGPR budget for 6 waves per SIMD)
    if (dfr && pl.total) atomicAdd(&sh_dcand, (unsigned long long)pl.total);
    fold = M::fp_fold(s);
    if (OWN) sh_proj[threadIdx.x] = M::owner_proj(s);
    if (ABL == 0) {
      const uint64_t pidx = base + i;
      if (pl.fail_pos >= 0)
        atomicMin(&C->err_key, (pidx << 16) | ((uint64_t)pl.fail_pos << 8) | E_ASSERT);
      else if (pl.total == 0 && check_deadlock)
        atomicMin(&C->err_key, (pidx << 16) | E_DEADLOCK);
#pragma unroll
      for (int slot = 0; slot < M::NSLOT; ++slot) {      // per-action "generated" (msg 2772)
        const int c = (int)((pl.counts >> (6 * slot)) & 63);
        if (c) atomicAdd(&sh_act[M::slot_action(s, slot) * AS + (threadIdx.x & (AS - 1))], (unsigned)c);
      }
    }
    tot = pl.total;
    if (tot > M::MAXSUCC) {
      if (ABL == 0) atomicAdd(&C->overflow, 1ull);
      tot = M::MAXSUCC;
    }
    counts = pl.counts;
    if (ABL == 3) tot = 0;
  }
#ifdef KC_DIAG
  {
    const int diag_tot = live ? tot : 0;
    int mx = diag_tot, sm = diag_tot;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      mx = max(mx, __shfl_xor(mx, off, 64));
      sm += __shfl_xor(sm, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&stripe(C).loop_max, (unsigned long long)mx);
      atomicAdd(&stripe(C).loop_sum, (unsigned long long)sm);
    }
    __shared__ unsigned int sh_hist[M::MAXSUCC + 1];
    if (threadIdx.x <= M::MAXSUCC) sh_hist[threadIdx.x] = 0;
    __syncthreads();
    if (live) atomicAdd(&sh_hist[diag_tot], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long srt = 0;
      unsigned int seen = 0, next = 0;
      for (int v = M::MAXSUCC; v >= 0; --v) {
        seen += sh_hist[v];
        while (next < seen) { srt += v; next += 64; }
      }
      atomicAdd(&stripe(C).loop_sorted, srt);
    }
  }
#endif
  // Deal: a wave runs its successor loop as many times as its busiest lane
  // needs.  Counting-sort the tile's parents by successor count (descending)
  // and give lane k the k-th, so each wave's lanes need about the same number
  // of trips.  The parent's state, fold and plan move through the (not yet
  // used) LDS table; every key and mask below uses the parent's own index lp.
  // (the parent's index travels in bits 56-63 of its plan, which locate()
  // never reads: one register more across the loop spills k_claim)
  static_assert(!DEAL || (M::NSLOT * 6 <= 56 && CLAIM_TILE <= 256), "deal: lp in the plan word");
  KC_CT(1);
  if (DEAL) {
    const unsigned int pos = live ? atomicAdd(&deal_cnt[tot], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned int at = 0;
      for (int v = M::MAXSUCC; v >= 0; --v) {
        deal_start[v] = at;
        at += deal_cnt[v];
      }
    }
    __syncthreads();
    if (live) {
      const unsigned int d = deal_start[tot] + pos;
#pragma unroll
      for (int k = 0; k < M::W; ++k) sh_fp[k * CLAIM_TILE + d] = s.w[k];
      const uint64_t cl = counts | ((uint64_t)threadIdx.x << 56);
      if (DEAL_FP) {
        sh_fp[M::W * CLAIM_TILE + d] = fold;
        sh_fp[(M::W + 1) * CLAIM_TILE + d] = cl;
      } else {
        sh_key[DEAL_KEY0 + d] = (unsigned)fold;
        sh_key[DEAL_KEY0 + CLAIM_TILE + d] = (unsigned)(fold >> 32);
        sh_key[DEAL_KEY0 + 2 * CLAIM_TILE + d] = (unsigned)cl;
        sh_key[DEAL_KEY0 + 3 * CLAIM_TILE + d] = (unsigned)(cl >> 32);
      }
      sh_key[d] = (unsigned)tot;
    }
    __syncthreads();
    if (live) {   // (the live lanes are a prefix of the tile: slot threadIdx.x was written)
#pragma unroll
      for (int k = 0; k < M::W; ++k) s.w[k] = sh_fp[k * CLAIM_TILE + threadIdx.x];
      if (DEAL_FP) {
        fold = sh_fp[M::W * CLAIM_TILE + threadIdx.x];
        counts = sh_fp[(M::W + 1) * CLAIM_TILE + threadIdx.x];
      } else {
        fold = sh_key[DEAL_KEY0 + threadIdx.x] | ((uint64_t)sh_key[DEAL_KEY0 + CLAIM_TILE + threadIdx.x] << 32);
        counts = sh_key[DEAL_KEY0 + 2 * CLAIM_TILE + threadIdx.x] |
                 ((uint64_t)sh_key[DEAL_KEY0 + 3 * CLAIM_TILE + threadIdx.x] << 32);
      }
      tot = (int)sh_key[threadIdx.x];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < NT; k += CLAIM_TILE) {
      sh_fp[k] = 0ull;
      sh_key[k] = ~0u;
    }
    __syncthreads();
  }
  KC_CT(2);
  if (live) {
#define KC_LP (DEAL ? (unsigned)(counts >> 56) : (unsigned)threadIdx.x)
    // KC_LOCATE_SWAR: the slot lookup from cumulative counts (its top byte
    // keeps the dealt parent's index)
    constexpr bool SWAR = KC_LOCATE_SWAR && M::CUM_OK;
    if (SWAR) counts = M::plan_cum(counts);
    const typename M::Plan pl{counts, tot, -1, -1};
    uint64_t acc = fold ^ counts;
    // (walking (slot, j) along with t instead of locate() measured slower:
    // its three live registers spill at k_claim's 80-VGPR budget; r03w)
    for (int t = 0; t < tot; ++t) {
      int slot, j;
      if (SWAR)
        M::locate_cum(counts, t, slot, j);
      else
        M::locate(pl, t, slot, j);
      typename M::State x;
      int who;
      if (ABL == 5) {
#pragma unroll
        for (int k = 0; k < M::W; ++k) x.w[k] = s.w[k];
        who = slot % M::A;
#pragma unroll
        for (int k = 0; k < M::A; ++k)
          if (k == who) x.w[1 + k] ^= (uint64_t)(j + 1) << (slot & 31);
      } else {
        M::apply(s, slot, j, f, x, who);
      }
      uint64_t fp;
      if (ABL == 4) {
        fp = 0;
#pragma unroll
        for (int k = 0; k < M::W; ++k) fp ^= x.w[k] << k;
      } else {
        fp = OWN ? M::template fingerprint_succ<1>(s, fold, x, who, sh_proj[KC_LP])
                 : M::template fingerprint_succ<0>(s, fold, x, who);
      }
      if (ABL == 2 || ABL == 4 || ABL == 5) {
        acc ^= fp;
        continue;
      }
      if (lds_claim<NT>(sh_fp, sh_key, fp, (KC_LP << 5) | (unsigned)t) < 0 && ABL == 0) {
        // LDS table full: claim (or send) this copy directly
        if (SH) {
          const uint32_t o = owner_of(fp, sh.world);
          if (o != sh.rank) {
            atomicOr(&sh_rep[KC_LP], 1u << t);
            atomicAdd(&sh_cnt[(o >> 2) * CLAIM_TILE + KC_LP], 1u << (8 * (o & 3)));
            continue;
          }
        }
        ++probes;
        const uint64_t pidx = base + tile0 + KC_LP;
        const uint64_t b = C8 ? fpslots_home(fp, nbuckets) : bucket_of(fp, nbuckets);
        const int r = C8      ? fpslots_insert_pair(cs8, nbuckets, fp, b, fpslots_first(cs8, b))
                    : FIRST ? claimset_insert_from(cs, nbuckets, fp, b, cs[b].fp)
                            : claimset_claim_store(cs, nbuckets, fp, make_claim(level, okey(pidx, (uint64_t)t)), level);
        KC_DIAG_OUT(r);
        if (r == CL_NEW)
          atomicOr(&sh_cur[KC_LP], 1u << t);
        else if (r == CL_CUR && !FIRST)
          push_candidate(&sh_rc, tile, rec_fp, rec_lk, fp, (KC_LP << 5) | (unsigned)t, sh.ovf, C);
        else if (r == CL_FULL)
          atomicAdd(&C->overflow, 1ull);
      }
    }
    if (ABL >= 2) sh_cur[KC_LP] = (unsigned)acc;
#undef KC_LP
  }
  __syncthreads();
  KC_CT(3);
  if (ABL != 0) {
    if (live) scratch[i] = sh_cur[threadIdx.x] ^ sh_key[threadIdx.x] ^ (unsigned)sh_fp[threadIdx.x];
    return;
  }
  // compact the tile representatives to the front of the LDS table, so a
  // lane claims ~3 dense entries in a row instead of scanning 8 sparse ones
  // (each scan step costs its wave one probe round trip)
  {
    constexpr int PER = NT / CLAIM_TILE;
    unsigned long long efp[PER];
    unsigned int ekey[PER];
    unsigned int mine = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      efp[j] = sh_fp[threadIdx.x + j * CLAIM_TILE];
      ekey[j] = sh_key[threadIdx.x + j * CLAIM_TILE];
      mine += efp[j] != 0ull;
    }
    unsigned int pos = mine ? atomicAdd(&sh_nrep, mine) : 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (efp[j]) {
        sh_fp[pos] = efp[j];
        sh_key[pos] = ekey[j];
        ++pos;
      }
    }
    __syncthreads();
  }
  KC_CT(4);
  // every tile representative claims its fp in the ClaimSet.  A lane takes
  // representatives k = tid, tid + 256, ... in groups of KC_CLAIM_BATCH:
  // the first probe loads of a group are issued back to back, then each
  // claim runs from its loaded pair (a stale pair only shows a slot empty
  // or a claim larger; the CAS and the settle passes decide).
  const int nrep = (int)sh_nrep;
  for (int k0 = threadIdx.x; k0 < nrep; k0 += CLAIM_TILE * KC_CLAIM_BATCH) {
    unsigned long long fpq[KC_CLAIM_BATCH];
    ulonglong2 eq[KC_CLAIM_BATCH];
    uint64_t iq[KC_CLAIM_BATCH];
#pragma unroll
    for (int q = 0; q < KC_CLAIM_BATCH; ++q) {
      const int k = k0 + q * CLAIM_TILE;
      fpq[q] = k < nrep ? sh_fp[k] : 0ull;
      if (fpq[q] && (!SH || owner_of(fpq[q], sh.world) == sh.rank)) {
        iq[q] = C8 ? fpslots_home(fpq[q], nbuckets) : bucket_of(fpq[q], nbuckets);
        eq[q] = C8 ? fpslots_first(cs8, iq[q]) : claimset_first(cs, iq[q]);
      }
    }
#if KC_CLAIM_PIPE
    unsigned long long cq[KC_CLAIM_BATCH];     // CAS results (~0: no CAS issued)
#pragma unroll
    for (int q = 0; q < KC_CLAIM_BATCH; ++q) {
      const int k = k0 + q * CLAIM_TILE;
      cq[q] = ~0ull;
      if (C8) {                                   // (the pair's first empty slot)
        const uint64_t j = k < nrep && fpq[q] && (!SH || owner_of(fpq[q], sh.world) == sh.rank)
                               ? fpslots_pair_target(iq[q], eq[q], fpq[q]) : ~0ull;
        if (j < ~1ull) cq[q] = atomicCAS(&cs8[j], 0ull, fpq[q]);
      } else if (k < nrep && fpq[q] && (!SH || owner_of(fpq[q], sh.world) == sh.rank) && eq[q].x == 0ull) {
        cq[q] = atomicCAS(&cs[iq[q]].fp, 0ull, fpq[q]);
      }
    }
#endif
#pragma unroll
    for (int q = 0; q < KC_CLAIM_BATCH; ++q) {
      const int k = k0 + q * CLAIM_TILE;
      if (k >= nrep) break;
      const unsigned long long fp = fpq[q];
      const unsigned int lk = sh_key[k];
      const unsigned int lp = lk >> 5, t = lk & 31;
      const uint64_t pidx = base + tile0 + lp;
      if (SH) {
        const uint32_t o = owner_of(fp, sh.world);
        if (o != sh.rank) {
          atomicOr(&sh_rep[lp], 1u << t);
          atomicAdd(&sh_cnt[(o >> 2) * CLAIM_TILE + lp], 1u << (8 * (o & 3)));
          continue;
        }
      }
      ++probes;
#if KC_CLAIM_PIPE
      int r;
      const uint64_t claim = make_claim(level, okey(pidx, t));
      if (C8) {
        r = fpslots_insert_pair(cs8, nbuckets, fp, iq[q], eq[q], cq[q]);
      } else if (cq[q] == 0ull) {                 // this lane's CAS inserted fp (fingerprints are never ~0)
        if (!FIRST)
          __hip_atomic_store(&cs[iq[q]].nclaim, ~(unsigned long long)claim, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        r = CL_NEW;
      } else if (FIRST) {
        r = claimset_insert_from(cs, nbuckets, fp, iq[q], cq[q] != ~0ull ? cq[q] : eq[q].x);
      } else {
        ulonglong2 e = eq[q];
        if (cq[q] != ~0ull) e = make_ulonglong2(cq[q], 0ull);   // another claimant's fp took the slot first
        r = claimset_claim_store_from(cs, nbuckets, fp, claim, level, iq[q], e);
      }
#else
      const int r = claimset_claim_store_from(cs, nbuckets, fp, make_claim(level, okey(pidx, t)), level,
                                              iq[q], eq[q]);
#endif
      KC_DIAG_OUT(r);
      if (r == CL_NEW)
        atomicOr(&sh_cur[lp], 1u << t);
      else if (r == CL_CUR && !FIRST)
        push_candidate(&sh_rc, tile, rec_fp, rec_lk, fp, lk, sh.ovf, C);
      else if (r == CL_FULL)
        atomicAdd(&C->overflow, 1ull);
    }
  }
  __syncthreads();
  KC_CT(5);
  if (SH && sh.stage)
    // (the parents reloaded from the frontier, or from the states rebuilt above)
    stage_records<M, NT, TLC>(sh, live, fold, counts, DEAL ? (unsigned)(counts >> 56) : (unsigned)threadIdx.x, f,
                              sh_rep, sh_cnt, sh_proj, sh_fp, sh_key, tile,
                              dfr ? reinterpret_cast<const typename M::State*>(df.out) : cur,
                              dfr ? base + tile0 : tile0, base + tile0, C);
  KC_CT(6);
  if (threadIdx.x == 0) rcount[tile] = FIRST ? 0u : sh_rc < (unsigned)CLAIM_RCAP ? sh_rc : (unsigned)CLAIM_RCAP;
  if (live) newmask[i] = sh_cur[threadIdx.x];
  if (FIRST) {
    // the tile's new states (sh_cur is final: the barrier after the claims)
    unsigned int c = live ? (unsigned)__builtin_popcount(sh_cur[threadIdx.x]) : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += (unsigned)__shfl_xor((int)c, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&sh_rc, c);   // (sh_rc is 0: no candidates)
    __syncthreads();
    if (threadIdx.x == 0) {
      sh.ttot[tile] = sh_rc;
      if (sh.csum && sh_rc) atomicAdd(&sh.csum[tile / CSUM_TILES], sh_rc);
    }
  }
  if (SH && live) {
    sh.repmask[i] = sh_rep[threadIdx.x];
    for (uint32_t o = 0; o < sh.world; ++o)
      sh.cnt[(uint64_t)o * n + i] = (uint8_t)((sh_cnt[(o >> 2) * CLAIM_TILE + threadIdx.x] >> (8 * (o & 3))) & 0xffu);
  }
  unsigned long long pw = probes;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) pw += __shfl_down(pw, off, 64);
  if ((threadIdx.x & 63) == 0 && pw) atomicAdd(&stripe(C).probes, pw);
  if (threadIdx.x < A_COUNT) {
    const unsigned int v = act_sum<AS>(sh_act, threadIdx.x);
    if (v) atomicAdd(&stripe(C).act_gen[threadIdx.x], (unsigned long long)v);
  }
  if (dfr) {
    if (threadIdx.x < A_COUNT) {
      const unsigned int v = act_sum<AS>(sh_actd, threadIdx.x);
      if (v) atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)v);
    }
    if (threadIdx.x == 0 && sh_dcand) atomicAdd(&stripe(C).next_cand, sh_dcand);
  }
#ifdef KC_CLAIM_TRACE
  KC_CT(7);
  if (threadIdx.x == 0) {
    atomicAdd(&g_ctrace[0], 1ull);
    for (int k = 1; k < 8; ++k) atomicAdd(&g_ctrace[k], ct[k] - ct[k - 1]);
    atomicMax(&g_ctrace[8], ct[7] - ct[0]);
    atomicMin(&g_ctrace[9], ct[0]);
    atomicMax(&g_ctrace[10], ct[7]);
  }
#endif
#ifdef KC_DIAG
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    unsigned long long v = (outc >> (16 * r)) & 0xffffull;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&stripe(C).claim_out[r], v);
  }
  __syncthreads();
  if (threadIdx.x < 8 && sh_odist[threadIdx.x])
    atomicAdd(&stripe(C).old_dist[threadIdx.x], (unsigned long long)sh_odist[threadIdx.x]);
#endif
#undef KC_DIAG_OUT
}

// A claim displaced the stored ~prev in settle pass A: clear the displaced
// claim's newmask bit when it is this rank's (parent index - base, position),
// and flag the displacer (*flag_at = flag_val).
__device__ __forceinline__ void settle_displace(unsigned long long prev, uint32_t level, const ClaimKeys& rank,
                                                uint64_t base, uint64_t n, uint32_t* __restrict__ newmask,
                                                Counters* __restrict__ C, unsigned int* flag_at,
                                                unsigned int flag_val) {
  const uint64_t pkey = (~prev) & ((1ull << CLAIM_KEY_BITS) - 1);
  if (prev == 0ull || ((~prev) >> CLAIM_KEY_BITS) != level) {
    atomicAdd(&C->overflow, 1ull);               // protocol violation: fail loudly
    return;
  }
  uint64_t pp;
  uint32_t t;
  if (rank.mine(pkey, pp, t)) {
    pp -= base;
    if (pp >= n) {
      atomicAdd(&C->overflow, 1ull);
      return;
    }
    atomicAnd(&newmask[pp], ~(1u << t));
  }
  *flag_at = flag_val;
}

// k_settle_rec<PASS>: one workgroup per claim tile (STORE-claim protocol,
// fpset_dev.h).  PASS 0: every candidate folds its claim into its slot; one
// that lowers the stored claim clears the displaced claim's newmask bit and
// flags itself.  PASS 1 (a later launch): every displacer whose claim is
// still the stored one sets its newmask bit.  Displaced claims always belong
// to this chunk: earlier chunks' claims are smaller and final.  Sharded: a
// displaced claim of another rank (a received record's) has no bit here;
// records re-read their claims themselves (shard.hip).
//
// PASS 1 with tile_total (the engine's default): also the tile's new-state count
// (popcount of its newmask words after pass A, plus this pass's winners),
// the input of k_tile_scan.
// (The body takes the tile index, so the sharded insert can run it in one
// launch with the records' settle pass.)
// One candidate record of tile `tile`.  PASS 0 folds its claim into its
// slot (a displacer flags itself in *lkp); PASS 1 a displacer whose claim is
// still the stored one sets its newmask bit.  Returns 1 for a record it
// processed (PASS 1: 2 for a winner), 0 for one PASS 1 skips.
template <int PASS>
__device__ __forceinline__ int settle_record(uint32_t tile, unsigned long long fp, unsigned int* lkp, uint64_t n,
                                             uint64_t base, ClaimEntry* __restrict__ cs, uint64_t nbuckets,
                                             uint32_t level, uint32_t* __restrict__ newmask, Counters* __restrict__ C,
                                             const ClaimKeys& rank) {
  const unsigned int lk = *lkp;
  if (PASS == 1 && !(lk & CAND_DISPLACER)) return 0;
  const uint64_t tile0 = (uint64_t)tile * CLAIM_TILE;
  const unsigned int lp = (lk >> 5) & (CLAIM_TILE - 1), t = lk & 31;
  const uint64_t claim = make_claim(level, rank.own(base + tile0 + lp, t));
  if (PASS == 0) {
    const unsigned long long prev = claimset_store_claim(cs, nbuckets, fp, claim);
    if (prev < ~claim)                           // displaced ~prev (or found no claim)
      settle_displace(prev, level, rank, base, n, newmask, C, lkp, lk | CAND_DISPLACER);
    return 1;
  }
  if (~claimset_get(cs, nbuckets, fp) == claim) {
    atomicOr(&newmask[tile0 + lp], 1u << t);     // a candidate's bit is never set before
    return 2;
  }
  return 1;
}

template <int PASS>
__device__ __forceinline__ void settle_tile(uint32_t tile, uint64_t n, uint64_t base, ClaimEntry* __restrict__ cs,
                                            uint64_t nbuckets, uint32_t level, const unsigned int* __restrict__ rcount,
                                            const unsigned long long* __restrict__ rec_fp,
                                            unsigned int* __restrict__ rec_lk, uint32_t* __restrict__ newmask,
                                            Counters* __restrict__ C, ClaimKeys rank, uint32_t* __restrict__ tile_total) {
  __shared__ unsigned int sh_tot[CLAIM_TILE / 64];
  const unsigned int cnt = rcount[tile];
  const uint64_t tile0 = (uint64_t)tile * CLAIM_TILE;
  unsigned reads = 0, newc = 0;
  if (PASS == 1 && tile_total) {
    // read before any of this pass's bit sets (the barrier orders them)
    if (tile0 + threadIdx.x < n) newc = (unsigned)__builtin_popcount(newmask[tile0 + threadIdx.x]);
    __syncthreads();
  }
  for (unsigned int k = threadIdx.x; k < cnt; k += CLAIM_TILE) {
    const uint64_t r = (uint64_t)tile * CLAIM_RCAP + k;
    const int v = settle_record<PASS>(tile, rec_fp[r], &rec_lk[r], n, base, cs, nbuckets, level, newmask, C, rank);
    reads += v ? 1u : 0u;
    newc += v == 2 ? 1u : 0u;
  }
  unsigned long long rw = reads;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) rw += __shfl_down(rw, off, 64);
  if ((threadIdx.x & 63) == 0 && rw) atomicAdd(&stripe(C).settles, rw);
  if (PASS == 1 && tile_total) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) newc += __shfl_down(newc, off, 64);
    if ((threadIdx.x & 63) == 0) sh_tot[threadIdx.x >> 6] = newc;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned int t = 0;
#pragma unroll
      for (int w = 0; w < CLAIM_TILE / 64; ++w) t += sh_tot[w];
      tile_total[tile] = t;
    }
  }
}
// The same passes over the chunk's overflow list (after k_settle_rec<PASS>:
// a PASS-1 winner then adds itself to its tile's count).
template <int PASS>
__device__ __forceinline__ void settle_ovf_blocks(uint32_t blk, uint32_t nblk, const CandOvf& ovf, uint64_t n,
                                                  uint64_t base, ClaimEntry* __restrict__ cs, uint64_t nbuckets,
                                                  uint32_t level, uint32_t* __restrict__ newmask,
                                                  Counters* __restrict__ C, ClaimKeys rank,
                                                  uint32_t* __restrict__ tile_total) {
  const unsigned long long c = *ovf.count;
  const uint64_t cnt = c < ovf.cap ? c : ovf.cap;
  if (PASS == 0 && blk == 0 && threadIdx.x == 0 && cnt) atomicAdd(&stripe(C).cand_ovf, (unsigned long long)cnt);
  unsigned long long reads = 0;
  for (uint64_t k = (uint64_t)blk * blockDim.x + threadIdx.x; k < cnt; k += (uint64_t)nblk * blockDim.x) {
    const unsigned int tile = ovf.tile[k];
    const int v = settle_record<PASS>(tile, ovf.fp[k], &ovf.lk[k], n, base, cs, nbuckets, level, newmask, C, rank);
    reads += v ? 1 : 0;
    if (v == 2 && tile_total) atomicAdd(&tile_total[tile], 1u);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) reads += __shfl_down(reads, off, 64);
  if ((threadIdx.x & 63) == 0 && reads) atomicAdd(&stripe(C).settles, reads);
}
template <int PASS>
static __global__ void __launch_bounds__(256)
k_settle_ovf(CandOvf ovf, uint64_t n, uint64_t base, ClaimEntry* __restrict__ cs, uint64_t nbuckets, uint32_t level,
             uint32_t* __restrict__ newmask, Counters* __restrict__ C, ClaimKeys rank,
             uint32_t* __restrict__ tile_total) {
  settle_ovf_blocks<PASS>(blockIdx.x, gridDim.x, ovf, n, base, cs, nbuckets, level, newmask, C, rank, tile_total);
}
constexpr unsigned SETTLE_OVF_GRID = 1024;
// blocks of settle pass A's launch that take the overflow list (pass A needs
// no counts, so its overflow work shares the tiles' launch; pass B's adds to
// the tile counts the tile blocks compute, so it runs in a launch of its own)
constexpr unsigned SETTLE_OVF_BLOCKS = 256;

template <int PASS>
static __global__ void __launch_bounds__(CLAIM_TILE)
k_settle_rec(uint64_t n, uint64_t base, ClaimEntry* __restrict__ cs, uint64_t nbuckets,
             uint32_t level, const unsigned int* __restrict__ rcount,
             const unsigned long long* __restrict__ rec_fp, unsigned int* __restrict__ rec_lk,
             uint32_t* __restrict__ newmask, Counters* __restrict__ C, ClaimKeys rank,
             uint32_t* __restrict__ tile_total = nullptr, uint32_t tiles = 0, CandOvf ovf = CandOvf{}) {
  // PASS 0 launched with tiles + SETTLE_OVF_BLOCKS blocks: the blocks past
  // the tiles settle the overflow list
  if (PASS == 0 && blockIdx.x >= tiles && tiles) {
    settle_ovf_blocks<0>(blockIdx.x - tiles, gridDim.x - tiles, ovf, n, base, cs, nbuckets, level, newmask, C, rank,
                         nullptr);
    return;
  }
  settle_tile<PASS>(blockIdx.x, n, base, cs, nbuckets, level, rcount, rec_fp, rec_lk, newmask, C, rank, tile_total);
}

// Exclusive prefix sum of the tiles' new-state counts (engine default; one
// workgroup): off[t] = sum of tot[0..t), off[T] = the chunk's total (a chunk
// is at most 2^27 parents, so the totals fit u32).  Each thread takes a
// contiguous run of 16-B groups (4 tiles); up to TS_REG groups per thread
// (T <= 65,536 tiles) stay in registers, all their loads in flight at once.
constexpr int TSCAN_THREADS = 1024;
// Marks of a tile scan (the sharded levels): the exclusive prefix at
// positions m_k = k * stride for k = 0 .. nmark - 1, plus at `extra`, go to
// LDS (mark[k], mark[nmark]); k * stride = T reads the total.  nmark <= 16.
struct ScanMarks {
  uint32_t stride = 0, nmark = 0, extra = ~0u;
};
__device__ __forceinline__ void tile_scan_body(const uint32_t* __restrict__ tot, uint32_t T, uint32_t* __restrict__ off,
                                               int reg_ok, const ScanMarks& mk, unsigned int* sh_mark) {
  __shared__ unsigned int sh_w[TSCAN_THREADS / 64];
  const uint32_t G = (T + 3) / 4, per = (G + TSCAN_THREADS - 1) / TSCAN_THREADS;
  const uint32_t b = threadIdx.x * per, e = min(G, b + per);
  const uint4* t4 = reinterpret_cast<const uint4*>(tot);
  auto grp = [&](uint32_t g) {                    // tiles >= T read as 0
    uint4 v = t4[g];
    const uint32_t k = 4 * g;
    if (k + 1 >= T) v.y = 0;
    if (k + 2 >= T) v.z = 0;
    if (k + 3 >= T) v.w = 0;
    return v;
  };
  constexpr uint32_t TS_REG = 16;
  const bool inreg = reg_ok && per <= TS_REG;   // (reg_ok = 0: KC_TSCAN_REG=0, tests the loop path)
  uint4 rv[TS_REG];
  unsigned int sum = 0;
  if (inreg) {
#pragma unroll
    for (uint32_t j = 0; j < TS_REG; ++j) rv[j] = b + j < e ? grp(b + j) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t j = 0; j < TS_REG; ++j) sum += rv[j].x + rv[j].y + rv[j].z + rv[j].w;
  } else {
    for (uint32_t g = b; g < e; ++g) {
      const uint4 v = grp(g);
      sum += v.x + v.y + v.z + v.w;
    }
  }
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  unsigned int incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) sh_w[wv] = incl;
  __syncthreads();
  unsigned int run = incl - sum;
  for (int w = 0; w < wv; ++w) run += sh_w[w];
  uint4* o4 = reinterpret_cast<uint4*>(off);
  auto mark = [&](uint32_t c0, const unsigned int (&ex)[4]) {   // cells c0 .. c0 + 3 start at ex[]
    if (!mk.nmark && mk.extra == ~0u) return;
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t c = c0 + q;
      if (c >= T) break;
      if (c == mk.extra) sh_mark[mk.nmark] = ex[q];
      if (mk.stride && c % mk.stride == 0 && c / mk.stride < mk.nmark) sh_mark[c / mk.stride] = ex[q];
    }
  };
  auto put = [&](uint32_t g, const uint4& v) {
    uint4 r;
    r.x = run;
    r.y = run + v.x;
    r.z = r.y + v.y;
    r.w = r.z + v.z;
    run = r.w + v.w;
    o4[g] = r;
    const unsigned int ex[4] = {r.x, r.y, r.z, r.w};
    mark(4 * g, ex);
  };
  if (inreg) {
#pragma unroll
    for (uint32_t j = 0; j < TS_REG; ++j)
      if (b + j < e) put(b + j, rv[j]);
  } else {
    for (uint32_t g = b; g < e; ++g) put(g, grp(g));
  }
  if (threadIdx.x == TSCAN_THREADS - 1) {
    off[T] = run;
    // marks at T (the total): k * stride == T, or extra == T
    if (mk.extra == T) sh_mark[mk.nmark] = run;
    if (mk.stride && T % mk.stride == 0 && T / mk.stride < mk.nmark) sh_mark[T / mk.stride] = run;
  }
  __syncthreads();
}
// Exclusive prefix sum of the tiles' new-state counts (engine default; one
// workgroup): off[t] = sum of tot[0..t), off[T] = the chunk's total (a chunk
// is at most 2^27 parents, so the totals fit u32).  Each thread takes a
// contiguous run of 16-B groups (4 tiles); up to TS_REG groups per thread
// (T <= 65,536 tiles) stay in registers, all their loads in flight at once.
static __global__ void __launch_bounds__(TSCAN_THREADS)
k_tile_scan(const uint32_t* __restrict__ tot, uint32_t T, uint32_t* __restrict__ off, int reg_ok) {
  tile_scan_body(tot, T, off, reg_ok, ScanMarks{}, nullptr);
}

// The chunk-sum scan (round 6; the engine's first-claim levels): coff =
// exclusive prefix of the CSUM_TILES-tile chunk sums k_claim accumulated
// (coff[C] the total), and the sums zeroed for the next level.  The link
// emit adds a tile's offset inside its chunk from the tile counts.  One
// workgroup, as k_tile_scan, over 64x fewer cells.
static __global__ void __launch_bounds__(TSCAN_THREADS)
k_chunk_scan(uint32_t* __restrict__ csum, uint32_t nchunk, uint32_t* __restrict__ coff, int reg_ok) {
  tile_scan_body(csum, nchunk, coff, reg_ok, ScanMarks{}, nullptr);
  for (uint32_t c = threadIdx.x; c < nchunk; c += TSCAN_THREADS) csum[c] = 0u;
}

// A small chunk's settle pass B over its candidate overflow list and the
// tile scan in one workgroup (round 5): the list of a chunk of <= 2^16
// parents is short (usually empty), so the 1,024-workgroup k_settle_ovf<1>
// launch and k_tile_scan's launch become one.  The overflow winners' tile
// counts are this workgroup's own atomics, visible to its scan after the
// barrier.  (A long list is still settled correctly, only by one workgroup.)
constexpr uint64_t FUSE_OVF_SCAN_MAX = 1ull << 16;
static __global__ void __launch_bounds__(TSCAN_THREADS)
k_ovf_tile_scan(CandOvf ovf, uint64_t n, uint64_t base, ClaimEntry* __restrict__ cs, uint64_t nbuckets,
                uint32_t level, uint32_t* __restrict__ newmask, Counters* __restrict__ C, ClaimKeys rank,
                uint32_t* __restrict__ tile_total, uint32_t T, uint32_t* __restrict__ off, int reg_ok) {
  settle_ovf_blocks<1>(0, 1, ovf, n, base, cs, nbuckets, level, newmask, C, rank, tile_total);
  __syncthreads();
  tile_scan_body(tile_total, T, off, reg_ok, ScanMarks{}, nullptr);
}

// popcount(newmask): the scan's input (new states per parent)
struct NewCount {
  __host__ __device__ __forceinline__ uint32_t operator()(uint32_t m) const {
    return (uint32_t)__builtin_popcount(m);
  }
};

// ABL (diagnostic builds of the same kernel, KC_ABLATE=1, on scratch
// counters): 1 = no plan of the new state (the next level's candidate
// count), 2 = also no invariant check, 3 = also no successor rebuild and no
// state store (parent pointers only).
// SH (the sharded insert's own winners, shard.hip k_shard_emit): `parent`
// takes the parent keys rank << 60 | parent << 16 | position << 8 | action,
// error keys carry the rank, the output starts at offset 0 (chunk_base is
// the records' base there), and there is no outdegree (a rank sees only the
// successors it owns).
template <class M, int ABL, bool SH = false>
__device__ __forceinline__ void emit_body(const typename M::State* __restrict__ cur, uint64_t n, uint64_t base, Flags f,
       const uint32_t* __restrict__ newmask, const uint32_t* __restrict__ offsets,
       typename M::State* __restrict__ next, uint64_t next_base, uint64_t level_gidx, uint64_t next_gidx,
       unsigned long long* __restrict__ parent, uint8_t* __restrict__ ord, int keep_trace,
       Counters* __restrict__ C, const uint32_t* __restrict__ tile_off, uint64_t rank = 0) {
  // offsets: per-parent exclusive offsets; or (tile_off != nullptr) per
  // 256-parent block, the wave bases then come from the block's own counts
  __shared__ unsigned int sh_act[A_COUNT];
  __shared__ unsigned int sh_deg[OUTDEG_BINS];
  __shared__ unsigned long long sh_cand;
  __shared__ unsigned int sh_wtot[4];
  if (threadIdx.x < A_COUNT) sh_act[threadIdx.x] = 0;
  if (threadIdx.x < OUTDEG_BINS) sh_deg[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh_cand = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long cand = 0;
  // Wave-balanced like k_claim: the wave's new states are dealt out 64 per
  // round in order, lane g of a round writes next[obase + g], so the stores
  // of a round are one contiguous run.
  uint32_t mask = 0;
  uint64_t counts = 0;
  uint32_t obase = 0;
  if (i < n) {
    mask = newmask[i];
    if (mask) counts = M::plan(load_state<M>(cur, i), f).counts;
  }
  const int cnt = __builtin_popcount(mask);
  if (!SH && i < n) atomicAdd(&sh_deg[cnt < OUTDEG_BINS ? cnt : OUTDEG_BINS - 1], 1u);
  const int lane = (int)(threadIdx.x & 63);
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  const int wtot = __shfl(incl, 63, 64);
  const int excl = incl - cnt;
  if (tile_off) {
    if (lane == 0) sh_wtot[threadIdx.x >> 6] = (unsigned int)wtot;
    __syncthreads();
    obase = tile_off[blockIdx.x];
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) obase += sh_wtot[w];
  } else if (wtot) {
    obase = __shfl(i < n ? offsets[i] - (uint32_t)excl : 0u, 0, 64);
  }
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
    const uint64_t pidx = base + pi;
    const uint64_t o = (SH ? 0ull : C->chunk_base) + obase + (uint64_t)g;
    if (!SH && keep_trace) {
      parent[next_gidx + o] = level_gidx + pidx;
      ord[next_gidx + o] = (uint8_t)t;
    }
    if (ABL >= 3) continue;
    const typename M::State s = load_state<M>(cur, pi);
    const typename M::Plan pl{pc, 0, -1, -1};
    int slot, j;
    M::locate(pl, t, slot, j);
    typename M::State x;
    M::apply(s, slot, j, f, x);
    store_state<M>(next, o - next_base, x);   // next_base: the StateQueue run starts at o = next_base
    const int act = M::slot_action(s, slot);
    const uint64_t key = (SH ? rank << 60 : 0ull) | (pidx << 16) | ((uint64_t)t << 8);
    if (SH) parent[next_gidx + o] = key | (uint64_t)act;
    if (ABL < 2 && M::check(x, f.inv_mask) >= 0) atomicMin(&C->err_key, key | E_INVARIANT);
    atomicAdd(&sh_act[act], 1u);
    if (ABL == 0) {
      const typename M::Plan px = M::plan(x, f);
      cand += (unsigned long long)px.total;
    }
  }
  // wave reduction of the candidate count, then one LDS atomic per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cand += __shfl_down(cand, off, 64);
  if ((threadIdx.x & 63) == 0 && cand) atomicAdd(&sh_cand, cand);
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_act[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_act[threadIdx.x]);
  if (!SH && threadIdx.x < OUTDEG_BINS && sh_deg[threadIdx.x])
    atomicAdd(&stripe(C).outdeg[threadIdx.x], (unsigned long long)sh_deg[threadIdx.x]);
  if (threadIdx.x == 0 && sh_cand) atomicAdd(&stripe(C).next_cand, sh_cand);
}

// Deferred frontier's emit (DeferArgs): per new state only its link — the
// trace entry (global parent index, position) with keep_trace, and/or a
// level-local parent index << 8 | position (`link`, when the trace is off or
// in host memory) — plus the outdegree histogram.
// No state is loaded or built here; the next level's k_claim rebuilds them.
// Entries at or past `cap` (the host's estimate of the level's new states)
// are not written and set DF_CAPACITY: the host re-runs on the exact path.
// Same wave-balanced dealing as emit_body: lane g of a round writes entry
// obase + g, so a round's stores are contiguous.
// A workgroup takes EMIT_TPB consecutive 256-parent tiles (round 6): all
// their masks and tile offsets are loaded at once, then the tiles are dealt
// one after another — one dependent round trip per workgroup instead of one
// per tile (a tile's work is a few stores; its time was its round trips).
constexpr int EMIT_TPB = 4;
static __global__ void __launch_bounds__(256)
k_emit_links(uint64_t n, uint64_t base, const uint32_t* __restrict__ newmask, const uint32_t* __restrict__ tile_off,
             uint64_t level_gidx, uint64_t next_gidx, unsigned long long* __restrict__ parent,
             uint8_t* __restrict__ ord, unsigned long long* __restrict__ link, uint64_t cap,
             Counters* __restrict__ C, const uint32_t* __restrict__ ttot = nullptr) {
  // tile offsets: tile_off[tile] (k_tile_scan), or with ttot (k_chunk_scan)
  // tile_off[chunk] + the tile counts of its chunk before it (each wave
  // scans the chunk's <= 64 counts; a workgroup's tiles share one chunk)
  static_assert(CSUM_TILES == 64 && CSUM_TILES % EMIT_TPB == 0, "a workgroup's tiles in one chunk");
  __shared__ unsigned int sh_deg[OUTDEG_BINS * ACT_STRIPES];   // (striped by lane, as k_claim's counters)
  __shared__ unsigned int sh_wtot[EMIT_TPB][4];
  const uint64_t cb = C->chunk_base;
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  const uint64_t T = (n + 255) / 256, tile0 = (uint64_t)blockIdx.x * EMIT_TPB;
  uint32_t mask[EMIT_TPB], toff[EMIT_TPB];
  uint32_t cnt_in_chunk = 0, coff = 0;
  if (ttot) {
    const uint64_t c0 = tile0 / CSUM_TILES * CSUM_TILES;
    cnt_in_chunk = c0 + lane < T ? ttot[c0 + lane] : 0u;
    coff = tile_off[tile0 / CSUM_TILES];
  }
#pragma unroll
  for (int k = 0; k < EMIT_TPB; ++k) {
    const uint64_t tile = tile0 + k;
    const uint64_t i = tile * 256 + threadIdx.x;
    mask[k] = i < n ? newmask[i] : 0u;
    toff[k] = !ttot && tile < T ? tile_off[tile] : 0u;
  }
  if (ttot) {
    uint32_t x = cnt_in_chunk;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t v = (uint32_t)__shfl_up((int)x, off, 64);
      if (lane >= off) x += v;
    }
    const int j0 = (int)(tile0 % CSUM_TILES);
#pragma unroll
    for (int k = 0; k < EMIT_TPB; ++k)
      toff[k] = coff + (uint32_t)__shfl((int)(x - cnt_in_chunk), j0 + k, 64);
  }
  if (threadIdx.x < OUTDEG_BINS * ACT_STRIPES) sh_deg[threadIdx.x] = 0;
  __syncthreads();
  int excl[EMIT_TPB], wtot[EMIT_TPB];
#pragma unroll
  for (int k = 0; k < EMIT_TPB; ++k) {
    const uint64_t i = ((uint64_t)blockIdx.x * EMIT_TPB + k) * 256 + threadIdx.x;
    const int cnt = __builtin_popcount(mask[k]);
    if (i < n) atomicAdd(&sh_deg[(cnt < OUTDEG_BINS ? cnt : OUTDEG_BINS - 1) * ACT_STRIPES + (threadIdx.x & (ACT_STRIPES - 1))], 1u);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    wtot[k] = __shfl(incl, 63, 64);
    excl[k] = incl - cnt;
    if (lane == 0) sh_wtot[k][wv] = (unsigned int)wtot[k];
  }
  __syncthreads();
  bool over = false;
#pragma unroll
  for (int k = 0; k < EMIT_TPB; ++k) {
    uint64_t obase = cb + toff[k];
    for (int w = 0; w < wv; ++w) obase += sh_wtot[k][w];
    const uint64_t wave0 = ((uint64_t)blockIdx.x * EMIT_TPB + k) * 256 + (uint64_t)(threadIdx.x - lane);
    for (int r = 0; r < wtot[k]; r += 64) {
      const int g = r + lane;
      int p = 0;                                       // last lane with excl <= g
#pragma unroll
      for (int b = 32; b > 0; b >>= 1) {
        const int e = __shfl(excl[k], p + b, 64);
        if (e <= g) p += b;
      }
      int q = g - __shfl(excl[k], p, 64);
      uint32_t m = (uint32_t)__shfl((int)mask[k], p, 64);
      if (g >= wtot[k]) continue;
      for (; q > 0; --q) m &= m - 1;
      const int t = __ffs(m) - 1;
      const uint64_t pidx = base + wave0 + (uint64_t)p;
      const uint64_t o = obase + (uint64_t)g;
      if (o >= cap) {
        over = true;
        continue;
      }
      if (link) link[o] = (pidx << 8) | (uint64_t)t;
      if (parent) {
        parent[next_gidx + o] = level_gidx + pidx;
        ord[next_gidx + o] = (uint8_t)t;
      }
    }
  }
  if (over) atomicOr(&C->defer_flags, DF_CAPACITY);
  __syncthreads();
  if (threadIdx.x < OUTDEG_BINS) {
    const unsigned int v = act_sum(sh_deg, threadIdx.x);
    if (v) atomicAdd(&stripe(C).outdeg[threadIdx.x], (unsigned long long)v);
  }
}

// Pinned to 8 waves per SIMD (64 VGPRs; unpinned it took 68 = 7 waves):
// NP=2 emit 31.6 -> 28.7 ms on the same box (profiles/r02o_ab2.txt).
template <class M, int ABL = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_emit(const typename M::State* __restrict__ cur, uint64_t n, uint64_t base, Flags f,
       const uint32_t* __restrict__ newmask, const uint32_t* __restrict__ offsets,
       typename M::State* __restrict__ next, uint64_t next_base, uint64_t level_gidx, uint64_t next_gidx,
       unsigned long long* __restrict__ parent, uint8_t* __restrict__ ord, int keep_trace,
       Counters* __restrict__ C, const uint32_t* __restrict__ tile_off = nullptr) {
  emit_body<M, ABL>(cur, n, base, f, newmask, offsets, next, next_base, level_gidx, next_gidx, parent, ord,
                    keep_trace, C, tile_off);
}
}  // namespace kc
