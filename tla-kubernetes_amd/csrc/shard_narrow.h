// shard_narrow.h — device-driven narrow levels of the fingerprint-owner-
// sharded BFS (gfx950).  The sharded loop's counterpart of engine_narrow.h.
//
// A counted level of the sharded loop (shard.hip, shard_driver.hip) costs
// ~12 launches, two host synchronisations, an all-gather and a sized
// all-to-all, whatever its width: ~77 us per level at one rank, 185 levels
// for NP=2, 124 (all narrow) for Model_1.  While every rank's frontier is
// small (<= SN_MAX states) the levels run here instead, with no host in the
// loop: the host enqueues SN_BATCH levels at a time and synchronises once.
//
// The exchange of a narrow level has a FIXED size, so it can be enqueued
// before anyone knows the counts: each rank sends every peer one slot of
// slot_cap + 1 records; record 0 is a header carrying the slot's record
// count and the sender's status (its previous level's new-state count and
// error key, and whether it can run this level narrow).  Every rank reads
// the same R headers (its own from its control block) and takes the same
// decision, before any ClaimSet write:
//   some rank reports an error        -> SN_ERROR
//   the level is globally empty       -> SN_DONE
//   some rank cannot run it narrow    -> SN_STOP (too wide, no room, a slot
//                                        overflowed, max_levels, a failure)
//   otherwise the level runs.
// A level that does not run has changed nothing but scratch (its own
// successors went into the level table, the records into the slots): the
// host hands it to the counted path, whose all-gather then reports the
// error or the end exactly as before.  Every rank enqueues the same
// exchanges whatever its device state, so the collectives always match.
//
// Per level L (the kernels return at once once the control block is
// inactive):
//   k_sn_expand   lanes (parent, sub): plan (Assert / deadlock keys, per-
//                 action counts held until the level runs), successors,
//                 fingerprints (owner projection OWN = 1).  Own successors go
//                 into the level table (min key = rank << 18 | parent << 5 |
//                 t: the order of the counted path's claims); the others are
//                 marked per parent and counted per owner (8-bit counts).
//   k_sn_pack     (R > 1) lane = parent: the slot headers, and the records
//                 bit-packed (record.h) at positions from per-owner sums.
//   (exchange: RCCL grouped send/recv of whole slots, enqueued by the host)
//   k_sn_recv     (R > 1) the decision; received records into the table.
//   k_sn_claim    the decision (authoritative); every copy holding its
//                 fingerprint's minimum key inserts it into the ClaimSet:
//                 new unless an earlier level stored it.
//   k_sn_emit     new states (own first, in parent order; then the
//                 records', by sender and slot order), parent keys,
//                 invariants, per-action distinct counts, the next level's
//                 successor count; the last workgroup to finish closes the
//                 level.
// Three launches per level at R = 1, five at R > 1 (plus the exchange).
// No kernel waits for another workgroup of its own grid, so any number of
// ranks' kernels may share the GPU (the emulated ranks do).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_kernels.h"
#include "engine_narrow.h"
#include "record.h"

namespace kc {

constexpr int SN_MAX = 8192;                                 // parents of a narrow level, per rank
constexpr int SN_THREADS = 256;
constexpr int SN_SUB = 8;                                    // k_sn_expand lanes per parent
constexpr int SN_XWG = SN_MAX * SN_SUB / SN_THREADS;
constexpr int SN_ESUB = 4;                                   // k_sn_claim lanes per parent
constexpr int SN_CWG = SN_MAX * SN_ESUB / SN_THREADS;
constexpr int SN_PWG = SN_MAX / SN_THREADS;                  // lane = parent kernels
constexpr int SN_EMSUB = 4;                                  // k_sn_emit lanes per parent (own new states)
constexpr int SN_EWG = SN_MAX * SN_EMSUB / SN_THREADS;
constexpr uint64_t SN_CAND_MAX = 32768;                      // own successors of a narrow level
constexpr int SN_MAX_R = 16;
constexpr uint32_t SN_SLOT_MAX = 4096;                       // records per peer slot (upper bound)
constexpr uint32_t SN_SLOT_DEFAULT = 2048;
constexpr int SN_LT_BITS = 17;                               // level table: <= 47% full at R = 15
constexpr uint64_t SN_LT = 1ull << SN_LT_BITS;
constexpr int SN_NLT = 3;
constexpr int SN_LT_PROBES = 256;
constexpr int SN_BATCH = 32;                                 // levels enqueued per host sync
static_assert((uint64_t)SN_MAX * 32 < (1u << 20), "keys: parent 13 bits, t 5 bits");
static_assert(SN_EWG + SN_MAX_R * SN_SLOT_MAX / SN_THREADS < 512 &&
              SN_CAND_MAX + (uint64_t)SN_MAX_R * SN_SLOT_MAX < (1u << 20), "k_sn_emit's arrival word");

enum SNReason : int { SN_RUN = 0, SN_ERROR = 1, SN_DONE = 2, SN_STOP = 3 };

// The control block of one rank (device memory; the host fills it before a
// batch, the kernels advance it level by level).
struct SNCtl {
  uint32_t active;            // 1 while levels run here
  int32_t reason;             // SNReason once inactive
  uint32_t level;             // the level about to be expanded (1 = Init)
  uint32_t world, rank;
  uint32_t slot_cap;          // records per peer slot
  uint32_t stop_level;        // do not expand a level >= this (0: none)
  uint32_t levels;            // levels run in this batch
  uint32_t fail;              // set by the host (a failure on this rank): stop at the next level
  uint32_t k1_over;           // k_sn_expand: an over-wide state or a full level table
  uint64_t n;                 // local width of `level`
  uint64_t level_gidx;        // parent-key index of its first state
  uint64_t cand;              // successors of its states
  uint64_t room, buf_cap, par_cap;
  uint64_t new_total;         // new states of this batch
  uint64_t sent, sent_total;  // records this level sends (k_sn_pack); of the levels run
  // by level parity: [L & 1] = level L's errors (its parents' Assert /
  // deadlock keys, its successors' invariant keys); sent as the status of
  // level L in the headers of level L + 1
  unsigned long long err[2];
  uint64_t hdr[4];            // what k_sn_pack put in this level's headers (count 0)
  uint64_t gw;                // k_sn_claim: the level's global width
  unsigned long long close_acc;   // k_sn_emit: workgroups done << 55 | new states << 35 | successors
  unsigned int act_pend[A_COUNT]; // the level's per-action successor counts, kept if it runs
  uint64_t lwidths[KC_MAX_LEVELS];    // [k] = local new states of the k-th level of the batch
  uint64_t gwidths[KC_MAX_LEVELS];    // [k] = global width of the level the k-th step expanded
};

struct SNScratch {
  NarrowLT lt[SN_NLT][SN_LT];        // by level mod 3: k_sn_emit of L clears L + 2's
  unsigned long long pcnt[SN_MAX];   // plan slot counts of each parent
  unsigned char ptot[SN_MAX];        // its successor total (<= MAXSUCC)
  uint32_t hidx[SN_MAX * 32];        // table slot of each own successor
  uint32_t rmask[SN_MAX];            // successors owned by other ranks
  uint32_t cnt4[SN_MAX_R / 4][SN_MAX];     // per parent, remote successors per owner: 4 x 8 bits
  uint32_t soff[SN_MAX_R][SN_MAX];         // per owner and parent: first slot position
  uint32_t newmask[SN_MAX], offsets[SN_MAX];
  uint32_t rhidx[SN_MAX_R][SN_SLOT_MAX];   // table slot of each received record
  uint32_t isnew[SN_MAX_R][SN_SLOT_MAX], ioff[SN_MAX_R][SN_SLOT_MAX];
};

__host__ __device__ __forceinline__ uint32_t sn_key(uint32_t rank, uint64_t parent, uint32_t t) {
  return (rank << 18) | ((uint32_t)parent << 5) | t;
}
// claim key of the counted path's record claims (shard.hip record_ckey)
__device__ __forceinline__ uint64_t sn_record_ckey(uint64_t key) {
  return ((key >> 60) << CLAIM_RANK_SHIFT) | (((key >> 16) & 0xffffffffull) << 8) | ((key >> 8) & 0xff);
}

// This rank cannot run `level` narrow (the host applies the same rule).
__host__ __device__ __forceinline__ bool sn_local_stop(const SNCtl& c) {
  const uint64_t in = (uint64_t)(c.world - 1) * c.slot_cap;     // records it may receive
  return c.fail || c.n > (uint64_t)SN_MAX || c.cand > SN_CAND_MAX ||
         (c.stop_level && c.level >= c.stop_level) || c.cand + in > c.buf_cap || c.cand + in > c.room ||
         c.level_gidx + c.n + c.cand + in + 1 > c.par_cap;
}

__device__ __forceinline__ uint64_t sn_slot_words(uint32_t cap, int rw) { return (uint64_t)(cap + 1) * rw; }

// The decision of level `level` from this rank's own status and the peers'
// headers (identical on every rank).  *bad: a header of another level (a
// protocol fault: the run fails loudly).
// This rank's own status is what k_sn_pack put in its headers (ctl->hdr);
// at R = 1 (no pack, no headers) it is computed here the same way.
template <int RW>
__device__ __forceinline__ int sn_decide(const SNCtl* __restrict__ ctl, const uint64_t* __restrict__ recv,
                                         uint32_t world, uint32_t rank, uint32_t cap, uint32_t level,
                                         uint64_t* gnew_out, bool* bad) {
  uint64_t gerr, gnew;
  bool stop;
  if (world == 1) {
    gerr = ctl->err[(level - 1) & 1];
    gnew = ctl->n;
    stop = sn_local_stop(*ctl) || ctl->k1_over;
  } else {
    gerr = ctl->hdr[3];
    gnew = ctl->hdr[2];
    stop = (ctl->hdr[1] & 1) != 0;
  }
  *bad = false;
  for (uint32_t s = 0; s < world; ++s) {
    if (s == rank) continue;
    const uint64_t* h = recv + s * sn_slot_words(cap, RW);
    const uint64_t w1 = h[1];
    if ((w1 >> 8) != (uint64_t)level) {
      *bad = true;
      stop = true;
      continue;
    }
    stop |= (w1 & 1) != 0;
    gnew += h[2];
    gerr = h[3] < gerr ? h[3] : gerr;
  }
  *gnew_out = gnew;
  if (gerr != ~0ull) return SN_ERROR;
  if (gnew == 0) return SN_DONE;
  return stop ? SN_STOP : SN_RUN;
}

// Enter fingerprint fp with order key `key` into a level table (minimum
// key kept as the maximum complement); the slot, or -1 past SN_LT_PROBES.
__device__ __forceinline__ int64_t sn_enter(NarrowLT* __restrict__ lt, uint64_t fp, uint32_t key) {
  uint64_t h = (fp * 0xd6e8feb86659fd93ull) >> (64 - SN_LT_BITS);
  for (int q = 0; q < SN_LT_PROBES; ++q) {
    const unsigned long long e = atomicCAS(&lt[h].fp, 0ull, (unsigned long long)fp);
    if (e == 0ull || e == fp) {
      atomicMax(&lt[h].nkey, ~key);
      return (int64_t)h;
    }
    h = (h + 1) & (SN_LT - 1);
  }
  return -1;
}

__device__ __forceinline__ uint32_t sn_block_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) lds[wv] = x;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (uint32_t k = 0; k < nw; ++k) {
    const uint32_t t = lds[k];
    if (k < wv) before += t;
    total += t;
  }
  __syncthreads();
  return before + x - v;
}

// The host marks a failed rank: its next level stops every rank.
static __global__ void k_sn_fail(SNCtl* __restrict__ ctl) {
  if (threadIdx.x == 0) ctl->fail = 1;
}

// grid SN_XWG x SN_THREADS; lane g: parent g / SN_SUB, successors
// t = g % SN_SUB (+ SN_SUB ...)
template <class M>
__global__ void __launch_bounds__(SN_THREADS)
k_sn_expand(const typename M::State* __restrict__ bufA, const typename M::State* __restrict__ bufB, Flags f,
            int check_deadlock, uint32_t lev, SNCtl* __restrict__ ctl, SNScratch* __restrict__ sc) {
  using State = typename M::State;
  const uint64_t g = (uint64_t)blockIdx.x * SN_THREADS + threadIdx.x;
  const uint64_t i = g / SN_SUB;
  const int sub = (int)(g % SN_SUB);
  const State* __restrict__ cur = (lev & 1) ? bufB : bufA;
  if (!ctl->active) return;
  // clear level L + 2's table (level L - 1 used it; the stores overlap the
  // rest of the kernel)
  {
    NarrowLT* __restrict__ other = sc->lt[(lev + 2) % SN_NLT];
    for (uint64_t h = g; h < SN_LT; h += (uint64_t)SN_XWG * SN_THREADS)
      *reinterpret_cast<ulonglong2*>(&other[h]) = make_ulonglong2(0ull, 0ull);
  }
  if (sn_local_stop(*ctl)) return;   // (the headers report the stop)
  const uint64_t n = ctl->n;
  const uint32_t world = ctl->world, rank = ctl->rank, level = ctl->level;
  __shared__ unsigned int sh_act[A_COUNT];
  if (threadIdx.x < A_COUNT) sh_act[threadIdx.x] = 0;
  __syncthreads();
  NarrowLT* __restrict__ lt = sc->lt[lev % SN_NLT];
  const bool live = i < n;
  uint32_t rm = 0, oc[SN_MAX_R / 4] = {0u, 0u, 0u, 0u};
  bool over = false;
  if (live) {
    const State s = load_state<M>(cur, i);
    const typename M::Plan pl = M::plan(s, f);
    if (sub == 0) {
      sc->pcnt[i] = pl.counts;
      sc->ptot[i] = (unsigned char)(pl.total < M::MAXSUCC ? pl.total : M::MAXSUCC);
      const uint64_t kb = ((uint64_t)rank << 60) | (i << 16);
      if (pl.fail_pos >= 0)
        atomicMin(&ctl->err[level & 1], kb | ((uint64_t)pl.fail_pos << 8) | E_ASSERT);
      else if (pl.total == 0 && check_deadlock)
        atomicMin(&ctl->err[level & 1], kb | E_DEADLOCK);
#pragma unroll
      for (int slot = 0; slot < M::NSLOT; ++slot) {
        const int c = (int)((pl.counts >> (6 * slot)) & 63);
        if (c) atomicAdd(&sh_act[M::slot_action(s, slot)], (unsigned)c);
      }
      if (pl.total > M::MAXSUCC) over = true;      // (the counted path reports it)
    }
    const int tot = pl.total < M::MAXSUCC ? pl.total : M::MAXSUCC;
    const uint64_t fold = M::fp_fold(s);
    const uint32_t proj = M::owner_proj(s);
    for (int t = sub; t < tot; t += SN_SUB) {
      int slot, j, who;
      M::locate(pl, t, slot, j);
      State x;
      M::apply(s, slot, j, f, x, who);
      const uint64_t fp = M::template fingerprint_succ<1>(s, fold, x, who, proj);
      const uint32_t o = owner_of(fp, world);
      if (o == rank) {
        const int64_t h = sn_enter(lt, fp, sn_key(rank, i, (uint32_t)t));
        if (h < 0) over = true;
        else sc->hidx[i * 32 + t] = (uint32_t)h;
      } else {
        rm |= 1u << t;
        oc[o >> 2] += 1u << (8 * (o & 3));
      }
    }
  }
  // the parent's SN_SUB lanes are adjacent lanes of one wave
#pragma unroll
  for (int off = 1; off < SN_SUB; off <<= 1) {
    rm |= (uint32_t)__shfl_xor((int)rm, off, 64);
#pragma unroll
    for (int k = 0; k < SN_MAX_R / 4; ++k) oc[k] += (uint32_t)__shfl_xor((int)oc[k], off, 64);
  }
  if (live && sub == 0) {
    sc->rmask[i] = rm;
#pragma unroll
    for (int k = 0; k < SN_MAX_R / 4; ++k)
      if ((uint32_t)(4 * k) < world) sc->cnt4[k][i] = oc[k];
  }
  if (over) atomicOr(&ctl->k1_over, 1u);
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_act[threadIdx.x]) atomicAdd(&ctl->act_pend[threadIdx.x], sh_act[threadIdx.x]);
}

// (R > 1) lane = parent: the slot headers (workgroup 0) and the records of
// its remote successors.  Every workgroup sums the per-owner counts of all
// parents and of the parents before its own (at most 8192: cheaper than a
// separate scan launch), so the positions follow (owner, parent, t) order
// without any workgroup waiting for another.
template <class M>
__global__ void __launch_bounds__(SN_THREADS)
k_sn_pack(const typename M::State* __restrict__ bufA, const typename M::State* __restrict__ bufB, Flags f,
          uint32_t lev, SNCtl* __restrict__ ctl, const SNScratch* __restrict__ sc, uint64_t* __restrict__ send) {
  using State = typename M::State;
  constexpr int RW = Record<M>::RW;
  if (!ctl->active) return;
  const uint64_t n = ctl->n;
  const uint32_t world = ctl->world, cap = ctl->slot_cap, level = ctl->level;
  const uint64_t rank = ctl->rank;
  const bool stop0 = sn_local_stop(*ctl) || ctl->k1_over;
  __shared__ uint32_t sh_base[SN_MAX_R], sh_tot[SN_MAX_R];
  __shared__ uint32_t lds[SN_THREADS / 64];
  if (threadIdx.x < SN_MAX_R) sh_base[threadIdx.x] = sh_tot[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t first = (uint64_t)blockIdx.x * SN_THREADS;
  const uint32_t nk = (world + 3) / 4;
  if (!stop0) {
    uint32_t b[SN_MAX_R] = {}, t[SN_MAX_R] = {};
    for (uint64_t j = threadIdx.x; j < n; j += SN_THREADS) {
#pragma unroll
      for (uint32_t k = 0; k < SN_MAX_R / 4; ++k) {
        if (k >= nk) break;
        const uint32_t w = sc->cnt4[k][j];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t v = (w >> (8 * q)) & 0xffu;
          t[4 * k + q] += v;
          if (j < first) b[4 * k + q] += v;
        }
      }
    }
#pragma unroll
    for (uint32_t o = 0; o < SN_MAX_R; ++o) {
      if (o < world && t[o]) atomicAdd(&sh_tot[o], t[o]);
      if (o < world && b[o]) atomicAdd(&sh_base[o], b[o]);
    }
  }
  __syncthreads();
  bool stop = stop0;
  uint64_t sent = 0;
  for (uint32_t o = 0; o < world; ++o) {
    if (o == rank) continue;
    if (sh_tot[o] > cap) stop = true;                // a slot overflowed: the counted path takes the level
    sent += sh_tot[o];
  }
  if (blockIdx.x == 0) {
    const uint64_t w1 = ((uint64_t)level << 8) | (stop ? 1ull : 0ull), e = ctl->err[(level - 1) & 1];
    if (threadIdx.x == 0) {
      ctl->hdr[0] = 0;
      ctl->hdr[1] = w1;
      ctl->hdr[2] = n;
      ctl->hdr[3] = e;
      ctl->sent = sent;
    }
    if (threadIdx.x < world && threadIdx.x != rank) {
      uint64_t* h = send + threadIdx.x * sn_slot_words(cap, RW);
      h[0] = stop ? 0ull : (uint64_t)sh_tot[threadIdx.x];
      h[1] = w1;
      h[2] = n;
      h[3] = e;
#pragma unroll
      for (int k = 4; k < RW; ++k) h[k] = 0;
    }
  }
  if (stop) return;
  // the lane's first position in each owner's slot
  const uint64_t i = first + threadIdx.x;
  const bool live = i < n;
  uint32_t offs[SN_MAX_R] = {};
  for (uint32_t o = 0; o < world; ++o) {
    if (o == rank || sh_tot[o] == 0) continue;        // (uniform)
    const uint32_t v = live ? (sc->cnt4[o >> 2][i] >> (8 * (o & 3))) & 0xffu : 0u;
    uint32_t total;
    const uint32_t e = sn_block_scan(v, lds, total);
#pragma unroll
    for (uint32_t k = 0; k < SN_MAX_R; ++k)
      if (k == o) offs[k] = sh_base[o] + e;
  }
  if (!live) return;
  uint32_t rm = sc->rmask[i];
  if (!rm) return;
  const State* __restrict__ cur = (lev & 1) ? bufB : bufA;
  const State s = load_state<M>(cur, i);
  const typename M::Plan pl{sc->pcnt[i], 0, -1, -1};
  const uint64_t fold = M::fp_fold(s);
  const uint32_t proj = M::owner_proj(s);
  for (; rm; rm &= rm - 1) {
    const int t = __ffs(rm) - 1;
    int slot, j, who;
    M::locate(pl, t, slot, j);
    State x;
    M::apply(s, slot, j, f, x, who);
    const uint64_t fp = M::template fingerprint_succ<1>(s, fold, x, who, proj);
    const uint32_t o = owner_of(fp, world);
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t k = 0; k < SN_MAX_R; ++k)
      if (k == o) { pos = offs[k]; offs[k] = pos + 1; }
    if (pos >= cap) continue;                         // (cannot happen: the totals fit)
    uint64_t w[RW];
    record_pack<M>(x, (rank << 60) | (i << 16) | ((uint64_t)t << 8) | (uint64_t)M::slot_action(s, slot), w);
    ulonglong2* v = reinterpret_cast<ulonglong2*>(send + o * sn_slot_words(cap, RW) + (1 + (uint64_t)pos) * RW);
#pragma unroll
    for (int k = 0; k < RW / 2; ++k) v[k] = make_ulonglong2(w[2 * k], w[2 * k + 1]);
  }
}

// (R > 1) lane (sender, slot position): received records into the table
template <class M>
__global__ void __launch_bounds__(SN_THREADS)
k_sn_recv(uint32_t lev, const SNCtl* __restrict__ ctl, SNScratch* __restrict__ sc, const uint64_t* __restrict__ recv,
          Counters* __restrict__ C) {
  using State = typename M::State;
  constexpr int RW = Record<M>::RW;
  if (!ctl->active) return;
  const uint32_t world = ctl->world, rank = ctl->rank, cap = ctl->slot_cap, level = ctl->level;
  __shared__ int sh_d;
  if (threadIdx.x == 0) {
    uint64_t gnew;
    bool bad;
    sh_d = sn_decide<RW>(ctl, recv, world, rank, cap, level, &gnew, &bad);
  }
  __syncthreads();
  if (sh_d != SN_RUN) return;
  const uint64_t g = (uint64_t)blockIdx.x * SN_THREADS + threadIdx.x;
  const uint32_t s = (uint32_t)(g / cap), k = (uint32_t)(g % cap);
  if (s >= world || s == rank) return;
  const uint64_t* slot = recv + s * sn_slot_words(cap, RW);
  if (k >= slot[0]) return;             // (k < cap: a count past cap reads as cap)
  const ulonglong2* v = reinterpret_cast<const ulonglong2*>(slot + (1 + (uint64_t)k) * RW);
  uint64_t r[RW];
#pragma unroll
  for (int q = 0; q < RW / 2; ++q) {
    const ulonglong2 e = v[q];
    r[2 * q] = e.x;
    r[2 * q + 1] = e.y;
  }
  State x;
  uint64_t key;
  record_unpack<M>(r, x, key);
  const uint64_t p = (key >> 16) & 0xffffffffull, t = (key >> 8) & 0xff;
  int64_t h = -1;
  if (p < (uint64_t)SN_MAX && t < 32)       // (else not a record of a narrow level)
    h = sn_enter(sc->lt[lev % SN_NLT], M::template fingerprint<1>(x), sn_key(s, p, (uint32_t)t));
  if (h < 0) atomicAdd(&C->overflow, 1ull);            // fails the run loudly; no table slot
  sc->rhidx[s][k] = h < 0 ? ~0u : (uint32_t)h;
}

// grid SN_CWG + ceil(world * cap / SN_THREADS): the decision; then the
// level's first copy of every fingerprint this rank owns claims it
template <class M>
__global__ void __launch_bounds__(SN_THREADS)
k_sn_claim(uint32_t lev, SNCtl* __restrict__ ctl, SNScratch* __restrict__ sc, const uint64_t* __restrict__ recv,
           ClaimEntry* __restrict__ cs, uint64_t nslots, Counters* __restrict__ C, uint32_t csh = 1) {
  constexpr int RW = Record<M>::RW;
  // (csh: slot i's fp word is word i << csh — 0 for the compact set of the
  // first-claim mode, DevClaimSet::compact, which has no claim words and
  // even home slots)
  unsigned long long* const csw = reinterpret_cast<unsigned long long*>(cs);
  if (!ctl->active) return;
  const uint64_t n = ctl->n;
  const uint32_t world = ctl->world, rank = ctl->rank, cap = ctl->slot_cap, level = ctl->level;
  __shared__ int sh_d;
  if (threadIdx.x == 0) {
    uint64_t gnew;
    bool bad;
    const int d = sn_decide<RW>(ctl, recv, world, rank, cap, level, &gnew, &bad);
    sh_d = d;
    if (blockIdx.x == 0) {
      if (bad) atomicAdd(&C->overflow, 1ull);
      if (d != SN_RUN) {
        ctl->active = 0;
        ctl->reason = d;
      } else {
        ctl->gw = gnew;
        ctl->err[(level + 1) & 1] = ~0ull;         // (the next level's; its status went out in this level's headers)
        ctl->sent_total += ctl->sent;
      }
    }
  }
  __syncthreads();
  const int d = sh_d;
  if (blockIdx.x == 0 && threadIdx.x < A_COUNT) {      // the level's generated counts: kept if it runs
    const unsigned int v = ctl->act_pend[threadIdx.x];
    if (v && d == SN_RUN) atomicAdd(&C->s[0].act_gen[threadIdx.x], (unsigned long long)v);
    ctl->act_pend[threadIdx.x] = 0;
  }
  if (d != SN_RUN) return;
  const NarrowLT* __restrict__ lt = sc->lt[lev % SN_NLT];
  const uint32_t succ_level = level + 1;
  auto insert = [&](uint64_t fp, uint64_t ckey) -> bool {
    uint64_t ix = csh ? bucket_of(fp, nslots) : fpslots_home(fp, nslots);
    for (uint64_t q = 0; q < nslots; ++q) {
      const unsigned long long o = atomicCAS(&csw[ix << csh], 0ull, (unsigned long long)fp);
      if (o == 0ull) {
        if (csh) csw[(ix << 1) + 1] = ~make_claim(succ_level, ckey);
        return true;
      }
      if (o == fp) return false;
      ix = (ix + 1 == nslots) ? 0 : ix + 1;
    }
    atomicAdd(&C->overflow, 1ull);
    return false;
  };
  unsigned long long probes = 0;
  if (blockIdx.x < (unsigned)SN_CWG) {
    const uint64_t g = (uint64_t)blockIdx.x * SN_THREADS + threadIdx.x;
    const uint64_t i = g / SN_ESUB;
    const int sub = (int)(g % SN_ESUB);
    const bool live = i < n;
    uint32_t mine = 0;
    if (live) {
      const int tot = sc->ptot[i];
      const uint32_t rm = sc->rmask[i];
      // the lane's own first copies (an earlier copy of the level holds the
      // others; k_sn_expand wrote every own successor's slot): their first
      // ClaimSet CASes issued back to back, then linear probing for the few
      // that met another fingerprint
      constexpr int PT = 32 / SN_ESUB;
      uint64_t fps[PT], ixs[PT];
      unsigned long long os[PT];
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const int t = sub + k * SN_ESUB;
        fps[k] = 0;
        if (t < tot && !((rm >> t) & 1u)) {
          const uint32_t hx = sc->hidx[i * 32 + t];
          if (hx < SN_LT) {
            const NarrowLT e = lt[hx];
            if (~e.nkey == sn_key(rank, i, (uint32_t)t)) fps[k] = e.fp;
          }
        }
        ixs[k] = fps[k] ? (csh ? bucket_of(fps[k], nslots) : fpslots_home(fps[k], nslots)) : 0ull;
        os[k] = fps[k] ? atomicCAS(&csw[ixs[k] << csh], 0ull, (unsigned long long)fps[k]) : 0ull;
      }
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const uint64_t fp = fps[k];
        if (!fp) continue;
        const int t = sub + k * SN_ESUB;
        ++probes;
        uint64_t ix = ixs[k];
        unsigned long long o = os[k];
        uint64_t q = 1;
        for (; o != 0ull && o != fp && q < nslots; ++q) {
          ix = (ix + 1 == nslots) ? 0 : ix + 1;
          o = atomicCAS(&csw[ix << csh], 0ull, (unsigned long long)fp);
        }
        if (o == 0ull) {
          if (csh)
            csw[(ix << 1) + 1] = ~make_claim(succ_level, ((uint64_t)rank << CLAIM_RANK_SHIFT) | (i << 8) | (uint64_t)t);
          mine |= 1u << t;
        } else if (o != fp) {
          atomicAdd(&C->overflow, 1ull);               // a full table
        }
      }
    }
#pragma unroll
    for (int off = 1; off < SN_ESUB; off <<= 1) mine |= (uint32_t)__shfl_xor((int)mine, off, 64);
    if (live && sub == 0) sc->newmask[i] = mine;
  } else {
    const uint64_t g = (uint64_t)(blockIdx.x - SN_CWG) * SN_THREADS + threadIdx.x;
    const uint32_t s = (uint32_t)(g / cap), k = (uint32_t)(g % cap);
    if (s < world && s != rank) {
      const uint64_t* slot = recv + s * sn_slot_words(cap, RW);
      if (k < slot[0]) {
        const uint64_t key = slot[(1 + (uint64_t)k) * RW];
        const uint32_t hx = sc->rhidx[s][k];
        uint32_t w = 0;
        if (hx < SN_LT && ~lt[hx].nkey == sn_key(s, (key >> 16) & 0xffffffffull, (uint32_t)((key >> 8) & 0xff))) {
          const NarrowLT e = lt[hx];
          ++probes;
          w = insert(e.fp, sn_record_ckey(key)) ? 1u : 0u;
        }
        sc->isnew[s][k] = w;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off, 64);
  if ((threadIdx.x & 63) == 0 && probes) atomicAdd(&stripe(C).probes, probes);
}

// grid SN_EWG + ceil(world * cap / SN_THREADS): the new states (own in
// parent order, then the records' by sender and slot order), each at its
// position: a workgroup sums the new-state counts before its own first (at
// most 8192 parents and 15 x 4096 records: cheaper than a scan launch).
// Own new states: SN_EMSUB adjacent lanes per parent, lane `sub` taking the
// parent's new states of rank sub, sub + SN_EMSUB, ... (a narrow level's
// time is one lane's serial chain: measured 11.4 us per Model_1 level with
// one lane per parent).  The last workgroup to finish closes the level.
template <class M>
__global__ void __launch_bounds__(SN_THREADS)
k_sn_emit(typename M::State* __restrict__ bufA, typename M::State* __restrict__ bufB, Flags f, uint32_t lev,
          SNCtl* __restrict__ ctl, SNScratch* __restrict__ sc, const uint64_t* __restrict__ recv,
          unsigned long long* __restrict__ pkeys, Counters* __restrict__ C) {
  using State = typename M::State;
  constexpr int RW = Record<M>::RW;
  if (!ctl->active) return;
  const uint64_t n = ctl->n, level_gidx = ctl->level_gidx;
  const uint32_t world = ctl->world, rank = ctl->rank, cap = ctl->slot_cap, level = ctl->level;
  const State* __restrict__ cur = (lev & 1) ? bufB : bufA;
  State* __restrict__ nxt = (lev & 1) ? bufA : bufB;
  const uint64_t next_gidx = level_gidx + n;
  __shared__ unsigned int sh_dist[A_COUNT];
  __shared__ unsigned long long sh_cand;
  __shared__ uint32_t sh_sum[2];
  __shared__ uint32_t lds[SN_THREADS / 64];
  if (threadIdx.x < A_COUNT) sh_dist[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    sh_cand = 0;
    sh_sum[0] = sh_sum[1] = 0;
  }
  __syncthreads();
  const bool own = blockIdx.x < (unsigned)SN_EWG;
  const uint64_t rfirst = own ? 0 : (uint64_t)(blockIdx.x - SN_EWG) * SN_THREADS;   // flattened record index
  auto rec_new = [&](uint64_t g) -> uint32_t {          // 1 if flattened record g is a new state
    const uint32_t s = (uint32_t)(g / cap), k = (uint32_t)(g % cap);
    if (s >= world || s == rank) return 0u;
    return k < recv[s * sn_slot_words(cap, RW)] ? sc->isnew[s][k] : 0u;
  };
  // [0]: new states before this workgroup's first; [1] (records): all own new states
  {
    const uint64_t pend = own ? (uint64_t)blockIdx.x * (SN_THREADS / SN_EMSUB) : n;
    uint32_t a = 0, r = 0;
    for (uint64_t j = threadIdx.x; j < pend && j < n; j += SN_THREADS) a += (uint32_t)__builtin_popcount(sc->newmask[j]);
    if (!own)
      for (uint64_t g = threadIdx.x; g < rfirst; g += SN_THREADS) r += rec_new(g);
    if (a) atomicAdd(&sh_sum[own ? 0 : 1], a);
    if (r) atomicAdd(&sh_sum[0], r);
  }
  __syncthreads();
  unsigned long long cand = 0;
  uint32_t wnew = 0;                                  // this workgroup's new states
  auto emit = [&](const State& x, uint64_t o, uint64_t key, uint64_t act) {
    store_state<M>(nxt, o, x);
    pkeys[next_gidx + o] = key;
    if (M::check(x, f.inv_mask) >= 0) atomicMin(&ctl->err[level & 1], (key & ~0xffull) | E_INVARIANT);
    if (act < (uint64_t)A_COUNT) atomicAdd(&sh_dist[act], 1u);
    cand += (unsigned long long)M::plan(x, f).total;
  };
  if (own) {
    const uint64_t gl = (uint64_t)blockIdx.x * SN_THREADS + threadIdx.x;
    const uint64_t i = gl / SN_EMSUB;
    const uint32_t sub = (uint32_t)(gl % SN_EMSUB);
    uint32_t m = i < n ? sc->newmask[i] : 0u;
    uint32_t total;
    // the parent's count once (its lane 0), its base to all its lanes
    const uint32_t e0 = sn_block_scan(sub == 0 ? (uint32_t)__builtin_popcount(m) : 0u, lds, total);
    const uint32_t e = (uint32_t)__shfl((int)e0, (int)((threadIdx.x & 63u) & ~(uint32_t)(SN_EMSUB - 1)), 64);
    wnew = total;
    for (uint32_t k = 0; k < sub && m; ++k) m &= m - 1;      // skip to the lane's first rank
    if (m) {
      const State s = load_state<M>(cur, i);
      const typename M::Plan pl{sc->pcnt[i], 0, -1, -1};
      uint64_t o = (uint64_t)sh_sum[0] + e + sub;
      while (m) {
        const int t = __ffs(m) - 1;
        int slot, j;
        M::locate(pl, t, slot, j);
        State x;
        M::apply(s, slot, j, f, x);
        const uint64_t act = (uint64_t)M::slot_action(s, slot);
        emit(x, o, ((uint64_t)rank << 60) | (i << 16) | ((uint64_t)t << 8) | act, act);
        for (int k = 0; k < SN_EMSUB && m; ++k) m &= m - 1;  // the lane's next rank
        o += SN_EMSUB;
      }
    }
  } else {
    const uint64_t g = rfirst + threadIdx.x;
    const uint32_t w = rec_new(g);
    uint32_t total;
    const uint32_t e = sn_block_scan(w, lds, total);
    wnew = total;
    if (w) {
      const uint32_t s = (uint32_t)(g / cap), k = (uint32_t)(g % cap);
      const ulonglong2* v = reinterpret_cast<const ulonglong2*>(recv + s * sn_slot_words(cap, RW) + (1 + (uint64_t)k) * RW);
      uint64_t r[RW];
#pragma unroll
      for (int q = 0; q < RW / 2; ++q) {
        const ulonglong2 ev = v[q];
        r[2 * q] = ev.x;
        r[2 * q + 1] = ev.y;
      }
      State x;
      uint64_t key;
      record_unpack<M>(r, x, key);
      emit(x, (uint64_t)sh_sum[1] + sh_sum[0] + e, key, key & 0xff);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cand += __shfl_down(cand, off, 64);
  if ((threadIdx.x & 63) == 0 && cand) atomicAdd(&sh_cand, cand);
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_dist[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_dist[threadIdx.x]);
  // the last workgroup to get here closes the level: every wave's atomics
  // complete first (s_waitcnt), then one returning add carries this
  // workgroup's new states and successor count with the arrival count
  // (arrivals 9 bits | new states 20 | successors 35)
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const unsigned long long mine = (1ull << 55) | ((unsigned long long)wnew << 35) | sh_cand;
  const unsigned long long prev = atomicAdd(&ctl->close_acc, mine);
  if ((prev >> 55) == gridDim.x - 1) {
    const unsigned long long all = prev + mine;
    const uint64_t nn = (all >> 35) & ((1ull << 20) - 1);
    const unsigned long long cnext = all & ((1ull << 35) - 1);
    const uint32_t lv = ctl->levels;
    if (lv < (uint32_t)KC_MAX_LEVELS) {
      ctl->lwidths[lv] = nn;
      ctl->gwidths[lv] = ctl->gw;
    }
    ctl->close_acc = 0;
    ctl->levels = lv + 1;
    ctl->new_total += nn;
    ctl->room = ctl->room > nn ? ctl->room - nn : 0;
    ctl->level_gidx = next_gidx;
    ctl->n = nn;
    ctl->cand = cnext;
    ctl->level = level + 1;
    ctl->k1_over = 0;
  }
}

}  // namespace kc
