// shard.hip — fingerprint-owner-sharded BFS stages for one GPU of R (one
// process per GPU; kubecheck/distributed.py drives the levels and does the
// exchange with RCCL all-to-all through torch.distributed).
//
// owner(fp) = floor(fp * R / 2^63) (fps are uniform in [1, 2^63)), the top
// bits of the fingerprint as in TLC's MultiFPSet [ext-TLC].  Per level:
//   expand : the engine's k_claim in shard mode (engine_kernels.h): LDS tile
//            dedup, then every tile representative this rank owns claims its
//            fp in the local ClaimSet shard (STORE-claim + newmask protocol);
//            the others are marked and counted per owner -> one exclusive
//            scan over the owner-major count matrix
//   pack   : k_shard_pack writes one record per remote representative
//            {state words, key} into the caller's send buffer, grouped by
//            owner, each group in (parent, t) order
//   (all-to-all by the caller)
//   insert : received records claim their fp in the same ClaimSet
//            (k_rec_claim, same protocol), then settle pass A (local and
//            record candidates fold their claims; a displaced local claim
//            loses its newmask bit), pass B (local displacers, record
//            inserters and displacers re-read their claim), two scans, and
//            the emit of the winners — this rank's own successors first (in
//            parent order), then the records' (in receive order) — with parent
//            keys (TLC trace file), invariant checks and counters.
// With R = 1 nothing is sent and the level is the single-GPU engine's.
// Keys: rank << 60 | parent index << 16 | successor position << 8 | low byte
// (action id in records and parent keys, ErrKind in error keys); the
// ClaimSet claim orders them by (rank, parent, position), so the same minimum
// is taken everywhere and the result does not depend on arrival order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kubecheck.h"
#include "coldset.h"
#include "engine_kernels.h"
#include "engine_spill.h"
#include "engine_util.h"
#include "fpset_host.h"
#include "kc_common.h"
#include "record.h"
#include "shard.h"
#include "shard_narrow.h"

namespace kc {

constexpr uint64_t KEY_INIT = 0xFull << 60;   // parent key of an Init state (| init index)

template <class M>
__device__ __forceinline__ uint64_t record_key(const Record<M>* __restrict__ in, uint64_t i) {
  return in[i].w[0];
}


template <class M>
__global__ void __launch_bounds__(256)
k_shard_pack(const typename M::State* __restrict__ cur, uint64_t n, Flags f, uint32_t world,
             uint64_t rank, const uint32_t* __restrict__ off /* [world][n], one exclusive scan */,
             const uint32_t* __restrict__ repmask,
             Record<M>* __restrict__ out, const uint32_t* __restrict__ gpos /* TLC order: G per parent */) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t mask = repmask[i];
  if (!mask) return;
  const typename M::State s = load_state<M>(cur, i);
  const typename M::Plan pl = M::plan(s, f);
  const uint64_t fold = M::fp_fold(s);
  uint32_t c[16] = {};
  for (; mask; mask &= mask - 1) {
    const int t = __ffs(mask) - 1;
    int slot, j;
    M::locate(pl, t, slot, j);
    typename M::State x;
    int who;
    M::apply(s, slot, j, f, x, who);
    const uint64_t fp = M::template fingerprint_succ<1>(s, fold, x, who, M::owner_proj(s));
    const uint32_t o = owner_of(fp, world);
    uint32_t r = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
      if (k == o) { r = c[k]; c[k] = r + 1; }
    const uint64_t pos = (uint64_t)off[(uint64_t)o * n + i] + r;   // owner-major scan
    uint64_t w[Record<M>::RW];
    record_pack<M>(x, (rank << 60) | ((gpos ? (uint64_t)gpos[i] : i) << 16) | ((uint64_t)t << 8) |
                          (uint64_t)M::slot_action(s, slot), w);
    ulonglong2* v = reinterpret_cast<ulonglong2*>(out + pos);
#pragma unroll
    for (int k = 0; k < Record<M>::RW / 2; ++k) v[k] = make_ulonglong2(w[2 * k], w[2 * k + 1]);
  }
}

// Records per owner from the owner-major exclusive scan of cnt[world][n]
// (8-bit counts: a parent has at most 32 successors).
// Owner totals (world > 1; 0 at world 1) into tot and straight into pinned
// host memory, with the level head (error key, overflow flags): what the
// host reads after expand, with no copy launches.
// (device-scope loads: the last emit workgroup reads what the others' atomics wrote)
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void head_to_host(const Counters* __restrict__ C, unsigned long long* __restrict__ h) {
  h[0] = ld_agent(&C->err_key);
  h[1] = ld_agent(&C->chunk_base);
  h[2] = ld_agent(&C->overflow);
  h[3] = ld_agent(&C->batch_used);
  h[4] = ld_agent(&C->cand_total);
  h[5] = ld_agent(&C->level_new);
  h[7] = ld_agent(&C->defer_flags);
  h[9] = ld_agent(&C->defer_err);
}
// Level head reset at the start of expand (one launch instead of fills),
// with the candidate overflow list's count and the staging cursor.
__global__ void k_head_reset(Counters* __restrict__ C, unsigned long long* __restrict__ ovf_count,
                             unsigned long long* __restrict__ stage_cur) {
  if (threadIdx.x == 0) {
    C->err_key = ~0ull;
    C->chunk_base = 0;
    C->overflow = 0;
    C->batch_used = 0;
    C->emit_done = 0;
    C->defer_flags = 0;
    C->defer_err = ~0ull;
    *ovf_count = 0;
    *stage_cur = 0;
  }
}
// row != nullptr (ShardBase::expand_dev): the all-gather row too, in device
// memory: totals, status_new, status_err (level 1: an Init-state invariant
// key, 0x12, found by expand takes the status slot, as Group::run does), and
// the failure word.
// (thread o < 16: owner o's total v; thread 0 also the head and the status
// words.  status_err takes the deferred frontier's invariant key, an error
// of the level before, as the materialising emit would have reported it.)
__device__ __forceinline__ void owner_row(uint32_t o, uint64_t v, uint32_t world, uint64_t* __restrict__ tot,
                                          const Counters* __restrict__ C, uint64_t* __restrict__ host_tot,
                                          unsigned long long* __restrict__ host_head, uint64_t* __restrict__ row,
                                          uint64_t status_new, uint64_t status_err, int level1, uint64_t init_err) {
  if (o == 0) {
    head_to_host(C, host_head);
    if (row) {
      uint64_t se = status_err;
      const uint64_t de = C->defer_err;
      if (de < se) se = de;
      // an Init state's invariant violation is level 1's error, whatever
      // level 1's expansion found (an Assert of a lower-index Init state
      // must not hide it)
      if (level1 && init_err != ~0ull) se = init_err;
      row[world] = status_new;
      row[world + 1] = se;
      // failure word: a full table or an over-wide state found by this
      // level's claims, so every rank leaves the loop together (the host
      // overwrites it with its own failure code, if any)
      row[world + 2] = (C->overflow || C->batch_used) ? 1ull : 0ull;
    }
  }
  if (o >= 16) return;
  tot[o] = v;
  host_tot[o] = v;
  if (row && o < world) row[o] = v;
}
__device__ __forceinline__ void owner_totals(const uint32_t* __restrict__ off, const uint8_t* __restrict__ cnt,
                                             uint64_t n, uint32_t world, uint64_t* __restrict__ tot,
                                             const Counters* __restrict__ C, uint64_t* __restrict__ host_tot,
                                             unsigned long long* __restrict__ host_head, uint64_t* __restrict__ row,
                                             uint64_t status_new, uint64_t status_err, int level1,
                                             uint64_t init_err) {
  const uint32_t o = threadIdx.x;
  uint64_t v = 0;
  if (world > 1 && o < world && n > 0) {
    const uint64_t end = (o + 1 < world) ? (uint64_t)off[(uint64_t)(o + 1) * n]
                                         : (uint64_t)off[(uint64_t)world * n - 1] + cnt[(uint64_t)world * n - 1];
    v = end - off[(uint64_t)o * n];
  }
  owner_row(o, v, world, tot, C, host_tot, host_head, row, status_new, status_err, level1, init_err);
}
__global__ void k_owner_totals(const uint32_t* __restrict__ off, const uint8_t* __restrict__ cnt,
                               uint64_t n, uint32_t world, uint64_t* __restrict__ tot,
                               const Counters* __restrict__ C, uint64_t* __restrict__ host_tot,
                               unsigned long long* __restrict__ host_head, uint64_t* __restrict__ row,
                               uint64_t status_new, uint64_t status_err, int level1, uint64_t init_err) {
  owner_totals(off, cnt, n, world, tot, C, host_tot, host_head, row, status_new, status_err, level1, init_err);
}

// Owner-major exclusive scan of the tiles' per-owner record counts (k_claim
// with staging: tcnt[o][tile], world x T cells) -> toff, the send-buffer
// position of each (owner, tile) segment; the owner totals then go to the
// all-gather row and the host as in owner_totals.  One workgroup (the
// engine's k_tile_scan body), instead of a device scan over world x n
// per-parent cells and a totals launch.
__global__ void __launch_bounds__(TSCAN_THREADS)
k_owner_tscan(const uint32_t* __restrict__ tcnt, uint32_t T, uint32_t world, uint32_t* __restrict__ toff,
              uint64_t* __restrict__ tot, const Counters* __restrict__ C, uint64_t* __restrict__ host_tot,
              unsigned long long* __restrict__ host_head, uint64_t* __restrict__ row, uint64_t status_new,
              uint64_t status_err, int level1, uint64_t init_err) {
  __shared__ unsigned int sh_mark[17];
  const uint32_t cells = world * T;
  tile_scan_body(tcnt, cells, toff, 1, ScanMarks{T, world, cells}, sh_mark);
  if (threadIdx.x < 64) {
    const uint32_t o = threadIdx.x;
    const uint64_t v = o < world ? (uint64_t)(sh_mark[o + 1 < world ? o + 1 : world] - sh_mark[o]) : 0ull;
    owner_row(o, world > 1 ? v : 0ull, world, tot, C, host_tot, host_head, row, status_new, status_err, level1,
              init_err);
  }
}
// The same over the owner x chunk sums (round 6, ShardArgs::ocsum): world x
// C cells (C = ceil(T / CSUM_TILES)) instead of world x T; coff[o][chunk] is
// the send-buffer position of the chunk's first record of owner o, and the
// sums are zeroed for the next level.  k_shard_gather adds a tile's offset
// inside its chunk.
__global__ void __launch_bounds__(TSCAN_THREADS)
k_owner_cscan(uint32_t* __restrict__ ocsum, uint32_t C_, uint32_t world, uint32_t* __restrict__ coff,
              uint64_t* __restrict__ tot, const Counters* __restrict__ C, uint64_t* __restrict__ host_tot,
              unsigned long long* __restrict__ host_head, uint64_t* __restrict__ row, uint64_t status_new,
              uint64_t status_err, int level1, uint64_t init_err) {
  __shared__ unsigned int sh_mark[17];
  const uint32_t cells = world * C_;
  tile_scan_body(ocsum, cells, coff, 1, ScanMarks{C_, world, cells}, sh_mark);
  for (uint32_t c = threadIdx.x; c < cells; c += TSCAN_THREADS) ocsum[c] = 0u;
  if (threadIdx.x < 64) {
    const uint32_t o = threadIdx.x;
    const uint64_t v = o < world ? (uint64_t)(sh_mark[o + 1 < world ? o + 1 : world] - sh_mark[o]) : 0ull;
    owner_row(o, world > 1 ? v : 0ull, world, tot, C, host_tot, host_head, row, status_new, status_err, level1,
              init_err);
  }
}
// The staged records into the send buffer (pack without re-expansion): one
// workgroup per tile moves its segment, owner by owner, to toff[o][tile]
// (chunked: coff[o][chunk] + the tile counts of owner o before it in its
// chunk, one wave prefix per owner).
template <class M>
__global__ void __launch_bounds__(256)
k_shard_gather(const Record<M>* __restrict__ stage, const unsigned long long* __restrict__ stoff,
               const uint32_t* __restrict__ tcnt, const uint32_t* __restrict__ toff, uint32_t T, uint32_t world,
               Record<M>* __restrict__ out, int chunked) {
  constexpr int U = Record<M>::RW / 2;     // 16-B units per record
  __shared__ uint32_t sh_n[16], sh_src[16], sh_dst[16];
  const uint32_t tile = blockIdx.x;
  const unsigned long long b = stoff[tile];      // (loaded with the counts: one round trip less)
  if (!chunked) {
    if (threadIdx.x == 0) {
      uint32_t acc = 0;
      for (uint32_t o = 0; o < world; ++o) {
        const uint32_t c = tcnt[(uint64_t)o * T + tile];
        sh_n[o] = c;
        sh_src[o] = acc;
        sh_dst[o] = toff[(uint64_t)o * T + tile];
        acc += c;
      }
    }
  } else if (threadIdx.x < 64) {
    const uint32_t lane = threadIdx.x, c0 = tile / CSUM_TILES * CSUM_TILES, j = tile - c0;
    const uint32_t nC = (T + CSUM_TILES - 1) / CSUM_TILES;
    uint32_t v[16], base[16];
#pragma unroll
    for (uint32_t o = 0; o < 16; ++o) {          // (world <= 15) every owner's counts and chunk base at once
      v[o] = o < world && c0 + lane < T ? tcnt[(uint64_t)o * T + c0 + lane] : 0u;
      base[o] = o < world ? toff[(uint64_t)o * nC + tile / CSUM_TILES] : 0u;
    }
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t o = 0; o < 16; ++o) {
      if (o >= world) break;
      uint32_t x = v[o];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, off, 64);
        if (lane >= (uint32_t)off) x += y;
      }
      if (lane == j) {
        sh_n[o] = v[o];
        sh_src[o] = acc;
        sh_dst[o] = base[o] + x - v[o];
      }
      acc += (uint32_t)__shfl((int)v[o], (int)j, 64);
    }
  }
  __syncthreads();
  if (b == ~0ull) return;
  const ulonglong2* src = reinterpret_cast<const ulonglong2*>(stage + b);
  ulonglong2* dst = reinterpret_cast<ulonglong2*>(out);
  for (uint32_t o = 0; o < world; ++o) {
    const uint32_t units = sh_n[o] * U;
    const ulonglong2* s = src + (uint64_t)sh_src[o] * U;
    ulonglong2* d = dst + (uint64_t)sh_dst[o] * U;
    for (uint32_t u = threadIdx.x; u < units; u += blockDim.x) d[u] = s[u];
  }
}

// 8-bit per-owner counts widened for the owner-major scan
struct Widen8 {
  __host__ __device__ __forceinline__ uint32_t operator()(uint8_t v) const { return v; }
};

// Record flags: 0 = out, 1 = candidate, 2 = inserted its fp, 3 = displacer.
enum : unsigned int { RF_OUT = 0, RF_CAND = 1, RF_INSERTER = 2, RF_DISPLACER = 3 };

template <class M>
__global__ void __launch_bounds__(256)
k_rec_claim(const Record<M>* __restrict__ in, uint64_t n, ClaimEntry* __restrict__ cs,
            uint64_t nslots, uint32_t level, unsigned long long* __restrict__ rfp,
            unsigned int* __restrict__ flag, Counters* __restrict__ C, int tlc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long probes = 0;
  if (i < n) {
    typename M::State x;
    uint64_t key;
    load_record<M>(in, i, x, key);
    const uint64_t fp = M::template fingerprint<1>(x);
    rfp[i] = fp;
    const int r = claimset_claim_store(cs, nslots, fp, make_claim(level, record_ckey(key, tlc)), level);
    if (r == CL_FULL) atomicAdd(&C->overflow, 1ull);
    flag[i] = r == CL_NEW ? RF_INSERTER : (r == CL_CUR ? RF_CAND : RF_OUT);
    probes = 1;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off, 64);
  if ((threadIdx.x & 63) == 0 && probes) atomicAdd(&stripe(C).probes, probes);
}

// First-claim mode (cfg.first_claim; ShardT::first_): a received record is
// new iff its CAS inserts the fingerprint — no claim word, no candidates, no
// settle passes (a copy this rank's own k_claim inserted at expand, or an
// earlier record's, makes it old).  isnew[i] directly, and each block's
// winners into rtot[blk] (the record half of k_win_scan's input).
// (Two records per lane, their loads, probes and CASes issued together,
// measured slower at R = 8: Σ over the ranks 23.3 -> 26.5 ms, r06z — half
// the workgroups on the small levels.)
template <class M>
__global__ void __launch_bounds__(256)
k_rec_claim_first(const Record<M>* __restrict__ in, uint64_t n, ClaimEntry* __restrict__ cs, uint64_t nslots,
                  uint32_t* __restrict__ isnew, uint32_t* __restrict__ rtot, Counters* __restrict__ C,
                  int compact) {
  __shared__ unsigned int sh_rw[4];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t w = 0;
  if (i < n) {
    typename M::State x;
    uint64_t key;
    load_record<M>(in, i, x, key);
    const uint64_t fp = M::template fingerprint<1>(x);
    unsigned long long* const w8 = reinterpret_cast<unsigned long long*>(cs);
    const uint64_t b = compact ? fpslots_home(fp, nslots) : bucket_of(fp, nslots);
    const int r = compact ? fpslots_insert_pair(w8, nslots, fp, b, fpslots_first(w8, b))
                          : claimset_insert_from(cs, nslots, fp, b, cs[b].fp);
    if (r == CL_FULL) atomicAdd(&C->overflow, 1ull);
    w = r == CL_NEW ? 1u : 0u;
    isnew[i] = w;
  }
  const unsigned long long bw = __ballot(w != 0);
  const unsigned long long bp = __ballot(i < n);
  if ((threadIdx.x & 63) == 0) {
    sh_rw[threadIdx.x >> 6] = (unsigned)__popcll(bw);
    if (bp) atomicAdd(&stripe(C).probes, (unsigned long long)__popcll(bp));
  }
  __syncthreads();
  if (threadIdx.x == 0) rtot[blockIdx.x] = sh_rw[0] + sh_rw[1] + sh_rw[2] + sh_rw[3];
}

// PASS 0: candidates fold their claims (a displaced local claim loses its
// newmask bit, the displacer is flagged); PASS 1: inserters and displacers
// win iff the stored claim is still theirs.
// PASS 1 with rtot: the block's winners (the record half of k_win_scan's input).
template <class M, int PASS>
__device__ __forceinline__ void rec_settle(uint64_t blk, const Record<M>* __restrict__ in, uint64_t n,
                                           ClaimEntry* __restrict__ cs, uint64_t nslots, uint32_t level,
                                           const ClaimKeys& rank, const unsigned long long* __restrict__ rfp,
                                           unsigned int* __restrict__ flag, uint32_t* __restrict__ newmask,
                                           uint64_t nlocal, uint32_t* __restrict__ isnew, Counters* __restrict__ C,
                                           uint32_t* __restrict__ rtot) {
  const uint64_t i = blk * 256 + threadIdx.x;
  if (PASS == 0) {
    if (i >= n) return;
    const unsigned int fl = flag[i];
    if (fl != RF_CAND) return;
    const uint64_t claim = make_claim(level, record_ckey(record_key<M>(in, i), rank.gpos != nullptr));
    const unsigned long long prev = claimset_store_claim(cs, nslots, rfp[i], claim);
    if (prev < ~claim) settle_displace(prev, level, rank, 0, nlocal, newmask, C, &flag[i], RF_DISPLACER);
  } else {
    uint32_t w = 0;
    if (i < n) {
      const unsigned int fl = flag[i];
      if (fl >= RF_INSERTER) {
        const uint64_t claim = make_claim(level, record_ckey(record_key<M>(in, i), rank.gpos != nullptr));
        w = ~claimset_get(cs, nslots, rfp[i]) == claim ? 1u : 0u;
      }
      isnew[i] = w;
    }
    if (rtot) {
      __shared__ unsigned int sh_rw[4];
      const unsigned long long b = __ballot(w != 0);
      if ((threadIdx.x & 63) == 0) sh_rw[threadIdx.x >> 6] = (unsigned)__popcll(b);
      __syncthreads();
      if (threadIdx.x == 0) rtot[blk] = sh_rw[0] + sh_rw[1] + sh_rw[2] + sh_rw[3];
    }
  }
}
// One settle pass over this rank's own claim tiles (blocks [0, tiles)), the
// received records (the next rblocks) and the tiles' candidate overflow list
// (the blocks after those), in one launch: the passes of the three commute
// (atomicMax claims; a displaced candidate has no bit; with no per-tile
// counts here, overflow winners set their bits like tile winners).  Pass A
// also resets the level's error key for the emits.
// wtot != nullptr (PASS 1, the tile-count path): the own tiles' new-state
// counts go to wtot[0, tiles) and the record blocks' winners to
// wtot[tiles, tiles + rblocks) — k_win_scan's input — and the launch has no
// overflow-list blocks: their pass B adds to the tile counts afterwards
// (k_settle_ovf<1>), as the engine's does, so no winner is counted twice.
template <class M, int PASS>
__global__ void __launch_bounds__(256)
k_settle_both(uint32_t tiles, uint32_t rblocks, uint64_t n_local, ClaimEntry* __restrict__ cs, uint64_t nslots,
              uint32_t level, ClaimKeys rank, const unsigned int* __restrict__ rcount,
              const unsigned long long* __restrict__ rec_fp, unsigned int* __restrict__ rec_lk,
              uint32_t* __restrict__ newmask, const Record<M>* __restrict__ in, uint64_t n,
              const unsigned long long* __restrict__ rfp, unsigned int* __restrict__ flag,
              uint32_t* __restrict__ isnew, Counters* __restrict__ C, CandOvf ovf, uint32_t* __restrict__ wtot) {
  static_assert(CLAIM_TILE == 256, "one block size for both halves");
  if (PASS == 0 && blockIdx.x == 0 && threadIdx.x == 0) C->err_key = ~0ull;   // (nothing before the emits sets it)
  const uint32_t tb = tiles;
  if (blockIdx.x < tb) {
    settle_tile<PASS>(blockIdx.x, n_local, 0, cs, nslots, level, rcount, rec_fp, rec_lk, newmask, C, rank,
                      PASS == 1 ? wtot : nullptr);
  } else if (blockIdx.x < tb + rblocks) {
    rec_settle<M, PASS>(blockIdx.x - tb, in, n, cs, nslots, level, rank, rfp, flag, newmask, n_local, isnew, C,
                        PASS == 1 && wtot ? wtot + tiles : nullptr);
  } else {
    settle_ovf_blocks<PASS>(blockIdx.x - tb - rblocks, gridDim.x - tb - rblocks, ovf, n_local, 0, cs, nslots,
                            level, newmask, C, rank, nullptr);
  }
}
// Positions of the level's new states (the tile-count path): one scan over
// [own tiles' counts | record blocks' winners] -> woff; chunk_base = this
// rank's own new states (the records' emit base), level_new = all.
__global__ void __launch_bounds__(TSCAN_THREADS)
// (it also resets the level's error key for the emits — expand's Assert /
// deadlock keys were read from its own head copy; in the deterministic mode
// settle pass A did this already, first-claim mode runs no settle pass)
k_win_scan(const uint32_t* __restrict__ wtot, uint32_t tiles, uint32_t rblocks, uint32_t* __restrict__ woff,
           Counters* __restrict__ C) {
  __shared__ unsigned int sh_mark[4];
  const uint32_t cells = tiles + rblocks;
  tile_scan_body(wtot, cells, woff, 1, ScanMarks{cells, 2, tiles}, sh_mark);
  if (threadIdx.x == 0) {
    C->chunk_base = sh_mark[2];
    C->level_new = sh_mark[1];
    C->err_key = ~0ull;
  }
}
constexpr unsigned SHARD_OVF_BLOCKS = 256;
// A small level (<= FUSE_OVF_SCAN_MAX own parents): the overflow list's
// pass B and k_win_scan in one workgroup (engine_kernels.h k_ovf_tile_scan)
__global__ void __launch_bounds__(TSCAN_THREADS)
k_ovf_win_scan(CandOvf ovf, uint64_t n_local, ClaimEntry* __restrict__ cs, uint64_t nslots, uint32_t level,
               uint32_t* __restrict__ newmask, Counters* __restrict__ C, ClaimKeys rank, uint32_t* __restrict__ wtot,
               uint32_t tiles, uint32_t rblocks, uint32_t* __restrict__ woff) {
  settle_ovf_blocks<1>(0, 1, ovf, n_local, 0, cs, nslots, level, newmask, C, rank, wtot);
  __syncthreads();
  __shared__ unsigned int sh_mark[4];
  const uint32_t cells = tiles + rblocks;
  tile_scan_body(wtot, cells, woff, 1, ScanMarks{cells, 2, tiles}, sh_mark);
  if (threadIdx.x == 0) {
    C->chunk_base = sh_mark[2];
    C->level_new = sh_mark[1];
  }
}

// Narrow levels: both exclusive scans (own winners' popcounts, records'
// isnew flags) and k_shard_base's totals in one workgroup, instead of two
// device scans and a launch.
constexpr uint64_t SHARD_SMALL_SCAN = 16384;
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
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
// Narrow levels at world > 1: the owner-major exclusive scan of the count
// matrix and k_owner_totals in one workgroup (instead of a device scan's two
// launches and the totals launch).
constexpr uint64_t OWNER_SMALL_SCAN = 16384;
__global__ void __launch_bounds__(1024)
k_owner_scan_small(const uint8_t* __restrict__ cnt, uint32_t* __restrict__ off, uint64_t n, uint32_t world,
                   uint64_t* __restrict__ tot, const Counters* __restrict__ C, uint64_t* __restrict__ host_tot,
                   unsigned long long* __restrict__ host_head, uint64_t* __restrict__ row, uint64_t status_new,
                   uint64_t status_err, int level1, uint64_t init_err) {
  __shared__ uint32_t lds[16];
  const uint64_t cells = n * world;
  uint32_t carry = 0, total = 0;
  for (uint64_t b = 0; b < cells; b += blockDim.x) {
    const uint64_t i = b + threadIdx.x;
    const uint32_t v = i < cells ? (uint32_t)cnt[i] : 0u;
    const uint32_t e = block_exclusive_scan(v, lds, total);
    if (i < cells) off[i] = carry + e;
    carry += total;
  }
  __syncthreads();       // (the scan's global writes, for the totals' reads below)
  if (threadIdx.x < 64)
    owner_totals(off, cnt, n, world, tot, C, host_tot, host_head, row, status_new, status_err, level1, init_err);
}
__global__ void __launch_bounds__(1024)
k_shard_scan_small(const uint32_t* __restrict__ newmask, uint64_t nlocal, uint32_t* __restrict__ offsets,
                   const uint32_t* __restrict__ isnew, uint64_t nrec, uint32_t* __restrict__ ioff,
                   Counters* __restrict__ C) {
  __shared__ uint32_t lds[16];
  uint32_t carry = 0, tot = 0;
  for (uint64_t b = 0; b < nlocal; b += blockDim.x) {
    const uint64_t i = b + threadIdx.x;
    const uint32_t v = i < nlocal ? NewCount()(newmask[i]) : 0u;
    const uint32_t e = block_exclusive_scan(v, lds, tot);
    if (i < nlocal) offsets[i] = carry + e;
    carry += tot;
  }
  const uint32_t lt = carry;
  carry = 0;
  for (uint64_t b = 0; b < nrec; b += blockDim.x) {
    const uint64_t i = b + threadIdx.x;
    const uint32_t v = i < nrec ? isnew[i] : 0u;
    const uint32_t e = block_exclusive_scan(v, lds, tot);
    if (i < nrec) ioff[i] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    C->chunk_base = lt;
    C->level_new = (uint64_t)lt + carry;
  }
}

// chunk_base = this rank's own new states (the records' emit base);
// level_new = all new states of the level
__global__ void k_shard_base(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ newmask,
                             uint64_t nlocal, const uint32_t* __restrict__ ioff,
                             const uint32_t* __restrict__ isnew, uint64_t nrec, Counters* __restrict__ C) {
  if (threadIdx.x != 0) return;
  const uint64_t lt = nlocal ? (uint64_t)offsets[nlocal - 1] + NewCount()(newmask[nlocal - 1]) : 0;
  const uint64_t rt = nrec ? (uint64_t)ioff[nrec - 1] + isnew[nrec - 1] : 0;
  C->chunk_base = lt;
  C->level_new = lt + rt;
}

// The winners among the received records, after the local ones (one
// workgroup's share).
// (boff != nullptr, the tile-count path: the block's first position, the
// rest from the block's own isnew flags; else per-record offsets ioff after
// the own states, chunk_base)
__device__ __forceinline__ uint64_t rec_block_pos(uint64_t blk, uint64_t i, uint64_t n,
                                                  const uint32_t* __restrict__ isnew,
                                                  const uint32_t* __restrict__ ioff,
                                                  const uint32_t* __restrict__ boff, const Counters* __restrict__ C,
                                                  bool* won) {
  const bool w = i < n && isnew[i];
  *won = w;
  if (!boff) return w ? C->chunk_base + ioff[i] : 0ull;
  __shared__ unsigned int sh_rw[4];
  const unsigned long long b = __ballot(w);
  const unsigned lane = threadIdx.x & 63;
  if (lane == 0) sh_rw[threadIdx.x >> 6] = (unsigned)__popcll(b);
  __syncthreads();
  unsigned before = 0;
  for (unsigned k = 0; k < (threadIdx.x >> 6); ++k) before += sh_rw[k];
  return (uint64_t)boff[blk] + before + (unsigned)__popcll(b & ((1ull << lane) - 1ull));
}
template <class M>
__device__ __forceinline__ void emit_rec_block(uint64_t blk, const Record<M>* __restrict__ in, uint64_t n,
                                               const uint32_t* __restrict__ isnew, const uint32_t* __restrict__ ioff,
                                               const uint32_t* __restrict__ boff,
                                               Flags f, typename M::State* __restrict__ next,
                                               unsigned long long* __restrict__ pkeys, uint64_t next_gidx,
                                               Counters* __restrict__ C) {
  __shared__ unsigned int sh_act[A_COUNT];
  __shared__ unsigned long long sh_cand;
  if (threadIdx.x < A_COUNT) sh_act[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh_cand = 0;
  __syncthreads();
  const uint64_t i = blk * blockDim.x + threadIdx.x;
  unsigned long long cand = 0;
  bool won;
  const uint64_t o = rec_block_pos(blk, i, n, isnew, ioff, boff, C, &won);
  if (won) {
    typename M::State x;
    uint64_t key;
    load_record<M>(in, i, x, key);
    store_state<M>(next, o, x);
    pkeys[next_gidx + o] = key;
    if (M::check(x, f.inv_mask) >= 0) atomicMin(&C->err_key, (key & ~0xffull) | E_INVARIANT);
    // (a record's action byte indexes LDS: a zeroed record of a failed rank
    // reads 0; anything out of range would be a corrupt record, counted nowhere)
    if ((key & 0xff) < (uint64_t)A_COUNT) atomicAdd(&sh_act[key & 0xff], 1u);
    cand = (unsigned long long)M::plan(x, f).total;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cand += __shfl_down(cand, off, 64);
  if ((threadIdx.x & 63) == 0 && cand) atomicAdd(&sh_cand, cand);
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_act[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_act[threadIdx.x]);
  if (threadIdx.x == 0 && sh_cand) atomicAdd(&stripe(C).next_cand, sh_cand);
}
// cand_total = sum of the next_cand stripes (one lane per stripe), then the
// level head straight into pinned host memory
__device__ __forceinline__ void level_tail(Counters* __restrict__ C, unsigned long long* __restrict__ host_head) {
  static_assert(CTR_STRIPES == 64, "one lane per stripe");
  unsigned long long v = ld_agent(&C->s[threadIdx.x].next_cand);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if (threadIdx.x == 0) {
    C->cand_total = v;
    __threadfence();
    head_to_host(C, host_head);
  }
}
__global__ void __launch_bounds__(64) k_shard_cand(Counters* __restrict__ C,
                                                   unsigned long long* __restrict__ host_head) {
  level_tail(C, host_head);
}
// Both emits in one launch: blocks [0, lblocks) this rank's own winners
// (the engine's wave-balanced emit body, engine_kernels.h emit_body, with
// parent keys), the rest the records'.  Narrow levels (tail != 0): the last
// workgroup to finish runs k_shard_cand's tail; a wide level's grid would
// queue that many device-scope atomics and fences on one counter
// (measured: NP=2 sharded 172 -> 680 ms), so it takes the separate launch.
// woff != nullptr: the tile-count path (k_win_scan's offsets: own tiles,
// then record blocks); else per-parent offsets and per-record ioff.
template <class M>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_shard_emit(const typename M::State* __restrict__ cur, uint64_t n_local, uint32_t lblocks, Flags f, uint64_t rank,
             const uint32_t* __restrict__ newmask, const uint32_t* __restrict__ offsets,
             const Record<M>* __restrict__ in, uint64_t n, const uint32_t* __restrict__ isnew,
             const uint32_t* __restrict__ ioff, typename M::State* __restrict__ next,
             unsigned long long* __restrict__ pkeys, uint64_t next_gidx, Counters* __restrict__ C,
             unsigned long long* __restrict__ host_head, int tail, const uint32_t* __restrict__ woff) {
  __shared__ bool sh_last;
  if (blockIdx.x < lblocks)
    emit_body<M, 0, true>(cur, n_local, 0, f, newmask, offsets, next, 0, 0, next_gidx, pkeys, nullptr, 1, C, woff,
                          rank);
  else
    emit_rec_block<M>(blockIdx.x - lblocks, in, n, isnew, ioff, woff ? woff + lblocks : nullptr, f, next, pkeys,
                      next_gidx, C);
  if (!tail) return;
  // every thread's atomics (error key, stripes) before this workgroup counts as done
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) sh_last = atomicAdd(&C->emit_done, 1ull) == gridDim.x - 1;
  __syncthreads();
  if (!sh_last || threadIdx.x >= 64) return;
  __threadfence();
  if (threadIdx.x == 0) C->emit_done = 0;
  level_tail(C, host_head);
}
constexpr unsigned SHARD_TAIL_BLOCKS = 64;    // emit grids up to this size run the level tail themselves

// The deferred frontier's emit (round 5; the engine's k_emit_links on the
// sharded path): per new state only its link and its parent key (TLC's
// trace file) — own winners at their tile offsets in (parent, position)
// order (link parent << 8 | position), then the received records' winners
// in receive order (link bit 63 | record index: the next level's k_claim
// reads the state from this level's receive buffer).  No state is built,
// stored, checked or planned here: the next level's k_claim rebuilds each
// state as it expands it (shard_rebuild).  Entries at or past `cap` are not
// written and set DF_CAPACITY; the host grows the buffers and runs the
// launch again (it writes nothing else).
template <class M>
__global__ void __launch_bounds__(256)
k_shard_emit_links(uint64_t n_local, uint32_t lblocks, uint64_t rank, const uint32_t* __restrict__ gpos,
                   const uint32_t* __restrict__ newmask,
                   const Record<M>* __restrict__ in, uint64_t n, const uint32_t* __restrict__ isnew,
                   const uint32_t* __restrict__ woff, unsigned long long* __restrict__ link,
                   unsigned long long* __restrict__ pkeys, uint64_t next_gidx, uint64_t cap,
                   Counters* __restrict__ C, unsigned long long* __restrict__ host_head, int tail) {
  __shared__ unsigned int sh_wtot[4];
  __shared__ bool sh_last;
  bool over = false;
  if (blockIdx.x < lblocks) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t tbase = woff[blockIdx.x];         // (loaded with the masks: one round trip less)
    const uint32_t mask = i < n_local ? newmask[i] : 0u;
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
    uint64_t obase = tbase;
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
      if (g >= wtot) continue;
      for (; k > 0; --k) m &= m - 1;
      const uint64_t t = (uint64_t)(__ffs(m) - 1);
      const uint64_t pidx = wave0 + (uint64_t)p;
      const uint64_t o = obase + (uint64_t)g;
      if (o >= cap) {
        over = true;
        continue;
      }
      link[o] = (pidx << 8) | t;
      pkeys[next_gidx + o] = (rank << 60) | ((gpos ? (uint64_t)gpos[pidx] : pidx) << 16) | (t << 8);
    }
  } else {
    const uint64_t blk = blockIdx.x - lblocks;
    const uint64_t i = blk * blockDim.x + threadIdx.x;
    bool won;
    const uint64_t o = rec_block_pos(blk, i, n, isnew, nullptr, woff + lblocks, C, &won);
    if (won) {
      if (o >= cap) {
        over = true;
      } else {
        link[o] = (1ull << 63) | i;
        pkeys[next_gidx + o] = in[i].w[0];
      }
    }
  }
  if (over) atomicOr(&C->defer_flags, DF_CAPACITY);
  if (!tail) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) sh_last = atomicAdd(&C->emit_done, 1ull) == gridDim.x - 1;
  __syncthreads();
  if (!sh_last || threadIdx.x >= 64) return;
  __threadfence();
  if (threadIdx.x == 0) C->emit_done = 0;
  level_tail(C, host_head);
}

// A deferred frontier materialised outside k_claim (before a narrow batch,
// at a max_levels stop): the same rebuild, plus the level's successor count.
template <class M, bool TLC>
__global__ void __launch_bounds__(256) k_shard_materialize(DeferArgs df, uint64_t n, Flags f, uint64_t rank,
                                                           Counters* __restrict__ C) {
  __shared__ unsigned int sh_actd[A_COUNT];
  if (threadIdx.x < A_COUNT) sh_actd[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long cand = 0;
  if (i < n) {
    const typename M::State s = shard_rebuild<M, 1, TLC>(df, i, f, rank, sh_actd, C);
    cand = (unsigned long long)M::plan(s, f).total;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cand += __shfl_down(cand, off, 64);
  if ((threadIdx.x & 63) == 0 && cand) atomicAdd(&stripe(C).next_cand, cand);
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_actd[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_actd[threadIdx.x]);
}

// ---- seen-set spill (cfg.seen_hbm_bytes > 0), per rank: the engine's hot
// ClaimSet + cold runs (coldset.h, engine_spill.h) over this rank's share of
// the fingerprints.  After a level's settle passes and scans, its winners
// w.r.t. the hot table are checked against the cold tier in windows of
// emit positions [w0, w1): cold key + location (own successor: parent << 5 |
// position; received record: bit 63 | record index).
template <class M>
__global__ void __launch_bounds__(256)
k_shard_spill_queries(const typename M::State* __restrict__ cur, uint64_t n_local, uint32_t lblocks, Flags f,
                      const uint32_t* __restrict__ newmask, const uint32_t* __restrict__ offsets, uint64_t n,
                      const unsigned long long* __restrict__ rfp, const uint32_t* __restrict__ isnew,
                      const uint32_t* __restrict__ ioff, const Counters* __restrict__ C, uint64_t w0, uint64_t w1,
                      uint64_t* __restrict__ qkey, uint64_t* __restrict__ qloc) {
  if (blockIdx.x < lblocks) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_local) return;
    uint32_t mask = newmask[i];
    if (!mask) return;
    const uint64_t o = offsets[i];
    if (o >= w1 || o + (uint64_t)__builtin_popcount(mask) <= w0) return;
    const typename M::State s = load_state<M>(cur, i);
    const typename M::Plan pl = M::plan(s, f);
    const uint64_t fold = M::fp_fold(s);
    const uint32_t proj = M::owner_proj(s);
    for (uint64_t pos = o; mask; mask &= mask - 1, ++pos) {
      if (pos < w0 || pos >= w1) continue;
      const int t = __ffs(mask) - 1;
      int slot, j;
      M::locate(pl, t, slot, j);
      typename M::State x;
      int who;
      M::apply(s, slot, j, f, x, who);
      // (the fingerprint k_claim claimed: owner bits included, as at every world)
      qkey[pos - w0] = cold_key(M::template fingerprint_succ<1>(s, fold, x, who, proj));
      qloc[pos - w0] = (i << 5) | (uint64_t)t;
    }
    return;
  }
  const uint64_t r = (uint64_t)(blockIdx.x - lblocks) * blockDim.x + threadIdx.x;
  if (r >= n || !isnew[r]) return;
  const uint64_t pos = C->chunk_base + ioff[r];
  if (pos < w0 || pos >= w1) return;
  qkey[pos - w0] = cold_key(rfp[r]);
  qloc[pos - w0] = (1ull << 63) | r;
}
// Winners found in the cold tier lose: their newmask bit or isnew flag is
// cleared and their hot slot retired (engine_spill.h claimset_retire).
__global__ void k_shard_spill_apply(const uint64_t* __restrict__ qkey, const uint64_t* __restrict__ qloc,
                                    const uint8_t* __restrict__ found, uint64_t m, uint32_t* __restrict__ newmask,
                                    uint32_t* __restrict__ isnew, ClaimEntry* __restrict__ cs, uint64_t nslots,
                                    Counters* __restrict__ C) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !found[i]) return;
  const uint64_t loc = qloc[i];
  if (loc >> 63)
    isnew[loc & ~(1ull << 63)] = 0u;
  else
    atomicAnd(&newmask[loc >> 5], ~(1u << (loc & 31)));
  if (!claimset_retire(cs, nslots, cold_unkey(qkey[i]))) atomicAdd(&C->overflow, 1ull);
}

// ---- TLC order (ShardBase::tlc_*; cfg.tlc_order, world > 1).  Per level of
// global width W, after every rank's insert: k_tlc_mask sets, for each new
// state this rank won, its position bit in its parent's word (parent keys
// carry the parent's G); the words are summed over the ranks (bits of one
// parent are disjoint: every successor has one owner); then G of a new state
// = the winners of the parents before its parent (one scan over the W
// popcounts) + its parent's winners before it (k_tlc_pos), and its local
// index = the rank's G values before it (a bitmap over the next level's G
// and one scan of its word popcounts: k_tlc_perm).  The bitmap and its scan
// stay as the next level's G -> local index map (ClaimKeys::mine).
__global__ void __launch_bounds__(256) k_tlc_mask(const unsigned long long* __restrict__ pk, uint64_t nn,
                                                  uint32_t* __restrict__ wmask, uint64_t W,
                                                  Counters* __restrict__ C) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  const uint64_t key = pk[i];
  const uint64_t g = (key >> 16) & 0xffffffffull;
  const uint32_t t = (uint32_t)((key >> 8) & 0xff);
  if (g >= W || t >= 32) {
    atomicAdd(&C->overflow, 1ull);                // a parent key outside the level: fail loudly
    return;
  }
  atomicOr(&wmask[g], 1u << t);
}
__global__ void __launch_bounds__(256) k_tlc_pos(const unsigned long long* __restrict__ pk, uint64_t nn,
                                                 const uint32_t* __restrict__ wmask,
                                                 const uint32_t* __restrict__ wbase, uint32_t* __restrict__ gnew,
                                                 uint32_t* __restrict__ bits) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  const uint64_t key = pk[i];
  const uint64_t g = (key >> 16) & 0xffffffffull;
  const uint32_t t = (uint32_t)((key >> 8) & 31);
  const uint32_t gn = wbase[g] + (uint32_t)__builtin_popcount(wmask[g] & ((1u << t) - 1u));
  gnew[i] = gn;
  atomicOr(&bits[gn >> 5], 1u << (gn & 31));
}
__global__ void __launch_bounds__(256) k_tlc_perm(uint64_t nn, const uint32_t* __restrict__ gnew,
                                                  const uint32_t* __restrict__ bits,
                                                  const uint32_t* __restrict__ brank,
                                                  const unsigned long long* __restrict__ link_in,
                                                  const unsigned long long* __restrict__ pk_in,
                                                  unsigned long long* __restrict__ link_out,
                                                  unsigned long long* __restrict__ pk_out,
                                                  uint32_t* __restrict__ gpos_out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  const uint32_t gn = gnew[i];
  const uint64_t j = (uint64_t)brank[gn >> 5] + (uint64_t)__builtin_popcount(bits[gn >> 5] & ((1u << (gn & 31)) - 1u));
  link_out[j] = link_in[i];
  pk_out[j] = pk_in[i];
  gpos_out[j] = gn;
}

// drop_last_expand: take a level's per-action generated counts back out
// (what k_claim added: each parent's plan slot counts, by action), from the
// level's states and the plans k_claim kept
template <class M>
__global__ void __launch_bounds__(256) k_undo_gen(const typename M::State* __restrict__ st,
                                                  const unsigned long long* __restrict__ counts, uint64_t n,
                                                  Counters* __restrict__ C) {
  __shared__ unsigned int sh[A_COUNT];
  if (threadIdx.x < A_COUNT) sh[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const typename M::State s = load_state<M>(st, i);
    const unsigned long long c = counts[i];
#pragma unroll
    for (int slot = 0; slot < M::NSLOT; ++slot) {
      const unsigned v = (unsigned)((c >> (6 * slot)) & 63);
      if (v) atomicAdd(&sh[M::slot_action(s, slot)], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh[threadIdx.x])
    atomicAdd(&stripe(C).act_gen[threadIdx.x], 0ull - (unsigned long long)sh[threadIdx.x]);   // (mod 2^64)
}

template <class M>
class ShardT final : public ShardBase {
  using State = typename M::State;
  using Rec = Record<M>;

 public:
  ShardT(const kc_model_config& cfg, int rank, int world)
      : cfg_(cfg), rank_(rank), world_(world) {
    flags_ = flags_of(cfg);
    spill_ = cfg.seen_hbm_bytes > 0;
    if (cfg.spill_dir) spill_dir_ = cfg.spill_dir;   // (the seen-set's disk tier)
    cfg_.spill_dir = nullptr;      // (the caller's string is not kept)
    // A/B switches (round 5): KC_STAGE=0 packs every level with k_shard_pack
    // (re-expansion + per-parent owner scan); KC_SHARD_TSCAN=0 positions the
    // winners with per-parent / per-record device scans
    const char* sg = getenv("KC_STAGE");
    stage_on_ = !(sg && sg[0] == '0');
    const char* ts = getenv("KC_SHARD_TSCAN");
    tcount_ = !(ts && ts[0] == '0');
    const char* dc = getenv("KC_DEFER_CHECK");     // diagnostic: rebuilt states against materialised ones
    defer_check_ = dc && dc[0] == '1';
    tlc_ = cfg.tlc_order && world > 1;
    // first-claim mode on the counted levels (k_claim FIRST, k_rec_claim_first;
    // no candidates, no settle passes): the first inserter owns a state, as in
    // a TLC -workers N run
    first_ = cfg.first_claim != 0;
    const char* ck = getenv("KC_CHUNK_SCAN");
    ocscan_ = !(ck && ck[0] == '0');
    // (its ClaimSet holds fp words only, as the engine's in this mode: 8-B
    // slots, half the table to clear; the narrow levels write no claim words)
    cs_.compact = first_;
  }
  ~ShardT() override { release(); }

  int setup() override {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      set_error("kc_shard: no HIP device visible (no CPU fallback)");
      return -ENODEV;
    }
    if (world_ < 1 || world_ > 15 || rank_ < 0 || rank_ >= world_) {
      set_error("kc_shard: bad rank/world %d/%d (1..15 ranks)", rank_, world_);
      return -EINVAL;
    }
    if (cfg_.device < 0 || cfg_.device >= ndev) {
      set_error("kc_shard: bad device %d", cfg_.device);
      return -EINVAL;
    }
    if (tlc_ && (spill_ || !tcount_)) {
      set_error("kc_shard: tlc_order needs the deferred frontier (no seen-set spill, KC_SHARD_TSCAN on)");
      return -EINVAL;
    }
    if (first_ && (tlc_ || spill_ || !tcount_)) {
      set_error("kc_shard: first_claim cannot run with %s", tlc_ ? "tlc_order (a deterministic claim order)"
                                                         : spill_ ? "the seen-set spill (its cold check settles winners)"
                                                                  : "KC_SHARD_TSCAN=0 (it needs the tile counts)");
      return -EINVAL;
    }
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    KC_HIP_TRY(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    KC_HIP_TRY(hipMalloc(&d_ctr_, sizeof(Counters)));
    KC_HIP_TRY(hipHostMalloc(&h_ctr_, sizeof(Counters)));
    KC_HIP_TRY(hipHostMalloc(&h_exp_, kCtrHead));
    KC_HIP_TRY(hipMalloc(&d_owner_base_, 16 * sizeof(uint64_t)));
    KC_HIP_TRY(hipMalloc(&d_ovf_cnt_, 8));     // (zeroed by k_head_reset every level)
    KC_HIP_TRY(hipMalloc(&d_stage_cur_, 8));   // (likewise)
    KC_HIP_TRY(hipHostMalloc(&h_owner_base_, 16 * sizeof(uint64_t)));
    KC_HIP_TRY(hipEventCreate(&ev_[0]));
    KC_HIP_TRY(hipEventCreate(&ev_[1]));
    return 0;
  }

  // k_claim time (HIP events, cfg.timing != 0), launches and parents since
  // the last call to this function (reset on read).
  void claim_times(double* ms, uint64_t* launches, uint64_t* parents) override {
    *ms = claim_ms_;
    *launches = claim_launches_;
    *parents = claim_parents_;
    claim_ms_ = 0;
    claim_launches_ = claim_parents_ = 0;
  }

  int set_stream(hipStream_t st) override {
    if (own_st_ && st_) KC_HIP_TRY(hipStreamDestroy(st_));
    st_ = st;
    own_st_ = false;
    return 0;
  }

  int init(uint64_t* n_local) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    const uint64_t fp_slots = cfg_.fpset_slots ? cfg_.fpset_slots : (1ull << 20);
    if (spill_) {
      KC_TRY(spill_setup());
    } else if (cs_.t && cs_.capacity() >= fp_slots) {
      KC_TRY(cs_.clear(st_));
    } else {
      KC_TRY(cs_.init(fp_slots, st_));
    }
    KC_HIP_TRY(hipMemsetAsync(d_ctr_, 0, sizeof(Counters), st_));
    std::vector<State> mine;
    std::vector<unsigned long long> keys;
    std::vector<uint64_t> fps;
    cand_ = 0;
    for (int k = 0; k < M::num_init(); ++k) {
      State s;
      M::init_state(k, s, cfg_.variant);
      const uint64_t fp = M::template fingerprint<1>(s);
      const uint32_t o = (uint32_t)(((unsigned __int128)(fp << 1) * (uint64_t)world_) >> 64);
      if ((int)o != rank_) continue;
      mine.push_back(s);
      keys.push_back(KEY_INIT | (uint64_t)k);
      fps.push_back(fp);
      cand_ += (uint64_t)M::plan(s, flags_).total;
      // an Init-state violation's key orders by the Init state's index in
      // TLC's order (k << 16; the rank in bits 8-15), so the minimum over
      // the ranks is the first violating Init state TLC would report
      if (M::check(s, flags_.inv_mask) >= 0 && init_err_ == ~0ull)
        init_err_ = ((uint64_t)k << 16) | ((uint64_t)rank_ << 8) | 0x12;
    }
    n_ = mine.size();
    init_key_ = init_err_;
    cur_deferred_ = false;
    emitted_links_ = false;
    deferred_states_ = 0;
    cand_est_ = next_cand_est_ = false;
    last_new_ = 0;
    prev_rec_ = nullptr;
    defer_err_ = ~0ull;
    level_ = 1;
    level_base_.assign(1, 0);
    gen_init_ = n_;
    cand_total_ = 0;
    KC_TRY(grow_buffer(cur_, cur_cap_, std::max<uint64_t>(n_, 1), false, st_));
    KC_TRY(grow_buffer(pkeys_, pk_cap_, std::max<uint64_t>(n_, 1), false, st_));
    if (tlc_) {
      // level 1 in TLC order: Init states are distinct, each at its index
      // (G = k); this rank's in increasing k
      const uint64_t W = (uint64_t)M::num_init(), words = W / 32 + 1;
      std::vector<uint32_t> g, bits(words, 0), brank(words, 0);
      for (auto k : keys) {
        const uint32_t gk = (uint32_t)(k & 0xffffffffull);
        g.push_back(gk);
        bits[gk >> 5] |= 1u << (gk & 31);
      }
      for (uint64_t w = 1; w < words; ++w) brank[w] = brank[w - 1] + (uint32_t)__builtin_popcount(bits[w - 1]);
      KC_TRY(grow_buffer(gpos_all_, gp_cap_, pk_cap_, false, st_));
      KC_TRY(grow_buffer(gbits_cur_, gbits_cur_cap_, words, false, st_));
      KC_TRY(grow_buffer(grank_cur_, grank_cur_cap_, words, false, st_));
      if (n_) KC_HIP_TRY(hipMemcpyAsync(gpos_all_, g.data(), n_ * 4, hipMemcpyHostToDevice, st_));
      KC_HIP_TRY(hipMemcpyAsync(gbits_cur_, bits.data(), words * 4, hipMemcpyHostToDevice, st_));
      KC_HIP_TRY(hipMemcpyAsync(grank_cur_, brank.data(), words * 4, hipMemcpyHostToDevice, st_));
      KC_HIP_TRY(hipStreamSynchronize(st_));
    }
    if (n_) {
      KC_HIP_TRY(hipMemcpyAsync(cur_, mine.data(), n_ * sizeof(State), hipMemcpyHostToDevice, st_));
      KC_HIP_TRY(hipMemcpyAsync(pkeys_, keys.data(), n_ * 8, hipMemcpyHostToDevice, st_));
      uint64_t* d_fps = nullptr;
      KC_HIP_TRY(hipMalloc(&d_fps, n_ * 8));
      KC_HIP_TRY(hipMemcpyAsync(d_fps, fps.data(), n_ * 8, hipMemcpyHostToDevice, st_));
      launch_claimset_insert_list(d_fps, n_, cs_, 1u, nullptr, st_);
      KC_HIP_TRY(hipStreamSynchronize(st_));
      (void)hipFree(d_fps);
    }
    KC_HIP_TRY(hipStreamSynchronize(st_));
    cs_.count = n_;
    distinct_ = n_;
    *n_local = n_;
    return 0;
  }

  // Claims this rank's own successors of the level; counts the rest per owner.
  int expand(uint64_t* counts, uint64_t* err_key) override {
    KC_TRY(expand_dev(0, ~0ull, false, nullptr));
    if (!dev_empty_) KC_HIP_TRY(hipStreamSynchronize(st_));
    return expand_done(counts, err_key);
  }
  int expand_dev(uint64_t status_new, uint64_t status_err, bool level1, uint64_t* d_row) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    rebuilt_ = false;
    gen_snap_ok_ = false;
    hipLaunchKernelGGL(k_head_reset, dim3(1), dim3(64), 0, st_, d_ctr_, d_ovf_cnt_, d_stage_cur_);
    send_total_ = 0;
    dev_init_err_ = init_err_;
    init_err_ = ~0ull;
    dev_empty_ = n_ == 0;
    if (n_ == 0) {
      // nothing to claim; a device row still gets its status words
      if (d_row)
        hipLaunchKernelGGL(k_owner_totals, dim3(1), dim3(64), 0, st_, off_, cnt_, (uint64_t)0, (uint32_t)world_,
                           d_owner_base_, d_ctr_, h_owner_base_, reinterpret_cast<unsigned long long*>(h_exp_),
                           d_row, status_new, status_err, (int)level1, dev_init_err_);
      dev_empty_ = d_row == nullptr;
      dev_zero_ = true;
      return 0;
    }
    dev_zero_ = false;
    if (n_ >= (1ull << 32)) {
      set_error("kc_shard_expand: frontier wider than 2^32 states");
      return -ENOMEM;
    }
    if (spill_) {
      // the level's claims (own successors and received records: about
      // cand_ successors together, of which the last level's fraction
      // filled hot slots) go into the fixed hot table; flush it first when
      // they might take it past 1/2 load
      const uint64_t need = std::min<uint64_t>(cand_, (uint64_t)((double)cand_ * sp_ratio_ * 1.25) + 4096);
      if (cs_.count > 0 && cs_.count + need > hot_limit_) KC_TRY(spill_flush());
    } else {
      // (a deferred frontier's successor count is an estimate: 16 per parent
      // at least, so even MAXSUCC = 32 cannot fill the table, as the engine)
      KC_TRY(cs_.reserve(cand_est_ ? std::max<uint64_t>(cand_, 16 * n_) : cand_, st_));
    }
    const uint64_t tiles = (n_ + CLAIM_TILE - 1) / CLAIM_TILE;
    KC_TRY(grow_buffer(rcount_, rcount_cap_, tiles, false, st_));
    // (first-claim mode has no candidates: no records, no overflow list; its
    // k_claim writes each tile's new-state count, k_win_scan's input)
    if (first_) KC_TRY(grow_buffer(wtot_, wtot_cap_, tiles + 8, false, st_));
    if (!first_) KC_TRY(grow_buffer(rec_fp_, rec_fp_cap_, tiles * CLAIM_RCAP, false, st_));
    if (!first_) KC_TRY(grow_buffer(rec_lk_, rec_lk_cap_, tiles * CLAIM_RCAP, false, st_));
    // candidates past a tile's segment: one overflow list, bounded by the
    // level's successor count
    if (!first_) {
      // (estimated: at least two per parent; the list holds only the
      // candidates past a tile's first 256, a few percent of the successors)
      const uint64_t bound = cand_est_ ? std::max<uint64_t>(cand_, 2 * n_) : std::max<uint64_t>(cand_, 1);
      KC_TRY(grow_buffer_tight(ovf_fp_, ovf_fp_cap_, bound, st_));
      KC_TRY(grow_buffer_tight(ovf_lk_, ovf_lk_cap_, bound, st_));
      KC_TRY(grow_buffer_tight(ovf_tile_, ovf_tile_cap_, bound, st_));
      ovf_ = CandOvf{d_ovf_cnt_, ovf_fp_, ovf_lk_, ovf_tile_, std::min(ovf_fp_cap_, std::min(ovf_lk_cap_, ovf_tile_cap_))};
    }
    KC_TRY(grow_buffer(newmask_, mask_cap_, n_, false, st_));
    KC_TRY(grow_buffer(cnt_, cnt_cap_, n_ * world_, false, st_));
    KC_TRY(grow_buffer(repmask_, rm_cap_, n_, false, st_));
    ShardArgs sh;
    sh.world = (uint32_t)world_;
    sh.rank = (uint32_t)rank_;
    sh.repmask = repmask_;
    sh.cnt = cnt_;
    sh.ovf = ovf_;
    if (tlc_) sh.gpos = gpos_cur();
    if (first_) sh.ttot = wtot_;
    // record staging (world > 1): an estimate from the last level's records
    // per parent, at most the level's successors; a level past it packs the
    // old way (DF_STAGE, pack())
    stage_level_ = world_ > 1 && stage_on_;
    if (stage_level_) {
      const uint64_t est = std::min<uint64_t>(std::max<uint64_t>(cand_, 1),
                                              (uint64_t)((double)n_ * rec_ratio_ * 1.5) + 65536);
      KC_TRY(grow_buffer_tight(stage_, stage_cap_, est, st_));
      const uint64_t cells = tiles * (uint64_t)world_;
      KC_TRY(grow_buffer(tcnt_, tcnt_cap_, cells + 8, false, st_));
      KC_TRY(grow_buffer(toff_, toff_cap_, cells + 8, false, st_));
      KC_TRY(grow_buffer(stoff_, stoff_cap_, tiles, false, st_));
      ocscan_level_ = ocscan_;
      if (ocscan_level_) {
        const uint64_t old = ocsum_cap_;
        KC_TRY(grow_buffer(ocsum_, ocsum_cap_, (tiles / CSUM_TILES + 1) * (uint64_t)world_ + 8, false, st_));
        if (ocsum_cap_ != old) KC_HIP_TRY(hipMemsetAsync(ocsum_, 0, ocsum_cap_ * sizeof(uint32_t), st_));
        sh.ocsum = ocsum_;
      }
      sh.stage = stage_;
      sh.stage_cur = d_stage_cur_;
      sh.stage_cap = stage_cap_;
      sh.tcnt = tcnt_;
      sh.stoff = stoff_;
    }
    const size_t dyn = (size_t)(CLAIM_TILE + ((world_ + 3) / 4) * CLAIM_TILE) * sizeof(unsigned int);
    // the deferred frontier: this level's plans kept for the next level's
    // rebuild; a deferred frontier rebuilt into cur_ (the free buffer) from
    // the previous frontier (next_) and the last receive buffer
    DeferArgs df;
    if (defer_on_) {
      KC_TRY(grow_buffer(pc_cur_, pc_cur_cap_, n_, false, st_));
      df.counts_out = pc_cur_;
    }
    rebuilt_ = cur_deferred_;
    if (cur_deferred_) {
      KC_TRY(grow_buffer(cur_, cur_cap_, n_, false, st_));
      df.prev = next_;
      df.link = link_cur_;
      df.prev_rec = prev_rec_;
      df.out = cur_;
      df.prev_counts = pc_prev_;
      if (tlc_) df.prev_gpos = gpos_prev();
      cur_deferred_ = false;
      ++deferred_levels_;
      deferred_states_ += n_;     // (rebuilt inside this k_claim: its algorithmic bytes, bench.py)
      // (the solo path stops on this level's deferred invariant after the
      // expand has counted its successors, where the exact path stops before
      // it: drop_last_expand then subtracts them, from the rebuilt states
      // and the plans this k_claim keeps)
      gen_snap_ok_ = d_row == nullptr && df.counts_out != nullptr;
      if (defer_check_) {
        if (!d_dchk_) KC_HIP_TRY(hipMalloc(&d_dchk_, 32));
        const unsigned long long init[4] = {0ull, ~0ull, ~0ull, 0ull};
        KC_HIP_TRY(hipMemcpyAsync(d_dchk_, init, 32, hipMemcpyHostToDevice, st_));
        KC_HIP_TRY(hipStreamSynchronize(st_));
        df.check = d_dchk_;
      }
    }
    if (cfg_.timing) KC_HIP_TRY(hipEventRecord(ev_[0], st_));
    if (world_ == 1) {
      // one rank owns everything: the single-GPU engine's claim kernel (no
      // owner counting; claim keys then carry rank 0, which they do anyway)
      if (first_)
        hipLaunchKernelGGL((k_claim<M, 0, false, 1, false, true, true>), dim3((unsigned)tiles), dim3(CLAIM_TILE), 0, st_,
                           cur_, n_, (uint64_t)0, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                           (uint32_t)level_ + 1, (uint32_t*)nullptr, rcount_, rec_fp_, rec_lk_, newmask_,
                           d_ctr_, sh, df);
      else
        hipLaunchKernelGGL((k_claim<M, 0, false, 1>), dim3((unsigned)tiles), dim3(CLAIM_TILE), 0, st_,
                           cur_, n_, (uint64_t)0, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                           (uint32_t)level_ + 1, (uint32_t*)nullptr, rcount_, rec_fp_, rec_lk_, newmask_,
                           d_ctr_, sh, df);
    } else if (first_) {
      hipLaunchKernelGGL((k_claim<M, 0, true, 1, false, true, true>), dim3((unsigned)tiles), dim3(CLAIM_TILE), dyn, st_,
                         cur_, n_, (uint64_t)0, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                         (uint32_t)level_ + 1, (uint32_t*)nullptr, rcount_, rec_fp_, rec_lk_, newmask_,
                         d_ctr_, sh, df);
    } else {
      if (tlc_)
        hipLaunchKernelGGL((k_claim<M, 0, true, 1, true>), dim3((unsigned)tiles), dim3(CLAIM_TILE), dyn, st_,
                           cur_, n_, (uint64_t)0, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                           (uint32_t)level_ + 1, (uint32_t*)nullptr, rcount_, rec_fp_, rec_lk_, newmask_,
                           d_ctr_, sh, df);
      else
        hipLaunchKernelGGL((k_claim<M, 0, true>), dim3((unsigned)tiles), dim3(CLAIM_TILE), dyn, st_,
                           cur_, n_, (uint64_t)0, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                           (uint32_t)level_ + 1, (uint32_t*)nullptr, rcount_, rec_fp_, rec_lk_, newmask_,
                           d_ctr_, sh, df);
    }
    if (cfg_.timing) KC_HIP_TRY(hipEventRecord(ev_[1], st_));
#ifdef KC_CLAIM_TRACE
    {
      unsigned long long t[16];
      KC_HIP_TRY(hipStreamSynchronize(st_));
      KC_HIP_TRY(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_ctrace), sizeof t));
      if (t[0])
        fprintf(stderr, "ctrace rank %d level %d n %llu tiles %llu | us/block: prep %.2f deal %.2f succ %.2f compact %.2f "
                "claims %.2f stage %.2f tail %.2f | longest %.2f span %.2f\n", rank_, level_, (unsigned long long)n_,
                (unsigned long long)tiles, t[1] * 0.01 / t[0], t[2] * 0.01 / t[0], t[3] * 0.01 / t[0],
                t[4] * 0.01 / t[0], t[5] * 0.01 / t[0], t[6] * 0.01 / t[0], t[7] * 0.01 / t[0], t[8] * 0.01,
                (t[10] - t[9]) * 0.01);
      memset(t, 0, sizeof t);
      t[9] = ~0ull;
      KC_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_ctrace), t, sizeof t));
    }
#endif
    if (stage_level_) {
      // positions of the tiles' segments in the owner-grouped send buffer and
      // the owner totals (the all-gather row)
      if (tiles * (uint64_t)world_ >= (1ull << 31)) {
        set_error("kc_shard_expand: %llu tile x owner cells exceed one scan", (unsigned long long)(tiles * world_));
        return -ENOMEM;
      }
      if (ocscan_level_)
        hipLaunchKernelGGL(k_owner_cscan, dim3(1), dim3(TSCAN_THREADS), 0, st_, ocsum_,
                           (uint32_t)((tiles + CSUM_TILES - 1) / CSUM_TILES), (uint32_t)world_, toff_, d_owner_base_,
                           d_ctr_, h_owner_base_, reinterpret_cast<unsigned long long*>(h_exp_), d_row, status_new,
                           status_err, (int)level1, dev_init_err_);
      else
      hipLaunchKernelGGL(k_owner_tscan, dim3(1), dim3(TSCAN_THREADS), 0, st_, tcnt_, (uint32_t)tiles, (uint32_t)world_,
                         toff_, d_owner_base_, d_ctr_, h_owner_base_, reinterpret_cast<unsigned long long*>(h_exp_),
                         d_row, status_new, status_err, (int)level1, dev_init_err_);
      KC_HIP_TRY(hipGetLastError());
      return 0;
    }
    // one exclusive scan over the owner-major matrix = every record's position
    // in the owner-grouped send buffer (nothing to send at world 1)
    const uint64_t cells = n_ * (uint64_t)world_;
    KC_TRY(grow_buffer(off_, off_cap_, cells, false, st_));
    if (cells >= (1ull << 31)) {
      set_error("kc_shard_expand: frontier x world = %llu cells exceeds one scan (2^31)",
                (unsigned long long)cells);
      return -ENOMEM;
    }
    if (world_ > 1 && cells <= OWNER_SMALL_SCAN) {
      hipLaunchKernelGGL(k_owner_scan_small, dim3(1), dim3(1024), 0, st_, cnt_, off_, n_, (uint32_t)world_,
                         d_owner_base_, d_ctr_, h_owner_base_, reinterpret_cast<unsigned long long*>(h_exp_),
                         d_row, status_new, status_err, (int)level1, dev_init_err_);
    } else {
      if (world_ > 1) {
        size_t tmp_bytes = 0;
        const hipcub::TransformInputIterator<uint32_t, Widen8, const uint8_t*> cnt32(cnt_, Widen8());
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt32, off_, (int)cells, st_));
        KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, cnt32, off_, (int)cells, st_));
      }
      hipLaunchKernelGGL(k_owner_totals, dim3(1), dim3(64), 0, st_, off_, cnt_, n_, (uint32_t)world_,
                         d_owner_base_, d_ctr_, h_owner_base_, reinterpret_cast<unsigned long long*>(h_exp_),
                         d_row, status_new, status_err, (int)level1, dev_init_err_);
    }
    KC_HIP_TRY(hipGetLastError());
    return 0;
  }
  // after the stream sync that follows expand_dev
  int expand_done(uint64_t* counts, uint64_t* err_key) override {
    for (int o = 0; o < world_; ++o) counts[o] = 0;
    *err_key = dev_init_err_;
    defer_err_ = ~0ull;
    if (dev_zero_) return 0;
    defer_err_ = h_exp_->defer_err;
    const bool init_violated = dev_init_err_ != ~0ull;   // then it is THE error (see k_owner_totals)
    if (cfg_.timing) {
      float ms = 0;
      KC_HIP_TRY(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
      claim_ms_ += ms;
      ++claim_launches_;
    }
    claim_parents_ += n_;
    // (expand's head has a pinned copy of its own, h_exp_: a caller with
    // nothing to gather reads it only after insert's sync)
    if (h_exp_->overflow || h_exp_->batch_used) {
      set_error("kc_shard_expand: successor overflow or full table");
      return -ENOMEM;
    }
    staged_ = stage_level_ && !(h_exp_->defer_flags & DF_STAGE);
    if (defer_check_ && rebuilt_) {
      unsigned long long c[4];
      KC_HIP_TRY(hipMemcpy(c, d_dchk_, 32, hipMemcpyDeviceToHost));
      if (c[0])
        fprintf(stderr, "kc_shard rank %d level %d: %llu of %llu rebuilt states differ (first %lld, first record link %lld)\n",
                rank_, level_, c[0], (unsigned long long)n_, (long long)c[1], (long long)c[2]);
    }
    if (stage_level_ && !staged_) ++stage_fallbacks_;
    for (int o = 0; o < world_; ++o) {
      counts[o] = h_owner_base_[o];
      send_total_ += counts[o];
    }
    if (n_) rec_ratio_ = std::max(0.01, (double)(send_total_ - counts[rank_]) / (double)n_);
    if (h_exp_->err_key != ~0ull && !init_violated) {
      uint64_t e = ((uint64_t)rank_ << 60) | (uint64_t)h_exp_->err_key;
      if (tlc_) {
        // TLC order: the parent's G, no rank (the trace walk locates it)
        const uint64_t pidx = (h_exp_->err_key >> 16) & ((1ull << 44) - 1);
        uint32_t g = 0;
        KC_HIP_TRY(hipMemcpy(&g, gpos_cur() + pidx, 4, hipMemcpyDeviceToHost));
        e = ((uint64_t)g << 16) | (h_exp_->err_key & 0xffffull);
      }
      *err_key = std::min<uint64_t>(*err_key, e);
    }
    if (cfg_.verbose > 1)
      fprintf(stderr, "kc_shard rank %d level %d: expand n %llu rebuilt %d e1 %llx deferred-invariant %llx\n", rank_,
              level_, (unsigned long long)n_, (int)rebuilt_, (unsigned long long)*err_key,
              (unsigned long long)defer_err_);
    return 0;
  }

  uint64_t record_bytes() const override { return sizeof(Rec); }
  uint64_t init_error() const override { return init_key_; }
  hipStream_t stream() const override { return st_; }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  int device() const override { return cfg_.device; }
  int tuple_words() const override { return M::TUPLE_WORDS; }
  const kc_model_config& config() const override { return cfg_; }
  void set_async_pack(bool on) override { async_pack_ = on; }

  // Rebuild a counterexample on the host (TLC's trace file walk): from Init
  // state `init_idx` follow the successor ordinals, then add the violating
  // successor `pos` (invariant errors).  The same plan/apply code the
  // kernels run, compiled for the host.
  int replay(int init_idx, const std::vector<int>& ords, int kind, int pos,
             std::vector<std::vector<uint64_t>>& tuples, int* err_action, int* err_self,
             int* err_inv) override {
    if (init_idx < 0 || init_idx >= M::num_init()) {
      set_error("kc_shard replay: bad Init index %d", init_idx);
      return -EIO;
    }
    std::vector<State> path(1);
    M::init_state(init_idx, path[0], cfg_.variant);
    for (int t : ords) {
      const State& s = path.back();
      const typename M::Plan pl = M::plan(s, flags_);
      if (t < 0 || t >= pl.total) {
        set_error("kc_shard replay: ordinal %d out of %d", t, pl.total);
        return -EIO;
      }
      int slot, j;
      M::locate(pl, t, slot, j);
      State x;
      M::apply(s, slot, j, flags_, x);
      path.push_back(x);
    }
    *err_action = *err_self = *err_inv = -1;
    const State& s = path.back();
    const typename M::Plan pl = M::plan(s, flags_);
    if (kind == E_INVARIANT) {
      int slot, j;
      M::locate(pl, pos, slot, j);
      State x;
      M::apply(s, slot, j, flags_, x);
      path.push_back(x);
      *err_inv = M::check(x, flags_.inv_mask);
    } else if (kind == 0x12) {
      *err_inv = M::check(s, flags_.inv_mask);
    } else if (kind == E_ASSERT && pl.fail_slot >= 0) {
      *err_action = M::slot_action(s, pl.fail_slot);
      *err_self = pl.fail_slot < M::A ? pl.fail_slot
                  : pl.fail_slot < 2 * M::A ? pl.fail_slot - M::A
                                           : M::A + (pl.fail_slot - 2 * M::A);
    }
    tuples.assign(path.size(), std::vector<uint64_t>(M::TUPLE_WORDS));
    for (size_t k = 0; k < path.size(); ++k) M::to_tuple(path[k], tuples[k].data());
    return 0;
  }

  int pack(void* send) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    if (n_ && send_total_ && staged_) {
      // the tiles' staged segments, in tile order per owner
      const unsigned tiles = (unsigned)((n_ + CLAIM_TILE - 1) / CLAIM_TILE);
      hipLaunchKernelGGL(k_shard_gather<M>, dim3(tiles), dim3(256), 0, st_, stage_, stoff_, tcnt_, toff_, tiles,
                         (uint32_t)world_, (Rec*)send, ocscan_level_ ? 1 : 0);
      KC_HIP_TRY(hipGetLastError());
    } else if (n_ && send_total_) {
      if (stage_level_) {
        // (staging overflowed this level: the per-parent owner-major scan
        // that k_shard_pack positions its records with)
        const uint64_t cells = n_ * (uint64_t)world_;
        KC_TRY(grow_buffer(off_, off_cap_, cells, false, st_));
        size_t tmp_bytes = 0;
        const hipcub::TransformInputIterator<uint32_t, Widen8, const uint8_t*> cnt32(cnt_, Widen8());
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt32, off_, (int)cells, st_));
        KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, cnt32, off_, (int)cells, st_));
      }
      hipLaunchKernelGGL(k_shard_pack<M>, dim3((unsigned)((n_ + 255) / 256)), dim3(256), 0, st_,
                         cur_, n_, flags_, (uint32_t)world_, (uint64_t)rank_, off_, repmask_,
                         (Rec*)send, tlc_ ? gpos_cur() : (const uint32_t*)nullptr);
      KC_HIP_TRY(hipGetLastError());
    }
    // else stream-ordered with the caller (set_stream, or the native level
    // loop, which synchronises before it moves the records itself)
    if (own_st_ && !async_pack_) KC_HIP_TRY(hipStreamSynchronize(st_));
    return 0;
  }

  // Claims the received records, settles local and record claims together,
  // emits the winners.  `recv` must be complete (caller's stream synced).
  int insert(const void* recv, uint64_t n, uint64_t* n_new, uint64_t* err_key) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    const Rec* in = (const Rec*)recv;
    *n_new = 0;
    *err_key = ~0ull;
    next_n_ = 0;
    next_cand_ = 0;
    next_cand_est_ = false;
    last_new_ = 0;
    // (an empty level emits nothing: advance must not take the last level's
    // links or plans for this one's)
    emitted_links_ = false;
    if (n_ == 0 && n == 0) return 0;
    if (n >= (1ull << 31) || n_ >= (1ull << 31)) {
      set_error("kc_shard_insert: more than 2^31 records or parents in one level");
      return -ENOMEM;
    }
    if (!spill_) KC_TRY(cs_.reserve(cand_ + n, st_));     // count excludes this level's local inserts (<= cand_)
    const uint32_t succ_level = (uint32_t)level_ + 1;
    const unsigned tiles = (unsigned)((n_ + CLAIM_TILE - 1) / CLAIM_TILE);
    const unsigned rgrid = (unsigned)((n + 255) / 256);
    if (first_) {
      // first-claim mode: the records' CASes (their block counts after this
      // level's own tile counts, which k_claim wrote), one scan, the emit
      const unsigned lt = n_ ? tiles : 0u, rb = n ? rgrid : 0u;
      KC_TRY(grow_buffer(wtot_, wtot_cap_, (uint64_t)lt + rb + 8, true, st_));
      KC_TRY(grow_buffer(woff_, woff_cap_, (uint64_t)lt + rb + 8, false, st_));
      if (n) {
        KC_TRY(grow_buffer(isnew_, isnew_cap_, n, false, st_));
        hipLaunchKernelGGL(k_rec_claim_first<M>, dim3(rgrid), dim3(256), 0, st_, in, n, cs_.t, cs_.nslots, isnew_,
                           wtot_ + lt, d_ctr_, cs_.compact ? 1 : 0);
      }
      hipLaunchKernelGGL(k_win_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, wtot_, lt, rb, woff_, d_ctr_);
      return insert_emit(in, n, true, n_new, err_key);
    }
    if (n) {
      KC_TRY(grow_buffer(rfp_, rfp_cap_, n, false, st_));
      KC_TRY(grow_buffer(flag_, flag_cap_, n, false, st_));
      KC_TRY(grow_buffer(isnew_, isnew_cap_, n, false, st_));
      KC_TRY(grow_buffer(ioff_, ioff_cap_, n, false, st_));
      hipLaunchKernelGGL(k_rec_claim<M>, dim3(rgrid), dim3(256), 0, st_, in, n, cs_.t, cs_.nslots,
                         succ_level, rfp_, flag_, d_ctr_, (int)tlc_);
    }
    // settle pass A (own tiles, records and the tiles' overflow list in one
    // launch), then pass B; n_ = 0 with n > 0 still runs pass A's first
    // workgroup, which resets the error key
    const unsigned lt = n_ ? tiles : 0u, ob = n_ ? SHARD_OVF_BLOCKS : 0u, rb = n ? rgrid : 0u;
    const unsigned sgrid = std::max(lt + rb + ob, 1u);
    // the tile-count path (not with the seen-set spill, whose cold check
    // works on per-parent / per-record offsets): pass B counts each own
    // tile's and each record block's new states, the overflow list's pass B
    // adds its winners to their tiles, one scan positions them all
    const bool tc = tcount_ && !spill_;
    ClaimKeys ck((uint32_t)rank_);
    if (tlc_) {
      if (!(defer_on_ && tc)) {
        set_error("kc_shard_insert: tlc_order needs the deferred frontier");
        return -EINVAL;
      }
      ck.gpos = gpos_cur();
      ck.gbits = gbits_cur_;
      ck.grank = grank_cur_;
    }
    // (one workgroup per own tile: round 5 measured 4 tiles per workgroup
    // slower at R = 8)
    auto settle = [&](int pass, unsigned ob_blocks, uint32_t* wt) {
      const unsigned g = std::max(lt + rb + ob_blocks, 1u);
      if (pass == 0)
        hipLaunchKernelGGL((k_settle_both<M, 0>), dim3(g), dim3(256), 0, st_, lt, rb, n_, cs_.t, cs_.nslots,
                           succ_level, ck, rcount_, rec_fp_, rec_lk_, newmask_, in, n, rfp_, flag_, isnew_, d_ctr_,
                           ovf_, wt);
      else
        hipLaunchKernelGGL((k_settle_both<M, 1>), dim3(g), dim3(256), 0, st_, lt, rb, n_, cs_.t, cs_.nslots,
                           succ_level, ck, rcount_, rec_fp_, rec_lk_, newmask_, in, n, rfp_, flag_, isnew_, d_ctr_,
                           ovf_, wt);
    };
    settle(0, ob, (uint32_t*)nullptr);
    if (tc) {
      KC_TRY(grow_buffer(wtot_, wtot_cap_, (uint64_t)lt + rb + 8, false, st_));
      KC_TRY(grow_buffer(woff_, woff_cap_, (uint64_t)lt + rb + 8, false, st_));
      if (lt + rb) settle(1, 0, wtot_);
      if (n_ && n_ <= FUSE_OVF_SCAN_MAX) {
        hipLaunchKernelGGL(k_ovf_win_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, ovf_, n_, cs_.t, cs_.nslots,
                           succ_level, newmask_, d_ctr_, ck, wtot_, lt, rb, woff_);
      } else {
        if (n_)
          hipLaunchKernelGGL(k_settle_ovf<1>, dim3(SHARD_OVF_BLOCKS), dim3(256), 0, st_, ovf_, n_, (uint64_t)0, cs_.t,
                             cs_.nslots, succ_level, newmask_, d_ctr_, ck, wtot_);
        hipLaunchKernelGGL(k_win_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, wtot_, lt, rb, woff_, d_ctr_);
      }
    } else {
      hipLaunchKernelGGL((k_settle_both<M, 1>), dim3(sgrid), dim3(256), 0, st_, lt, rb, n_, cs_.t,
                         cs_.nslots, succ_level, ck, rcount_, rec_fp_, rec_lk_, newmask_, in, n, rfp_,
                         flag_, isnew_, d_ctr_, ovf_, (uint32_t*)nullptr);
      // positions: this rank's own winners first, then the records'
      KC_TRY(scan_winners(n));
      if (spill_) {
        bool changed = false;
        KC_TRY(spill_check(n, tiles, rgrid, &changed));
        if (changed) KC_TRY(scan_winners(n));
      }
    }
    return insert_emit(in, n, tc, n_new, err_key);
  }

  // The emit half of insert(): the winners' positions are known (woff_ on
  // the tile-count path `tc`, else offsets_ / ioff_).
  int insert_emit(const Rec* in, uint64_t n, bool tc, uint64_t* n_new, uint64_t* err_key) {
    const unsigned rgrid = (unsigned)((n + 255) / 256);
    // capacity: at most one new state per own successor and per record
    // (the deferred frontier: links and parent keys only, sized by the
    // estimate when the level's successor count is one; past it the emit
    // runs again with the exact count)
    const bool links = defer_on_ && tc;
    emitted_links_ = links;
    last_in_ = in;
    const uint64_t bound = cand_ + n;
    if (!links || defer_check_) KC_TRY(grow_buffer(next_, next_cap_, std::max<uint64_t>(bound, 1), false, st_));
    const uint64_t next_gidx = level_base_.back() + n_;
    KC_TRY(grow_buffer(pkeys_, pk_cap_, next_gidx + bound + 1, true, st_));
    if (tlc_) KC_TRY(grow_buffer(gpos_all_, gp_cap_, pk_cap_, true, st_));
    if (links) KC_TRY(grow_buffer(link_next_, link_next_cap_, std::max<uint64_t>(bound, 1), false, st_));
    const unsigned lb = (unsigned)((n_ + 255) / 256), eg = std::max(lb + (n ? rgrid : 0u), 1u);
    const int tail = eg <= SHARD_TAIL_BLOCKS;
    if (links && defer_check_) {
      // (diagnostic) the materialising emit too, into next_ — which the next
      // level's rebuild then compares with — on scratch counters and keys
      if (!d_ctr_dbg_) KC_HIP_TRY(hipMalloc(&d_ctr_dbg_, sizeof(Counters)));
      KC_TRY(grow_buffer(pk_dbg_, pk_dbg_cap_, bound + 1, false, st_));
      hipLaunchKernelGGL(k_shard_emit<M>, dim3(eg), dim3(256), 0, st_, cur_, n_, lb, flags_, (uint64_t)rank_, newmask_,
                         offsets_, in, n, isnew_, ioff_, next_, pk_dbg_, (uint64_t)0, d_ctr_dbg_,
                         (unsigned long long*)nullptr, 0, woff_);
    }
    auto emit = [&]() {
      if (links)
        hipLaunchKernelGGL(k_shard_emit_links<M>, dim3(eg), dim3(256), 0, st_, n_, lb, (uint64_t)rank_,
                           tlc_ ? gpos_cur() : (const uint32_t*)nullptr, newmask_, in, n,
                           isnew_, woff_, link_next_, pkeys_, next_gidx,
                           std::min<uint64_t>(link_next_cap_, pk_cap_ - next_gidx), d_ctr_,
                           reinterpret_cast<unsigned long long*>(h_ctr_), tail);
      else
        hipLaunchKernelGGL(k_shard_emit<M>, dim3(eg), dim3(256), 0, st_, cur_, n_, lb, flags_, (uint64_t)rank_,
                           newmask_, offsets_, in, n, isnew_, ioff_, next_, pkeys_, next_gidx, d_ctr_,
                           reinterpret_cast<unsigned long long*>(h_ctr_), tail,
                           tc ? woff_ : (const uint32_t*)nullptr);
      if (!tail)
        hipLaunchKernelGGL(k_shard_cand, dim3(1), dim3(64), 0, st_, d_ctr_,
                           reinterpret_cast<unsigned long long*>(h_ctr_));
    };
    emit();
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipStreamSynchronize(st_));
    if (links && (h_ctr_->defer_flags & DF_CAPACITY)) {
      const uint64_t need = h_ctr_->level_new;
      KC_TRY(grow_buffer(link_next_, link_next_cap_, need, false, st_));
      KC_TRY(grow_buffer(pkeys_, pk_cap_, next_gidx + need + 1, true, st_));
      if (tlc_) KC_TRY(grow_buffer(gpos_all_, gp_cap_, pk_cap_, true, st_));
      KC_HIP_TRY(hipMemsetAsync(&d_ctr_->defer_flags, 0, 8, st_));
      ++emit_retries_;
      emit();
      KC_HIP_TRY(hipGetLastError());
      KC_HIP_TRY(hipStreamSynchronize(st_));
      if (h_ctr_->defer_flags & DF_CAPACITY) {
        set_error("kc_shard_insert: %llu links do not fit %llu", (unsigned long long)need,
                  (unsigned long long)link_next_cap_);
        return -ENOMEM;
      }
    }
    if (h_ctr_->overflow || h_ctr_->batch_used) {
      set_error("kc_shard_insert: table full or claim protocol violation");
      return -ENOMEM;
    }
    next_n_ = h_ctr_->level_new;
    const uint64_t dc = h_ctr_->cand_total - cand_total_;
    cand_total_ = h_ctr_->cand_total;
    if (links) {
      // successors counted this level: those of this level's rebuilt states
      // (or none: a level k_claim did not rebuild has an exact count already);
      // the next level's, for its buffers, estimated from them
      const uint64_t cur_cand = rebuilt_ ? dc : cand_;
      if (n_ && (rebuilt_ || !cand_est_)) succ_ratio_ = std::max(1.0, (double)cur_cand / (double)n_);
      next_cand_ = next_n_ ? (uint64_t)((double)next_n_ * succ_ratio_ * 1.25) + 4096 : 0;
      next_cand_est_ = true;
    } else {
      next_cand_ = dc;
      next_cand_est_ = false;
    }
    last_new_ = next_n_;
    if (!spill_) cs_.count += next_n_;   // (spill: spill_check counted the hot slots)
    distinct_ += next_n_;
    if (h_ctr_->err_key != ~0ull) *err_key = h_ctr_->err_key;
    *n_new = next_n_;
    if (cfg_.verbose > 1)
      fprintf(stderr, "kc_shard rank %d level %d: insert records %llu new %llu links %d e2 %llx\n", rank_, level_,
              (unsigned long long)n, (unsigned long long)next_n_, (int)links, (unsigned long long)*err_key);
    return 0;
  }

  // Exclusive scans of the own winners' newmask popcounts (offsets_) and the
  // records' isnew flags (ioff_); C->chunk_base / level_new = the totals.
  int scan_winners(uint64_t n) {
    if (n_) KC_TRY(grow_buffer(offsets_, offsets_cap_, n_, false, st_));
    if (n_ <= SHARD_SMALL_SCAN && n <= SHARD_SMALL_SCAN) {
      hipLaunchKernelGGL(k_shard_scan_small, dim3(1), dim3(1024), 0, st_, newmask_, n_, offsets_, isnew_, n, ioff_,
                         d_ctr_);
    } else {
      size_t tmp_bytes = 0;
      if (n_) {
        const hipcub::TransformInputIterator<uint32_t, NewCount, const uint32_t*> newcnt(newmask_, NewCount());
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, newcnt, offsets_, (int)n_, st_));
        KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, newcnt, offsets_, (int)n_, st_));
      }
      if (n) {
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, isnew_, ioff_, (int)n, st_));
        KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, isnew_, ioff_, (int)n, st_));
      }
      hipLaunchKernelGGL(k_shard_base, dim3(1), dim3(64), 0, st_, offsets_, newmask_, n_, ioff_, isnew_, n, d_ctr_);
    }
    return 0;
  }

  // ---- seen-set spill (cfg.seen_hbm_bytes > 0; the engine's scheme,
  // engine.hip spill_setup/spill_flush/spill_check, with whole levels: the
  // sharded level cannot be cut into chunks without cutting every rank's).
  // Budget B per rank: the hot ClaimSet takes the largest power-of-two table
  // of <= B/2 bytes, flushed before a level whose claims might take it past
  // 1/2 load (a level may go on to 7/8: an estimate, not a bound, decides
  // the flush); one arena serves the flush (up to 7/8 of the slots' keys) and
  // the level's cold check (q_max_ queries per window); the rest is the cold
  // runs' directories and filters.
  int spill_setup() {
    if (!cs_.t) {
      const uint64_t B = cfg_.seen_hbm_bytes;
      uint64_t ns = 1ull << 12;
      while (ns * 2 * sizeof(ClaimEntry) <= B / 2) ns *= 2;
      KC_TRY(cs_.init(ns, st_));
      hot_limit_ = ns / 2;
      hot_hard_ = ns / 8 * 7;
      uint64_t arena = hot_hard_ * 8;
      q_max_ = std::max<uint64_t>(256, arena / 48 / 256 * 256);
      const char* qm = getenv("KC_SEEN_QMAX");        // queries per cold-check window (tests: many windows)
      if (qm && atoll(qm) >= 256) q_max_ = std::min<uint64_t>(q_max_, (uint64_t)atoll(qm) / 256 * 256);
      size_t tmp = 0;
      {
        hipcub::DoubleBuffer<uint64_t> k(nullptr, nullptr);
        hipcub::DoubleBuffer<uint64_t> v(nullptr, nullptr);
        KC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k, v, (int)q_max_, 0, 64, st_));
      }
      sp_qtmp_bytes_ = tmp;
      arena = std::max<uint64_t>(arena, q_max_ * 33 + tmp + 1024);
      sp_arena_bytes_ = arena;
      KC_HIP_TRY(hipMalloc(&sp_arena_, arena));
      KC_HIP_TRY(hipMalloc(&d_spctr_, 64));
      KC_HIP_TRY(hipHostMalloc(&h_spctr_, 64));
      const uint64_t used = ns * sizeof(ClaimEntry) + arena;
      if (used + (1ull << 20) > B) {
        set_error("kc_shard: seen_hbm_bytes %llu too small (hot table + scratch need %llu B)",
                  (unsigned long long)B, (unsigned long long)used);
        return -EINVAL;
      }
      ColdSet::Config cc;
      cc.device = cfg_.device;
      cc.meta_hbm_bytes = B - used;
      cc.host_bytes = cfg_.seen_host_bytes;
      cc.dir = spill_dir_;
      const char* wk = getenv("KC_COLD_WINDOW");      // disk-run staging window (keys); tests shrink it
      if (wk && atoll(wk) > 0) cc.window_keys = (uint64_t)atoll(wk);
      const char* bb = getenv("KC_COLD_BLOOM_BITS");  // filter bits per key (0 = no filters; A/B)
      if (bb) cc.bloom_bits = atoi(bb);
      const char* ck = getenv("KC_COLD_CACHE");       // KC_COLD_CACHE=0: no HBM copies of run keys (A/B)
      cc.cache_keys = !(ck && ck[0] == '0');
      KC_TRY(cold_.init(cc));
    } else {
      KC_TRY(cs_.clear(st_));
    }
    cold_.clear();
    sp_flushes_ = sp_queries_ = 0;
    sp_ratio_ = 1.0;
    KC_HIP_TRY(hipMemsetAsync(d_spctr_, 0, 64, st_));
    return 0;
  }

  // Hot table -> one sorted cold run; the table starts over empty.
  int spill_flush() {
    uint64_t* keys = reinterpret_cast<uint64_t*>(sp_arena_);
    KC_HIP_TRY(hipMemsetAsync(d_spctr_ + 1, 0, 8, st_));
    hipLaunchKernelGGL(k_claimset_keys, dim3(table_grid(cs_.nslots)), dim3(256), 0, st_, cs_.t, cs_.nslots, keys,
                       hot_hard_, d_spctr_ + 1);
    KC_HIP_TRY(hipMemcpyAsync(h_spctr_, d_spctr_, 16, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    const uint64_t c = h_spctr_[1];
    if (c > hot_hard_) {
      set_error("kc_shard: hot seen-set holds %llu > %llu fingerprints", (unsigned long long)c,
                (unsigned long long)hot_hard_);
      return -EIO;
    }
    if (c) {
      // sorted in place, the hot table (cleared right after) lending the
      // alternate buffer and the temporary storage
      uint64_t* alt = reinterpret_cast<uint64_t*>(cs_.t);
      const uint64_t tab = cs_.nslots * sizeof(ClaimEntry);
      const uint64_t off = (c * 8 + 255) / 256 * 256;
      hipcub::DoubleBuffer<uint64_t> kb(keys, alt);
      size_t tb = 0;
      KC_HIP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, kb, (int)c, 0, 64, st_));
      if (off + tb > tab) {
        set_error("kc_shard: seen-set flush sort needs %llu B > %llu", (unsigned long long)(off + tb),
                  (unsigned long long)tab);
        return -ENOMEM;
      }
      KC_HIP_TRY(hipcub::DeviceRadixSort::SortKeys(reinterpret_cast<uint8_t*>(cs_.t) + off, tb, kb, (int)c, 0, 64,
                                                   st_));
      KC_TRY(cold_.add_run(kb.Current(), c, st_));
    }
    KC_TRY(cs_.clear(st_));
    cs_.count = 0;
    ++sp_flushes_;
    return 0;
  }

  // The level's winners w.r.t. the hot table (C->level_new after the first
  // scans) against the cold tier; those found lose.  *changed: some did.
  int spill_check(uint64_t n, unsigned tiles, unsigned rgrid, bool* changed) {
    *changed = false;
    KC_HIP_TRY(hipMemcpyAsync(h_spctr_ + 2, &d_ctr_->level_new, 8, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    const uint64_t m = h_spctr_[2];
    cs_.count += m;                   // the hot slots this level filled
    sp_queries_ += m;
    if (cand_) sp_ratio_ = std::min(1.0, (double)m / (double)cand_);
    if (cs_.count > hot_hard_) {
      set_error("kc_shard: one level put %llu fingerprints into a hot seen-set of %llu slots; raise seen_hbm_bytes",
                (unsigned long long)m, (unsigned long long)cs_.nslots);
      return -ENOMEM;
    }
    if (m == 0 || cold_.empty()) return 0;
    uint64_t* qk = reinterpret_cast<uint64_t*>(sp_arena_);
    uint64_t* qk2 = qk + q_max_;
    uint64_t* ql = qk2 + q_max_;
    uint64_t* ql2 = ql + q_max_;
    uint8_t* found = reinterpret_cast<uint8_t*>(ql2 + q_max_);
    uint8_t* tmp = found + (q_max_ + 255) / 256 * 256;
    const unsigned lb = n_ ? tiles : 0u;
    // windows from the last to the first: a winner that loses clears its
    // bit, which would shift the positions of its parent's later winners,
    // so every window is taken before any lower one changes
    const uint64_t nwin = (m + q_max_ - 1) / q_max_;
    for (uint64_t wi = nwin; wi-- > 0;) {
      const uint64_t w0 = wi * q_max_, w1 = std::min(m, w0 + q_max_), c = w1 - w0;
      hipLaunchKernelGGL(k_shard_spill_queries<M>, dim3(std::max(lb + rgrid, 1u)), dim3(256), 0, st_, cur_, n_, lb,
                         flags_, newmask_, offsets_, n, rfp_, isnew_, ioff_, d_ctr_, w0, w1, qk, ql);
      hipcub::DoubleBuffer<uint64_t> kb(qk, qk2);
      hipcub::DoubleBuffer<uint64_t> vb(ql, ql2);
      size_t tb = sp_qtmp_bytes_;
      KC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kb, vb, (int)c, 0, 64, st_));
      KC_HIP_TRY(hipMemsetAsync(found, 0, c, st_));
      KC_TRY(cold_.probe(kb.Current(), c, found, d_spctr_, st_));
      hipLaunchKernelGGL(k_shard_spill_apply, dim3((unsigned)((c + 255) / 256)), dim3(256), 0, st_, kb.Current(),
                         vb.Current(), found, c, newmask_, isnew_, cs_.t, cs_.nslots, d_ctr_);
      KC_HIP_TRY(hipGetLastError());
    }
    *changed = true;
    return 0;
  }

  // ---- device-driven narrow levels (shard_narrow.h)
  int sn_setup(uint32_t cap) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    sn_cap_ = std::max<uint32_t>(1, std::min<uint32_t>(cap, SN_SLOT_MAX));
    KC_HIP_TRY(hipMalloc(&d_snc_, sizeof(SNCtl)));
    KC_HIP_TRY(hipHostMalloc(&h_snc_, sizeof(SNCtl)));
    KC_HIP_TRY(hipMalloc(&d_sns_, sizeof(SNScratch)));
    KC_HIP_TRY(hipMalloc(&sn_send_, (uint64_t)world_ * sn_slot_bytes()));
    KC_HIP_TRY(hipMalloc(&sn_recv_, (uint64_t)world_ * sn_slot_bytes()));
    KC_HIP_TRY(hipMemset(d_snc_, 0, sizeof(SNCtl)));
    KC_HIP_TRY(hipMemset(sn_send_, 0, (uint64_t)world_ * sn_slot_bytes()));
    KC_HIP_TRY(hipMemset(sn_recv_, 0, (uint64_t)world_ * sn_slot_bytes()));
    return 0;
  }
  uint64_t sn_slot_bytes() const override { return (uint64_t)(sn_cap_ + 1) * sizeof(Rec); }
  void* sn_send() override { return sn_send_; }
  void* sn_recv() override { return sn_recv_; }

  // A batch's control block.  It is written whatever happens: when a buffer
  // cannot be grown the block says "failed", so this rank's next level stops
  // every rank (through its headers) instead of running on short buffers.
  int sn_begin(uint64_t status_new, uint64_t status_err, int batch) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    int rc = 0;
    if (status_new != n_) {
      set_error("kc_shard narrow: status %llu is not the frontier's width %llu", (unsigned long long)status_new,
                (unsigned long long)n_);
      rc = -EIO;
    }
    const uint64_t in = (uint64_t)(world_ - 1) * sn_cap_;
    const uint64_t per = SN_CAND_MAX + in + 1;           // new states one level may add, at most
    const uint64_t bufs = std::max<uint64_t>(SN_MAX, per);
    const uint64_t base = level_base_.back();
    if (!rc) rc = grow_buffer(cur_, cur_cap_, bufs, true, st_);
    if (!rc) rc = grow_buffer(next_, next_cap_, bufs, false, st_);
    if (!rc) rc = grow_buffer(pkeys_, pk_cap_, base + n_ + (uint64_t)batch * per + 1, true, st_);
    // ClaimSet room for the batch: a few times the first level's bound, not
    // the batch's worst case (that forced ~2M entries on every model; ADVICE
    // r4).  The device stops a level whose claims might not fit (room below,
    // sn_local_stop: SN_STOP, the counted path takes it), so a reserve that
    // finds no memory is not a failure either (the table is unchanged then).
    if (!rc && cs_.reserve(std::min<uint64_t>((uint64_t)batch * per, 4 * (cand_ + in + 1) + (1u << 16)), st_) < 0)
      (void)hipGetLastError();
    SNCtl& h = *h_snc_;
    memset(&h, 0, offsetof(SNCtl, lwidths));
    h.active = 1;
    h.level = (uint32_t)level_;
    h.world = (uint32_t)world_;
    h.rank = (uint32_t)rank_;
    h.slot_cap = sn_cap_;
    h.stop_level = (uint32_t)cfg_.max_levels;
    h.n = n_;
    h.level_gidx = base;
    h.cand = cand_;
    h.err[(level_ - 1) & 1] = status_err;
    h.err[level_ & 1] = ~0ull;
    if (rc) {
      h.fail = 1;           // (buf_cap = room = par_cap = 0: nothing runs)
    } else {
      h.room = cs_.capacity() / 2 > cs_.count ? cs_.capacity() / 2 - cs_.count : 0;
      h.buf_cap = std::min(cur_cap_, next_cap_);
      h.par_cap = pk_cap_;
    }
    sn_n0_ = n_;
    KC_HIP_TRY(hipMemcpyAsync(d_snc_, h_snc_, offsetof(SNCtl, lwidths), hipMemcpyHostToDevice, st_));
    KC_HIP_TRY(hipMemsetAsync(d_sns_->lt, 0, sizeof(d_sns_->lt), st_));
    return rc;
  }
  int sn_pre(uint32_t lev, bool fail) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    if (fail) hipLaunchKernelGGL(k_sn_fail, dim3(1), dim3(64), 0, st_, d_snc_);
    hipLaunchKernelGGL(k_sn_expand<M>, dim3(SN_XWG), dim3(SN_THREADS), 0, st_, cur_, next_, flags_,
                       cfg_.check_deadlock, lev, d_snc_, d_sns_);
    if (world_ > 1)
      hipLaunchKernelGGL(k_sn_pack<M>, dim3(SN_PWG), dim3(SN_THREADS), 0, st_, cur_, next_, flags_, lev, d_snc_,
                         d_sns_, sn_send_);
    KC_HIP_TRY(hipGetLastError());
    return 0;
  }
  int sn_post(uint32_t lev) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    const unsigned rgrid = world_ > 1 ? (unsigned)(((uint64_t)world_ * sn_cap_ + SN_THREADS - 1) / SN_THREADS) : 0u;
    if (world_ > 1)
      hipLaunchKernelGGL(k_sn_recv<M>, dim3(rgrid), dim3(SN_THREADS), 0, st_, lev, d_snc_, d_sns_, sn_recv_, d_ctr_);
    hipLaunchKernelGGL(k_sn_claim<M>, dim3(SN_CWG + rgrid), dim3(SN_THREADS), 0, st_, lev, d_snc_, d_sns_, sn_recv_,
                       cs_.t, cs_.nslots, d_ctr_, cs_.word_shift());
    hipLaunchKernelGGL(k_sn_emit<M>, dim3(SN_EWG + rgrid), dim3(SN_THREADS), 0, st_, cur_, next_, flags_, lev, d_snc_,
                       d_sns_, sn_recv_, pkeys_, d_ctr_);
    KC_HIP_TRY(hipGetLastError());
    return 0;
  }
  int sn_end(SNOut* out) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    KC_HIP_TRY(hipMemcpyAsync(h_snc_, d_snc_, sizeof(SNCtl), hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, kCtrHead, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    const SNCtl& h = *h_snc_;
    // (the outcome is filled in before a failure is reported: the caller
    // keeps in step with its peers on it, shard_driver.hip)
    out->filled = true;
    out->levels = (int)h.levels;
    out->reason = h.active ? SN_RUN : h.reason;
    out->widths.assign(h.gwidths, h.gwidths + std::min<uint32_t>(h.levels, KC_MAX_LEVELS));
    uint64_t w = sn_n0_;
    for (uint32_t k = 0; k < h.levels; ++k) {
      level_base_.push_back(level_base_.back() + w);
      w = k < (uint32_t)KC_MAX_LEVELS ? h.lwidths[k] : 0;
    }
    cs_.count += h.new_total;
    distinct_ += h.new_total;
    level_ = (int)h.level;
    n_ = h.n;
    cand_ = h.cand;
    if (h.levels & 1) {
      std::swap(cur_, next_);
      std::swap(cur_cap_, next_cap_);
    }
    out->status_new = n_;
    out->status_err = h.err[(h.level - 1) & 1];
    out->sent = h.sent_total;
    if (h_ctr_->overflow) {
      set_error("kc_shard narrow: a full level table or ClaimSet, or a header of another level");
      return -ENOMEM;
    }
    return 0;
  }

  int advance() override {
    level_base_.push_back(level_base_.back() + n_);
    std::swap(cur_, next_);
    std::swap(cur_cap_, next_cap_);
    if (emitted_links_) {
      // the new frontier is links into the old one (now next_) and into the
      // receive buffer; this level's plans become the previous level's
      std::swap(link_cur_, link_next_);
      std::swap(link_cur_cap_, link_next_cap_);
      std::swap(pc_cur_, pc_prev_);
      std::swap(pc_cur_cap_, pc_prev_cap_);
      prev_rec_ = last_in_;
      cur_deferred_ = next_n_ > 0;
      emitted_links_ = false;
    }
    if (tlc_) {
      std::swap(gbits_cur_, gbits_next_);
      std::swap(gbits_cur_cap_, gbits_next_cap_);
      std::swap(grank_cur_, grank_next_);
      std::swap(grank_cur_cap_, grank_next_cap_);
    }
    n_ = next_n_;
    cand_ = next_cand_;
    cand_est_ = next_cand_est_;
    next_cand_ = 0;
    next_cand_est_ = false;
    ++level_;
    return 0;
  }

  void set_deferred(bool on) override { defer_on_ = on && !spill_ && tcount_; }
  uint64_t defer_error() const override { return defer_err_; }
  void drop_last_insert() override {
    distinct_ -= last_new_;
    last_new_ = 0;
  }
  int drop_last_expand() override {
    if (!gen_snap_ok_) return 0;
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    if (n_)
      hipLaunchKernelGGL(k_undo_gen<M>, dim3((unsigned)((n_ + 255) / 256)), dim3(256), 0, st_, cur_, pc_cur_, n_, d_ctr_);
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipStreamSynchronize(st_));
    gen_snap_ok_ = false;
    return 0;
  }
  int materialize(uint64_t* derr) override {
    *derr = ~0ull;
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    if (!cur_deferred_ || n_ == 0) {
      cur_deferred_ = false;
      return 0;
    }
    KC_TRY(grow_buffer(cur_, cur_cap_, n_, false, st_));
    DeferArgs df;
    df.prev = next_;
    df.link = link_cur_;
    df.prev_rec = prev_rec_;
    df.out = cur_;
    df.prev_counts = pc_prev_;
    if (tlc_) df.prev_gpos = gpos_prev();
    KC_HIP_TRY(hipMemsetAsync(&d_ctr_->defer_err, 0xff, 8, st_));
    if (tlc_)
      hipLaunchKernelGGL((k_shard_materialize<M, true>), dim3((unsigned)((n_ + 255) / 256)), dim3(256), 0, st_, df, n_,
                         flags_, (uint64_t)rank_, d_ctr_);
    else
      hipLaunchKernelGGL((k_shard_materialize<M, false>), dim3((unsigned)((n_ + 255) / 256)), dim3(256), 0, st_, df,
                         n_, flags_, (uint64_t)rank_, d_ctr_);
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, sizeof(Counters), hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    cur_deferred_ = false;
    ++deferred_levels_;
    const uint64_t tot = h_ctr_->next_cand();      // (the stripes: materialize added this level's successors)
    cand_ = tot - cand_total_;
    cand_total_ = tot;
    cand_est_ = false;
    if (n_) succ_ratio_ = std::max(1.0, (double)cand_ / (double)n_);
    *derr = h_ctr_->defer_err;
    return 0;
  }

  bool tlc() const override { return tlc_; }
  const uint32_t* gpos_cur() const { return gpos_all_ + level_base_.back(); }
  const uint32_t* gpos_prev() const {
    return gpos_all_ + (level_base_.size() >= 2 ? level_base_[level_base_.size() - 2] : 0);
  }
  int tlc_masks(uint64_t W, uint32_t** mask) override {
    *mask = nullptr;
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    if (!tlc_ || W >= (1ull << 31)) {
      set_error("kc_shard tlc_masks: %s", tlc_ ? "a level of 2^31 states or more" : "not in TLC order");
      return -EINVAL;
    }
    KC_TRY(grow_buffer(wmask_, wmask_cap_, W, false, st_));
    KC_HIP_TRY(hipMemsetAsync(wmask_, 0, W * 4, st_));
    const uint64_t next_gidx = level_base_.back() + n_;
    if (next_n_)
      hipLaunchKernelGGL(k_tlc_mask, dim3((unsigned)((next_n_ + 255) / 256)), dim3(256), 0, st_, pkeys_ + next_gidx,
                         next_n_, wmask_, W, d_ctr_);
    KC_HIP_TRY(hipGetLastError());
    *mask = wmask_;
    return 0;
  }
  int tlc_order(uint64_t W) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    // (the next level has at most 32 W states: W + 1 bitmap words)
    const uint64_t words = W + 1;
    KC_TRY(grow_buffer(gbits_next_, gbits_next_cap_, words, false, st_));
    KC_TRY(grow_buffer(grank_next_, grank_next_cap_, words, false, st_));
    KC_TRY(grow_buffer(wbase_, wbase_cap_, W, false, st_));
    KC_HIP_TRY(hipMemsetAsync(gbits_next_, 0, words * 4, st_));
    size_t tmp_bytes = 0;
    const hipcub::TransformInputIterator<uint32_t, NewCount, const uint32_t*> wc(wmask_, NewCount());
    KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, wc, wbase_, (int)W, st_));
    KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
    KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, wc, wbase_, (int)W, st_));
    const uint64_t nn = next_n_, next_gidx = level_base_.back() + n_;
    const unsigned g = (unsigned)((nn + 255) / 256);
    if (nn) {
      KC_TRY(grow_buffer(gnew_, gnew_cap_, nn, false, st_));
      hipLaunchKernelGGL(k_tlc_pos, dim3(g), dim3(256), 0, st_, pkeys_ + next_gidx, nn, wmask_, wbase_, gnew_,
                         gbits_next_);
    }
    const hipcub::TransformInputIterator<uint32_t, NewCount, const uint32_t*> bc(gbits_next_, NewCount());
    KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, bc, grank_next_, (int)words, st_));
    KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
    KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, bc, grank_next_, (int)words, st_));
    if (nn) {
      KC_TRY(grow_buffer(link_tmp_, link_tmp_cap_, std::max(nn, link_next_cap_), false, st_));
      KC_TRY(grow_buffer(pk_tmp_, pk_tmp_cap_, nn, false, st_));
      hipLaunchKernelGGL(k_tlc_perm, dim3(g), dim3(256), 0, st_, nn, gnew_, gbits_next_, grank_next_, link_next_,
                         pkeys_ + next_gidx, link_tmp_, pk_tmp_, gpos_all_ + next_gidx);
      KC_HIP_TRY(hipMemcpyAsync(pkeys_ + next_gidx, pk_tmp_, nn * 8, hipMemcpyDeviceToDevice, st_));
      std::swap(link_next_, link_tmp_);
      std::swap(link_next_cap_, link_tmp_cap_);
    }
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipStreamSynchronize(st_));
    KC_HIP_TRY(hipMemcpy(h_ctr_, d_ctr_, kCtrHead, hipMemcpyDeviceToHost));
    if (h_ctr_->overflow) {
      set_error("kc_shard tlc_order: a parent key outside its level");
      return -EIO;
    }
    return 0;
  }
  int tlc_locate(int level, uint64_t G, uint64_t* idx, bool* found) override {
    *found = false;
    if (!tlc_ || level < 1 || level > (int)level_base_.size()) {
      set_error("kc_shard tlc_locate: bad level %d", level);
      return -EINVAL;
    }
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    const uint64_t b = level_base_[level - 1];
    const uint64_t cnt = level < (int)level_base_.size() ? level_base_[level] - b : n_;
    // (a level's G values are sorted: tlc_order)
    uint64_t lo = 0, hi = cnt;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      uint32_t v = 0;
      KC_HIP_TRY(hipMemcpy(&v, gpos_all_ + b + mid, 4, hipMemcpyDeviceToHost));
      if ((uint64_t)v < G) lo = mid + 1; else hi = mid;
    }
    if (lo < cnt) {
      uint32_t v = 0;
      KC_HIP_TRY(hipMemcpy(&v, gpos_all_ + b + lo, 4, hipMemcpyDeviceToHost));
      if ((uint64_t)v == G) {
        *idx = lo;
        *found = true;
      }
    }
    return 0;
  }

  int parent_key(int level, uint64_t idx, uint64_t* key) override {
    if (level < 1 || level > (int)level_base_.size()) {
      set_error("kc_shard_parent_key: bad level %d", level);
      return -EINVAL;
    }
    const uint64_t g = level_base_[level - 1] + idx;
    KC_HIP_TRY(hipMemcpy(key, pkeys_ + g, 8, hipMemcpyDeviceToHost));
    return 0;
  }

  int frontier_tuple(uint64_t idx, uint64_t* out) override {
    if (idx >= n_) { set_error("kc_shard_frontier_tuple: index"); return -EINVAL; }
    State s;
    KC_HIP_TRY(hipMemcpy(&s, cur_ + idx, sizeof(State), hipMemcpyDeviceToHost));
    M::to_tuple(s, out);
    return M::TUPLE_WORDS;
  }

  int result(kc_result* r) override {
    KC_HIP_TRY(hipMemcpy(h_ctr_, d_ctr_, sizeof(Counters), hipMemcpyDeviceToHost));
    memset(r, 0, sizeof *r);
    uint64_t gen = 0;
    for (int a = 0; a < A_COUNT; ++a) {
      r->act_gen[a] = h_ctr_->act_gen(a);
      r->act_dist[a] = h_ctr_->act_dist(a);
      gen += r->act_gen[a];
    }
    r->init = gen_init_;
    r->generated = gen;                 // successors generated by this rank's parents
    r->distinct = distinct_;
    r->fpset_slots = cs_.capacity();
    if (spill_) {
      ColdStats cst;
      cold_.stats(&cst);
      unsigned long long hits = 0;
      KC_HIP_TRY(hipMemcpy(&hits, d_spctr_, 8, hipMemcpyDeviceToHost));
      r->seen_flushes = sp_flushes_;
      r->seen_cold_fps = cst.keys;
      r->seen_cold_runs = cst.runs;
      r->seen_cold_queries = sp_queries_;
      r->seen_cold_hits = hits;
      r->seen_merges = cst.merges;
      r->seen_disk_bytes = cst.disk_written;
    }
    r->fpset_probes = h_ctr_->probes();
    r->batch_inserts = h_ctr_->settles();
    r->nlevels = level_;
    r->claim_mode = first_ ? 1 : tlc_ ? 2 : 0;
    r->deferred_states = deferred_states_;
    return 0;
  }

 private:
  void release() {
    (void)hipSetDevice(cfg_.device);
    cs_.release();
    for (void* p : {(void*)cur_, (void*)next_, (void*)pkeys_, (void*)cnt_, (void*)off_,
                    (void*)ovf_fp_, (void*)ovf_lk_, (void*)ovf_tile_, (void*)d_ovf_cnt_,
                    (void*)repmask_, (void*)newmask_, (void*)offsets_, (void*)rcount_, (void*)rec_fp_,
                    (void*)rec_lk_, (void*)rfp_, (void*)flag_, (void*)isnew_, (void*)ioff_,
                    (void*)scan_tmp_, (void*)d_ctr_, (void*)d_owner_base_, (void*)stage_, (void*)d_stage_cur_,
                    (void*)tcnt_, (void*)toff_, (void*)stoff_, (void*)ocsum_, (void*)wtot_, (void*)woff_, (void*)link_cur_,
                    (void*)link_next_, (void*)pc_cur_, (void*)pc_prev_, (void*)d_dchk_, (void*)d_ctr_dbg_,
                    (void*)pk_dbg_, (void*)gpos_all_, (void*)gbits_cur_, (void*)grank_cur_, (void*)gbits_next_,
                    (void*)grank_next_, (void*)wmask_, (void*)wbase_, (void*)gnew_, (void*)link_tmp_,
                    (void*)pk_tmp_})
      if (p) (void)hipFree(p);
    if (h_ctr_) (void)hipHostFree(h_ctr_);
    if (h_exp_) (void)hipHostFree(h_exp_);
    if (h_owner_base_) (void)hipHostFree(h_owner_base_);
    for (void* p : {(void*)d_snc_, (void*)d_sns_, (void*)sn_send_, (void*)sn_recv_})
      if (p) (void)hipFree(p);
    if (h_snc_) (void)hipHostFree(h_snc_);
    if (sp_arena_) (void)hipFree(sp_arena_);
    if (d_spctr_) (void)hipFree(d_spctr_);
    if (h_spctr_) (void)hipHostFree(h_spctr_);
    for (auto& e : ev_)
      if (e) (void)hipEventDestroy(e);
    if (st_ && own_st_) (void)hipStreamDestroy(st_);
  }

  kc_model_config cfg_;
  int rank_, world_;
  Flags flags_{};
  hipStream_t st_ = nullptr;
  bool own_st_ = true;
  DevClaimSet cs_;
  State *cur_ = nullptr, *next_ = nullptr;
  uint64_t cur_cap_ = 0, next_cap_ = 0;
  unsigned long long* pkeys_ = nullptr;
  uint64_t pk_cap_ = 0;
  // expand: owner counts / scan, remote representatives, local claim tiles
  uint8_t* cnt_ = nullptr;
  uint32_t *off_ = nullptr, *repmask_ = nullptr, *newmask_ = nullptr, *offsets_ = nullptr;
  uint64_t cnt_cap_ = 0, off_cap_ = 0, rm_cap_ = 0, mask_cap_ = 0, offsets_cap_ = 0;
  unsigned int *rcount_ = nullptr, *rec_lk_ = nullptr;
  unsigned long long* rec_fp_ = nullptr;
  uint64_t rcount_cap_ = 0, rec_fp_cap_ = 0, rec_lk_cap_ = 0;
  CandOvf ovf_{};
  unsigned long long* ovf_fp_ = nullptr;
  unsigned int *ovf_lk_ = nullptr, *ovf_tile_ = nullptr;
  uint64_t ovf_fp_cap_ = 0, ovf_lk_cap_ = 0, ovf_tile_cap_ = 0;
  unsigned long long* d_ovf_cnt_ = nullptr;
  // insert: per received record
  unsigned long long* rfp_ = nullptr;
  unsigned int* flag_ = nullptr;
  uint32_t *isnew_ = nullptr, *ioff_ = nullptr;
  uint64_t rfp_cap_ = 0, flag_cap_ = 0, isnew_cap_ = 0, ioff_cap_ = 0;
  uint8_t* scan_tmp_ = nullptr;
  uint64_t scan_cap_ = 0;
  // record staging (ShardArgs::stage; world > 1)
  Rec* stage_ = nullptr;
  uint64_t stage_cap_ = 0;
  unsigned long long* d_stage_cur_ = nullptr;
  uint32_t *tcnt_ = nullptr, *toff_ = nullptr;
  uint64_t tcnt_cap_ = 0, toff_cap_ = 0;
  // owner x chunk sums of the staged record counts (k_owner_cscan; zeroed at
  // allocation and by each scan); KC_CHUNK_SCAN=0: k_owner_tscan per tile
  bool ocscan_ = true, ocscan_level_ = false;
  uint32_t* ocsum_ = nullptr;
  uint64_t ocsum_cap_ = 0;
  unsigned long long* stoff_ = nullptr;
  uint64_t stoff_cap_ = 0;
  bool stage_on_ = true, stage_level_ = false, staged_ = false;
  bool first_ = false;    // first-claim mode (cfg.first_claim)
  uint64_t stage_fallbacks_ = 0;       // levels packed the old way (staging estimate exceeded)
  double rec_ratio_ = 1.0;             // records sent per parent, last level (the staging estimate)
  // the tile-count insert path: own tiles' and record blocks' new-state counts, their scan
  bool tcount_ = true;
  uint32_t *wtot_ = nullptr, *woff_ = nullptr;
  uint64_t wtot_cap_ = 0, woff_cap_ = 0;
  // the deferred frontier (set_deferred; the native loop's counted levels)
  bool defer_on_ = false;
  bool cur_deferred_ = false;        // cur_ not built: link_cur_ into next_ (the previous frontier) / prev_rec_
  bool emitted_links_ = false;       // the last insert emitted links (advance swaps them in)
  bool rebuilt_ = false;             // this level's k_claim rebuilt its parents
  bool cand_est_ = false, next_cand_est_ = false;   // cand_ / next_cand_ estimated, not counted
  unsigned long long *link_cur_ = nullptr, *link_next_ = nullptr;
  uint64_t link_cur_cap_ = 0, link_next_cap_ = 0;
  unsigned long long *pc_cur_ = nullptr, *pc_prev_ = nullptr;   // plans of this / the previous level's parents
  uint64_t pc_cur_cap_ = 0, pc_prev_cap_ = 0;
  const Rec* prev_rec_ = nullptr;    // the receive buffer the links point into
  const Rec* last_in_ = nullptr;     // the last insert's receive buffer
  uint64_t defer_err_ = ~0ull;       // expand_done: the rebuild's invariant key
  double succ_ratio_ = 5.0;          // successors per state, last counted (the estimates)
  bool gen_snap_ok_ = false;        // drop_last_expand can undo the last expand's act_gen
  uint64_t last_new_ = 0;            // the last insert's new states (drop_last_insert)
  uint64_t deferred_levels_ = 0, emit_retries_ = 0;
  uint64_t deferred_states_ = 0;   // this run's states rebuilt inside k_claim (kc_result.deferred_states)
  bool defer_check_ = false;         // KC_DEFER_CHECK (diagnostic)
  // TLC order (tlc_*): G of every state (parallel to pkeys_), the current /
  // next level's G -> local index map, the per-parent masks and scratch
  bool tlc_ = false;
  uint32_t* gpos_all_ = nullptr;
  uint64_t gp_cap_ = 0;
  uint32_t *gbits_cur_ = nullptr, *grank_cur_ = nullptr, *gbits_next_ = nullptr, *grank_next_ = nullptr;
  uint64_t gbits_cur_cap_ = 0, grank_cur_cap_ = 0, gbits_next_cap_ = 0, grank_next_cap_ = 0;
  uint32_t *wmask_ = nullptr, *wbase_ = nullptr, *gnew_ = nullptr;
  uint64_t wmask_cap_ = 0, wbase_cap_ = 0, gnew_cap_ = 0;
  unsigned long long *link_tmp_ = nullptr, *pk_tmp_ = nullptr;
  uint64_t link_tmp_cap_ = 0, pk_tmp_cap_ = 0;
  unsigned long long* d_dchk_ = nullptr;
  Counters* d_ctr_dbg_ = nullptr;
  unsigned long long* pk_dbg_ = nullptr;
  uint64_t pk_dbg_cap_ = 0;
  uint64_t* d_owner_base_ = nullptr;   // per-owner record totals (device / pinned host)
  uint64_t* h_owner_base_ = nullptr;
  Counters *d_ctr_ = nullptr, *h_ctr_ = nullptr;
  Counters* h_exp_ = nullptr;          // pinned: expand's level head (kCtrHead bytes)
  uint64_t n_ = 0, next_n_ = 0, send_total_ = 0, gen_init_ = 0;
  uint64_t cand_ = 0, next_cand_ = 0, cand_total_ = 0;   // successors of the frontier
  uint64_t init_err_ = ~0ull;
  uint64_t init_key_ = ~0ull;       // init_error(): init_err_ as init() found it
  // expand_dev -> expand_done: the Init-state key taken, nothing launched
  // that needs a sync, no claims this level
  uint64_t dev_init_err_ = ~0ull;
  bool dev_empty_ = false, dev_zero_ = false;
  int level_ = 0;
  std::vector<uint64_t> level_base_;
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool async_pack_ = false;
  // device-driven narrow levels
  SNCtl *d_snc_ = nullptr, *h_snc_ = nullptr;
  SNScratch* d_sns_ = nullptr;
  uint64_t *sn_send_ = nullptr, *sn_recv_ = nullptr;
  uint32_t sn_cap_ = SN_SLOT_DEFAULT;
  uint64_t sn_n0_ = 0;
  double claim_ms_ = 0;
  uint64_t claim_launches_ = 0, claim_parents_ = 0;
  uint64_t distinct_ = 0;           // new states this rank owns (cs_.count is the hot table's, spilling)
  // seen-set spill
  bool spill_ = false;
  std::string spill_dir_;
  ColdSet cold_;
  uint64_t hot_limit_ = 0, hot_hard_ = 0, q_max_ = 0;
  uint8_t* sp_arena_ = nullptr;
  uint64_t sp_arena_bytes_ = 0;
  size_t sp_qtmp_bytes_ = 0;
  unsigned long long *d_spctr_ = nullptr, *h_spctr_ = nullptr;   // [0] cold hits, [1] flush count, [2] m
  uint64_t sp_flushes_ = 0, sp_queries_ = 0;
  double sp_ratio_ = 1.0;           // hot slots filled per successor, last level
};

std::unique_ptr<ShardBase> make_shard(const kc_model_config& cfg, int rank, int world) {
#define KC_MAKE(a, b, c)                                                   \
  if (cfg.nc == a && cfg.np == b && cfg.ns == c)                           \
    return std::unique_ptr<ShardBase>(new ShardT<Model<a, b, c>>(cfg, rank, world));
  KC_FOR_EACH_MODEL(KC_MAKE)
#undef KC_MAKE
  return nullptr;
}

}  // namespace kc

using namespace kc;

extern "C" {

int kc_shard_create(const kc_model_config* cfg, int rank, int world, kc_shard** out) {
  if (!cfg || !out) { set_error("kc_shard_create: NULL"); return -EINVAL; }
  *out = nullptr;
  auto impl = make_shard(*cfg, rank, world);
  if (!impl) {
    set_error("kc_shard_create: unsupported model nc=%d np=%d ns=%d", cfg->nc, cfg->np, cfg->ns);
    return -EINVAL;
  }
  KC_TRY(impl->setup());
  *out = new kc_shard{std::move(impl)};
  return 0;
}
void kc_shard_destroy(kc_shard* s) { delete s; }
int kc_shard_init(kc_shard* s, uint64_t* n_local) {
  if (!s || !n_local) { set_error("kc_shard_init: NULL"); return -EINVAL; }
  return s->impl->init(n_local);
}

int kc_shard_init_error(kc_shard* s, uint64_t* key) {
  if (!s || !key) { set_error("kc_shard_init_error: NULL"); return -EINVAL; }
  *key = s->impl->init_error();
  return 0;
}
int kc_shard_set_stream(kc_shard* s, void* stream) {
  if (!s) { set_error("kc_shard_set_stream: NULL"); return -EINVAL; }   // stream 0: the default stream
  return s->impl->set_stream((hipStream_t)stream);
}
int kc_shard_expand(kc_shard* s, uint64_t* counts, uint64_t* err_key) {
  if (!s || !counts || !err_key) { set_error("kc_shard_expand: NULL"); return -EINVAL; }
  return s->impl->expand(counts, err_key);
}
uint64_t kc_shard_record_bytes(kc_shard* s) { return s ? s->impl->record_bytes() : 0; }
int kc_shard_pack(kc_shard* s, void* send_dev) {
  if (!s) { set_error("kc_shard_pack: NULL"); return -EINVAL; }
  return s->impl->pack(send_dev);
}
int kc_shard_insert(kc_shard* s, const void* recv_dev, uint64_t n_records, uint64_t* n_new,
                    uint64_t* err_key) {
  if (!s || !n_new || !err_key) { set_error("kc_shard_insert: NULL"); return -EINVAL; }
  return s->impl->insert(recv_dev, n_records, n_new, err_key);
}
int kc_shard_advance(kc_shard* s) {
  if (!s) { set_error("kc_shard_advance: NULL"); return -EINVAL; }
  return s->impl->advance();
}
int kc_shard_parent_key(kc_shard* s, int level, uint64_t idx, uint64_t* key) {
  if (!s || !key) { set_error("kc_shard_parent_key: NULL"); return -EINVAL; }
  return s->impl->parent_key(level, idx, key);
}
int kc_shard_frontier_tuple(kc_shard* s, uint64_t idx, uint64_t* out) {
  if (!s || !out) { set_error("kc_shard_frontier_tuple: NULL"); return -EINVAL; }
  return s->impl->frontier_tuple(idx, out);
}
int kc_shard_result(kc_shard* s, kc_result* r) {
  if (!s || !r) { set_error("kc_shard_result: NULL"); return -EINVAL; }
  return s->impl->result(r);
}
int kc_shard_claim_times(kc_shard* s, double* ms, uint64_t* launches, uint64_t* parents) {
  if (!s || !ms || !launches || !parents) { set_error("kc_shard_claim_times: NULL"); return -EINVAL; }
  s->impl->claim_times(ms, launches, parents);
  return 0;
}
int kc_shard_owner(uint64_t fp, int world) {
  if (world < 1) return -EINVAL;
  return (int)(((unsigned __int128)((fp & 0x7fffffffffffffffull) << 1) * (uint64_t)world) >> 64);
}

}  // extern "C"
