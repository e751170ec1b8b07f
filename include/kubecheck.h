/*
 * kubecheck.h — C ABI of libkubecheck.so, the MI355X-native BFS model
 * checker for KubeAPI.tla (JohnStrunk/tla-kubernetes).
 *
 * Plain C, plain pointers and sizes; no torch, no C++ types.  Every entry
 * point returns 0 on success or a negative errno-style code (-EINVAL bad
 * argument, -ENOMEM device memory / table full, -EIO HIP failure, -ENODEV
 * no GPU) and leaves a thread-local message for kc_last_error().  Nothing
 * aborts and nothing throws across this boundary.
 *
 * What each group replaces in the reference's hot path.  The reference's
 * checker is TLC 2.16 (tla2tools.jar, rev cdddf55; KubeAPI.toolbox/Model_1/
 * MC.out:2), a third-party Java jar not vendored in the reference; its
 * plugin seams are named in the recorded run's banner (MC.out:5:
 * "OffHeapDiskFPSet, DiskStateQueue") and selected by TLC system properties
 * [ext-TLC].  INTEGRATION.md shows the Java (Panama FFM) binding a TLC
 * maintainer would add over these symbols.
 *
 *   kc_fpset_*   tlc2.tool.fp.FPSet (abstract class; impl chosen by
 *                -Dtlc2.tool.fp.FPSet.impl=<class>):
 *                  put(long fp)      -> boolean "was already present"
 *                  contains(long fp) -> boolean
 *                  size()            -> long
 *                  checkFPs()        -> double (collision estimate, MC.out:42)
 *                  init/close        -> create/destroy
 *                Batched: TLC's put() is per-state; the shim batches puts
 *                from all -workers threads (flat combining).  Within one
 *                batch, equal fps resolve exactly as sequential puts would:
 *                the lowest index gets seen=0, every later one seen=1.
 *                Fingerprints are normalised like TLC's disk FPSets: the
 *                MSB is ignored and 0 is mapped to 1 (documented merge).
 *   kc_squeue_*  tlc2.tool.queue.StateQueue (MC.out:5 "DiskStateQueue"):
 *                FIFO of packed states in HBM (enqueue/dequeue batches).
 *   kc_engine_*  tlc2.TLC's BFS ModelChecker run over Model_1-style inputs
 *                (MC.cfg:1-16, MC.tla:1-16, KubeAPI___Model_1.launch):
 *                counts, depth, per-action coverage and counterexamples.
 *   kc_spec_*    host-side access to the lowered spec (canonical tuples) —
 *                used for trace replay and by the parity tests.
 */
#ifndef KUBECHECK_H
#define KUBECHECK_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KC_ABI_VERSION 1
#define KC_NACTIONS 22
#define KC_MAX_LEVELS 4096

/* ------------------------------------------------------------------ misc */
/* Thread-local description of the last failure on this thread. */
const char *kc_last_error(void);
/* ABI version (KC_ABI_VERSION) and build string. */
int kc_abi_version(void);
const char *kc_build_info(void);
/* Number of visible HIP devices (0 without a GPU; never fails). */
int kc_device_count(void);

/* ---------------------------------------------------------------- FPSet */
typedef struct kc_fpset kc_fpset;

/* Create a set able to hold `capacity_fps` fingerprints at <= 75% load
 * (rounded up to whole 64-B buckets); it grows (rehash) when a batch would
 * push it past 75%.  `device` is a HIP device ordinal. */
int kc_fpset_create(uint64_t capacity_fps, int device, kc_fpset **out);
void kc_fpset_destroy(kc_fpset *s);
/* put: seen_out[i] = 1 iff fps[i] was already present (TLC FPSet.put). */
int kc_fpset_put_batch(kc_fpset *s, const uint64_t *fps, size_t n, uint8_t *seen_out);
/* contains: seen_out[i] = 1 iff present (TLC FPSet.contains). */
int kc_fpset_contains_batch(kc_fpset *s, const uint64_t *fps, size_t n, uint8_t *seen_out);
/* Device-pointer variants (HBM in and out, asynchronous on `hip_stream`,
 * which may be NULL for the handle's own stream; that stream is a blocking
 * one, ordered with the legacy default stream).  fps_dev may be rewritten
 * (normalised in place). */
int kc_fpset_put_batch_dev(kc_fpset *s, uint64_t *fps_dev, size_t n, uint8_t *seen_dev,
                           void *hip_stream);
int kc_fpset_contains_batch_dev(kc_fpset *s, uint64_t *fps_dev, size_t n, uint8_t *seen_dev,
                                void *hip_stream);
/* Distinct fingerprints stored. */
uint64_t kc_fpset_size(const kc_fpset *s);
/* Slot capacity (u64 fingerprint slots, linear probing). */
uint64_t kc_fpset_capacity(const kc_fpset *s);
/* TLC checkFPs(): the minimum gap between any two stored fingerprints
 * (sorted), from which TLC derives "based on the actual fingerprints"
 * (MC.out:42).  *prob_out = 1/min_gap (TLC's estimate). */
int kc_fpset_check_fps(kc_fpset *s, uint64_t *min_gap_out, double *prob_out);
/* Single-fingerprint put/contains, safe from many host threads at once
 * (TLC's -workers threads each call FPSet.put(long); MC.out:5 "4 workers").
 * Concurrent calls are flat-combined: one caller launches every pending
 * request as one batch (arrival order = sequential put order) while the
 * others wait for their result.  *seen_out = 1 iff already present. */
int kc_fpset_put(kc_fpset *s, uint64_t fp, int *seen_out);
int kc_fpset_contains(kc_fpset *s, uint64_t fp, int *seen_out);
/* Number of combined batches launched by kc_fpset_put/contains so far. */
uint64_t kc_fpset_combine_rounds(const kc_fpset *s);
/* Bulk insert / lookup of device-resident fingerprints without per-fp
 * results (a sharded or streaming caller that only needs the totals):
 * *n_new_out = fps newly inserted, *found_out = fps present.  Synchronous. */
int kc_fpset_insert_count_dev(kc_fpset *s, const uint64_t *fps_dev, size_t n, uint64_t *n_new_out,
                              void *hip_stream);
int kc_fpset_contains_count_dev(kc_fpset *s, const uint64_t *fps_dev, size_t n, uint64_t *found_out,
                                void *hip_stream);
/* Fingerprint-owner routing of a batch (multi-GPU FPSet): stable counting
 * sort of fps_dev by owner rank floor(fp * world / 2^63) (after the MSB/0
 * normalisation) into out_dev; counts_out[r] = fps for rank r (host array of
 * `world` entries, 1 <= world <= 16).  Synchronous. */
int kc_fpset_partition_dev(kc_fpset *s, const uint64_t *fps_dev, uint64_t n, int world,
                           uint64_t *out_dev, uint64_t *counts_out, void *hip_stream);
/* Synthetic stress, fingerprints generated on device:
 * insert stream i -> perm63(seed + i) for i in [0, n) (perm63 a bijection of
 * [0, 2^63), so the n fps are distinct and normalised), in batches of
 * `batch`; then n_lookup lookups, entry j present for even j and absent for
 * odd j.  So size() grows by exactly n and *found_out = ceil(n_lookup / 2).
 * Needs 1 <= seed and seed + n + n_lookup < 2^63.  Device times in seconds. */
int kc_fpset_stress(kc_fpset *s, uint64_t seed, uint64_t n, uint64_t batch,
                    uint64_t n_lookup, double *insert_seconds, double *lookup_seconds,
                    uint64_t *found_out);
/* The same streams written to device memory: kind 0 = insert stream entries
 * [start, start + n); kind 1 = lookup stream entries (n_ins = the insert
 * stream's length).  Asynchronous on hip_stream. */
int kc_stress_fps_dev(uint64_t seed, int kind, uint64_t n_ins, uint64_t start, uint64_t n,
                      uint64_t *out_dev, void *hip_stream);
/* Host copy of one stream entry (tests). */
uint64_t kc_stress_fp(uint64_t seed, int kind, uint64_t n_ins, uint64_t i);

/* ----------------------------------------------------------- StateQueue */
typedef struct kc_squeue kc_squeue;
/* FIFO of fixed-width packed states (words per state = `state_words`) in
 * segments over three tiers: HBM, pinned host RAM beyond `hbm_bytes`, and
 * spill files in `spill_dir` beyond `host_bytes` (DiskStateQueue's role).
 * The tail segment is always in HBM; a spilled segment comes back to HBM
 * when a reader reaches it.  The segments being read (front runs handed
 * out since the last pop) and written stay resident whatever the budget.
 * Every call takes a HIP stream (NULL = the queue's own blocking stream);
 * drive one queue from one stream: copies and kernels are then ordered
 * without events. */
typedef struct {
  int state_words;
  int device;
  uint64_t segment_states;  /* states per segment (0 = 2^20) */
  uint64_t hbm_bytes;       /* HBM budget of the segments (0 = unlimited) */
  uint64_t host_bytes;      /* pinned host RAM budget (0 = unlimited) */
  const char *spill_dir;    /* disk tier (NULL = none: past both budgets -ENOMEM) */
} kc_squeue_config;
typedef struct {
  uint64_t size, segments, seg_hbm, seg_host, seg_disk;
  uint64_t hbm_bytes, host_bytes, disk_bytes;      /* now */
  uint64_t spilled_host_bytes, spilled_disk_bytes, reloaded_bytes, peak_hbm_bytes;  /* cumulative */
} kc_squeue_stats;
int kc_squeue_create2(const kc_squeue_config *cfg, kc_squeue **out);
/* one HBM tier of `capacity_states`-state segments, no budget (round-1 API);
 * capacity_states is also a hard bound on the queue's size: enqueue,
 * enqueue_dev and reserve_dev past it fail with -ENOMEM ("StateQueue full") */
int kc_squeue_create(int state_words, uint64_t capacity_states, int device, kc_squeue **out);
void kc_squeue_destroy(kc_squeue *q);
/* host buffers (synchronous) */
int kc_squeue_enqueue(kc_squeue *q, const uint64_t *states, size_t n);
/* dequeue up to `max_n` states into `out`; *n_out = number dequeued */
int kc_squeue_dequeue(kc_squeue *q, uint64_t *out, size_t max_n, size_t *n_out);
/* device buffers, stream-ordered (TLC's sEnqueue / sDequeue(n) batches) */
int kc_squeue_enqueue_dev(kc_squeue *q, const uint64_t *dev_states, size_t n, void *hip_stream);
int kc_squeue_dequeue_dev(kc_squeue *q, uint64_t *dev_out, size_t max_n, size_t *n_out, void *hip_stream);
/* In place: a device run of n states at the tail for a kernel to write,
 * valid until the next call; commit(k <= n) appends its first k states. */
int kc_squeue_reserve_dev(kc_squeue *q, size_t n, uint64_t **dev_ptr, void *hip_stream);
int kc_squeue_commit(kc_squeue *q, size_t n, void *hip_stream);
/* In place: a contiguous device run of up to max_n states starting `offset`
 * states after the head (*n_out may be smaller, at a segment end), valid
 * until it is popped; pop(n) drops n states from the head. */
int kc_squeue_front_dev(kc_squeue *q, size_t offset, size_t max_n, const uint64_t **dev_ptr,
                        size_t *n_out, void *hip_stream);
int kc_squeue_pop(kc_squeue *q, size_t n, void *hip_stream);
/* host copy of states [offset, offset + n) after the head, from any tier */
int kc_squeue_peek(kc_squeue *q, size_t offset, size_t n, uint64_t *host_out, void *hip_stream);
int kc_squeue_get_stats(kc_squeue *q, kc_squeue_stats *out);
uint64_t kc_squeue_size(const kc_squeue *q);

/* -------------------------------------------------------------- Engine */
typedef struct {
  int nc, np, ns;          /* clients, PVC controllers, API servers (Model_1: 1,1,1) */
  int can_fail;            /* REQUESTS_CAN_FAIL  (MC.tla:5-7) */
  int can_timeout;         /* REQUESTS_CAN_TIMEOUT (MC.tla:10-12) */
  int check_deadlock;      /* launch:16 */
  int variant;             /* 0 = KubeAPI.tla as written; seeded bugs: 1 = Update w/o
                              HasRead, 2 = Force w/o replace, 3 = C1 ignores the
                              reply status, 4 = list ignores kind, 5 = Init store
                              with two Secret versions (kubeapi_spec.h Flags) */
  int device;              /* HIP device ordinal */
  int keep_trace;          /* parent pointers (TLC's trace file); default 1 */
  int max_levels;          /* 0 = to completion */
  uint64_t fpset_slots;    /* initial FPSet slots; 0 = default */
  uint64_t chunk_states;   /* parents per expansion chunk; 0 = default */
  int verbose;             /* progress lines to stderr */
  int timing;              /* 1 = time every kernel launch with HIP events,
                              2 = only k_claim (the roofline kernel) */
  int invariants;          /* MC.cfg INVARIANT list: bit 0 TypeOK, bit 1
                              OnlyOneVersion (default 3; 0 = check none), bit 2
                              the build-defined NoLostUpdate (with its lostUpdate
                              history variable; models of <= 3 actors) */
  /* Frontier spill (single-GPU engine).  frontier_hbm_bytes > 0 keeps the
   * frontiers in a kc_squeue with that HBM budget: levels run in chunks of
   * <= frontier_segment_states parents, read from the queue's head and
   * written into its tail; segments past the budget go to pinned host RAM
   * (up to frontier_host_bytes, 0 = unlimited), then to files in spill_dir.
   * trace_host = 1 keeps the trace file (parent index + ordinal, 9 B per
   * state) in pinned host RAM instead of HBM. */
  uint64_t frontier_hbm_bytes;
  uint64_t frontier_host_bytes;
  uint64_t frontier_segment_states;   /* 0 = 2^22 */
  const char *spill_dir;
  int trace_host;
  /* Seen-set spill (single-GPU engine, and every rank of the sharded loop
   * for its own share of the fingerprints; TLC's OffHeapDiskFPSet role,
   * MC.out:5).  seen_hbm_bytes > 0 caps the HBM the seen-set uses: a fixed
   * hot ClaimSet (<= half of it), scratch, and the HBM directories and
   * filters of the cold tier.  When the hot table fills, its fingerprints are
   * flushed into sorted runs in pinned host RAM (up to seen_host_bytes,
   * 0 = unlimited), then in files in spill_dir; every level's new states are
   * checked against the runs on the GPU.  Results are identical to the
   * unbounded seen-set's. */
  uint64_t seen_hbm_bytes;
  uint64_t seen_host_bytes;
  /* Sharded loop at world > 1 (kc_group_*, kc_shard_*): 1 = claims ordered
   * by each parent's position in sequential-BFS order instead of (rank, local
   * index), so the first discoverer of every state, the error reported and
   * its trace are TLC -workers 1's (KubeAPI___Model_1.launch:4-7); costs a
   * per-level all-reduce of per-parent masks and a sort of each rank's new
   * frontier.  Counted levels only, with the deferred frontier; not with the
   * seen-set spill.  Ignored at world 1, where the order is TLC's anyway. */
  int tlc_order;
  /* 1 = the first inserter of a fingerprint owns it, as in a TLC -workers N
   * run (KubeAPI___Model_1.launch:33): no settle passes.  Counts, widths,
   * per-action generated counts, error kinds and levels and trace lengths are
   * unchanged; which same-level copy wins (its parent, the per-action
   * distinct split, which of several equal-level errors is reported) is not
   * deterministic.  Single-GPU engine: in-HBM wide levels only (ignored with
   * the seen-set spill or a frontier HBM budget; KC_FIRST_CLAIM=1 sets it
   * too).  Sharded loop (kc_shard_*, kc_group_*): every counted level, at any
   * world; kc_shard_create fails with -EINVAL together with tlc_order or the
   * seen-set spill.  kc_result.claim_mode reports what ran.  The seen-set
   * then holds 8-B fingerprint words (16-B {fp, claim} slots otherwise): the
   * same slot count and load in half the HBM, half the per-run clear. */
  int first_claim;
} kc_model_config;

typedef struct {
  uint64_t init, generated, distinct, queue_left;
  int depth;               /* BFS levels, init = level 1 (TLC msg 2194) */
  int complete;
  uint64_t act_gen[KC_NACTIONS];
  uint64_t act_dist[KC_NACTIONS];
  int nlevels;
  uint64_t level_width[KC_MAX_LEVELS];
  int err_kind;            /* 0 none, 1 assertion, 2 invariant, 3 deadlock */
  int err_action;          /* action id (assertion) */
  int err_self;            /* process index of the failing action */
  int err_invariant;       /* 0 TypeOK, 1 OnlyOneVersion */
  int err_level;           /* BFS level of the last trace state */
  int trace_len;           /* states in the counterexample */
  double seconds;          /* wall time of the BFS (device work + host loop) */
  double collision_optimistic; /* TLC's calculated estimate d*(g-d)/2^64 */
  uint64_t fpset_slots;
  uint64_t peak_frontier;
  uint64_t fpset_probes;   /* FPSet insert probes (level-unique successors) */
  uint64_t batch_inserts;  /* batch-table inserts (= generated successors) */
  uint64_t levels_chunks;  /* expansion chunks over the whole run */
  uint64_t outdeg_hist[16]; /* TLC outdegree (msg 2268): expanded states by the number of
                              new states first reached from them; [15] = 15 or more
                              (single-GPU engine; zero in the sharded path) */
  uint64_t frontier_spilled_bytes;   /* frontier bytes written to host RAM or disk */
  uint64_t frontier_reloaded_bytes;  /* ... and read back into HBM */
  uint64_t frontier_peak_hbm_bytes;  /* peak HBM held by the frontier queue */
  /* seen-set spill (cfg.seen_hbm_bytes > 0) */
  uint64_t seen_flushes;        /* hot-table flushes into the cold tier */
  uint64_t seen_cold_fps;       /* fingerprints in cold runs at the end */
  uint64_t seen_cold_runs;      /* cold runs at the end (host + disk) */
  uint64_t seen_cold_queries;   /* new-to-the-hot-table fingerprints checked against the cold tier */
  uint64_t seen_cold_hits;      /* ... found there (states already seen) */
  uint64_t seen_merges;         /* run merges */
  uint64_t seen_filter_tests;   /* (query, run) pairs tested by a run's Bloom filter */
  uint64_t seen_filter_passed;  /* ... that the filter let through to the run */
  uint64_t seen_disk_bytes;     /* cold-run bytes written to spill files */
  uint64_t seen_peak_hbm_bytes; /* peak HBM of the seen-set (hot table + scratch + cold metadata) */
  double seen_seconds;          /* host wall time in chunk planning, flushes and cold checks */
  double seen_flush_seconds;    /* ... of it in flushes (sort, copy out, merges, files) */
  double seen_merge_seconds;    /* ... of that in the host merges of runs */
  double seen_check_seconds;    /* ... in the per-chunk cold checks (queries, sort, probe) */
  uint64_t cand_overflow_records;  /* settle candidates beyond their tile's segment (overflow list) */
  uint64_t cand_buffer_peak_bytes; /* HBM of the candidate-record buffers (tile segments + overflow list) */
  /* deferred frontier (the default wide path): states rebuilt from their
   * links inside k_claim (which then also writes them), and whether this run
   * was redone on the materialising path (an error or a capacity estimate
   * exceeded; the reported result is the redone run's) */
  uint64_t deferred_states;
  uint64_t defer_fallback;
  /* the level an exact redo of a deferred-frontier anomaly started from (the
   * anomaly's level; 1 = from Init), 0 if there was none */
  uint64_t defer_redo_level;
  /* levels run by a device-driven narrow path (single-GPU engine: k_nfinish;
   * sharded loop: the fixed-slot exchange levels, shard_narrow.h) */
  uint64_t narrow_levels;
  /* the claim protocol the wide (counted) levels ran with: 0 = the
   * sequential-BFS minimum key (TLC -workers 1's first discoverer on one GPU;
   * (rank, parent) order on shards), 1 = first inserter (cfg.first_claim),
   * 2 = TLC order on shards (cfg.tlc_order at world > 1) */
  int claim_mode;
} kc_result;

typedef struct kc_engine kc_engine;
/* Fill a config with Model_1 defaults (1,1,1, both constants TRUE, deadlock on). */
void kc_model_config_default(kc_model_config *cfg);
int kc_engine_create(const kc_model_config *cfg, kc_engine **out);
void kc_engine_destroy(kc_engine *e);
/* Run BFS to completion (or error / max_levels). */
int kc_engine_run(kc_engine *e, kc_result *res);
/* Counterexample as TLC-style text ("State 1: ..."); returns bytes needed. */
size_t kc_engine_trace_text(kc_engine *e, char *buf, size_t cap);
/* Canonical tuple of trace state i (see kc_spec_tuple_words). */
int kc_engine_trace_tuple(kc_engine *e, int i, uint64_t *out);
/* Canonical tuples of the states of BFS level `level` (1-based) from the
 * last run's frontier buffers, if still resident (only the final level and
 * levels captured with kc_engine_capture_level).  Returns count or <0. */
int64_t kc_engine_level_tuples(kc_engine *e, int level, uint64_t *out, uint64_t cap_states);
/* Ask run() to keep a host copy of level `level`'s packed states. */
int kc_engine_capture_level(kc_engine *e, int level);
/* Per-kernel device timings of the last run (ms; needs cfg.timing=1, or 2
 * for expand alone):
 * expand, resolve, scan, emit; and the number of launches of each. */
int kc_engine_kernel_times(kc_engine *e, double *ms4, uint64_t *launches4);
/* The narrow-level kernel of the last run (frontiers <= 8192 states run as
 * whole levels inside one single-workgroup launch): its device time in ms
 * (with cfg.timing), launches, and the BFS levels it expanded. */
int kc_engine_narrow_times(kc_engine *e, double *ms, uint64_t *launches, uint64_t *levels);
/* TLC's checkFPs on the last run's seen-set ("based on the actual
 * fingerprints", MC.out:42): the minimum gap between sorted fingerprints;
 * *prob_out = 1/min_gap. */
int kc_engine_check_fps(kc_engine *e, uint64_t *min_gap_out, double *prob_out);

/* --------------------------------------------------- Sharded (multi-GPU) */
/* Fingerprint-owner-sharded BFS, one process per GPU (replaces TLC's
 * single-host worker pool; TLC's own distributed mode is off in Model_1,
 * KubeAPI___Model_1.launch:4-7).  The caller drives the levels and does the
 * exchange between pack() and insert() (kubecheck/distributed.py: RCCL
 * all-to-all through torch.distributed).  owner(fp) = floor(fp*R/2^63).
 * Per level:  expand -> pack(send) -> [all-to-all] -> insert(recv) ->
 * [all-reduce of new counts / error keys] -> advance.
 * Keys (records and errors): rank<<60 | parent index<<16 | successor<<8 |
 * low byte (action id in records; 1 assertion, 2 invariant, 3 deadlock,
 * 0x12 invariant violated by an Init state in error keys). */
typedef struct kc_shard kc_shard;
int kc_shard_create(const kc_model_config *cfg, int rank, int world, kc_shard **out);
void kc_shard_destroy(kc_shard *s);
/* Adopt (insert + enqueue) the Init states this rank owns. */
int kc_shard_init(kc_shard *s, uint64_t *n_local);
/* After kc_shard_init: the error key (low byte 0x12) of this rank's first
 * Init state that violates an invariant, ~0 if none.  It is level 1's error
 * and takes precedence over anything level 1's expansion reports. */
int kc_shard_init_error(kc_shard *s, uint64_t *key_out);
/* Run every stage on the caller's HIP stream (e.g. the one its RCCL
 * collectives use) instead of the shard's own: pack() then returns without a
 * host sync and insert() may read a recv buffer written earlier on that
 * stream (NULL = the default stream).  Call before kc_shard_init. */
int kc_shard_set_stream(kc_shard *s, void *hip_stream);
/* Expand the frontier: claim the successors this rank owns in place;
 * counts_out[r] = records destined to rank r (world entries, 0 for this
 * rank); *err_key_out = this rank's min Assert/deadlock key or ~0. */
int kc_shard_expand(kc_shard *s, uint64_t *counts_out, uint64_t *err_key_out);
/* Bytes per record: the state's canonical words and the key, padded to 16 B
 * (the receiver recomputes the fingerprint). */
uint64_t kc_shard_record_bytes(kc_shard *s);
/* Write sum(counts) records, grouped by owner rank, into device memory
 * (complete on return unless a caller stream was set). */
int kc_shard_pack(kc_shard *s, void *send_dev);
/* Dedup + insert `n_records` received records (device memory, grouped by
 * source rank) together with this rank's own claims of the level;
 * *n_new = states added to this rank's next frontier.  Without a caller
 * stream the library reads recv_dev on its own HIP stream: the caller must
 * have completed every write to it (e.g. synchronised its all-to-all). */
int kc_shard_insert(kc_shard *s, const void *recv_dev, uint64_t n_records, uint64_t *n_new,
                    uint64_t *err_key_out);
/* The new states become the frontier (after the caller's agreement step). */
int kc_shard_advance(kc_shard *s);
/* Parent key of local state `idx` of BFS level `level` (trace walk-back). */
int kc_shard_parent_key(kc_shard *s, int level, uint64_t idx, uint64_t *key_out);
/* Canonical tuple of current-frontier state `idx`. */
int kc_shard_frontier_tuple(kc_shard *s, uint64_t idx, uint64_t *out);
/* This rank's counters: act_gen (its parents), act_dist (its new states),
 * generated, distinct (owned), fpset_slots. */
int kc_shard_result(kc_shard *s, kc_result *res);
/* k_claim device time in ms (HIP events; needs cfg.timing != 0), launches
 * and parents expanded since the previous call (counters reset on read). */
int kc_shard_claim_times(kc_shard *s, double *ms, uint64_t *launches, uint64_t *parents);
/* owner rank of a fingerprint */
int kc_shard_owner(uint64_t fp, int world);

/* ------------------------------------------- Native sharded level loop */
/* The whole level-synchronous sharded BFS in C++ (the protocol above, with
 * one all-gather and one all-to-all per level and no caller in the loop).
 * A group is the set of shards one process drives plus their collectives:
 *   - kc_group_create_rccl: one shard per process (one process per GPU) and
 *     an RCCL communicator; every rank passes the same 128-byte id, made by
 *     kc_rccl_unique_id on one rank and sent to the others by the caller
 *     (e.g. a torch.distributed broadcast).  RCCL is loaded at run time.
 *   - kc_group_create_local: ranks 0..n-1 of one process on one GPU, the
 *     collectives done by device copies (multi-rank emulation, tests).
 * kc_group_run fills the GLOBAL result (the same on every rank): totals,
 * per-action counts, level widths, depth, and any error with its trace. */
#define KC_RCCL_ID_BYTES 128
typedef struct kc_group kc_group;
int kc_rccl_unique_id(uint8_t *id_out /* KC_RCCL_ID_BYTES */);
int kc_group_create_rccl(kc_shard *s, const uint8_t *id, kc_group **out);
int kc_group_create_local(kc_shard **shards, int nshards, kc_group **out);
/* One shard per process with the caller's own transport (MPI, gloo,
 * sockets) instead of RCCL: the loop calls these on host buffers, from the
 * thread that called kc_group_run; each returns 0 or < 0 (the run then fails
 * with -EIO on every rank that sees it; like RCCL's, a transport failure on
 * one rank only is the transport's to surface).  Every rank makes the same
 * sequence of calls.
 *   all_gather:     out[r * n + k] = rank r's in[k]  (n words)
 *   exchange:       this rank's all-to-all as kc_exchange_plan lists it, in
 *                   BYTES: xfers[4k..4k+3] = peer, 1 send / 0 receive, byte
 *                   offset into sendbuf / recvbuf, bytes; post all of them,
 *                   then wait (the k-th send from s to d pairs with the k-th
 *                   receive at d from s)
 *   broadcast:      *v from rank `root` to every rank
 *   all_reduce_sum: v[0..n) summed over ranks, in place
 * kubecheck.distributed.GlooHostComm implements it over torch.distributed. */
typedef struct kc_host_comm {
  void *ctx;
  int (*all_gather)(void *ctx, const uint64_t *in, uint64_t n, uint64_t *out);
  int (*exchange)(void *ctx, const uint64_t *xfers, int nxfers, const void *sendbuf, void *recvbuf);
  int (*broadcast)(void *ctx, int root, uint64_t *v);
  int (*all_reduce_sum)(void *ctx, uint64_t *v, uint64_t n);
} kc_host_comm;
int kc_group_create_host(kc_shard *s, const kc_host_comm *comm, kc_group **out);
void kc_group_destroy(kc_group *g);
int kc_group_run(kc_group *g, kc_result *res);
/* Canonical tuple of trace state i of the last run's error; returns words. */
int kc_group_trace_tuple(kc_group *g, int i, uint64_t *out);
/* Records this group's ranks sent to other ranks in the last run (global). */
uint64_t kc_group_records_sent(const kc_group *g);
/* The all-to-all of rank `me` as issued to RCCL (and replayed by the
 * one-process emulation): for each peer in rank order, its sends then its
 * receives, each cut into pieces of <= piece_records records (the native loop
 * uses 256 MiB / record bytes, or KC_PIECE_BYTES).  Mx = world x world
 * record counts (row = source rank).  out[4k..4k+3] = peer, 1 send / 0 receive,
 * offset and count in records (offsets into the destination-grouped send /
 * source-grouped receive buffer); fills at most `cap` transfers and returns
 * how many there are.  Host only (no GPU): the CPU tests check every rank's
 * plan pairs with its peers' for world 1..9. */
int kc_exchange_plan(int world, int me, const uint64_t *Mx, uint64_t piece_records, uint64_t *out, int cap);

/* ----------------------------------------------- Seen-set spill (tests) */
/* Host self-check of the cold tier's run search (coldset.hip run_find, the
 * search every GPU lookup of a spilled fingerprint runs): n sorted random
 * keys and their directory; every key must be found and absent keys not,
 * whole-run and through staging windows.  Returns the number of wrong
 * answers (0 expected).  No GPU needed. */
int64_t kc_cold_find_selftest(uint64_t n, uint64_t seed);

/* ---------------------------------------------------------- Spec (host) */
/* Words of the canonical tuple for a model: 1 + 19 * (nc + np + ns). */
int kc_spec_tuple_words(int nc, int np, int ns);
/* Words of the packed state (GPU layout) for a model. */
int kc_spec_state_words(int nc, int np, int ns);
/* Init states as canonical tuples; returns count. */
int kc_spec_init(const kc_model_config *cfg, uint64_t *tuples_out, int cap);
/* Successors of a canonical tuple in TLC order; returns count, or -2 when
 * the state raises an Assert failure (*fail_action set), <0 on error. */
int kc_spec_successors(const kc_model_config *cfg, const uint64_t *tuple, int *actions_out,
                       uint64_t *succ_tuples_out, int cap, int *fail_action);
/* TypeOK/OnlyOneVersion: -1 = both hold, 0 = TypeOK fails, 1 = OOV fails. */
int kc_spec_check(const kc_model_config *cfg, const uint64_t *tuple);
/* Fingerprint of the packed form of a canonical tuple. */
int kc_spec_fingerprint(const kc_model_config *cfg, const uint64_t *tuple, uint64_t *fp_out);
/* Self-check of the kernels' incremental fingerprint: the number of
 * successors of `tuple` whose fingerprint_succ differs from a full
 * fingerprint (0 expected), <0 on error. */
int kc_spec_fp_selfcheck(const kc_model_config *cfg, const uint64_t *tuple);
/* Packed <-> canonical conversion. */
int kc_spec_pack(const kc_model_config *cfg, const uint64_t *tuple, uint64_t *packed_out);
int kc_spec_unpack(const kc_model_config *cfg, const uint64_t *packed, uint64_t *tuple_out);

#ifdef __cplusplus
}
#endif
#endif
