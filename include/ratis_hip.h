/*
 * ratis_hip.h -- C ABI of libratis_hip, the MI355X (gfx950) leader-bookkeeping engine for
 * Apache Ratis (OneSizeFitsQuorum/ratis).
 *
 * Two hot paths of the reference are served, each as a batched HIP kernel over HBM-resident
 * struct-of-arrays data:
 *
 *   1. Quorum commit -- LeaderStateImpl.updateCommit() / getMajorityMin() / MinMajorityMax and
 *      RaftLogBase.updateCommitIndex(), including joint-consensus (old+new) confs and the
 *      current-term check, evaluated for millions of RaftGroups per launch.
 *   2. Log-entry CRC32C -- PureJavaCrc32C as used by SegmentedRaftLogOutputStream.write (frame
 *      trailer) and SegmentedRaftLogReader.decodeEntry (frame verification).
 *
 * Reference paths cited below are relative to the ratis tree:
 *   LSI = ratis-server/src/main/java/org/apache/ratis/server/impl/LeaderStateImpl.java
 *   RLB = ratis-server/src/main/java/org/apache/ratis/server/raftlog/RaftLogBase.java
 *   RCI = ratis-server/src/main/java/org/apache/ratis/server/impl/RaftConfigurationImpl.java
 *   FII = ratis-server/src/main/java/org/apache/ratis/server/impl/FollowerInfoImpl.java
 *   PJC = ratis-common/src/main/java/org/apache/ratis/util/PureJavaCrc32C.java
 *   OUT = ratis-server/.../raftlog/segmented/SegmentedRaftLogOutputStream.java
 *   RDR = ratis-server/.../raftlog/segmented/SegmentedRaftLogReader.java
 *
 * Conventions (all entry points):
 *   - Plain C types only; no exception crosses the ABI.  Every int-returning function returns
 *     RH_OK (0) or a negative RH_E_* code; rh_last_error() then holds a message for the calling
 *     thread (the Java binding maps RH_E_INVAL and RH_E_RANGE to IllegalArgumentException, the
 *     others to IOException -- see INTEGRATION.md).
 *   - "_launch" functions take DEVICE pointers, enqueue work on `stream` (a hipStream_t, used
 *     as given: NULL is the HIP null stream; rh_ctx_stream() returns the context's own stream)
 *     and return without synchronising.
 *   - All log indices are signed 64-bit (Java long); INVALID_LOG_INDEX = -1 is a legal value.
 */
#ifndef RATIS_HIP_H
#define RATIS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RH_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------------------- */
#define RH_OK        0
#define RH_E_INVAL  -1  /* bad argument (null pointer, size out of range, ...)               */
#define RH_E_RANGE  -2  /* value outside what the engine supports (e.g. > 14 follower slots) */
#define RH_E_DEVICE -3  /* HIP runtime failure (message carries hipGetErrorString)           */
#define RH_E_NOMEM  -4  /* device or pinned host allocation failed                          */
#define RH_E_STATE  -5  /* object used after destroy / on the wrong device                   */

typedef struct rh_ctx rh_ctx;       /* one per (process, GPU): device, stream, constant tables */
typedef struct rh_groups rh_groups; /* a resident table of leader divisions on one GPU       */

int rh_abi_version(void);
/* Message describing the last failure on the calling thread ("" if none). */
const char* rh_last_error(void);
/* Number of visible GPUs. */
int rh_device_count(int* out);
/* Binds device `device`, creates the context stream and uploads the CRC tables. */
int rh_init(int device, rh_ctx** out);
int rh_shutdown(rh_ctx* ctx);
/* Waits for all work enqueued on the context stream. */
int rh_synchronize(rh_ctx* ctx);
/* The context's hipStream_t, for callers that order their own work against it. */
void* rh_ctx_stream(rh_ctx* ctx);

/* ===================================================================================== */
/* 1. Quorum commit                                                                      */
/* ===================================================================================== */

/* Per-group membership word (one uint32 per group), host-built from RaftConfigurationImpl on
 * every conf or leadership change (RCI:142-195, PeerConfiguration.java:96-128):
 *   bits  0..13  follower slot k is a voter of conf (new/current) AND has a FollowerInfo
 *                (LSI:274-293 getFollowerInfos: peers.streamPeerIds().map(map::get).filter(nonNull))
 *   bit   14     includeSelf          = conf.containsInConf(selfId)          (LSI:963)
 *   bit   15     transitional         = conf.isTransitional() (oldConf != null, RCI:142-144)
 *   bits 16..29  follower slot k is a voter of oldConf with a FollowerInfo
 *   bit   30     includeSelfInOldConf = conf.containsInOldConf(selfId)       (LSI:975)
 *   bit   31     active: this division is LEADER and should be evaluated (inactive => no result)
 * Listeners are never voters (PeerConfiguration keeps them in a separate map).
 * A word is MALFORMED for a tier of F follower slots when bits 0..13 or 16..29 name a slot >= F:
 * the commit and lease kernels then treat the group as inactive (no result, no commit, no lease)
 * rather than evaluating a quorum over fewer voters. */
#define RH_MAX_FOLLOWERS    14u
#define RH_CONF_SELF        (1u << 14)
#define RH_CONF_TRANSITIONAL (1u << 15)
#define RH_CONF_OLD_SHIFT   16u
#define RH_CONF_SELF_OLD    (1u << 30)
#define RH_CONF_ACTIVE      (1u << 31)

static inline uint32_t rh_conf_pack(uint32_t new_mask, int include_self, int transitional,
                                    uint32_t old_mask, int include_self_old, int active) {
    return (new_mask & 0x3FFFu) | (include_self ? RH_CONF_SELF : 0u) |
           (transitional ? RH_CONF_TRANSITIONAL : 0u) | ((old_mask & 0x3FFFu) << RH_CONF_OLD_SHIFT) |
           (include_self_old ? RH_CONF_SELF_OLD : 0u) | (active ? RH_CONF_ACTIVE : 0u);
}

/* Which reference computation a launch performs. */
#define RH_MODE_COMMIT 0 /* LSI:946-950 updateCommit(): getMajorityMin(matchIndex, flushIndex, gap)
                            -> LSI:1015-1026 updateCommit(majority, min) -> RLB:121-142        */
#define RH_MODE_WATCH  1 /* LSI:612-622 commitIndexChanged(): getMajorityMin(commitIndex,
                            lastCommittedIndex) with gap -1 -> {min, majority, max} levels     */

/* One struct-of-arrays table ("tier") of G groups with F follower slots each.  All pointers are
 * device pointers.  Groups whose voter union needs more slots live in a wider tier; a launch
 * takes up to RH_MAX_TIERS tiers and runs them in one kernel.  Per group, reads
 * 8*(F+1) + 8 + 8 + 4 bytes and writes 16 bytes (COMMIT) -- the "8P+36 B" of SURVEY 8(d). */
typedef struct rh_commit_soa {
    uint64_t n;                    /* groups in this tier                                       */
    uint32_t n_followers;          /* F, 1..RH_MAX_FOLLOWERS                                    */
    int32_t  mode;                 /* RH_MODE_COMMIT or RH_MODE_WATCH                           */
    int64_t  gap_threshold;        /* followerMaxGapThreshold (LSI:390-401), -1 = off; COMMIT only */
    const int64_t* follower_index; /* [F][col_stride], column k = follower slot k:
                                      FollowerInfo.getMatchIndex (COMMIT) or getCommitIndex
                                      (WATCH) -- FII:87-105                                     */
    uint64_t col_stride;           /* elements between follower columns; 0 means n             */
    const int64_t* self_index;     /* [n] COMMIT: raftLog.getFlushIndex(); WATCH: getLastCommittedIndex() */
    const int64_t* commit_in;      /* [n] raftLog.getLastCommittedIndex()  (COMMIT only)          */
    const int64_t* term_start;     /* [n] first log index of the leader's current term (the
                                      StartupLogEntry index, LSI:296-301); termAt(i)==currentTerm
                                      <=> i >= term_start for i <= flushIndex (COMMIT only)       */
    const uint32_t* conf;          /* [n] membership words (above)                               */
    int64_t* commit_out;           /* [n] new commit index (COMMIT); may alias commit_in          */
    int64_t* min_out;              /* [n] optional: min (watch ALL / ALL_COMMITTED level)         */
    int64_t* maj_out;              /* [n] optional: majority (MAJORITY_COMMITTED level)           */
    int64_t* max_out;              /* [n] optional: max (MAJORITY level)                          */
    uint64_t* valid_bits;          /* [ceil(n/64)] optional: bit g = getMajorityMin was present  */
    uint64_t* advanced_bits;       /* [ceil(n/64)] optional: bit g = updateCommitIndex stored     */
    /* optional compacted list of advanced groups (COMMIT): entries appended in unspecified
     * order; *adv_count must be zeroed by the caller (rh_groups does it). */
    uint64_t* adv_rows;            /* [cap] row index within this tier                          */
    int64_t*  adv_commit;          /* [cap] new commit index                                    */
    unsigned long long* adv_count; /* single counter, shared by all tiers of a launch OK        */
    uint64_t adv_cap;
    uint64_t adv_row_base;         /* added to each row written to adv_rows (tier slot offset)   */
    uint64_t tile_stride;          /* 0: every column is a plain array over the groups.  Else the
                                      TILED layout: groups come in tiles of RH_TILE_GROUPS, every
                                      per-group column (follower_index .. max_out) holds its 128
                                      elements of a tile contiguously at its pointer + tile *
                                      tile_stride bytes, and follower column k lies col_stride
                                      elements after column 0 within the tile (col_stride >= 128).
                                      tile_stride is a multiple of 16; every column must cover
                                      ceil(n / 128) whole tiles.  One wave then reads one
                                      contiguous run per tile instead of F + 4 separate ones.    */
} rh_commit_soa;
#define RH_TILE_GROUPS 128u

#define RH_MAX_TIERS 4

/* Evaluates every group of every tier (one kernel launch).  Invalid groups (inactive or
 * Optional.empty()) keep commit_out = commit_in and get INT64_MIN in min/maj/max_out. */
int rh_commit_soa_launch(rh_ctx* ctx, const rh_commit_soa* tiers, int n_tiers, void* stream);

/* ---- resident group table (the object the Java ratis-hip module holds) ------------------
 *
 * One table per (process, GPU) holds the leader-side commit state of up to `capacity` leader
 * divisions ("slots", the handle the Java module keeps per RaftGroup).  A slot owns its
 * FollowerInfo matchIndex / commitIndex per follower slot k (0..13; k is the module's numbering
 * of the division's peers), the leader's flushIndex, commitIndex, the current term's first log
 * index, and the membership word.  Internally the slot lives in the narrowest SoA tier whose
 * width (2, 4, 6, ..., 14 follower columns) covers every slot its conf word names; a conf change
 * that needs a different width moves it (rh_group_reconf).  Everything below is asynchronous on
 * the context stream in call order, except where a call says it blocks.
 *
 * Event model (LeaderStateImpl's UPDATE_COMMIT event queue, LSI:155-166, 846-854, 900-902): a
 * delta to matchIndex / flushIndex / commitIndex, a start or a reconf marks the slot dirty, and
 * rh_commit_batch evaluates updateCommit() for the dirty slots only (each once, however many
 * deltas it received), reporting just the groups whose result changed.  The same holds for
 * follower commitIndex deltas and rh_watch_levels (commitIndexChanged, LSI:606-622).
 * Evaluating a clean slot again could not change its result, so this is exactly the reference's
 * event-driven behaviour. */

/* Column ids for deltas (FollowerInfo / RaftLog producers). */
#define RH_COL_MATCH(k)   ((uint8_t)(k))        /* follower k matchIndex (FII:87-95)            */
#define RH_COL_FCOMMIT(k) ((uint8_t)(16u + (k))) /* follower k commitIndex (FII:97-105)         */
#define RH_COL_FLUSH      ((uint8_t)32u)         /* leader flushIndex (SegmentedRaftLogWorker
                                                    .java:419-431)                              */
#define RH_COL_COMMITTED  ((uint8_t)33u)         /* leader commitIndex raised outside the kernel
                                                    (RaftLogBase.updateSnapshotIndex, RLB:155-166) */
/* Operations (RaftLogIndex, ratis-server-api/.../raftlog/RaftLogIndex.java). */
#define RH_OP_MAX 0u  /* updateToMax: matchIndex / commitIndex updates (FII:93-105)              */
#define RH_OP_SET 1u  /* setUnconditionally: FollowerInfo.setSnapshotIndex sets matchIndex,
                         possibly lower (FII:147-151)                                           */
typedef struct rh_delta {  /* 16 bytes */
    uint32_t slot;         /* division slot in the table                                        */
    uint8_t  column;       /* RH_COL_*                                                          */
    uint8_t  op;           /* RH_OP_*                                                           */
    uint16_t reserved;     /* 0                                                                 */
    int64_t  value;
} rh_delta;
/* Ordering: every batch the device applies (a staging slot of rh_push_deltas calls, or one
 * rh_deltas_submit) leaves each (slot, column) where applying its deltas one by one in batch order
 * leaves it -- the last SET wins and only the MAX deltas after it count (RaftLogIndex semantics per
 * call, FollowerInfoImpl.java:93-105, 147-151) -- whatever mix of SETs and MAXes, repeated SETs
 * included, the batch holds. */

/* An event of rh_commit_batch: `slot` and an index (the new commitIndex, or the changed
 * watch-ALL level). 16 bytes. */
typedef struct rh_index_event {
    uint32_t slot;
    uint32_t reserved;
    int64_t  value;
} rh_index_event;
/* An event of rh_watch_levels: the changed commitIndexChanged() levels of one slot. 32 bytes.
 * valid = 0 is Optional.empty() (levels INT64_MIN). */
typedef struct rh_watch_event {
    uint32_t slot;
    uint32_t valid;
    int64_t  min;       /* ALL_COMMITTED      */
    int64_t  majority;  /* MAJORITY_COMMITTED */
    int64_t  max;       /* MAJORITY           */
} rh_watch_event;

/* Results of one rh_commit_batch: library-owned pinned host memory, valid until the third
 * rh_commit_batch_async after the one that produced them (three result buffers rotate, so a
 * producer can keep two evaluations in flight while it reads the third's events). */
typedef struct rh_commit_out {
    const rh_index_event* advanced;   /* slots whose commitIndex was stored, new value (LSI:1017-1021,
                                         RLB:121-142); the Java follow-up runs for these only    */
    uint64_t n_advanced;
    const rh_index_event* watch_all;  /* slots whose watch-ALL level (min, LSI:1025) changed       */
    uint64_t n_watch_all;
} rh_commit_out;

/* Creates a table of `capacity` slots (< 2^28); every slot starts stopped. */
int rh_groups_create(rh_ctx* ctx, uint64_t capacity, int64_t gap_threshold, rh_groups** out);
/* Waits for the table's work and frees it; RH_E_DEVICE if that work faulted (freed anyway). */
int rh_groups_destroy(rh_groups* g);
/* Leader start for `slot` (a new LeaderStateImpl: every FollowerInfo is new, matchIndex =
 * commitIndex = -1, FII:42-43, LSI:421-430; StartupLogEntry's index is term_start, LSI:296-301).
 * Also the way to re-arm a slot for a new leadership term.  Marks the slot dirty. */
int rh_group_start(rh_groups* g, uint32_t slot, uint32_t conf, int64_t flush_index, int64_t commit_index,
                   int64_t term_start);
/* Conf change of a started slot (applyOldNewConf / replicateNewConf, LSI:624-633, 1064-1074;
 * addSenders LSI:681-692; restart of a LogAppender LSI:704-724).  `src` (RH_MAX_FOLLOWERS
 * entries, or NULL = identity) maps every new follower slot k to the old slot whose
 * matchIndex / commitIndex it keeps (src[k] = k: the peer stays; another old slot: the module
 * renumbered it), or -1 for a new FollowerInfo (index -1: a newcomer, or a recycled slot).  The
 * slot moves to another tier when the new word needs a different width.  Marks it dirty. */
int rh_group_reconf(rh_groups* g, uint32_t slot, uint32_t conf, const int8_t* src);
/* Step down / group removal: the slot stops (no further results) and releases its row. */
int rh_group_stop(rh_groups* g, uint32_t slot);
/* Bulk start of slots [first, first + n) with explicit follower state (checkpoint restore, bench):
 * host arrays, match / fcommit are [n_host_followers][n] (column k = follower slot k; columns a
 * slot's tier has beyond n_host_followers start at -1).  NULL match / fcommit = all -1. */
int rh_groups_load(rh_groups* g, uint32_t first, uint32_t n, uint32_t n_host_followers, const int64_t* match,
                   const int64_t* fcommit, const int64_t* flush, const int64_t* commit,
                   const int64_t* term_start, const uint32_t* conf);
/* Copies deltas into the pinned staging ring (RaftLogIndex semantics per op, see Ordering above).
 * Deltas of stopped slots or of follower columns the slot's tier does not have are rejected
 * (RH_E_INVAL, nothing applied).  A call with more deltas than the open slot's room is staged
 * chunk by chunk; a control call may take effect between two chunks, and each later chunk is checked
 * again against the slot states it finds -- a delta rejected then fails the call with the earlier
 * chunks staged (the message names them).  Returns once the caller's buffer may be reused.  Multi-producer:
 * concurrent calls copy into ranges of the open slot reserved with one atomic each, never waiting
 * for an evaluation, a _wait call or another producer's copy; a call's deltas keep their order and
 * calls that do not overlap in time keep theirs.  Staged deltas reach the device when the slot is
 * full or before the next evaluation, read, zero-copy acquire or control call -- always before
 * anything issued after the push returned. */
int rh_push_deltas(rh_groups* g, const rh_delta* deltas, size_t n);
/* Zero-copy producer path over the same staging ring (two pinned slots of RH_DELTA_SLOT deltas):
 * rh_deltas_acquire hands out the next slot to fill in place (waiting until its previous H2D has
 * completed); rh_deltas_submit enqueues the H2D of its first n deltas and the device apply and
 * returns without waiting, so the producer fills the other slot while this one is in flight.  One
 * acquire/submit pair at a time per table.  Submitted deltas are not validated on the host: the
 * device ignores a delta with a slot >= capacity, a stopped slot, an unknown column or op. */
#define RH_DELTA_SLOT (1u << 20)
int rh_deltas_acquire(rh_groups* g, rh_delta** out_buf, size_t* out_cap);
int rh_deltas_submit(rh_groups* g, size_t n);
/* Batched LeaderStateImpl.updateCommit() over the dirty slots (see the event model above): stores
 * advanced commit indices in the table and fills *out.  Blocks until *out is ready.
 * flags: RH_COMMIT_WATCH_ALL also reports the changed watch-ALL levels (the module sets it while
 * the server has ALL-level watch requests, WatchRequests.java:146-219); without it out->watch_all
 * is empty and the levels are neither compared nor stored, so the next batch that sets it reports
 * every dirty slot whose level differs from the last one reported. */
#define RH_COMMIT_WATCH_ALL 1u
int rh_commit_batch(rh_groups* g, uint32_t flags, rh_commit_out* out);
/* The same split in two: _async enqueues the evaluation and returns a ticket; _wait blocks until that
 * ticket's results are ready.  Deltas and other calls may be issued in between (they are ordered
 * after it).  No call holds the table's locks while it waits on the device: producers pushing
 * deltas during any _wait (or an _async waiting for an unread earlier result) proceed at once. */
int rh_commit_batch_async(rh_groups* g, uint32_t flags, uint64_t* ticket);
int rh_commit_batch_wait(rh_groups* g, uint64_t ticket, rh_commit_out* out);
/* Where the result lists are assembled.  HOST_MAPPED: the evaluation kernels write the records
 * straight into the pinned result buffers (one range per workgroup, PCIe writes by the GPU),
 * visible when the ticket completes.  AUTO (the default): an evaluation over every tile (up to one
 * record per row) runs without writing records at all -- it stores two event bits per row
 * (updateCommit: advanced, watch-ALL changed; commitIndexChanged: changed, valid) and a gather
 * kernel right behind it on the table's stream rebuilds the records from the table's columns into
 * the pinned buffers (the ticket completes after the gather; no host-issued copy; the table's next
 * writers of those columns come after it in stream order); an evaluation over the dirty-row
 * lists (at most capacity / 32 marked rows) writes its records into the pinned buffers directly.
 * DEVICE: as AUTO, except that a list evaluation writes event bits per listed row, rebuilt the same
 * way from the list entries.  Results are identical.  Not while
 * an evaluation is outstanding (RH_E_STATE). */
#define RH_EVENTS_HOST_MAPPED 0
#define RH_EVENTS_DEVICE      1
#define RH_EVENTS_AUTO        2
int rh_groups_set_event_sink(rh_groups* g, int sink);
/* Diagnostics (benchmarks, tests): with timing enabled every evaluation's kernel launch(es) carry HIP
 * events stamped at the dispatch's start and completion (hipExtLaunchKernel: the kernel boundaries,
 * as a profiler reports them); rh_groups_last_timing returns the last evaluation's device time in ms
 * (blocks until it has completed; RH_E_STATE before any timed evaluation) and, if list_evaluated is
 * not NULL, whether it ran over the dirty-row lists (1: only the rows marked since the previous
 * evaluation of its kind were visited; 2: both kinds' lists in one launch, rh_tick_async; 0: every
 * tile). */
int rh_groups_timing(rh_groups* g, int enable);
int rh_groups_last_timing(rh_groups* g, float* eval_ms, int* list_evaluated);
/* The last timed rh_commit_batch_async / rh_watch_levels_async split (ms, device events): submit =
 * the deltas staged before it (H2D + apply), eval = the evaluation kernels (as above), events = from
 * the evaluation's end until its event records are in the pinned result lists (the REGION gather or
 * the drain on the side stream, their launch and cross-stream wait included; ~0 when the evaluation
 * kernel wrote them itself; the DEVICE sink's copy in _wait not included), gather = the REGION
 * gather kernel alone, at its kernel boundaries (0: none ran).  Blocks until they have completed. */
int rh_groups_last_timing_split(rh_groups* g, float* submit_ms, float* eval_ms, float* events_ms,
                                float* gather_ms, int* list_evaluated);
/* Diagnostics: GPU stores into mapped pinned host memory -- the path the event records take --
 * `bytes` from HBM by the library's 16-byte copy kernel, `reps` launches; *ms = the median one. */
int rh_pcie_write_probe(rh_ctx* ctx, uint64_t bytes, int reps, float* ms);
/* Batched commitIndexChanged() over the slots whose follower commitIndex or leader commitIndex
 * changed: the slots whose {min, majority, max} levels changed, into library-owned pinned memory
 * valid until the next rh_watch_levels / rh_watch_levels_async.  Blocks. */
int rh_watch_levels(rh_groups* g, const rh_watch_event** out_events, uint64_t* out_n);
/* The same split in two (one evaluation outstanding per table: a second _async first waits for the
 * first, whose list it then replaces).  _wait fails with RH_E_STATE when none is outstanding. */
int rh_watch_levels_async(rh_groups* g);
int rh_watch_levels_wait(rh_groups* g, const rh_watch_event** out_events, uint64_t* out_n);
/* A pump tick's two evaluations in one call: rh_commit_batch_async(g, flags, ticket) followed by
 * rh_watch_levels_async(g), collected with rh_commit_batch_wait(g, *ticket, ..) and
 * rh_watch_levels_wait(g, ..) -- the same results (each list in its own order; the _wait calls sort
 * nothing).  When every row marked since the last evaluation of either kind is listed (the sparse
 * tick: the marks since then fit the dirty-row lists, no control op in between) and the sink is not
 * DEVICE, both run in ONE kernel launch: each listed row's updateCommit, then its commitIndexChanged
 * right after in the same lane (the row's levels depend on its new commit index only), then the watch
 * list's other rows (LeaderStateImpl.java:946-950, 612-622 per division); otherwise as the two calls.
 * Replaces the two JNI crossings of LeaderStateImpl's updateCommit + commitIndexChanged per tick. */
int rh_tick_async(rh_groups* g, uint32_t flags, uint64_t* ticket);
/* Reads back one column of slots [first, first + n) (debug / checkpoint / tests): column =
 * RH_COL_MATCH(k) / RH_COL_FCOMMIT(k) / RH_COL_FLUSH / RH_COL_COMMITTED, or RH_COL_CONF (the
 * membership word, as int64) and RH_COL_TERM_START.  Stopped slots read INT64_MIN; follower
 * columns beyond a slot's tier read -1.  Blocks. */
#define RH_COL_CONF       ((uint8_t)34u)
#define RH_COL_TERM_START ((uint8_t)35u)
/* Lease columns (readable, and writable through deltas: RH_OP_SET = Timestamp/AtomicBoolean set,
 * RH_OP_MAX = the later timestamp / OR of the flag).  A new or re-armed slot starts with the lease
 * disabled, no lease and no follower timestamps (INT64_MIN: never active) -- see rh_group_lease_start. */
#define RH_COL_LEASE      ((uint8_t)36u)         /* LeaderLease.lease (System.nanoTime nanos, LL:38)   */
#define RH_COL_LEASE_ON   ((uint8_t)37u)         /* LeaderLease.enabled 0/1 (LL:37; getAndSetEnabled,
                                                    LSI:478, 744, 1042, 1226)                           */
#define RH_COL_TS(k)      ((uint8_t)(48u + (k))) /* follower k lastRespondedAppendEntriesSendTime (nanos,
                                                    FII:236-243; LogAppenderDefault.java:102)           */
int rh_groups_read(rh_groups* g, uint32_t first, uint32_t n, uint8_t column, int64_t* out);
/* Follower width of the tier a slot lives in (0 = stopped), for tests and diagnostics. */
int rh_group_tier(rh_groups* g, uint32_t slot, uint32_t* out_width);

/* ---- leader lease on the resident table (LeaderStateImpl.hasLease LSI:1229-1249, LeaderLease) --
 * A started slot's LeaderLease (new with the LeaderStateImpl, LSI:388): lease = now, enabled as
 * given, and every follower slot of its tier stamped with now (a new FollowerInfoImpl's
 * lastRpcTime, FII:58).  Queued like deltas (after the calls before it).  Later responses arrive
 * as RH_COL_TS(k) deltas; a follower added by rh_group_reconf starts unstamped until its delta. */
int rh_group_lease_start(rh_groups* g, uint32_t slot, int64_t now_nanos, int enabled);
/* hasLease() of every started slot at now_nanos (isRunning() && isReady() stay with the caller):
 * if the lease is enabled and not valid, LeaderLease.extend from the followers' timestamps (majority
 * of the current and old confs active within timeout_ms -> lease = the earliest majority-ack time),
 * stored in the table.  *out_bits: library-owned pinned bitmap, bit s = slot s has the lease, valid
 * until the next rh_lease_batch; *out_words = ceil(capacity / 64).  Blocks. */
int rh_lease_batch(rh_groups* g, int64_t now_nanos, int64_t timeout_ms, const uint64_t** out_bits,
                   uint64_t* out_words);
/* The same split in two, as rh_watch_levels_async / _wait (one batch outstanding per table; the
 * bitmap stays valid until the next rh_lease_batch / rh_lease_batch_async). */
int rh_lease_batch_async(rh_groups* g, int64_t now_nanos, int64_t timeout_ms);
int rh_lease_batch_wait(rh_groups* g, const uint64_t** out_bits, uint64_t* out_words);

/* ---- one RaftServer across several GPUs ---------------------------------------------------
 * A node owns one context and one resident table per device of `device_mask` (bit d = GPU d).
 * A RaftGroup is placed on shard floorMod(UUID.hashCode(), n_shards) of its RaftGroupId
 * (RaftId.hashCode = UUID.hashCode, RaftId.java:119-122), with no inter-GPU traffic on the hot
 * path.  Node slot = shard * capacity_per_shard + table slot; every rh_groups call above has a
 * node form that routes by it. */
typedef struct rh_node rh_node;
/* floorMod(UUID.hashCode(), n): hashCode = (int)(hilo >> 32) ^ (int)hilo, hilo = msb ^ lsb
 * (java.util.UUID.hashCode).  Pure host function; no device needed. */
int rh_shard_of(uint64_t uuid_msb, uint64_t uuid_lsb, int n_shards);
int rh_node_create(uint32_t device_mask, uint64_t capacity_per_shard, int64_t gap_threshold, rh_node** out);
/* The same with an explicit device per shard: shard i lives on GPU devices[i] (1 <= n_shards <= 64;
 * a device may repeat -- several shards on one GPU, each with its own context, stream and table:
 * how a one-GPU box runs the routing, gathering and lease bitmap of an 8-GPU server). */
int rh_node_create_devices(const int* devices, int n_shards, uint64_t capacity_per_shard, int64_t gap_threshold,
                           rh_node** out);
/* Destroys every shard (rh_groups_destroy) and context; the first shard's failure is returned. */
int rh_node_destroy(rh_node* node);
int rh_node_shards(rh_node* node);
/* The shard table (for per-shard calls such as the zero-copy ring) and its context. */
rh_groups* rh_node_groups(rh_node* node, int shard);
rh_ctx* rh_node_ctx(rh_node* node, int shard);
int rh_node_group_start(rh_node* node, uint32_t node_slot, uint32_t conf, int64_t flush_index,
                        int64_t commit_index, int64_t term_start);
int rh_node_group_reconf(rh_node* node, uint32_t node_slot, uint32_t conf, const int8_t* src);
int rh_node_group_stop(rh_node* node, uint32_t node_slot);
/* Splits the deltas by shard (node slots) and pushes each part to its shard's table. */
int rh_node_push_deltas(rh_node* node, const rh_delta* deltas, size_t n);
/* updateCommit on every shard (all launched before any is awaited); the events of all shards,
 * with node slots, are gathered into the caller's arrays (up to the caps; the n_* counts are the
 * totals).  flags as rh_commit_batch.  Blocks. */
int rh_node_commit_batch(rh_node* node, uint32_t flags, rh_index_event* advanced, uint64_t adv_cap,
                         uint64_t* n_advanced, rh_index_event* watch_all, uint64_t watch_cap, uint64_t* n_watch_all);
/* commitIndexChanged() on every shard (all launched before any is awaited): the changed levels of
 * all shards, with node slots, into the caller's array (up to cap; *out_n = the total).  Blocks. */
int rh_node_watch_levels(rh_node* node, rh_watch_event* out, uint64_t cap, uint64_t* out_n);
/* rh_group_lease_start / rh_lease_batch on every shard (all shards' passes in flight before any
 * wait); bit s of the caller's out_bits (at least ceil(shards * capacity_per_shard / 64) words) =
 * node slot s has the lease.  Blocks. */
int rh_node_group_lease_start(rh_node* node, uint32_t node_slot, int64_t now_nanos, int enabled);
int rh_node_lease_batch(rh_node* node, int64_t now_nanos, int64_t timeout_ms, uint64_t* out_bits, uint64_t out_words);

/* ===================================================================================== */
/* 2. CRC32C (PureJavaCrc32C) over SegmentedRaftLog frames                               */
/* ===================================================================================== */

/* Frame = varint32(n) || LogEntryProto (n bytes) || big-endian u32 CRC32C(varint||proto)
 * (OUT:86-110).  Flags: */
#define RH_CRC_VERIFY 1u /* compare with the stored trailer, set bad bit on mismatch (RDR:327-336) */
#define RH_CRC_STAMP  2u /* write the computed CRC into the trailer, big-endian (OUT:100-107)      */
/* With neither flag, frame_len is a plain span length and only crc_out is produced. */

typedef struct rh_frames {
    uint8_t* buf;                 /* device pointer to segment bytes (read-only unless STAMP)   */
    uint64_t buf_len;
    const uint64_t* frame_off;    /* [n] offset of each frame's first varint byte               */
    const uint32_t* frame_len;    /* [n] whole frame length = varint + proto + 4 (VERIFY/STAMP) */
    uint64_t n;
    uint32_t init_state;          /* PureJavaCrc32C state before update(): 0xFFFFFFFF = reset() */
    uint32_t reserved;
    uint32_t* crc_out;            /* [n] optional: getValue() after update(frame bytes)          */
    uint64_t* bad_bits;           /* [ceil(n/64)] optional: stored != computed (VERIFY), or the
                                     frame is malformed (any flags; see rh_crc32c_frames_launch) */
    unsigned long long* n_bad;    /* optional: such frames are atomically added here             */
} rh_frames;

/* CRC of every frame (one call; asynchronous on `stream`).  Lengths <= 2^31; spans shorter than 4
 * bytes are supported; n < 2^32 (else RH_E_RANGE).  When the mean frame length buf_len / n is at
 * most 2 KiB the call sorts the frames by length (20 B of stream-ordered scratch per frame from the
 * context's pool) and folds spans up to 1536 B on 4 or 8 lanes per frame; every other frame, and
 * every frame of a log of longer entries, on 16 lanes per 1 KiB window.  Results do not depend on
 * the split.
 * A MALFORMED frame -- one that does not lie inside [0, buf_len), or (VERIFY/STAMP) is shorter
 * than its 4-byte trailer -- gets crc_out = 0 and, under EVERY flag setting, its bad bit set and
 * n_bad incremented; in STAMP mode it is not stamped.  So bad_bits / n_bad report "mismatch or
 * malformed" for VERIFY and "malformed" for STAMP and flags = 0. */
int rh_crc32c_frames_launch(rh_ctx* ctx, const rh_frames* frames, uint32_t flags, void* stream);

/* Host-buffer convenience (PCIe-inclusive): copies the segment image and frame table to the
 * device, verifies every frame, copies results back.  Returns RH_OK; *n_bad = mismatches. */
int rh_crc32c_verify_host(rh_ctx* ctx, const uint8_t* seg, uint64_t seg_len, const uint64_t* frame_off,
                          const uint32_t* frame_len, uint64_t n, uint32_t* crc_out, uint64_t* bad_bits,
                          uint64_t* n_bad);

/* The write side over a HOST buffer (PCIe-inclusive; what the Java module's flush seam calls,
 * SegmentedRaftLogOutputStream.write OUT:86-110 deferred to BufferedWriteChannel's flush): frame i =
 * buf[frame_off[i], frame_off[i] + frame_len[i]), varint + entry + a 4-byte trailer; every trailer
 * is overwritten with the big-endian PureJavaCrc32C of the bytes before it (reset() state), exactly
 * what write() puts there.  Only the span the frames cover is copied to the device and only the
 * CRCs come back.  Every frame must hold its trailer and lie inside the buffer (RH_E_INVAL, nothing
 * stamped).  Blocks.  A buffer registered with rh_host_register (the worker's reused write buffer)
 * crosses PCIe without staging. */
int rh_crc32c_stamp_host(rh_ctx* ctx, uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off,
                         const uint32_t* frame_len, uint64_t n);
/* Page-locks a host buffer for direct DMA from every GPU (hipHostRegister, portable) until
 * rh_host_unregister. */
int rh_host_register(rh_ctx* ctx, void* p, uint64_t n);
int rh_host_unregister(rh_ctx* ctx, void* p);

/* Checksum.update over one host span (PJC:54-91 update(byte[], off, len)): crc_state is the
 * PureJavaCrc32C `crc` field before the call (0xFFFFFFFF after reset()); *out_state receives it
 * after, so getValue() = ~*out_state.  Reentrant: the span is staged through per-call
 * stream-ordered scratch from the context's pool (no shared staging buffer) and folded by the frame
 * kernel on the context stream, so concurrent callers are safe but run one after another (and
 * after other work on that stream); the call returns when done, as does rh_crc32c_verify_host.  For
 * per-entry call sites prefer batching frames through rh_crc32c_frames_launch (RH_CRC_STAMP /
 * RH_CRC_VERIFY); this entry serves the odd single span (e.g. a snapshot-file checksum). */
int rh_crc32c(rh_ctx* ctx, uint32_t crc_state, const void* data, uint64_t n, uint32_t* out_state);
/* The SURVEY 8(b) `rh_crc32c` contract as a pure host function: Checksum.update over one span on
 * PureJavaCrc32C's internal state (0xFFFFFFFF after reset(); getValue() = ~state), returning the
 * new state.  Pure and reentrant, no context, no device (the CPU's CRC32 instruction, SSE4.2, or a
 * byte table without it); NULL or empty spans return crc_state.  For one-off spans -- the batched
 * paths above stay on the GPU. */
uint32_t rh_crc32c_update(uint32_t crc_state, const void* data, uint64_t n);

/* ---- leader lease (LeaderStateImpl.hasLease LSI:1229-1249; LeaderLease LL:60-103) ------------
 * One tier = groups with the same follower-slot count F (0..14), same conf word as the commit
 * path.  For every active group whose lease is enabled: if the lease is not valid and the conf is
 * not a singleton, try LeaderLease.extend from the followers' lastRespondedAppendEntriesSendTime
 * (majority of the peers responded within the timeout -> lease = earliest majority-ack time of the
 * current and old confs); report hasLease (isRunning()/isReady() stay the caller's).  Times are
 * System.nanoTime() values frozen at now_nanos; elapsed ms truncate like Java long division.
 * Exact for |now - t| < 2^62 ns, where Timestamp.compareTo is a total order. */
typedef struct rh_lease_soa {
    uint64_t n;
    uint32_t n_followers;          /* F, 0..14                                                    */
    uint32_t reserved;
    int64_t now_nanos;
    int64_t timeout_ms;            /* leaseTimeoutMs = rpc.timeout.min x read.leader.lease.timeout.ratio */
    const int64_t* follower_ts;    /* [F][col_stride]: lastRespondedAppendEntriesSendTime (nanos)  */
    uint64_t col_stride;           /* elements between columns, >= n                              */
    const uint32_t* conf;          /* [n] membership word (RH_CONF_*)                             */
    const int64_t* lease_in;       /* [n] current lease timestamp (nanos)                         */
    const uint64_t* enabled_bits;  /* optional [ceil(n/64)] LeaderLease.isEnabled; NULL = enabled */
    int64_t* lease_out;            /* [n] lease after extension; may alias lease_in               */
    uint64_t* has_lease_bits;      /* [ceil(n/64)] hasLease()                                     */
    uint64_t* extended_bits;       /* optional [ceil(n/64)]: the lease was set by extend()        */
    uint64_t tile_stride;          /* 0: plain columns.  Else the TILED layout of rh_commit_soa:
                                      every per-group column (follower_ts, conf, lease_in,
                                      lease_out) holds its RH_TILE_GROUPS elements of a tile
                                      contiguously at its pointer + tile * tile_stride bytes,
                                      follower column k col_stride elements after column 0 within
                                      the tile (col_stride >= 128); a multiple of 16.  Bit columns
                                      stay plain. */
} rh_lease_soa;

int rh_lease_soa_launch(rh_ctx* ctx, const rh_lease_soa* tiers, int n_tiers, void* stream);

/* The leader's per-heartbeat bookkeeping in ONE launch: updateCommit over the commit tiers and
 * hasLease over the lease tiers (typically the same divisions, sharing their conf words).  Same
 * results as rh_commit_soa_launch + rh_lease_soa_launch; commit tiers with F <= 6 and lease tiers
 * with F <= 7 share one kernel (one launch ramp and tail instead of two), wider tiers of either
 * kind run in their own launches on the same stream. */
int rh_leader_soa_launch(rh_ctx* ctx, const rh_commit_soa* commit, int n_commit, const rh_lease_soa* lease,
                         int n_lease, void* stream);

/* ---- segment framing (SegmentedRaftLogReader.verifyHeader / decodeEntry / verifyTerminator) --
 * Walks each segment image: header "RaftLog1" (RDR:179-205), then frames varint32(n) || n bytes ||
 * 4-byte CRC while the first byte is non-zero (RDR:291-323), then checks that the terminator
 * padding is all zero (RDR:251-280).  The walk applies decodeEntry's size rules (maxOpSize, the
 * LimitedInputStream limit) and EOF rules; it does NOT check CRCs -- feed the produced frame table
 * to rh_crc32c_frames_launch(RH_CRC_VERIFY), exactly as readSegmentFile would verify each entry.
 * One 256-thread block per segment; the serial varint chain is walked out of LDS windows. */
#define RH_SEG_END          1   /* clean end: EOF at an entry boundary or zero padding to EOF  */
#define RH_SEG_PARTIAL      2   /* last entry truncated (readEntry returns null, RDR:221-229)  */
#define RH_SEG_E_OVERSIZE  -1   /* entry larger than maxOpSize (RDR:314-317, limit checks)      */
#define RH_SEG_E_PADDING   -3   /* non-zero byte after the terminator (RDR:251-280)            */
#define RH_SEG_E_VARINT    -4   /* malformed / truncated varint (CodedInputStream)             */
#define RH_SEG_E_HEADER    -5   /* corrupted header (CorruptedFileException, RDR:201-204)       */
#define RH_SEG_E_CAPACITY  -6   /* more frames than frames_per_seg_cap                          */
#define RH_SEG_E_RANGE     -7   /* seg_off / seg_len outside [0, buf_len): a caller error, the
                                   segment is not walked (nothing is clamped)                    */

typedef struct rh_segments {
    const uint8_t* buf;           /* device: segment images                                     */
    uint64_t buf_len;
    const uint64_t* seg_off;      /* [n_seg] start of each segment image in buf                 */
    const uint64_t* seg_len;      /* [n_seg] file length of each segment                        */
    uint64_t n_seg;
    uint32_t max_op;              /* raft.server.log.appender.buffer.byte-limit (default 4 MiB) */
    uint32_t frames_per_seg_cap;  /* capacity of each segment's slot in the scratch table      */
    uint64_t* scratch_off;        /* [n_seg * cap] per-segment slotted frame offsets           */
    uint32_t* scratch_len;        /* [n_seg * cap]                                              */
    uint64_t* frame_off;          /* [frame_cap] dense output: absolute offset in buf           */
    uint32_t* frame_len;          /* [frame_cap] whole frame length (varint + proto + 4)        */
    uint64_t frame_cap;
    uint64_t* seg_first;          /* [n_seg] index of the segment's first frame in the output   */
    uint32_t* seg_nframes;        /* [n_seg] frames found before the walk stopped               */
    int32_t* seg_status;          /* [n_seg] RH_SEG_*                                           */
    uint64_t* seg_stop;           /* [n_seg] offset (within the segment) where the walk stopped */
    unsigned long long* total_frames; /* single counter (sum of seg_nframes)                    */
} rh_segments;

int rh_segments_scan_launch(rh_ctx* ctx, const rh_segments* segs, void* stream);

/* ---- read path (LogSegment.readSegmentFile, LogSegment.java:166-196) ----------------------
 * Framing walk + CRC32C verification of every frame (decodeEntry's checksum, RDR:327-336) in one
 * call: fills every rh_segments output exactly as rh_segments_scan_launch does, plus the per-frame
 * CRCs and the reader's verdict per segment -- the reader stops at the first frame whose CRC does
 * not verify (ChecksumException at that frame's offset). */
#define RH_SEG_E_CHECKSUM  -2   /* a frame's stored CRC != computed (ChecksumException, RDR:330-336) */
typedef struct rh_segments_crc {
    uint32_t* scratch_crc;        /* [n_seg * frames_per_seg_cap] computed CRC (getValue()) per slot */
    uint32_t* seg_ok;             /* [n_seg] frames the reader accepts: those before the first CRC failure */
    int32_t*  seg_read_status;    /* [n_seg] RH_SEG_E_CHECKSUM if a frame failed, else seg_status     */
    uint64_t* seg_read_stop;      /* [n_seg] offset (in the segment) of that frame, else seg_stop     */
    uint32_t* crc_out;            /* [frame_cap] optional: computed CRC per frame, dense order        */
    uint64_t* bad_bits;           /* [ceil(frame_cap/64)] optional: stored != computed (zeroed here) */
    unsigned long long* n_bad;    /* optional: CRC mismatches over all found frames (added)          */
} rh_segments_crc;
int rh_segments_read_launch(rh_ctx* ctx, const rh_segments* segs, const rh_segments_crc* crc, void* stream);

/* One segment's outcome of rh_segments_read_host: what LogSegment.readSegmentFile's reader loop
 * (SegmentedRaftLogInputStream.nextEntry -> SegmentedRaftLogReader.readEntry / decodeEntry,
 * LogSegment.java:166-196) meets in that file, minus the LogEntryProto parse. */
typedef struct rh_segment_result {
    int32_t  status;       /* RH_SEG_END / RH_SEG_PARTIAL (the reader returns null: normal end);
                              RH_SEG_E_CHECKSUM (ChecksumException at `stop`, RDR:330-336),
                              RH_SEG_E_OVERSIZE / _PADDING / _VARINT / _HEADER (IOException /
                              CorruptedFileException); RH_SEG_E_CAPACITY / _RANGE: not read here    */
    uint32_t n_ok;         /* entries the reader returns before it stops                           */
    uint64_t stop;         /* offset in the segment where it stopped (the failing frame, or the end) */
    uint64_t first_frame;  /* index of the segment's first frame in frame_off / frame_len / frame_crc */
    uint32_t n_frames;     /* frames the framing walk found (>= n_ok)                              */
    uint32_t reserved;
} rh_segment_result;

/* The read path over HOST segment images (PCIe-inclusive; what the Java module's bulk segment load
 * calls): copies `image` and the segment table to the device, runs rh_segments_read_launch, and
 * copies back each segment's result and the frame table in segment order -- offsets relative to
 * the start of `image`, whole frame lengths (varint + entry + 4), computed CRCs.  Segment i is
 * image[seg_off[i], seg_off[i] + seg_len[i]).  frames_per_seg_cap bounds the frames of one segment
 * (a segment with more reports RH_SEG_E_CAPACITY: read it with the Java reader); the frame arrays
 * hold frame_cap entries and *n_frames_total receives the total found.  Blocks. */
int rh_segments_read_host(rh_ctx* ctx, const uint8_t* image, uint64_t image_len, const uint64_t* seg_off,
                          const uint64_t* seg_len, uint64_t n_seg, uint32_t max_op, uint32_t frames_per_seg_cap,
                          uint64_t* frame_off, uint32_t* frame_len, uint32_t* frame_crc, uint64_t frame_cap,
                          rh_segment_result* results, uint64_t* n_frames_total);
#ifdef __cplusplus
}
#endif
#endif /* RATIS_HIP_H */
