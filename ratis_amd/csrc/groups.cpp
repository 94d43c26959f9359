// Host side of the resident group table (rh_groups) and of the multi-GPU node (rh_node), see
// include/ratis_hip.h.  Device kernels: table.hip.
//
// Reference (ratis tree): the per-division leader commit state this replaces is LeaderStateImpl's
// FollowerInfoMap (LeaderStateImpl.java:262-294), FollowerInfoImpl (FollowerInfoImpl.java:42-151),
// the UPDATE_COMMIT event queue (LeaderStateImpl.java:111-188, 846-854, 900-902) and the
// RaftServerProxy's map of divisions (RaftServerProxy.java:89-150) for the multi-GPU node.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <shared_mutex>
#include <string>
#include <vector>

#include "rh_internal.h"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define RH_EXPORT extern "C" __attribute__((visibility("default")))

#ifndef RH_DELTA_ZC_MAX   // batches of at most this many deltas are applied from the pinned slot in place (A/B:
#define RH_DELTA_ZC_MAX 65536   // profiles/r06/zc_ab/ -- 1 % of 1M rows 68 -> 47 us, 1M-delta streaming 3x slower)
#endif
#ifndef RH_LIST_DIV   // A/B: list mode while at most capacity / RH_LIST_DIV rows can be dirty
#define RH_LIST_DIV 32
#endif

namespace {

using rh::CtrlOp;
using rh::kNoRow;
using rh::kTableTiers;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Highest follower slot a conf word names (new or old mask), + 1; 0 for none.
uint32_t needed_width(uint32_t conf) {
    const uint32_t m = (conf & 0x3FFFu) | ((conf >> RH_CONF_OLD_SHIFT) & 0x3FFFu);
    return m ? 32u - (uint32_t)__builtin_clz(m) : 0u;
}

struct TierHost {
    uint32_t hw = 0;                      // rows handed out so far (high-water mark)
    std::vector<uint32_t> free_rows;      // released rows, reusable
    std::vector<uint32_t> pending_free;   // released by queued ops: reusable after the next flush
};

constexpr int kEvSets = 3;  // results of the last three rh_commit_batch_async calls stay readable

struct EvSet {
    rh_index_event* adv = nullptr;   // host-mapped pinned [cap]: the contiguous result lists
    rh_index_event* wall = nullptr;
    rh_index_event* d_adv = nullptr;  // device views of the same memory
    rh_index_event* d_wall = nullptr;
    rh_index_event* hbm_adv = nullptr;   // the lists in HBM (RH_EVENTS_DEVICE, RH_EVENTS_AUTO's tile evaluations)
    rh_index_event* hbm_wall = nullptr;
    uint32_t* bdesc = nullptr;           // REGION mode: the evaluation's per-workgroup counts
    uint32_t nblocks = 0;                // REGION mode: its workgroups (0: the lists are contiguous)
    uint64_t* h_cnt = nullptr;       // host-mapped [2]: list lengths, written by the gather kernel
    uint64_t* d_cnt = nullptr;
    hipEvent_t done = nullptr;
    uint64_t ticket = 0;
    bool pending = false;
    bool hbm = false;   // this ticket's lists are in hbm_adv / hbm_wall (copied out by _wait)
};

// HBM list capacity: the table's capacity plus room for the REGION mode's per-workgroup regions
// (every tier's last workgroup may be partial and the tiers round their rows up to 128).
uint64_t hbm_records(uint64_t capacity) { return capacity + (uint64_t)(rh::kTableTiers + 1) * rh::kTableRecs; }
uint64_t region_blocks(uint64_t capacity) { return hbm_records(capacity) / rh::kTableRecs + rh::kTableTiers + 1; }
// list capacity: a list evaluation is chosen while at most capacity / RH_LIST_DIV rows can be dirty
uint32_t list_cap(uint64_t capacity) { return (uint32_t)std::max<uint64_t>(1024, capacity / RH_LIST_DIV); }
// words between the two hasLease bitmaps (an even number: both 16-byte aligned)
uint64_t lbits_stride(uint64_t capacity) { return ((capacity + 63) / 64 + 1) / 2 * 2; }
// REGION-mode descriptors per result set: a tile evaluation's workgroups or a list evaluation's
uint64_t desc_blocks(uint64_t capacity) {
    return std::max<uint64_t>(region_blocks(capacity), rh::table_list_desc_blocks(list_cap(capacity)));
}

}  // namespace

struct rh_groups {
    rh_ctx* ctx = nullptr;
    uint64_t capacity = 0;
    int64_t gap = -1;
    std::mutex mu;
    // Delta staging (rh_push_deltas, multi-producer): `smu` shared = producers validating and copying
    // into the open host slot at ranges reserved with one CAS on `fill`; exclusive = whoever
    // submits the staged deltas (a full slot, an evaluation, a control op on a staged slot, a read,
    // the zero-copy path).  Lock order: smu, then mu.  `mu` guards everything else.
    std::shared_mutex smu;
    rh::TableDev dev;                         // device pointers (copied into every launch)
    std::vector<uint32_t> slot_map;           // host mirror of dev.slot_map
    std::vector<uint32_t> slot_conf;          // host mirror of each started slot's conf word
    TierHost tiers[kTableTiers];
    // control ops: queued on the host, applied by table_control_kernel in stream order
    std::vector<CtrlOp> ops;
    std::vector<uint32_t> op_stamp;           // slot -> batch generation that holds an op for it
    uint32_t op_gen = 1;
    CtrlOp* h_ops = nullptr;                  // pinned staging
    CtrlOp* d_ops = nullptr;
    size_t ops_cap = 0;
    hipEvent_t ops_free = nullptr;
    bool ops_used = false;
    // delta staging: two pinned host slots, each with its own device buffer; the H2D copies run on
    // a copy stream, so the copy of batch s+1 overlaps the apply / evaluation of batch s
    rh_delta* h_ring[2] = {nullptr, nullptr};
    rh_delta* d_ring[2] = {nullptr, nullptr};
    const rh_delta* d_hring[2] = {nullptr, nullptr};   // device views of h_ring (small batches: read in place)
    hipEvent_t ring_free[2] = {nullptr, nullptr};   // H2D of the slot done (host slot reusable)
    hipEvent_t ring_read[2] = {nullptr, nullptr};   // apply of the slot done (device slot reusable)
    bool ring_used[2] = {false, false};
    // the host slot is free again when ring_done[i] completes: ring_free[i], or -- after an in-place
    // apply, which records no event of its own (an event record is ~4.6 us on the stream's timeline) --
    // the done event of the next evaluation issued behind it (ring_lazy[i] until then)
    hipEvent_t ring_done[2] = {nullptr, nullptr};
    bool ring_lazy[2] = {false, false};
    // the slot was filled by rh_push_deltas, which stores each delta's row code (tier << 28 | row, the
    // host slot map's) in its slot field: the apply skips the device slot map (false: rh_deltas_acquire)
    bool ring_resolved[2] = {false, false};
    int ring_next = 0;
    int ring_acquired = -1;
    int open = -1;                            // host slot open for rh_push_deltas (-1: none)
    std::atomic<uint64_t> fill{0};            // deltas reserved in the open slot
    std::atomic<bool> staged_set{false};      // some staged delta is a SET
    uint32_t apply_gen = 0;                   // order-key generation of the last batch with SETs
    hipStream_t copy_stream = nullptr;       // H2D of delta slots and control ops
    hipStream_t d2h_stream = nullptr;        // the result lists' way to the host: RH_EVENTS_DEVICE's D2H in
                                             // _wait, RH_EVENTS_AUTO's drain kernel after the evaluation
    hipEvent_t evaluated = nullptr;          // recorded after an evaluation: orders the drain behind it
    // REGION-mode updateCommit records are rebuilt from the table's row-slot / commit / watch-ALL
    // columns by rh_table_gather_commit on d2h_stream: every later launch that writes those columns
    // (an updateCommit evaluation, control ops, a delta batch, a load, a tier's move) is ordered
    // after it (gather_fence)
    hipEvent_t gathered = nullptr;
    bool gather_pending = false;
    // the same for commitIndexChanged's records (row-slot, wmin / wmaj / wmax columns: written by a
    // watch evaluation, control ops, a load)
    hipEvent_t wgathered = nullptr;
    bool wgather_pending = false;
    bool wgather_list = false;   // ... and it reads the commitIndexChanged list's entries (list_fence)
    uint64_t* d_lbits = nullptr;  // rh_lease_batch: two slot bitmaps (device; a pass clears the other) and the pinned copy
    int lbuf = 0;                 // the bitmap the next pass sets (zero)
    uint64_t* h_lbits = nullptr;
    uint64_t* d_hlbits = nullptr;  // device view of h_lbits (the pass's last kernel writes it across PCIe)
    // events (rh_internal.h, TableEvents): the evaluation counter words, result sets
    EvSet ev[kEvSets];
    uint64_t next_ticket = 1;
    unsigned long long* d_evw = nullptr;      // [2 * kHeadStride]: counter word, then the done word
    rh_watch_event* watch = nullptr;          // host-mapped pinned [cap]: rh_watch_levels' list
    rh_watch_event* d_watch = nullptr;
    rh_watch_event* hbm_watch = nullptr;      // in HBM (as hbm_adv)
    uint32_t* wbdesc = nullptr;               // REGION mode (as EvSet::bdesc)
    uint32_t wnblocks = 0;
    uint64_t* h_wcnt = nullptr;               // host-mapped [2]: its length (the evaluation's last workgroup)
    uint64_t* d_wcnt = nullptr;
    hipEvent_t wdone = nullptr;
    // the watch list of a fused tick completes with that tick's result set: wtick = its ticket (0: the
    // list has its own wdone), wseen = the commit wait of that ticket has seen it complete
    uint64_t wtick = 0;
    bool wseen = false;
    bool wpending = false, whbm = false;
    uint64_t wgen = 0;                        // watch evaluations started (a waiter re-validates it)
    hipEvent_t ldone = nullptr;               // rh_lease_batch_async's bitmap D2H
    bool lpending = false;
    uint64_t lgen = 0;
    // dirty-row lists (rh_internal.h, TableLists), per kind (0 = updateCommit, 1 = commitIndexChanged)
    uint32_t* d_lrows[2] = {nullptr, nullptr};   // [kHeads][lcap]: (tier << 28) | row
    unsigned long long* d_lheads = nullptr;      // [2 kinds][2 sets][kHeads * kHeadStride]
    uint32_t lcap = 0;
    int lpar[2] = {0, 0};       // the set appends go to
    bool lvalid[2] = {true, true};   // every row marked since the kind's last evaluation is listed
    uint64_t lmarks[2] = {0, 0};     // bound on the rows marked since then
    uint64_t marks[2] = {0, 0};      // deltas of each kind since its last evaluation (lists or not)
    int last_list = 0;          // the last evaluation: 0 tiles, 1 the dirty-row lists, 2 both kinds' lists in one launch
    // rh_groups_timing: [0] / [1] the evaluation's kernel boundaries, [2] before the staged deltas'
    // submission (H2D + apply), [3] after the event records reached the pinned lists (gather / drain,
    // or the evaluation itself when its kernel wrote them)
    // [4] / [5] the gather kernel's boundaries (gathered: whether the last timed _async ran one)
    hipEvent_t tev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool timing = false, timed = false, gathered_timed = false;
    int event_sink = RH_EVENTS_AUTO;
    uint32_t cbits = 28;   // bits per list count in the evaluation's counter word (TableEvents)
    int64_t* d_read = nullptr;
    size_t read_cap = 0;
    unsigned long long* d_tick = nullptr;   // [3 * kHeadStride]: the fused tick's counters (rh::TickEvents)
    uint64_t map_gen = 0;   // bumped by every slot_map change (exclusive side): a push's checks stay valid while it holds
};

namespace {

template <typename T>
int dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) return RH_OK;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
    if (e != hipSuccess) return rh::fail(RH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return RH_OK;
}

template <typename T>
int halloc_mapped(T** host, T** dev, size_t count) {
    *host = nullptr;
    *dev = nullptr;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(host), std::max<size_t>(count, 1) * sizeof(T), hipHostMallocMapped);
    if (e != hipSuccess) return rh::fail(RH_E_NOMEM, "hipHostMalloc(mapped event buffer)");
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(dev), *host, 0);
    if (e != hipSuccess) return rh::hip_fail(e, "hipHostGetDevicePointer");
    return RH_OK;
}

void free_tier(rh::TableTier& t) {
    (void)hipFree(t.base);
    (void)hipFree(t.sum);
    (void)hipFree(t.shadow);
    t = rh::TableTier{};
}

void free_groups(rh_groups* g) {
    for (auto& t : g->dev.tier) free_tier(t);
    (void)hipFree(g->dev.slot_map);
    (void)hipFree(g->d_ops);
    if (g->h_ops) (void)hipHostFree(g->h_ops);
    if (g->ops_free) (void)hipEventDestroy(g->ops_free);
    for (int i = 0; i < 2; ++i) {
        if (g->h_ring[i]) (void)hipHostFree(g->h_ring[i]);
        (void)hipFree(g->d_ring[i]);
        if (g->ring_free[i]) (void)hipEventDestroy(g->ring_free[i]);
        if (g->ring_read[i]) (void)hipEventDestroy(g->ring_read[i]);
    }
    for (int i = 0; i < kEvSets; ++i) {
        if (g->ev[i].adv) (void)hipHostFree(g->ev[i].adv);
        if (g->ev[i].wall) (void)hipHostFree(g->ev[i].wall);
        if (g->ev[i].h_cnt) (void)hipHostFree(g->ev[i].h_cnt);
        if (g->ev[i].done) (void)hipEventDestroy(g->ev[i].done);
        (void)hipFree(g->ev[i].hbm_adv);
        (void)hipFree(g->ev[i].hbm_wall);
        (void)hipFree(g->ev[i].bdesc);
    }
    (void)hipFree(g->d_lrows[0]);
    (void)hipFree(g->d_lrows[1]);
    (void)hipFree(g->d_lheads);
    (void)hipFree(g->hbm_watch);
    (void)hipFree(g->wbdesc);
    (void)hipFree(g->d_evw);
    (void)hipFree(g->d_tick);
    if (g->watch) (void)hipHostFree(g->watch);
    if (g->h_wcnt) (void)hipHostFree(g->h_wcnt);
    if (g->wdone) (void)hipEventDestroy(g->wdone);
    if (g->ldone) (void)hipEventDestroy(g->ldone);
    for (hipEvent_t e : g->tev)
        if (e) (void)hipEventDestroy(e);
    (void)hipFree(g->d_read);
    if (g->copy_stream) (void)hipStreamDestroy(g->copy_stream);
    if (g->d2h_stream) (void)hipStreamDestroy(g->d2h_stream);
    if (g->evaluated) (void)hipEventDestroy(g->evaluated);
    if (g->gathered) (void)hipEventDestroy(g->gathered);
    if (g->wgathered) (void)hipEventDestroy(g->wgathered);
    (void)hipFree(g->d_lbits);
    if (g->h_lbits) (void)hipHostFree(g->h_lbits);
}

// Orders the table stream's next launch after the last updateCommit record gather (see `gathered`).
// A gather of a list evaluation also reads that list's entries, which the next appends overwrite:
// the delta apply (every kind) and an updateCommit list evaluation (the commitIndexChanged list).
#ifndef RH_GATHER_SIDE   // A/B: a REGION gather on the side stream behind an event (1) or on the table stream (0)
#define RH_GATHER_SIDE 0
#endif
#ifndef RH_GATHER_FENCE   // test-sensitivity builds only (0: no fence -- wrong results)
#define RH_GATHER_FENCE 1
#endif
int gather_fence(rh_groups* g) {
    if (!RH_GATHER_FENCE || !g->gather_pending) return RH_OK;
    RH_HIP(hipStreamWaitEvent(g->ctx->stream, g->gathered, 0));
    g->gather_pending = false;
    return RH_OK;
}

// The same for the last commitIndexChanged record gather (see `wgathered`).
int wgather_fence(rh_groups* g) {
    if (!RH_GATHER_FENCE || !g->wgather_pending) return RH_OK;
    RH_HIP(hipStreamWaitEvent(g->ctx->stream, g->wgathered, 0));
    g->wgather_pending = false;
    g->wgather_list = false;
    return RH_OK;
}

// Before a launch that appends to the commitIndexChanged list: the last watch gather, if it reads
// that list's entries.
int list_fence(rh_groups* g) { return g->wgather_list ? wgather_fence(g) : RH_OK; }

// (Re)allocates tier t with `rows` rows (a multiple of 128), keeping the old rows' contents: tiles
// keep their position, so the old tiles and summaries are one copy each and the new tiles start
// free.  Blocks (the old arrays are released after the stream has drained every launch that still
// names them).
int grow_tier(rh_groups* g, int t, uint32_t rows) {
    rh::TableTier n{};
    const rh::TableTier& o = g->dev.tier[t];
    n.width = rh::width_of_tier(t);
    n.rows = rows;
    const uint64_t TB = rh::tile::bytes(n.width);
    const uint32_t tiles = rows / rh::kTileRows, keep = o.rows / rh::kTileRows;
    int rc = dalloc(&n.base, (size_t)tiles * TB);
    if (rc == RH_OK) rc = dalloc(&n.sum, (size_t)tiles * 2);
    if (rc == RH_OK) rc = dalloc(&n.shadow, (size_t)tiles * TB);
    if (rc != RH_OK) {
        free_tier(n);
        return rc;
    }
    hipStream_t s = g->ctx->stream;
    hipError_t e = hipSuccess;
    if (keep) {
        e = hipMemcpyAsync(n.base, o.base, (size_t)keep * TB, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(n.sum, o.sum, (size_t)keep * 2, hipMemcpyDeviceToDevice, s);
    }
    // order keys of earlier batches never matter again (a key counts only within its generation)
    if (e == hipSuccess) e = hipMemsetAsync(n.shadow, 0, (size_t)tiles * TB, s);
    if (e == hipSuccess) rc = rh_table_init_tiles(n, keep, tiles - keep, s);
    if (e == hipSuccess && rc == RH_OK) e = hipStreamSynchronize(s);
    if (e == hipSuccess && rc == RH_OK) e = hipStreamSynchronize(g->d2h_stream);   // a gather may read the old tiles
    if (e != hipSuccess || rc != RH_OK) {
        free_tier(n);
        return rc != RH_OK ? rc : rh::hip_fail(e, "rh_groups: tier growth");
    }
    rh::TableTier old = o;
    g->dev.tier[t] = n;
    free_tier(old);
    return RH_OK;
}

// The table with each tier cut at its high-water mark (rounded up to a tile): rows past it were
// never handed out, so passes over every row skip them; *rows: the rows left.
rh::TableDev clipped(const rh_groups* g, uint64_t* rows) {
    rh::TableDev ed = g->dev;
    uint64_t n = 0;
    for (int t = 0; t < rh::kTableTiers; ++t) {
        const uint64_t hw = ((uint64_t)g->tiers[t].hw + rh::kTileRows - 1) / rh::kTileRows * rh::kTileRows;
        ed.tier[t].rows = (uint32_t)std::min<uint64_t>(ed.tier[t].rows, hw);
        n += ed.tier[t].rows;
    }
    if (rows) *rows = n;
    return ed;
}

// A row of tier t for a new occupant.
int alloc_row(rh_groups* g, int t, uint32_t* row) {
    TierHost& h = g->tiers[t];
    if (!h.free_rows.empty()) {
        *row = h.free_rows.back();
        h.free_rows.pop_back();
        return RH_OK;
    }
    if (h.hw >= g->dev.tier[t].rows) {
        const uint64_t want = std::max<uint64_t>(1024, (uint64_t)g->dev.tier[t].rows * 2);
        const uint64_t cap = (g->capacity + 127) / 128 * 128;
        const uint32_t rows = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(want, h.hw + 128), std::max<uint64_t>(cap, 128));
        if (rows <= h.hw) return rh::fail(RH_E_RANGE, "rh_groups: tier full");
        int rc = grow_tier(g, t, (rows + 127) / 128 * 128);
        if (rc != RH_OK) return rc;
    }
    *row = h.hw++;
    return RH_OK;
}

// Enqueues the H2D of the queued control ops and their kernel; rows they released become reusable.
int flush_ops(rh_groups* g) {
    const size_t n = g->ops.size();
    if (n) {
        hipStream_t s = g->ctx->stream;
        if (g->ops_used) RH_HIP(hipEventSynchronize(g->ops_free));  // staging still being read
        if (n > g->ops_cap) {
            if (g->h_ops) (void)hipHostFree(g->h_ops);
            (void)hipFree(g->d_ops);
            g->h_ops = nullptr;
            g->d_ops = nullptr;
            g->ops_cap = 0;
            const size_t cap = std::max<size_t>(n, 4096);
            if (hipHostMalloc(reinterpret_cast<void**>(&g->h_ops), cap * sizeof(CtrlOp)) != hipSuccess)
                return rh::fail(RH_E_NOMEM, "rh_groups: control-op staging");
            int rc = dalloc(&g->d_ops, cap);
            if (rc != RH_OK) return rc;
            g->ops_cap = cap;
        }
        std::memcpy(g->h_ops, g->ops.data(), n * sizeof(CtrlOp));
        RH_HIP(hipMemcpyAsync(g->d_ops, g->h_ops, n * sizeof(CtrlOp), hipMemcpyHostToDevice, s));
        RH_HIP(hipEventRecord(g->ops_free, s));
        g->ops_used = true;
        int rc = gather_fence(g);   // control ops write row slots, commit indices and levels
        if (rc == RH_OK) rc = wgather_fence(g);
        if (rc != RH_OK) return rc;
        rc = rh_table_control(g->dev, g->d_ops, n, s);
        if (rc != RH_OK) return rc;
        g->ops.clear();
        g->lvalid[0] = g->lvalid[1] = false;   // control ops mark rows with plain stores: no lists
    }
    ++g->op_gen;
    for (auto& t : g->tiers) {
        t.free_rows.insert(t.free_rows.end(), t.pending_free.begin(), t.pending_free.end());
        t.pending_free.clear();
    }
    return RH_OK;
}

// Queues one control op for `slot` (flushing first if the current batch already holds one).
int queue_op(rh_groups* g, const CtrlOp& op) {
    if (g->op_stamp[op.slot] == g->op_gen) {
        int rc = flush_ops(g);
        if (rc != RH_OK) return rc;
    }
    g->op_stamp[op.slot] = g->op_gen;
    g->ops.push_back(op);
    if (g->ops.size() >= (1u << 16)) return flush_ops(g);
    return RH_OK;
}

uint32_t enc(int t, uint32_t row) { return ((uint32_t)t << 28) | row; }

constexpr size_t kListRegions = (size_t)rh::kHeads;   // one list region per XCD head (entries carry their tier)

unsigned long long* lheads_of(rh_groups* g, int kind, int set) {
    return g->d_lheads + (size_t)(kind * 2 + set) * kListRegions * rh::kHeadStride;
}

// The list `kind` for `n_marks` more possible markings: maintained while the bound stays within the
// list capacity; past it the kind's list is given up until its next evaluation (a tile evaluation).
rh::TableLists lists_for(rh_groups* g, int kind, uint64_t n_marks) {
    rh::TableLists l;
    if (g->lvalid[kind] && g->lmarks[kind] + n_marks <= g->lcap) {
        g->lmarks[kind] += n_marks;
        l.rows = g->d_lrows[kind];
        l.heads = lheads_of(g, kind, g->lpar[kind]);
        l.cap = g->lcap;
    } else {
        g->lvalid[kind] = false;
    }
    return l;
}

// After a failed evaluation launch (some workgroups may have counted, a later launch of the
// evaluation may not have run): drain the stream and zero the counter words and every list head,
// so the next evaluation starts from clean counters.
int reset_heads(rh_groups* g) {
    hipStream_t s = g->ctx->stream;
    (void)hipStreamSynchronize(s);
    RH_HIP(hipMemsetAsync(g->d_evw, 0, (size_t)2 * rh::kHeadStride * 8, s));
    RH_HIP(hipMemsetAsync(g->d_lheads, 0, (size_t)4 * kListRegions * rh::kHeadStride * 8, s));
    RH_HIP(hipMemsetAsync(g->d_tick, 0, (size_t)3 * rh::kHeadStride * 8, s));
    RH_HIP(hipStreamSynchronize(s));
    g->lvalid[0] = g->lvalid[1] = false;   // the next evaluations run the tile kernels
    return RH_OK;
}

// The result lists an evaluation may write: [0] the pinned buffers (device pointers of the host
// mapping), [1] their HBM twins.
struct EvTargets {
    rh_index_event* adv[2] = {nullptr, nullptr};
    rh_index_event* wall[2] = {nullptr, nullptr};
    rh_watch_event* watch[2] = {nullptr, nullptr};
};

#ifndef RH_SPEC_DIV   // SPEC tile evaluations from marks >= rows / RH_SPEC_DIV (A/B)
#define RH_SPEC_DIV 4
#endif
#ifndef RH_LIST_REGION   // A/B: list evaluations into HBM in REGION mode (1) or with the counter atomic (0)
#define RH_LIST_REGION 1
#endif
// AUTO: list evaluations of fewer marked rows write the pinned lists directly (A/B).  Round 6: every
// list evaluation does -- what the host waits for, from _async to the records in the pinned lists,
// at 1 % of 1M rows 67 us against 95 us by REGION masks + the gather (the kernel itself 10.1 against
// 9.0 us), at 3 % 83 against 112 us (profiles/r06/pin_ab/)
#ifndef RH_LIST_PINNED_MAX
#define RH_LIST_PINNED_MAX (~0ull)
#endif

// Enqueues one evaluation (mode) of the dirty rows, its events written into the lists adv / wall
// or watch of `t` (their lengths to counts_out, host-mapped).  The sink picks the set: HOST_MAPPED
// [0], DEVICE [1], AUTO [1] for a tile evaluation (up to every row's records: written at HBM speed,
// gathered into the pinned lists afterwards) and [0] for a list evaluation (few records: written
// across PCIe by the kernel, no copy).  *hbm: whether [1] was used.  A tile evaluation into [1]
// runs in REGION mode (rh_internal.h, TableEvents): per-workgroup masks and totals in `bdesc`, no
// counter atomic, no records: the caller's rh_table_gather_commit / _watch rebuilds them and
// publishes the lengths; *nblocks = its workgroups (else 0), *ed_out its clipped table.
int evaluate(rh_groups* g, int mode, bool wall_on, const EvTargets& t, uint64_t* counts_out, uint64_t* h_counts,
             bool* hbm, uint32_t* bdesc, uint32_t* nblocks, rh::TableDev* ed_out = nullptr, rh::ListRegion* lr_out = nullptr) {
    hipStream_t s = g->ctx->stream;
    *hbm = false;
    *nblocks = 0;
    if (lr_out) *lr_out = rh::ListRegion{};
    int rc = flush_ops(g);
    if (rc == RH_OK) rc = mode != RH_MODE_WATCH ? gather_fence(g) : wgather_fence(g);   // it rewrites the values a gather reads
    // an updateCommit list evaluation appends to the commitIndexChanged list a watch gather may read
    if (rc == RH_OK && mode != RH_MODE_WATCH && g->lvalid[0]) rc = list_fence(g);
    if (rc != RH_OK) return rc;
    const uint32_t blocks = rh::table_commit_blocks(g->dev);
    if (blocks == 0) {   // no tier has rows: nothing can be dirty
        h_counts[0] = h_counts[1] = 0;
        return RH_OK;
    }
    const int m = mode == RH_MODE_WATCH ? 1 : 0;
    const bool list = g->lvalid[m];   // every row marked since the last evaluation is listed
    // AUTO: HBM lists (gathered / drained on the side stream) for a tile evaluation; a list
    // evaluation writes its records across PCIe itself (RH_LIST_PINNED_MAX above)
    const bool few = list && g->marks[m] < RH_LIST_PINNED_MAX;
    const int k = (g->event_sink == RH_EVENTS_DEVICE || (g->event_sink == RH_EVENTS_AUTO && !few)) ? 1 : 0;
    rh::TableEvents ev;
    ev.adv = t.adv[k];
    ev.wall = wall_on ? t.wall[k] : nullptr;
    ev.watch = t.watch[k];
    ev.cap = g->capacity;
    ev.cnt = g->d_evw;
    ev.done = reinterpret_cast<unsigned int*>(g->d_evw + rh::kHeadStride);
    ev.counts_out = counts_out;
    ev.cbits = g->cbits;
    ev.lheads_next = lheads_of(g, m, g->lpar[m] ^ 1);
    hipEvent_t t0 = g->timing ? g->tev[0] : nullptr, t1 = g->timing ? g->tev[1] : nullptr;
    if (list) {
        rh::TableLists l;
        l.rows = g->d_lrows[m];
        l.heads = lheads_of(g, m, g->lpar[m]);
        l.cap = g->lcap;
        // COMMIT marks the rows whose commit advanced for commitIndexChanged: at most the listed ones
        const rh::TableLists lw = m == 0 ? lists_for(g, 1, g->lmarks[0]) : rh::TableLists{};
        // REGION mode into [1] (masks per wave and pass, no counter atomic, no records): the
        // caller's gather rebuilds the records from the list entries and the table
        const uint32_t grid = rh::table_list_grid(g->lmarks[m]);
        const uint32_t passes = rh::table_list_passes(grid, std::min<uint64_t>(g->lmarks[m], g->lcap));
        if (RH_LIST_REGION && k == 1 && lr_out && ed_out && passes && (uint64_t)passes * grid <= desc_blocks(g->capacity)) {
            ev.bdesc = bdesc;
            ev.list_passes = passes;
            *nblocks = passes * grid;
            *ed_out = g->dev;
            lr_out->rows = g->d_lrows[m];
            lr_out->cap = g->lcap;
            lr_out->grid = grid;
        }
        rc = rh_table_commit_lists(g->dev, mode, l, lw, ev, s, t0, t1, g->lmarks[m]);
    } else {
        if (m == 0) g->lvalid[1] = false;   // the tile kernel marks wdirty with plain stores
        // tiles at or past a tier's high-water mark hold no row ever handed out (clean): the
        // evaluation covers the tiles below it only
        uint64_t rows = 0;
        const rh::TableDev ed = clipped(g, &rows);
        const uint32_t nb = rh::table_commit_blocks(ed);
        if (k == 1 && nb <= region_blocks(g->capacity) && (uint64_t)nb * rh::kTableRecs <= hbm_records(g->capacity)) {
            ev.bdesc = bdesc;
            ev.cap = hbm_records(g->capacity);
            *nblocks = nb;
            if (ed_out) *ed_out = ed;
        }
        // a quarter of the rows or more possibly dirty: the loads go out with the flag loads
        rc = rh_table_commit(ed, mode, ev, g->marks[m] * RH_SPEC_DIV >= rows, s, t0, t1);
    }
    if (rc == RH_OK && g->timing) g->timed = true;
    if (rc != RH_OK) {
        const std::string msg = rh_last_error();
        (void)reset_heads(g);
        return rh::fail(rc, msg);
    }
    *hbm = k == 1;
    g->lpar[m] ^= 1;  // ... and the other list set of this kind: fresh lists from here on
    g->lmarks[m] = 0;
    if (m == 0) g->marks[1] += g->marks[0];   // rows whose commit advanced are marked for commitIndexChanged
    g->marks[m] = 0;
    g->lvalid[m] = true;
    g->last_list = list ? 1 : 0;
    return RH_OK;
}

int do_stop(rh_groups* g, uint32_t slot) {
    const uint32_t m = g->slot_map[slot];
    if (m == kNoRow) return RH_OK;
    CtrlOp op{};
    op.kind = rh::kCtrlStop;
    op.slot = slot;
    op.src = m;
    int rc = queue_op(g, op);
    if (rc != RH_OK) return rc;
    g->tiers[m >> 28].pending_free.push_back(m & rh::kRowMask);
    g->slot_map[slot] = kNoRow;
    ++g->map_gen;
    g->slot_conf[slot] = 0;
    return RH_OK;
}

// The event whose completion frees host slot i (nullptr: never used).  A slot applied in place with
// no evaluation issued since gets ring_free[i] recorded now, behind that apply.
int slot_event(rh_groups* g, int i, hipEvent_t* ev) {
    *ev = nullptr;
    if (!g->ring_used[i]) return RH_OK;
    if (g->ring_lazy[i]) {
        RH_HIP(hipEventRecord(g->ring_free[i], g->ctx->stream));
        g->ring_done[i] = g->ring_free[i];
        g->ring_lazy[i] = false;
    }
    *ev = g->ring_done[i];
    return RH_OK;
}

// An evaluation's done event `ev`, recorded behind every apply enqueued so far, frees the slots applied
// in place (any later re-record of `ev` completes later still).
void slots_freed_by(rh_groups* g, hipEvent_t ev) {
    for (int i = 0; i < 2; ++i)
        if (g->ring_lazy[i]) {
            g->ring_done[i] = ev;
            g->ring_lazy[i] = false;
        }
}

int ring_wait(rh_groups* g, int i) {
    hipEvent_t ev = nullptr;
    int rc = slot_event(g, i, &ev);
    if (rc == RH_OK && ev) RH_HIP(hipEventSynchronize(ev));
    return rc;
}

// H2D of the first n deltas of ring slot i on the copy stream (after the previous apply that read
// device slot i), then the apply phases on the table stream (after that H2D).  has_set: the batch
// may hold SET deltas (their order keys are recorded first, rh_internal.h ApplyPhase).
int ring_submit(rh_groups* g, int i, size_t n, bool has_set) {
    hipStream_t s = g->ctx->stream, cs = g->copy_stream;
    int rc = flush_ops(g);
    if (rc != RH_OK) return rc;
    // a small batch (a pump tick's replies) is read by the apply kernels straight from the pinned
    // slot across PCIe: no DMA set-up and no cross-stream wait on the tick's path; the host slot is
    // free again once they are done.  Large batches go by DMA on the copy stream (overlapping the
    // previous batch's apply), read from HBM by the apply phases.
    const bool zc = n <= (size_t)RH_DELTA_ZC_MAX && g->d_hring[i] != nullptr;
    const rh_delta* src = zc ? g->d_hring[i] : g->d_ring[i];
    if (!zc) {
        if (g->ring_used[i]) RH_HIP(hipStreamWaitEvent(cs, g->ring_read[i], 0));
        RH_HIP(hipMemcpyAsync(g->d_ring[i], g->h_ring[i], n * sizeof(rh_delta), hipMemcpyHostToDevice, cs));
        RH_HIP(hipEventRecord(g->ring_free[i], cs));
        RH_HIP(hipStreamWaitEvent(s, g->ring_free[i], 0));
    }
    rc = gather_fence(g);   // RH_COL_COMMITTED deltas write the commit column; appends, the lists
    if (rc == RH_OK) rc = list_fence(g);
    if (rc != RH_OK) return rc;
    g->ring_used[i] = true;
    g->ring_next = i ^ 1;
    // every delta marks at most one row per kind
    const rh::TableLists lc = lists_for(g, 0, n), lw = lists_for(g, 1, n);
    g->marks[0] += n;
    g->marks[1] += n;
    uint32_t gen = 0;
    if (has_set) {
        if (g->apply_gen == 0xFFFFFFFFu) {   // generations wrapped: no stale key may look current
            for (const rh::TableTier& t : g->dev.tier)
                if (t.shadow) RH_HIP(hipMemsetAsync(t.shadow, 0, (size_t)(t.rows / rh::kTileRows) * rh::tile::bytes(t.width), s));
            g->apply_gen = 0;
        }
        gen = ++g->apply_gen;
        rc = rh_table_apply_deltas(g->dev, src, n, kApplyKeys, gen, lc, lw, s, g->ring_resolved[i]);
        if (rc == RH_OK) rc = rh_table_apply_deltas(g->dev, src, n, kApplySet, gen, lc, lw, s, g->ring_resolved[i]);
        if (rc != RH_OK) return rc;
    }
    rc = rh_table_apply_deltas(g->dev, src, n, kApplyMax, gen, lc, lw, s, g->ring_resolved[i]);
    if (rc != RH_OK) return rc;
    if (zc) {   // the host slot was read by the apply itself: freed by the next evaluation's event
        g->ring_lazy[i] = true;   // (the device slot was not read: ring_read[i] stays the last DMA apply's)
        g->ring_done[i] = nullptr;
    } else {
        RH_HIP(hipEventRecord(g->ring_read[i], s));
        g->ring_lazy[i] = false;
        g->ring_done[i] = g->ring_free[i];
    }
    return RH_OK;
}

// ---- delta staging (callers hold smu exclusively and mu) ----
// Submits the deltas staged in the open slot (H2D + apply, ordered after every call before this).
int stage_submit(rh_groups* g) {
    if (g->open < 0) return RH_OK;
    const int i = g->open;
    const uint64_t n = std::min<uint64_t>(g->fill.load(std::memory_order_relaxed), RH_DELTA_SLOT);
    g->open = -1;
    g->fill.store(0, std::memory_order_relaxed);
    const bool has_set = g->staged_set.exchange(false, std::memory_order_relaxed);
    if (n == 0) return RH_OK;
    return ring_submit(g, i, n, has_set);
}

// The exclusive side of the staging: both locks, staged deltas submitted first.
struct Exclusive {
    std::unique_lock<std::shared_mutex> x;
    std::unique_lock<std::mutex> m;
    explicit Exclusive(rh_groups* g) : x(g->smu), m(g->mu) {}
    void unlock() {
        m.unlock();
        x.unlock();
    }
    void lock() {
        x.lock();
        m.lock();
    }
};

// Waits for `ev` with both locks released (producers and readers go on meanwhile), then takes them
// again.
int wait_unlocked(Exclusive& ex, hipEvent_t ev) {
    ex.unlock();
    const hipError_t e = hipEventSynchronize(ev);
    ex.lock();
    return e == hipSuccess ? RH_OK : rh::hip_fail(e, "hipEventSynchronize");
}

int check_conf(uint32_t conf, const char* who) {
    if (needed_width(conf) > RH_MAX_FOLLOWERS) return rh::fail(RH_E_RANGE, std::string(who) + ": conf names a slot > 13");
    return RH_OK;
}

}  // namespace

// ---- lifecycle -------------------------------------------------------------------------------------
RH_EXPORT int rh_groups_create(rh_ctx* ctx, uint64_t capacity, int64_t gap_threshold, rh_groups** out) {
    if (!ctx || !out) return rh::fail(RH_E_INVAL, "rh_groups_create: ctx/out == NULL");
    *out = nullptr;
    if (capacity == 0 || capacity >= (1ull << 28)) return rh::fail(RH_E_RANGE, "rh_groups_create: capacity must be in [1, 2^28)");
    if (gap_threshold < -1) return rh::fail(RH_E_INVAL, "rh_groups_create: gap_threshold must be -1 or >= 0");
    DeviceGuard dg(ctx->device);
    rh_groups* g = new (std::nothrow) rh_groups();
    if (!g) return rh::fail(RH_E_NOMEM, "rh_groups_create: out of host memory");
    g->ctx = ctx;
    g->capacity = capacity;
    g->gap = gap_threshold;
    g->dev.capacity = capacity;
    g->dev.gap = gap_threshold;
    for (int t = 0; t < kTableTiers; ++t) g->dev.tier[t].width = rh::width_of_tier(t);
    int rc = RH_OK;
    try {
        g->slot_map.assign(capacity, kNoRow);
        g->slot_conf.assign(capacity, 0);
        g->op_stamp.assign(capacity, 0);
    } catch (...) {
        rc = rh::fail(RH_E_NOMEM, "rh_groups_create: out of host memory");
    }
    hipStream_t s = ctx->stream;
    if (rc == RH_OK) rc = dalloc(&g->dev.slot_map, capacity);
    if (rc == RH_OK && hipMemsetAsync(g->dev.slot_map, 0xFF, capacity * 4, s) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: init");
    if (rc == RH_OK && hipStreamCreateWithFlags(&g->d2h_stream, hipStreamNonBlocking) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: result copy stream");
    if (rc == RH_OK && hipEventCreateWithFlags(&g->evaluated, hipEventDisableTiming) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: evaluation event");
    if (rc == RH_OK && hipEventCreateWithFlags(&g->gathered, hipEventDisableTiming) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: gather event");
    if (rc == RH_OK && hipEventCreateWithFlags(&g->wgathered, hipEventDisableTiming) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: gather event");
    if (rc == RH_OK && hipStreamCreateWithFlags(&g->copy_stream, hipStreamNonBlocking) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: copy stream");
    for (int i = 0; i < 2 && rc == RH_OK; ++i) {
        rc = dalloc(&g->d_ring[i], (size_t)RH_DELTA_SLOT);
        if (rc == RH_OK && hipEventCreateWithFlags(&g->ring_read[i], hipEventDisableTiming) != hipSuccess)
            rc = rh::fail(RH_E_DEVICE, "hipEventCreate(delta staging)");
        if (rc != RH_OK) break;
        if (hipHostMalloc(reinterpret_cast<void**>(&g->h_ring[i]), (size_t)RH_DELTA_SLOT * sizeof(rh_delta)) != hipSuccess)
            rc = rh::fail(RH_E_NOMEM, "hipHostMalloc(delta staging)");
        void* dv = nullptr;   // no device view: every batch goes by DMA
        if (rc == RH_OK && hipHostGetDevicePointer(&dv, g->h_ring[i], 0) == hipSuccess) g->d_hring[i] = static_cast<const rh_delta*>(dv);
        if (rc == RH_OK && hipEventCreateWithFlags(&g->ring_free[i], hipEventDisableTiming) != hipSuccess)
            rc = rh::fail(RH_E_DEVICE, "hipEventCreate(delta staging)");
    }
    for (int i = 0; i < kEvSets && rc == RH_OK; ++i) {
        if (rc == RH_OK) rc = halloc_mapped(&g->ev[i].adv, &g->ev[i].d_adv, capacity);
        if (rc == RH_OK) rc = halloc_mapped(&g->ev[i].wall, &g->ev[i].d_wall, capacity);
        if (rc == RH_OK) rc = dalloc(&g->ev[i].hbm_adv, hbm_records(capacity));
        if (rc == RH_OK) rc = dalloc(&g->ev[i].hbm_wall, hbm_records(capacity));
        if (rc == RH_OK) rc = dalloc(&g->ev[i].bdesc, rh::kTableDesc * desc_blocks(capacity));
        if (rc == RH_OK) rc = halloc_mapped(&g->ev[i].h_cnt, &g->ev[i].d_cnt, 2);
        if (rc == RH_OK && hipEventCreateWithFlags(&g->ev[i].done, hipEventDisableTiming) != hipSuccess)
            rc = rh::fail(RH_E_DEVICE, "hipEventCreate(commit batch)");
    }
    if (rc == RH_OK) rc = halloc_mapped(&g->watch, &g->d_watch, capacity);
    if (rc == RH_OK) rc = dalloc(&g->hbm_watch, hbm_records(capacity));
    if (rc == RH_OK) rc = dalloc(&g->wbdesc, rh::kTableDesc * desc_blocks(capacity));
    if (rc == RH_OK) rc = halloc_mapped(&g->h_wcnt, &g->d_wcnt, 2);
    if (rc == RH_OK && hipEventCreateWithFlags(&g->wdone, hipEventDisableTiming) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "hipEventCreate(watch levels)");
    if (rc == RH_OK && hipEventCreateWithFlags(&g->ldone, hipEventDisableTiming) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "hipEventCreate(lease batch)");
    // 24-bit counts leave 16 bits of done count in the word (every tile workgroup packed); the
    // environment can force 28 (tests: the separate done word of large tables)
    g->cbits = capacity < (1ull << 24) ? 24u : 28u;
    if (const char* e = std::getenv("RATIS_HIP_TABLE_CNT_BITS"))
        if (std::atoi(e) == 28) g->cbits = 28u;
    g->lcap = list_cap(capacity);
    for (int k = 0; k < 2 && rc == RH_OK; ++k) rc = dalloc(&g->d_lrows[k], kListRegions * g->lcap);
    if (rc == RH_OK) rc = dalloc(&g->d_lheads, (size_t)4 * kListRegions * rh::kHeadStride);
    if (rc == RH_OK && hipMemsetAsync(g->d_lheads, 0, (size_t)4 * kListRegions * rh::kHeadStride * 8, s) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: list counters");
    if (rc == RH_OK) rc = dalloc(&g->d_tick, (size_t)3 * rh::kHeadStride);
    if (rc == RH_OK && hipMemsetAsync(g->d_tick, 0, (size_t)3 * rh::kHeadStride * 8, s) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: tick counters");
    if (rc == RH_OK) rc = dalloc(&g->d_evw, (size_t)2 * rh::kHeadStride);
    if (rc == RH_OK && hipMemsetAsync(g->d_evw, 0, (size_t)2 * rh::kHeadStride * 8, s) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: counters");
    // two bitmaps, each at a 16-byte aligned stride (the copy to the host moves 16 bytes a step)
    if (rc == RH_OK) rc = dalloc(&g->d_lbits, 2 * lbits_stride(capacity));
    if (rc == RH_OK && hipMemsetAsync(g->d_lbits, 0, 2 * lbits_stride(capacity) * 8, s) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "rh_groups_create: lease bitmaps");
    if (rc == RH_OK) rc = halloc_mapped(&g->h_lbits, &g->d_hlbits, (capacity + 63) / 64);
    if (rc == RH_OK && hipEventCreateWithFlags(&g->ops_free, hipEventDisableTiming) != hipSuccess)
        rc = rh::fail(RH_E_DEVICE, "hipEventCreate(control ops)");
    if (rc == RH_OK && hipStreamSynchronize(s) != hipSuccess) rc = rh::fail(RH_E_DEVICE, "rh_groups_create: sync");
    if (rc != RH_OK) {
        free_groups(g);
        delete g;
        return rc;
    }
    *out = g;
    return RH_OK;
}

RH_EXPORT int rh_groups_destroy(rh_groups* g) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_groups_destroy: NULL");
    DeviceGuard dg(g->ctx->device);
    // a fault of the table's last work is reported here, not swallowed (the table is freed anyway)
    hipError_t e = hipStreamSynchronize(g->ctx->stream);
    if (g->copy_stream) {
        const hipError_t e1 = hipStreamSynchronize(g->copy_stream);
        if (e == hipSuccess) e = e1;
    }
    if (g->d2h_stream) {
        const hipError_t e2 = hipStreamSynchronize(g->d2h_stream);
        if (e == hipSuccess) e = e2;
    }
    free_groups(g);
    delete g;
    if (e != hipSuccess) return rh::hip_fail(e, "rh_groups_destroy: the table's last work failed");
    return RH_OK;
}

RH_EXPORT int rh_groups_set_event_sink(rh_groups* g, int sink) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_groups_set_event_sink: groups == NULL");
    if (sink != RH_EVENTS_HOST_MAPPED && sink != RH_EVENTS_DEVICE && sink != RH_EVENTS_AUTO)
        return rh::fail(RH_E_INVAL, "rh_groups_set_event_sink: unknown sink");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    for (const EvSet& e : g->ev)
        if (e.pending) return rh::fail(RH_E_STATE, "rh_groups_set_event_sink: an evaluation is in flight");
    if (g->wpending) return rh::fail(RH_E_STATE, "rh_groups_set_event_sink: a watch evaluation is in flight");
    g->event_sink = sink;
    return RH_OK;
}

RH_EXPORT int rh_groups_timing(rh_groups* g, int enable) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_groups_timing: groups == NULL");
    DeviceGuard dg(g->ctx->device);
    std::lock_guard<std::mutex> lk(g->mu);
    for (hipEvent_t& e : g->tev)
        if (!e && hipEventCreate(&e) != hipSuccess) return rh::fail(RH_E_DEVICE, "hipEventCreate(timing)");
    g->timing = enable != 0;
    g->timed = false;
    return RH_OK;
}

RH_EXPORT int rh_groups_last_timing_split(rh_groups* g, float* submit_ms, float* eval_ms, float* events_ms,
                                          float* gather_ms, int* list_evaluated) {
    if (!g || !submit_ms || !eval_ms || !events_ms || !gather_ms)
        return rh::fail(RH_E_INVAL, "rh_groups_last_timing_split: NULL argument");
    DeviceGuard dg(g->ctx->device);
    std::unique_lock<std::mutex> lk(g->mu);
    if (!g->timed) return rh::fail(RH_E_STATE, "rh_groups_last_timing_split: no timed evaluation");
    hipEvent_t ev[6] = {g->tev[0], g->tev[1], g->tev[2], g->tev[3], g->tev[4], g->tev[5]};
    const int was_list = g->last_list;
    const bool gathered = g->gathered_timed;
    lk.unlock();   // no table lock across a device wait
    RH_HIP(hipEventSynchronize(ev[3]));
    RH_HIP(hipEventSynchronize(ev[1]));
    RH_HIP(hipEventElapsedTime(submit_ms, ev[2], ev[0]));
    RH_HIP(hipEventElapsedTime(eval_ms, ev[0], ev[1]));
    RH_HIP(hipEventElapsedTime(events_ms, ev[1], ev[3]));
    if (*events_ms < 0) *events_ms = 0;   // the evaluation wrote the records itself
    *gather_ms = 0;
    if (gathered) {
        RH_HIP(hipEventSynchronize(ev[5]));
        RH_HIP(hipEventElapsedTime(gather_ms, ev[4], ev[5]));
    }
    if (list_evaluated) *list_evaluated = was_list;
    return RH_OK;
}

RH_EXPORT int rh_groups_last_timing(rh_groups* g, float* eval_ms, int* list_evaluated) {
    if (!g || !eval_ms) return rh::fail(RH_E_INVAL, "rh_groups_last_timing: NULL argument");
    DeviceGuard dg(g->ctx->device);
    std::unique_lock<std::mutex> lk(g->mu);
    if (!g->timed) return rh::fail(RH_E_STATE, "rh_groups_last_timing: no timed evaluation");
    const hipEvent_t t0 = g->tev[0], t1 = g->tev[1];
    const int was_list = g->last_list;
    lk.unlock();   // no table lock across a device wait
    RH_HIP(hipEventSynchronize(t1));
    RH_HIP(hipEventElapsedTime(eval_ms, t0, t1));
    if (list_evaluated) *list_evaluated = was_list;
    return RH_OK;
}

// ---- control ---------------------------------------------------------------------------------------
RH_EXPORT int rh_group_start(rh_groups* g, uint32_t slot, uint32_t conf, int64_t flush_index, int64_t commit_index,
                             int64_t term_start) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_group_start: groups == NULL");
    if (slot >= g->capacity) return rh::fail(RH_E_INVAL, "rh_group_start: slot out of range");
    int rc = check_conf(conf, "rh_group_start");
    if (rc != RH_OK) return rc;
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    rc = stage_submit(g);   // the deltas pushed before this call apply before it
    if (rc != RH_OK) return rc;
    rc = do_stop(g, slot);  // a re-armed slot drops its old row (and every FollowerInfo with it)
    if (rc != RH_OK) return rc;
    const int t = rh::tier_of_width(needed_width(conf));
    uint32_t row = 0;
    rc = alloc_row(g, t, &row);
    if (rc != RH_OK) return rc;
    CtrlOp op{};
    op.kind = rh::kCtrlStart;
    op.slot = slot;
    op.dst = enc(t, row);
    op.conf = conf;
    op.flush = flush_index;
    op.commit = commit_index;
    op.tstart = term_start;
    rc = queue_op(g, op);
    if (rc != RH_OK) return rc;
    g->slot_map[slot] = op.dst;
    ++g->map_gen;
    g->slot_conf[slot] = conf;
    return RH_OK;
}

RH_EXPORT int rh_group_reconf(rh_groups* g, uint32_t slot, uint32_t conf, const int8_t* src) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_group_reconf: groups == NULL");
    if (slot >= g->capacity) return rh::fail(RH_E_INVAL, "rh_group_reconf: slot out of range");
    int rc = check_conf(conf, "rh_group_reconf");
    if (rc != RH_OK) return rc;
    if (src)
        for (int k = 0; k < (int)RH_MAX_FOLLOWERS; ++k)
            if (src[k] < -1 || src[k] >= (int)RH_MAX_FOLLOWERS)
                return rh::fail(RH_E_INVAL, "rh_group_reconf: src entries must be -1 or a follower slot");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    const uint32_t m = g->slot_map[slot];
    if (m == kNoRow) return rh::fail(RH_E_STATE, "rh_group_reconf: slot not started");
    rc = stage_submit(g);   // the deltas pushed before this call apply under the old conf
    if (rc != RH_OK) return rc;
    const int t_old = (int)(m >> 28);
    const int t_new = rh::tier_of_width(needed_width(conf));
    CtrlOp op{};
    op.slot = slot;
    op.src = m;
    op.conf = conf;
    for (int k = 0; k < (int)RH_MAX_FOLLOWERS; ++k) op.map[k] = src ? src[k] : (int8_t)k;
    if (t_new == t_old) {
        op.kind = rh::kCtrlReconf;
        op.dst = m;
    } else {
        uint32_t row = 0;
        rc = alloc_row(g, t_new, &row);
        if (rc != RH_OK) return rc;
        op.kind = rh::kCtrlMove;
        op.dst = enc(t_new, row);
    }
    rc = queue_op(g, op);
    if (rc != RH_OK) return rc;
    if (op.kind == rh::kCtrlMove) g->tiers[t_old].pending_free.push_back(m & rh::kRowMask);
    g->slot_map[slot] = op.dst;
    ++g->map_gen;
    g->slot_conf[slot] = conf;
    return RH_OK;
}

RH_EXPORT int rh_group_stop(rh_groups* g, uint32_t slot) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_group_stop: groups == NULL");
    if (slot >= g->capacity) return rh::fail(RH_E_INVAL, "rh_group_stop: slot out of range");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    int rc = stage_submit(g);
    return rc != RH_OK ? rc : do_stop(g, slot);
}

RH_EXPORT int rh_group_tier(rh_groups* g, uint32_t slot, uint32_t* out_width) {
    if (!g || !out_width) return rh::fail(RH_E_INVAL, "rh_group_tier: NULL argument");
    if (slot >= g->capacity) return rh::fail(RH_E_INVAL, "rh_group_tier: slot out of range");
    std::lock_guard<std::mutex> lk(g->mu);
    const uint32_t m = g->slot_map[slot];
    *out_width = m == kNoRow ? 0u : rh::width_of_tier((int)(m >> 28));
    return RH_OK;
}

namespace {

__global__ void table_load_kernel(rh::TableDev T, int t, const uint32_t* __restrict__ rows,
                                  const uint32_t* __restrict__ slots, const int64_t* __restrict__ cols, uint32_t m) {
    // cols: [F match][F fcommit][flush][commit][tstart][conf] x m, column-major
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    namespace tl = rh::tile;
    const rh::TableTier& D = T.tier[t];
    const uint32_t r = rows[i];
    const uint32_t F = D.width;
    for (uint32_t k = 0; k < F; ++k) {
        *D.i64(tl::match(k), r) = cols[(uint64_t)k * m + i];
        *D.i64(tl::fcommit(F, k), r) = cols[(F + k) * m + i];
        *D.i64(tl::fts(F, k), r) = rh::kNoTimestamp;  // lease state as a fresh start: rh_group_lease_start
    }
    *D.i64(tl::lease(F), r) = rh::kNoTimestamp;
    *D.u8(tl::kLon, r) = 0;
    *D.i64(tl::flush(F), r) = cols[(2 * F) * m + i];
    *D.i64(tl::commit(F), r) = cols[(2 * F + 1) * m + i];
    *D.i64(tl::tstart(F), r) = cols[(2 * F + 2) * m + i];
    *D.u32(tl::kConf, r) = (uint32_t)cols[(2 * F + 3) * m + i];
    *D.i64(tl::wall(F), r) = INT64_MIN;
    *D.i64(tl::wmin(F), r) = INT64_MIN;
    *D.i64(tl::wmaj(F), r) = INT64_MIN;
    *D.i64(tl::wmax(F), r) = INT64_MIN;
    *D.u8(tl::kDirty, r) = 1;
    *D.u8(tl::kWdirty, r) = 1;
    *D.summary(r, 0) = 1;
    *D.summary(r, 1) = 1;
    *D.u32(tl::kSlot, r) = slots[i];
    T.slot_map[slots[i]] = ((uint32_t)t << 28) | r;
}

}  // namespace

RH_EXPORT int rh_groups_load(rh_groups* g, uint32_t first, uint32_t n, uint32_t n_host_followers, const int64_t* match,
                             const int64_t* fcommit, const int64_t* flush, const int64_t* commit,
                             const int64_t* term_start, const uint32_t* conf) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_groups_load: groups == NULL");
    if ((uint64_t)first + n > g->capacity) return rh::fail(RH_E_INVAL, "rh_groups_load: slots out of range");
    if (n == 0) return RH_OK;
    if (!flush || !commit || !term_start || !conf)
        return rh::fail(RH_E_INVAL, "rh_groups_load: flush, commit, term_start and conf are required");
    if (n_host_followers > RH_MAX_FOLLOWERS) return rh::fail(RH_E_RANGE, "rh_groups_load: n_host_followers > 14");
    for (uint32_t i = 0; i < n; ++i) {
        int rc = check_conf(conf[i], "rh_groups_load");
        if (rc != RH_OK) return rc;
    }
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    int rc = stage_submit(g);
    if (rc != RH_OK) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        rc = do_stop(g, first + i);
        if (rc != RH_OK) return rc;
    }
    rc = flush_ops(g);  // launches the stops; the rows they released are reusable now
    if (rc != RH_OK) return rc;
    g->lvalid[0] = g->lvalid[1] = false;   // the load marks its rows with plain stores
    hipStream_t s = g->ctx->stream;
    std::vector<std::vector<uint32_t>> members(kTableTiers);
    for (uint32_t i = 0; i < n; ++i) members[rh::tier_of_width(needed_width(conf[i]))].push_back(i);
    for (int t = 0; t < kTableTiers; ++t) {
        const std::vector<uint32_t>& mem = members[t];
        if (mem.empty()) continue;
        const uint32_t m = (uint32_t)mem.size(), F = rh::width_of_tier(t);
        std::vector<uint32_t> rows(m), slots(m);
        for (uint32_t j = 0; j < m; ++j) {
            rc = alloc_row(g, t, &rows[j]);
            if (rc != RH_OK) return rc;
            slots[j] = first + mem[j];
        }
        std::vector<int64_t> cols((size_t)(2 * F + 4) * m);
        for (uint32_t j = 0; j < m; ++j) {
            const uint32_t i = mem[j];
            for (uint32_t k = 0; k < F; ++k) {
                const bool have = k < n_host_followers;
                cols[(size_t)k * m + j] = (have && match) ? match[(size_t)k * n + i] : -1;
                cols[(size_t)(F + k) * m + j] = (have && fcommit) ? fcommit[(size_t)k * n + i] : -1;
            }
            cols[(size_t)(2 * F) * m + j] = flush[i];
            cols[(size_t)(2 * F + 1) * m + j] = commit[i];
            cols[(size_t)(2 * F + 2) * m + j] = term_start[i];
            cols[(size_t)(2 * F + 3) * m + j] = (int64_t)conf[i];
        }
        uint32_t *d_rows = nullptr, *d_slots = nullptr;
        int64_t* d_cols = nullptr;
        rc = dalloc(&d_rows, m);
        if (rc == RH_OK) rc = dalloc(&d_slots, m);
        if (rc == RH_OK) rc = dalloc(&d_cols, cols.size());
        hipError_t e = hipSuccess;
        if (rc == RH_OK) {
            // host vectors: through the context's bounce buffers (rh::h2d), never page-locked in place
            rc = rh::h2d(g->ctx, d_rows, rows.data(), (uint64_t)m * 4, s);
            if (rc == RH_OK) rc = rh::h2d(g->ctx, d_slots, slots.data(), (uint64_t)m * 4, s);
            if (rc == RH_OK) rc = rh::h2d(g->ctx, d_cols, cols.data(), cols.size() * 8, s);
            if (rc == RH_OK) e = g->gather_pending ? hipStreamWaitEvent(s, g->gathered, 0) : hipSuccess;
            if (rc == RH_OK && e == hipSuccess) e = g->wgather_pending ? hipStreamWaitEvent(s, g->wgathered, 0) : hipSuccess;
            if (rc == RH_OK && e == hipSuccess) {
                g->gather_pending = g->wgather_pending = false;
                hipLaunchKernelGGL(table_load_kernel, dim3((m + 255) / 256), dim3(256), 0, s, g->dev, t, d_rows, d_slots,
                                   d_cols, m);
                e = hipGetLastError();
            }
            const hipError_t es = hipStreamSynchronize(s);   // the bounce copies and the load (error paths too)
            if (e == hipSuccess) e = es;
        }
        (void)hipFree(d_rows);
        (void)hipFree(d_slots);
        (void)hipFree(d_cols);
        if (rc != RH_OK) return rc;
        if (e != hipSuccess) return rh::hip_fail(e, "rh_groups_load");
        ++g->map_gen;
        for (uint32_t j = 0; j < m; ++j) {
            g->slot_map[slots[j]] = enc(t, rows[j]);
            g->slot_conf[slots[j]] = conf[mem[j]];
        }
    }
    return RH_OK;
}

// ---- deltas ------------------------------------------------------------------------------------------
#ifndef RH_PUSH_NT   // A/B: producers copy into the pinned slot with streaming stores (1) or memcpy (0)
#define RH_PUSH_NT 1
#endif

// A producer's copy into the pinned staging slot.  Streaming (non-temporal) stores: the slot is
// written once here and read next by the H2D DMA, so allocating its lines in the writer's cache
// (a read for ownership per line, then a write-back) only halves the copy rate -- with 8 producers
// the cached copy saturated near 30 GB/s (scripts/push_probe.py).  The fence orders the streaming
// stores before the staging lock is released (the submitter takes it exclusively before the H2D).
static_assert(sizeof(rh_delta) == 16, "one 16-byte store per delta");
// The deltas into the staging slot with each slot field replaced by its row code (`codes`, from the
// validation against the host slot map).
static void stage_copy(rh_delta* dst, const rh_delta* src, const uint32_t* codes, size_t n) {
#if defined(__x86_64__)
    if (RH_PUSH_NT && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        __m128i* d = reinterpret_cast<__m128i*>(dst);
        const __m128i* s = reinterpret_cast<const __m128i*>(src);
        for (size_t i = 0; i < n; ++i) {
            __m128i v = _mm_loadu_si128(s + i);
            v = _mm_insert_epi16(v, (int)(codes[i] & 0xFFFFu), 0);   // slot field: bytes 0..3
            v = _mm_insert_epi16(v, (int)(codes[i] >> 16), 1);
            _mm_stream_si128(d + i, v);
        }
        _mm_sfence();
        return;
    }
#endif
    for (size_t i = 0; i < n; ++i) {
        dst[i] = src[i];
        dst[i].slot = codes[i];
    }
}

// Multi-producer: each call validates its deltas and copies them into the open pinned slot at a range
// it reserved with one CAS, holding the staging lock SHARED -- producers on other threads copy at the
// same time, and no producer waits for an evaluation, a watch or lease wait, or another producer's
// copy.  Nothing per delta is written outside the caller's reserved range (a per-slot stamp array
// written by every producer thrashed its cache lines between cores: 10 ms per 4M deltas).  The slot
// goes to the device (H2D + apply) when it is full or when an evaluation, a read, a control op or the
// zero-copy path needs the deltas before it; the device applies a batch in slot order with
// one-by-one semantics (rh_internal.h, ApplyPhase), so a call's deltas keep their array order and
// calls that do not overlap in time keep theirs.
RH_EXPORT int rh_push_deltas(rh_groups* g, const rh_delta* deltas, size_t n) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_push_deltas: groups == NULL");
    if (n == 0) return RH_OK;
    if (!deltas) return rh::fail(RH_E_INVAL, "rh_push_deltas: deltas == NULL");
    // deltas [lo, hi) against the current slot map (caller holds smu); a producer's deltas come in
    // runs per division (a reply's SET + MAXes): the slot map is read once per run
    bool any_set = false;
    size_t done = 0;
    thread_local std::vector<uint32_t> codes;   // each delta's row code, as the check found it
    struct Trim {   // a thread keeps at most 1 MiB of codes between calls (one large push frees its own)
        std::vector<uint32_t>& v;
        ~Trim() {
            if (v.capacity() > (1u << 18)) std::vector<uint32_t>().swap(v);
        }
    } trim{codes};
    if (codes.size() < n) codes.resize(n);
    auto validate = [&](size_t lo, size_t hi) -> int {
        uint32_t last = kNoRow, m = kNoRow, w = 0;
        constexpr size_t kAhead = 16;   // the slot map's lines requested ahead (random slots: ~L3 latency each)
        for (size_t i = lo; i < std::min(hi, lo + kAhead); ++i)
            if (deltas[i].slot < g->capacity) __builtin_prefetch(&g->slot_map[deltas[i].slot]);
        for (size_t i = lo; i < hi; ++i) {
            if (i + kAhead < hi && deltas[i + kAhead].slot < g->capacity)
                __builtin_prefetch(&g->slot_map[deltas[i + kAhead].slot]);
            const rh_delta& d = deltas[i];
            if (d.slot != last || i == lo) {
                last = d.slot;
                m = d.slot < g->capacity ? g->slot_map[d.slot] : kNoRow;
                w = m == kNoRow ? 0u : rh::width_of_tier((int)(m >> 28));
            }
            const uint32_t c = d.column;
            const bool ok_col = c < w || (c >= 16 && c < 16 + w) || c == RH_COL_FLUSH || c == RH_COL_COMMITTED ||
                                (c >= 48 && c < 48 + w) || c == RH_COL_LEASE || c == RH_COL_LEASE_ON;
            if (m == kNoRow || !ok_col || d.op > RH_OP_SET)
                return rh::fail(RH_E_INVAL, "rh_push_deltas: delta " + std::to_string(i) +
                                                " names a stopped slot, a column outside its tier or an unknown op" +
                                                (done ? " (deltas [0, " + std::to_string(done) + ") were staged)" : ""));
            any_set |= d.op == RH_OP_SET;
            codes[i] = m;
        }
        return RH_OK;
    };
    // The whole call is checked first: a rejected call stages nothing.  A call longer than the open
    // slot's room is staged chunk by chunk, and between two chunks the exclusive side below runs
    // (and so may a control call): if the slot map changed meanwhile (map_gen), the deltas not staged
    // yet are checked again against the map they will be applied with.
    bool validated = false;
    uint64_t gen = 0;   // the slot map the remaining deltas were checked against
    while (done < n) {
        {
            std::shared_lock<std::shared_mutex> sl(g->smu);   // the slot map changes only under exclusive
            if (g->ring_acquired >= 0) return rh::fail(RH_E_STATE, "rh_push_deltas: a staging slot is acquired");
            if (!validated || gen != g->map_gen) {   // first, or a control call changed the map meanwhile
                const int rc = validate(done, n);   // everything not staged yet, against this map
                if (rc != RH_OK) return rc;
                validated = true;
                gen = g->map_gen;
            }
            if (g->open >= 0) {
                uint64_t r = g->fill.load(std::memory_order_relaxed), take = 0;
                do {
                    if (r >= RH_DELTA_SLOT) {
                        take = 0;
                        break;
                    }
                    take = std::min<uint64_t>(n - done, RH_DELTA_SLOT - r);
                } while (!g->fill.compare_exchange_weak(r, r + take, std::memory_order_relaxed));
                if (take) {
                    if (any_set) g->staged_set.store(true, std::memory_order_relaxed);
                    stage_copy(g->h_ring[g->open] + r, deltas + done, codes.data() + done, take);
                    done += take;
                    continue;
                }
            }
        }
        // no open slot, or it is full: submit it and open the next one -- waiting for the next slot's
        // previous H2D / in-place apply with both locks released (no producer blocks the
        // others, nor the _async / _wait callers, on device work)
        DeviceGuard dg(g->ctx->device);
        Exclusive ex(g);
        if (g->ring_acquired >= 0) return rh::fail(RH_E_STATE, "rh_push_deltas: a staging slot is acquired");
        if (g->open < 0 || g->fill.load(std::memory_order_relaxed) >= RH_DELTA_SLOT) {
            int rc = stage_submit(g);
            if (rc != RH_OK) return rc;
            const int i = g->ring_next;
            hipEvent_t fe = nullptr;
            rc = slot_event(g, i, &fe);
            if (rc != RH_OK) return rc;
            if (fe) {
                const hipError_t q = hipEventQuery(fe);
                if (q == hipErrorNotReady) {
                    (void)hipGetLastError();
                    rc = wait_unlocked(ex, fe);
                    if (rc != RH_OK) return rc;
                    continue;   // re-checked from the top (another producer may have opened a slot)
                }
                if (q != hipSuccess) return rh::hip_fail(q, "rh_push_deltas: staging slot");   // a device fault
            }
            g->open = i;
            g->ring_resolved[i] = true;   // pushes store row codes
            g->fill.store(0, std::memory_order_relaxed);
        }
    }
    return RH_OK;
}

RH_EXPORT int rh_deltas_acquire(rh_groups* g, rh_delta** out_buf, size_t* out_cap) {
    if (!g || !out_buf || !out_cap) return rh::fail(RH_E_INVAL, "rh_deltas_acquire: NULL argument");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    if (g->ring_acquired >= 0) return rh::fail(RH_E_STATE, "rh_deltas_acquire: a slot is already acquired");
    int rc = stage_submit(g);   // the pushed deltas precede the acquired slot's
    if (rc != RH_OK) return rc;
    const int i = g->ring_next;
    rc = ring_wait(g, i);
    if (rc != RH_OK) return rc;
    g->ring_acquired = i;
    g->ring_resolved[i] = false;   // producers write slots, not row codes
    *out_buf = g->h_ring[i];
    *out_cap = RH_DELTA_SLOT;
    return RH_OK;
}

RH_EXPORT int rh_deltas_submit(rh_groups* g, size_t n) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_deltas_submit: groups == NULL");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    const int i = g->ring_acquired;
    if (i < 0) return rh::fail(RH_E_STATE, "rh_deltas_submit: no slot acquired");
    if (n > RH_DELTA_SLOT) return rh::fail(RH_E_INVAL, "rh_deltas_submit: n exceeds the slot capacity");
    g->ring_acquired = -1;
    if (n == 0) return RH_OK;
    return ring_submit(g, i, n, true);
}

// ---- evaluation -------------------------------------------------------------------------------------
// No table lock is held across a device wait: a wait for an earlier evaluation (its result buffers
// are about to be rewritten) and the _wait calls release both locks first, then re-validate.
namespace {
// The staged deltas go first, every evaluation of this call after them.
int submit_staged(rh_groups* g) {
    if (g->timing) RH_HIP(hipEventRecord(g->tev[2], g->ctx->stream));
    g->gathered_timed = false;
    return stage_submit(g);   // the deltas pushed before this call
}

// Frees result set `e` (ticket `tk`) for a new evaluation: an unread earlier result set is waited for
// before its buffers are rewritten (both locks released while waiting).
int claim_set(rh_groups* g, Exclusive& ex, EvSet& e) {
    while (e.pending) {
        const uint64_t was = e.ticket;
        int rc = wait_unlocked(ex, e.done);
        if (rc != RH_OK) return rc;
        if (e.pending && e.ticket == was) e.pending = false;
    }
    e.ticket = 0;
    return RH_OK;
}

// The event the outstanding commitIndexChanged list completes with.
hipEvent_t watch_done(rh_groups* g) { return g->wtick ? g->ev[g->wtick % kEvSets].done : g->wdone; }

// The same for the commitIndexChanged list.
int claim_watch(rh_groups* g, Exclusive& ex) {
    while (g->wpending) {   // the previous list is about to be rewritten: wait for it, unlocked
        const uint64_t was = g->wgen;
        int rc = wait_unlocked(ex, watch_done(g));
        if (rc != RH_OK) return rc;
        if (g->wpending && g->wgen == was) g->wpending = false;
    }
    return RH_OK;
}

// updateCommit of the dirty rows into result set e under ticket tk (locks held, set claimed, staged
// deltas submitted).
int commit_issue(rh_groups* g, uint32_t flags, uint64_t tk, EvSet& e) {
    const bool wall_on = (flags & RH_COMMIT_WATCH_ALL) != 0;
    EvTargets t;
    t.adv[0] = e.d_adv, t.adv[1] = e.hbm_adv;
    t.wall[0] = e.d_wall, t.wall[1] = e.hbm_wall;
    bool hbm = false;
    rh::TableDev ed;
    rh::ListRegion lr;
    int rc = evaluate(g, RH_MODE_COMMIT, wall_on, t, e.d_cnt, e.h_cnt, &hbm, e.bdesc, &e.nblocks, &ed, &lr);
    if (rc != RH_OK) return rc;
    if (hbm && e.nblocks) {   // REGION mode (DEVICE and AUTO): the records rebuilt into the pinned lists
        hipStream_t gs = RH_GATHER_SIDE ? g->d2h_stream : g->ctx->stream;
        if (RH_GATHER_SIDE) {
            RH_HIP(hipEventRecord(g->evaluated, g->ctx->stream));
            RH_HIP(hipStreamWaitEvent(gs, g->evaluated, 0));
        }
        rc = rh_table_gather_commit(ed, e.bdesc, e.nblocks, e.d_adv, wall_on ? e.d_wall : nullptr, e.d_cnt, gs, lr,
                                    g->timing ? g->tev[4] : nullptr, g->timing ? g->tev[5] : nullptr);
        g->gathered_timed = g->timing;
        if (rc != RH_OK) return rc;
        RH_HIP(hipEventRecord(e.done, gs));
        if (RH_GATHER_SIDE) {
            RH_HIP(hipEventRecord(g->gathered, gs));
            g->gather_pending = true;
        }
        if (g->timing) RH_HIP(hipEventRecord(g->tev[3], gs));
        hbm = false;   // nothing left for _wait to copy
    } else if (hbm && g->event_sink == RH_EVENTS_AUTO) {   // contiguous HBM lists: drained on the side stream
        RH_HIP(hipEventRecord(g->evaluated, g->ctx->stream));
        RH_HIP(hipStreamWaitEvent(g->d2h_stream, g->evaluated, 0));
        rc = rh_table_drain(e.d_cnt, e.hbm_adv, e.d_adv, wall_on ? e.hbm_wall : nullptr, e.d_wall, 16, g->capacity,
                            g->d2h_stream);
        if (rc != RH_OK) return rc;
        RH_HIP(hipEventRecord(e.done, g->d2h_stream));
        if (g->timing) RH_HIP(hipEventRecord(g->tev[3], g->d2h_stream));
        hbm = false;   // nothing left for _wait to copy
    } else {
        RH_HIP(hipEventRecord(e.done, g->ctx->stream));
        if (g->timing) RH_HIP(hipEventRecord(g->tev[3], g->ctx->stream));   // (DEVICE sink: _wait's copy not included)
    }
    slots_freed_by(g, e.done);
    e.ticket = tk;
    e.hbm = hbm;
    e.pending = true;
    return RH_OK;
}
}  // namespace

RH_EXPORT int rh_commit_batch_async(rh_groups* g, uint32_t flags, uint64_t* ticket) {
    if (!g || !ticket) return rh::fail(RH_E_INVAL, "rh_commit_batch_async: NULL argument");
    if (flags & ~RH_COMMIT_WATCH_ALL) return rh::fail(RH_E_INVAL, "rh_commit_batch_async: unknown flags");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    const uint64_t tk = g->next_ticket++;
    EvSet& e = g->ev[tk % kEvSets];
    int rc = claim_set(g, ex, e);
    if (rc == RH_OK) rc = submit_staged(g);
    if (rc == RH_OK) rc = commit_issue(g, flags, tk, e);
    if (rc != RH_OK) return rc;
    *ticket = tk;
    return RH_OK;
}

RH_EXPORT int rh_commit_batch_wait(rh_groups* g, uint64_t ticket, rh_commit_out* out) {
    if (!g || !out) return rh::fail(RH_E_INVAL, "rh_commit_batch_wait: NULL argument");
    DeviceGuard dg(g->ctx->device);
    EvSet* e;
    hipEvent_t done;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        e = &g->ev[ticket % kEvSets];
        if (e->ticket != ticket || ticket == 0) return rh::fail(RH_E_STATE, "rh_commit_batch_wait: ticket unknown or superseded");
        done = e->done;
    }
    RH_HIP(hipEventSynchronize(done));
    std::unique_lock<std::mutex> lk(g->mu);
    if (e->ticket != ticket) return rh::fail(RH_E_STATE, "rh_commit_batch_wait: ticket superseded while waiting");
    if (g->wpending && g->wtick == ticket) g->wseen = true;   // a fused tick's watch list is complete too
    uint64_t na = std::min<uint64_t>(e->h_cnt[0], g->capacity);
    uint64_t nw = std::min<uint64_t>(e->h_cnt[1], g->capacity);
    if (e->hbm) {  // lists in HBM (DEVICE sink): into the pinned result buffers
        e->hbm = false;
        hipStream_t s = g->d2h_stream;
        // contiguous lists (counter mode into HBM; REGION mode was gathered at _async): the counted prefixes
        if (na) RH_HIP(hipMemcpyAsync(e->adv, e->hbm_adv, na * sizeof(rh_index_event), hipMemcpyDeviceToHost, s));
        if (nw) RH_HIP(hipMemcpyAsync(e->wall, e->hbm_wall, nw * sizeof(rh_index_event), hipMemcpyDeviceToHost, s));
        RH_HIP(hipEventRecord(e->done, s));
        done = e->done;
        lk.unlock();   // the set stays this ticket's (pending) while the copy runs
        RH_HIP(hipEventSynchronize(done));
        lk.lock();
        if (e->ticket != ticket) return rh::fail(RH_E_STATE, "rh_commit_batch_wait: ticket superseded while waiting");
        na = std::min<uint64_t>(e->h_cnt[0], g->capacity);
        nw = std::min<uint64_t>(e->h_cnt[1], g->capacity);
    }
    e->pending = false;
    out->advanced = e->adv;
    out->n_advanced = na;
    out->watch_all = e->wall;
    out->n_watch_all = nw;
    return RH_OK;
}

RH_EXPORT int rh_commit_batch(rh_groups* g, uint32_t flags, rh_commit_out* out) {
    if (!g || !out) return rh::fail(RH_E_INVAL, "rh_commit_batch: NULL argument");
    uint64_t tk = 0;
    int rc = rh_commit_batch_async(g, flags, &tk);
    return rc != RH_OK ? rc : rh_commit_batch_wait(g, tk, out);
}

namespace {
// commitIndexChanged of the watch-dirty rows into the watch list (locks held, list claimed, staged
// deltas submitted).
int watch_issue(rh_groups* g) {
    EvTargets t;
    t.watch[0] = g->d_watch, t.watch[1] = g->hbm_watch;
    bool hbm = false;
    rh::TableDev ed;
    rh::ListRegion lr;
    int rc = evaluate(g, RH_MODE_WATCH, false, t, g->d_wcnt, g->h_wcnt, &hbm, g->wbdesc, &g->wnblocks, &ed, &lr);
    if (rc != RH_OK) return rc;
    if (hbm && g->wnblocks) {   // REGION mode (DEVICE and AUTO): the records rebuilt into the pinned list
        hipStream_t gs = RH_GATHER_SIDE ? g->d2h_stream : g->ctx->stream;
        if (RH_GATHER_SIDE) {
            RH_HIP(hipEventRecord(g->evaluated, g->ctx->stream));
            RH_HIP(hipStreamWaitEvent(gs, g->evaluated, 0));
        }
        rc = rh_table_gather_watch(ed, g->wbdesc, g->wnblocks, g->d_watch, g->d_wcnt, gs, lr,
                                   g->timing ? g->tev[4] : nullptr, g->timing ? g->tev[5] : nullptr);
        g->gathered_timed = g->timing;
        if (rc != RH_OK) return rc;
        RH_HIP(hipEventRecord(g->wdone, gs));
        if (RH_GATHER_SIDE) {
            RH_HIP(hipEventRecord(g->wgathered, gs));
            g->wgather_pending = true;
            g->wgather_list = lr.rows != nullptr;
        }
        if (g->timing) RH_HIP(hipEventRecord(g->tev[3], gs));
        hbm = false;
    } else if (hbm && g->event_sink == RH_EVENTS_AUTO) {   // contiguous HBM list: drained on the side stream
        RH_HIP(hipEventRecord(g->evaluated, g->ctx->stream));
        RH_HIP(hipStreamWaitEvent(g->d2h_stream, g->evaluated, 0));
        rc = rh_table_drain(g->d_wcnt, g->hbm_watch, g->d_watch, nullptr, nullptr, 32, g->capacity, g->d2h_stream);
        if (rc != RH_OK) return rc;
        RH_HIP(hipEventRecord(g->wdone, g->d2h_stream));
        if (g->timing) RH_HIP(hipEventRecord(g->tev[3], g->d2h_stream));
        hbm = false;
    } else {
        RH_HIP(hipEventRecord(g->wdone, g->ctx->stream));
        if (g->timing) RH_HIP(hipEventRecord(g->tev[3], g->ctx->stream));
    }
    slots_freed_by(g, g->wdone);
    g->whbm = hbm;
    g->wtick = 0;
    g->wseen = false;
    ++g->wgen;
    g->wpending = true;
    return RH_OK;
}

#ifndef RH_TICK_FUSE   // rh_tick_async: both evaluations in one launch when both kinds run over their lists
#define RH_TICK_FUSE 1
#endif

// Both evaluations of a tick in one launch (table_tick_kernel): every row marked for updateCommit
// since its last evaluation and every row marked for commitIndexChanged since its last evaluation is
// listed, and the records go to the pinned lists (not the DEVICE sink).  Locks held, result set e and
// the watch list claimed, staged deltas submitted.
int tick_issue(rh_groups* g, uint32_t flags, uint64_t tk, EvSet& e) {
    hipStream_t s = g->ctx->stream;
    int rc = flush_ops(g);   // control ops before: they drop the lists (-> the two launches)
    if (rc == RH_OK) rc = gather_fence(g);
    if (rc == RH_OK) rc = wgather_fence(g);
    if (rc != RH_OK) return rc;
    if (!(RH_TICK_FUSE && g->event_sink != RH_EVENTS_DEVICE && g->lvalid[0] && g->lvalid[1] &&
          rh::table_commit_blocks(g->dev) > 0)) {   // the two evaluations one after the other
        rc = commit_issue(g, flags, tk, e);
        return rc != RH_OK ? rc : watch_issue(g);
    }
    rh::TableLists lc, lw;
    lc.rows = g->d_lrows[0], lc.heads = lheads_of(g, 0, g->lpar[0]), lc.cap = g->lcap;
    lw.rows = g->d_lrows[1], lw.heads = lheads_of(g, 1, g->lpar[1]), lw.cap = g->lcap;
    rh::TickEvents ev;
    ev.adv = e.d_adv;
    ev.wall = (flags & RH_COMMIT_WATCH_ALL) ? e.d_wall : nullptr;
    ev.watch = g->d_watch;
    ev.cap = g->capacity;
    ev.cnt = g->d_tick;
    ev.counts_c = e.d_cnt;
    ev.counts_w = g->d_wcnt;
    ev.lheads_next_c = lheads_of(g, 0, g->lpar[0] ^ 1);
    ev.lheads_next_w = lheads_of(g, 1, g->lpar[1] ^ 1);
    rc = rh_table_tick_lists(g->dev, lc, lw, ev, s, g->timing ? g->tev[0] : nullptr, g->timing ? g->tev[1] : nullptr,
                             std::max(g->lmarks[0], g->lmarks[1]));
    if (rc != RH_OK) {
        const std::string msg = rh_last_error();
        (void)reset_heads(g);
        return rh::fail(rc, msg);
    }
    if (g->timing) {
        g->timed = true;
        RH_HIP(hipEventRecord(g->tev[3], s));
    }
    RH_HIP(hipEventRecord(e.done, s));   // both lists complete with it (watch_done)
    slots_freed_by(g, e.done);
    for (int m = 0; m < 2; ++m) {   // both kinds' lists consumed; the next marks go to the fresh sets
        g->lpar[m] ^= 1;
        g->lmarks[m] = 0;
        g->marks[m] = 0;
        g->lvalid[m] = true;
    }
    g->last_list = 2;
    e.nblocks = 0;
    e.ticket = tk;
    e.hbm = false;
    e.pending = true;
    g->wnblocks = 0;
    g->whbm = false;
    g->wtick = tk;
    g->wseen = false;
    ++g->wgen;
    g->wpending = true;
    return RH_OK;
}
}  // namespace

RH_EXPORT int rh_watch_levels_async(rh_groups* g) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_watch_levels_async: groups == NULL");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    int rc = claim_watch(g, ex);
    if (rc == RH_OK) rc = submit_staged(g);
    return rc != RH_OK ? rc : watch_issue(g);
}

RH_EXPORT int rh_tick_async(rh_groups* g, uint32_t flags, uint64_t* ticket) {
    if (!g || !ticket) return rh::fail(RH_E_INVAL, "rh_tick_async: NULL argument");
    if (flags & ~RH_COMMIT_WATCH_ALL) return rh::fail(RH_E_INVAL, "rh_tick_async: unknown flags");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    const uint64_t tk = g->next_ticket++;
    EvSet& e = g->ev[tk % kEvSets];
    int rc = claim_set(g, ex, e);
    if (rc == RH_OK) rc = claim_watch(g, ex);
    if (rc == RH_OK && e.pending) rc = rh::fail(RH_E_STATE, "rh_tick_async: result set taken while waiting");
    if (rc == RH_OK) rc = submit_staged(g);
    if (rc == RH_OK) rc = tick_issue(g, flags, tk, e);
    if (rc != RH_OK) return rc;
    *ticket = tk;
    return RH_OK;
}

RH_EXPORT int rh_watch_levels_wait(rh_groups* g, const rh_watch_event** out_events, uint64_t* out_n) {
    if (!g || !out_events || !out_n) return rh::fail(RH_E_INVAL, "rh_watch_levels_wait: NULL argument");
    DeviceGuard dg(g->ctx->device);
    std::unique_lock<std::mutex> lk(g->mu);
    if (!g->wpending) return rh::fail(RH_E_STATE, "rh_watch_levels_wait: no watch evaluation in flight");
    const uint64_t gen = g->wgen;
    if (!g->wseen) {   // (a fused tick's commit wait may have seen it complete already)
        hipEvent_t done = watch_done(g);
        lk.unlock();   // no table lock across a device wait
        RH_HIP(hipEventSynchronize(done));
        lk.lock();
        if (!g->wpending || g->wgen != gen) return rh::fail(RH_E_STATE, "rh_watch_levels_wait: superseded while waiting");
    }
    uint64_t n = std::min<uint64_t>(g->h_wcnt[0], g->capacity);
    if (g->whbm && n) {   // DEVICE sink, contiguous HBM list (REGION mode was gathered at _async)
        g->whbm = false;
        RH_HIP(hipMemcpyAsync(g->watch, g->hbm_watch, n * sizeof(rh_watch_event), hipMemcpyDeviceToHost, g->d2h_stream));
        RH_HIP(hipEventRecord(g->wdone, g->d2h_stream));
        hipEvent_t done = g->wdone;
        lk.unlock();
        RH_HIP(hipEventSynchronize(done));
        lk.lock();
        if (!g->wpending || g->wgen != gen) return rh::fail(RH_E_STATE, "rh_watch_levels_wait: superseded while waiting");
        n = std::min<uint64_t>(g->h_wcnt[0], g->capacity);
    }
    g->wpending = false;
    *out_events = g->watch;
    *out_n = n;
    return RH_OK;
}

RH_EXPORT int rh_watch_levels(rh_groups* g, const rh_watch_event** out_events, uint64_t* out_n) {
    if (!g || !out_events || !out_n) return rh::fail(RH_E_INVAL, "rh_watch_levels: NULL argument");
    int rc = rh_watch_levels_async(g);
    return rc != RH_OK ? rc : rh_watch_levels_wait(g, out_events, out_n);
}

RH_EXPORT int rh_groups_read(rh_groups* g, uint32_t first, uint32_t n, uint8_t column, int64_t* out) {
    if (!g || (!out && n)) return rh::fail(RH_E_INVAL, "rh_groups_read: NULL argument");
    if ((uint64_t)first + n > g->capacity) return rh::fail(RH_E_INVAL, "rh_groups_read: slots out of range");
    const uint32_t c = column;
    if (!(c < RH_MAX_FOLLOWERS || (c >= 16 && c < 16 + RH_MAX_FOLLOWERS) || c == RH_COL_FLUSH || c == RH_COL_COMMITTED ||
          c == RH_COL_CONF || c == RH_COL_TERM_START || c == RH_COL_LEASE || c == RH_COL_LEASE_ON ||
          (c >= 48 && c < 48 + RH_MAX_FOLLOWERS)))
        return rh::fail(RH_E_INVAL, "rh_groups_read: unknown column");
    if (n == 0) return RH_OK;
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    hipStream_t s = g->ctx->stream;
    int rc = stage_submit(g);   // the deltas pushed before this call
    if (rc == RH_OK) rc = flush_ops(g);
    if (rc != RH_OK) return rc;
    if (g->read_cap < n) {
        (void)hipFree(g->d_read);
        g->read_cap = 0;
        rc = dalloc(&g->d_read, n);
        if (rc != RH_OK) return rc;
        g->read_cap = n;
    }
    rc = rh_table_read(g->dev, first, n, column, g->d_read, s);
    if (rc != RH_OK) return rc;
    // the read-back buffer is the table's: keep the lock (a read is a diagnostic, not the hot path);
    // the caller's array through the context's bounce buffers (rh::d2h waits for the stream)
    return rh::d2h(g->ctx, out, g->d_read, (uint64_t)n * 8, s);
}

// ---- leader lease ------------------------------------------------------------------------------------
RH_EXPORT int rh_group_lease_start(rh_groups* g, uint32_t slot, int64_t now_nanos, int enabled) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_group_lease_start: groups == NULL");
    if (slot >= g->capacity) return rh::fail(RH_E_INVAL, "rh_group_lease_start: slot out of range");
    uint32_t width = 0;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        const uint32_t m = g->slot_map[slot];
        if (m == kNoRow) return rh::fail(RH_E_INVAL, "rh_group_lease_start: slot is stopped");
        width = rh::width_of_tier((int)(m >> 28));
    }
    // LeaderLease(properties): lease = currentTime(), enabled per config (LL:37-38); every
    // FollowerInfoImpl: lastRespondedAppendEntriesSendTime = lastRpcTime (FII:58) -- as SET deltas,
    // ordered after the calls before this one
    rh_delta d[RH_MAX_FOLLOWERS + 2];
    size_t n = 0;
    for (uint32_t k = 0; k < width; ++k) d[n++] = rh_delta{slot, RH_COL_TS(k), RH_OP_SET, 0, now_nanos};
    d[n++] = rh_delta{slot, RH_COL_LEASE, RH_OP_SET, 0, now_nanos};
    d[n++] = rh_delta{slot, RH_COL_LEASE_ON, RH_OP_SET, 0, enabled ? 1 : 0};
    return rh_push_deltas(g, d, n);
}

RH_EXPORT int rh_lease_batch_async(rh_groups* g, int64_t now_nanos, int64_t timeout_ms) {
    if (!g) return rh::fail(RH_E_INVAL, "rh_lease_batch_async: groups == NULL");
    if (timeout_ms < 0) return rh::fail(RH_E_INVAL, "rh_lease_batch_async: timeout_ms < 0");
    DeviceGuard dg(g->ctx->device);
    Exclusive ex(g);
    while (g->lpending) {   // the pinned bitmap is about to be rewritten: wait for it, unlocked
        const uint64_t was = g->lgen;
        int rc = wait_unlocked(ex, g->ldone);
        if (rc != RH_OK) return rc;
        if (g->lpending && g->lgen == was) g->lpending = false;
    }
    hipStream_t s = g->ctx->stream;
    int rc = stage_submit(g);
    if (rc == RH_OK) rc = flush_ops(g);
    if (rc != RH_OK) return rc;
    const uint64_t words = (g->capacity + 63) / 64;
    // this pass sets bitmap lbuf (zeroed by the previous pass, or at creation) and zeroes the other
    uint64_t* bits = g->d_lbits + (size_t)g->lbuf * lbits_stride(g->capacity);
    uint64_t* other = g->d_lbits + (size_t)(g->lbuf ^ 1) * lbits_stride(g->capacity);
    rc = rh_table_lease(clipped(g, nullptr), now_nanos, timeout_ms, bits, other, (uint32_t)words, s);   // rows below the high-water marks
    if (rc != RH_OK) {   // a launch failed: the bitmaps' state is unknown
        (void)hipStreamSynchronize(s);
        (void)hipMemsetAsync(g->d_lbits, 0, 2 * lbits_stride(g->capacity) * 8, s);
        return rc;
    }
    g->lbuf ^= 1;
    // the bitmap to the host by GPU writes into the mapped pinned copy (no DMA setup on the path)
    rc = rh_table_copy_words(bits, g->d_hlbits, words, s);
    if (rc != RH_OK) return rc;
    RH_HIP(hipEventRecord(g->ldone, s));
    ++g->lgen;
    g->lpending = true;
    return RH_OK;
}

RH_EXPORT int rh_lease_batch_wait(rh_groups* g, const uint64_t** out_bits, uint64_t* out_words) {
    if (!g || !out_bits || !out_words) return rh::fail(RH_E_INVAL, "rh_lease_batch_wait: NULL argument");
    DeviceGuard dg(g->ctx->device);
    std::unique_lock<std::mutex> lk(g->mu);
    if (!g->lpending) return rh::fail(RH_E_STATE, "rh_lease_batch_wait: no lease batch in flight");
    const uint64_t gen = g->lgen;
    const hipEvent_t done = g->ldone;
    lk.unlock();   // no table lock across a device wait
    RH_HIP(hipEventSynchronize(done));
    lk.lock();
    if (!g->lpending || g->lgen != gen) return rh::fail(RH_E_STATE, "rh_lease_batch_wait: superseded while waiting");
    g->lpending = false;
    *out_bits = g->h_lbits;
    *out_words = (g->capacity + 63) / 64;
    return RH_OK;
}

RH_EXPORT int rh_lease_batch(rh_groups* g, int64_t now_nanos, int64_t timeout_ms, const uint64_t** out_bits,
                             uint64_t* out_words) {
    if (!g || !out_bits || !out_words) return rh::fail(RH_E_INVAL, "rh_lease_batch: NULL argument");
    int rc = rh_lease_batch_async(g, now_nanos, timeout_ms);
    return rc != RH_OK ? rc : rh_lease_batch_wait(g, out_bits, out_words);
}

// ---- multi-GPU node ----------------------------------------------------------------------------------
struct rh_node {
    std::vector<rh_ctx*> ctx;
    std::vector<rh_groups*> tab;
    uint64_t cap = 0;
    std::mutex batch_mu;                       // guards `tickets`
    std::vector<uint64_t> tickets;
};

RH_EXPORT int rh_shard_of(uint64_t msb, uint64_t lsb, int n_shards) {
    if (n_shards < 1) return rh::fail(RH_E_INVAL, "rh_shard_of: n_shards < 1");
    const uint64_t hilo = msb ^ lsb;  // java.util.UUID.hashCode
    const int32_t h = (int32_t)(uint32_t)(hilo >> 32) ^ (int32_t)(uint32_t)hilo;
    const int32_t r = h % n_shards;   // Math.floorMod
    return r < 0 ? r + n_shards : r;
}

RH_EXPORT int rh_node_create_devices(const int* devices, int n_shards, uint64_t capacity_per_shard,
                                     int64_t gap_threshold, rh_node** out) {
    if (!out) return rh::fail(RH_E_INVAL, "rh_node_create_devices: out == NULL");
    *out = nullptr;
    if (!devices || n_shards < 1 || n_shards > 64)
        return rh::fail(RH_E_INVAL, "rh_node_create_devices: need 1..64 devices");
    if (capacity_per_shard * (uint64_t)n_shards > 0xFFFFFFFFull)
        return rh::fail(RH_E_RANGE, "rh_node_create_devices: node slots must fit 32 bits");
    int ndev = 0;
    int rc = rh_device_count(&ndev);
    if (rc != RH_OK) return rc;
    for (int i = 0; i < n_shards; ++i)
        if (devices[i] < 0 || devices[i] >= ndev)
            return rh::fail(RH_E_INVAL, "rh_node_create_devices: no such device " + std::to_string(devices[i]));
    rh_node* nd = new (std::nothrow) rh_node();
    if (!nd) return rh::fail(RH_E_NOMEM, "rh_node_create_devices: out of host memory");
    nd->cap = capacity_per_shard;
    try {
        nd->tickets.resize((size_t)n_shards);
    } catch (...) {
        delete nd;
        return rh::fail(RH_E_NOMEM, "rh_node_create_devices: out of host memory");
    }
    for (int i = 0; i < n_shards && rc == RH_OK; ++i) {
        rh_ctx* c = nullptr;
        rc = rh_init(devices[i], &c);
        if (rc != RH_OK) break;
        nd->ctx.push_back(c);
        rh_groups* t = nullptr;
        rc = rh_groups_create(c, capacity_per_shard, gap_threshold, &t);
        if (rc == RH_OK) nd->tab.push_back(t);
    }
    if (rc != RH_OK) {
        (void)rh_node_destroy(nd);
        return rc;
    }
    *out = nd;
    return RH_OK;
}

RH_EXPORT int rh_node_create(uint32_t device_mask, uint64_t capacity_per_shard, int64_t gap_threshold, rh_node** out) {
    if (!out) return rh::fail(RH_E_INVAL, "rh_node_create: out == NULL");
    *out = nullptr;
    if (device_mask == 0) return rh::fail(RH_E_INVAL, "rh_node_create: empty device mask");
    int devs[32];
    int n = 0;
    for (int d = 0; d < 32; ++d)
        if ((device_mask >> d) & 1u) devs[n++] = d;
    return rh_node_create_devices(devs, n, capacity_per_shard, gap_threshold, out);
}

RH_EXPORT int rh_node_destroy(rh_node* nd) {
    if (!nd) return rh::fail(RH_E_INVAL, "rh_node_destroy: NULL");
    int rc = RH_OK;
    std::string msg;
    for (rh_groups* t : nd->tab) {
        const int r = rh_groups_destroy(t);
        if (r != RH_OK && rc == RH_OK) rc = r, msg = rh_last_error();   // the first shard's failure
    }
    for (rh_ctx* c : nd->ctx) {   // rh_shutdown reports a fault of the shard's last work as well
        const int r = rh_shutdown(c);
        if (r != RH_OK && rc == RH_OK) rc = r, msg = rh_last_error();
    }
    delete nd;
    return rc == RH_OK ? RH_OK : rh::fail(rc, msg);
}

RH_EXPORT int rh_node_shards(rh_node* nd) { return nd ? (int)nd->tab.size() : rh::fail(RH_E_INVAL, "rh_node_shards: NULL"); }

RH_EXPORT rh_groups* rh_node_groups(rh_node* nd, int shard) {
    return (nd && shard >= 0 && shard < (int)nd->tab.size()) ? nd->tab[shard] : nullptr;
}

RH_EXPORT rh_ctx* rh_node_ctx(rh_node* nd, int shard) {
    return (nd && shard >= 0 && shard < (int)nd->ctx.size()) ? nd->ctx[shard] : nullptr;
}

namespace {
int route(rh_node* nd, uint32_t node_slot, rh_groups** t, uint32_t* slot) {
    if (!nd) return rh::fail(RH_E_INVAL, "rh_node: NULL");
    const uint64_t sh = node_slot / nd->cap;
    if (sh >= nd->tab.size()) return rh::fail(RH_E_INVAL, "rh_node: node slot out of range");
    *t = nd->tab[sh];
    *slot = (uint32_t)(node_slot % nd->cap);
    return RH_OK;
}
}  // namespace

RH_EXPORT int rh_node_group_start(rh_node* nd, uint32_t node_slot, uint32_t conf, int64_t flush_index,
                                  int64_t commit_index, int64_t term_start) {
    rh_groups* t;
    uint32_t s;
    int rc = route(nd, node_slot, &t, &s);
    return rc != RH_OK ? rc : rh_group_start(t, s, conf, flush_index, commit_index, term_start);
}

RH_EXPORT int rh_node_group_reconf(rh_node* nd, uint32_t node_slot, uint32_t conf, const int8_t* src) {
    rh_groups* t;
    uint32_t s;
    int rc = route(nd, node_slot, &t, &s);
    return rc != RH_OK ? rc : rh_group_reconf(t, s, conf, src);
}

RH_EXPORT int rh_node_group_stop(rh_node* nd, uint32_t node_slot) {
    rh_groups* t;
    uint32_t s;
    int rc = route(nd, node_slot, &t, &s);
    return rc != RH_OK ? rc : rh_group_stop(t, s);
}

RH_EXPORT int rh_node_push_deltas(rh_node* nd, const rh_delta* deltas, size_t n) {
    if (!nd || (n && !deltas)) return rh::fail(RH_E_INVAL, "rh_node_push_deltas: NULL argument");
    const size_t S = nd->tab.size();
    const uint64_t limit = (uint64_t)nd->cap * S;   // node slots [0, cap x shards): no division per delta
    for (size_t i = 0; i < n; ++i)  // validate every delta before any shard receives one
        if (deltas[i].slot >= limit)
            return rh::fail(RH_E_INVAL, "rh_node_push_deltas: delta " + std::to_string(i) + " has a bad slot");
    if (S == 1) return rh_push_deltas(nd->tab[0], deltas, n);  // node slot == table slot
    // per-shard partitions in the calling thread's own buffers (producers share nothing here; the
    // capacity stays between calls: no allocation once warmed up)
    thread_local std::vector<std::vector<rh_delta>> part;
    try {
        if (part.size() < S) part.resize(S);
        for (size_t sh = 0; sh < S; ++sh) part[sh].clear();
        for (size_t i = 0; i < n; ++i) {
            rh_delta d = deltas[i];
            const uint64_t sh = d.slot / nd->cap;
            d.slot = (uint32_t)(d.slot % nd->cap);
            part[sh].push_back(d);
        }
    } catch (...) {
        return rh::fail(RH_E_NOMEM, "rh_node_push_deltas: out of host memory");
    }
    for (size_t sh = 0; sh < S; ++sh) {
        if (part[sh].empty()) continue;
        int rc = rh_push_deltas(nd->tab[sh], part[sh].data(), part[sh].size());
        if (rc != RH_OK) return rc;
    }
    return RH_OK;
}

RH_EXPORT int rh_node_commit_batch(rh_node* nd, uint32_t flags, rh_index_event* advanced, uint64_t adv_cap,
                                   uint64_t* n_advanced, rh_index_event* watch_all, uint64_t watch_cap,
                                   uint64_t* n_watch_all) {
    if (!nd || !n_advanced || !n_watch_all) return rh::fail(RH_E_INVAL, "rh_node_commit_batch: NULL argument");
    if ((adv_cap && !advanced) || (watch_cap && !watch_all))
        return rh::fail(RH_E_INVAL, "rh_node_commit_batch: output arrays required");
    const size_t S = nd->tab.size();
    std::lock_guard<std::mutex> lk(nd->batch_mu);
    std::vector<uint64_t>& tk = nd->tickets;
    for (size_t sh = 0; sh < S; ++sh) {  // every shard's evaluation is in flight before any wait
        int rc = rh_commit_batch_async(nd->tab[sh], flags, &tk[sh]);
        if (rc != RH_OK) return rc;
    }
    uint64_t na = 0, nw = 0;
    for (size_t sh = 0; sh < S; ++sh) {
        rh_commit_out o{};
        int rc = rh_commit_batch_wait(nd->tab[sh], tk[sh], &o);
        if (rc != RH_OK) return rc;
        const uint32_t base = (uint32_t)(sh * nd->cap);
        for (uint64_t i = 0; i < o.n_advanced; ++i, ++na)
            if (na < adv_cap) advanced[na] = rh_index_event{o.advanced[i].slot + base, 0u, o.advanced[i].value};
        for (uint64_t i = 0; i < o.n_watch_all; ++i, ++nw)
            if (nw < watch_cap) watch_all[nw] = rh_index_event{o.watch_all[i].slot + base, 0u, o.watch_all[i].value};
    }
    *n_advanced = na;
    *n_watch_all = nw;
    return RH_OK;
}

RH_EXPORT int rh_node_group_lease_start(rh_node* nd, uint32_t node_slot, int64_t now_nanos, int enabled) {
    rh_groups* t;
    uint32_t s;
    int rc = route(nd, node_slot, &t, &s);
    return rc != RH_OK ? rc : rh_group_lease_start(t, s, now_nanos, enabled);
}

RH_EXPORT int rh_node_lease_batch(rh_node* nd, int64_t now_nanos, int64_t timeout_ms, uint64_t* out_bits,
                                  uint64_t out_words) {
    if (!nd || !out_bits) return rh::fail(RH_E_INVAL, "rh_node_lease_batch: NULL argument");
    if (timeout_ms < 0) return rh::fail(RH_E_INVAL, "rh_node_lease_batch: timeout_ms < 0");
    const uint64_t total = nd->cap * nd->tab.size();
    if (out_words < (total + 63) / 64) return rh::fail(RH_E_INVAL, "rh_node_lease_batch: out_bits too small");
    std::lock_guard<std::mutex> lk(nd->batch_mu);
    for (size_t sh = 0; sh < nd->tab.size(); ++sh) {  // every shard's pass in flight before any wait
        int rc = rh_lease_batch_async(nd->tab[sh], now_nanos, timeout_ms);
        if (rc != RH_OK) return rc;
    }
    std::memset(out_bits, 0, (total + 63) / 64 * 8);
    for (size_t sh = 0; sh < nd->tab.size(); ++sh) {
        const uint64_t* bits = nullptr;
        uint64_t words = 0;
        int rc = rh_lease_batch_wait(nd->tab[sh], &bits, &words);
        if (rc != RH_OK) return rc;
        const uint64_t base = sh * nd->cap;  // node slot of the shard's slot 0
        for (uint64_t w = 0; w < words; ++w) {
            uint64_t x = bits[w];
            while (x) {
                const uint64_t s = w * 64 + (uint64_t)__builtin_ctzll(x);
                x &= x - 1;
                if (s < nd->cap) out_bits[(base + s) >> 6] |= 1ull << ((base + s) & 63);
            }
        }
    }
    return RH_OK;
}

RH_EXPORT int rh_node_watch_levels(rh_node* nd, rh_watch_event* out, uint64_t cap, uint64_t* out_n) {
    if (!nd || !out_n || (cap && !out)) return rh::fail(RH_E_INVAL, "rh_node_watch_levels: NULL argument");
    std::lock_guard<std::mutex> lk(nd->batch_mu);
    for (size_t sh = 0; sh < nd->tab.size(); ++sh) {  // every shard's evaluation in flight before any wait
        int rc = rh_watch_levels_async(nd->tab[sh]);
        if (rc != RH_OK) return rc;
    }
    uint64_t n = 0;
    for (size_t sh = 0; sh < nd->tab.size(); ++sh) {
        const rh_watch_event* ev = nullptr;
        uint64_t k = 0;
        int rc = rh_watch_levels_wait(nd->tab[sh], &ev, &k);
        if (rc != RH_OK) return rc;
        const uint32_t base = (uint32_t)(sh * nd->cap);
        for (uint64_t i = 0; i < k; ++i, ++n)
            if (n < cap) {
                out[n] = ev[i];
                out[n].slot += base;
            }
    }
    *out_n = n;
    return RH_OK;
}
