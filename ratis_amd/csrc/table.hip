// Device side of the resident group table (rh_groups, include/ratis_hip.h) for gfx950.
//
//   table_apply_kernel    FollowerInfo.updateMatchIndex / updateCommitIndex (RaftLogIndex.updateToMax,
//                         FollowerInfoImpl.java:93-105), setSnapshotIndex's setUnconditionally
//                         (FollowerInfoImpl.java:147-151), the flush-index advance
//                         (SegmentedRaftLogWorker.java:419-431) -- and the event each one submits
//                         (submitUpdateCommitEvent, LeaderStateImpl.java:846-854, 900-902): the
//                         touched row is marked dirty.
//   table_control_kernel  leader start (new FollowerInfos at -1, FollowerInfoImpl.java:42-43),
//                         conf change with follower carry-over / reset, step down.
//   table_commit_kernel   LeaderStateImpl.updateCommit() (COMMIT) or commitIndexChanged() (WATCH)
//                         over the DIRTY rows of every tier; only changed results become events,
//                         written straight into the result lists (host-mapped pinned memory or
//                         HBM) with one counter atomic per workgroup.
//   table_list_kernel     the same over the dirty-row lists (list mode: work ~ the dirty rows).
//   table_lease_kernel    LeaderStateImpl.hasLease() (LSI:1229-1249) with LeaderLease.extend (LL:67-84)
//                         for every started slot: lease_eval.h's arithmetic over the follower
//                         timestamp columns, the lease stored in place, a slot-indexed bitmap out.
//   table_read_kernel     slot-ordered read-back of one column.
//
// Rows of a tier are laid out in 128-row tiles (rh_internal.h, tile::), the TILED layout of the
// raw rh_commit_soa kernels; the per-group arithmetic is commit_eval.h's, shared with them.
// Integer compare/select work, no MFMA; HBM-bound over the dirty rows.
#include <hip/hip_ext.h>

#include "rh_internal.h"
#include "commit_eval.h"
#include "lease_eval.h"

namespace {

using rh::CtrlOp;
using rh::TableDev;
using rh::TableEvents;
using rh::TableTier;
using rh::TableLists;
namespace tile = rh::tile;

typedef int64_t v2i64 __attribute__((ext_vector_type(2)));
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool locate(const TableDev& T, uint32_t slot, const TableTier*& tt, uint32_t& row) {
    if ((uint64_t)slot >= T.capacity) return false;
    const uint32_t m = T.slot_map[slot];
    if (m == rh::kNoRow) return false;
    const uint32_t t = m >> 28;
    if (t >= (uint32_t)rh::kTableTiers) return false;
    tt = &T.tier[t];
    row = m & rh::kRowMask;
    return row < tt->rows;
}

// Marks a row dirty for updateCommit (watch = 0) or commitIndexChanged (watch = 1), with its tile's
// summary byte (plain byte stores: every writer stores 1).
__device__ __forceinline__ void mark(const TableTier& tt, uint64_t r, int watch) {
    *tt.u8(watch ? tile::kWdirty : tile::kDirty, r) = 1;
    *tt.summary(r, watch) = 1;
}

// The same with a dirty-row list maintained (list mode): the flag is set through its 32-bit word
// with an atomicOr, and the return value says whether this call made the 0 -> 1 transition (the
// caller then appends the row).  Without a list: plain stores, no transition reported.
__device__ __forceinline__ bool mark_listed(const TableTier& tt, uint64_t r, int watch, bool listed) {
    uint8_t* f = tt.u8(watch ? tile::kWdirty : tile::kDirty, r);
    *tt.summary(r, watch) = 1;
    if (!listed) {
        *f = 1;
        return false;
    }
    uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(f) & ~(uintptr_t)3);
    const uint32_t sh = 8u * (uint32_t)(reinterpret_cast<uintptr_t>(f) & 3);
    const uint32_t old = atomicOr(w, 1u << sh);
    return ((old >> sh) & 0xFFu) == 0u;
}

// Appends the rows of the lanes with `want` to list l, region h (an XCD head): one returning
// atomic per wave.  An entry is the row with its tier in the top 4 bits (rh::kRowMask below).
// Every lane of the wave must call it (ballot).
__device__ __forceinline__ void list_append(const TableLists& l, bool want, int t, uint32_t row, uint32_t h) {
    const int lane = threadIdx.x & 63;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint64_t grp = __ballot(want);
    if (!grp) return;
    uint32_t base = 0;
    if (lane == 0) base = (uint32_t)atomicAdd(l.heads + (uint64_t)h * rh::kHeadStride, (unsigned long long)__popcll(grp));
    base = (uint32_t)__shfl((int)base, 0);
    if (want) {
        const uint32_t idx = base + (uint32_t)__popcll(grp & lt);
        if (idx < l.cap) l.rows[(uint64_t)h * l.cap + idx] = ((uint32_t)t << 28) | row;   // the host's bound keeps idx < cap
    }
}

// ---- deltas --------------------------------------------------------------------------------------
// One batch is applied in call order (its index in the batch) with the semantics of applying the
// deltas one by one: per target cell, the LAST SET wins and only the MAX deltas after it count.
// kApplyKeys: every SET raises its cell's key to (gen << 32) | index (64-bit atomicMax: the last SET
// holds the highest key); kApplySet: the SET holding its cell's key stores its value; kApplyMax: a
// MAX before its cell's last SET is dropped, the others atomicMax -- stream order puts the store
// before them.  A batch without SETs (gen == 0) runs kApplyMax alone, unchecked.  Every delta of a
// phase that applies (SET: kApplySet, MAX: kApplyMax) marks its row dirty -- the UPDATE_COMMIT event
// of LSI:846-854 -- and with dirty-row lists (lc / lw .rows non-null) appends a row it newly marks.
// resolved: the batch's slot fields already hold the row code (tier << 28 | row) the host's slot map
// gave at push time (rh_push_deltas; the device map is that map in stream order) -- no slot-map trip.
__global__ __launch_bounds__(256) void table_apply_kernel(TableDev Targ, const rh_delta* __restrict__ d, uint64_t n,
                                                          int phase, uint32_t gen, TableLists lc, TableLists lw,
                                                          int resolved) {
    // the tier is picked per thread: index the argument in the kernarg segment (scalar loads), not
    // the by-value copy, which the compiler spilled whole into scratch (984 B per lane, 8x slower)
    const TableDev& T = rh::kernarg_struct<TableDev>();
    (void)Targ;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool ac = false, aw = false;   // this delta newly marked its row (list mode)
    int t = 0;
    uint32_t row = 0;
    const unsigned long long key = ((unsigned long long)gen << 32) | (unsigned long long)i;
    do {   // one pass; `break` = the delta has no (further) effect
        if (i >= n) break;
        const rh_delta x = d[i];
        if (x.op != (phase == kApplyMax ? RH_OP_MAX : RH_OP_SET)) break;
        const TableTier* tt;
        if (resolved) {   // kernel argument: uniform
            t = (int)(x.slot >> 28);
            row = x.slot & rh::kRowMask;
            if (t >= rh::kTableTiers) break;
            tt = &T.tier[t];
            if (row >= tt->rows) break;
        } else {
            if (!locate(T, x.slot, tt, row)) break;  // stopped slot / out of range: ignored
            t = (int)(T.slot_map[x.slot] >> 28);
        }
        uint32_t off = 0xFFFFFFFFu;
        bool commit_ev = false, watch_ev = false;
        const uint32_t c = x.column, F = tt->width;
        if (c == RH_COL_LEASE_ON) {
            off = tile::kLon;
        } else if (c >= 48 && c < 64) {
            if (c - 48 < F) off = tile::fts(F, c - 48);
        } else if (c == RH_COL_LEASE) {
            off = tile::lease(F);
        } else if (c < 16) {
            if (c < F) off = tile::match(c);
            commit_ev = true;
        } else if (c < 32) {
            if (c - 16 < F) off = tile::fcommit(F, c - 16);
            watch_ev = true;
        } else if (c == RH_COL_FLUSH) {
            off = tile::flush(F);
            commit_ev = true;
        } else if (c == RH_COL_COMMITTED) {
            off = tile::commit(F);
            commit_ev = watch_ev = true;
        }
        if (off == 0xFFFFFFFFu) break;
        if (phase == kApplyKeys) {
            atomicMax(tt->key(off, row), key);
            break;
        }
        const bool last = phase == kApplySet ? *tt->key(off, row) == key
                                             : (gen == 0 || !(*tt->key(off, row) > key && (*tt->key(off, row) >> 32) == gen));
        if (last) {
            if (off == tile::kLon) {  // AtomicBoolean: SET stores, MAX ORs
                uint8_t* f = tt->u8(tile::kLon, row);
                if (phase == kApplySet)
                    *f = x.value != 0;
                else if (x.value != 0)
                    *f = 1;
            } else {
                int64_t* p = tt->i64(off, row);
                if (phase == kApplySet)
                    *p = x.value;
                else
                    atomicMax(reinterpret_cast<long long*>(p), (long long)x.value);
            }
        }
        if (commit_ev) ac = mark_listed(*tt, row, 0, lc.rows != nullptr);
        if (watch_ev) aw = mark_listed(*tt, row, 1, lw.rows != nullptr);
    } while (false);
    if (phase == kApplyKeys) return;   // uniform: marks come with the SET phase
    const uint32_t h = blockIdx.x & (rh::kHeads - 1);
    if (lc.rows) list_append(lc, ac, t, row, h);   // kernel arguments: uniform branches
    if (lw.rows) list_append(lw, aw, t, row, h);
}

// ---- control ops ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void table_control_kernel(TableDev Targ, const CtrlOp* __restrict__ ops, uint64_t n) {
    const TableDev& T = rh::kernarg_struct<TableDev>();
    (void)Targ;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const CtrlOp op = ops[i];
    if (op.kind == rh::kCtrlStop) {
        const TableTier& s = T.tier[op.src >> 28];
        const uint32_t r = op.src & rh::kRowMask;
        *s.u32(tile::kConf, r) = 0u;
        *s.u8(tile::kDirty, r) = 0;
        *s.u8(tile::kWdirty, r) = 0;
        *s.u8(tile::kLon, r) = 0;
        *s.u32(tile::kSlot, r) = rh::kNoRow;
        T.slot_map[op.slot] = rh::kNoRow;
        return;
    }
    const TableTier& D = T.tier[op.dst >> 28];
    const uint32_t r = op.dst & rh::kRowMask;
    const uint32_t DF = D.width;
    if (op.kind == rh::kCtrlStart) {
        for (uint32_t k = 0; k < DF; ++k) {
            *D.i64(tile::match(k), r) = -1;   // RaftLog.INVALID_LOG_INDEX (FollowerInfoImpl.java:42-43)
            *D.i64(tile::fcommit(DF, k), r) = -1;
            *D.i64(tile::fts(DF, k), r) = rh::kNoTimestamp;
        }
        *D.i64(tile::lease(DF), r) = rh::kNoTimestamp;  // rh_group_lease_start sets the LeaderLease
        *D.u8(tile::kLon, r) = 0;
        *D.i64(tile::flush(DF), r) = op.flush;
        *D.i64(tile::commit(DF), r) = op.commit;
        *D.i64(tile::tstart(DF), r) = op.tstart;
        *D.i64(tile::wall(DF), r) = INT64_MIN;
        *D.i64(tile::wmin(DF), r) = INT64_MIN;
        *D.i64(tile::wmaj(DF), r) = INT64_MIN;
        *D.i64(tile::wmax(DF), r) = INT64_MIN;
    } else {  // MOVE (to another tier) or RECONF (same row): follower columns through the map
        const TableTier& S = T.tier[op.src >> 28];
        const uint32_t sr = op.src & rh::kRowMask;
        const uint32_t SF = S.width;
        int64_t m[RH_MAX_FOLLOWERS], f[RH_MAX_FOLLOWERS], ts[RH_MAX_FOLLOWERS];
        for (uint32_t k = 0; k < DF; ++k) {  // read all first: RECONF may permute in place
            const int src = op.map[k];
            const bool keep = src >= 0 && (uint32_t)src < SF;
            m[k] = keep ? *S.i64(tile::match(src), sr) : -1;
            f[k] = keep ? *S.i64(tile::fcommit(SF, src), sr) : -1;
            ts[k] = keep ? *S.i64(tile::fts(SF, src), sr) : rh::kNoTimestamp;
        }
        for (uint32_t k = 0; k < DF; ++k) {
            *D.i64(tile::match(k), r) = m[k];
            *D.i64(tile::fcommit(DF, k), r) = f[k];
            *D.i64(tile::fts(DF, k), r) = ts[k];
        }
        if (op.kind == rh::kCtrlMove) {
            *D.i64(tile::flush(DF), r) = *S.i64(tile::flush(SF), sr);
            *D.i64(tile::commit(DF), r) = *S.i64(tile::commit(SF), sr);
            *D.i64(tile::tstart(DF), r) = *S.i64(tile::tstart(SF), sr);
            *D.i64(tile::wall(DF), r) = *S.i64(tile::wall(SF), sr);
            *D.i64(tile::wmin(DF), r) = *S.i64(tile::wmin(SF), sr);
            *D.i64(tile::wmaj(DF), r) = *S.i64(tile::wmaj(SF), sr);
            *D.i64(tile::wmax(DF), r) = *S.i64(tile::wmax(SF), sr);
            *D.i64(tile::lease(DF), r) = *S.i64(tile::lease(SF), sr);
            *D.u8(tile::kLon, r) = *S.u8(tile::kLon, sr);
            *S.u8(tile::kLon, sr) = 0;
            *S.u32(tile::kConf, sr) = 0u;
            *S.u8(tile::kDirty, sr) = 0;
            *S.u8(tile::kWdirty, sr) = 0;
            *S.u32(tile::kSlot, sr) = rh::kNoRow;
        }
    }
    *D.u32(tile::kConf, r) = op.conf;
    *D.u32(tile::kSlot, r) = op.slot;
    mark(D, r, 0);
    mark(D, r, 1);
    T.slot_map[op.slot] = op.dst;
}

// Fresh tiles: every row free (conf 0, unowned), clean, lease off; summaries clear.
__global__ __launch_bounds__(128) void table_init_tiles_kernel(TableTier tt, uint32_t first_tile) {
    const uint64_t r = (uint64_t)(first_tile + blockIdx.x) * rh::kTileRows + threadIdx.x;
    *tt.u8(tile::kDirty, r) = 0;
    *tt.u8(tile::kWdirty, r) = 0;
    *tt.u8(tile::kLon, r) = 0;
    *tt.u32(tile::kConf, r) = 0u;
    *tt.u32(tile::kSlot, r) = rh::kNoRow;
    if (threadIdx.x < 2) *tt.summary(r, (int)threadIdx.x) = 0;
}

// ---- updateCommit / commitIndexChanged over the dirty rows ---------------------------------------
// One workgroup = kTWaves waves, one 128-row tile per wave.  Every wave evaluates its rows' results
// in registers.  REGION mode (the DEVICE / AUTO sinks' tile evaluations): no records -- each wave's
// event masks go through LDS into its workgroup's descriptor, and rh_table_gather_commit / _watch
// rebuild the records from the masks and the values stored in the table.  Counter mode (the lists
// in pinned memory): the block gathers its events in LDS in wave order, takes ONE range of each
// result list with ONE device-scope atomic on the evaluation's counter word (rh_internal.h,
// TableEvents) and copies the records out as contiguous 16-byte-per-lane stores.
// Workgroup size (same box, 1M rows, profiles/r05/table_eval/): 12 waves 20.4 us all dirty, 6
// waves 20.2, 4 waves 19.3, 2 waves 19.1, 1 wave 19.3 -- small workgroups leave no CU holding a
// workgroup slot for its slowest wave at the tail.
struct TierRange {
    uint32_t block_begin[rh::kTableTiers + 1];  // blocks of launch slot i: [block_begin[i], block_begin[i+1])
    int8_t tier[rh::kTableTiers];               // tier of launch slot i (widest first)
    int32_t n_slots;
};

#ifndef RH_TABLE_WPE                         // A/B: waves per SIMD the widths-2..6 kernel is pinned to
#define RH_TABLE_WPE 6
#endif
#ifndef RH_TABLE_SUMMARY                     // A/B: skip clean tiles by their summary byte (1) or not (0)
#define RH_TABLE_SUMMARY 1
#endif
constexpr int kTWaves = RH_TABLE_BLOCK_WAVES;
constexpr int kTBlock = kTWaves * 64;
constexpr uint32_t kTRows = kTWaves * 128;   // rows per workgroup
static_assert(kTRows <= rh::kTableRecs && 2 + 8 * kTWaves == rh::kTableDesc,
              "REGION mode: a workgroup's records fit its region, its counts its descriptor");
#ifndef RH_TABLE_NT                          // A/B: non-temporal column loads (1) or plain (0)
#define RH_TABLE_NT 0
#endif

#ifndef RH_TABLE_ABL   // ablation only (wrong results): 2 = no events, 3 = no table stores, 4 = trivial arithmetic
#define RH_TABLE_ABL 0   // list kernel: 6 / 7 = 5 / 3 lines per row, 8 = no counter atomic or records, 9 = 6 + 8, 10 = no watch-list appends
#endif

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
#ifndef RH_TABLE_STAGE   // A/B: SPEC evaluations stage their section through LDS (1) or load per lane (0)
#define RH_TABLE_STAGE 0
#endif

template <typename V>
__device__ __forceinline__ V tload(const uint8_t* p) {
    if (RH_TABLE_NT) return __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
    return *reinterpret_cast<const V*>(p);
}

// Event staging of one workgroup in LDS: wave w owns 128 records of each kind at w * 128 (kind 0 =
// advanced commit (COMMIT) / changed levels (WATCH), kind 1 = changed watch-ALL level (COMMIT)), so
// a wave writes its records as soon as it has them and keeps nothing live across the barrier.
struct Stage {
    unsigned long long mask[kTWaves][4];   // REGION mode, COMMIT: each wave's event masks (zero: none)
    uint32_t cnt[2][kTWaves];
    uint32_t pre[2][kTWaves + 1];  // exclusive prefix of cnt over the waves
    unsigned long long base;        // the block's first record in list 0 (REGION mode: in both lists)
    unsigned long long base1;       // counter mode: its first record in list 1
};

// SPEC (chosen per evaluation by the host, rh_table_commit): the evaluation follows deltas that
// may have marked a large part of the table, so nearly every tile and most of its column lines hold
// a dirty row -- the column loads are issued with the flag load instead of after it (one dependent
// HBM trip per wave fewer) and the tile summary is not consulted.  Measured (1M rows, same box,
// profiles/r04/table_spec/): 100 % dirty 23.7 -> 22.2 us, but 4 % dirty 18.3 -> 21.4 us (clean
// lines loaded): hence the host's choice.
template <int F, bool RANK, bool WATCH, bool SPEC>
__device__ __forceinline__ void table_wave(const TableDev& T, const TableTier& tt, uint64_t tl, bool wall_on,
                                           unsigned char* ws, Stage& sc, const TableEvents& ev, uint64_t gb) {
    constexpr int N = F + 1;
    constexpr uint64_t TB = tile::bytes(F);
    const int lane = threadIdx.x & 63;
    uint8_t* tb = tt.base + tl * TB;   // this wave's tile: rows 128 tl .. 128 tl + 127
    uint8_t* sump = tt.sum + 2 * tl + (WATCH ? 1 : 0);
    if (!SPEC && RH_TABLE_SUMMARY && *sump == 0) return;  // clean tile: its flag line is not read
    uint8_t* dflag = tb + (WATCH ? tile::kWdirty : tile::kDirty) + 2 * lane;
    const uint16_t dd = *reinterpret_cast<const uint16_t*>(dflag);
    const bool d0 = (dd & 0xFFu) != 0, d1 = (dd >> 8) != 0;
    const bool need = d0 || d1;
    if (!SPEC && !__any(need)) {
        if (lane == 0) *sump = 0;
        return;
    }
    int64_t fv[2][F], self[2] = {0, 0}, cin[2] = {0, 0}, ts[2] = {0, 0};
    int64_t p0[2] = {0, 0}, p1[2] = {0, 0}, p2[2] = {0, 0};
    uint32_t w[2] = {0u, 0u}, slot[2] = {0u, 0u};
    const uint32_t l8 = 8u * lane;
    if (SPEC || need) {  // every load of the row pair is issued before any result is used
        // the lane's row-pair record of its evaluation's section (rh_internal.h, tile::pair_off):
        // [match[F] flush tstart wall] or [fcommit[F] wmin wmaj wmax], NS 16-byte pairs
        constexpr uint32_t NS = F + 3;
        constexpr uint32_t c0 = WATCH ? tile::fcommit(F, 0) : tile::match(0);
        constexpr uint32_t s0 = tile::pair_off(F, c0, 0);
        const uint8_t* sb = tb + s0;   // the section: in the tile, or staged in LDS
#if RH_TABLE_STAGE
        if constexpr (SPEC) {
            // nearly every row pair is dirty: the section moves as one coalesced run into the wave's
            // LDS region (LDS-DMA, 64 x 16 B per instruction), each lane then reads its record --
            // NS odd: 16-byte reads at a stride of NS x 16 B hit every bank group once per 16 lanes
#pragma unroll
            for (uint32_t i = 0; i < NS; ++i)
                __builtin_amdgcn_global_load_lds((gbl_void_t*)(tb + s0 + 1024u * i + 16u * lane), (lds_void_t*)(ws + 1024u * i), 16, 0, 0);
        }
#endif
        const v2u32 c = tload<v2u32>(tb + tile::kConf + l8);
        // row slots only for records this kernel writes (REGION mode: the gather reads them)
        const v2u32 sl = ev.bdesc ? v2u32{0u, 0u} : tload<v2u32>(tb + tile::kSlot + l8);
        const v2i64 cm = tload<v2i64>(tb + tile::pair_off(F, tile::commit(F), lane));
#if RH_TABLE_STAGE
        if constexpr (SPEC) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the wave's LDS-DMA has landed
            sb = ws;
        }
#endif
        auto sec = [&](uint32_t col) {   // the lane's row pair of column col
            return *reinterpret_cast<const v2i64*>(sb + (tile::pair_off(F, col, lane) - s0));
        };
#pragma unroll
        for (int k = 0; k < F; ++k) {
            const v2i64 x = sec(WATCH ? tile::fcommit(F, k) : tile::match(k));
            fv[0][k] = x.x;
            fv[1][k] = x.y;
        }
        slot[0] = sl.x;
        slot[1] = sl.y;
        w[0] = d0 ? c.x : 0u;  // a clean row is evaluated as inactive and produces nothing
        w[1] = d1 ? c.y : 0u;
        cin[0] = cm.x;
        cin[1] = cm.y;
        if (WATCH) {
            self[0] = cm.x;  // lastCommittedIndex is the self value (LSI:613)
            self[1] = cm.y;
            const v2i64 a = sec(tile::wmin(F));
            const v2i64 b = sec(tile::wmaj(F));
            const v2i64 e = sec(tile::wmax(F));
            p0[0] = a.x, p0[1] = a.y, p1[0] = b.x, p1[1] = b.y, p2[0] = e.x, p2[1] = e.y;
        } else {
            const v2i64 fl = sec(tile::flush(F));
            const v2i64 st = sec(tile::tstart(F));
            self[0] = fl.x, self[1] = fl.y, ts[0] = st.x, ts[1] = st.y;
            if (wall_on) {  // watch-ALL levels are compared only when reported (RH_COMMIT_WATCH_ALL)
                const v2i64 wa = sec(tile::wall(F));
                p0[0] = wa.x, p0[1] = wa.y;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < F; ++k) fv[0][k] = fv[1][k] = 0;
    }
    const int64_t gap = WATCH ? -1 : T.gap;  // commitIndexChanged uses the 2-arg overload (gap -1)
    bool trans[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) trans[g] = (w[g] & RH_CONF_ACTIVE) && (w[g] & RH_CONF_TRANSITIONAL);
    const bool any_trans = __any(trans[0] || trans[1]);
    bool e0[2], e1[2] = {false, false};
    uint32_t valid[2];
    int64_t x0[2], x1[2], x2[2];  // COMMIT: new commit, min; WATCH: min, majority, max
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        int64_t vals[N];
#pragma unroll
        for (int k = 0; k < F; ++k) vals[k] = fv[g][k];
        vals[F] = self[g];
        bool v;
        int64_t mn, mj, mx;
#if RH_TABLE_ABL == 4
        (void)any_trans;
        v = (w[g] & RH_CONF_ACTIVE) != 0;
        mn = vals[0];
#pragma unroll
        for (int k = 1; k < N; ++k) mn ^= vals[k];
        mj = mn + 1;
        mx = mn + 2;
#else
        rh_eval::eval_group<F, RANK>(vals, w[g], gap, any_trans, v, mn, mj, mx);
#endif
        const bool dg = g ? d1 : d0;
        valid[g] = v ? 1u : 0u;
        if (WATCH) {
            e0[g] = dg && (mn != p0[g] || mj != p1[g] || mx != p2[g]);
            x0[g] = mn, x1[g] = mj, x2[g] = mx;
        } else {
            int64_t nc = cin[g];
            e0[g] = dg && rh_eval::commit_decision(v, mj, cin[g], self[g], ts[g], nc);
            e1[g] = dg && wall_on && mn != p0[g];  // watch-ALL level changed (LSI:1025)
            x0[g] = nc, x1[g] = mn, x2[g] = 0;
        }
    }
    // table stores: only what changed, plus clearing this lane's dirty flags and the tile summary
    const uint64_t a0 = __ballot(e0[0]), a1 = __ballot(e0[1]);
#if RH_TABLE_ABL == 3
    if (lane == 64) {
#else
    {
#endif
    if (need) *reinterpret_cast<uint16_t*>(dflag) = 0;
    if (lane == 0) *sump = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const uint32_t ro = 2u * lane + g;
        if (WATCH) {
            if (e0[g]) {
                *reinterpret_cast<int64_t*>(tb + tile::pair_off(F, tile::wmin(F), lane) + 8u * g) = x0[g];
                *reinterpret_cast<int64_t*>(tb + tile::pair_off(F, tile::wmaj(F), lane) + 8u * g) = x1[g];
                *reinterpret_cast<int64_t*>(tb + tile::pair_off(F, tile::wmax(F), lane) + 8u * g) = x2[g];
            }
        } else {
            if (e0[g]) {
                *reinterpret_cast<int64_t*>(tb + tile::pair_off(F, tile::commit(F), lane) + 8u * g) = x0[g];
                tb[tile::kWdirty + ro] = 1;  // the commit index changed: commitIndexChanged follows (LSI:1003)
            }
            if (e1[g]) *reinterpret_cast<int64_t*>(tb + tile::pair_off(F, tile::wall(F), lane) + 8u * g) = x1[g];
        }
    }
    if (!WATCH && (a0 | a1) && lane == 0) tt.sum[2 * tl + 1] = 1;
    }
#if RH_TABLE_ABL == 2
    if (lane == 0) sc.cnt[0][threadIdx.x >> 6] = 0;
    return;
#endif
    // events: in REGION mode the wave's masks (into the workgroup's descriptor); else compacted into
    // this wave's LDS region, in row order, for the workgroup's copy-out
    const int wave = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t p = (uint32_t)(__popcll(a0 & lt) + __popcll(a1 & lt));
    if (ev.bdesc) {
        if (WATCH) {   // no records: the changed rows and their valid flags (levels: in the table)
            const uint64_t v0 = __ballot(e0[0] && valid[0]), v1 = __ballot(e0[1] && valid[1]);
            if (lane == 0) {
                sc.mask[wave][0] = a0;
                sc.mask[wave][1] = a1;
                sc.mask[wave][2] = v0;
                sc.mask[wave][3] = v1;
            }
        } else {
            // no records: the wave's masks (the values are in the table, rh_table_gather_commit),
            // staged in LDS: a wave that returned early (clean tile) leaves the block's zeros
            const uint64_t c0 = __ballot(e1[0]), c1 = __ballot(e1[1]);
            if (lane == 0) {
                sc.mask[wave][0] = a0;
                sc.mask[wave][1] = a1;
                sc.mask[wave][2] = c0;
                sc.mask[wave][3] = c1;
                sc.cnt[1][wave] = (uint32_t)(__popcll(c0) + __popcll(c1));
            }
        }
    } else if (WATCH) {
        rh_watch_event* sw = reinterpret_cast<rh_watch_event*>(ws);   // this wave's LDS region
#pragma unroll
        for (int g = 0; g < 2; ++g)
            if (e0[g]) sw[p++] = rh_watch_event{slot[g], valid[g], x0[g], x1[g], x2[g]};
    } else {
        rh_index_event* sa = reinterpret_cast<rh_index_event*>(ws);   // this wave's LDS region
        rh_index_event* sw = sa + 128;
        const uint64_t c0 = __ballot(e1[0]), c1 = __ballot(e1[1]);
        uint32_t q = (uint32_t)(__popcll(c0 & lt) + __popcll(c1 & lt));
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            if (e0[g]) sa[p++] = rh_index_event{slot[g], 0u, x0[g]};
            if (e1[g]) sw[q++] = rh_index_event{slot[g], 0u, x1[g]};
        }
        if (lane == 0) sc.cnt[1][wave] = (uint32_t)(__popcll(c0) + __popcll(c1));
    }
    if (lane == 0) sc.cnt[0][wave] = (uint32_t)(__popcll(a0) + __popcll(a1));
}

template <int F, int FHI, bool RANK, bool WATCH, bool SPEC>
__device__ __forceinline__ void table_dispatch(const TableDev& T, int t, uint64_t tl, bool wall_on,
                                               unsigned char* ws, Stage& sc, const TableEvents& ev, uint64_t gb) {
    if ((int)rh::width_of_tier(t) == F)
        table_wave<F, RANK, WATCH, SPEC>(T, T.tier[t], tl, wall_on, ws, sc, ev, gb);
    else if constexpr (F + 2 <= FHI)
        table_dispatch<F + 2, FHI, RANK, WATCH, SPEC>(T, t, tl, wall_on, ws, sc, ev, gb);
}

// LDS per wave of a tile workgroup whose widths reach FHI: the staged section (SPEC) or, in counter
// mode, the wave's records (128 of 32 B, or 2 x 128 of 16 B) -- one region, used in that order
template <int FHI, bool SPEC>
constexpr uint32_t wave_lds() { return SPEC && RH_TABLE_STAGE && 1024u * (FHI + 3) > 4096u ? 1024u * (FHI + 3) : 4096u; }

// The evaluation's counter word (rh_internal.h, TableEvents): kind 0 in bits [0, cbits), kind 1 in
// [cbits, 2 cbits), workgroups done above when the count fits there (`packed`; the list kernel
// always: at most kListMaxGrid workgroups < 2^8).
#ifndef RH_LIST_WAVES   // A/B: waves per list-kernel workgroup
#define RH_LIST_WAVES 2
#endif
constexpr uint32_t kListWaves = RH_LIST_WAVES;
#ifndef RH_LIST_TOTAL_WAVES   // A/B: waves of the list grid (960 before round 5: 0.1 % dirty 8.0 -> 7.5 us, 1 % unchanged)
#define RH_LIST_TOTAL_WAVES 480
#endif
constexpr uint32_t kListMaxGrid = RH_LIST_TOTAL_WAVES / kListWaves;   // < 2^8 workgroups: the done count's byte
static_assert(kListMaxGrid < 256, "the done count's byte");
static_assert(kListWaves >= 2, "thread 64 (wave 1) stages the tier table while wave 0 does the bookkeeping");

__device__ __forceinline__ void publish_counts(const TableEvents& ev, unsigned long long c) {
    const unsigned long long m = (1ull << ev.cbits) - 1;
    ev.counts_out[0] = c & m;
    ev.counts_out[1] = (c >> ev.cbits) & m;
}

// Thread 0 of a tile-kernel workgroup after its counter atomic, when the done count has its own
// word: counts the workgroup done; the one completing the evaluation's count (done_target, 0 in
// a launch that does not end the evaluation) zeroes both words and publishes the list lengths.
// `after` is the counter atomic's return value (0 without one): the done increment depends on it,
// so it issues only once the counter atomic has been performed (both execute at the memory side,
// MI355X_MICROARCH.md 'Global float atomics') -- no fence, which at agent scope would write back
// this XCD's L2.
__device__ __forceinline__ void block_done(const TableEvents& ev, unsigned long long after) {
    if (atomicAdd(ev.done, 1u + (unsigned int)(after >> 63)) + 1u != ev.done_target) return;
    atomicExch(ev.done, 0u);
    publish_counts(ev, atomicExch(ev.cnt, 0ull));
}

// One workgroup (block index b of the launch).
template <bool WATCH, int FLO, int FHI, bool SPEC>
__device__ __forceinline__ void table_block_iter(const TableDev& T, const TierRange& tr, const TableEvents& ev,
                                                 uint32_t b, unsigned char* stage, Stage& sc) {
    const int wave = threadIdx.x >> 6;
    const bool wall_on = !WATCH && ev.wall != nullptr;
    int i = 0;
#pragma unroll
    for (int k = 1; k < rh::kTableTiers; ++k)
        if (k < tr.n_slots && b >= tr.block_begin[k]) i = k;
    const int t = tr.tier[i];
    const uint64_t tl = (uint64_t)(b - tr.block_begin[i]) * kTWaves + wave;   // tile of this wave
    if (threadIdx.x < 2 * kTWaves) (&sc.cnt[0][0])[threadIdx.x] = 0u;
    if (threadIdx.x < 4 * kTWaves) (&sc.mask[0][0])[threadIdx.x] = 0ull;
    if (b == 0 && threadIdx.x < rh::kHeads && ev.lheads_next)
        ev.lheads_next[threadIdx.x * rh::kHeadStride] = 0ull;  // the next list set of this kind
    __syncthreads();
    const uint64_t gb = (uint64_t)ev.block_base + b;   // REGION mode: the evaluation's workgroup number
    constexpr uint32_t WL = wave_lds<FHI, SPEC>();
    if (tl * rh::kTileRows < T.tier[t].rows)
        table_dispatch<FLO, FHI, FLO <= 6, WATCH, SPEC>(T, t, tl, wall_on, stage + wave * WL, sc, ev, gb);
    __syncthreads();

    if (ev.bdesc) {   // ---- REGION mode: the descriptor: totals, the waves' masks
        uint64_t* md = reinterpret_cast<uint64_t*>(ev.bdesc) + gb * (rh::kTableDesc / 2);
        if (threadIdx.x == 0) {
            uint64_t v0 = 0, v1 = 0;
#pragma unroll
            for (int w = 0; w < kTWaves; ++w) v0 += sc.cnt[0][w], v1 += sc.cnt[1][w];
            md[0] = v0 | v1 << 32;
        } else if (threadIdx.x <= 4 * kTWaves) {
            md[threadIdx.x] = (&sc.mask[0][0])[threadIdx.x - 1];
        }
        return;
    }
    // ---- one range of each list per block (one device-scope atomic), then a contiguous copy
    if (threadIdx.x == 0) {
        uint32_t a0 = 0, a1 = 0;
        for (int k = 0; k < kTWaves; ++k) {
            sc.pre[0][k] = a0;
            sc.pre[1][k] = a1;
            a0 += sc.cnt[0][k];
            a1 += sc.cnt[1][k];
        }
        sc.pre[0][kTWaves] = a0;
        sc.pre[1][kTWaves] = a1;
        {   // counter mode (REGION mode returned above)
            const uint32_t cb = ev.cbits;
            const unsigned long long add = (unsigned long long)a0 | ((unsigned long long)a1 << cb) |
                                           (ev.packed ? 1ull << (2 * cb) : 0ull);
            const unsigned long long old = add ? atomicAdd(ev.cnt, add) : 0ull;
            const unsigned long long cm = (1ull << cb) - 1;
            sc.base = old & cm;
            sc.base1 = (old >> cb) & cm;
            if (!ev.packed) {
                block_done(ev, old);
            } else if (ev.done_target && ((old + add) >> (2 * cb)) == ev.done_target) {   // the last workgroup
                publish_counts(ev, old + add);
                atomicExch(ev.cnt, 0ull);   // the next evaluation's counter
            }
        }
    }
    __syncthreads();
    const uint32_t tot0 = sc.pre[0][kTWaves], tot1 = sc.pre[1][kTWaves];
    if (!(tot0 | tot1)) return;
    const uint64_t R = ev.cap;   // a list holds one record per row at most: never reached
    const uint64_t b0 = sc.base, b1 = sc.base1;
    const uint64_t lim0 = b0 >= R ? 0 : (b0 + tot0 <= R ? tot0 : R - b0);
    const uint64_t lim1 = b1 >= R ? 0 : (b1 + tot1 <= R ? tot1 : R - b1);
    // record e of the block lives in the region of wave k with pre[k] <= e < pre[k + 1]
    typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
    const v4u32* src = reinterpret_cast<const v4u32*>(stage);
    if (WATCH) {  // 32-byte records: two 16-byte words each
        v4u32* dst = reinterpret_cast<v4u32*>(ev.watch + b0);
        for (uint32_t j = threadIdx.x; j < 2 * lim0; j += kTBlock) {
            const uint32_t e = j >> 1;
            uint32_t k = 0;
#pragma unroll
            for (int m = 1; m < kTWaves; ++m) k += e >= sc.pre[0][m] ? 1u : 0u;
            dst[j] = src[k * (WL / 16) + 2 * (e - sc.pre[0][k]) + (j & 1)];
        }
    } else {
        v4u32* da = reinterpret_cast<v4u32*>(ev.adv + b0);
        for (uint32_t e = threadIdx.x; e < lim0; e += kTBlock) {
            uint32_t k = 0;
#pragma unroll
            for (int m = 1; m < kTWaves; ++m) k += e >= sc.pre[0][m] ? 1u : 0u;
            da[e] = src[k * (WL / 16) + (e - sc.pre[0][k])];
        }
        if (ev.wall) {
            v4u32* dw = reinterpret_cast<v4u32*>(ev.wall + b1);
            for (uint32_t e = threadIdx.x; e < lim1; e += kTBlock) {
                uint32_t k = 0;
#pragma unroll
                for (int m = 1; m < kTWaves; ++m) k += e >= sc.pre[1][m] ? 1u : 0u;
                dw[e] = src[k * (WL / 16) + 128 + (e - sc.pre[1][k])];
            }
        }
    }
}

template <bool WATCH, int FLO, int FHI, bool SPEC>
__device__ __forceinline__ void table_commit_block(const TierRange& tr, const TableEvents& ev) {
    const TableDev& T = rh::kernarg_struct<TableDev>();  // block-uniform tier index: scalar loads
    // per wave (wave_lds): the staged section, then (counter mode) its records
    __shared__ __attribute__((aligned(16))) unsigned char stage[kTWaves * wave_lds<FHI, SPEC>()];
    __shared__ Stage sc;
    table_block_iter<WATCH, FLO, FHI, SPEC>(T, tr, ev, blockIdx.x, stage, sc);
}

// Widths 2..6: rank-mask order statistics, 6 waves per SIMD (<= 84 VGPRs: the row pair's columns
// are all in flight before the compute; at 64 VGPRs the compiler spilled 52 B per lane; pinned to
// 8 waves per SIMD, 19.9 us vs 19.3 at 4-wave workgroups).  Widths 8..14: Batcher networks
// (commit.hip's split) with the registers their 15-value networks need; these tiers are rare.
template <bool WATCH, bool SPEC>
__global__ __launch_bounds__(kTBlock) __attribute__((amdgpu_waves_per_eu(RH_TABLE_WPE, 8))) void table_commit_kernel_rank(
    TableDev Targ, TierRange tr, TableEvents ev) {
    (void)Targ;
    table_commit_block<WATCH, 2, 6, SPEC>(tr, ev);
}

template <bool WATCH, bool SPEC>
__global__ __launch_bounds__(kTBlock) void table_commit_kernel_net(TableDev Targ, TierRange tr, TableEvents ev) {
    (void)Targ;
    table_commit_block<WATCH, 8, 14, SPEC>(tr, ev);
}

// ---- list mode: updateCommit / commitIndexChanged over the listed rows only ---------------------
// One lane per listed row (random rows: each lane loads its row's 8-byte column elements).  The
// lanes of a wave may hold rows of different tiers (widths): the row evaluation is instantiated per
// width and the wave runs the widths its lanes hold.  Entries are dealt per region: wave wg takes
// head region r = wg % kHeads at rank k = wg / kHeads, and in pass p lane j takes the region's
// entry (64 p + j) Wr + k (Wr = the region's waves: a sparse list spreads over all of them, a few
// rows per wave on nearly every CU) -- so a wave loads its region's count and its first entries in
// one trip (the entries speculatively, below the capacity), with no scan of the counts before the
// rows are loaded; wave 0 of each workgroup loads all eight counts for the bookkeeping (passes,
// workgroups holding entries, this workgroup's last pass).  Events: per pass one counter atomic per
// workgroup (its waves' counts summed in LDS), records written straight into the result lists;
// the last pass's atomic also counts the workgroup done (the counter word's top bits), so the
// workgroup that completes the count knows the list lengths from its own atomic's return.
template <int F, bool WATCH>
__device__ __forceinline__ void list_row(const TableDev& T, const TableTier& tt, uint32_t r, bool wall_on,
                                         bool wlisted, bool& e0, bool& e1, bool& wtrans, int64_t& x0, int64_t& x1,
                                         int64_t& x2, uint32_t& valid, uint32_t& slot, bool need_slot) {
    int64_t vals[F + 1];
    const uint32_t w = *tt.u32(tile::kConf, r);
    slot = need_slot ? *tt.u32(tile::kSlot, r) : 0u;   // REGION mode: the gather reads it
    const int64_t cm = *tt.i64(tile::commit(F), r);
#if RH_TABLE_ABL == 6 || RH_TABLE_ABL == 7 || RH_TABLE_ABL == 9   // ablation (wrong results): a row's lines cut to conf, slot, commit (+ flags)
#pragma unroll
    for (int k = 0; k < F; ++k) vals[k] = cm + k;
#else
#pragma unroll
    for (int k = 0; k < F; ++k) vals[k] = *tt.i64(WATCH ? tile::fcommit(F, k) : tile::match(k), r);
#endif
    // the row's commitIndexChanged flag, read with its columns: a listed row is in this list once,
    // so its lane alone may set the flag here (plain store; no atomic to find the transition)
#if RH_TABLE_ABL == 7
    const uint8_t wd = 0;
#else
    const uint8_t wd = WATCH ? 0 : *tt.u8(tile::kWdirty, r);
#endif
    int64_t self, ts = 0, p0 = 0, p1 = 0, p2 = 0;
    if (WATCH) {
        self = cm;  // lastCommittedIndex is the self value (LSI:613)
        p0 = *tt.i64(tile::wmin(F), r);
        p1 = *tt.i64(tile::wmaj(F), r);
        p2 = *tt.i64(tile::wmax(F), r);
    } else {
#if RH_TABLE_ABL == 6 || RH_TABLE_ABL == 7 || RH_TABLE_ABL == 9
        self = cm + 7, ts = 0, p0 = cm;
#else
        self = *tt.i64(tile::flush(F), r);
        ts = *tt.i64(tile::tstart(F), r);
        if (wall_on) p0 = *tt.i64(tile::wall(F), r);
#endif
    }
    vals[F] = self;
    const bool trans = (w & RH_CONF_ACTIVE) && (w & RH_CONF_TRANSITIONAL);   // lane-local: always exact
    bool v;
    int64_t mn, mj, mx;
    rh_eval::eval_group<F, (F <= 6)>(vals, w, WATCH ? -1 : T.gap, trans, v, mn, mj, mx);
    valid = v ? 1u : 0u;
    if (WATCH) {
        e0 = mn != p0 || mj != p1 || mx != p2;
        x0 = mn, x1 = mj, x2 = mx;
        if (e0) {
            *tt.i64(tile::wmin(F), r) = mn;
            *tt.i64(tile::wmaj(F), r) = mj;
            *tt.i64(tile::wmax(F), r) = mx;
        }
        *tt.u8(tile::kWdirty, r) = 0;
    } else {
        int64_t nc;
        e0 = rh_eval::commit_decision(v, mj, cm, self, ts, nc);
        e1 = wall_on && mn != p0;  // watch-ALL level changed (LSI:1025)
        x0 = nc, x1 = mn, x2 = 0;
#if RH_TABLE_ABL != 7
        *tt.u8(tile::kDirty, r) = 0;
#endif
        if (e0) {
            *tt.i64(tile::commit(F), r) = nc;
            // the commit index changed: commitIndexChanged follows (listed if the flag was clear)
            *tt.u8(tile::kWdirty, r) = 1;
            *tt.summary(r, 1) = 1;
            wtrans = wlisted && wd == 0;
        }
        if (e1) *tt.i64(tile::wall(F), r) = mn;
    }
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d));
    return v;
}

// REGION mode: this workgroup's descriptors of passes [from, list_passes) -- passes the evaluation
// does not run -- zeroed, so the gather (launched over the host's bound) finds no events there.
__device__ __forceinline__ void zero_list_desc(const TableEvents& ev, uint32_t from) {
    constexpr uint32_t S = rh::kTableDesc / 2;
    uint64_t* d = reinterpret_cast<uint64_t*>(ev.bdesc);
    const uint32_t n = ev.list_passes > from ? (ev.list_passes - from) * S : 0u;
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x)
        d[((uint64_t)(from + j / S) * gridDim.x + blockIdx.x) * S + j % S] = 0ull;
}
static_assert(kListWaves == kTWaves, "REGION mode: a list workgroup's masks fill a tile workgroup's descriptor");

template <bool WATCH>
__global__ __launch_bounds__(kListWaves * 64) void table_list_kernel(TableDev Targ, TableLists L, TableLists Lw, TableEvents ev) {
    const TableDev& T = rh::kernarg_struct<TableDev>();
    (void)Targ;
    constexpr uint32_t NR = rh::kHeads;
    // lanes pick tiers per row: from LDS, not by per-lane loads of the kernarg segment
    __shared__ __attribute__((aligned(16))) unsigned char tiers_mem[sizeof(TableTier) * rh::kTableTiers];
    TableTier* tiers = reinterpret_cast<TableTier*>(tiers_mem);
    __shared__ uint32_t wcnt[2][kListWaves];   // per pass: the waves' record counts
    __shared__ unsigned long long lbase;       // per pass: the workgroup's range of the lists
    __shared__ uint32_t book[3];               // passes, workgroups holding entries, this one's last pass + 1
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * kListWaves, wg = blockIdx.x * kListWaves + (uint32_t)wave;
    const uint32_t r = wg % NR, k = wg / NR, Wr = (W - r + NR - 1) / NR;
    // one trip: this wave's region count and first entries; wave 0 also every region's count
    const unsigned long long hr = L.heads[(uint64_t)r * rh::kHeadStride];
    const uint32_t i0 = (uint32_t)lane * Wr + k;
    const uint32_t ent0 = i0 < L.cap ? L.rows[(uint64_t)r * L.cap + i0] : 0u;
    uint32_t cl = 0;
    if (wave == 0 && lane < (int)NR) {
        const unsigned long long x = L.heads[(uint64_t)lane * rh::kHeadStride];
        cl = (uint32_t)(x < L.cap ? x : L.cap);
    }
    if (threadIdx.x == 64) {
#pragma unroll
        for (int q = 0; q < rh::kTableTiers; ++q) tiers[q] = T.tier[q];   // uniform index: scalar loads
    }
    if (blockIdx.x == 0 && threadIdx.x < NR && ev.lheads_next)
        ev.lheads_next[(uint64_t)threadIdx.x * rh::kHeadStride] = 0ull;   // the next list set of this kind
    const uint32_t cnt = (uint32_t)(hr < L.cap ? hr : L.cap);
    if (wave == 0) {
        // wave g holds entries in pass p iff 64 p Wr(g % NR) + g / NR < count[g % NR]
        uint32_t np = 0;
        if (lane < (int)NR) {
            const uint32_t wr = (W - (uint32_t)lane + NR - 1) / NR;
            np = (cl + wr * 64u - 1) / (wr * 64u);
        }
        np = wave_max_u32(np);
        uint32_t act = 0;
        for (uint32_t b0 = 0; b0 < gridDim.x; b0 += 64) {   // uniform trip count: every lane shuffles
            const uint32_t b = b0 + (uint32_t)lane;
            bool any = false;
#pragma unroll
            for (uint32_t w = 0; w < kListWaves; ++w) {
                const uint32_t g = b * kListWaves + w;
                const uint32_t cg = (uint32_t)__shfl((int)cl, (int)(g % NR));
                any |= b < gridDim.x && g / NR < cg;
            }
            act += (uint32_t)__popcll(__ballot(any));
        }
        // this workgroup's last pass holding entries, + 1 (0: none): lane w < kListWaves for wave w
        const uint32_t g = blockIdx.x * kListWaves + (uint32_t)(lane % kListWaves), rg = g % NR, kg = g / NR;
        const uint32_t wr = (W - rg + NR - 1) / NR;
        const uint32_t cg = (uint32_t)__shfl((int)cl, (int)rg);
        uint32_t lp1 = kg < cg ? (cg - 1 - kg) / (wr * 64u) + 1 : 0u;
        lp1 = wave_max_u32(lane < (int)kListWaves ? lp1 : 0u);
        if (lane == 0) {
            book[0] = np;
            book[1] = act;
            book[2] = lp1;
        }
    }
    __syncthreads();   // the tier table and the bookkeeping (the loads above are still in flight)
    const uint32_t np = book[0], active = book[1], lp1 = book[2];
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t h = blockIdx.x & (rh::kHeads - 1);   // the watch-list region rows are appended to
    const uint64_t R = ev.cap;
    const bool wall_on = !WATCH && ev.wall != nullptr;
    const bool wl = Lw.rows != nullptr;
    const bool region = ev.bdesc != nullptr;   // REGION mode (kernel argument: uniform)
    if (active == 0) {   // empty lists
        if (region) zero_list_desc(ev, 0);
        else if (blockIdx.x == 0 && threadIdx.x == 0) publish_counts(ev, 0ull);
        return;
    }
    for (uint32_t pass = 0; pass < np; ++pass) {
        const uint32_t idx = (pass * 64u + (uint32_t)lane) * Wr + k;
        const bool has = idx < cnt;
        bool e0 = false, e1 = false, wtrans = false;
        int64_t x0 = 0, x1 = 0, x2 = 0;
        uint32_t valid = 0, slot = 0, row = 0;
        int t = 0;
        if (has) {
            const uint32_t ent = pass == 0 ? ent0 : L.rows[(uint64_t)r * L.cap + idx];
            t = (int)(ent >> 28);
            row = ent & rh::kRowMask;
            const TableTier tt = tiers[t < rh::kTableTiers ? t : 0];
            switch (tt.width) {
                case 2: list_row<2, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
                case 4: list_row<4, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
                case 6: list_row<6, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
                case 8: list_row<8, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
                case 10: list_row<10, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
                case 12: list_row<12, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
                default: list_row<14, WATCH>(T, tt, row, wall_on, wl, e0, e1, wtrans, x0, x1, x2, valid, slot, !region); break;
            }
        }
        // events: one range of the lists per workgroup and pass
        const uint64_t a = __ballot(e0), c = WATCH ? 0ull : __ballot(e1);
        if (region) {
            // no records, no counter atomic: the wave's masks (COMMIT: advanced, watch-ALL changed;
            // WATCH: changed, valid) and the workgroup's totals into its descriptor of this pass --
            // rh_table_gather_commit / _watch rebuild the records from the list entries and the table
            const uint64_t cv = WATCH ? __ballot(e0 && valid != 0u) : c;
            const bool rec = pass < ev.list_passes;   // the host's bound: never exceeded
            uint64_t* md = reinterpret_cast<uint64_t*>(ev.bdesc) + ((uint64_t)pass * gridDim.x + blockIdx.x) * (rh::kTableDesc / 2);
            if (rec && lane < 4) md[1 + 4 * wave + lane] = lane == 0 ? a : (lane == 2 ? cv : 0ull);
            if (lane == 0) {
                wcnt[0][wave] = (uint32_t)__popcll(a);
                wcnt[1][wave] = (uint32_t)__popcll(c);
            }
            __syncthreads();
#if RH_TABLE_ABL != 10   // ablation (wrong results): no watch-list appends
            if (!WATCH && wl) list_append(Lw, wtrans, t, row, h);   // kernel argument: uniform
#endif
            if (threadIdx.x == 0 && rec) {
                unsigned long long s0 = 0, s1 = 0;
#pragma unroll
                for (uint32_t q = 0; q < kListWaves; ++q) s0 += wcnt[0][q], s1 += wcnt[1][q];
                md[0] = s0 | (s1 << 32);
            }
            if (pass + 1 < np) __syncthreads();   // wcnt is the next pass's (np: uniform)
            continue;
        }
        if (lane == 0) {
            wcnt[0][wave] = (uint32_t)__popcll(a);
            wcnt[1][wave] = (uint32_t)__popcll(c);
        }
        __syncthreads();
        // the watch list's appends and the counter atomic are in flight together
        if (!WATCH && wl) list_append(Lw, wtrans, t, row, h);   // kernel argument: uniform
        if (threadIdx.x == 0) {
            const bool last = pass + 1 == lp1;
            unsigned long long s0 = 0, s1 = 0;
#pragma unroll
            for (uint32_t q = 0; q < kListWaves; ++q) s0 += wcnt[0][q], s1 += wcnt[1][q];
            const uint32_t cb = ev.cbits;
            const unsigned long long add = s0 | (s1 << cb) | (last ? 1ull << (2 * cb) : 0ull);
#if RH_TABLE_ABL == 8 || RH_TABLE_ABL == 9   // ablation (wrong results): no counter atomic, no records
            const unsigned long long old = 0ull;
            if (blockIdx.x == 0) publish_counts(ev, 0ull);
            if (false) {
#else
            const unsigned long long old = add ? atomicAdd(ev.cnt, add) : 0ull;
            lbase = old;
            if (last && ((old + add) >> (2 * cb)) == active) {   // every workgroup holding entries has counted
#endif
                publish_counts(ev, old + add);
                atomicExch(ev.cnt, 0ull);   // the next evaluation's counter
            }
        }
        __syncthreads();
        const unsigned long long cm = (1ull << ev.cbits) - 1;
        uint32_t b0 = (uint32_t)(lbase & cm), b1 = (uint32_t)((lbase >> ev.cbits) & cm);
        for (int q = 0; q < wave; ++q) b0 += wcnt[0][q], b1 += wcnt[1][q];
        if (pass + 1 < np) __syncthreads();   // wcnt / lbase are the next pass's (np: uniform)
#if RH_TABLE_ABL == 8 || RH_TABLE_ABL == 9
        continue;
#endif
        if (e0) {
            const uint64_t kk = b0 + (uint64_t)__popcll(a & lt);
            if (kk < R) {
                if (WATCH)
                    ev.watch[kk] = rh_watch_event{slot, valid, x0, x1, x2};
                else
                    ev.adv[kk] = rh_index_event{slot, 0u, x0};
            }
        }
        if (!WATCH && e1) {
            const uint64_t kk = b1 + (uint64_t)__popcll(c & lt);
            if (kk < R) ev.wall[kk] = rh_index_event{slot, 0u, x1};
        }
    }
    if (region) zero_list_desc(ev, np);
}

// ---- the pump's tick in one launch (rh_tick_async) --------------------------------------------------
// updateCommit over the commit list, then commitIndexChanged of every row whose levels may have moved
// -- the watch list's rows (a follower commitIndex delta) and the rows whose commit advanced -- in the
// same launch: a row's commitIndexChanged reads only that row (its followers' commitIndex, its new
// commit index, its levels), so the lane that evaluated its updateCommit evaluates it right after,
// from the same load batch (LeaderStateImpl.java:946-950, then 612-622, per division).  A wave serves
// one list: the commit list's waves and the watch list's run side by side.  Each row's
// commitIndexChanged runs exactly once, after its updateCommit.  The two flags are touched only by
// atomics here (performed at the device's coherence point: no fence, no cross-XCD staleness): a
// commit-list lane claims the row by clearing its watch flag (or by its commit having advanced), waits
// for that atomic to return, then clears the row's updateCommit flag; a watch-list lane reads the
// updateCommit flag with an atomic and claims only a row whose flag it finds clear -- so a commit-list
// lane has claimed it already (the claim fails) or the row is not in the commit list (the claim
// succeeds once).  A watch-list lane evaluates only rows whose commit index this launch does not write
// (its loads go out with the flag fetch and are used only then).  Records go straight into the pinned
// lists (one counter atomic per list kind per workgroup and pass); the last workgroup to finish
// publishes both lists' lengths and zeroes the counters.

// Clears byte `f` of its 32-bit word with one atomic; whether it was set.
__device__ __forceinline__ bool claim_flag(uint8_t* f) {
    uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(f) & ~(uintptr_t)3);
    const uint32_t sh = 8u * (uint32_t)(reinterpret_cast<uintptr_t>(f) & 3);
    return ((atomicAnd(w, ~(0xFFu << sh)) >> sh) & 0xFFu) != 0u;
}

// Byte `f` as the device's coherence point holds it (a returning atomic that changes nothing).
__device__ __forceinline__ uint8_t fetch_flag(uint8_t* f) {
    uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(f) & ~(uintptr_t)3);
    const uint32_t sh = 8u * (uint32_t)(reinterpret_cast<uintptr_t>(f) & 3);
    return (uint8_t)(atomicOr(w, 0u) >> sh);
}

// A commit-list row of the tick: every load of both evaluations and the claim of its watch flag
// issued together, then updateCommit (list_row<F, false>'s arithmetic), then -- claimed, or its
// commit advanced -- commitIndexChanged from the same registers with the new commit index as the
// self value (list_row<F, true>'s), so the second evaluation costs no second trip to the row.
template <int F>
__device__ __forceinline__ void tick_row(const TableDev& T, const TableTier& tt, uint32_t r, bool wall_on, bool& claimed,
                                         bool& e0, bool& e1, int64_t& x0, int64_t& x1, bool& ew, int64_t& y0,
                                         int64_t& y1, int64_t& y2, uint32_t& wvalid, uint32_t& slot) {
    int64_t m[F + 1], c[F + 1];
    const uint32_t w = *tt.u32(tile::kConf, r);
    slot = *tt.u32(tile::kSlot, r);
    const int64_t cm = *tt.i64(tile::commit(F), r);
#pragma unroll
    for (int k = 0; k < F; ++k) {
        m[k] = *tt.i64(tile::match(k), r);
        c[k] = *tt.i64(tile::fcommit(F, k), r);
    }
    const int64_t self = *tt.i64(tile::flush(F), r), ts = *tt.i64(tile::tstart(F), r);
    const int64_t p0 = wall_on ? *tt.i64(tile::wall(F), r) : 0;
    const int64_t q0 = *tt.i64(tile::wmin(F), r), q1 = *tt.i64(tile::wmaj(F), r), q2 = *tt.i64(tile::wmax(F), r);
    claimed = claim_flag(tt.u8(tile::kWdirty, r));
    const bool trans = (w & RH_CONF_ACTIVE) && (w & RH_CONF_TRANSITIONAL);
    bool v;
    int64_t mn, mj, mx, nc;
    m[F] = self;
    rh_eval::eval_group<F, (F <= 6)>(m, w, T.gap, trans, v, mn, mj, mx);
    e0 = rh_eval::commit_decision(v, mj, cm, self, ts, nc);
    e1 = wall_on && mn != p0;  // watch-ALL level changed (LSI:1025)
    x0 = nc, x1 = mn;
    if (e0) *tt.i64(tile::commit(F), r) = nc;
    if (e1) *tt.i64(tile::wall(F), r) = mn;
    if (claimed || e0) {   // commitIndexChanged: lastCommittedIndex (now nc if it advanced) is the self value (LSI:613)
        c[F] = e0 ? nc : cm;
        rh_eval::eval_group<F, (F <= 6)>(c, w, -1, trans, v, mn, mj, mx);
        wvalid = v ? 1u : 0u;
        ew = mn != q0 || mj != q1 || mx != q2;
        y0 = mn, y1 = mj, y2 = mx;
        if (ew) {
            *tt.i64(tile::wmin(F), r) = mn;
            *tt.i64(tile::wmaj(F), r) = mj;
            *tt.i64(tile::wmax(F), r) = mx;
        }
    }
}

// A watch-list row of the tick: its loads issued with the atomic fetch of its updateCommit flag, then
// -- the flag clear and the watch flag claimed -- commitIndexChanged (list_row<F, true>'s arithmetic).
template <int F>
__device__ __forceinline__ void tick_watch_row(const TableTier& tt, uint32_t r, bool& ew, int64_t& y0, int64_t& y1,
                                               int64_t& y2, uint32_t& wvalid, uint32_t& slot) {
    int64_t c[F + 1];
    const uint32_t w = *tt.u32(tile::kConf, r);
    slot = *tt.u32(tile::kSlot, r);
    c[F] = *tt.i64(tile::commit(F), r);   // lastCommittedIndex is the self value (LSI:613)
#pragma unroll
    for (int k = 0; k < F; ++k) c[k] = *tt.i64(tile::fcommit(F, k), r);
    const int64_t q0 = *tt.i64(tile::wmin(F), r), q1 = *tt.i64(tile::wmaj(F), r), q2 = *tt.i64(tile::wmax(F), r);
    if (fetch_flag(tt.u8(tile::kDirty, r)) != 0 || !claim_flag(tt.u8(tile::kWdirty, r))) return;
    const bool trans = (w & RH_CONF_ACTIVE) && (w & RH_CONF_TRANSITIONAL);
    bool v;
    int64_t mn, mj, mx;
    rh_eval::eval_group<F, (F <= 6)>(c, w, -1, trans, v, mn, mj, mx);
    wvalid = v ? 1u : 0u;
    ew = mn != q0 || mj != q1 || mx != q2;
    y0 = mn, y1 = mj, y2 = mx;
    if (ew) {
        *tt.i64(tile::wmin(F), r) = mn;
        *tt.i64(tile::wmaj(F), r) = mj;
        *tt.i64(tile::wmax(F), r) = mx;
    }
}

__device__ __forceinline__ void tick_watch_row_any(const TableTier& tt, uint32_t r, bool& ew, int64_t& y0, int64_t& y1,
                                                   int64_t& y2, uint32_t& wvalid, uint32_t& slot) {
    switch (tt.width) {
        case 2: tick_watch_row<2>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
        case 4: tick_watch_row<4>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
        case 6: tick_watch_row<6>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
        case 8: tick_watch_row<8>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
        case 10: tick_watch_row<10>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
        case 12: tick_watch_row<12>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
        default: tick_watch_row<14>(tt, r, ew, y0, y1, y2, wvalid, slot); break;
    }
}

__device__ __forceinline__ void tick_row_any(const TableDev& T, const TableTier& tt, uint32_t r, bool wall_on,
                                             bool& claimed, bool& e0, bool& e1, int64_t& x0, int64_t& x1, bool& ew,
                                             int64_t& y0, int64_t& y1, int64_t& y2, uint32_t& wvalid, uint32_t& slot) {
    switch (tt.width) {
        case 2: tick_row<2>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
        case 4: tick_row<4>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
        case 6: tick_row<6>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
        case 8: tick_row<8>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
        case 10: tick_row<10>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
        case 12: tick_row<12>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
        default: tick_row<14>(T, tt, r, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot); break;
    }
}


__global__ __launch_bounds__(kListWaves * 64) void table_tick_kernel(TableDev Targ, TableLists Lc, TableLists Lw,
                                                                     rh::TickEvents ev) {
    const TableDev& T = rh::kernarg_struct<TableDev>();
    (void)Targ;
    constexpr uint32_t NR = rh::kHeads;
    __shared__ __attribute__((aligned(16))) unsigned char tiers_mem[sizeof(TableTier) * rh::kTableTiers];
    TableTier* tiers = reinterpret_cast<TableTier*>(tiers_mem);
    __shared__ uint32_t wcnt[3][kListWaves];   // per pass: the waves' advanced / watch-ALL / level records
    __shared__ unsigned long long bc, bw;      // per pass: the workgroup's ranges of the lists
    __shared__ uint32_t book[2];               // passes over the commit list, over the watch list
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * kListWaves, wg = blockIdx.x * kListWaves + (uint32_t)wave;
    const uint32_t r = wg % NR, k = wg / NR, Wr = (W - r + NR - 1) / NR;
    // a wave serves one list (wave-uniform: the two row chains run on different waves, side by side):
    // the region's even ranks its commit list, the odd ranks its watch list (the host's grid gives
    // every region at least two waves)
    const uint32_t role = k & 1u, kr = k >> 1, Wrr = role ? Wr / 2 : (Wr + 1) / 2;
    const TableLists& L = role ? Lw : Lc;
    const unsigned long long hl = L.heads[(uint64_t)r * rh::kHeadStride];
    // the first pass's entry loaded with the count (speculatively: below the capacity it is in bounds)
    const uint32_t i0 = (uint32_t)lane * Wrr + kr;
    const uint32_t ent0 = i0 < L.cap ? L.rows[(uint64_t)r * L.cap + i0] : 0u;
    uint32_t cl = 0;
    if (wave == 0 && lane < (int)(2 * NR)) {   // lanes 0..7: the commit list's regions, 8..15: the watch list's
        const TableLists& Lq = lane < (int)NR ? Lc : Lw;
        const unsigned long long x = Lq.heads[(uint64_t)(lane % NR) * rh::kHeadStride];
        cl = (uint32_t)(x < Lq.cap ? x : Lq.cap);
    }
    if (threadIdx.x == 64) {
#pragma unroll
        for (int q = 0; q < rh::kTableTiers; ++q) tiers[q] = T.tier[q];   // uniform index: scalar loads
    }
    if (blockIdx.x == 0 && threadIdx.x < NR) {   // the next list sets of both kinds
        ev.lheads_next_c[(uint64_t)threadIdx.x * rh::kHeadStride] = 0ull;
        ev.lheads_next_w[(uint64_t)threadIdx.x * rh::kHeadStride] = 0ull;
    }
    const uint32_t cnt = (uint32_t)(hl < L.cap ? hl : L.cap);
    if (wave == 0) {
        uint32_t np = 0;
        if (lane < (int)(2 * NR)) {
            const uint32_t rr = (uint32_t)lane % NR, wr = (W - rr + NR - 1) / NR;
            const uint32_t wrr = lane < (int)NR ? (wr + 1) / 2 : wr / 2;
            np = (cl + wrr * 64u - 1) / (wrr * 64u);
        }
        const uint32_t npc = wave_max_u32(lane < (int)NR ? np : 0u), npw = wave_max_u32(lane >= (int)NR ? np : 0u);
        if (lane == 0) {
            book[0] = npc;
            book[1] = npw;
        }
    }
    __syncthreads();
    const uint32_t np_c = book[0], np_w = book[1];
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const bool wall_on = ev.wall != nullptr;
    const uint64_t R = ev.cap;
    const uint32_t np = np_c > np_w ? np_c : np_w;   // uniform over the workgroup (its barriers)
    for (uint32_t pass = 0; pass < np; ++pass) {
        const uint32_t idx = (pass * 64u + (uint32_t)lane) * Wrr + kr;
        bool e0 = false, e1 = false, ew = false;
        int64_t x0 = 0, x1 = 0, y0 = 0, y1 = 0, y2 = 0;
        uint32_t slot = 0, wvalid = 0;
        if (idx < cnt) {
            const uint32_t ent = pass == 0 ? ent0 : L.rows[(uint64_t)r * L.cap + idx];
            const uint32_t t = ent >> 28, row = ent & rh::kRowMask;
            const TableTier tt = tiers[t < (uint32_t)rh::kTableTiers ? t : 0u];
            if (row < tt.rows) {
                if (role == 0) {   // updateCommit, then (watch flag claimed, or advanced) commitIndexChanged
                    bool claimed = false;
                    tick_row_any(T, tt, row, wall_on, claimed, e0, e1, x0, x1, ew, y0, y1, y2, wvalid, slot);
                    // the claim performed (returned: its value in a register) before the updateCommit flag
                    // clears -- the watch side reads it; no memory access moves across
                    asm volatile("" ::"v"((uint32_t)claimed) : "memory");
                    (void)claim_flag(tt.u8(tile::kDirty, row));
                } else {   // commitIndexChanged, if no commit-list lane holds the row
                    tick_watch_row_any(tt, row, ew, y0, y1, y2, wvalid, slot);
                }
            }
        }
        const uint64_t a = __ballot(e0), c = __ballot(e1), w = __ballot(ew);
        if (lane == 0) {
            wcnt[0][wave] = (uint32_t)__popcll(a);
            wcnt[1][wave] = (uint32_t)__popcll(c);
            wcnt[2][wave] = (uint32_t)__popcll(w);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
            for (uint32_t q = 0; q < kListWaves; ++q) s0 += wcnt[0][q], s1 += wcnt[1][q], s2 += wcnt[2][q];
            bc = (s0 | s1) ? atomicAdd(ev.cnt, s0 | (s1 << 32)) : 0ull;
            bw = s2 ? atomicAdd(ev.cnt + rh::kHeadStride, s2) : 0ull;
        }
        __syncthreads();
        uint64_t b0 = bc & 0xFFFFFFFFull, b1 = bc >> 32, b2 = bw;
        for (int q = 0; q < wave; ++q) b0 += wcnt[0][q], b1 += wcnt[1][q], b2 += wcnt[2][q];
        __syncthreads();   // wcnt / bc / bw are the next pass's
        if (e0) {
            const uint64_t kk = b0 + (uint64_t)__popcll(a & lt);
            if (kk < R) ev.adv[kk] = rh_index_event{slot, 0u, x0};
        }
        if (e1) {
            const uint64_t kk = b1 + (uint64_t)__popcll(c & lt);
            if (kk < R) ev.wall[kk] = rh_index_event{slot, 0u, x1};
        }
        if (ew) {
            const uint64_t kk = b2 + (uint64_t)__popcll(w & lt);
            if (kk < R) ev.watch[kk] = rh_watch_event{slot, wvalid, y0, y1, y2};
        }
    }
    // the last workgroup to finish publishes both lists' lengths and zeroes the counters (every other
    // workgroup's counter atomics returned before its done atomic was issued)
    if (threadIdx.x == 0) {
        const unsigned int prev = atomicAdd(reinterpret_cast<unsigned int*>(ev.cnt + 2 * rh::kHeadStride), 1u);
        if (prev + 1u == gridDim.x) {
            const unsigned long long c = atomicExch(ev.cnt, 0ull), w = atomicExch(ev.cnt + rh::kHeadStride, 0ull);
            atomicExch(reinterpret_cast<unsigned int*>(ev.cnt + 2 * rh::kHeadStride), 0u);
            ev.counts_c[0] = c & 0xFFFFFFFFull;
            ev.counts_c[1] = c >> 32;
            ev.counts_w[0] = w;
            ev.counts_w[1] = 0;
        }
    }
}

// ---- hasLease over every started row -------------------------------------------------------------
#ifndef RH_LEASE_BITS_WAVE   // A/B: the hasLease bitmap set per wave (1) or per row (0)
#define RH_LEASE_BITS_WAVE 1
#endif
template <int F>
__global__ __launch_bounds__(256) void table_lease_kernel(TableTier tt, int64_t now, int64_t timeout_ms,
                                                          uint64_t* __restrict__ slot_bits,
                                                          uint64_t* __restrict__ clear, uint32_t clear_words) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the other bitmap, the next pass's, cleared here (no memset launch of its own)
    for (uint64_t j = r; j < clear_words; j += (uint64_t)gridDim.x * blockDim.x) clear[j] = 0ull;
    bool has = false;
    uint32_t slot = 0;
    if (r < tt.rows) {   // no early return: the bitmap words are set wave-wide below
        const uint32_t w = *tt.u32(tile::kConf, r);
        if (w & RH_CONF_ACTIVE) {   // a started row
            int64_t ts[F];
            uint32_t never = 0;
#pragma unroll
            for (int k = 0; k < F; ++k) {
                ts[k] = *tt.i64(tile::fts(F, k), r);
                never |= (ts[k] == rh::kNoTimestamp ? 1u : 0u) << k;
            }
            rh_lease_soa t{};
            t.now_nanos = now;
            t.timeout_ms = timeout_ms;
            int64_t lout;
            bool ext;
            int64_t* lease = tt.i64(tile::lease(F), r);
            rh_lease::lease_one<F>(t, ts, w, *lease, *tt.u8(tile::kLon, r) != 0, true, lout, has, ext, never);
            if (ext) *lease = lout;
            if (has) slot = *tt.u32(tile::kSlot, r);
        }
    }
#if RH_LEASE_BITS_WAVE
    // the wave's rows usually hold consecutive slots (a load or a start fills rows in slot order):
    // lanes whose bit lands in the first pending lane's word OR their bits together and one lane
    // sets the word -- one atomic per word instead of one per row (64 same-address atomics a wave)
    const int lane = threadIdx.x & 63;
    uint64_t pend = __ballot(has);
    for (int round = 0; pend && round < 2; ++round) {
        const int lead = __ffsll((long long)pend) - 1;
        const uint32_t word = (uint32_t)__shfl((int)(slot >> 6), lead);
        const bool mine = has && (slot >> 6) == word && ((pend >> lane) & 1ull);
        uint64_t v = mine ? 1ull << (slot & 63) : 0ull;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) v |= __shfl_xor(v, d);
        if (lane == lead) atomicOr(reinterpret_cast<unsigned long long*>(slot_bits + word), v);
        pend &= ~__ballot(mine);
    }
    if (has && ((pend >> lane) & 1ull))   // slots spread wider: one atomic per row
        atomicOr(reinterpret_cast<unsigned long long*>(slot_bits + (slot >> 6)), 1ull << (slot & 63));
#else
    if (has) atomicOr(reinterpret_cast<unsigned long long*>(slot_bits + (slot >> 6)), 1ull << (slot & 63));
#endif
}

template <int F>
void launch_lease_width(const TableTier& tt, int64_t now, int64_t timeout_ms, uint64_t* bits, uint64_t* clear,
                        uint32_t clear_words, hipStream_t s) {
    hipLaunchKernelGGL((table_lease_kernel<F>), dim3((tt.rows + 255) / 256), dim3(256), 0, s, tt, now, timeout_ms, bits,
                       clear, clear_words);
}

// ---- read-back -------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void table_read_kernel(TableDev Targ, uint32_t first, uint32_t n, uint32_t column,
                                                         int64_t* __restrict__ out) {
    const TableDev& T = rh::kernarg_struct<TableDev>();
    (void)Targ;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const TableTier* tt;
    uint32_t row;
    int64_t v = INT64_MIN;
    if (locate(T, first + i, tt, row)) {
        const uint32_t F = tt->width;
        if (column < 16) v = column < F ? *tt->i64(tile::match(column), row) : -1;
        else if (column < 32) v = column - 16 < F ? *tt->i64(tile::fcommit(F, column - 16), row) : -1;
        else if (column == RH_COL_FLUSH) v = *tt->i64(tile::flush(F), row);
        else if (column == RH_COL_COMMITTED) v = *tt->i64(tile::commit(F), row);
        else if (column == RH_COL_CONF) v = (int64_t)*tt->u32(tile::kConf, row);
        else if (column == RH_COL_TERM_START) v = *tt->i64(tile::tstart(F), row);
        else if (column == RH_COL_LEASE) v = *tt->i64(tile::lease(F), row);
        else if (column == RH_COL_LEASE_ON) v = (int64_t)*tt->u8(tile::kLon, row);
        else if (column >= 48 && column < 64) v = column - 48 < F ? *tt->i64(tile::fts(F, column - 48), row) : rh::kNoTimestamp;
    }
    out[i] = v;
}

}  // namespace

int rh_table_apply_deltas(const rh::TableDev& t, const rh_delta* d_deltas, uint64_t n, int phase, uint32_t gen,
                          const rh::TableLists& lc, const rh::TableLists& lw, hipStream_t stream, bool resolved) {
    if (n == 0) return RH_OK;
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(table_apply_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, t, d_deltas, n, phase, gen, lc,
                       lw, resolved ? 1 : 0);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_table_control(const rh::TableDev& t, const rh::CtrlOp* d_ops, uint64_t n, hipStream_t stream) {
    if (n == 0) return RH_OK;
    hipLaunchKernelGGL(table_control_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, t, d_ops, n);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

static uint32_t class_blocks(const rh::TableDev& t, int cls) {
    uint32_t blocks = 0;
    for (int i = 0; i < rh::kTableTiers; ++i)
        if ((cls == 0 ? i <= 2 : i >= 3) && t.tier[i].rows) blocks += (t.tier[i].rows + kTRows - 1) / kTRows;
    return blocks;
}

uint32_t rh::table_commit_blocks(const rh::TableDev& t) { return class_blocks(t, 0) + class_blocks(t, 1); }

// The block -> tier map of width class cls's evaluation launch (widest tier first); its blocks.
static uint32_t tier_range(const rh::TableDev& t, int cls, TierRange& tr) {
    tr = TierRange{};
    uint32_t blocks = 0;
    for (int i = rh::kTableTiers - 1; i >= 0; --i) {
        const bool in_cls = cls == 0 ? i <= 2 : i >= 3;
        if (!in_cls || !t.tier[i].rows) continue;
        tr.block_begin[tr.n_slots] = blocks;
        tr.tier[tr.n_slots++] = (int8_t)i;
        blocks += (t.tier[i].rows + kTRows - 1) / kTRows;
    }
    for (int s = tr.n_slots; s <= rh::kTableTiers; ++s) tr.block_begin[s] = blocks;
    return blocks;
}

// Evaluation launches.  With timing events (rh_groups_timing) hipExtLaunchKernel stamps them at
// the dispatch's own start and completion (the kernel boundaries rocprof reports), not as separate
// stream packets around it: t0 on the evaluation's first launch, t1 on its last.
template <typename K, typename... A>
hipError_t eval_launch(K kernel, dim3 g, dim3 b, hipStream_t stream, hipEvent_t t0, hipEvent_t t1, A... args) {
    if (t0 || t1) hipExtLaunchKernelGGL(kernel, g, b, 0, stream, t0, t1, 0u, args...);
    else hipLaunchKernelGGL(kernel, g, b, 0, stream, args...);
    return hipGetLastError();
}

int rh_table_commit(const rh::TableDev& t, int mode, const rh::TableEvents& ev_in, bool spec, hipStream_t stream,
                    hipEvent_t t0, hipEvent_t t1) {
    // one launch per width class over every non-empty tier of the class, widest tier first (a
    // joint-consensus tier's rows cost several times a stable row's compute: dispatched last they
    // were the launch's tail, commit.hip build_args)
    rh::TableEvents ev = ev_in;
    const int first_cls = class_blocks(t, 0) ? 0 : 1;
    const int last_cls = class_blocks(t, 1) ? 1 : 0;   // its launch publishes the list lengths
    const uint32_t total = rh::table_commit_blocks(t);
    // the done count rides in the counter word when the evaluation's workgroups fit above the counts
    ev.packed = 2 * ev.cbits < 64 && (uint64_t)total < (1ull << (64 - 2 * ev.cbits)) ? 1 : 0;
    for (int cls = 0; cls < 2; ++cls) {
        TierRange tr{};
        const uint32_t blocks = tier_range(t, cls, tr);
        if (blocks == 0) continue;
        ev.done_target = cls == last_cls ? total : 0u;   // workgroups of both launches count
        ev.block_base = cls == 0 ? 0u : class_blocks(t, 0);   // REGION mode: workgroup numbering
        const dim3 g(blocks), b(kTBlock);
        const hipEvent_t a0 = cls == first_cls ? t0 : nullptr, a1 = cls == last_cls ? t1 : nullptr;
        hipError_t e;
        if (mode == RH_MODE_WATCH) {
            if (cls == 0 && spec) e = eval_launch(table_commit_kernel_rank<true, true>, g, b, stream, a0, a1, t, tr, ev);
            else if (cls == 0) e = eval_launch(table_commit_kernel_rank<true, false>, g, b, stream, a0, a1, t, tr, ev);
            else if (spec) e = eval_launch(table_commit_kernel_net<true, true>, g, b, stream, a0, a1, t, tr, ev);
            else e = eval_launch(table_commit_kernel_net<true, false>, g, b, stream, a0, a1, t, tr, ev);
        } else {
            if (cls == 0 && spec) e = eval_launch(table_commit_kernel_rank<false, true>, g, b, stream, a0, a1, t, tr, ev);
            else if (cls == 0) e = eval_launch(table_commit_kernel_rank<false, false>, g, b, stream, a0, a1, t, tr, ev);
            else if (spec) e = eval_launch(table_commit_kernel_net<false, true>, g, b, stream, a0, a1, t, tr, ev);
            else e = eval_launch(table_commit_kernel_net<false, false>, g, b, stream, a0, a1, t, tr, ev);
        }
        RH_HIP(e);
    }
    return RH_OK;
}

// List grid by the marked rows (an upper bound of the listed ones): about kListRowsPerWave rows per
// wave, between kListMinGrid and kListMaxGrid workgroups (same box, 1M rows: 240 waves 9.5-10.0 us
// at 1 %, 7.9-8.0 at 0.3 %, but 17.5-18.5 at 3 %, where 480 waves take 14.0-15.1;
// profiles/r05/table_eval/)
#ifndef RH_LIST_ROWS_PER_WAVE
#define RH_LIST_ROWS_PER_WAVE 48
#endif
#ifndef RH_LIST_MIN_GRID
#define RH_LIST_MIN_GRID (kListMaxGrid / 2)
#endif
constexpr uint32_t kListMinGrid = RH_LIST_MIN_GRID;
static_assert(kListMinGrid >= rh::kHeads, "a workgroup per list region at least");

uint32_t rh::table_list_grid(uint64_t rows_hint) {
    const uint64_t want = (rows_hint + (uint64_t)RH_LIST_ROWS_PER_WAVE * kListWaves - 1) / ((uint64_t)RH_LIST_ROWS_PER_WAVE * kListWaves);
    return (uint32_t)std::min<uint64_t>(kListMaxGrid, std::max<uint64_t>(kListMinGrid, want));
}

// A region r's entries are dealt over its Wr = (W - r + 7) / 8 >= W / 8 waves, 64 per wave and pass.
uint32_t rh::table_list_passes(uint32_t grid, uint64_t rows) {
    const uint64_t per_pass = 64ull * ((uint64_t)grid * kListWaves / rh::kHeads);
    return (uint32_t)((rows + per_pass - 1) / per_pass);
}

uint64_t rh::table_list_desc_blocks(uint64_t cap) {
    uint64_t most = 0;
    for (uint32_t g = kListMinGrid; g <= kListMaxGrid; ++g) most = std::max<uint64_t>(most, (uint64_t)g * table_list_passes(g, cap));
    return most;
}

int rh_table_commit_lists(const rh::TableDev& t, int mode, const rh::TableLists& l, const rh::TableLists& lw,
                          const rh::TableEvents& ev_in, hipStream_t stream, hipEvent_t t0, hipEvent_t t1,
                          uint64_t rows_hint) {
    // the listed rows are dealt lane-major over every wave of a near-chip-wide grid: a few rows per
    // wave on ~every CU (random rows: the chain of dependent loads is latency-bound per CU, so the
    // rows are spread, not packed into few waves)
    const dim3 g(rh::table_list_grid(rows_hint)), b(kListWaves * 64);
    rh::TableEvents ev = ev_in;
    hipError_t e;
    if (mode == RH_MODE_WATCH)
        e = eval_launch(table_list_kernel<true>, g, b, stream, t0, t1, t, l, rh::TableLists{}, ev);
    else
        e = eval_launch(table_list_kernel<false>, g, b, stream, t0, t1, t, l, lw, ev);
    RH_HIP(e);
    return RH_OK;
}

int rh_table_tick_lists(const rh::TableDev& t, const rh::TableLists& lc, const rh::TableLists& lw, const rh::TickEvents& ev,
                        hipStream_t stream, hipEvent_t t0, hipEvent_t t1, uint64_t rows_hint) {
    // every region at least two waves: one per list (table_tick_kernel's roles)
    const dim3 g(std::max<uint32_t>(rh::table_list_grid(rows_hint), 2 * rh::kHeads / kListWaves)), b(kListWaves * 64);
    RH_HIP(eval_launch(table_tick_kernel, g, b, stream, t0, t1, t, lc, lw, ev));
    return RH_OK;
}

// ---- AUTO sink: a tile evaluation's HBM lists drained into the pinned lists ------------------------
// On its own stream after the evaluation: the counted prefixes (lengths from the host-mapped counts
// the evaluation published) move across PCIe as GPU writes, 16 B per thread and step, while the table
// stream goes on (the next deltas' apply, the next evaluation) and no host thread issues a copy.
__global__ __launch_bounds__(256) void table_drain_kernel(const uint64_t* __restrict__ counts, const uint4* __restrict__ a,
                                                          uint4* __restrict__ a_out, const uint4* __restrict__ b,
                                                          uint4* __restrict__ b_out, uint32_t words0, uint64_t cap) {
    const uint64_t n0 = (counts[0] < cap ? counts[0] : cap) * words0;
    const uint64_t n1 = b ? (counts[1] < cap ? counts[1] : cap) : 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n0 + n1; j += stride) {
        if (j < n0) a_out[j] = a[j];
        else b_out[j - n0] = b[j - n0];
    }
}

__global__ __launch_bounds__(256) void table_copy_words_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                               uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n2 = n / 2;   // 16 bytes per thread and step (both pointers 16-byte aligned)
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n2; j += stride)
        reinterpret_cast<uint4*>(dst)[j] = reinterpret_cast<const uint4*>(src)[j];
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) dst[n - 1] = src[n - 1];
}

int rh_table_copy_words(const uint64_t* src, uint64_t* dst, uint64_t n, hipStream_t stream) {
    if (n == 0) return RH_OK;
    if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15)
        return rh::fail(RH_E_STATE, "rh_table_copy_words: buffers not 16-byte aligned");
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(64, (n / 2 + 255) / 256 + 1);
    hipLaunchKernelGGL(table_copy_words_kernel, dim3(blocks), dim3(256), 0, stream, src, dst, n);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_table_drain(const uint64_t* counts, const void* a, void* a_out, const void* b, void* b_out, uint32_t rec_bytes0,
                   uint64_t cap, hipStream_t stream) {
    hipLaunchKernelGGL(table_drain_kernel, dim3(512), dim3(256), 0, stream, counts, static_cast<const uint4*>(a),
                       static_cast<uint4*>(a_out), static_cast<const uint4*>(b), static_cast<uint4*>(b_out),
                       rec_bytes0 / 16u, cap);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

// ---- REGION mode gathers: one gather workgroup per kGatherWGs evaluation workgroups ----------------
#ifndef RH_GATHER_CHUNKS   // evaluation waves (chunks) per gather workgroup of 4 waves: one per wave (round 6:
                           // 10 % dirty 34.7 -> 23.2 us, 100 % 128.4 -> 126.2 us; profiles/r06/gather_ab/)
#define RH_GATHER_CHUNKS 4
#endif
constexpr uint32_t kGatherWGs = kTWaves >= RH_GATHER_CHUNKS ? 1u : RH_GATHER_CHUNKS / kTWaves;
constexpr uint32_t kGatherChunks = kGatherWGs * kTWaves;


// ---- REGION mode: the records rebuilt from the masks and the table ---------------------------------
// One gather workgroup per kGatherWGs evaluation workgroups: its offsets in the packed lists are
// the sums of the totals before its first evaluation workgroup (summed by the 256 threads, reduced
// in LDS), its parts' counts -- popcounts of the masks -- scanned in LDS; then each wave takes
// parts round robin: the part's tile (its launch, tier slot and tile, as the evaluation's block
// map), lane L the rows 2L, 2L + 1: their row slots and the values the evaluation stored -- one
// coalesced load per column per wave -- written in row order.  updateCommit: list a = advanced
// (the commit column), list b = changed watch-ALL levels (the watch-ALL column).  commitIndexChanged:
// list a = changed levels (wmin / wmaj / wmax) with the valid flag from the mask's second pair.
struct GatherRowsArgs {
    TableDev t;             // the evaluation's (clipped) table
    TierRange tr[2];        // its launches' block -> tier maps
    uint32_t cls1_base;     // the second launch's first workgroup number
    uint32_t n_blocks;
    const uint64_t* desc;   // per workgroup: totals (a | b << 32), per wave 4 masks
    void* a;                // rh_index_event (updateCommit) / rh_watch_event (commitIndexChanged) list
    rh_index_event* b;      // updateCommit's watch-ALL list (null: none)
    uint64_t* counts_out;
    rh::ListRegion lr;      // a list evaluation's (rows null: a tile evaluation)
};

template <bool WATCH>
__global__ __launch_bounds__(256) void table_gather_rows_kernel(GatherRowsArgs arg) {
    (void)arg;
    const GatherRowsArgs& A = rh::kernarg_struct<GatherRowsArgs>();
    constexpr uint32_t S = rh::kTableDesc / 2;   // u64 per descriptor
    __shared__ unsigned long long red[2][256 / 64];
    __shared__ uint32_t pre[2][kGatherChunks + 1];
    const bool has_b = !WATCH && A.b != nullptr;
    const uint32_t first = blockIdx.x * kGatherWGs;
    const uint32_t upto = blockIdx.x == 0 ? A.n_blocks : first;   // gather workgroup 0 sums them all
    unsigned long long s0 = 0, s1 = 0;
    for (uint32_t j = threadIdx.x; j < upto; j += blockDim.x) {
        const uint64_t v = A.desc[(uint64_t)j * S];
        s0 += (uint32_t)v;
        s1 += v >> 32;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_down(s0, o);
        s1 += __shfl_down(s1, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = s0;
        red[1][threadIdx.x >> 6] = s1;
    }
    for (uint32_t c = threadIdx.x; c < kGatherChunks; c += blockDim.x) {   // the parts' counts
        const uint32_t gb = first + c / kTWaves, w = c % kTWaves;
        uint32_t n0 = 0, n1 = 0;
        if (gb < A.n_blocks) {
            const uint64_t* m = A.desc + (uint64_t)gb * S + 1 + 4 * w;
            n0 = (uint32_t)(__popcll(m[0]) + __popcll(m[1]));
            n1 = has_b ? (uint32_t)(__popcll(m[2]) + __popcll(m[3])) : 0u;
        }
        pre[0][c + 1] = n0;
        pre[1][c + 1] = n1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {   // exclusive scan of one list's part counts
        uint32_t* p = pre[threadIdx.x];
        p[0] = 0;
        for (uint32_t c = 1; c <= kGatherChunks; ++c) p[c] += p[c - 1];
    }
    s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    uint64_t p0 = s0, p1 = s1;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            A.counts_out[0] = s0;
            A.counts_out[1] = has_b ? s1 : 0;
        }
        p0 = p1 = 0;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t c = wv; c < kGatherChunks; c += blockDim.x / 64) {
        const uint32_t gb = first + c / kTWaves, w = c % kTWaves;
        if (gb >= A.n_blocks) break;   // wave-uniform
        const uint64_t* m = A.desc + (uint64_t)gb * S + 1 + 4 * w;
        const uint64_t a0 = m[0], a1 = m[1], c0 = (WATCH || has_b) ? m[2] : 0ull, c1 = (WATCH || has_b) ? m[3] : 0ull;
        if (!(a0 | a1 | (WATCH ? 0ull : (c0 | c1)))) continue;
        if (A.lr.rows) {   // a list evaluation: lane j's listed row of that wave and pass (a1 = c1 = 0)
            const bool e0 = (a0 >> lane) & 1u, e1 = !WATCH && ((c0 >> lane) & 1u);
            if (!(e0 || e1)) continue;
            const uint32_t pass = gb / A.lr.grid, wg = (gb % A.lr.grid) * kListWaves + w;
            const uint32_t W = A.lr.grid * kListWaves, r = wg % rh::kHeads, k = wg / rh::kHeads;
            const uint32_t Wr = (W - r + rh::kHeads - 1) / rh::kHeads;
            const uint32_t ent = A.lr.rows[(uint64_t)r * A.lr.cap + (pass * 64u + lane) * Wr + k];
            const TableTier& tt = A.t.tier[(ent >> 28) < (uint32_t)rh::kTableTiers ? (ent >> 28) : 0u];
            const uint32_t row = ent & rh::kRowMask, F = tt.width;
            if (row >= tt.rows) continue;   // never: the entry was listed by this evaluation (no stray access)
            const uint32_t sl = *tt.u32(rh::tile::kSlot, row);
            if (WATCH) {
                rh_watch_event* out = static_cast<rh_watch_event*>(A.a);
                out[p0 + pre[0][c] + (uint64_t)__popcll(a0 & lt)] =
                    rh_watch_event{sl, (uint32_t)((c0 >> lane) & 1u), *tt.i64(rh::tile::wmin(F), row),
                                   *tt.i64(rh::tile::wmaj(F), row), *tt.i64(rh::tile::wmax(F), row)};
            } else {
                if (e0)
                    static_cast<rh_index_event*>(A.a)[p0 + pre[0][c] + (uint64_t)__popcll(a0 & lt)] =
                        rh_index_event{sl, 0u, *tt.i64(rh::tile::commit(F), row)};
                if (e1) A.b[p1 + pre[1][c] + (uint64_t)__popcll(c0 & lt)] = rh_index_event{sl, 0u, *tt.i64(rh::tile::wall(F), row)};
            }
            continue;
        }
        const int cls = gb < A.cls1_base ? 0 : 1;
        const uint32_t b = gb - (cls ? A.cls1_base : 0u);
        const TierRange& tr = A.tr[cls];
        int i = 0;
#pragma unroll
        for (int k = 1; k < rh::kTableTiers; ++k)
            if (k < tr.n_slots && b >= tr.block_begin[k]) i = k;
        const TableTier& tt = A.t.tier[tr.tier[i]];
        const uint64_t tl = (uint64_t)(b - tr.block_begin[i]) * kTWaves + w;
        const uint8_t* tb = tt.base + tl * rh::tile::bytes(tt.width);
        const uint32_t F = tt.width;
        const bool e00 = (a0 >> lane) & 1u, e01 = (a1 >> lane) & 1u;
        const bool e10 = !WATCH && ((c0 >> lane) & 1u), e11 = !WATCH && ((c1 >> lane) & 1u);
        if (!(e00 || e01 || e10 || e11)) continue;
        const uint2 sl = *reinterpret_cast<const uint2*>(tb + rh::tile::kSlot + 8u * lane);
        if (WATCH) {
            const int64_t* mn = reinterpret_cast<const int64_t*>(tb + rh::tile::pair_off(F, rh::tile::wmin(F), lane));
            const int64_t* mj = reinterpret_cast<const int64_t*>(tb + rh::tile::pair_off(F, rh::tile::wmaj(F), lane));
            const int64_t* mx = reinterpret_cast<const int64_t*>(tb + rh::tile::pair_off(F, rh::tile::wmax(F), lane));
            rh_watch_event* out = static_cast<rh_watch_event*>(A.a);
            uint64_t p = p0 + pre[0][c] + (uint64_t)(__popcll(a0 & lt) + __popcll(a1 & lt));
            if (e00) out[p++] = rh_watch_event{sl.x, (uint32_t)((c0 >> lane) & 1u), mn[0], mj[0], mx[0]};
            if (e01) out[p] = rh_watch_event{sl.y, (uint32_t)((c1 >> lane) & 1u), mn[1], mj[1], mx[1]};
        } else {
            if (e00 || e01) {
                const int64_t* cp = reinterpret_cast<const int64_t*>(tb + rh::tile::pair_off(F, rh::tile::commit(F), lane));
                rh_index_event* out = static_cast<rh_index_event*>(A.a);
                uint64_t p = p0 + pre[0][c] + (uint64_t)(__popcll(a0 & lt) + __popcll(a1 & lt));
                if (e00) out[p++] = rh_index_event{sl.x, 0u, cp[0]};
                if (e01) out[p] = rh_index_event{sl.y, 0u, cp[1]};
            }
            if (e10 || e11) {
                const int64_t* wp = reinterpret_cast<const int64_t*>(tb + rh::tile::pair_off(F, rh::tile::wall(F), lane));
                uint64_t q = p1 + pre[1][c] + (uint64_t)(__popcll(c0 & lt) + __popcll(c1 & lt));
                if (e10) A.b[q++] = rh_index_event{sl.x, 0u, wp[0]};
                if (e11) A.b[q] = rh_index_event{sl.y, 0u, wp[1]};
            }
        }
    }
}

static int gather_rows(bool watch, const rh::TableDev& t, const uint32_t* bdesc, uint32_t n_blocks, void* a,
                       rh_index_event* b, uint64_t* counts_out, hipStream_t stream, const rh::ListRegion& lr,
                       hipEvent_t t0, hipEvent_t t1) {
    if (n_blocks == 0) return rh::fail(RH_E_INVAL, "rh_table_gather_rows: no workgroups");
    GatherRowsArgs g{};
    g.t = t;
    g.lr = lr;
    if (lr.rows) {   // descriptors: passes x the list grid
        if (lr.grid == 0 || n_blocks % lr.grid) return rh::fail(RH_E_STATE, "rh_table_gather_rows: descriptors differ from the list grid's");
    } else {
        const uint32_t b0 = tier_range(t, 0, g.tr[0]), b1 = tier_range(t, 1, g.tr[1]);
        if (b0 + b1 != n_blocks) return rh::fail(RH_E_STATE, "rh_table_gather_rows: workgroups differ from the evaluation's");
        g.cls1_base = b0;
    }
    g.n_blocks = n_blocks;
    g.desc = reinterpret_cast<const uint64_t*>(bdesc);
    g.a = a;
    g.b = b;
    g.counts_out = counts_out;
    const dim3 grid((n_blocks + kGatherWGs - 1) / kGatherWGs), blk(256);
    hipError_t e;
    if (watch)
        e = eval_launch(table_gather_rows_kernel<true>, grid, blk, stream, t0, t1, g);
    else
        e = eval_launch(table_gather_rows_kernel<false>, grid, blk, stream, t0, t1, g);
    RH_HIP(e);
    return RH_OK;
}

int rh_table_gather_commit(const rh::TableDev& t, const uint32_t* bdesc, uint32_t n_blocks, rh_index_event* adv_out,
                           rh_index_event* wall_out, uint64_t* counts_out, hipStream_t stream, const rh::ListRegion& lr,
                           hipEvent_t t0, hipEvent_t t1) {
    return gather_rows(false, t, bdesc, n_blocks, adv_out, wall_out, counts_out, stream, lr, t0, t1);
}

int rh_table_gather_watch(const rh::TableDev& t, const uint32_t* bdesc, uint32_t n_blocks, rh_watch_event* out,
                          uint64_t* counts_out, hipStream_t stream, const rh::ListRegion& lr, hipEvent_t t0, hipEvent_t t1) {
    return gather_rows(true, t, bdesc, n_blocks, out, nullptr, counts_out, stream, lr, t0, t1);
}

int rh_table_init_tiles(const rh::TableTier& t, uint32_t first_tile, uint32_t n_tiles, hipStream_t stream) {
    if (n_tiles == 0) return RH_OK;
    hipLaunchKernelGGL(table_init_tiles_kernel, dim3(n_tiles), dim3(rh::kTileRows), 0, stream, t, first_tile);
    RH_HIP(hipGetLastError());
    return RH_OK;
}

int rh_table_lease(const rh::TableDev& t, int64_t now_nanos, int64_t timeout_ms, uint64_t* d_slot_bits,
                   uint64_t* d_clear_bits, uint32_t clear_words, hipStream_t stream) {
    bool cleared = false;
    for (int i = 0; i < rh::kTableTiers; ++i) {
        const TableTier& tt = t.tier[i];
        if (!tt.rows) continue;
        uint64_t* clear = cleared ? nullptr : d_clear_bits;   // the first launch clears the other bitmap
        const uint32_t cw = cleared ? 0u : clear_words;
        cleared = true;
        switch (tt.width) {
            case 2: launch_lease_width<2>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            case 4: launch_lease_width<4>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            case 6: launch_lease_width<6>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            case 8: launch_lease_width<8>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            case 10: launch_lease_width<10>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            case 12: launch_lease_width<12>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            case 14: launch_lease_width<14>(tt, now_nanos, timeout_ms, d_slot_bits, clear, cw, stream); break;
            default: return rh::fail(RH_E_STATE, "rh_lease_batch: unexpected tier width");
        }
        RH_HIP(hipGetLastError());
    }
    if (!cleared && d_clear_bits && clear_words) RH_HIP(hipMemsetAsync(d_clear_bits, 0, (size_t)clear_words * 8, stream));
    return RH_OK;
}

int rh_table_read(const rh::TableDev& t, uint32_t first, uint32_t n, uint8_t column, int64_t* d_out,
                  hipStream_t stream) {
    if (n == 0) return RH_OK;
    hipLaunchKernelGGL(table_read_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, t, first, n, (uint32_t)column, d_out);
    RH_HIP(hipGetLastError());
    return RH_OK;
}
